set -o pipefail
out=gpurun_out/r6i; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-extra --no-cpu-baseline > $out/plain.json 2> $out/plain.err || exit $?
python scripts/bench_summary.py plain $out/plain.json
for v in base slot64 bal0; do
  case $v in base) envs="";; slot64) envs="DG_TAB_SLOT=64";; bal0) envs="DG_TAB_BALANCE=0";; esac
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run -- \
    python3 bench.py --steps 200 --warmup 20 --no-extra --no-cpu-baseline --kernel-reps 200 > $out/$v.json 2> $out/$v.log || exit $?
  python scripts/bench_summary.py prof_$v $out/$v.json
  python - "$out/$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "tab_kernel" in r["Name"] or "decoder_hinge" in r["Name"]:
        print("   ", r["Name"][:40], r["Calls"], "avg us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
done
