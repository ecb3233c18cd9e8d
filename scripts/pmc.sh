# PMC passes over bench.py (config via BENCH_ARGS), one rocprofv3 run per counter set, summary
# of the kernels whose name contains $1.   bash scripts/pmc.sh <kernel-substr> "<ctr ctr ..>" ...
set -e
cd "$GRAFT_REPO_ROOT"
filt=$1; shift
out=gpurun_out/pmc_$filt
rm -rf $out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
n=0
for set in "$@"; do
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $out/s$n -o run -- \
    python3 bench.py ${BENCH_ARGS:---config P} --no-graph --steps 2 --warmup 1 --kernel-reps 1 --no-cpu-baseline > /dev/null 2> $out/s$n.log || echo "pmc set $n failed"
done
python3 - "$out" "$filt" <<'PY'
import csv, glob, sys, collections
out, filt = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if filt in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), "mean %.4g" % (sum(v) / len(v)))
PY
