# Kernel-trace stats of one bench config (tuning aid).  Usage on the GPU box:
#   bash scripts/trace.sh <tag> <config> [extra bench args]   -> gpurun_out/trace_<tag>/
set -e
tag=$1; cfg=$2; shift 2
cd "$GRAFT_REPO_ROOT"
out=$GRAFT_REPO_ROOT/gpurun_out/trace_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t -o run -- \
  python3 bench.py --config $cfg --no-cpu-baseline "$@" > $out/bench.json 2> $out/trace.log
python3 - $out <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/t/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{n[:60]:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} us {float(r['Percentage']):6.1f}%")
PY
