# Kernel-trace stats of config P in several trees (tuning aid): AB_OTHER="<tree> ..." bash scripts/ab_trace.sh <kernel substring>
set -e
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for tree in . ${AB_OTHER}; do
  tag=$(basename $(cd $tree && pwd))
  out=$GRAFT_REPO_ROOT/gpurun_out/abt_$tag
  mkdir -p $out
  (cd $tree && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t -o run -- \
    python3 bench.py --config P --steps 10 --warmup 2 --kernel-reps 5 --no-cpu-baseline > $out/bench.json 2> $out/trace.log)
  python3 -c "
import csv,glob,sys
f=glob.glob('$out/t/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if '$1' in r['Name']: print('$tag', r['Name'].split('(')[0][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
done
