set -e
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for nb in 256 512 1024 2048 4096; do
  out=gpurun_out/pb_$nb; mkdir -p $out
  DG_PROJ_BLOCKS=$nb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t -o run -- python3 bench.py --config P --steps 10 --warmup 2 --kernel-reps 5 --no-cpu-baseline > $out/bench.json 2> $out/log
  python3 -c "
import csv,glob,json
f=glob.glob('$out/t/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'gemm_f32_proj' in r['Name']: print('$nb', round(float(r['AverageNs'])/1e3,1))
"
done
