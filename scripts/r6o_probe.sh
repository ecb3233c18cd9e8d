# Config P at N = 8: per-kernel trace of rank shares 0, 4 and 5 (4 and 5 are the slow ranks)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6o
for r in 0 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6o/rank$r -o run -- python3 bench.py --config P --simulate-world 8 --simulate-rank $r --steps 20 --warmup 5 --no-graph > gpurun_out/r6o/rank$r.json 2> gpurun_out/r6o/rank$r.err || exit 1
done
