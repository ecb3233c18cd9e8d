set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r48
for r in 0 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r48/rank$r -o run -- python3 bench.py --config P --simulate-world 8 --simulate-rank $r --steps 20 --warmup 5 --no-graph > gpurun_out/r48/rank$r.json 2> gpurun_out/r48/rank$r.err || exit 1
done
