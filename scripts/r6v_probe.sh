set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6v
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6v/rank1 -o run -- python3 bench.py --config P --simulate-world 8 --simulate-rank 1 --steps 20 --warmup 5 --no-graph > gpurun_out/r6v/rank1.json 2> gpurun_out/r6v/rank1.err || exit 1
