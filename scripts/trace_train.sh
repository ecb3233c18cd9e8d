# Kernel trace of the training-step bench (tuning aid).  -> gpurun_out/trace_<tag>/
set -e
tag=$1; shift
cd "$GRAFT_REPO_ROOT"
out=$GRAFT_REPO_ROOT/gpurun_out/trace_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t -o run -- \
  python3 bench.py --train "$@" > $out/bench.json 2> $out/trace.log
python3 scripts/trace_table.py $out
