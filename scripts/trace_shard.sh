# Kernel trace of the one-GPU rehearsal of the sharded (N > 1) step.  -> gpurun_out/trace_<tag>/
set -e
tag=$1; shift
cd "$GRAFT_REPO_ROOT"
out=$GRAFT_REPO_ROOT/gpurun_out/trace_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t -o run -- \
  python3 bench.py --force-shard --no-cpu-baseline "$@" > $out/bench.json 2> $out/trace.log
python3 scripts/trace_table.py $out
