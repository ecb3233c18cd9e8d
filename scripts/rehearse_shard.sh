# One-GPU rehearsal of the N > 1 bench step (relation-sharded plan + RCCL world-1 all-reduces):
# eager collectives vs all-reduces captured in the hipGraph.  Results: gpurun_out/shard/
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/shard
for mode in eager graph; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 1 --force-shard --collectives $mode --no-cpu-baseline \
    ${CFG_ARGS:-} > gpurun_out/shard/S_$mode.json 2> gpurun_out/shard/S_$mode.err
  python -c "import json; d=json.load(open('gpurun_out/shard/S_$mode.json')); print('$mode', d['ms_per_step']*1e3, 'us/step', d['config']['launch'])"
done
