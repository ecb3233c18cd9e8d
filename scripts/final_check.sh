# Round-end rehearsal: smoke(), the sharded step over RCCL at world size 1 (torchrun), and the
# sharded training step; outputs under gpurun_out/final/
set -o pipefail
out=gpurun_out/final; mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --force-shard --steps 20 --warmup 5 --no-cpu-baseline \
  > $out/force_shard.json 2> $out/force_shard.err || exit $?
head -c 400 $out/force_shard.json; echo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --gpus 1 --force-shard --train --steps 10 --warmup 2 \
  > $out/force_shard_train.json 2> $out/force_shard_train.err || exit $?
head -c 300 $out/force_shard_train.json; echo
