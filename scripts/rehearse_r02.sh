# Multi-GPU rehearsals on the one-GPU box (round 2):
#  1. the sharded step over RCCL at world size 1 (torchrun, --force-shard): every collective of
#     the N > 1 path — the all-reduce, the protein all-gather, the config-5 loss all-reduce —
#     captured in the hipGraphs exactly as at N = 8, on one rank;
#  2. each rank's share of the N-GPU config-P step timed alone (--simulate-world N).
set -o pipefail
out=gpurun_out/${1:-r02c}
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 1 --force-shard --steps 20 --warmup 5 --no-cpu-baseline \
  > $out/force_shard.json 2> $out/force_shard.err || exit $?
cat $out/force_shard.json
for N in 2 4 8; do
  timeout -k 10 400 python bench.py --config P --simulate-world $N --steps 20 --warmup 3 \
    > $out/sim$N.json 2> $out/sim$N.err || exit $?
  echo "sim $N done"
done
