# Training checks on one GPU: the training / sharded / ingestion tests, then the training bench
# (S, P) on one GPU and the relation-sharded training step over RCCL at world size 1.
set -o pipefail
out=gpurun_out/${1:-trainchk}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_sharded.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --steps 20 --warmup 3 > $out/trainS.json 2> $out/trainS.err || exit $?
timeout -k 10 300 python bench.py --train --config P --steps 10 --warmup 2 > $out/trainP.json 2> $out/trainP.err || exit $?
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --train --force-shard --steps 20 --warmup 3 > $out/trainS_shard1.json 2> $out/trainS_shard1.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --train --config P --force-shard --steps 10 --warmup 2 > $out/trainP_shard1.json 2> $out/trainP_shard1.err || exit $?
for f in trainS trainP trainS_shard1 trainP_shard1; do python3 -c "import json; d=json.load(open('$out/$f.json')); print('$f', round(d['ms_per_step']*1e3,1), 'us', d['config']['parallelism'], d['loss_first_step'], d['loss_last_step'])"; done
