# Sharded-path check on one GPU: the sharded GPU tests, rank 0's share of the 8-GPU P plan
# (timeline), and one-rank RCCL rehearsals of S and P with the per-phase breakdown.
# Usage on the box: bash scripts/gpu_shard_check.sh <tag>
set -o pipefail
out=gpurun_out/${1:-shard}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_config5.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/tl_env.sh ${1:-shard}/tl "" 2>&1 | sed -n '/P8r0/,$p' || exit $?
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
for cfg in S P; do
  timeout -k 10 300 python3 bench.py --force-shard --config $cfg --no-cpu-baseline --no-extra --steps 20 --warmup 3 \
    > $out/rehearse_$cfg.json 2> $out/rehearse_$cfg.err || exit $?
  python3 -c "import json; d=json.load(open('$out/rehearse_$cfg.json')); print('$cfg', round(d['ms_per_step']*1e3,1), 'us', {k: (v if not isinstance(v, list) else [round(x,1) if isinstance(x,float) else x for x in v]) for k, v in d['phases'].items()})"
done
