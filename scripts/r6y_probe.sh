# Drug-target relation dealt by rows over every rank (DG_SHARD_DEAL_ROWS): sharded parity
# (forward, training), then config P's rank shares at N = 8 / 4 against the LPT owner form
set -o pipefail
mkdir -p gpurun_out/r6y
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py -x -v -m gpu -k "P_shaped or full_size_P or training" --timeout 400 --timeout-method thread > gpurun_out/r6y/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r6y/pytest.log | head -20; tail -5 gpurun_out/r6y/pytest.log; exit 1; }
tail -1 gpurun_out/r6y/pytest.log
bash scripts/simP_ab.sh r6y 8 base DG_SHARD_DEAL_ROWS=0 base DG_SHARD_DEAL_ROWS=0 || exit $?
bash scripts/simP_ab.sh r6y4 4 base DG_SHARD_DEAL_ROWS=0 || exit $?
