# Variable staged output chunks: kernel parity, then config P's rank shares at N = 8 and 4 and the
# one-GPU config P step, each against DG_STAGED_VAR=0 (fixed snake-binned runs)
set -o pipefail
mkdir -p gpurun_out/r6p
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k staged --timeout 120 --timeout-method thread > gpurun_out/r6p/pytest.log 2>&1 || { tail -20 gpurun_out/r6p/pytest.log; exit 1; }
tail -1 gpurun_out/r6p/pytest.log
bash scripts/simP_ab.sh r6p 8 base DG_STAGED_VAR=0 || exit $?
bash scripts/simP_ab.sh r6p4 4 base DG_STAGED_VAR=0 || exit $?
REPS=1 bash scripts/ab.sh r6pP "--config P --steps 50 --warmup 5" DG_STAGED_VAR=0 || exit $?
