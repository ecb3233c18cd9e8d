# Staged row pieces of heavy relations (DG_STAGED_PIECE): sharded-P parity, rank shares at N = 8, 4
set -o pipefail
mkdir -p gpurun_out/r6r
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -x -v -m gpu -k "full_size_P or P_shaped or training" --timeout 300 --timeout-method thread > gpurun_out/r6r/pytest.log 2>&1 || { tail -30 gpurun_out/r6r/pytest.log; exit 1; }
tail -1 gpurun_out/r6r/pytest.log
bash scripts/simP_ab.sh r6r 8 base DG_STAGED_PIECE=0 DG_STAGED_PIECE=0.35 || exit $?
bash scripts/simP_ab.sh r6r4 4 base DG_STAGED_PIECE=0 || exit $?
