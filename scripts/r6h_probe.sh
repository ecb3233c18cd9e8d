set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_tab.py tests/test_gpu_model.py tests/test_gpu_peer.py tests/test_gpu_sharded.py -m gpu > gpurun_out/r6h/pytest.log 2>&1 || { tail -30 gpurun_out/r6h/pytest.log; exit 1; }
tail -1 gpurun_out/r6h/pytest.log
REPS=3 bash scripts/ab.sh r6h "--steps 200 --warmup 20 --no-extra --no-cpu-baseline" DG_TAB_SLOT=64 DG_TAB_SLOT=32 || exit $?
timeout -k 10 120 python scripts/fseg_prof.py 20 > gpurun_out/r6h/fseg_prof.json || exit $?
bash scripts/sim_ab.sh r6h_s8 8 rccl:base rccl:DG_TAB_SLOT=64 peer:base || exit $?
