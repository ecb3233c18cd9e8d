set -o pipefail
mkdir -p gpurun_out/r6j
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tab.py tests/test_gpu_model.py -m gpu > gpurun_out/r6j/pytest.log 2>&1 || { tail -30 gpurun_out/r6j/pytest.log; exit 1; }
tail -1 gpurun_out/r6j/pytest.log
REPS=3 bash scripts/ab.sh r6j "--steps 200 --warmup 20 --no-extra --no-cpu-baseline" DG_TAB_WLDS=0 || exit $?
timeout -k 10 120 python scripts/fseg_prof.py 20 > gpurun_out/r6j/fseg_prof.json || exit $?
