set -o pipefail
mkdir -p gpurun_out/r6l
timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_kernels.py tests/test_gpu_train.py -m gpu > gpurun_out/r6l/pytest.log 2>&1 || { tail -30 gpurun_out/r6l/pytest.log; exit 1; }
tail -1 gpurun_out/r6l/pytest.log
REPS=3 bash scripts/ab.sh r6l "--steps 200 --warmup 20 --no-extra --no-cpu-baseline" decr5 || exit $?
timeout -k 10 120 python scripts/dec_prof.py 20 > gpurun_out/r6l/dec_prof.json || exit $?
