# Row-table epilogue's long-chunk loop: 8 loads in flight (default) vs 4 (epitab4); bitwise tests
set -o pipefail
mkdir -p gpurun_out/r6aa
timeout -k 10 600 python -u -m pytest tests/test_gpu_tab.py tests/test_gpu_kernels.py -x -q -m gpu -k "epilogue" --timeout 300 --timeout-method thread > gpurun_out/r6aa/pytest.log 2>&1 || { tail -20 gpurun_out/r6aa/pytest.log; exit 1; }
tail -1 gpurun_out/r6aa/pytest.log
REPS=2 bash scripts/ab.sh r6aaP "--config P --steps 50 --warmup 5" epitab4 || exit $?
