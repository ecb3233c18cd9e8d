# Many-chunk plain reduce in one workgroup per row (chunk_reduce_kernel) vs one wave per row
set -o pipefail
mkdir -p gpurun_out/r6u
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "epilogue or staged" --timeout 120 --timeout-method thread > gpurun_out/r6u/pytest.log 2>&1 || { tail -20 gpurun_out/r6u/pytest.log; exit 1; }
tail -1 gpurun_out/r6u/pytest.log
bash scripts/simP_ab.sh r6u 8 base rowwave base rowwave || exit $?
REPS=1 bash scripts/ab.sh r6uP "--config P --steps 50 --warmup 5" rowwave || exit $?
