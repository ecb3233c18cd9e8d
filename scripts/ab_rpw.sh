# Partial-mode SpMM rows per wave: parity tests on the default build, then config P's step and
# per-launch times with each variant build (DG_LIB) and the default.
set -o pipefail
out=gpurun_out/rpw; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in default rpw1 rpw4 default; do
  lib=""; [ $v != default ] && lib=scripts/prof_build/lib_$v.so
  DG_LIB=$lib timeout -k 10 300 python bench.py --config P --steps 20 --warmup 3 --kernel-reps 20 --no-cpu-baseline \
    > $out/P_$v.json 2> $out/P_$v.err || exit $?
  python -c "import json; r=json.load(open('$out/P_$v.json')); print('$v', round(r['ms_per_step']*1e3,1), 'us/step; layer1 spmm', round(r['spmm_layer1']['ms']*1e3,1), 'layer2 spmm', round(r['spmm_layer2_ms']*1e3,1))"
done
