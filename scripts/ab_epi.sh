# Epilogue: 16 partial loads in flight (default build) vs 4 (scripts/prof_build/lib_epi4.so):
# parity tests on the default build, then config P's step with each.
set -o pipefail
out=gpurun_out/epi; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -k "epilogue or polypharmacy or full_size or training_sums" \
  --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in default epi4 default epi4; do
  lib=""; [ $v != default ] && lib=scripts/prof_build/lib_$v.so
  DG_LIB=$lib timeout -k 10 300 python bench.py --config P --steps 20 --warmup 3 --kernel-reps 20 --no-cpu-baseline \
    > $out/P_$v.json 2> $out/P_$v.err || exit $?
  python -c "import json; r=json.load(open('$out/P_$v.json')); print('$v', round(r['ms_per_step']*1e3,1), 'us/step')"
done
