# Config 5 scorer: paired-kernel parity tests, then --config D with the paired kernel (default)
set -o pipefail
out=gpurun_out/decp; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_config5.py -m gpu -x -q -k "bf16 or config5" \
  --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline > $out/D_$i.json 2> $out/D_$i.err || exit $?
  python -c "import json; r=json.load(open('$out/D_$i.json')); print('D', round(r['ms_per_step']*1e3,1), 'us/step', r['value'], 'kernel', round(r['roofline']['kernel_ms']*1e3,1), 'us', round(r['roofline']['frac'],3))"
done
