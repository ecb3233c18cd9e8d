# Config S step against the fused kernel's waves per group (DG_WPG override), two passes each.
set -o pipefail
out=gpurun_out/wpg; mkdir -p $out
for v in 0 2 4 8 0 2 4 8; do
  env=""; [ $v -gt 0 ] && env="DG_WPG=$v"
  env $env timeout -k 10 300 python bench.py --config S --steps 200 --warmup 20 --kernel-reps 200 --no-extra \
    --no-cpu-baseline > $out/S_$v.json 2> $out/S_$v.err || exit $?
  python -c "import json; r=json.load(open('$out/S_$v.json')); print('wpg $v', round(r['ms_per_step']*1e3,2), 'us/step; L1', round(r['roofline']['kernel_ms']*1e3,2), 'L2', round(r['spmm_layer2_ms']*1e3,2))"
done
