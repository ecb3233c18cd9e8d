# A/B of config-P launch options (env-controlled), forward step + per-layer SpMM times.
# Usage on the box: bash scripts/ab_r02.sh <tag> "ENV=.. ENV=.." ...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python3 bench.py --config P --no-cpu-baseline --steps 20 --warmup 3 --kernel-reps 20 \
    > $out/v$i.json 2> $out/v$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open('$out/v$i.json')); r=d['roofline']; print('$v', 'step %.1f us' % (d['ms_per_step']*1e3), 'L1 %.1f us' % (d['spmm_layer1']['ms']*1e3), 'L2 %.1f us' % (d['spmm_layer2_ms']*1e3), 'staged %.1f us' % (r['kernel_ms']*1e3))"
done
