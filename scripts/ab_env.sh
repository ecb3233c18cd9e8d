# Config P forward under different environment settings (A/B of host-side layout knobs).
# Usage on the box: bash scripts/ab_env.sh <tag> "VAR=a VAR2=b" "VAR=c" ...   ("" = defaults)
set -o pipefail
out=gpurun_out/${1:-abE}; shift; mkdir -p $out
for envs in "$@"; do
  env $envs timeout -k 10 300 python bench.py --config P --no-cpu-baseline --steps 20 --warmup 3 --kernel-reps 20 \
    > $out/run.json 2>> $out/err.log || exit $?
  python3 - $out/run.json "$envs" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read()); r = d['roofline']
print('[%s] step %.1f us  staged L1 %.1f us (%.1f%%)  L1 %.1f  L2 %.1f' % (sys.argv[2], d['ms_per_step']*1e3, r['kernel_ms']*1e3, 100*r['frac'], d['spmm_layer1']['ms']*1e3, d['spmm_layer2_ms']*1e3))
PY
done
