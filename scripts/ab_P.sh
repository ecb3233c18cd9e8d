# Config P forward: step, staged layer-1 kernel, layer-1 / layer-2 SpMM for every variant build.
set -o pipefail
out=gpurun_out/${1:-abP}; mkdir -p $out
timeout -k 10 900 python scripts/variants.py run bench.py --config P --no-cpu-baseline --steps 20 --warmup 3 --kernel-reps 20 > $out/v.jsonl 2> $out/v.err || exit $?
python3 - $out/v.jsonl <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line); r = d['roofline']
    print('step %.1f us  staged L1 %.1f us (%.1f%%)  L1 %.1f  L2 %.1f' % (d['ms_per_step']*1e3, r['kernel_ms']*1e3, 100*r['frac'], d['spmm_layer1']['ms']*1e3, d['spmm_layer2_ms']*1e3))
PY
