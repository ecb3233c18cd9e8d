# A/B of DG_PROJ_UNROLL (W2 loads per batch of the fused kernel's projection epilogue) on
# configs S and P; build decagon_amd/lib/ab_u32.so / ab_u64.so with -DDG_PROJ_UNROLL=32 / 64 first
set -o pipefail
out=gpurun_out/ab_unroll; mkdir -p $out
for rep in 1 2; do
  for v in 16 32 64; do
    lib=""; [ $v = 16 ] || lib=$PWD/decagon_amd/lib/ab_u$v.so
    DG_LIB=$lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --config S \
      > $out/S_$v$rep.json 2> $out/S_$v$rep.err || exit $?
    DG_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --config P \
      > $out/P_$v$rep.json 2> $out/P_$v$rep.err || exit $?
    python -c "import json; d=json.load(open('$out/S_$v$rep.json')); p=json.load(open('$out/P_$v$rep.json')); print('unroll $v S', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), 'P', round(p['ms_per_step']*1e3,1))"
  done
done
