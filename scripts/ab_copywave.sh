# A/B of the staged kernel's copy-wave form (config P): default build vs DG_STAGED_COPYWAVE=1/2/3
# build with the layout's lanes at 960 (wave 15 left without pairs) and at 1024; then the
# staged parity tests on the variant.  Usage on the box: bash scripts/ab_copywave.sh <tag>
set -o pipefail
# Build the variants first: python scripts/variants.py build cwN -DDG_STAGED_COPYWAVE=N (N = 1, 2, 3)
out=gpurun_out/${1:-abcw}; mkdir -p $out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config P --no-cpu-baseline --steps 20 --warmup 3 --kernel-reps 20 \
    > $out/$name.json 2> $out/$name.err || return $?
  python3 - $out/$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d['roofline']
print('%-12s step %.1f us  staged L1 %.1f us (%.1f%%)  L1 %.1f  L2 %.1f' % (sys.argv[2], d['ms_per_step']*1e3, r['kernel_ms']*1e3, 100*r['frac'], d['spmm_layer1']['ms']*1e3, d['spmm_layer2_ms']*1e3), flush=True)
PY
}
run base DG_STAGED_LANES=1024 || exit $?
run base896 DG_STAGED_LANES=896 || exit $?
run base832 DG_STAGED_LANES=832 || exit $?
run cw1_960 DG_LIB=scripts/prof_build/lib_cw1.so DG_STAGED_LANES=960 || exit $?
run cw2_896 DG_LIB=scripts/prof_build/lib_cw2.so DG_STAGED_LANES=896 || exit $?
run cw3_832 DG_LIB=scripts/prof_build/lib_cw3.so DG_STAGED_LANES=832 || exit $?
run base_again DG_STAGED_LANES=1024 || exit $?
DG_LIB=scripts/prof_build/lib_cw2.so DG_STAGED_LANES=896 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "staged or P" > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; exit $rc
