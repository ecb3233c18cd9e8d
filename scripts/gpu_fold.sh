# Layer 2 + decoder in one launch: its GPU tests, S bench folded vs not, then the -m gpu suite
# and the default bench line.  Usage on the box: bash scripts/gpu_fold.sh <tag>
set -o pipefail
tag=${1:-fold}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step_fold.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/fold.log 2>&1
rc=$?; tail -15 $out/fold.log; [ $rc -eq 0 ] || exit $rc
for v in step.a layer2.a none.a step.b layer2.b none.b; do
  extra="--fold ${v%.*}"
  timeout -k 10 300 python bench.py --config S --steps 200 --warmup 20 --no-extra --no-cpu-baseline $extra \
    > $out/S_$v.json 2> $out/S_$v.err || exit $?
  python -c "import json,sys; r=json.load(open('$out/S_$v.json')); print('$v', r['ms_per_step']*1e3, 'us/step', r['spmm_layer2_ms']*1e3, r['folded'])"
done
[ "$2" = quick ] && exit 0
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -5 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?; cat $out/bench.json | head -c 600; exit $rc
