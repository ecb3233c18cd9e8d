# One GPU call: the -m gpu suite (optionally a subset), then the default bench line.
# Usage on the box: bash scripts/gpu_check.sh <tag> [pytest selection...]
set -o pipefail
tag=${1:-check}; shift
out=gpurun_out/$tag
mkdir -p $out
sel=${@:-tests}
timeout -k 10 1000 python -u -m pytest $sel -m gpu -x -v -s --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -5 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
rc=$?
cat $out/bench.json
exit $rc
