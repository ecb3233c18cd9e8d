# Quick GPU check: a pytest selection (-m gpu), then config S per-launch times of every variant
# build.  Usage on the box: bash scripts/gpu_quick.sh <tag> [pytest args...]
set -o pipefail
tag=${1:-quick}; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/variants.py run scripts/s_times.py > $out/variants.jsonl 2> $out/variants.err || exit $?
cat $out/variants.jsonl
