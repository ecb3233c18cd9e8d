# A/B of the S launches (scripts/prof_build variants vs the default build), then a GPU test
# selection.  Usage on the box: bash scripts/ab_r02b.sh <tag> [pytest selection...]
set -o pipefail
tag=${1:-ab}; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python scripts/variants.py run scripts/s_times.py > $out/variants.jsonl 2> $out/variants.err || exit $?
cat $out/variants.jsonl
sel=${@:-tests}
timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -5 $out/pytest.log; exit $rc
