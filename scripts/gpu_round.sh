# One GPU call's core: the -m gpu suite (test failures are reported, not fatal: the timing
# steps after it still run; a crash, abort or time limit ends the call), smoke(), the default
# bench line.  Usage on the box: bash scripts/gpu_round.sh <tag> [pytest selection...]
set -o pipefail
tag=${1:-round}; shift
out=gpurun_out/$tag
mkdir -p $out
sel=${@:-tests}
timeout -k 10 900 python -u -m pytest $sel -m gpu -v --maxfail=20 --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $out/pytest.log | head -20
tail -1 $out/pytest.log
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -5 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
python scripts/bench_summary.py default $out/bench.json
