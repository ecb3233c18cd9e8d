# Layer 2's tab projection: one W round trip (vmcnt(0) before the slice) and the W L1 touch before
# the gathers; nowtouch = the wait only, nowfix = neither (the tree before)
set -o pipefail
mkdir -p gpurun_out/r6ac
timeout -k 10 600 python -u -m pytest tests/test_gpu_tab.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6ac/pytest.log 2>&1 || { tail -20 gpurun_out/r6ac/pytest.log; exit 1; }
tail -1 gpurun_out/r6ac/pytest.log
REPS=3 bash scripts/ab.sh r6ac "--steps 200 --warmup 20 --no-extra" nowtouch nowfix || exit $?
REPS=2 bash scripts/ab.sh r6ac20 "--steps 20 --warmup 5 --no-extra" nowfix || exit $?
