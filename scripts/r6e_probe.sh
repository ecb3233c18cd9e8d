set -o pipefail
mkdir -p gpurun_out/r6e
PEER_WAIT_LOG=gpurun_out/r6e/peer_waits.jsonl timeout -k 10 600 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_tab.py tests/test_gpu_model.py tests/test_gpu_peer.py tests/test_gpu_sharded.py -m gpu > gpurun_out/r6e/pytest.log 2>&1 || { tail -30 gpurun_out/r6e/pytest.log; exit 1; }
tail -1 gpurun_out/r6e/pytest.log
REPS=3 bash scripts/ab.sh r6e "--steps 200 --warmup 20 --no-extra --no-cpu-baseline" DG_TAB_BALANCE=0 DG_TAB_BALANCE=2 pdpp@DG_TAB_PROJ_DPP=1 pdpp@DG_TAB_PROJ_DPP=1,DG_TAB_BALANCE=0 || exit $?
timeout -k 10 120 python scripts/fseg_prof.py 20 > gpurun_out/r6e/fseg_prof.json || exit $?
bash scripts/sim_ab.sh r6e_s8 8 rccl:base peer:base || exit $?
