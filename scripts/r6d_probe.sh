set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_tab.py tests/test_gpu_model.py -m gpu > gpurun_out/r6d/pytest_tab.log 2>&1 || { tail -30 gpurun_out/r6d/pytest_tab.log; exit 1; }
tail -1 gpurun_out/r6d/pytest_tab.log
REPS=3 bash scripts/ab.sh r6d "--steps 200 --warmup 20 --no-extra --no-cpu-baseline" twophase serlds DG_TAB_BALANCE=0 pdpp@DG_TAB_PROJ_DPP=1 wpre || exit $?
timeout -k 10 120 python scripts/fseg_prof.py 20 > gpurun_out/r6d/fseg_prof.json || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_peer.py -m gpu -k "device_tensor or loopback" > gpurun_out/r6d/pytest_kinds.log 2>&1; tail -1 gpurun_out/r6d/pytest_kinds.log
bash scripts/sim_ab.sh r6d_s8 8 peer:base peer:DG_PEER_REGION_KIND=1 peer:DG_PEER_REGION_KIND=2 || exit $?
EXCHANGE=peer bash scripts/simP_ab.sh r6d_p8 8 base DG_PEER_REGION_KIND=1 DG_PEER_REGION_KIND=2 || exit $?
bash scripts/simP_ab.sh r6d_p8c 8 base DG_CONCURRENT=1 DG_CONCURRENT=1,DG_STAGED_FIRST=0 || exit $?
timeout -k 10 300 python bench.py --config D --simulate-world 8 --steps 50 --warmup 5 > gpurun_out/r6d/simD8.json 2> gpurun_out/r6d/simD8.err || exit $?
python -c "import json; r=json.load(open('gpurun_out/r6d/simD8.json')); print('D8 max rank %.1f us' % (1e3*r['max_rank_ms_per_step']), [round(1e3*x['ms_per_step'],1) for x in r['ranks']])"
REPS=2 bash scripts/ab.sh r6d_p "--config P --steps 50 --warmup 5 --no-cpu-baseline --kernel-reps 20" ntcsr || exit $?
