set -o pipefail
mkdir -p gpurun_out/r6g
timeout -k 10 120 python scripts/fseg_prof.py 20 > gpurun_out/r6g/fseg_prof.json || exit $?
REPS=3 bash scripts/ab.sh r6g "--steps 200 --warmup 20 --no-extra --no-cpu-baseline" tab_up8 tab_u8 tab_up2 || exit $?
