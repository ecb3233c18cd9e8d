# gpu_check.sh, then the 8-rank config-P rehearsal (rank shares timed one at a time).
set -o pipefail
tag=${1:-check}; shift
bash scripts/gpu_check.sh $tag "$@" || exit $?
timeout -k 10 400 python3 bench.py --config P --simulate-world 8 --steps 20 --warmup 3 \
  > gpurun_out/$tag/sim8.json 2> gpurun_out/$tag/sim8.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/$tag/sim8.json')); print('sim8 max rank us', d['max_rank_ms_per_step']*1e3)"
