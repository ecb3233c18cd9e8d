# Final tree re-check after the engine/sharding edits: the -m gpu suite, smoke, default bench line
set -o pipefail
bash scripts/gpu_round.sh r6z || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r6z/bench_noargs.json 2> gpurun_out/r6z/bench_noargs.err || exit $?
python scripts/bench_summary.py noargs gpurun_out/r6z/bench_noargs.json
