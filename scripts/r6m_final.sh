set -o pipefail
bash scripts/gpu_round.sh r6m || exit $?
for i in 2 3; do
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r6m/bench$i.json 2> gpurun_out/r6m/bench$i.err || exit $?
  python scripts/bench_summary.py default$i gpurun_out/r6m/bench$i.json
done
timeout -k 10 300 python bench.py > gpurun_out/r6m/bench_noargs.json 2> gpurun_out/r6m/bench_noargs.err || exit $?
python scripts/bench_summary.py noargs gpurun_out/r6m/bench_noargs.json
