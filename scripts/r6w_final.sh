# Final tree: the -m gpu suite, smoke, default bench; config P one GPU (3 runs) and its N = 8 / 4
# rank shares; rocprofv3 kernel stats of config P and of its N = 8 rank 0
set -o pipefail
bash scripts/gpu_round.sh r6w || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --config P --steps 20 --warmup 5 > gpurun_out/r6w/benchP$i.json 2> gpurun_out/r6w/benchP$i.err || exit $?
  python scripts/bench_summary.py P$i gpurun_out/r6w/benchP$i.json
done
bash scripts/simP_ab.sh r6w_p8 8 base || exit $?
bash scripts/simP_ab.sh r6w_p4 4 base || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6w/P_trace -o run -- python3 bench.py --config P --steps 20 --warmup 3 --kernel-reps 20 --no-cpu-baseline > gpurun_out/r6w/P_prof.json 2> gpurun_out/r6w/P_prof.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6w/P8_trace -o run -- python3 bench.py --config P --simulate-world 8 --simulate-rank 0 --steps 50 --warmup 5 > gpurun_out/r6w/P8_prof.json 2> gpurun_out/r6w/P8_prof.err || exit 1
echo done
