# Epilogue partial loads in flight (8 default; variants 4, 16) and the drug-target LPT cost sweep
set -o pipefail
bash scripts/simP_ab.sh r6t 8 base epib4 epib16 DG_SHARD_GROUP_TAIL=150000 DG_SHARD_GROUP_TAIL=250000 || exit $?
REPS=1 bash scripts/ab.sh r6tP "--config P --steps 50 --warmup 5" epib4 || exit $?
REPS=2 bash scripts/ab.sh r6tS "--steps 200 --warmup 20 --no-extra" epib4 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6t_trace
for r in 0 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6t_trace/rank$r -o run -- python3 bench.py --config P --simulate-world 8 --simulate-rank $r --steps 20 --warmup 5 --no-graph > gpurun_out/r6t_trace/rank$r.json 2> gpurun_out/r6t_trace/rank$r.err || exit 1
done
