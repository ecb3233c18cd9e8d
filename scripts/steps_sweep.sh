# Step time vs the number of timed steps and steps per hipGraph (fixed per-call / per-replay
# overheads of bench.py's host-clocked timing), one summary line per run.
# Usage on the box: bash scripts/steps_sweep.sh <tag> <config> "<steps:graph_steps> ..."
set -o pipefail
tag=$1; cfg=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for sg in $1; do
  s=${sg%%:*}; g=${sg##*:}
  timeout -k 10 300 python bench.py --config $cfg --steps $s --warmup 5 --graph-steps $g --no-cpu-baseline \
    > $out/${cfg}_${s}_${g}.json 2> $out/${cfg}_${s}_${g}.err || exit $?
  python scripts/bench_summary.py "$cfg steps=$s graph=$g" $out/${cfg}_${s}_${g}.json
done
