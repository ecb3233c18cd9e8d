# A/B of variant builds on the GPU box: for each decagon_amd/lib/var_<name>.so (built on the
# CPU container with `python -m decagon_amd._build <name> DEFINE...`) and the default library,
# run the same bench command REPS times and print one summary line per run.
# Usage: bash scripts/ab.sh <tag> "<bench args>" <name>... ; env REPS (default 2)
set -o pipefail
tag=$1; shift
args=$1; shift
out=gpurun_out/ab_$tag; mkdir -p $out
for rep in $(seq 1 ${REPS:-2}); do
  for v in base "$@"; do
    lib=""; [ $v = base ] || lib=$PWD/decagon_amd/lib/var_$v.so
    DG_LIB=$lib timeout -k 10 300 python bench.py $args > $out/${v}_$rep.json 2> $out/${v}_$rep.err || exit $?
    python scripts/bench_summary.py $v $out/${v}_$rep.json
  done
done
