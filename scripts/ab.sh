# A/B timing on the GPU box: the same bench command with the default library and each variant,
# REPS rounds (default 2), one summary line per run (scripts/bench_summary.py).
# A variant is NAME — decagon_amd/lib/var_NAME.so, built on the CPU container with
# `python -m decagon_amd._build NAME FLAG[=VALUE]...` — or VAR=value, an environment setting (knobs
# such as DG_S_ROWS_FORM, DG_PROJ_BLOCKS, DG_WPG; several joined by commas) with the default library,
# or NAME@VAR=value[,VAR=value], both.
# Usage: bash scripts/ab.sh <tag> "<bench args>" VARIANT...
set -o pipefail
tag=$1; shift
args=$1; shift
out=gpurun_out/ab_$tag; mkdir -p $out
for rep in $(seq 1 ${REPS:-2}); do
  for v in base "$@"; do
    lib=""; envs=""
    case $v in base) ;; *@*) lib=$PWD/decagon_amd/lib/var_${v%%@*}.so; envs=$(echo "${v#*@}" | tr ',' ' ');;
      *=*) envs=$(echo "$v" | tr ',' ' ');; *) lib=$PWD/decagon_amd/lib/var_$v.so;; esac
    name=$(echo "$v" | tr -c 'A-Za-z0-9_.-' '_')
    env DG_LIB=$lib $envs timeout -k 10 300 python bench.py $args > $out/${name}_$rep.json 2> $out/${name}_$rep.err || exit $?
    python scripts/bench_summary.py "$v" $out/${name}_$rep.json
  done
done
