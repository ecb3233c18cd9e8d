# Config P's N-GPU rank share on one GPU (bench.py --config P --simulate-world N, collectives as
# no-ops), one summary line per variant: "base", a library variant NAME (decagon_amd/lib/var_NAME.so)
# or VAR=value settings (several joined by commas).
# Usage on the box: bash scripts/simP_ab.sh <tag> <N> VARIANT ...
set -o pipefail
tag=$1; N=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for v in "$@"; do
  lib=""; envs=""
  case $v in base) ;; *=*) envs=$(echo "$v" | tr ',' ' ');; *) lib=$PWD/decagon_amd/lib/var_$v.so;; esac
  name=$(echo "$v" | tr -c 'A-Za-z0-9_.-' '_')
  env DG_LIB=$lib $envs timeout -k 10 300 python bench.py --config P --simulate-world $N --exchange ${EXCHANGE:-rccl} --steps 50 --warmup 5 \
      > $out/simP_$name.json 2> $out/simP_$name.err || { tail -5 $out/simP_$name.err; exit 1; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], 'max rank %.2f us' % (1e3*r['max_rank_ms_per_step']), 'ranks', [round(1e3*x['ms_per_step'],1) for x in r['ranks']])" $out/simP_$name.json "$v"
done
