# Loopback rehearsals of config S's N-GPU rank share (bench.py --simulate-world N) for several
# exchange forms / library variants, one summary line each.
# Usage on the box: bash scripts/sim_ab.sh <tag> <N> "<exchange>:<VARIANT or VAR=value or base>" ...
set -o pipefail
tag=$1; N=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
for spec in "$@"; do
  ex=${spec%%:*}; v=${spec#*:}
  lib=""; envs=""
  case $v in base) ;; *=*) envs=$v;; *) lib=$PWD/decagon_amd/lib/var_$v.so;; esac
  name=$(echo "$spec" | tr -c 'A-Za-z0-9_.-' '_')
  env DG_LIB=$lib $envs timeout -k 10 300 python bench.py --config S --simulate-world $N --exchange $ex \
      --steps 100 --warmup 10 > $out/sim_$name.json 2> $out/sim_$name.err || { tail -5 $out/sim_$name.err; exit 1; }
  python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], 'max rank %.2f us' % (1e3*r['max_rank_ms_per_step']), 'ranks', [round(1e3*x['ms_per_step'],1) for x in r['ranks']], 'err', sorted({x.get('peer_error_word') for x in r['ranks']}, key=str))" $out/sim_$name.json "$spec"
done
