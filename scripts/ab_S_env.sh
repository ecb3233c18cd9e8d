# Config S per-launch and step times (scripts/s_times.py) under environment settings.
# Usage on the box: bash scripts/ab_S_env.sh <tag> "VAR=a" "" ...
set -o pipefail
out=gpurun_out/${1:-abSE}; shift; mkdir -p $out
for envs in "$@"; do
  for rep in 1 2; do
    env $envs timeout -k 10 300 python scripts/s_times.py >> $out/s.jsonl 2>> $out/s.err || exit $?
  done
done
cat $out/s.jsonl
