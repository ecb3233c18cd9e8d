# Config S weak-scaling rank share (--simulate-world N: rank 0's launches on one GPU, the
# collectives as copies) under rocprofv3 kernel-trace stats.  Usage: bash scripts/prof_s8.sh <tag>
set -o pipefail
tag=${1:-s8}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 1 8; do
  sim=""; [ $n -gt 1 ] && sim="--simulate-world $n"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/S$n -o run -- \
    python3 bench.py --config S $sim --steps 100 --warmup 10 --kernel-reps 20 --no-extra --no-cpu-baseline \
    > $out/S$n.json 2> $out/S$n.log || exit $?
  echo "S$n done"
done
