# One-step kernel timelines of config P and of rank 0 of the 8-GPU plan (rehearsed on one GPU)
# under environment settings.  Usage on the box: bash scripts/tl_env.sh <tag> "VAR=a" "" ...
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-tlE}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
k=0
for envs in "$@"; do
  k=$((k + 1))
  for run in "P --config P" "P8r0 --config P --simulate-world 8 --simulate-rank 0"; do
    set -- $run; n=$1; shift
    env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$n.$k -o run -- \
      python3 bench.py --no-cpu-baseline --no-extra --kernel-reps 5 --steps 20 --warmup 3 "$@" \
      > $out/$n.$k.json 2> $out/$n.$k.log || exit $?
    echo "== $n [$envs]"; python3 scripts/timeline.py $out/$n.$k decoder_hinge 40
  done
done
