# Kernel timelines of one step: config S, config P, and rank 0 of the 8-GPU config-P plan
# (rehearsed on one GPU).  Usage on the box: bash scripts/trace_r02.sh <tag>
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-tl}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/$n -o run -- \
    python3 bench.py --no-cpu-baseline --no-extra --kernel-reps 5 "$@" > $out/$n.json 2> $out/$n.log || return $?
  python3 scripts/timeline.py $out/$n decoder_hinge 40 > $out/$n.timeline.txt
  echo "== $n"; cat $out/$n.timeline.txt
}
run S --steps 50 --warmup 5 && run P --config P --steps 20 --warmup 3 && \
  run P8r0 --config P --simulate-world 8 --simulate-rank 0 --steps 20 --warmup 3
