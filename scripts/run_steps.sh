# Run GPU steps in order, each under its own time limit; a step that ends with a signal / abort /
# time limit (exit >= 124, or 134/139) stops the call (nothing more runs on the GPU after a fault),
# a plain failure (exit 1-123: a failing test, a refused argument) is reported and the next step runs.
# Usage on the box: bash scripts/run_steps.sh <tag> "<cmd 1>" "<cmd 2>" ...
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
i=0
for cmd in "$@"; do
  i=$((i + 1))
  echo "== step $i: $cmd"
  bash -c "$cmd" > $out/step$i.log 2>&1
  rc=$?
  tail -${TAILN:-12} $out/step$i.log
  echo "== step $i rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after step $i (rc=$rc)"; exit $rc; fi
done
