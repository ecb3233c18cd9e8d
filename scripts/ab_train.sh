# A/B the training step between this tree and another checkout (tuning aid):
#   AB_OTHER=<tree> bash scripts/ab_train.sh [bench args]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for tree in . ${AB_OTHER}; do
    tag=$(basename $(cd $tree && pwd))_$rep
    (cd $tree && timeout -k 10 200 python bench.py --train --no-cpu-baseline "$@") > gpurun_out/ab/T_$tag.json 2>gpurun_out/ab/T_$tag.err
    python -c "import json; d=json.load(open('gpurun_out/ab/T_$tag.json')); print('train $tag', round(d['ms_per_step']*1e3,1))"
  done
done
