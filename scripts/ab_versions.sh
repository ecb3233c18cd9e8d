# A/B config P between this tree and another checkout (tuning aid): AB_OTHER=<tree> bash scripts/ab_versions.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for tree in . ${AB_OTHER}; do
    tag=$(basename $(cd $tree && pwd))_$rep
    (cd $tree && timeout -k 10 200 python bench.py --config P --steps 10 --warmup 2 --kernel-reps 10 --no-cpu-baseline) > gpurun_out/ab/V_$tag.json 2>gpurun_out/ab/V_$tag.err
    python -c "import json; d=json.load(open('gpurun_out/ab/V_$tag.json')); print('P $tag', round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1), round(d['spmm_layer2_ms']*1e3,1))"
  done
done
