# A/B the config-5 decoder between this tree and other checkouts (tuning aid):
#   AB_OTHER="<tree> ..." bash scripts/ab_dec.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for tree in . ${AB_OTHER}; do
    tag=$(basename $(cd $tree && pwd))_$rep
    (cd $tree && timeout -k 10 200 python bench.py --config D --no-cpu-baseline) > gpurun_out/ab/D_$tag.json 2>gpurun_out/ab/D_$tag.err
    python -c "import json; d=json.load(open('gpurun_out/ab/D_$tag.json')); print('D $tag', round(d['ms_per_step']*1e3,1), d['roofline'].get('frac'), d['value'])"
  done
done
