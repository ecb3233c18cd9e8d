# A/B the LDS-staged kernel on config P (tuning aid; results under gpurun_out/ab)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
# AB_CFGS: comma-separated "DG_STAGED BINS SPLIT" triples
IFS=, read -ra cfgs <<< "${AB_CFGS:-0 128 1,1 128 1,1 128 0,1 64 1,1 256 1}"
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  tag=st$1_b$2_s$3
  DG_STAGED=$1 DG_STAGED_BINS=$2 DG_STAGED_SPLIT=$3 timeout -k 10 200 python bench.py --config P --steps 10 --warmup 2 --kernel-reps 10 --no-cpu-baseline > gpurun_out/ab/P_$tag.json 2>gpurun_out/ab/P_$tag.err
  python -c "import json; d=json.load(open('gpurun_out/ab/P_$tag.json')); print('P $tag', round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1), round(d['spmm_layer2_ms']*1e3,1), round(d['roofline']['achieved']), 'GB/s')"
done
