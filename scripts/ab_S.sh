# S-config A/B: waves per group and steps per graph (tuning aid; results under gpurun_out/abS)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abS
for gs in 1 10; do for w in 1 2 4 8; do
  DG_WPG=$w timeout -k 10 200 python bench.py --graph-steps $gs --no-cpu-baseline > gpurun_out/abS/w${w}_g${gs}.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/abS/w${w}_g${gs}.json')); print('S wpg=$w gs=$gs', round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2), round(d['spmm_layer2_ms']*1e3,2))"
done; done
