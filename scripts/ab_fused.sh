# A/B of the fused-kernel knobs on config S and P (tuning aid; results under gpurun_out/ab)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for cfg in "1 64" "2 64" "1 0" "2 0"; do
  set -- $cfg
  DG_WPG=$1 DG_FUSED_PROJ_MAX=$2 timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ab/S_w$1_p$2.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ab/S_w$1_p$2.json')); print('S wpg=$1 proj=$2', round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1), round(d['spmm_layer2_ms']*1e3,1))"
done
for cfg in "1 64" "3 64"; do
  set -- $cfg
  DG_WPG=$1 DG_FUSED_PROJ_MAX=$2 timeout -k 10 200 python bench.py --config P --steps 10 --warmup 2 --kernel-reps 10 --no-cpu-baseline > gpurun_out/ab/P_w$1_p$2.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ab/P_w$1_p$2.json')); print('P wpg=$1 proj=$2', round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1), round(d['spmm_layer2_ms']*1e3,1))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DG_WPG=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/profS -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > /dev/null 2>&1
echo prof done
