# A/B the LDS-staged kernel on config P (tuning aid; results under gpurun_out/ab)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for cfg in "0 16" "1 16" "1 32"; do
  set -- $cfg
  DG_STAGED=$1 DG_STAGED_SLICE=$2 timeout -k 10 200 python bench.py --config P --steps 10 --warmup 2 --kernel-reps 10 --no-cpu-baseline > gpurun_out/ab/P_st$1_$2.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/ab/P_st$1_$2.json')); print('P staged=$1 slice=$2', round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1), round(d['spmm_layer2_ms']*1e3,1), round(d['roofline']['achieved']), 'GB/s')"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/profP -o run -- python3 bench.py --config P --steps 10 --warmup 2 --kernel-reps 2 --no-cpu-baseline > /dev/null 2>&1
echo prof done
