# Sweep relations-per-chunk for config P (tuning aid; results under gpurun_out/sweep)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for c in 6 12 20 37 64; do
  timeout -k 10 200 python bench.py --config P --steps 10 --warmup 2 --kernel-reps 10 --no-cpu-baseline --chunk $c > gpurun_out/sweep/P_chunk$c.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/sweep/P_chunk$c.json')); print('chunk $c', round(d['ms_per_step']*1e3,1), round(d['roofline']['kernel_ms']*1e3,1), round(d['spmm_layer2_ms']*1e3,1))"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in 12 37; do
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm|fused" --output-format csv -d gpurun_out/sweep/pmc_c$c -o run -- python3 bench.py --config P --steps 3 --warmup 1 --kernel-reps 2 --no-cpu-baseline --chunk $c > /dev/null 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep/trace -o run -- python3 bench.py --config P --steps 10 --warmup 2 --kernel-reps 2 --no-cpu-baseline > /dev/null 2>&1
echo pmc done
