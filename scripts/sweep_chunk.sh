set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for c in 4 8 16 37; do
  timeout -k 10 200 python bench.py --config P --steps 10 --warmup 2 --kernel-reps 10 --no-cpu-baseline --chunk $c > gpurun_out/sweep/P_chunk$c.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/sweep/P_chunk$c.json')); print('chunk $c', d['ms_per_step'], d['roofline']['kernel_ms'], d['spmm_layer2_ms'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "spmm|fused" --output-format csv -d gpurun_out/sweep/pmc -o run -- python3 bench.py --config P --steps 3 --warmup 1 --kernel-reps 2 --no-cpu-baseline > /dev/null 2>&1
echo pmc done
