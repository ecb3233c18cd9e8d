# Config S rank share at N = 8 (--simulate-world 8) against the projection GEMM's grid knob.
set -o pipefail
out=gpurun_out/s8sweep; mkdir -p $out
for pb in 512 128 32 2048 512; do
  DG_PROJ_BLOCKS=$pb timeout -k 10 300 python3 bench.py --config S --simulate-world 8 --steps 100 --warmup 10 \
    --kernel-reps 20 --no-extra --no-cpu-baseline > $out/pb$pb.json 2> $out/pb$pb.err || exit $?
  python3 -c "import json; r=json.load(open('$out/pb$pb.json')); print($pb, round(r['max_rank_ms_per_step']*1e3,2), [round(x['ms_per_step']*1e3,1) for x in r['ranks']])"
done
