# Round profile: rocprofv3 kernel-trace stats of the default bench (config S) and of config P,
# then one PMC pass per TCC counter (FETCH_SIZE, WRITE_SIZE: they do not fit one pass).
# Usage on the GPU box:  bash scripts/profile_round.sh <tag>      (outputs: gpurun_out/prof_<tag>/)
set -e
tag=${1:-r01}
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in S P; do
  if [ $cfg = S ]; then steps="--steps 200 --warmup 20 --kernel-reps 200 --no-extra"; else steps="--steps 20 --warmup 3 --kernel-reps 20"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${cfg}_trace -o run -- \
    python3 bench.py --config $cfg $steps --no-cpu-baseline > $out/${cfg}_bench.json 2> $out/${cfg}_trace.log
  echo "$cfg trace done"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $out/${cfg}_$ctr -o run -- \
      python3 bench.py --config $cfg --no-graph --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline \
      > /dev/null 2> $out/${cfg}_$ctr.log
    echo "$cfg $ctr done"
  done
done
# the staged kernel's LDS bank-conflict ratio (config P, both layers; one pass, SQ block only)
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS --kernel-trace \
  --output-format csv -d $out/P_LDS -o run -- \
  python3 bench.py --config P --no-graph --steps 5 --warmup 1 --kernel-reps 3 --no-cpu-baseline \
  > /dev/null 2> $out/P_LDS.log
echo "P LDS done"
for cfg in S P; do
  if [ $cfg = S ]; then steps="--steps 100 --warmup 10"; else steps="--steps 5 --warmup 1 --graph-steps 1"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/train${cfg}_trace -o run -- \
    python3 bench.py --train --config $cfg $steps > $out/train${cfg}_bench.json 2> $out/train${cfg}_trace.log
  echo "train $cfg trace done"
done
# rank 0's share of the 8-GPU step (collectives as no-ops), configs S and P
for cfg in S P; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${cfg}8_trace -o run -- \
    python3 bench.py --config $cfg --simulate-world 8 --simulate-rank 0 --steps 50 --warmup 5 \
    > $out/${cfg}8_bench.json 2> $out/${cfg}8_trace.log
  echo "$cfg N=8 rank 0 trace done"
done
# config 5 (bf16 DEDICOM scorer): kernel trace, then MFMA busy cycles against the GPU clock
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/D_trace -o run -- \
  python3 bench.py --config D --steps 50 --warmup 5 --no-cpu-baseline > $out/D_bench.json 2> $out/D_trace.log
echo "D trace done"
timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d $out/D_MFMA -o run -- \
  python3 bench.py --config D --no-graph --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> $out/D_MFMA.log
echo "D mfma done"
python3 scripts/prof_summary.py $out > $out/summary.md
python3 scripts/prof_summary.py $out --json $out/traffic.json
echo summary done
