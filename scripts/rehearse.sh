# Multi-GPU and training rehearsals on the one-GPU box, one step per argument; outputs under
# gpurun_out/<tag>/, one summary line per step (scripts/bench_summary.py).
# Usage on the box: bash scripts/rehearse.sh <tag> STEP...
#   test:<pytest -k expr>   the -m gpu tests matching expr
#   bench:<cfg>             bench.py --config cfg (one GPU)
#   sim:<cfg>:<N>           every rank's share of the N-GPU step on this GPU, collectives as
#                           no-ops (bench.py --simulate-world N)
#   prof:<cfg>:<N>          rank 0's share (N = 1: the one-GPU step) under rocprofv3
#                           --kernel-trace --stats (per-kernel times: gpurun_out/<tag>/prof_<cfg><N>/)
#   rccl:<cfg>              bench.py --force-shard over RCCL at world size 1 (torchrun): every
#                           collective of the N > 1 step captured in the hipGraph
#   train:<cfg>             bench.py --train (one GPU)
#   trainrccl:<cfg>         bench.py --train --force-shard over RCCL at world size 1
# Environment settings for one step: prefix it, e.g. DG_S_ROWS_FORM=fused@sim:S:8
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
port=29540
for step in "$@"; do
  envs=""; body=$step
  case $step in *@*) envs=${step%%@*}; body=${step#*@};; esac
  IFS=: read -r kind a b <<< "$body"
  name=$(echo "$step" | tr -c 'A-Za-z0-9_.=-' '_')
  run() { env $envs timeout -k 10 600 "$@" > $out/$name.json 2> $out/$name.err; }
  case $kind in
    test) env $envs timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$a" --timeout 400 \
            --timeout-method thread > $out/$name.log 2>&1 || { tail -30 $out/$name.log; exit 1; }
          tail -1 $out/$name.log; continue;;
    bench) run python bench.py --config $a --steps 50 --warmup 5 || exit $?;;
    sim) run python bench.py --config $a --simulate-world $b --steps 100 --warmup 10 || exit $?
         python3 -c "import json; r=json.load(open('$out/$name.json')); print('$step', 'max', round(r['max_rank_ms_per_step']*1e3,2), 'us', [round(x['ms_per_step']*1e3,1) for x in r['ranks']])"
         continue;;
    prof) sim=""; [ "$b" -gt 1 ] && sim="--simulate-world $b --simulate-rank 0"
          cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
          env $envs timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$a$b -o run -- \
            python3 bench.py --config $a $sim --steps 100 --warmup 10 --no-extra --no-cpu-baseline \
            > $out/$name.json 2> $out/$name.err || exit $?
          python3 scripts/trace_table.py $out/prof_$a$b | head -20; continue;;
    rccl) port=$((port + 1))
          run python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
            --master-port $port bench.py --config $a --force-shard --steps 20 --warmup 3 --no-cpu-baseline || exit $?;;
    train) run python bench.py --train --config $a --steps 10 --warmup 2 || exit $?;;
    trainrccl) port=$((port + 1))
          run python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
            --master-port $port bench.py --train --config $a --force-shard --steps 10 --warmup 2 || exit $?;;
    *) echo "unknown step $step"; exit 2;;
  esac
  python3 scripts/bench_summary.py "$step" $out/$name.json
done
