# One-step kernel timeline of the sharded (N > 1) config-S / config-P step, rehearsed as one
# rank over RCCL on one GPU.  Usage on the box: bash scripts/tl_shard.sh <tag> [bench args]
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-tlS}; shift
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/t -o run -- \
  python3 bench.py --force-shard --no-cpu-baseline --no-extra --kernel-reps 5 --steps 20 --warmup 3 "$@" \
  > $out/bench.json 2> $out/bench.log || exit $?
python3 scripts/timeline.py $out/t decoder_hinge 40
python3 -c "import json; d=json.load(open('$out/bench.json')); print('step us', d['ms_per_step']*1e3, d['config']['launch'])"
