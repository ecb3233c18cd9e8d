# The peer-store exchange on the one-GPU box: its -m gpu tests (ranks = processes sharing the
# GPU, IPC-mapped regions), then the loopback rehearsal of config S's N-GPU rank share with the
# exchange in it beside the RCCL-free share (collectives as no-ops).
# Usage on the box: bash scripts/peer_round.sh <tag> [N]
set -o pipefail
tag=${1:-peer}
N=${2:-8}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_peer.py -m gpu -v -x --timeout 400 --timeout-method thread \
    > $out/peer_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $out/peer_tests.log | head -30
tail -1 $out/peer_tests.log
[ $rc -eq 0 ] || exit $rc
for ex in rccl peer peer-kernel; do
    timeout -k 10 300 python bench.py --config S --simulate-world $N --exchange $ex --steps 100 --warmup 10 \
        > $out/sim_S${N}_$ex.json 2> $out/sim_S${N}_$ex.err || { tail -5 $out/sim_S${N}_$ex.err; exit 1; }
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], 'max rank us/step %.2f' % (1e3*r['max_rank_ms_per_step']), [round(1e3*x['ms_per_step'],2) for x in r['ranks']], [x.get('peer_error_word') for x in r['ranks']])" $out/sim_S${N}_$ex.json $ex
done
