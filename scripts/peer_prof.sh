# Loopback rehearsal of an 8-GPU rank share (config S or P) under rocprofv3 (kernel trace +
# stats): where the peer exchange's time goes inside the finishing launches.
# Usage on the box: bash scripts/peer_prof.sh <tag> <exchange> [S|P]
set -o pipefail
tag=${1:-peerprof}
ex=${2:-peer}
cfg=${3:-S}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$ex -o run -- python3 bench.py --config $cfg \
    --simulate-world 8 --simulate-rank 0 --exchange $ex --steps 100 --warmup 10 > $out/prof_$ex.json 2> $out/prof_$ex.err \
    || { tail -5 $out/prof_$ex.err; exit 1; }
f=$(find $out/prof_$ex -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print('%-80s %6s calls  avg %8.2f us' % (r['Name'][:80], r['Calls'], float(r['AverageNs'])/1e3))
" $f
