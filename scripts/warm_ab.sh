# Untimed replays after capture (DG_WARM_REPLAYS) against the timed region's wall clock and the
# device span of the same replays (bench's timing_split), for config S and config 5.
# Usage on the box: bash scripts/warm_ab.sh <tag>
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for rep in 1 2; do
  for w in 1 2 4; do
    for cfg in S D; do
      if [ $cfg = S ]; then a="--steps 20 --warmup 5"; else a="--config D --steps 100 --warmup 10"; fi
      DG_WARM_REPLAYS=$w timeout -k 10 300 python bench.py $a --no-extra --no-cpu-baseline > $out/${cfg}_w${w}_$rep.json 2> $out/${cfg}_w${w}_$rep.err || exit $?
      python -c "import json,sys; r=json.load(open(sys.argv[1])); t=r['timing_split']; print(sys.argv[2], 'wall %.2f us device %.2f us enqueue %.1f us' % (1e3*r['ms_per_step'], 1e3*t['device_ms_per_step'], 1e3*t['host_enqueue_ms']))" $out/${cfg}_w${w}_$rep.json "$cfg warm=$w"
    done
  done
done
