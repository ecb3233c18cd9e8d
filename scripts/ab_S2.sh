# Config S per-launch times for every variant build under scripts/prof_build/ and a few env knobs.
set -o pipefail
out=gpurun_out/${1:-abS2}; mkdir -p $out
timeout -k 10 600 python scripts/variants.py run scripts/s_times.py > $out/variants.jsonl 2> $out/variants.err || exit $?
for w in 1 4; do DG_WPG=$w timeout -k 10 120 python scripts/s_times.py >> $out/variants.jsonl 2>> $out/variants.err || exit $?; done
cat $out/variants.jsonl
