# Config 5's scorer under PMC passes (one pass per counter group, rocprofv3 does not split):
# wave-cycle buckets and MFMA busy, then the TA / TD busy counters — what bounds the kernel.
# Usage on the box: [DG_LIB=<variant .so>] bash scripts/d_pmc.sh <tag>
set -o pipefail
tag=${1:-dpmc}
out=gpurun_out/$tag; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rocprofv3 -L > $out/counters.txt 2>&1 || true
grep -oE "^[[:space:]]*(TA|TD|TCP)_[A-Z_]+(BUSY|STALL)[A-Za-z_]*" $out/counters.txt | sort -u | head -40
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $out/$name -o run -- \
    python3 bench.py --config D --no-graph --steps 3 --warmup 1 --kernel-reps 3 > /dev/null 2> $out/$name.log
  echo "$name rc=$?"
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS
run ta TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum
run td TD_TD_BUSY_sum TD_LOAD_WAVEFRONTS_sum
run lds SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA
python3 - $out <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "cs16" in r["Kernel_Name"] or "slot_score" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), "mean %.6g" % (sum(v) / len(v)))
PY
