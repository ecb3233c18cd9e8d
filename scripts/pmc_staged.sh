# LDS counters of the staged kernel on config P (profiling aid)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
for set in ${PMC_SETS:-"SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" "SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"}; do
  tag=$(echo $set | cut -d' ' -f1)
  DG_STAGED=1 timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/$tag -o run -- \
    python3 bench.py --config P --no-graph --steps 2 --warmup 1 --kernel-reps 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc/$tag.log || echo "pmc $tag failed"
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "staged" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, len(v), "mean %.4g" % (sum(v) / len(v)))
PY
