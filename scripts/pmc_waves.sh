cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for set in "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | cut -d' ' -f1)
  DG_STAGED=1 timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc/$tag -o run -- python3 bench.py --config P --no-graph --steps 2 --warmup 1 --kernel-reps 1 --no-cpu-baseline > /dev/null 2> gpurun_out/pmc/$tag.log || echo "pmc $tag failed"
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
