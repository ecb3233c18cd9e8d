"""Per-kernel, per-grid mean durations from a rocprofv3 --kernel-trace csv directory."""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:56]
    d[(n, int(r["Grid_Size_X"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{n:56s} grid {g:8d} calls {len(v):6d} avg {sum(v) / len(v):9.2f} us")
