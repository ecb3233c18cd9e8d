"""One step's kernel timeline (start/end relative to the end of the previous step's last
kernel) from a rocprofv3 --kernel-trace directory:
    python3 scripts/timeline.py <dir> [last-kernel-substring] [max kernels]"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
anchor = sys.argv[2] if len(sys.argv) > 2 else "decoder_hinge"
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
i0 = idx[len(idx) // 2]
t0 = int(rows[i0]["End_Timestamp"])
for r in rows[i0 + 1:i0 + int(sys.argv[3] if len(sys.argv) > 3 else 16)]:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:34]
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{n:36s} grid {int(r['Grid_Size_X']):8d} start {s:8.1f} end {e:8.1f} dur {e - s:7.1f}")
    if "decoder_hinge" in r["Kernel_Name"]:
        break
