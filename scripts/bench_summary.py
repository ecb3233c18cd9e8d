"""One line per bench JSON record: step time, dominant-kernel time and fraction, and the P /
D blocks when present (scripts/ab.sh)."""
import json
import sys


def line(tag, d):
    out = [tag]
    if "ms_per_step" in d:
        out.append(f"step {d['ms_per_step'] * 1e3:.2f} us")
    rf = d.get("roofline") or {}
    if rf.get("kernel_ms"):
        out.append(f"kernel {rf['kernel_ms'] * 1e3:.2f} us frac {rf.get('frac', 0):.4f}")
    if "spmm_layer2_ms" in d:
        out.append(f"L2 {d['spmm_layer2_ms'] * 1e3:.2f} us")
    if "max_rank_ms_per_step" in d:  # bench.py --simulate-world
        out.append(f"max rank step {d['max_rank_ms_per_step'] * 1e3:.2f} us")
        r = max(d["ranks"], key=lambda x: x["ms_per_step"])
        out.append(f"its layer-1 / layer-2 SpMM {r['layer1_spmm_ms'] * 1e3:.2f} / {r['layer2_spmm_ms'] * 1e3:.2f} us")
    return " | ".join(out)


tag, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
print(line(tag, d))
for k in ("P", "D"):
    if k in d:
        print(line(f"{tag}.{k}", d[k]))
