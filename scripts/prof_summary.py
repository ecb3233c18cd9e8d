"""Summarise a scripts/profile_round.sh output directory: per-kernel launch count and mean
duration (kernel-trace stats) and per-launch mean FETCH_SIZE / WRITE_SIZE (PMC passes).

    python3 scripts/prof_summary.py gpurun_out/prof_r01 > profiles/r01_summary.md
    python3 scripts/prof_summary.py gpurun_out/prof_r01 --json profiles/r01_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "(" in name else name


def stats(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        return []
    return list(csv.DictReader(open(f[0])))


def pmc(d, by_grid=False):
    """(kernel, counter) -> values per dispatch (or (kernel, counter, grid) with by_grid)."""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(list)
    if not f:
        return acc
    for r in csv.DictReader(open(f[0])):
        key = (short(r["Kernel_Name"]), r["Counter_Name"])
        if by_grid:
            key = key + (int(r.get("Grid_Size", 0) or 0),)
        acc[key].append(float(r["Counter_Value"]))
    return acc


def traffic_json(root, out):
    """Per-kernel mean FETCH_SIZE / WRITE_SIZE per launch (KiB, raw counter values) for each
    config, plus mean durations — what bench.py reads to fill roofline.traffic."""
    rec = {}
    for cfg in ("S", "P"):
        counters, grids = {}, {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            counters.update(pmc(os.path.join(root, f"{cfg}_{ctr}")))
            grids.update(pmc(os.path.join(root, f"{cfg}_{ctr}"), by_grid=True))
        kern = {}
        for (k, c), v in counters.items():
            kern.setdefault(k, {})[c.lower() + "_kib"] = sum(v) / len(v)
        for (k, c, gsz), v in grids.items():  # one kernel launched with several grids (layers)
            kern.setdefault(k, {}).setdefault("by_grid", {}).setdefault(str(gsz), {})[c.lower() + "_kib"] = sum(v) / len(v)
        for r in stats(os.path.join(root, f"{cfg}_trace")):
            kern.setdefault(short(r["Name"]), {})["avg_us"] = float(r["AverageNs"]) / 1e3
        rec[cfg] = kern
    json.dump(rec, open(out, "w"), indent=1, sort_keys=True)


def main(root):
    if len(sys.argv) > 3 and sys.argv[2] == "--json":
        traffic_json(root, sys.argv[3])
        return
    print(f"# rocprofv3 summary: {os.path.basename(root.rstrip('/'))}\n")
    for cfg in ("S", "P", "trainS", "trainP"):
        st = stats(os.path.join(root, f"{cfg}_trace"))
        if not st:
            continue
        if cfg.startswith("train"):
            bj = os.path.join(root, f"{cfg}_bench.json")
            if os.path.exists(bj):
                try:
                    rec = json.loads(open(bj).read().strip().splitlines()[-1])
                    print(f"## {cfg}: training step (bench.py --train) under the profiler\n")
                    print(f"{rec['ms_per_step']*1e3:.1f} us/step, {rec['value']:.4g} edges/s\n")
                except Exception:
                    pass
            print("| kernel | calls | avg us | total % |")
            print("|---|---|---|---|")
            for r in st[:16]:
                print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                      f"{float(r['Percentage']):.1f} |")
            print()
            continue
        bj = os.path.join(root, f"{cfg}_bench.json")
        if os.path.exists(bj):
            try:
                rec = json.loads(open(bj).read().strip().splitlines()[-1])
                print(f"## config {cfg}: bench line under the profiler\n")
                ro = rec["roofline"]
                print(f"value {rec['value']:.4g} edges/s, {rec['ms_per_step']*1e3:.1f} us/step; "
                      f"dominant kernel {ro['kernel']} {ro['kernel_ms']*1e3:.2f} us, "
                      f"{ro['algorithmic_bytes']} algorithmic B, {ro['achieved']:.0f} GB/s "
                      f"({100 * ro['frac']:.1f} % of {ro['peak']:.0f})")
                l1 = rec.get("spmm_layer1")
                if l1:
                    print(f"; whole layer-1 SpMM {l1['ms']*1e3:.2f} us, {l1['GB_s']:.0f} GB/s "
                          f"({100 * l1['frac']:.1f} %)")
                print()
            except Exception:
                pass
        counters = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            counters.update(pmc(os.path.join(root, f"{cfg}_{ctr}")))
        print(f"## config {cfg}: kernels (kernel-trace --stats)\n")
        print("| kernel | calls | avg us | total % | FETCH_SIZE/launch (raw) | WRITE_SIZE/launch (raw) |")
        print("|---|---|---|---|---|---|")
        for r in st[:14]:
            k = short(r["Name"])
            f = counters.get((k, "FETCH_SIZE"), [])
            w = counters.get((k, "WRITE_SIZE"), [])
            fs = f"{sum(f)/len(f):.1f}" if f else "-"
            ws = f"{sum(w)/len(w):.1f}" if w else "-"
            print(f"| `{k}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.1f} | {fs} | {ws} |")
        print()
    config_d(root)


def config_d(root):
    """Config 5: bench line, kernel stats and MFMA utilisation of the scorer =
    SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs × 1024 SIMDs)."""
    st = stats(os.path.join(root, "D_trace"))
    if not st:
        return
    print("## config 5 (bench.py --config D): bf16 DEDICOM scorer\n")
    bj = os.path.join(root, "D_bench.json")
    if os.path.exists(bj):
        try:
            rec = json.loads(open(bj).read().strip().splitlines()[-1])
            ro = rec["roofline"]
            print(f"value {rec['value']:.4g} pairs/s, {rec['ms_per_step']*1e3:.1f} us/step; scorer "
                  f"{ro['achieved']:.0f} {ro['unit']} ({100 * ro['frac']:.1f} % of {ro['peak']:.0f})\n")
        except Exception:
            pass
    c = pmc(os.path.join(root, "D_MFMA"))
    print("| kernel | calls | avg us | total % | MFMA busy / (GPU cycles × 1024 SIMDs) |")
    print("|---|---|---|---|---|")
    for r in st[:8]:
        k = short(r["Name"])
        busy, gui = c.get((k, "SQ_VALU_MFMA_BUSY_CYCLES"), []), c.get((k, "GRBM_GUI_ACTIVE"), [])
        util = "-"
        if busy and gui and sum(gui) > 0:
            util = f"{100 * sum(busy) / (sum(gui) / 8 * 1024):.1f} %"
        print(f"| `{k}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['Percentage']):.1f} | {util} |")
    print()


if __name__ == "__main__":
    main(sys.argv[1])
