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
        if by_grid:  # grid / workgroup / LDS bytes: the two layers differ in at least one
            key = key + ("%s/%s/%s" % (r.get("Grid_Size", 0) or 0, r.get("Workgroup_Size", 0) or 0,
                                       r.get("LDS_Block_Size", 0) or 0),)
        acc[key].append(float(r["Counter_Value"]))
    return acc


def launches(d):
    """Per-launch rows of a --kernel-trace directory, keyed by (kernel, grid, workgroup, LDS
    bytes) — the two layers launch one kernel with different grids or LDS sizes — each split
    into launches that ran alone and launches that overlapped another kernel (config P runs
    the staged and the protein-row launches concurrently; bench.py times each layer-1 launch
    alone, so the "alone" mean is the number its roofline uses)."""
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        return {}
    rows = []
    for r in csv.DictReader(open(f[0])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                     int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0),
                     int(r.get("LDS_Block_Size", 0) or 0)))
    rows.sort()
    out = {}
    end_max = 0  # latest end among earlier-starting launches
    for i, (s, e, k, g, w, lds) in enumerate(rows):
        overl = end_max > s or (i + 1 < len(rows) and rows[i + 1][0] < e)
        end_max = max(end_max, e)
        rec = out.setdefault((k, g, w, lds), {"alone": [], "overlapped": []})
        rec["overlapped" if overl else "alone"].append((e - s) / 1e3)
    return out


def launch_table(d, top=12):
    """Markdown table: per (kernel, grid, workgroup, LDS) launch class, mean µs alone / overlapped."""
    ls = launches(d)
    if not ls:
        return
    tot = {key: sum(v["alone"]) + sum(v["overlapped"]) for key, v in ls.items()}
    print("Per launch class (from the kernel trace; alone = no other kernel overlapped it):\n")
    print("| kernel | grid | wg | LDS B | alone: n, mean us | overlapped: n, mean us |")
    print("|---|---|---|---|---|---|")
    for key in sorted(tot, key=lambda x: -tot[x])[:top]:
        k, g, w, lds = key
        v = ls[key]
        a = f"{len(v['alone'])}, {sum(v['alone']) / len(v['alone']):.2f}" if v["alone"] else "0, -"
        o = f"{len(v['overlapped'])}, {sum(v['overlapped']) / len(v['overlapped']):.2f}" if v["overlapped"] else "0, -"
        print(f"| `{k}` | {g} | {w} | {lds} | {a} | {o} |")
    print()


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
        for (k, g, w, lds), v in launches(os.path.join(root, f"{cfg}_trace")).items():
            kern.setdefault(k, {}).setdefault("by_launch", {})[f"{g}/{w}/{lds}"] = {
                "alone_n": len(v["alone"]), "overlapped_n": len(v["overlapped"]),
                "alone_avg_us": sum(v["alone"]) / len(v["alone"]) if v["alone"] else None,
                "overlapped_avg_us": sum(v["overlapped"]) / len(v["overlapped"]) if v["overlapped"] else None}
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
            launch_table(os.path.join(root, f"{cfg}_trace"))
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
        launch_table(os.path.join(root, f"{cfg}_trace"))
    lds_table(root)
    config_d(root)
    rank_share(root)


def rank_share(root):
    """Rank 0's share of the 8-GPU step on one GPU (bench.py --simulate-world 8, the
    collectives as no-ops): kernel-trace stats of configs S and P."""
    for cfg in ("S8", "P8"):
        st = stats(os.path.join(root, f"{cfg}_trace"))
        if not st:
            continue
        print(f"## config {cfg[0]} at N = 8: rank 0's share on one GPU (--simulate-world 8 --simulate-rank 0)\n")
        bj = os.path.join(root, f"{cfg}_bench.json")
        if os.path.exists(bj):
            try:
                rec = json.loads(open(bj).read().strip().splitlines()[-1])
                print(f"{rec['max_rank_ms_per_step']*1e3:.1f} us/step under the profiler\n")
            except Exception:
                pass
        print("| kernel | calls | avg us | total % |")
        print("|---|---|---|---|")
        for r in st[:12]:
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                  f"{float(r['Percentage']):.1f} |")
        print()


def lds_table(root):
    """Config P: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per launch class of the LDS kernels."""
    c = pmc(os.path.join(root, "P_LDS"), by_grid=True)
    if not c:
        return
    print("## config P: LDS bank conflicts (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE)\n")
    print("| kernel | grid/wg/LDS | launches | conflict cycles | LDS active cycles | ratio |")
    print("|---|---|---|---|---|---|")
    for (k, ctr, cls), v in sorted(c.items()):
        if ctr != "SQ_LDS_BANK_CONFLICT":
            continue
        act = c.get((k, "SQ_LDS_IDX_ACTIVE", cls), [])
        if not act or sum(act) == 0:
            continue
        print(f"| `{k}` | {cls} | {len(v)} | {sum(v) / len(v):.4g} | {sum(act) / len(act):.4g} | "
              f"{sum(v) / sum(act):.3f} |")
    print()


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
