"""Where config S's fused-seg launches spend their time (profiling aid, GPU box).

Build (here):  python -m decagon_amd._build fsprof DG_FSEG_PROF=1   -> decagon_amd/lib/var_fsprof.so
Run (box):     python scripts/fseg_prof.py [steps]                   -> one JSON line on stdout

The profiling build stamps s_memrealtime (100 MHz, 10 ns) per wave at: start (0), target /
group found (1), segment bounds loaded (2, layer 2 only), the wave's relation sum done (3),
the workgroup's first barrier (4), groups normalised (5), row stored (6), plus the XCC id (7)
— with s_waitcnt before stamps 2, 3 and 6, so each stamp marks completed loads.  The forward
(both layers + decoder) runs `steps` times back to back in one hipGraph, as bench.py times it;
the buffers then hold the last step's two launches.  Reported per launch: its span (first wave
start to last row stored), the spread of workgroup start times (dispatch), and the median /
90th-percentile duration of each phase over the waves that own a relation.
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("DG_LIB", str(ROOT / "decagon_amd" / "lib" / "var_fsprof.so"))
sys.path.insert(0, str(ROOT))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402


def main():
    import torch

    import bench
    from decagon_amd import _lib

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = _lib.load()
    lib.dg_fseg_prof_copy.restype = ctypes.c_int64
    lib.dg_fseg_prof_copy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64]
    args = bench.parse(["--config", "S"])
    dev = torch.device("cuda", 0)
    graph, shard, _, _ = bench.build_workload("S", 0, 1, False)
    plan, dg = bench.make_plan(args, graph, shard, dev)
    dec = bench.Decoder(graph, plan, dev, 0)
    stream = torch.cuda.Stream(dev)

    def step():
        plan.run()
        dec()

    with torch.cuda.stream(stream):
        for _ in range(3):
            step()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            for _ in range(steps):
                step()
        for _ in range(3):
            g.replay()
        stream.synchronize()
    from decagon_amd import kernels
    forms = sorted({type(l).__name__ for L in plan.spmm_launches for l in L})
    out = {"steps_per_graph": steps, "launch_forms": forms,
           "note": "the table form (PreparedFusedTab = gcn_tab_kernel) has no search or bounds phase: "
                   "'search' is its first round trip (descriptor + first 64 pairs); in layer 2 'bounds' "
                   "is its gathers (first pairs in registers -> aggregate folded) and 'relation' the "
                   "projection by W2_k (W slice load, LDS hand-off, FMAs, butterfly); 'normalise' is the "
                   "finishing wave's group sums, norms and cross-group sum (no second barrier since round 6)",
           "launches": {}}
    bufs = {}
    for proj in (0, 1):
        buf = np.zeros((4096, 16, 8), np.uint64)
        n = lib.dg_fseg_prof_copy(proj, buf.ctypes.data, 4096)
        assert n > 0
        bufs[proj] = buf
    t_ref = min(int(b[b[:, :, 0] > 0][:, 0].min()) for b in bufs.values())
    for proj, buf in bufs.items():
        live = buf[:, :, 0] > 0
        blocks = np.nonzero(live.any(1))[0]
        st = buf.astype(np.int64)
        t0 = np.where(live, st[:, :, 0], np.iinfo(np.int64).max)
        wg_start = t0.min(1)[blocks]
        wg_end = st[:, :, 6].max(1)[blocks]
        k0, k1 = wg_start.min(), wg_end.max()
        ph = {}
        names = ["search", "bounds", "relation", "barrier1", "normalise", "store"]
        pairs = [(0, 1), (1, 2), (2 if proj else 1, 3), (3, 4), (4, 5), (5, 6)]
        for nm, (a, b) in zip(names, pairs):
            if nm == "bounds" and not proj:
                continue
            m = live & (st[:, :, b] > 0) & (st[:, :, a] > 0)
            d = (st[:, :, b] - st[:, :, a])[m] * 10.0 / 1e3  # us
            ph[nm] = {"median_us": float(np.median(d)), "p90_us": float(np.percentile(d, 90)),
                      "max_us": float(d.max())}
        xcc = buf[blocks, 0, 7].astype(int)
        out["launches"]["layer2 (reassociated)" if proj else "layer1"] = {
            "workgroups": int(len(blocks)),
            "start_us_after_first_layer1_wave": (k0 - t_ref) * 0.01,
            "span_us": (k1 - k0) * 0.01,
            "wg_start_spread_us": {"p50": float(np.percentile(wg_start - k0, 50)) * 0.01,
                                   "p90": float(np.percentile(wg_start - k0, 90)) * 0.01,
                                   "max": float((wg_start - k0).max()) * 0.01},
            "wg_duration_us": {"p50": float(np.percentile(wg_end - wg_start, 50)) * 0.01,
                               "p90": float(np.percentile(wg_end - wg_start, 90)) * 0.01,
                               "max": float((wg_end - wg_start).max()) * 0.01},
            "last_wg_start_to_end_us": float((k1 - wg_start.max()) * 0.01),
            "phases": ph,
            "workgroups_per_xcc": np.bincount(xcc, minlength=8).tolist(),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
