"""Where config S's decoder launch (dg_decoder_hinge_f32) spends its time (profiling aid).

Build (here):  python -m decagon_amd._build decprof DG_DEC_PROF=1   -> decagon_amd/lib/var_decprof.so
Run (box):     python scripts/dec_prof.py [steps]                   -> one JSON object on stdout

Stamps (s_memrealtime, 10 ns; each after an s_waitcnt, so it marks completed loads) per wave:
0 start, 1 indices / negative draws landed, 2 the tile's rows and parameters landed, 3 MFMA
chain + products, 4 reduce-scatter, 5 the block's ticket returned, 6 loss stored (last block).
The forward (both layers + decoder) runs `steps` times in one hipGraph as bench.py times it.
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("DG_LIB", str(ROOT / "decagon_amd" / "lib" / "var_decprof.so"))
sys.path.insert(0, str(ROOT))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402


def main():
    import torch

    import bench
    from decagon_amd import _lib

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = _lib.load()
    lib.dg_dec_prof_copy.restype = ctypes.c_int64
    lib.dg_dec_prof_copy.argtypes = [ctypes.c_void_p]
    args = bench.parse(["--config", "S"])
    dev = torch.device("cuda", 0)
    graph, shard, _, _ = bench.build_workload("S", 0, 1, False)
    plan, _ = bench.make_plan(args, graph, shard, dev)
    dec = bench.Decoder(graph, plan, dev, 0)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        for _ in range(3):
            plan.run()
            dec()
        stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
            for _ in range(steps):
                plan.run()
                dec()
        for _ in range(3):
            g.replay()
        stream.synchronize()
    buf = np.zeros((256, 2, 8), np.uint64)
    assert lib.dg_dec_prof_copy(buf.ctypes.data) > 0
    st = buf.astype(np.int64)
    live = st[:, :, 0] > 0
    blocks = np.nonzero(live.any(1))[0]
    st = st[blocks]
    k0 = st[:, :, 0].min()
    names = ["indices", "rows", "mfma", "reduce", "hinge+ticket"]
    out = {"blocks": int(len(blocks)), "span_us": float((st[:, :, 5].max() - k0) * 0.01),
           "last_block_loss_us_after_start": float((st[:, :, 6].max() - k0) * 0.01),
           "wave_start_spread_us": float((st[:, :, 0].max() - k0) * 0.01), "phases": {}}
    for j, nm in enumerate(names):
        d = (st[:, :, j + 1] - st[:, :, j]).ravel() * 0.01
        out["phases"][nm] = {"median_us": float(np.median(d)), "max_us": float(d.max())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
