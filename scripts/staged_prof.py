"""Cycle breakdown of dg_spmm_staged_f32 on config P (profiling aid).

Build (here):   python scripts/staged_prof.py build [NAME -DFLAG ...]
                                 -> scripts/prof_build/libdecagon_hip_prof[_NAME].so
Run (GPU box):  python scripts/staged_prof.py run [bins]   (DG_PROF_LIB=<.so> for a named build)
Per wave of each workgroup: cycles at the relation barrier, filling the other buffers and
issuing the next prefetch, reading the relation tables, gathering, and accumulating; printed
per relation as means over blocks, one column per wave, for layer 1 and layer 2.
"""
import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "scripts" / "prof_build" / "libdecagon_hip_prof.so"


def build():
    sys.path.insert(0, str(ROOT))
    from decagon_amd import _build
    OUT.parent.mkdir(exist_ok=True)
    out, flags = OUT, []
    if len(sys.argv) > 2:
        out = OUT.with_name(f"libdecagon_hip_prof_{sys.argv[2]}.so")
        flags = sys.argv[3:]
    cmd = [_build.hipcc(), "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared", "-DDG_STAGED_PROF",
           *flags, f"-I{ROOT / 'include'}", f"-I{_build.CSRC}", "-o", str(out), *map(str, _build._sources())]
    subprocess.run(cmd, check=True)


def run():
    os.environ["DG_LIB"] = os.environ.get("DG_PROF_LIB", str(OUT))
    os.environ["DG_STAGED"] = "1"
    if len(sys.argv) > 2:
        os.environ["DG_STAGED_BINS"] = sys.argv[2]
    sys.path.insert(0, str(ROOT))
    import numpy as np
    import torch

    import bench
    from decagon_amd import _lib, kernels

    lib = _lib.load()
    lib.dg_staged_prof_copy.restype = ctypes.c_int64
    lib.dg_staged_prof_copy.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
    sys.argv = [sys.argv[0], "--config", "P"]
    args = bench.parse()
    graph, shard, _, _ = bench.build_workload("P", 0, 1, False)
    plan, dg = bench.make_plan(args, graph, shard, torch.device("cuda", 0))
    l1, l2 = plan.spmm_launches
    clock = 100e6  # s_memtime/readcyclecounter ticks (shader clock): report raw and per stage
    for name, launches in (("layer1", l1), ("layer2", l2)):
        st = [x for x in launches if isinstance(x, kernels.PreparedStaged)]
        for rep in range(3):
            st[0]()
        torch.cuda.synchronize()
        buf = np.zeros((1 << 12, 16, 6), np.uint64)   # [block][wave][slot]
        n = lib.dg_staged_prof_copy(buf.ctypes.data, 1 << 12)
        b = buf[:n]
        b = b[b[:, 0, 5] > 0].astype(np.float64)
        nk = b[:, 0, 5].mean()
        tot = b[:, 0, :5].sum(1)
        print(f"{name}: blocks {len(b)}  relations/block {nk:.1f}  cycles/block mean {tot.mean():.0f} max {tot.max():.0f}")
        names = ("barrier", "put", "tables", "gather", "accum")
        print("   per relation, mean over blocks; columns = waves 0..15")
        for j, nm in enumerate(names):
            row = " ".join(f"{v:6.0f}" for v in b[:, :, j].mean(0) / nk)
            print(f"   {nm:8s} {row}")

if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
