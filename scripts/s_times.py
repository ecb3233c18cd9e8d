"""Per-launch device times of config S's forward step (profiling aid):
    python scripts/s_times.py [--reps N]        (DG_LIB=<variant .so> to time a variant build)
Prints one JSON line: each launch of the step alone (HIP events over a hipGraph of N launches)
and the whole step (hipGraph of 10 steps)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import argparse

    import torch

    import bench

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--config", default="S")
    a = ap.parse_args()
    args = bench.parse(["--config", a.config])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    graph, shard, _, _ = bench.build_workload(a.config, 0, 1, False)
    plan, dg = bench.make_plan(args, graph, None, dev)
    dec = bench.Decoder(graph, plan, dev, 0)
    st = torch.cuda.Stream(dev)
    out = {"lib": os.environ.get("DG_LIB", "default")}
    out["layer1_us"] = bench.time_kernel(plan._layer1.run, a.reps, st) * 1e3
    out["layer2_us"] = bench.time_kernel(plan._layer2.run, a.reps, st) * 1e3
    out["decoder_us"] = bench.time_kernel(dec, a.reps, st) * 1e3

    def step():
        plan.run()
        dec()
    out["step_us"] = bench.time_kernel(step, max(10, a.reps // 4), st) * 1e3
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()
