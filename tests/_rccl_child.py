"""Child of tests/test_gpu_rccl.py, launched in a FRESH process under
`torch.distributed.run --nproc-per-node 1` (no GPU call happens in this process before the
launcher starts it): the sharded forward exactly as `bench.py --force-shard` builds it —
bench.build_workload / make_plan, collectives issued straight to RCCL through
decagon_amd.rccl.RcclComm — with every step (kernels AND collectives) captured into one
hipGraph and replayed, as bench.timed_steps does at N > 1 over RCCL.

Both sharded forms run: config S's weak-scaling row-split plan (two all-gathers per step) and
the scaled-down config P (proteins row-split, drug×drug relations in the staged kernel: one
all-reduce + one all-gather per layer).  After the replays the process sleeps past
ProcessGroupNCCL's watchdog period (the abort this guards against — hipErrorCapturedEvent on a
captured collective — came from that thread), then checks hidden1 / embeddings against the
float64 oracle (oracle/decagon_oracle.py, restating decagon/deep/layers.py:85-118 and
model.py:64-88) at 1e-4 and prints one line `RCCL_CHILD_OK {...}`.
"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    import torch
    import torch.distributed as dist

    import bench
    from decagon_amd import rccl, synthetic
    from decagon_amd.sharding import RelationShard
    from test_gpu_sharded import _oracle, _weights

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    comm = rccl.world_comm()
    args = bench.parse(["--force-shard", "--steps", "10", "--warmup", "2"])
    report = {}
    for kind in ("S-rows", "P-small"):
        if kind == "S-rows":
            graph, shard, _, _ = bench.build_workload("S", rank, world, True, "nccl")
        else:
            graph = synthetic.make_P(seed=3, n_proteins=1500, n_drugs=150, n_side_effects=60, ppi_edges=12000,
                                     target_edges=1200)
            shard = RelationShard.split(graph.edge_types, graph.n_nodes,
                                        {et: [len(c[1]) for c in rels] for et, rels in graph.adj.items()},
                                        rank, world, *comm.collectives(), row_split_min=1000)
        plan, dg = bench.make_plan(args, graph, shard, dev)
        # the test's weights (bench draws its own glorot stacks): loaded in place
        w1, w2 = _weights(graph, 5)
        for et in graph.edge_types:
            plan.w1.stacks[et].copy_(torch.from_numpy(w1[et]))
            plan.w2.stacks[et].copy_(torch.from_numpy(w2[et]))
        stream = torch.cuda.Stream(dev)
        with torch.cuda.stream(stream):
            plan.run()  # eager warm-up (RCCL's first calls set up its channels)
            stream.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream, capture_error_mode="thread_local"):
                for _ in range(3):
                    plan.run()
            for h in list(plan.hidden1.values()) + list(plan.embeddings.values()):
                h.fill_(float("nan"))
            for _ in range(4):
                g.replay()
            stream.synchronize()
        dist.barrier()
        time.sleep(float(os.environ.get("DG_CHILD_WATCHDOG_S", "3")))
        torch.cuda.synchronize()
        h1, emb = _oracle(kind, graph)
        errs = {}
        for t in (0, 1):
            for name, got, want in (("hidden1", plan.hidden1[t], h1[t]), ("embeddings", plan.embeddings[t], emb[t])):
                a = got.cpu().numpy().astype(np.float64)
                errs[f"{name}_{t}"] = float(np.max(np.abs(a - want)) / np.max(np.abs(want)))
        bad = {k: v for k, v in errs.items() if not v <= 1e-4}
        if bad:
            raise SystemExit(f"{kind}: parity failed {bad}")
        report[kind] = {"parallelism": plan.parallelism("nccl"), "max_rel_err": max(errs.values())}
        del plan, dg, g
    comm.destroy()
    rccl._COMM = None
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL_CHILD_OK " + json.dumps(report), flush=True)


if __name__ == "__main__":
    main()
