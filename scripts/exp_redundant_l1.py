"""Config S at N = 8, VERDICT r5 item 1 (a): what layer 1 computed REDUNDANTLY over all 8 relation
sets would cost each rank (profiling aid, GPU box).

Every rank would then hold every hidden1 row without an exchange: layer 1 over the whole 8-set
graph (8 × 105,974 nnz, every row) on one GPU, in the launch forms the one-GPU plan picks for
it, against the row-split rank share it would replace (seg launch + finishing epilogue + the
exchange).  Run (box):  python scripts/exp_redundant_l1.py [N]   -> one JSON object.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import torch

    import bench
    from decagon_amd import synthetic

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    graph = synthetic.replicate_sets(synthetic.load_S(), n)
    args = bench.parse(["--config", "S"])
    plan, dg = bench.make_plan(args, graph, None, dev)
    out = {"sets": n, "nnz_per_layer": int(dg.total_nnz),
           "layer1_launches": [type(l).__name__ for l in plan._layer1.launches],
           "layer1_epilogues": [type(l).__name__ for l in plan._layer1.epilogues],
           "layer2_launches": [type(l).__name__ for l in plan._layer2.launches]}
    plan.run()
    torch.cuda.synchronize()
    out["layer1_us"] = bench.time_kernel(plan._layer1.run, 50, stream) * 1e3
    out["layer1_spmm_us"] = bench.time_kernel(plan._layer1.run_spmm, 50, stream) * 1e3
    out["forward_us"] = bench.time_kernel(plan.run, 50, stream) * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
