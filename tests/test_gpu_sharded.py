"""GPU: the relation-sharded forward (sharding.py + ForwardPlan(allreduce=...)) on two
ranks sharing the one GPU of the test box, collectives over gloo (RCCL refuses two ranks on
one device; the 8-GPU RCCL run is the driver's).  Both ranks must end with the same
hidden1 / embeddings as the single-device fused plan.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _plan(g, shard, device):
    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights

    rng = np.random.default_rng(5)
    n = g.n_nodes
    w1 = LayerWeights({et: torch.from_numpy(
        rng.uniform(-0.1, 0.1, (K, n[et[1]], 64)).astype(np.float32)).to(device) for et, K in g.edge_types.items()})
    w2 = LayerWeights({et: torch.from_numpy(
        rng.uniform(-0.3, 0.3, (K, 64, 32)).astype(np.float32)).to(device) for et, K in g.edge_types.items()})
    csr = g.csr()
    dg = DeviceGraph(g.edge_types, csr, device, None if shard is None else shard.local)
    return ForwardPlan(dg, {0: None, 1: None}, w1, w2, 64, 32,
                       allreduce=None if shard is None else shard.allreduce)


def _worker(rank, world, port, q, chunk_small):
    import torch.distributed as dist

    from decagon_amd.sharding import RelationShard, torch_allreduce
    from decagon_amd.synthetic import load_S

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_S()
    nnz = {et: [len(c[1]) for c in rels] for et, rels in g.adj.items()}
    shard = RelationShard.lpt(g.edge_types, nnz, rank, world, torch_allreduce())
    plan = _plan(g, shard, torch.device("cuda", 0))
    plan.run()
    torch.cuda.synchronize()
    eager = (plan.hidden1[1].cpu().numpy(), plan.embeddings[0].cpu().numpy(), plan.embeddings[1].cpu().numpy())
    # the bench's N > 1 form: each compute phase captured in a hipGraph, exchanges eager
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        seq = []
        for kind, fn in plan.phases():
            if kind == "exchange":
                seq.append(fn)
                continue
            fn()
            stream.synchronize()
            gph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gph, stream=stream):
                fn()
            seq.append(gph.replay)
        for h in list(plan.hidden1.values()) + list(plan.embeddings.values()):
            h.fill_(float("nan"))
        for f in seq:
            f()
        stream.synchronize()
    graphed = (plan.hidden1[1].cpu().numpy(), plan.embeddings[0].cpu().numpy(), plan.embeddings[1].cpu().numpy())
    for x, y in zip(eager, graphed):
        assert np.array_equal(x, y), "graph-captured phases differ from the eager forward"
    q.put((rank,) + eager)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_forward_matches_single_device():
    import torch.multiprocessing as mp

    from decagon_amd.synthetic import load_S

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = load_S()
    ref = _plan(g, None, torch.device("cuda", 0))
    ref.run()
    torch.cuda.synchronize()
    want = (ref.hidden1[1].cpu().numpy(), ref.embeddings[0].cpu().numpy(), ref.embeddings[1].cpu().numpy())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, False)) for r in range(2)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(2):
        r, *arrs = q.get(timeout=240)
        got[r] = arrs
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in (0, 1):
        for a, b in zip(got[r], want):
            assert np.max(np.abs(a - b)) <= 1e-5 * np.max(np.abs(b))
