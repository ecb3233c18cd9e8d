"""CPU: the multi-GPU path's host logic and its collective, with world_size-2 gloo.

The sharded forward computes, per rank, the pre-normalisation group sums of its own
relations and sum-all-reduces them before the L2 normalisation (layers.py:92-93).  Here
each rank computes its local sums with the float64 oracle (the checker) and reduces them
through the product's collective wrapper (decagon_amd.sharding.torch_allreduce) over gloo;
the result must equal the single-process sum over all relations.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from decagon_amd.sharding import RelationShard, lpt_assign


def test_lpt_balances_and_covers():
    rng = np.random.default_rng(0)
    costs = rng.integers(1, 1000, 200).tolist() + [50000, 40000]
    owner = lpt_assign(costs, 8)
    loads = np.zeros(8)
    for c, r in zip(costs, owner):
        loads[r] += c
    assert sorted(set(owner)) == list(range(8))
    assert loads.max() <= max(costs) + loads.mean()  # LPT bound
    assert lpt_assign(costs, 8) == owner  # deterministic


def test_relation_shard_lpt_partitions_every_relation():
    et = {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 1928}
    rng = np.random.default_rng(1)
    cost = {k: rng.integers(500, 30000, v).tolist() for k, v in et.items()}
    cost[(0, 0)] = [1_450_000, 1_450_000]
    seen = {k: [] for k in et}
    for r in range(8):
        s = RelationShard.lpt(et, cost, r, 8)
        for k, v in s.local.items():
            seen[k] += v
    for k, v in et.items():
        assert sorted(seen[k]) == list(range(v))


def test_weak_sets_shard():
    et, n = {(0, 0): 8, (0, 1): 4, (1, 0): 4, (1, 1): 24}, {0: 500, 1: 400}
    seen = {0: [], 1: []}
    for r in range(4):
        s = RelationShard.weak_sets(et, n, r, 4, form="seg")
        assert s.seg_rows and not s.fused_rows
        assert s.chunks == {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 6}  # one chunk per relation set
        assert s.local == {k: list(range(v)) for k, v in et.items()}    # every relation, on a row block
        for t in (0, 1):
            a, b, blk = s.row_block[t]
            assert blk == -(-n[t] // 4)
            seen[t] += list(range(a, b))
    assert seen == {0: list(range(500)), 1: list(range(400))}
    f = RelationShard.weak_sets(et, n, 1, 4, form="fused")
    assert f.fused_rows and f.chunks == et
    with pytest.raises(ValueError):
        RelationShard.weak_sets({(0, 0): 3}, {0: 10}, 0, 2, form="seg")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from decagon_amd.sharding import RelationShard, torch_allreduce
    from decagon_amd.synthetic import load_S
    from oracle import decagon_oracle as orc

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = load_S()
    nnz = {et: [len(c[1]) for c in rels] for et, rels in g.adj.items()}
    shard = RelationShard.lpt(g.edge_types, nnz, rank, world, torch_allreduce())
    rng = np.random.default_rng(7)
    X = {et: rng.standard_normal((K, g.n_nodes[et[1]], 64)) for et, K in g.edge_types.items()}
    flat = []
    for et in g.edge_types:
        s = np.zeros((g.n_nodes[et[0]], 64))
        for k in shard.local[et]:
            s += orc.sparse_dense_matmul(g.adj[et][k], X[et][k])
        flat.append(s.ravel())
    buf = torch.from_numpy(np.concatenate(flat))
    shard.allreduce(buf)
    q.put((rank, buf.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_rank_group_sums_equal_single_device():
    from decagon_amd.synthetic import load_S
    from oracle import decagon_oracle as orc

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = load_S()
    rng = np.random.default_rng(7)
    X = {et: rng.standard_normal((K, g.n_nodes[et[1]], 64)) for et, K in g.edge_types.items()}
    want = np.concatenate([sum(orc.sparse_dense_matmul(g.adj[et][k], X[et][k]) for k in range(K)).ravel()
                           for et, K in g.edge_types.items()])
    for r in (0, 1):
        assert np.allclose(res[r], want, rtol=1e-12, atol=1e-12)


# ---------------------------------------------------------------- row-split + relation shard
def test_row_blocks_cover_rows_once():
    from decagon_amd.sharding import row_block

    for n, world in ((19085, 8), (19085, 3), (1500, 2), (10, 4)):
        seen = np.zeros(n, int)
        for r in range(world):
            a, b, blk = row_block(n, r, world)
            assert blk == -(-n // world) and 0 <= b - a <= blk
            seen[a:b] += 1
        assert (seen == 1).all()


def test_split_row_splits_proteins_and_lpts_drug_relations():
    from decagon_amd.sharding import slot_range

    et = {(0, 0): 2, (0, 1): 1, (1, 0): 1, (1, 1): 1928}
    n = {0: 19085, 1: 645}
    rng = np.random.default_rng(1)
    cost = {k: rng.integers(500, 30000, v).tolist() for k, v in et.items()}
    cost[(0, 0)] = [1_450_000, 1_450_000]
    seen = {k: [] for k in et}
    for r in range(8):
        s = RelationShard.split(et, n, cost, r, 8)
        assert set(s.row_block) == {0}
        assert s.local[(0, 0)] == [0, 1] and s.local[(0, 1)] == [0]  # all relations, row block
        for k in ((1, 0), (1, 1)):
            seen[k] += s.local[k]
            assert s.local[k] == sorted(s.local[k])
        # drug-side loads balance within one relation of each other
        assert max(s.loads) - min(s.loads) <= max(cost[(1, 1)])
    for k in ((1, 0), (1, 1)):
        assert sorted(seen[k]) == list(range(et[k]))
    # config 5 slot blocks
    blocks = [slot_range(1928, r, 8) for r in range(8)]
    assert blocks[0][0] == 0 and blocks[-1][1] == 1928
    assert all(blocks[r][1] == blocks[r + 1][0] for r in range(7))
    assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1


def test_split_small_node_types_stay_relation_sharded():
    s = RelationShard.split({(0, 0): 2, (1, 1): 6}, {0: 500, 1: 400}, {(0, 0): [5, 5], (1, 1): [1] * 6}, 0, 2)
    assert s.row_block == {}
    assert len(s.local[(0, 0)]) == 1


def test_row_slice_keeps_rows_and_columns():
    import scipy.sparse as sp

    from decagon_amd.engine import row_slice
    from decagon_amd.sparse import coo_to_csr

    m = sp.random(50, 30, density=0.2, random_state=0, format="coo")
    c = coo_to_csr(np.stack([m.row, m.col], 1), m.data, m.shape)
    s = row_slice(c, 13, 37)
    dense = sp.csr_matrix((s.val, s.col, s.rowptr), shape=s.shape).toarray()
    assert s.shape == (24, 30)
    assert np.array_equal(dense, m.toarray()[13:37].astype(np.float32))


def _ag_worker(rank, world, port, q):
    import torch.distributed as dist

    from decagon_amd.sharding import row_block, torch_allgather

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, d = 11, 3
    a, b, blk = row_block(n, rank, world)
    out = torch.full((world * blk, d), -1.0)
    out[rank * blk:rank * blk + (b - a)] = torch.arange(a, b, dtype=torch.float32)[:, None]
    torch_allgather()(out, out[rank * blk:(rank + 1) * blk])
    q.put((rank, out[:n].numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_row_block_allgather_in_place():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ag_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(3):
        assert np.array_equal(res[r], np.repeat(np.arange(11, dtype=np.float32)[:, None], 3, 1))


def _fail_on_rank1(rank, world):
    if rank == 1:
        raise RuntimeError("boom")
    import torch.distributed as dist

    dist.barrier()  # would wait forever for rank 1
    return rank


def test_run_ranks_reports_a_failing_rank_at_once():
    import time

    from conftest import run_ranks

    t0 = time.time()
    with pytest.raises(AssertionError, match="boom"):
        run_ranks(_fail_on_rank1, 2, timeout=120)
    assert time.time() - t0 < 60
