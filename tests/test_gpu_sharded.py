"""GPU: the sharded forward (sharding.py + ForwardPlan(shard=...)) against the float64 oracle.

Ranks share the one GPU of the test box and talk over gloo (RCCL refuses two ranks on one
device; the 8-GPU RCCL run is the driver's).  Every rank must end with the full hidden1 /
embeddings, equal to oracle/decagon_oracle.py's restatement of the reference forward
(decagon/deep/layers.py:85-118, model.py:64-88) within 1e-4 relative — for

  * config S, relations LPT-sharded;
  * config S's weak-scaling form (bench.py at N GPUs): one relation set per rank, every node
    type row-split and finished in the fused kernel, the blocks all-gathered, on 2 and 3 ranks;
  * a scaled-down config P with the proteins row-split and the drug×drug relations
    LPT-sharded into the LDS-staged kernel (configs[3]'s plan), on 2 and 3 ranks (uneven
    row blocks, a short last block);
  * config P at full size on 2 and 8 ranks (configs[3], every output row; 8 is the partition
    the driver's 8-GPU run executes: 241 staged drug×drug relations and a 2,386-row protein
    block per rank);
  * config S's weak-scaling form and the scaled-down P at 4 and 8 ranks;
  * h1 == h2 on a row-split graph (each layer keeps its own padded output).

Each is run eagerly and as the bench's N > 1 form (each compute phase captured in a
hipGraph, the collectives eager between replays).
"""
import numpy as np
import pytest

from conftest import rel_err, run_ranks

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
TOL = 1e-4


def _weights(g, seed, s1=0.1, s2=0.3, h2=32):
    rng = np.random.default_rng(seed)
    n = g.n_nodes
    w1 = {et: rng.uniform(-s1, s1, (K, n[et[1]], 64)).astype(np.float32) for et, K in g.edge_types.items()}
    w2 = {et: rng.uniform(-s2, s2, (K, 64, h2)).astype(np.float32) for et, K in g.edge_types.items()}
    return w1, w2


def _graph(kind, world=1):
    from decagon_amd import synthetic

    if kind == "S":
        return synthetic.load_S()
    if kind in ("S-rows", "S-rows-fused"):
        return synthetic.replicate_sets(synthetic.load_S(), world)
    if kind == "P-small":
        return synthetic.make_P(seed=3, n_proteins=1500, n_drugs=150, n_side_effects=60, ppi_edges=12000,
                                target_edges=1200)
    return synthetic.make_P(seed=0)


def _shard(kind, g, rank, world):
    from decagon_amd.sharding import RelationShard, torch_allgather, torch_allreduce

    nnz = {et: [len(c[1]) for c in rels] for et, rels in g.adj.items()}
    if kind == "S":
        return RelationShard.lpt(g.edge_types, nnz, rank, world, torch_allreduce())
    if kind in ("S-rows", "S-rows-fused"):
        return RelationShard.weak_sets(g.edge_types, g.n_nodes, rank, world, torch_allreduce(), torch_allgather(),
                                       form="fused" if kind == "S-rows-fused" else "seg")
    if kind == "P":  # the driver's partition (bench.py): proteins row-split, drug×drug LPT
        return RelationShard.polypharmacy(g, rank, world, collectives=(torch_allreduce(), torch_allgather()))
    # P-small: at 3 and 8 ranks the drug-target relation dealt by rows as well (RelationShard.dealt)
    return RelationShard.split(g.edge_types, g.n_nodes, nnz, rank, world, torch_allreduce(), torch_allgather(),
                               row_split_min=1000, deal_rows=[(1, 0)] if world in (3, 8) else ())


def _rank(rank, world, kind, h2=32):
    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights

    dev = torch.device("cuda", 0)
    g = _graph(kind, world)
    shard = _shard(kind, g, rank, world)
    w1, w2 = _weights(g, 5, h2=h2)
    dg = DeviceGraph(g.edge_types, shard.local_csr(g.csr()), dev, shard.local, row_block=shard.row_block,
                     chunk=shard.chunks, segments=shard.seg_rows)
    plan = ForwardPlan(dg, {0: None, 1: None},
                       LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w1.items()}),
                       LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w2.items()}), 64, h2,
                       shard=shard)
    from decagon_amd import engine, kernels

    info = {"row_split": sorted(shard.row_block), "dealt": sorted(shard.dealt), "staged": dg.groups[(1, 1)].staged,
            "local": {et: len(v) for et, v in shard.local.items()}, "fused": sorted(plan.fused),
            "seg": plan.seg_mode, "gemms": len(plan._gemm2)}
    plan.run()
    torch.cuda.synchronize()

    def grab(p=plan):
        return ({t: p.hidden1[t].cpu().numpy() for t in (0, 1)},
                {t: p.embeddings[t].cpu().numpy() for t in (0, 1)})

    eager = grab()
    # the bench's N > 1 form: each compute phase captured in a hipGraph, exchanges eager
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        seq = []
        for kind_, fn in plan.phases():
            if kind_ == "exchange":
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
    return info, eager, grab()


def _oracle(kind, g, h2=32):
    import scipy.sparse as sp

    from oracle import decagon_oracle as orc

    w1, w2 = _weights(g, 5, h2=h2)
    if kind == "P":
        csr = {et: [sp.csr_matrix((v.astype(np.float32).astype(np.float64), (c[:, 0], c[:, 1])), shape=s)
                    for c, v, s in mats] for et, mats in g.adj.items()}
        return orc.decagon_forward_csr(g.edge_types, csr, {et: w.astype(np.float64) for et, w in w1.items()},
                                       {et: w.astype(np.float64) for et, w in w2.items()})
    n = g.n_nodes
    feats = {t: (np.stack([np.arange(n[t])] * 2, 1), np.ones(n[t]), (n[t], n[t])) for t in n}
    adj = {et: [(c, v.astype(np.float32).astype(np.float64), s) for c, v, s in mats] for et, mats in g.adj.items()}
    return orc.decagon_forward(g.edge_types, adj, feats,
                               {et: [x.astype(np.float64) for x in w] for et, w in w1.items()},
                               {et: [x.astype(np.float64) for x in w] for et, w in w2.items()})


def _check(kind, world, h2=32):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    got = run_ranks(_rank, world, (kind, h2))
    g = _graph(kind, world)
    h1, emb = _oracle(kind, g, h2)
    for r in range(world):
        info, eager, graphed = got[r]
        if kind == "S-rows":  # row blocks in dg_spmm_seg_f32, layer 2 reassociated: no projection GEMM
            assert info["row_split"] == [0, 1] and info["seg"] and not info["fused"] and info["gemms"] == 0, info
        elif kind == "S-rows-fused":
            assert info["row_split"] == [0, 1] and info["fused"] == [0, 1] and not info["seg"], info
        elif kind != "S":
            assert info["row_split"] == [0], info          # proteins row-split
            # drug×drug in the LDS-staged kernel whenever the rank holds enough of them (P-small
            # at 4 / 8 ranks leaves 30 / 15 per rank: those run in the partial-mode SpMM)
            from decagon_amd.engine import STAGED_MIN_RELS
            assert info["staged"] == (info["local"][1, 1] >= STAGED_MIN_RELS), info
        for form in (eager, graphed):
            for t in (0, 1):
                assert rel_err(form[0][t], h1[t]) <= TOL, (r, "hidden1", t)
                assert rel_err(form[1][t], emb[t]) <= TOL, (r, "embeddings", t)
        for t in (0, 1):  # SURVEY §8c's elementwise pass-rate, |y − y_ref| <= 1e-4·|y_ref| + 1e-6
            for got_, want_ in ((eager[0][t], h1[t]), (eager[1][t], emb[t])):
                ok = np.abs(got_ - want_) <= 1e-4 * np.abs(want_) + 1e-6
                assert ok.mean() >= 0.9999, (r, t, ok.mean())
        for t in (0, 1):  # the graph-captured phases reproduce the eager forward bit for bit
            assert np.array_equal(eager[0][t], graphed[0][t]) and np.array_equal(eager[1][t], graphed[1][t])
    # every relation of a relation-sharded group is owned by exactly one rank; a row-split
    # group's relations by every rank (each over its row block)
    split = got[0][0]["row_split"]
    for et in g.edge_types:
        owned = sum(got[r][0]["local"][et] for r in range(world))
        dealt = et in got[0][0]["dealt"]  # (every rank holds a row-dealt group's relations)
        assert owned == (g.edge_types[et] * (world if et[0] in split or dealt else 1))


def test_sharded_S_forward_matches_oracle():
    _check("S", 2)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_weak_scaling_S_row_split_matches_oracle(world):
    """bench.py's config S at N GPUs: N relation sets, every node type row-split; each rank's
    block in dg_spmm_seg_f32 (one chunk per relation set) + the epilogue, layer 2
    reassociated as Σ_k (Â_k·H1)·W2_k, blocks all-gathered."""
    _check("S-rows", world)


@pytest.mark.parametrize("world", [2, 8])
def test_weak_scaling_S_fused_form_matches_oracle(world):
    """The same partition in the fused kernel (one workgroup per row, projection GEMM on every
    rank) — RelationShard.weak_sets(form="fused"), DG_S_ROWS_FORM=fused."""
    _check("S-rows-fused", world)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_P_shaped_row_split_matches_oracle(world):
    _check("P-small", world)


def test_sharded_row_split_equal_layer_widths():
    """h1 == h2 on a row-split graph: hidden1 and the embeddings keep separate padded
    buffers (the layer-2 operand is not overwritten by the layer-2 output)."""
    _check("P-small", 2, h2=64)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_full_size_P_matches_oracle(world):
    """configs[3]'s plan at full size (19,085 + 645 nodes, 1,932 matrices, ≈23 M nnz) on 2
    and 8 ranks: proteins row-split, 1,928 drug×drug relations LPT-sharded (staged kernel) —
    at 8, the partition of the driver's 8-GPU run."""
    _check("P", world)


# ---------------------------------------------------------------------------- training
def _train_rank(rank, world, kind, split=False, dropout=0.0):
    """One sharded training step (train.py): forward (flat mode: all-reduces, and with `split`
    the proteins row-split — all-gathers), the DEDICOM decoder + hinge on a fixed batch of
    relation (1,1)_0 with given negatives, the backward (dH1 all-reduce; row-split groups'
    partial weight gradients all-reduced) and TF-Adam on the rank's relations, with dropout
    masks drawn under each relation's global id.  Returns the local gradients by global
    relation id, the decoder gradients, the loss and the updated local weights."""
    from decagon_amd import kernels, train
    from decagon_amd.engine import DeviceGraph, ForwardPlan, LayerWeights
    from decagon_amd.sharding import RelationShard, torch_allgather, torch_allreduce

    dev = torch.device("cuda", 0)
    g = _graph(kind)
    nnz = {et: [len(c[1]) for c in rels] for et, rels in g.adj.items()}
    if split:
        shard = RelationShard.split(g.edge_types, g.n_nodes, nnz, rank, world, torch_allreduce(), torch_allgather(),
                                    row_split_min=1000, deal_rows=[(1, 0)] if split == "deal" else ())
    else:
        shard = RelationShard.lpt(g.edge_types, nnz, rank, world, torch_allreduce())
    w1, w2 = _weights(g, 5)
    W1 = LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w1.items()})
    W2 = LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w2.items()})
    dg = DeviceGraph(g.edge_types, shard.local_csr(g.csr()), dev, shard.local, row_block=shard.row_block)
    drop = None
    if dropout > 0:
        drop = (1.0 - dropout, torch.tensor([20180701, 0], dtype=torch.int64, device=dev))
    fwd = ForwardPlan(dg, {0: None, 1: None}, W1, W2, 64, 32, shard=shard, keep_sums=True, dropout=drop)
    tp = train.TrainPlan(fwd, W1, W2, {0: None, 1: None})
    R, l, rows, cols, neg = _train_batch(g)
    E = fwd.embeddings[1]
    Rt, lt = torch.from_numpy(R).to(dev), torch.from_numpy(l).to(dev)
    rows_t, cols_t, neg_t = (torch.from_numpy(x.astype(np.int32)).to(dev) for x in (rows, cols, neg))
    hinge = kernels.PreparedDecoderHinge(E, E, rows_t, cols_t, Rt, lt, 0.1, neg_rows=neg_t)
    dR, dl = torch.zeros_like(Rt), torch.zeros_like(lt)
    dgrad = kernels.PreparedDecoderGrad(E, E, rows_t, cols_t, neg_t, hinge.pos, hinge.neg, Rt, lt, 0.1,
                                        dG=dR.view(-1), dl=dl)

    def decoder_grad(dE):
        dgrad()
        kernels.scatter_rows(dgrad.row_idx, dgrad.grad_rows, dE[1])
        kernels.scatter_rows(cols_t, dgrad.grad_cols, dE[1])

    pairs = tp.adam_pairs(W1, W2)
    adam = train.AdamState([p for p, _ in pairs], lr=0.001)
    prep = adam.prepared([gr for _, gr in pairs])
    fwd.run()
    hinge()
    tp.backward(decoder_grad)
    torch.cuda.synchronize()
    grads = {"w1": {}, "w2": {}}
    for name, gw in (("w1", tp.gW1), ("w2", tp.gW2)):
        for et, ids in tp.local_ids.items():
            for c, k in enumerate(ids):
                grads[name][et[0], et[1], int(k)] = gw[et][c].cpu().numpy()
    adam.apply(prep)
    torch.cuda.synchronize()
    after = {}
    for name, st in (("w1", W1), ("w2", W2)):
        for et, ids in tp.local_ids.items():
            for k in ids:
                after[name, et[0], et[1], int(k)] = st.stacks[et][int(k)].cpu().numpy()
    info = {"row_split": sorted(shard.row_block), "dealt": sorted(shard.dealt)}
    return grads, {"R": dR.cpu().numpy(), "l": dl.cpu().numpy()}, float(hinge.loss[0]), after, info


def _train_batch(g):
    rng = np.random.default_rng(17)
    R = rng.uniform(-0.3, 0.3, (32, 32)).astype(np.float32)
    l = rng.uniform(0.5, 1.5, 32).astype(np.float32)
    coords = g.adj[1, 1][0][0]
    pick = coords[rng.choice(len(coords), 128, replace=False)]
    neg = rng.integers(0, g.n_nodes[1], 128)
    return R, l, pick[:, 0], pick[:, 1], neg


def _train_oracle(kind, g, dropout=0.0):
    from oracle import decagon_oracle as orc
    from test_cpu_train_oracle import _masks

    w1, w2 = _weights(g, 5)
    R, l, rows, cols, neg = _train_batch(g)
    ets = list(g.edge_types)
    decoders = {et: "dedicom" for et in ets}
    rng = np.random.default_rng(1)
    dec = {et: {"global_interaction": rng.uniform(-0.3, 0.3, (32, 32)),
                **{"local_variation_%d" % k: rng.uniform(0.5, 1.5, 32) for k in range(K)}}
           for et, K in g.edge_types.items()}
    dec[1, 1]["global_interaction"] = R.astype(np.float64)
    dec[1, 1]["local_variation_0"] = l.astype(np.float64)
    e = sum(g.edge_types[et] for et in ets[:ets.index((1, 1))])  # flat index of (1,1)_0
    n = g.n_nodes
    feats = {t: None for t in n}
    adj = {et: [(c, v.astype(np.float32).astype(np.float64), s) for c, v, s in mats] for et, mats in g.adj.items()}
    drop1, drop2 = _masks(g.edge_types, adj, 1.0 - dropout, step=1) if dropout > 0 else (None, None)
    cost, ref = orc.train_grads(g.edge_types, adj, feats,
                                {et: [x.astype(np.float64) for x in w] for et, w in w1.items()},
                                {et: [x.astype(np.float64) for x in w] for et, w in w2.items()},
                                decoders, dec, 32, np.stack([rows, cols], 1), neg, e, 1, 1, 0.1,
                                drop1=drop1, drop2=drop2)
    return cost, ref, w1, w2


@pytest.mark.parametrize("kind,split,dropout", [("S", False, 0.0), ("S", False, 0.1), ("P-small", True, 0.1),
                                                ("P-small", True, 0.0), ("P-small", "deal", 0.1)])
def test_sharded_training_step_matches_oracle(kind, split, dropout):
    """Sharded training on 2 ranks: config S relations LPT-sharded (with and without the
    reference's default dropout 0.1, main.py:305-308), and the scaled-down config P with its
    proteins row-split (the multi-GPU plan of config P, optimizer.py:108-114 on it).  Every
    rank's gradients of its relations and the (replicated) decoder gradients equal the float64
    oracle's TF-minimize gradients (oracle.train_grads, on the same dropout masks) within 1e-4;
    a relation-sharded relation is updated by exactly one rank, a row-split group's relations
    by every rank identically (all-reduced gradients), each by one TF-Adam step (oracle.adam_tf)."""
    from oracle import decagon_oracle as orc

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    world = 2
    got = run_ranks(_train_rank, world, (kind, split, dropout))
    g = _graph(kind)
    cost, ref, w1, w2 = _train_oracle(kind, g, dropout)
    seen = {}
    for r in range(world):
        grads, dec, loss, after, info = got[r]
        assert info["row_split"] == ([0] if split else []), info
        assert abs(loss - cost) <= TOL * abs(cost)
        assert rel_err(dec["R"], ref["dec"][1, 1]["global_interaction"]) <= TOL
        assert rel_err(dec["l"], ref["dec"][1, 1]["local_variation_0"]) <= TOL
        for name, wref, wsrc in (("w1", ref["w1"], w1), ("w2", ref["w2"], w2)):
            for (i, j, k), gv in grads[name].items():
                want = wref[i, j][k]
                scale = np.max(np.abs(want))
                assert np.max(np.abs(gv - want)) <= TOL * max(scale, 1e-30), (r, name, i, j, k)
                p1, _, _ = orc.adam_tf(wsrc[i, j][k], gv, np.zeros_like(gv), np.zeros_like(gv), 1)
                assert np.max(np.abs(after[name, i, j, k] - p1)) <= 1e-6 * max(1.0, np.max(np.abs(p1)))
                key = (name, i, j, k)
                if key in seen:  # only a row-split group's relations live on several ranks
                    assert split and (i in info["row_split"] or (i, j) in info["dealt"]), key
                    assert np.array_equal(seen[key], after[key]), key
                seen[key] = after[name, i, j, k]
    assert len(seen) == 2 * sum(g.edge_types.values())  # every relation
