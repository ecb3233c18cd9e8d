"""Model-level parity on config S through the drop-in surface, driven the way the
reference's drivers drive it (main.py:244-315, DecagonTrainableBuilder.py:80-118): build
placeholders, DecagonModel, DecagonOptimizer; feed the reference-normalised adjacency
tuples (tests/golden/synthetic_S.npz, produced by the reference's EdgeMinibatchIterator);
load the fixture's seeded weights into the model variables; inject the negatives; compare
hidden1 / embeddings / outputs / neg_outputs / cost / predictions with the fixture
(float64 restatement) at ≤ 1e-4 relative.
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TOL = 1e-4


def _setup(z, edge_order=None):
    import decagon_amd as dg

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    et_rows = z["edge_types"]
    edge_types = {(int(i), int(j)): int(k) for i, j, k in et_rows}
    decoders = {et: str(d) for et, d in zip(edge_types, z["decoders"])}
    if edge_order is not None:
        edge_types = {et: edge_types[et] for et in edge_order}
        decoders = {et: decoders[et] for et in edge_order}
    n = {0: int(z["n_nodes"][0]), 1: int(z["n_nodes"][1])}
    ph = dg.construct_placeholders(edge_types)
    model = dg.DecagonModel(placeholders=ph, num_feat=n, nonzero_feat=n, edge_types=edge_types,
                            decoders=decoders)
    degrees = {0: [z["deg_0_0_0"], z["deg_0_0_1"]], 1: [z[f"deg_1_1_{k}"] for k in range(6)]}
    edge_type2dim = {et: [tuple(int(s) for s in z[f"adj_{et[0]}_{et[1]}_{k}_shape"]) for k in range(K)]
                     for et, K in edge_types.items()}
    opt = dg.DecagonOptimizer(embeddings=model.embeddings, latent_inters=model.latent_inters,
                              latent_varies=model.latent_varies, degrees=degrees, edge_types=edge_types,
                              edge_type2dim=edge_type2dim, placeholders=ph, batch_size=512, margin=0.1)
    # weights from the fixture
    for et, K in edge_types.items():
        i, j = et
        for k in range(K):
            model.layers1[et].vars["weights_%d" % k].load(z[f"w1_{i}_{j}_{k}"])
            model.layers2[et].vars["weights_%d" % k].load(z[f"w2_{i}_{j}_{k}"])
        for name, var in model.edge_type2decoder[et].vars.items():
            var.load(z[f"dec_{i}_{j}_{name}"])
    feed = {}
    for et, K in edge_types.items():
        i, j = et
        for k in range(K):
            feed[ph["adj_mats_%d,%d,%d" % (i, j, k)]] = (z[f"adj_{i}_{j}_{k}_coords"], z[f"adj_{i}_{j}_{k}_values"],
                                                          tuple(z[f"adj_{i}_{j}_{k}_shape"]))
    for t in (0, 1):
        feed[ph["feat_%d" % t]] = (np.stack([np.arange(n[t])] * 2, 1), np.ones(n[t]), (n[t], n[t]))
    feed[ph["dropout"]] = 0.0
    return dg, ph, model, opt, feed


@pytest.mark.parametrize("fused_seg,tab", [(True, True), (True, False), (False, False)])
def test_forward_matches_golden(golden_S, monkeypatch, fused_seg, tab):
    """Config S's golden forward through the Session, in dg_gcn_fused_tab_f32 (the default: the
    fused-seg layer from a host-built wave table), dg_gcn_fused_seg_f32 (layer 2 reassociated)
    and dg_gcn_fused_f32 with the projection epilogue."""
    from decagon_amd import engine

    monkeypatch.setattr(engine, "FUSED_SEG", fused_seg)
    monkeypatch.setattr(engine, "WAVE_TABLE", tab)
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    sess = dg.Session()
    h1_0, h1_1, e0, e1 = sess.run([model.hidden1[0], model.hidden1[1], model.embeddings[0], model.embeddings[1]],
                                  feed_dict=feed)
    assert rel_err(h1_0, z["hidden1_0"]) <= TOL
    assert rel_err(h1_1, z["hidden1_1"]) <= TOL
    assert rel_err(e0, z["emb_0"]) <= TOL
    assert rel_err(e1, z["emb_1"]) <= TOL
    # elementwise pass-rate reported by SURVEY §8c
    for got, want in ((e0, z["emb_0"]), (e1, z["emb_1"])):
        ok = np.abs(got - want) <= 1e-4 * np.abs(want) + 1e-6
        assert ok.mean() == 1.0


def test_decoder_and_loss_match_golden(golden_S):
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    sess = dg.Session()
    for b in range(4):
        e, rt, ct = (int(v) for v in z[f"batch{b}_meta"])
        fd = dict(feed)
        fd[ph["batch"]] = z[f"batch{b}_edges"]
        fd[ph["batch_edge_type_idx"]] = e
        fd[ph["batch_row_edge_type"]] = rt
        fd[ph["batch_col_edge_type"]] = ct
        fd[opt.neg_samples] = z[f"batch{b}_neg"]
        out, neg, cost, idx = sess.run([opt.outputs, opt.neg_outputs, opt.cost, opt.batch_edge_type_idx], fd)
        assert int(idx) == e
        assert rel_err(out, z[f"batch{b}_outputs"]) <= TOL
        assert rel_err(neg, z[f"batch{b}_neg_outputs"]) <= TOL
        assert abs(float(cost) - float(z[f"batch{b}_cost"])) <= TOL * max(1.0, abs(float(z[f"batch{b}_cost"])))
        xent = sess.run(opt._xent_loss(opt.outputs, opt.neg_outputs), fd)
        assert abs(float(xent) - float(z[f"batch{b}_xent"])) <= TOL * abs(float(z[f"batch{b}_xent"]))


def test_predictions_match_golden(golden_S):
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    sess = dg.Session()
    for e, rt, ct in ((2, 0, 1), (7, 1, 1)):
        fd = dict(feed)
        fd[ph["batch_edge_type_idx"]] = e
        fd[ph["batch_row_edge_type"]] = rt
        fd[ph["batch_col_edge_type"]] = ct
        pred = sess.run(opt.predictions, fd)
        assert rel_err(pred, z[f"predictions_{e}"]) <= TOL


def test_edge_type_order_of_main_framework(golden_S):
    """DecagonDataSet orders edge types (0,0),(0,1),(1,1),(1,0); the sums over
    edge types then run in that order — same values within tolerance."""
    z = golden_S
    dg, ph, model, opt, feed = _setup(z, edge_order=[(0, 0), (0, 1), (1, 1), (1, 0)])
    e1 = dg.Session().run(model.embeddings[1], feed)
    assert rel_err(e1, z["emb_1"]) <= TOL


def test_sampled_negatives_in_range(golden_S):
    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    fd = dict(feed)
    fd[ph["batch"]] = z["batch3_edges"]
    e, rt, ct = (int(v) for v in z["batch3_meta"])
    fd[ph["batch_edge_type_idx"]] = e
    fd[ph["batch_row_edge_type"]] = rt
    fd[ph["batch_col_edge_type"]] = ct
    neg, cost = dg.Session().run([opt.neg_samples, opt.cost], fd)
    assert neg.shape == (512,) and neg.min() >= 0 and neg.max() < 400
    assert np.isfinite(cost)


def test_standalone_layer_matches_oracle(golden_S):
    """Calling a layer object directly (layers.py:85-94 / 109-118) — including the class's
    default act=relu applied per relation before add_n."""
    import decagon_amd as dg
    from oracle import decagon_oracle as orc

    z = golden_S
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ph = dg.construct_placeholders({(1, 1): 6})
    adj = {(1, 1): [ph["adj_mats_1,1,%d" % k] for k in range(6)]}
    lay = dg.GraphConvolutionSparseMulti({1: 400}, 64, adj, {1: 400}, edge_type=(1, 1), num_types=6)
    for k in range(6):
        lay.vars["weights_%d" % k].load(z[f"w1_1_1_{k}"])
    node = lay(ph["feat_1"])
    feed = {ph["adj_mats_1,1,%d" % k]: (z[f"adj_1_1_{k}_coords"], z[f"adj_1_1_{k}_values"], (400, 400))
            for k in range(6)}
    feed[ph["feat_1"]] = (np.stack([np.arange(400)] * 2, 1), np.ones(400), (400, 400))
    got = dg.Session().run(node, feed)
    outs = [np.maximum(orc.sparse_dense_matmul((z[f"adj_1_1_{k}_coords"], z[f"adj_1_1_{k}_values"], (400, 400)),
                                               z[f"w1_1_1_{k}"].astype(np.float64)), 0) for k in range(6)]
    assert rel_err(got, orc.l2_normalize_rows(np.sum(outs, 0))) <= TOL


def test_sparse_features_path(golden_S):
    """Non-identity sparse features (T2 = X_j·W_k, layers.py:89) through the fused plan."""
    from oracle import decagon_oracle as orc
    import scipy.sparse as sp

    z = golden_S
    dg, ph, model, opt, feed = _setup(z)
    rng = np.random.default_rng(0)
    fd = dict(feed)
    feats = {}
    for t, n in ((0, 500), (1, 400)):
        m = sp.random(n, n, density=0.02, random_state=rng, format="coo") + sp.eye(n)
        m = m.tocoo()
        feats[t] = (np.stack([m.row, m.col], 1), m.data, (n, n))
        fd[ph["feat_%d" % t]] = feats[t]
    e0, e1 = dg.Session().run([model.embeddings[0], model.embeddings[1]], fd)
    edge_types = {(int(i), int(j)): int(k) for i, j, k in z["edge_types"]}
    adj = {et: [(z[f"adj_{et[0]}_{et[1]}_{k}_coords"], z[f"adj_{et[0]}_{et[1]}_{k}_values"],
                 tuple(z[f"adj_{et[0]}_{et[1]}_{k}_shape"])) for k in range(K)] for et, K in edge_types.items()}
    w1 = {et: [z[f"w1_{et[0]}_{et[1]}_{k}"].astype(np.float64) for k in range(K)] for et, K in edge_types.items()}
    w2 = {et: [z[f"w2_{et[0]}_{et[1]}_{k}"].astype(np.float64) for k in range(K)] for et, K in edge_types.items()}
    f64 = {t: (f[0], f[1].astype(np.float64), f[2]) for t, f in feats.items()}
    _, emb = orc.decagon_forward(edge_types, adj, f64, w1, w2)
    assert rel_err(e0, emb[0]) <= TOL
    assert rel_err(e1, emb[1]) <= TOL


def test_dedicom_kat_reference_parameters(golden_kat):
    """DEDICOM on the reference's own trained R and D_r (ndarray-dump*.np*) against the
    reference's numpy predictor formula E·D·R·D·Eᵀ (NpPredictor.py:304)."""
    from decagon_amd import kernels

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    z = golden_kat
    E = torch.from_numpy(z["E"]).cuda()
    R = torch.from_numpy(z["R"]).cuda()
    n = E.shape[0]
    ri = torch.arange(n, device="cuda", dtype=torch.int32).repeat_interleave(n)
    ci = torch.arange(n, device="cuda", dtype=torch.int32).repeat(n)
    for r in range(z["Ddiag"].shape[0]):
        l = torch.from_numpy(z["Ddiag"][r]).cuda()
        want = z[f"scores_{r}"]
        pairs = kernels.decoder_score(E, E, ri, ci, R, l).cpu().numpy().reshape(n, n)
        assert rel_err(pairs, want) <= TOL
        from decagon_amd import runtime
        full = runtime.full_scores(E, E, R, l).cpu().numpy()
        assert rel_err(full, want) <= TOL


@pytest.mark.parametrize("staged", ["1", "0"])
def test_polypharmacy_shaped_plan_matches_oracle(monkeypatch, staged):
    """A scaled-down config P (drug×drug group large enough for the LDS-staged kernel and
    for partial mode + epilogue; proteins fused) against the float64 restatement."""
    import importlib

    from oracle import decagon_oracle as orc
    from decagon_amd import engine, synthetic

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    monkeypatch.setenv("DG_STAGED", staged)
    g = synthetic.make_P(seed=3, n_proteins=900, n_drugs=120, n_side_effects=40, ppi_edges=6000,
                         target_edges=700)
    rng = np.random.default_rng(1)
    n = g.n_nodes
    w1 = {et: rng.uniform(-0.2, 0.2, (K, n[et[1]], 64)).astype(np.float32) for et, K in g.edge_types.items()}
    w2 = {et: rng.uniform(-0.3, 0.3, (K, 64, 32)).astype(np.float32) for et, K in g.edge_types.items()}
    dev = torch.device("cuda")
    dg = engine.DeviceGraph(g.edge_types, g.csr(), dev)
    assert dg.groups[(1, 1)].staged == (staged == "1")
    plan = engine.ForwardPlan(dg, {0: None, 1: None},
                              engine.LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w1.items()}),
                              engine.LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w2.items()}), 64, 32)
    plan.run()
    torch.cuda.synchronize()
    feats = {t: (np.stack([np.arange(n[t])] * 2, 1), np.ones(n[t]), (n[t], n[t])) for t in n}
    h1, emb = orc.decagon_forward(g.edge_types, g.adj, feats,
                                  {et: [x.astype(np.float64) for x in w] for et, w in w1.items()},
                                  {et: [x.astype(np.float64) for x in w] for et, w in w2.items()})
    assert rel_err(plan.hidden1[1].cpu().numpy(), h1[1]) <= TOL
    assert rel_err(plan.embeddings[0].cpu().numpy(), emb[0]) <= TOL
    assert rel_err(plan.embeddings[1].cpu().numpy(), emb[1]) <= TOL


def test_full_size_config_P_matches_oracle():
    """BASELINE configs[2] at full size — 19,085 proteins, 645 drugs, 1,932 matrices, ≈23 M
    nnz per layer, the plan bench.py times (staged drug×drug SpMM, PPI windows, projection
    GEMM) — against the float64 restatement with scipy products, every output row."""
    import scipy.sparse as sp

    from oracle import decagon_oracle as orc
    from decagon_amd import engine, synthetic

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    g = synthetic.make_P(seed=0)
    rng = np.random.default_rng(11)
    n = g.n_nodes
    w1 = {et: rng.uniform(-0.1, 0.1, (K, n[et[1]], 64)).astype(np.float32) for et, K in g.edge_types.items()}
    w2 = {et: rng.uniform(-0.2, 0.2, (K, 64, 32)).astype(np.float32) for et, K in g.edge_types.items()}
    dev = torch.device("cuda")
    dg = engine.DeviceGraph(g.edge_types, g.csr(), dev)
    assert dg.groups[(1, 1)].staged
    plan = engine.ForwardPlan(dg, {0: None, 1: None},
                              engine.LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w1.items()}),
                              engine.LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w2.items()}), 64, 32)
    plan.run()
    torch.cuda.synchronize()
    # the adjacency values as fed: float64 preprocess_graph output cast to float32
    csr = {et: [sp.csr_matrix((v.astype(np.float32).astype(np.float64), (c[:, 0], c[:, 1])), shape=s)
                for c, v, s in mats] for et, mats in g.adj.items()}
    h1, emb = orc.decagon_forward_csr(g.edge_types, csr, {et: w.astype(np.float64) for et, w in w1.items()},
                                      {et: w.astype(np.float64) for et, w in w2.items()})
    for t in (0, 1):
        got_h1, got_e = plan.hidden1[t].cpu().numpy(), plan.embeddings[t].cpu().numpy()
        assert rel_err(got_h1, h1[t]) <= TOL
        assert rel_err(got_e, emb[t]) <= TOL
        # SURVEY §8c's elementwise pass-rate: |y − y_ref| <= 1e-4·|y_ref| + 1e-6, every element
        # (23 M-nonzero fp32 sums against float64: a few near-zero elements may miss the floor)
        for got_, want_ in ((got_h1, h1[t]), (got_e, emb[t])):
            ok = np.abs(got_ - want_) <= 1e-4 * np.abs(want_) + 1e-6
            assert ok.mean() >= 0.9999, (t, ok.mean())


def test_training_sums_mode_matches_oracle(monkeypatch):
    """ForwardPlan(keep_sums=True) on one GPU with no fused node type (config P's shape): the
    partial-mode layers' single epilogue launch also writes every group's pre-normalisation
    sum S_ij (the backward's input) — checked group by group against the float64 sums, with
    H1 and the embeddings."""
    from oracle import decagon_oracle as orc
    from decagon_amd import engine, synthetic

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    monkeypatch.setattr(engine, "FUSED_MAX_ROWS", 0)  # every node type in partial mode
    g = synthetic.make_P(seed=5, n_proteins=700, n_drugs=110, n_side_effects=30, ppi_edges=4000,
                         target_edges=500)
    rng = np.random.default_rng(2)
    n = g.n_nodes
    w1 = {et: rng.uniform(-0.2, 0.2, (K, n[et[1]], 64)).astype(np.float32) for et, K in g.edge_types.items()}
    w2 = {et: rng.uniform(-0.3, 0.3, (K, 64, 32)).astype(np.float32) for et, K in g.edge_types.items()}
    dev = torch.device("cuda")
    dg = engine.DeviceGraph(g.edge_types, g.csr(), dev)
    plan = engine.ForwardPlan(dg, {0: None, 1: None},
                              engine.LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w1.items()}),
                              engine.LayerWeights({et: torch.from_numpy(w).to(dev) for et, w in w2.items()}),
                              64, 32, keep_sums=True)
    assert plan.sums_mode and not plan.flat_mode
    plan.run()
    torch.cuda.synchronize()
    feats = {t: (np.stack([np.arange(n[t])] * 2, 1), np.ones(n[t]), (n[t], n[t])) for t in n}
    h1, emb = orc.decagon_forward(g.edge_types, g.adj, feats,
                                  {et: [x.astype(np.float64) for x in w] for et, w in w1.items()},
                                  {et: [x.astype(np.float64) for x in w] for et, w in w2.items()})
    for t in (0, 1):
        assert rel_err(plan.hidden1[t].cpu().numpy(), h1[t]) <= TOL
        assert rel_err(plan.embeddings[t].cpu().numpy(), emb[t]) <= TOL
    for et, K in g.edge_types.items():
        i, j = et
        s1 = sum(orc.sparse_dense_matmul(g.adj[et][k], w1[et][k].astype(np.float64)) for k in range(K))
        s2 = sum(orc.sparse_dense_matmul(g.adj[et][k], h1[j] @ w2[et][k].astype(np.float64)) for k in range(K))
        assert rel_err(plan._layer1.views[et].view(n[i], 64).cpu().numpy(), s1) <= TOL
        assert rel_err(plan._layer2.views[et].view(n[i], 32).cpu().numpy(), s2) <= TOL


@pytest.mark.parametrize("dense", [False, True])
def test_standalone_layer_dropout_matches_oracle(golden_S, dense):
    """A layer called on its own with dropout > 0 (layers.py:88 dropout_sparse on the identity
    features, :112 tf.nn.dropout of the dense inputs), drawn per relation with the device's
    counter-based masks: each run against the float64 layer on the SAME masks, regenerated by
    oracle.dropout_scale from the layer's state {seed, step}; two runs draw different masks."""
    import decagon_amd as dg
    from decagon_amd.layers import _GraphConvBase
    from oracle import decagon_oracle as orc

    z = golden_S
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    keep = 0.75
    ph = dg.construct_placeholders({(1, 1): 6})
    adj = {(1, 1): [ph["adj_mats_1,1,%d" % k] for k in range(6)]}
    feed = {ph["adj_mats_1,1,%d" % k]: (z[f"adj_1_1_{k}_coords"], z[f"adj_1_1_{k}_values"], (400, 400))
            for k in range(6)}
    A = [(z[f"adj_1_1_{k}_coords"], z[f"adj_1_1_{k}_values"], (400, 400)) for k in range(6)]
    if dense:
        rng = np.random.default_rng(5)
        H = rng.standard_normal((400, 64)).astype(np.float32)
        W = [rng.uniform(-0.2, 0.2, (64, 32)).astype(np.float32) for _ in range(6)]
        lay = dg.GraphConvolutionMulti(64, 32, adj, dropout=1 - keep, edge_type=(1, 1), num_types=6)
        x = dg.placeholder(np.float32, name="h_in")
        feed[x] = H
        tag, n_mask = 2 << 16, 6 * 400 * 64
    else:
        W = [z[f"w1_1_1_{k}"] for k in range(6)]
        lay = dg.GraphConvolutionSparseMulti({1: 400}, 64, adj, {1: 400}, dropout=1 - keep, edge_type=(1, 1),
                                             num_types=6)
        x = ph["feat_1"]
        feed[x] = (np.stack([np.arange(400)] * 2, 1), np.ones(400), (400, 400))
        tag, n_mask = 1 << 16, 6 * 400
    for k in range(6):
        lay.vars["weights_%d" % k].load(W[k])
    node = lay(x)
    sess = dg.Session()
    runs = [sess.run(node, feed) for _ in range(2)]
    for step, got in enumerate(runs, start=1):
        m = orc.dropout_scale(_GraphConvBase.dropout_seed, step, tag, n_mask, keep).astype(np.float64)
        outs = []
        for k in range(6):
            if dense:
                xk = (H.astype(np.float64) * m.reshape(6, 400, 64)[k]) @ W[k].astype(np.float64)
            else:
                xk = m.reshape(6, 400)[k][:, None] * W[k].astype(np.float64)
            outs.append(np.maximum(orc.sparse_dense_matmul(A[k], xk), 0))
        assert rel_err(got, orc.l2_normalize_rows(np.sum(outs, 0))) <= TOL, step
    assert not np.allclose(runs[0], runs[1])
