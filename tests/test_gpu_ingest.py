"""GPU: the model on an ingested DecagonPublicData-format graph (decagon_amd/ingest.py) with
sparse mono side-effect features for the drugs (general layer 1: X_j·W_k, layers.py:85-94):
forward against the float64 oracle, and the training gradients (including X_jᵀ·(Â_kᵀ·dS)
for the feature weights) against oracle.train_grads.

Tolerance: per tensor max|y − y_ref| ≤ 1e-4·max|y_ref| (fp32 path)."""
import numpy as np
import pytest

from conftest import rel_err
from oracle import decagon_oracle as orc

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

TOL = 1e-4
DECODERS = {(0, 0): "bilinear", (0, 1): "bilinear", (1, 1): "dedicom", (1, 0): "bilinear"}


def _build(tmp_path, seed=3):
    import decagon_amd as dg
    from decagon_amd import ingest

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    paths = ingest.write_public_csvs(str(tmp_path / "pd"), seed=seed, n_proteins=400, n_drugs=70,
                                     n_side_effects=5, n_ppi=2000, n_targets=300, n_mono=700,
                                     n_mono_effects=90)
    data = ingest.load_public_data(*paths, min_edges=100)
    adj = ingest.normalized(data)
    edge_types = data.edge_types
    n = {0: len(data.node_lists.proteins), 1: len(data.node_lists.drugs)}
    f1 = data.features[1]
    ph = dg.construct_placeholders(edge_types)
    model = dg.DecagonModel(placeholders=ph, num_feat={0: n[0], 1: f1[2][1]},
                            nonzero_feat={0: n[0], 1: len(f1[1])}, edge_types=edge_types,
                            decoders={et: DECODERS[et] for et in edge_types})
    edge_type2dim = {et: [m.shape for m in ms] for et, ms in data.adj.items()}
    opt = dg.DecagonOptimizer(embeddings=model.embeddings, latent_inters=model.latent_inters,
                              latent_varies=model.latent_varies, degrees=data.degrees, edge_types=edge_types,
                              edge_type2dim=edge_type2dim, placeholders=ph, batch_size=64, margin=0.1)
    feed = {ph["adj_mats_%d,%d,%d" % (et[0], et[1], k)]: t for et, ts in adj.items() for k, t in enumerate(ts)}
    feed[ph["feat_0"]] = data.features[0]
    feed[ph["feat_1"]] = f1
    feed[ph["dropout"]] = 0.0
    return dg, data, adj, ph, model, opt, feed


def _weights(model, edge_types):
    w1 = {et: [model.layers1[et].vars["weights_%d" % k].eval().astype(np.float64) for k in range(K)]
          for et, K in edge_types.items()}
    w2 = {et: [model.layers2[et].vars["weights_%d" % k].eval().astype(np.float64) for k in range(K)]
          for et, K in edge_types.items()}
    dec = {et: {nm: v.eval().astype(np.float64) for nm, v in model.edge_type2decoder[et].vars.items()}
           for et in edge_types}
    return w1, w2, dec


def test_forward_on_ingested_graph_with_mono_features(tmp_path):
    dg, data, adj, ph, model, opt, feed = _build(tmp_path)
    assert model.edge_types[(1, 1)] >= 4 and data.features[1][2][1] > 10
    sess = dg.Session()
    got = sess.run([model.hidden1[0], model.hidden1[1], model.embeddings[0], model.embeddings[1]], feed_dict=feed)
    w1, w2, _ = _weights(model, model.edge_types)
    feats = {0: data.features[0], 1: data.features[1]}
    hidden1, emb = orc.decagon_forward(model.edge_types, adj, feats, w1, w2)
    for g, w in zip(got, [hidden1[0], hidden1[1], emb[0], emb[1]]):
        assert rel_err(g, w) <= TOL


def test_grads_with_sparse_features_match_oracle(tmp_path):
    dg, data, adj, ph, model, opt, feed = _build(tmp_path)
    edge_types = model.edge_types
    rng = np.random.default_rng(5)
    e = 3  # the first drug-drug relation: (0,0)×2, (0,1)×1 come first
    r, c = data.adj[(1, 1)][0].nonzero()
    pick = rng.choice(len(r), 64, replace=False)
    batch = np.stack([r[pick], c[pick]], 1).astype(np.int32)
    neg = rng.integers(0, len(data.node_lists.drugs), 64).astype(np.int32)
    f = dict(feed)
    f.update({ph["batch"]: batch, ph["batch_edge_type_idx"]: e, ph["batch_row_edge_type"]: 1,
              ph["batch_col_edge_type"]: 1, opt.neg_samples: neg})
    sess = dg.Session()
    gv = sess.run(opt.grads_vars, feed_dict=f)
    w1, w2, dec = _weights(model, edge_types)
    feats = {0: None, 1: data.features[1]}
    cost, ref = orc.train_grads(edge_types, adj, feats, w1, w2, model.decoders, dec, 32, batch, neg, e, 1, 1, 0.1)
    want = []
    for et, K in edge_types.items():
        want += [ref["w1"][et][k] for k in range(K)]
    for et, K in edge_types.items():
        want += [ref["w2"][et][k] for k in range(K)]
    for et in edge_types:
        want += [ref["dec"][et][nm] for nm in model.edge_type2decoder[et].vars]
    assert len(gv) == len(want)
    checked = 0
    for (g, _), w in zip(gv, want):
        assert g.shape == w.shape
        scale = np.max(np.abs(w))
        if scale == 0:
            assert np.max(np.abs(g)) == 0.0
        else:
            checked += 1
            assert np.max(np.abs(g - w)) <= TOL * scale, f"gradient off by {rel_err(g, w):.2e}"
    assert checked > 0
    # the feature weights of drug-sourced relations carry gradient
    order = list(edge_types)
    k0 = sum(edge_types[et] for et in order[:order.index((1, 1))])
    assert any(np.max(np.abs(gv[i][0])) > 0 for i in range(k0, k0 + edge_types[(1, 1)]))


def test_grads_with_sparse_features_and_dropout_match_oracle(tmp_path):
    """main.py's training setting on the ingested graph: FLAGS.dropout = 0.1 (main.py:235, :307)
    with sparse mono side-effect drug features — dropout_sparse draws, per relation, a mask
    over X_j's values (layers.py:23-31, :88) on the device (DG_GROUP_DROPOUT in the X_j·W_k
    SpMM, the same masks in the X_jᵀ·(Â_kᵀ·dS) backward).  Every gradient against the oracle
    on the same masks (the device's step-1 draw, regenerated by oracle.dropout_scale)."""
    from decagon_amd.sparse import coo_to_csr

    dg, data, adj, ph, model, opt, feed = _build(tmp_path)
    edge_types = model.edge_types
    rng = np.random.default_rng(6)
    e = 3
    r, c = data.adj[(1, 1)][0].nonzero()
    pick = rng.choice(len(r), 64, replace=False)
    batch = np.stack([r[pick], c[pick]], 1).astype(np.int32)
    neg = rng.integers(0, len(data.node_lists.drugs), 64).astype(np.int32)
    f = dict(feed)
    f.update({ph["batch"]: batch, ph["batch_edge_type_idx"]: e, ph["batch_row_edge_type"]: 1,
              ph["batch_col_edge_type"]: 1, opt.neg_samples: neg, ph["dropout"]: 0.1})
    sess = dg.Session()
    gv = sess.run(opt.grads_vars, feed_dict=f)
    w1, w2, dec = _weights(model, edge_types)
    # the feature tuple in the device's nonzero order (rows ascending, feed order inside a row)
    fc, fv, fs = data.features[1]
    order = np.argsort(np.asarray(fc)[:, 0], kind="stable")
    feat1 = (np.asarray(fc)[order], np.asarray(fv, np.float32)[order], fs)
    assert np.array_equal(coo_to_csr(*feat1).val, np.asarray(feat1[1], np.float32))
    nnz = len(feat1[1])
    drop1, drop2 = {}, {}
    for g, (et, K) in enumerate(edge_types.items()):
        n_j = len(data.node_lists.proteins) if et[1] == 0 else len(data.node_lists.drugs)
        m1 = nnz if et[1] == 1 else n_j
        drop1[et] = orc.dropout_scale(20180701, 1, (1 << 16) | g, K * m1, 0.9).reshape(K, m1)
        drop2[et] = orc.dropout_scale(20180701, 1, (2 << 16) | g, K * n_j * 64, 0.9).reshape(K, n_j, 64)
    feats = {0: None, 1: feat1}
    cost, ref = orc.train_grads(edge_types, adj, feats, w1, w2, model.decoders, dec, 32, batch, neg, e, 1, 1, 0.1,
                                drop1=drop1, drop2=drop2)
    want = []
    for et, K in edge_types.items():
        want += [ref["w1"][et][k] for k in range(K)]
    for et, K in edge_types.items():
        want += [ref["w2"][et][k] for k in range(K)]
    for et in edge_types:
        want += [ref["dec"][et][nm] for nm in model.edge_type2decoder[et].vars]
    checked = 0
    for (g_, _), w in zip(gv, want):
        scale = np.max(np.abs(w))
        if scale == 0:
            assert np.max(np.abs(g_)) == 0.0
        else:
            checked += 1
            assert np.max(np.abs(g_ - w)) <= TOL * scale, f"gradient off by {rel_err(g_, w):.2e}"
    assert checked > 0
    # the masks matter: the dropout-free gradient of the drug feature weights differs
    _, ref0 = orc.train_grads(edge_types, adj, feats, w1, w2, model.decoders, dec, 32, batch, neg, e, 1, 1, 0.1)
    assert any(rel_err(ref0["w1"][(1, 1)][k], ref["w1"][(1, 1)][k]) > 1e-3 for k in range(edge_types[(1, 1)])
               if np.any(ref["w1"][(1, 1)][k]))
    # and opt_op trains with it (main.py's loop)
    c0 = float(sess.run(opt.cost, feed_dict={**f, ph["dropout"]: 0.0}))
    for _ in range(5):
        sess.run(opt.opt_op, feed_dict=f)
    assert float(sess.run(opt.cost, feed_dict={**f, ph["dropout"]: 0.0})) < c0
