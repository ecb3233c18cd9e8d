"""CPU: the oracle's hand-written training gradients (oracle/decagon_oracle.train_grads)
against torch.autograd in float64 on the same config-S inputs, and its TF-Adam restatement
against the closed form of the first step.

The reference delegates both to TensorFlow 1.8 (tf.train.AdamOptimizer(...).minimize(cost),
decagon/deep/optimizer.py:108-114), which is not installable here: the gradients are pinned
by an independent autodiff of the same forward (TF op semantics written out below), not by
TF-produced values.
"""
import numpy as np
import pytest

from conftest import rel_err
from oracle import decagon_oracle as orc

torch = pytest.importorskip("torch")


def _inputs(z, b=3):
    edge_types = {(int(i), int(j)): int(k) for i, j, k in z["edge_types"]}
    decoders = {et: str(d) for et, d in zip(edge_types, z["decoders"])}
    adj = {et: [(z[f"adj_{et[0]}_{et[1]}_{k}_coords"], z[f"adj_{et[0]}_{et[1]}_{k}_values"],
                 tuple(int(s) for s in z[f"adj_{et[0]}_{et[1]}_{k}_shape"])) for k in range(K)]
           for et, K in edge_types.items()}
    w1 = {et: [z[f"w1_{et[0]}_{et[1]}_{k}"].astype(np.float64) for k in range(K)] for et, K in edge_types.items()}
    w2 = {et: [z[f"w2_{et[0]}_{et[1]}_{k}"].astype(np.float64) for k in range(K)] for et, K in edge_types.items()}
    dec = {et: {k[len(f"dec_{et[0]}_{et[1]}_"):]: z[k].astype(np.float64) for k in z.files
                if k.startswith(f"dec_{et[0]}_{et[1]}_")} for et in edge_types}
    e, rt, ct = (int(v) for v in z[f"batch{b}_meta"])
    return edge_types, decoders, adj, w1, w2, dec, z[f"batch{b}_edges"], z[f"batch{b}_neg"], e, rt, ct


def _torch_cost(edge_types, decoders, adj, w1, w2, dec, batch, neg, e, rt, ct, margin, drop1=None, drop2=None,
                feats=None):
    """The same cost with torch autograd (float64, dense adjacencies; optional dropout masks
    applied as layers.py:87-88 / :112 do; feats[j]: sparse features, whose values drop1
    masks per relation)."""
    feats = feats or {}
    T = lambda a: torch.tensor(np.asarray(a), dtype=torch.float64, requires_grad=True)  # noqa: E731
    tw1 = {et: [T(w) for w in ws] for et, ws in w1.items()}
    tw2 = {et: [T(w) for w in ws] for et, ws in w2.items()}
    tdec = {et: {k: T(v) for k, v in p.items()} for et, p in dec.items()}

    def dense(coo):
        c, v, s = coo
        m = torch.zeros(s, dtype=torch.float64)
        m.index_put_((torch.as_tensor(c[:, 0]).long(), torch.as_tensor(c[:, 1]).long()),
                     torch.as_tensor(v, dtype=torch.float64), accumulate=True)
        return m

    A = {et: [dense(a) for a in v] for et, v in adj.items()}

    def l2n(x):  # tf.nn.l2_normalize
        return x * torch.rsqrt(torch.maximum((x * x).sum(1, keepdim=True), torch.tensor(1e-12, dtype=torch.float64)))

    D1 = (lambda et, k: torch.as_tensor(drop1[et][k], dtype=torch.float64)[:, None]) if drop1 is not None \
        else (lambda et, k: 1.0)
    D2 = (lambda et, k: torch.as_tensor(drop2[et][k], dtype=torch.float64)) if drop2 is not None \
        else (lambda et, k: 1.0)
    def x1(et, k, w):
        f = feats.get(et[1])
        if f is None:
            return D1(et, k) * w
        c, v, sh = f
        v = np.asarray(v, np.float64) * (1.0 if drop1 is None else np.asarray(drop1[et][k], np.float64))
        return dense((c, v, sh)) @ w

    pre1 = {}
    for (i, j) in edge_types:
        s = sum(a @ x1((i, j), k, w) for k, (a, w) in enumerate(zip(A[i, j], tw1[i, j])))
        pre1[i] = pre1.get(i, 0) + l2n(s)
    h1 = {i: torch.relu(v) for i, v in pre1.items()}
    E = {}
    for (i, j) in edge_types:
        s = sum(a @ ((D2((i, j), k) * h1[j]) @ w) for k, (a, w) in enumerate(zip(A[i, j], tw2[i, j])))
        E[i] = E.get(i, 0) + l2n(s)
    flat = 0
    G = L = None
    d = 32
    for et in edge_types:
        for k in range(edge_types[et]):
            if flat == e:
                kind, p = decoders[et], tdec[et]
                if kind == "dedicom":
                    G, L = p["global_interaction"], torch.diag(p["local_variation_%d" % k])
                elif kind == "bilinear":
                    G, L = p["relation_%d" % k], torch.eye(d, dtype=torch.float64)
                elif kind == "distmult":
                    G, L = torch.diag(p["relation_%d" % k]), torch.eye(d, dtype=torch.float64)
                else:
                    G = L = torch.eye(d, dtype=torch.float64)
            flat += 1
    rows, cols = torch.as_tensor(batch[:, 0]).long(), torch.as_tensor(batch[:, 1]).long()
    negr = torch.as_tensor(np.asarray(neg)).long()
    M = L @ G @ L
    pos = ((E[rt][rows] @ M) * E[ct][cols]).sum(1)
    ng = ((E[rt][negr] @ M) * E[ct][cols]).sum(1)
    cost = torch.relu(ng - (pos - margin)).sum()
    cost.backward()
    return cost, tw1, tw2, tdec


def _masks(edge_types, adj, keep, step=1):
    """Dropout masks of every group as the device draws them (tags: decagon_amd.engine.drop_tag)."""
    drop1, drop2 = {}, {}
    for g, (et, K) in enumerate(edge_types.items()):
        n_j = int(adj[et][0][2][1])
        drop1[et] = orc.dropout_scale(20180701, step, (1 << 16) | g, K * n_j, keep).reshape(K, n_j)
        drop2[et] = orc.dropout_scale(20180701, step, (2 << 16) | g, K * n_j * 64, keep).reshape(K, n_j, 64)
    return drop1, drop2


@pytest.mark.parametrize("b,dropout", [(0, False), (3, False), (3, True)])
def test_oracle_grads_match_autograd(golden_S, b, dropout):
    args = _inputs(golden_S, b)
    edge_types, decoders, adj, w1, w2, dec, batch, neg, e, rt, ct = args
    feats = {0: None, 1: None}
    drop1, drop2 = _masks(edge_types, adj, 0.9) if dropout else (None, None)
    cost, g = orc.train_grads(edge_types, adj, feats, w1, w2, decoders, dec, 32, batch, neg, e, rt, ct, 0.1,
                              drop1=drop1, drop2=drop2)
    tcost, tw1, tw2, tdec = _torch_cost(*args, 0.1, drop1=drop1, drop2=drop2)
    assert abs(cost - float(tcost)) <= 1e-12 * max(1.0, abs(cost))
    if not dropout:
        assert abs(cost - float(golden_S[f"batch{b}_cost"])) <= 1e-9 * max(1.0, abs(cost))
    for et in edge_types:
        for k in range(edge_types[et]):
            for mine, t in ((g["w1"][et][k], tw1[et][k]), (g["w2"][et][k], tw2[et][k])):
                # autograd leaves .grad None where the cost does not reach; TF's concat /
                # gather gradients make those dense zeros
                ref = t.grad.numpy() if t.grad is not None else np.zeros_like(mine)
                assert np.max(np.abs(mine - ref)) <= 1e-10 * max(1e-30, np.max(np.abs(ref)))
        for name, t in tdec[et].items():
            ref = t.grad.numpy() if t.grad is not None else np.zeros_like(g["dec"][et][name])
            assert np.max(np.abs(g["dec"][et][name] - ref)) <= 1e-10 * max(1e-30, np.max(np.abs(ref)))
    # the batch's relation moves: some W2 of the batch's row type has a nonzero gradient
    assert any(np.any(w) for ws in g["w2"].values() for w in ws)


def test_adam_first_step_closed_form():
    rng = np.random.default_rng(0)
    p = rng.standard_normal(100).astype(np.float32)
    g = rng.standard_normal(100).astype(np.float32)
    z = np.zeros(100, np.float32)
    p1, m1, v1 = orc.adam_tf(p, g, z, z, 1)
    # t = 1: m = 0.1 g, v = 0.001 g², alpha = lr·sqrt(0.001)/0.1 → step ≈ lr·sign(g)
    assert np.allclose(m1, 0.1 * g, rtol=1e-6) and np.allclose(v1, 0.001 * g * g, rtol=1e-4)
    assert np.allclose(p - p1, 0.001 * np.sign(g), rtol=1e-4, atol=1e-7)
    # zero gradient on fresh slots leaves the parameter unchanged; on warm slots it moves
    p2, m2, v2 = orc.adam_tf(p1, z, m1, v1, 2)
    assert np.all(np.abs(p2 - p1) > 0)
    p3, _, _ = orc.adam_tf(p, z, z, z, 1)
    assert np.array_equal(p3, p)


def test_dropout_masks_distribution():
    """The restated draw keeps ~keep of the elements, independently per stream and step."""
    a = orc.dropout_scale(7, 1, 3, 200000, 0.9)
    b = orc.dropout_scale(7, 2, 3, 200000, 0.9)
    c = orc.dropout_scale(7, 1, 4, 200000, 0.9)
    for m in (a, b, c):
        assert abs((m > 0).mean() - 0.9) < 0.005
        assert set(np.unique(m)) <= {np.float32(0.0), np.float32(1 / np.float32(0.9))}
    assert 0.79 < ((a > 0) == (b > 0)).mean() < 0.85  # independent draws agree on ~0.82
    assert 0.79 < ((a > 0) == (c > 0)).mean() < 0.85


def test_apk_restatement_matches_reference():
    """oracle.apk against the reference's own rank_metrics.apk (decagon/utility/rank_metrics.py,
    numpy-only, imported from /root/reference when present — this container)."""
    import importlib.util
    import os

    path = "/root/reference/decagon/utility/rank_metrics.py"
    if not os.path.exists(path):
        pytest.skip("reference tree not present (GPU box)")
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    spec = importlib.util.spec_from_file_location("ref_rank_metrics", path)
    mod = importlib.util.module_from_spec(spec)
    import sys
    sys.dont_write_bytecode = True
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(4)
    for n, k in ((100, 50), (30, 50), (500, 10)):
        scores = rng.integers(0, 15, n).astype(float)
        actual = list(range(n // 3))
        predicted = [i for _, i in sorted(zip(scores.tolist(), range(n)), reverse=True, key=lambda t: t[0])]
        assert orc.apk(actual, predicted, k) == mod.apk(actual, predicted, k)


@pytest.mark.parametrize("dropout", [False, True])
def test_oracle_grads_with_sparse_feature_dropout_match_autograd(golden_S, dropout):
    """dropout_sparse on sparse drug features (layers.py:23-31, :88): relation k's own mask
    over X_j's values (oracle drop1[et] [K, nnz]) — forward and every gradient against
    autograd of the masked dense product."""
    edge_types, decoders, adj, w1, w2, dec, batch, neg, e, rt, ct = _inputs(golden_S, 3)
    rng = np.random.default_rng(9)
    F = 37
    m = (rng.random((400, F)) < 0.15) * rng.uniform(0.2, 1.0, (400, F))
    r, c = np.nonzero(m)
    feat = (np.stack([r, c], 1), m[r, c], (400, F))
    feats = {0: None, 1: feat}
    for et in edge_types:
        if et[1] == 1:
            w1[et] = [rng.uniform(-0.2, 0.2, (F, 64)) for _ in range(edge_types[et])]
    drop1 = None
    if dropout:
        drop1, _ = _masks(edge_types, adj, 0.9)
        for g, (et, K) in enumerate(edge_types.items()):
            if et[1] == 1:
                drop1[et] = orc.dropout_scale(20180701, 1, (1 << 16) | g, K * len(r), 0.9).reshape(K, len(r))
    cost, g = orc.train_grads(edge_types, adj, feats, w1, w2, decoders, dec, 32, batch, neg, e, rt, ct, 0.1,
                              drop1=drop1)
    tcost, tw1, tw2, tdec = _torch_cost(edge_types, decoders, adj, w1, w2, dec, batch, neg, e, rt, ct, 0.1,
                                        drop1=drop1, feats=feats)
    assert abs(cost - float(tcost)) <= 1e-12 * max(1.0, abs(cost))
    for et in edge_types:
        for k in range(edge_types[et]):
            for mine, t in ((g["w1"][et][k], tw1[et][k]), (g["w2"][et][k], tw2[et][k])):
                want = t.grad.numpy() if t.grad is not None else np.zeros_like(mine)
                assert np.max(np.abs(mine - want)) <= 1e-10 * max(1.0, np.max(np.abs(want)))
