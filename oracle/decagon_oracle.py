"""ORACLE — test infrastructure only.  CPU restatement of the reference's GCN forward,
edge decoders and losses, in float64 numpy.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
and only as the checker (or the timed CPU baseline) — never as the product path.

What it restates (paths relative to the reference root, jrectorb/decagon):
  GraphConvolutionSparseMulti._call   decagon/deep/layers.py:85-94
  GraphConvolutionMulti._call         decagon/deep/layers.py:109-118
  DecagonModel._build                 decagon/deep/model.py:64-137
  DecagonOptimizer.batch_predict      decagon/deep/optimizer.py:63-85
  DecagonOptimizer.predict            decagon/deep/optimizer.py:87-106
  DecagonOptimizer._hinge_loss/_xent  decagon/deep/optimizer.py:116-127
with TF 1.8 op semantics: l2_normalize = x * rsqrt(max(sum x², 1e-12));
sparse_tensor_dense_matmul visits nonzeros in feed order; dropout = 0 is the identity.

Parity pinning: TensorFlow 1.8 — the library that executes these ops in
the reference (requirements.txt:22) — is absent from this image and not installable
offline, so the reference's forward cannot be run.  The INPUTS of every golden fixture are
produced by the reference's own code (EdgeMinibatchIterator / preprocess_graph imported
from /root/reference by tests/golden/make_golden.py); the OUTPUTS are this restatement.  The
DEDICOM contraction is additionally cross-checked against the reference's numpy predictor
formula E·D·R·D·Eᵀ (main/Predictor/NpPredictor.py:304) on the reference's own trained R and
D_r artifacts.  Output parity is therefore pinned on reference inputs + restated outputs,
not on TF-produced outputs.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

EPS_L2 = 1e-12


def sparse_dense_matmul(coo, dense: np.ndarray) -> np.ndarray:
    """tf.sparse_tensor_dense_matmul(A, X) (layers.py:89-90, :114): out[r] += v * X[c] in
    nonzero order (float64 here)."""
    coords, values, shape = coo
    coords = np.asarray(coords, dtype=np.int64).reshape(-1, 2)
    values = np.asarray(values, dtype=np.float64)
    out = np.zeros((int(shape[0]), dense.shape[1]), dtype=np.float64)
    if coords.shape[0]:
        np.add.at(out, coords[:, 0], values[:, None] * dense[coords[:, 1]])
    return out


def l2_normalize_rows(x: np.ndarray) -> np.ndarray:
    """tf.nn.l2_normalize(x, dim=1) (layers.py:93, :117)."""
    ss = np.sum(x * x, axis=1, keepdims=True)
    return x / np.sqrt(np.maximum(ss, EPS_L2))


def _features_times(feat, w: np.ndarray) -> np.ndarray:
    # dropout_sparse at keep_prob 1 is the identity (layers.py:23-31, :88)
    return sparse_dense_matmul(feat, w)


def gcn_layer_sparse(adj: Sequence, feat, weights: Sequence[np.ndarray]) -> np.ndarray:
    """GraphConvolutionSparseMulti._call, act = identity as DecagonModel passes it
    (layers.py:85-94, model.py:71)."""
    outs = [sparse_dense_matmul(a, _features_times(feat, w)) for a, w in zip(adj, weights)]
    return l2_normalize_rows(np.sum(outs, axis=0))


def gcn_layer_dense(adj: Sequence, h: np.ndarray, weights: Sequence[np.ndarray]) -> np.ndarray:
    """GraphConvolutionMulti._call, act = identity (layers.py:109-118, model.py:83)."""
    outs = [sparse_dense_matmul(a, h @ w) for a, w in zip(adj, weights)]
    return l2_normalize_rows(np.sum(outs, axis=0))


def decagon_forward(edge_types: Dict[Tuple[int, int], int], adj: Dict[Tuple[int, int], List],
                    feats: Dict[int, tuple], w1: Dict[Tuple[int, int], List[np.ndarray]],
                    w2: Dict[Tuple[int, int], List[np.ndarray]]):
    """DecagonModel._build forward (model.py:64-88).  Returns (hidden1 dict, embeddings list)."""
    hidden1: Dict[int, List[np.ndarray]] = {}
    for (i, j) in edge_types:
        hidden1.setdefault(i, []).append(gcn_layer_sparse(adj[i, j], feats[j], w1[i, j]))
    h1 = {i: np.maximum(np.sum(v, axis=0), 0.0) for i, v in hidden1.items()}  # model.py:74-75
    emb: Dict[int, List[np.ndarray]] = {}
    for (i, j) in edge_types:
        emb.setdefault(i, []).append(gcn_layer_dense(adj[i, j], h1[j], w2[i, j]))
    n_types = max(i for i, _ in edge_types) + 1
    embeddings = [None] * n_types
    for i, v in emb.items():
        embeddings[i] = np.sum(v, axis=0)  # model.py:85-88 (no relu)
    return h1, embeddings


def decagon_forward_csr(edge_types: Dict[Tuple[int, int], int], adj_csr: Dict[Tuple[int, int], List],
                        w1: Dict[Tuple[int, int], np.ndarray], w2: Dict[Tuple[int, int], np.ndarray]):
    """decagon_forward for identity features at full size: the same layers (layers.py:85-94,
    109-118; model.py:64-88) with each Â_k a float64 scipy CSR and W stacks [K, F, d]
    (float64), products by scipy (summation order is immaterial in float64)."""
    def layer(x_of):
        acc: Dict[int, np.ndarray] = {}
        for (i, j) in edge_types:
            s = sum(adj_csr[i, j][k] @ x_of(i, j, k) for k in range(edge_types[i, j]))
            acc[i] = acc.get(i, 0) + l2_normalize_rows(np.asarray(s))
        return acc
    h1 = {i: np.maximum(v, 0.0) for i, v in layer(lambda i, j, k: w1[i, j][k]).items()}
    emb = layer(lambda i, j, k: h1[j] @ w2[i, j][k])
    return h1, emb


def latent_matrices(edge_types, decoders, dec_params, d: int):
    """latent_inters / latent_varies in edge-type order (model.py:116-137).

    dec_params[(i,j)] holds the decoder variables: 'relation_k' (distmult: [d], bilinear:
    [d,d]), 'global_interaction' [d,d] and 'local_variation_k' [d] (dedicom)."""
    inters, varies = [], []
    for et in edge_types:
        kind = decoders[et]
        p = dec_params.get(et, {})
        for k in range(edge_types[et]):
            if kind == "innerproduct":
                g, l = np.eye(d), np.eye(d)
            elif kind == "distmult":
                g, l = np.diag(p["relation_%d" % k]), np.eye(d)
            elif kind == "bilinear":
                g, l = p["relation_%d" % k], np.eye(d)
            elif kind == "dedicom":
                g, l = p["global_interaction"], np.diag(p["local_variation_%d" % k])
            else:
                raise ValueError("Unknown decoder type")
            inters.append(np.asarray(g, np.float64))
            varies.append(np.asarray(l, np.float64))
    return inters, varies


def batch_predict(embeddings, row_type: int, col_type: int, G: np.ndarray, L: np.ndarray,
                  rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    """optimizer.py:63-85 literally: the full B×B product, then its diagonal (:51-57)."""
    u = embeddings[row_type][np.asarray(rows)]
    v = embeddings[col_type][np.asarray(cols)]
    preds = ((u @ L) @ G @ L) @ v.T
    return np.diag(preds).copy()


def predict(embeddings, row_type: int, col_type: int, G: np.ndarray, L: np.ndarray) -> np.ndarray:
    """optimizer.py:87-106: E_i·L·G·L·E_jᵀ."""
    return ((embeddings[row_type] @ L) @ G @ L) @ embeddings[col_type].T


def hinge_loss(pos: np.ndarray, neg: np.ndarray, margin: float) -> float:
    """optimizer.py:116-120: sum(relu(neg - (pos - margin)))."""
    return float(np.sum(np.maximum(neg - (pos - margin), 0.0)))


def xent_loss(pos: np.ndarray, neg: np.ndarray, neg_weight: float) -> float:
    """optimizer.py:122-127 with sigmoid_cross_entropy_with_logits."""
    def sce(x, z):
        return np.maximum(x, 0) - x * z + np.log1p(np.exp(-np.abs(x)))
    return float(np.sum(sce(pos, 1.0)) + neg_weight * np.sum(sce(neg, 0.0)))


def np_predictor_dedicom(e_row: np.ndarray, e_col: np.ndarray, D: np.ndarray, R: np.ndarray):
    """The reference's offline numpy DEDICOM scorer, E·D·R·D·Eᵀ
    (main/Predictor/NpPredictor.py:304), used to cross-check `predict`."""
    return e_row @ D @ R @ D @ e_col.T


def unigram_distribution(degrees: np.ndarray, distortion: float = 0.75) -> np.ndarray:
    """Probabilities of tf.nn.fixed_unigram_candidate_sampler (optimizer.py:40-47)."""
    w = np.power(np.asarray(degrees, np.float64), distortion)
    return w / w.sum()


# ----------------------------------------------------------------------------------------
# Training step: gradients of the hinge cost and TF 1.8's Adam update
# (DecagonOptimizer._build, decagon/deep/optimizer.py:108-114).  The reference delegates
# both to TensorFlow (tf.train.AdamOptimizer(...).minimize(cost)); restated here by hand:
# reverse-mode through model.py:64-88 and optimizer.py:51-57, 116-120.
# ----------------------------------------------------------------------------------------
def sparse_t_dense_matmul(coo, dense: np.ndarray, n_cols: int) -> np.ndarray:
    """Aᵀ·G: the gradient of tf.sparse_tensor_dense_matmul(A, X) w.r.t. X."""
    coords, values, _ = coo
    coords = np.asarray(coords, dtype=np.int64).reshape(-1, 2)
    values = np.asarray(values, dtype=np.float64)
    out = np.zeros((n_cols, dense.shape[1]), dtype=np.float64)
    if coords.shape[0]:
        np.add.at(out, coords[:, 1], values[:, None] * dense[coords[:, 0]])
    return out


def l2_normalize_rows_grad(x: np.ndarray, dy: np.ndarray) -> np.ndarray:
    """Gradient of tf.nn.l2_normalize(x, dim=1) = x·rsqrt(max(Σx², ε)): the max passes its
    gradient to Σx² where Σx² >= ε (tf.maximum's gradient mask), so
        dx = dy·inv − x·inv³·(x·dy)·[Σx² >= ε],  inv = rsqrt(max(Σx², ε))."""
    ss = np.sum(x * x, axis=1, keepdims=True)
    inv = 1.0 / np.sqrt(np.maximum(ss, EPS_L2))
    dot = np.sum(x * dy, axis=1, keepdims=True)
    return dy * inv - x * (inv ** 3) * dot * (ss >= EPS_L2)


def _lowbias32(x):
    x = np.asarray(x, np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = (x * np.uint32(0x7FEB352D)).astype(np.uint32)
    x = x ^ (x >> np.uint32(15))
    x = (x * np.uint32(0x846CA68B)).astype(np.uint32)
    return x ^ (x >> np.uint32(16))


def dropout_scale(seed: int, step: int, tag: int, n: int, keep: float) -> np.ndarray:
    """The dropout masks of stream `tag` at (seed, step), elements 0..n-1, as the device draws
    them (decagon_amd/csrc/dropout.h): element idx kept iff lowbias32(key ^ idx) >> 8 <
    (uint32)(keep·2^24), scaled by 1/keep (float32).  TF's own RNG stream cannot be reproduced;
    this restates the device's draw so forward and backward are checked on identical masks."""
    with np.errstate(over="ignore"):
        lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
        k1 = _lowbias32(lo ^ np.uint32((tag * 0x9E3779B9) & 0xFFFFFFFF))
        key = _lowbias32(k1 ^ np.uint32((int(hi) + step * 0x85EBCA6B) & 0xFFFFFFFF))
        h = _lowbias32(key ^ np.arange(n, dtype=np.uint32))
    thr = np.uint32(np.float32(keep) * np.float32(16777216.0))
    inv = np.float32(1.0) / np.float32(keep)
    return np.where((h >> np.uint32(8)) < thr, inv, np.float32(0.0)).astype(np.float32)


def train_grads(edge_types, adj, feats, w1, w2, decoders, dec_params, d2: int, batch, neg, e: int,
                rt: int, ct: int, margin: float, drop1=None, drop2=None):
    """Forward (model.py:64-88, optimizer.py:51-57) and the hinge cost's gradient w.r.t.
    every variable, as TF's minimize() computes it (float64).

    feats[j] is None for identity features.  batch [B, 2] local (row, col) ids of the edge
    type; neg [B] the negative row ids; e the flat relation index (edge-type order).
    Returns (cost, grads) with grads = {"w1": {et: [K arrays]}, "w2": {...},
    "dec": {et: {var name: array}}} — every variable gets a gradient (zeros when the cost
    does not reach it: TF's gather/concat gradients are dense zeros, not None).
    Dropout (layers.py:87-88, :112): drop1[et] [K, n_j] scales rows of relation k's layer-1
    operand (dropout_sparse on the identity features) — or, for sparse features, drop1[et]
    [K, nnz_j] scales relation k's copy of X_j's values (dropout_sparse on the feature tuple,
    in its nonzero order); drop2[et] [K, n_j, h1] the elements of H1_j fed to relation k's
    projection (tf.nn.dropout); None = no dropout."""
    ets = list(edge_types)
    n_nodes = {}
    for (i, j) in ets:
        n_nodes[i] = int(adj[i, j][0][2][0])
        n_nodes[j] = int(adj[i, j][0][2][1])
    def feat_k(j, et, k):  # relation k's (dropped-out) copy of X_j
        c, v, sh = feats[j]
        if drop1 is None:
            return feats[j]
        return c, np.asarray(v, np.float64) * np.asarray(drop1[et][k], np.float64), sh

    x1 = {}
    for (i, j) in ets:
        if feats.get(j) is None:
            x1[i, j] = list(w1[i, j])
            if drop1 is not None:
                x1[i, j] = [x * drop1[i, j][k][:, None] for k, x in enumerate(x1[i, j])]
        else:
            x1[i, j] = [_features_times(feat_k(j, (i, j), k), w) for k, w in enumerate(w1[i, j])]
    hin = (lambda et, k, h: h * drop2[et][k]) if drop2 is not None else (lambda et, k, h: h)
    S1 = {et: np.sum([sparse_dense_matmul(a, x) for a, x in zip(adj[et], x1[et])], axis=0) for et in ets}
    pre1 = {}
    for (i, j) in ets:
        pre1[i] = pre1.get(i, 0.0) + l2_normalize_rows(S1[i, j])
    H1 = {i: np.maximum(v, 0.0) for i, v in pre1.items()}
    P = {(i, j): [hin((i, j), k, H1[j]) @ w for k, w in enumerate(w2[i, j])] for (i, j) in ets}
    S2 = {et: np.sum([sparse_dense_matmul(a, p) for a, p in zip(adj[et], P[et])], axis=0) for et in ets}
    E = {}
    for (i, j) in ets:
        E[i] = E.get(i, 0.0) + l2_normalize_rows(S2[i, j])

    inters, varies = latent_matrices(edge_types, decoders, dec_params, d2)
    G, L = inters[e], varies[e]
    M = L @ G @ L
    rows, cols = np.asarray(batch)[:, 0], np.asarray(batch)[:, 1]
    neg = np.asarray(neg)
    u, v, un = E[rt][rows], E[ct][cols], E[rt][neg]
    pos = np.sum((u @ M) * v, axis=1)
    negs = np.sum((un @ M) * v, axis=1)
    z = negs - (pos - margin)
    cost = float(np.sum(np.maximum(z, 0.0)))
    act = (z > 0).astype(np.float64)           # tf.nn.relu's gradient mask
    dpos, dneg = -act, act
    dM = u.T @ (dpos[:, None] * v) + un.T @ (dneg[:, None] * v)
    dE = {i: np.zeros_like(E[i]) for i in E}
    np.add.at(dE[rt], rows, dpos[:, None] * (v @ M.T))
    np.add.at(dE[rt], neg, dneg[:, None] * (v @ M.T))
    np.add.at(dE[ct], cols, dpos[:, None] * (u @ M) + dneg[:, None] * (un @ M))
    dG = L.T @ dM @ L.T                          # M = L·G·L
    dL = dM @ (G @ L).T + (L @ G).T @ dM

    # decoder variables: only relation e's entries of latent_inters / latent_varies get a
    # nonzero gradient; the rest are zeros of the variables' shapes
    dec = {}
    flat = 0
    for et in ets:
        kind = decoders[et]
        p = dec_params.get(et, {})
        g = {name: np.zeros_like(np.asarray(val, np.float64)) for name, val in p.items()}
        for k in range(edge_types[et]):
            if flat == e:
                if kind == "distmult":
                    g["relation_%d" % k] += np.diag(dG)
                elif kind == "bilinear":
                    g["relation_%d" % k] += dG
                elif kind == "dedicom":
                    g["global_interaction"] += dG
                    g["local_variation_%d" % k] += np.diag(dL)
            flat += 1
        dec[et] = g

    gw2, dH1 = {}, {j: np.zeros_like(H1[j]) for j in H1}
    for (i, j) in ets:
        dS2 = l2_normalize_rows_grad(S2[i, j], dE[i])
        gw2[i, j] = []
        for k, (a, w) in enumerate(zip(adj[i, j], w2[i, j])):
            dP = sparse_t_dense_matmul(a, dS2, n_nodes[j])
            gw2[i, j].append(hin((i, j), k, H1[j]).T @ dP)
            dH1[j] += hin((i, j), k, dP @ w.T)
    dpre1 = {i: dH1[i] * (pre1[i] > 0) for i in dH1}   # tf.nn.relu's gradient mask (model.py:75)
    gw1 = {}
    for (i, j) in ets:
        dS1 = l2_normalize_rows_grad(S1[i, j], dpre1[i])
        gw1[i, j] = []
        for k, a in enumerate(adj[i, j]):
            dX = sparse_t_dense_matmul(a, dS1, n_nodes[j])
            if feats.get(j) is not None:
                fk = feat_k(j, (i, j), k)
                dX = sparse_t_dense_matmul(fk, dX, int(fk[2][1]))
            elif drop1 is not None:
                dX = dX * drop1[i, j][k][:, None]
            gw1[i, j].append(dX)
    return cost, {"w1": gw1, "w2": gw2, "dec": dec}


def adam_tf(param: np.ndarray, grad: np.ndarray, m: np.ndarray, v: np.ndarray, t: int,
            lr: float = 0.001, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
    """One tf.train.AdamOptimizer step (TF 1.8 ApplyAdam, use_nesterov=False) in float32,
    as TF runs it on float32 variables; t is the 1-based step.  The beta powers are float32
    variables multiplied by beta once per step, and
        alpha = lr·sqrt(1 − β2^t)/(1 − β1^t);  m += (g − m)(1 − β1);  v += (g² − v)(1 − β2);
        param −= alpha·m / (sqrt(v) + ε).
    Returns new (param, m, v) as float32."""
    f = np.float32
    b1p, b2p = f(beta1), f(beta2)
    for _ in range(t - 1):
        b1p, b2p = f(b1p * f(beta1)), f(b2p * f(beta2))
    alpha = f(f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p))
    g = np.asarray(grad, np.float32)
    m = (m + (g - m) * (f(1) - f(beta1))).astype(np.float32)
    v = (v + (g * g - v) * (f(1) - f(beta2))).astype(np.float32)
    p = (param - (m * alpha) / (np.sqrt(v) + f(eps))).astype(np.float32)
    return p, m, v


# ----------------------------------------------------------------------------------------
# Evaluation path: get_accuracy_scores (main.py:38-80)
# ----------------------------------------------------------------------------------------
def apk(actual, predicted, k: int = 10) -> float:
    """rank_metrics.apk (decagon/utility/rank_metrics.py:4-40), restated."""
    if len(predicted) > k:
        predicted = predicted[:k]
    score, num_hits = 0.0, 0.0
    seen = set()
    actual = set(actual)
    for i, p in enumerate(predicted):
        if p in actual and p not in seen:
            num_hits += 1.0
            score += num_hits / (i + 1.0)
        seen.add(p)
    if not actual:
        return 0.0
    return score / min(len(actual), k)


def sigmoid_np114(logits, form: str = "main") -> np.ndarray:
    """The scores the reference ranks, from TF's float32 logits, under numpy 1.14
    (requirements.txt:14; value-based casting, pre-NEP 50):

      "main"       main.py:51-52 `1. / (1 + np.exp(-x))` on a float32 scalar rec[u, v]:
                   np.exp runs in float32 (libm expf — correctly rounded, restated as the
                   float64 exp rounded to float32), `1 + e` and `1. / …` promote to float64;
                   then np.nan_to_num (main.py:81)
      "evaluator"  MathUtils.sigmoid (main/Utils/MathUtils.py:3-4) on the float32 decoder
                   output ARRAY (DecagonAccuracyEvaluator.py:123): every step stays float32
    """
    x = np.asarray(logits, np.float32)
    with np.errstate(over="ignore", invalid="ignore"):
        e = np.exp(-x.astype(np.float64)).astype(np.float32)
    if form == "main":
        with np.errstate(over="ignore"):
            return np.nan_to_num(1.0 / (1.0 + e.astype(np.float64)))
    if form == "evaluator":
        with np.errstate(over="ignore"):
            return (np.float32(1.0) / (np.float32(1.0) + e)).astype(np.float32)
    raise ValueError(form)


def accuracy_scores(pos_scores: np.ndarray, neg_scores: np.ndarray, k: int = 50, sigmoid="main"):
    """(roc, auprc, apk@k) as get_accuracy_scores forms them (main.py:38-90): the LOGITS of the
    positive and negative edges go through the reference's sigmoid (`sigmoid_np114`; None:
    ranked as given), labels 1 for the positives then 0 for the negatives; `predicted` = edge
    indices sorted by score, descending, Python's stable sort (main.py:84)."""
    from sklearn import metrics

    if sigmoid is not None:
        pos_scores, neg_scores = sigmoid_np114(pos_scores, sigmoid), sigmoid_np114(neg_scores, sigmoid)
    pos = np.asarray(pos_scores, np.float64)
    neg = np.asarray(neg_scores, np.float64)
    preds_all = np.hstack([pos, neg])
    labels_all = np.hstack([np.ones(len(pos)), np.zeros(len(neg))])
    predicted = [i for _, i in sorted(zip(preds_all.tolist(), range(len(preds_all))), reverse=True,
                                      key=lambda t: t[0])]
    roc = metrics.roc_auc_score(labels_all, preds_all)
    aupr = metrics.average_precision_score(labels_all, preds_all)
    return roc, aupr, apk(list(range(len(pos))), predicted, k=k)
