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
