"""The evaluation path: link-prediction accuracy on the device.

Reference: `get_accuracy_scores(edges_pos, edges_neg, edge_type)` (main.py:38-80) runs
`sess.run(opt.predictions)` — the full N_i×N_j score matrix of the edge type — then, on the
host, takes sigmoid(rec[u, v]) of the sampled positive and negative edges and calls sklearn's
roc_auc_score / average_precision_score and rank_metrics.apk(k=50)
(decagon/utility/rank_metrics.py:4-40); DecagonAccuracyEvaluator (main/AccuracyEvaluators/
Tensorflow/DecagonAccuracyEvaluator.py:58-150) does the same over the drug×drug relations.

Here only the sampled pairs are scored (dg_decoder_score_f32: u·L·G·L·v per pair, no
N_i×N_j matrix) and the three metrics come from one dg_rank_metrics_f32 launch.  The sigmoid is
monotonic, so it is not applied: rankings — and so all three metrics — are those of the
logits (the reference's float64 sigmoid can only merge scores above |x| ≈ 36).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from . import _lib, kernels
from ._lib import check
from .graph import Node, RunContext


def rank_metrics_device(pos: torch.Tensor, neg: torch.Tensor, k: int = 50) -> torch.Tensor:
    """float64 device tensor [AUROC, AUPRC, AP@k] of device score vectors (asynchronous)."""
    for t, nm in ((pos, "pos"), (neg, "neg")):
        kernels._dev(t, torch.float32, nm)
    lib = _lib.load()
    P, N = pos.numel(), neg.numel()
    ws = torch.empty(max(4, int(lib.dg_rank_metrics_workspace(P)) // 4), dtype=torch.int32, device=pos.device)
    out = torch.empty(3, dtype=torch.float64, device=pos.device)
    check(lib.dg_rank_metrics_f32(pos.data_ptr() if P else None, P, neg.data_ptr() if N else None, N, int(k),
                                  out.data_ptr(), ws.data_ptr(), ws.numel() * 4,
                                  kernels._stream_ptr(None)), "dg_rank_metrics_f32")
    return out


def rank_metrics(pos: torch.Tensor, neg: torch.Tensor, k: int = 50) -> Tuple[float, float, float]:
    """(AUROC, AUPRC, AP@k) of device score vectors, as roc_auc_score,
    average_precision_score and rank_metrics.apk(range(P), order of all scores) compute them."""
    au, ap, apk = rank_metrics_device(pos, neg, k).cpu().tolist()
    return au, ap, apk


def _pairs(edges) -> Tuple[np.ndarray, np.ndarray]:
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    return e[:, 0].astype(np.int32), e[:, 1].astype(np.int32)


def accuracy_scores(sess, opt, placeholders, feed_dict, edges_pos, edges_neg, edge_type, edge_type2idx,
                    k: int = 50) -> Tuple[float, float, float]:
    """get_accuracy_scores (main.py:38-80) on the device: (roc, auprc, apk@k) of the edge
    type's sampled positive edges `edges_pos[edge_type[:2]][edge_type[2]]` against the sampled
    negatives, scored with the optimizer's decoder for that relation (dropout 0)."""
    fd = dict(feed_dict)
    fd[placeholders["dropout"]] = 0.0
    fd[placeholders["batch_edge_type_idx"]] = edge_type2idx[edge_type]
    fd[placeholders["batch_row_edge_type"]] = edge_type[0]
    fd[placeholders["batch_col_edge_type"]] = edge_type[1]
    pr, pc = _pairs(edges_pos[edge_type[:2]][edge_type[2]])
    nr, nc = _pairs(edges_neg[edge_type[:2]][edge_type[2]])

    def fn(ctx: RunContext):
        e, rt, ct = opt._edge(ctx)
        row_t, col_t = opt._tables(ctx, rt, ct)
        G, l = opt._latent(ctx, e)
        dev = ctx.session.device
        out = []
        for r, c in ((pr, pc), (nr, nc)):
            if r.size and (r.min() < 0 or r.max() >= row_t.shape[0] or c.min() < 0 or c.max() >= col_t.shape[0]):
                raise ValueError("edge sample outside the embedding tables")
            rd, cd = torch.from_numpy(r).to(dev), torch.from_numpy(c).to(dev)
            out.append(kernels.decoder_score(row_t, col_t, rd, cd, G, l) if r.size
                       else torch.empty(0, device=dev))
        return rank_metrics_device(out[0], out[1], k)

    au, ap, apk = sess.run(Node("evaluate/accuracy", fn), feed_dict=fd).tolist()
    return au, ap, apk
