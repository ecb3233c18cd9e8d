"""The evaluation path: link-prediction accuracy on the device.

Reference: `get_accuracy_scores(edges_pos, edges_neg, edge_type)` (main.py:38-80) runs
`sess.run(opt.predictions)` — the full N_i×N_j score matrix of the edge type — then, on the
host, takes sigmoid(rec[u, v]) of the sampled positive and negative edges and calls sklearn's
roc_auc_score / average_precision_score and rank_metrics.apk(k=50)
(decagon/utility/rank_metrics.py:4-40); DecagonAccuracyEvaluator (main/AccuracyEvaluators/
Tensorflow/DecagonAccuracyEvaluator.py:58-150) does the same over the drug×drug relations.

Here only the sampled pairs are scored (dg_decoder_score_f32: u·L·G·L·v per pair, no
N_i×N_j matrix) and the three metrics come from dg_rank_metrics_ex_f32, which ranks the scores
the reference ranks — not the logits: the sigmoid is monotonic but it saturates, and the
resulting ties move AUROC, AUPRC and AP@k.  `sigmoid` selects the reference's form:

  "main"       get_accuracy_scores (main.py:51-52,60,70,81) under numpy 1.14
               (requirements.txt:14): float32 exp of TF's float32 logit, float64 1/(1+e),
               nan_to_num — logits > ≈36.7 score exactly 1.0, < ≈-88.7 exactly 0.0
  "evaluator"  DecagonAccuracyEvaluator (MathUtils.sigmoid on the float32 decoder output,
               DecagonAccuracyEvaluator.py:123): all float32, logits > ≈16.6 score 1.0
  None         the raw logits
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib, kernels
from ._lib import check
from .graph import Node, RunContext


SIGMOID_MODES = {"main": _lib.DG_RANK_SIGMOID64, "evaluator": _lib.DG_RANK_SIGMOID32, None: _lib.DG_RANK_LOGIT}


def rank_metrics_device(pos: torch.Tensor, neg: torch.Tensor, k: int = 50,
                        sigmoid: Optional[str] = "main") -> torch.Tensor:
    """float64 device tensor [AUROC, AUPRC, AP@k] of device LOGIT vectors, ranked by the
    reference's sigmoid scores (module docstring; asynchronous)."""
    for t, nm in ((pos, "pos"), (neg, "neg")):
        kernels._dev(t, torch.float32, nm)
    if sigmoid not in SIGMOID_MODES:
        raise ValueError(f"sigmoid must be one of {list(SIGMOID_MODES)}")
    lib = _lib.load()
    P, N = pos.numel(), neg.numel()
    nbytes = int(lib.dg_rank_metrics_ex_workspace(P, N))
    ws = torch.empty(-(-nbytes // 8), dtype=torch.float64, device=pos.device)
    out = torch.empty(3, dtype=torch.float64, device=pos.device)
    check(lib.dg_rank_metrics_ex_f32(pos.data_ptr() if P else None, P, neg.data_ptr() if N else None, N, int(k),
                                     SIGMOID_MODES[sigmoid], out.data_ptr(), ws.data_ptr(), ws.numel() * 8,
                                     kernels._stream_ptr(None)), "dg_rank_metrics_ex_f32")
    return out


def rank_metrics(pos: torch.Tensor, neg: torch.Tensor, k: int = 50,
                 sigmoid: Optional[str] = "main") -> Tuple[float, float, float]:
    """(AUROC, AUPRC, AP@k) of device logit vectors, as roc_auc_score,
    average_precision_score and rank_metrics.apk(range(P), order of all scores) compute them
    on the reference's sigmoid scores."""
    au, ap, apk = rank_metrics_device(pos, neg, k, sigmoid).cpu().tolist()
    return au, ap, apk


def _pairs(edges) -> Tuple[np.ndarray, np.ndarray]:
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    return e[:, 0].astype(np.int32), e[:, 1].astype(np.int32)


def accuracy_scores(sess, opt, placeholders, feed_dict, edges_pos, edges_neg, edge_type, edge_type2idx,
                    k: int = 50, sigmoid: Optional[str] = "main") -> Tuple[float, float, float]:
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
        return rank_metrics_device(out[0], out[1], k, sigmoid)

    au, ap, apk = sess.run(Node("evaluate/accuracy", fn), feed_dict=fd).tolist()
    return au, ap, apk
