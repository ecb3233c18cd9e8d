"""Negative-sampling tables (host side, built once per relation).

tf.nn.fixed_unigram_candidate_sampler(distortion=0.75, unique=False)
(decagon/deep/optimizer.py:40-47) draws class c with probability ∝ degree_c^0.75.  The
device sampler (dg_unigram_sample / dg_decoder_hinge_f32) draws from a Walker alias table:
entry j = {acceptance probability q_j (float32 bits), alias a_j}; a draw picks j uniformly
and keeps it with probability q_j, else takes a_j — O(1), one 8-byte load per draw.
Built with Vose's method in float64; zero-weight classes are never drawn.
"""
from __future__ import annotations

import numpy as np


def alias_table(degrees, distortion: float = 0.75) -> np.ndarray:
    """uint32 [range, 2] table for p ∝ degrees^distortion."""
    w = np.power(np.asarray(degrees, np.float64), distortion)
    n = w.shape[0]
    if n == 0 or not np.isfinite(w).all() or w.sum() <= 0:
        raise ValueError("unigram sampler needs finite, non-negative degrees with a positive sum")
    prob = w * (n / w.sum())
    alias = np.arange(n, dtype=np.int64)
    q = np.ones(n, np.float64)
    small = [i for i in range(n) if prob[i] < 1.0]
    large = [i for i in range(n) if prob[i] >= 1.0]
    while small and large:
        s, l = small.pop(), large.pop()
        q[s] = prob[s]
        alias[s] = l
        prob[l] = (prob[l] + prob[s]) - 1.0
        (small if prob[l] < 1.0 else large).append(l)
    for i in small + large:  # numerical leftovers keep themselves
        q[i] = 1.0
        alias[i] = i
    # a zero-weight entry must never keep itself: its alias carries all of its mass
    q[w == 0] = 0.0
    out = np.empty((n, 2), np.uint32)
    out[:, 0] = q.astype(np.float32).view(np.uint32)
    out[:, 1] = alias.astype(np.uint32)
    return out


def table_distribution(table: np.ndarray) -> np.ndarray:
    """The exact distribution an alias table encodes (for tests)."""
    n = table.shape[0]
    q = table[:, 0].view(np.float32).astype(np.float64)
    a = table[:, 1].astype(np.int64)
    p = q / n
    np.add.at(p, a, (1.0 - q) / n)
    return p
