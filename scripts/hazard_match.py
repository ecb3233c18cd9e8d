"""Explain config 5's wrong scores term by term ("The config-5 miscompile").

Input: the directory scripts/hazard_harness writes with HZ_DUMP=DIR — its inputs, the reference
build's scores (ref.bin) and a failing variant's first failing run (got_<variant>.bin).

A positive score is pp = sum_i T[i] * (u_p[i] * D_k[i]), T = R.bf16(D_k o v), and lane group g
of the wave (lanes 16g .. 16g+15, one lane per pair) accumulates the elements
i = 32q + 8g + e of q iteration q, e = 0..7.  In the failing build the odd elements' products
u_p[i] * D_k[i] are the low results of `v_pk_mul_f32 D, A, B op_sel:[0,1]`.  For every failing
half tile this script finds the smallest set (one, else two) of terms (q, e, g) whose removal
turns the reference's scores into the failing ones for all 16 pairs, and reports how well that
explains them (residual relative to the error) and which lane groups, elements and q iterations
the removed terms fall on.

Usage: python scripts/hazard_match.py DIR VARIANT
"""
from __future__ import annotations

import collections
import itertools
import sys
from pathlib import Path

import numpy as np

D, ND, SLOTS, B = 256, 645, 1928, 512


def bf16_to_f32(a: np.ndarray) -> np.ndarray:
    return (a.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16_rne(x: np.ndarray) -> np.ndarray:
    u = x.astype(np.float32).view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def main(argv) -> int:
    d, variant = Path(argv[0]), argv[1]
    E = bf16_to_f32(np.fromfile(d / "E.bin", np.uint16)).reshape(ND, D)
    R = bf16_to_f32(np.fromfile(d / "R.bin", np.uint16)).reshape(D, D).astype(np.float64)
    L = bf16_to_f32(np.fromfile(d / "L.bin", np.uint16)).reshape(SLOTS, D)
    rows = np.fromfile(d / "rows.bin", np.int32)
    cols = np.fromfile(d / "cols.bin", np.int32)
    ref = np.fromfile(d / "ref.bin", np.float32)
    got = np.fromfile(d / f"got_{variant}.bin", np.float32)
    nh = rows.size
    bad = np.flatnonzero((got[:nh].view(np.uint32) != ref[:nh].view(np.uint32)).reshape(-1, 16).any(1))
    terms_hist, where, rel = collections.Counter(), collections.Counter(), []
    for h in bad:
        tile, half = divmod(int(h), 2)
        p = tile * 32 + 16 * half + np.arange(16)
        Dk = L[p // B]
        vD = bf16_to_f32(f32_to_bf16_rne(Dk * E[cols[p]])).astype(np.float64)  # the MFMA's B operand
        T = vD @ R.T
        prod = T * (E[rows[p]].astype(np.float64) * Dk)                         # [16 pairs, D]
        obs = got[p].astype(np.float64) - ref[p]
        scale = np.abs(obs).max()
        keys = [(q, e, g) for q in range(8) for e in range(8) for g in range(4)]
        term = {k: -prod[:, 32 * k[0] + 8 * k[2] + k[1]] for k in keys}
        res, best = min((np.abs(term[k] - obs).max(), (k,)) for k in keys)
        if res > 1e-4 * scale:
            res2, best2 = min((np.abs(term[a] + term[b] - obs).max(), (a, b)) for a, b in itertools.combinations(keys, 2))
            if res2 < res:
                res, best = res2, best2
        ok = res <= 1e-3 * scale
        terms_hist[len(best) if ok else "unexplained"] += 1
        rel.append(res / scale)
        if ok:
            for q, e, g in best:
                where[("lane group", g)] += 1
                where[("element", e)] += 1
                where[("q", q)] += 1
    rel = np.array(rel)
    print(f"{variant}: {bad.size} failing half tiles; explained by removing terms: {dict(terms_hist)}")
    if bad.size:
        print(f"residual / error: median {np.median(rel):.2e}, 99th pct {np.percentile(rel, 99):.2e}, "
              f"max {rel.max():.2e}")
    for key in ("lane group", "element", "q"):
        print(key, {k[1]: v for k, v in sorted(where.items()) if k[0] == key})
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
