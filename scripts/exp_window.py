"""Experiment: the PPI group of config P in partial mode, relations merged into one chunk vs
column windows (one chunk per window, windows mapped to XCDs) — does L2 residency of the
gathered operand rows pay for the window partials?"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from decagon_amd import kernels, synthetic  # noqa: E402
from decagon_amd.sparse import merge_chunks, MergedCSR  # noqa: E402


def windowed(csrs, n_win):
    n_r, n_c = csrs[0].shape
    K = len(csrs)
    edges = np.linspace(0, n_c, n_win + 1).astype(np.int64)
    rows_l, vcol_l, val_l, key_l = [], [], [], []
    for k, c in enumerate(csrs):
        lens = np.diff(c.rowptr.astype(np.int64))
        r = np.repeat(np.arange(n_r), lens)
        w = np.searchsorted(edges, c.col, side="right") - 1
        rows_l.append(r); vcol_l.append(k * n_c + c.col.astype(np.int64)); val_l.append(c.val)
        key_l.append(w * n_r + r)
    key = np.concatenate(key_l); vcol = np.concatenate(vcol_l); val = np.concatenate(val_l)
    order = np.argsort(key, kind="stable")
    counts = np.bincount(key, minlength=n_win * n_r)
    rowptr = np.zeros(n_win * n_r + 1, np.int64); np.cumsum(counts, out=rowptr[1:])
    return MergedCSR(rowptr.astype(np.int32), vcol[order].astype(np.int32), val[order].astype(np.float32),
                     n_r, n_c, n_win, K, K * n_c)


def bench(fn, reps=50):
    fn(); torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn(); s.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay(); s.synchronize()
        t0 = torch.cuda.Event(enable_timing=True); t1 = torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            t0.record(s); g.replay(); t1.record(s); t1.synchronize()
            best = min(best, t0.elapsed_time(t1) / reps)
    return best * 1e3


def main():
    dev = torch.device("cuda", 0)
    g = synthetic.make_P(seed=0)
    csr = g.csr()
    ppi = csr[(0, 0)]
    n = 19085
    for d in (64, 32):
        X = torch.randn((2, n, d), device=dev)
        res = {}
        for name, m in [("merged", merge_chunks(ppi, [0, 1], 2, 2))] + \
                       [(f"win{w}", windowed(ppi, w)) for w in (2, 4, 8, 16)]:
            out = torch.empty((m.n_chunks, n, d), device=dev)
            spec = kernels.RelGroupSpec(torch.from_numpy(m.rowptr).to(dev), torch.from_numpy(m.vcol).to(dev),
                                        torch.from_numpy(m.val).to(dev), X, out, n, m.n_chunks, d, 2 * n,
                                        vcol_max=int(m.vcol.max()))
            op = kernels.PreparedSpmm([spec], d)
            us = bench(op)
            outs = out.sum(0)
            res[name] = outs
            epi = kernels.PreparedEpilogue([(out, m.n_chunks)], torch.empty((n, d), device=dev), n, d, 0)
            us_e = bench(epi)
            print(f"d={d} {name:7s} chunks={m.n_chunks:2d} spmm {us:7.1f} us  epilogue {us_e:6.1f} us", flush=True)
        ref = res["merged"]
        for k, v in res.items():
            assert torch.allclose(v, ref, rtol=1e-4, atol=1e-5), k


if __name__ == "__main__":
    main()
