"""ORACLE — test infrastructure only.  Drives the scalar C restatement (gcn_ref.c) through
one full two-layer GCN forward in TF 1.8's CPU op order — per relation: X·W (identity
features: W itself), sparse_tensor_dense_matmul into a fresh buffer, add_n; then
l2_normalize, the sum over edge types and relu (decagon/deep/layers.py:85-118,
decagon/deep/model.py:64-88).  Used as bench.py's timed CPU baseline ("port", 1 thread)
and as a second checker in tests.
"""
from __future__ import annotations

import ctypes
import subprocess
from ctypes import POINTER, c_float, c_int32, c_int64, c_void_p
from pathlib import Path

import numpy as np
import scipy.sparse as sp

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "liboracle_gcn.so"


def load() -> ctypes.CDLL:
    if not LIB.exists():
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    lib = ctypes.CDLL(str(LIB))
    lib.oracle_spmm_f32.argtypes = [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int64, c_int32, c_void_p]
    lib.oracle_add_f32.argtypes = [c_void_p, c_void_p, c_int64]
    lib.oracle_l2norm_rows_f32.argtypes = [c_void_p, c_int32, c_int32]
    lib.oracle_relu_f32.argtypes = [c_void_p, c_int64]
    lib.oracle_gemm_f32.argtypes = [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32]
    for f in (lib.oracle_spmm_f32, lib.oracle_add_f32, lib.oracle_l2norm_rows_f32, lib.oracle_relu_f32,
              lib.oracle_gemm_f32):
        f.restype = None
    return lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


class Forward:
    def __init__(self, lib, graph, h1: int, h2: int, seed: int = 1234, w1=None, w2=None):
        self.lib = lib
        self.h1, self.h2 = h1, h2
        self.edge_types = dict(graph.edge_types)
        self.n = dict(graph.n_nodes)
        self.adj = {}
        memo = {}
        for et, rels in graph.adj.items():
            lst = []
            for coo in rels:
                key = (id(coo[0]), id(coo[1]))
                if key not in memo:
                    c, v, s = coo
                    m = sp.csr_matrix((np.asarray(v, np.float32), (c[:, 0], c[:, 1])), shape=s)
                    memo[key] = (m.indptr.astype(np.int32), m.indices.astype(np.int32),
                                 m.data.astype(np.float32), int(s[0]))
                lst.append(memo[key])
            self.adj[et] = lst
        rng = np.random.default_rng(seed)

        def glorot(k, a, b):
            r = np.sqrt(6.0 / (a + b))
            return rng.uniform(-r, r, size=(k, a, b)).astype(np.float32)

        self.w1 = w1 or {et: glorot(K, self.n[et[1]], h1) for et, K in self.edge_types.items()}
        self.w2 = w2 or {et: glorot(K, h1, h2) for et, K in self.edge_types.items()}
        self.tmp = {}

    def _buf(self, key, shape):
        b = self.tmp.get(key)
        if b is None or b.shape != shape:
            b = np.empty(shape, np.float32)
            self.tmp[key] = b
        return b

    def _layer(self, xs, d, relu):
        L = self.lib
        out = {}
        for et in self.edge_types:
            i, j = et
            n_i = self.n[i]
            acc = np.zeros((n_i, d), np.float32)
            y = self._buf(("y", n_i, d), (n_i, d))
            for k, (rp, ci, va, nr) in enumerate(self.adj[et]):
                x = xs(et, k)
                L.oracle_spmm_f32(_p(rp), _p(ci), _p(va), nr, _p(x), x.shape[1], d, _p(y))
                L.oracle_add_f32(_p(acc), _p(y), acc.size)
            L.oracle_l2norm_rows_f32(_p(acc), n_i, d)
            if i in out:
                L.oracle_add_f32(_p(out[i]), _p(acc), acc.size)
            else:
                out[i] = acc
        if relu:
            for v in out.values():
                L.oracle_relu_f32(_p(v), v.size)
        return out

    def run(self):
        h1 = self._layer(lambda et, k: self.w1[et][k], self.h1, True)

        def proj(et, k):
            j = et[1]
            p = self._buf(("p", j), (self.n[j], self.h2))
            self.lib.oracle_gemm_f32(_p(h1[j]), _p(self.w2[et][k]), _p(p), self.n[j], self.h1, self.h2)
            return p

        emb = self._layer(proj, self.h2, False)
        return h1, emb
