"""Host-side sparse formats at the drop-in boundary.

The reference feeds every adjacency matrix as a COO tuple `(coords[nnz,2], values[nnz],
shape)` (decagon/utility/preprocessing.py:20-26, decagon/deep/minibatch.py:259-267) into a
`tf.sparse_placeholder(tf.float32)` (main.py:103-104).  Here those tuples are converted
once to CSR (rows ascending, the order of the nonzeros inside a row preserved — TF's
SparseTensorDenseMatMul visits nonzeros in feed order) and uploaded; the values are cast
float64 -> float32 exactly as the placeholder's dtype does.
"""
from __future__ import annotations

from collections import namedtuple
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp

SparseTensorValue = namedtuple("SparseTensorValue", ["indices", "values", "dense_shape"])


def sparse_to_tuple(sparse_mx) -> Tuple[np.ndarray, np.ndarray, Tuple[int, int]]:
    """COO wire format of the reference (decagon/utility/preprocessing.py:20-26)."""
    m = sparse_mx.tocoo() if not sp.isspmatrix_coo(sparse_mx) else sparse_mx
    coords = np.stack([m.row, m.col], axis=1)
    return coords, m.data, tuple(int(s) for s in m.shape)


def preprocess_graph(adj) -> Tuple[np.ndarray, np.ndarray, Tuple[int, int]]:
    """Normalized adjacency, restating EdgeMinibatchIterator.preprocess_graph
    (decagon/deep/minibatch.py:80-93) in float64:

      square   (N×N):  Â = D^-½ (A+I)ᵀ D^-½,  D = diag(rowsum(A+I))
      rectangular:     Â = Dr^-½ A Dc^-½ (nan_to_num on the degrees, as the reference;
                       a zero-degree row/column holds no entry, so its factor is never used)

    For the square case each stored value is (v·d[c])·d[r] for entry (r,c) of A+I, stored
    at (c,r) — the same product order as the reference's `adj_.dot(D).transpose().dot(D)`.
    Returns the COO tuple; entry order is row-major (the CSR build does not depend on it).
    """
    a = sp.coo_matrix(adj, dtype=np.float64)
    n_r, n_c = a.shape
    if n_r == n_c:
        a = (a + sp.eye(n_r, dtype=np.float64)).tocsr()
        a.sum_duplicates()
        rowsum = np.asarray(a.sum(axis=1)).ravel()
        with np.errstate(divide="ignore"):
            dinv = np.power(rowsum, -0.5)
        a = a.tocoo()
        vals = (a.data * dinv[a.col]) * dinv[a.row]
        out = sp.coo_matrix((vals, (a.col, a.row)), shape=(n_c, n_r)).tocsr()
    else:
        rowsum = np.asarray(a.sum(axis=1)).ravel()
        colsum = np.asarray(a.sum(axis=0)).ravel()
        with np.errstate(divide="ignore"):
            rinv = np.nan_to_num(np.power(rowsum, -0.5))
            cinv = np.nan_to_num(np.power(colsum, -0.5))
        a = a.tocsr()
        a.sum_duplicates()
        a = a.tocoo()
        vals = (rinv[a.row] * a.data) * cinv[a.col]
        out = sp.coo_matrix((vals, (a.row, a.col)), shape=(n_r, n_c)).tocsr()
    out.sort_indices()
    return sparse_to_tuple(out)


def as_coo_tuple(value) -> Tuple[np.ndarray, np.ndarray, Tuple[int, int]]:
    """Accept what a tf.sparse_placeholder accepts: (coords, values, shape), a
    SparseTensorValue, or a scipy sparse matrix."""
    if sp.issparse(value):
        return sparse_to_tuple(value)
    if isinstance(value, SparseTensorValue):
        return np.asarray(value.indices), np.asarray(value.values), tuple(value.dense_shape)
    if isinstance(value, (tuple, list)) and len(value) == 3:
        c, v, s = value
        return np.asarray(c), np.asarray(v), tuple(int(x) for x in s)
    raise TypeError(f"cannot feed {type(value).__name__} to a sparse placeholder")


@dataclass
class HostCSR:
    """One relation in CSR, int32 indices, float32 values."""

    rowptr: np.ndarray
    col: np.ndarray
    val: np.ndarray
    shape: Tuple[int, int]

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])


def coo_to_csr(coords, values, shape) -> HostCSR:
    coords = np.asarray(coords)
    values = np.asarray(values)
    n_r, n_c = int(shape[0]), int(shape[1])
    if coords.size == 0:
        return HostCSR(np.zeros(n_r + 1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32), (n_r, n_c))
    if coords.ndim != 2 or coords.shape[1] != 2 or coords.shape[0] != values.shape[0]:
        raise ValueError("coords must be [nnz, 2] and match values")
    rows = coords[:, 0].astype(np.int64)
    cols = coords[:, 1].astype(np.int64)
    if rows.min() < 0 or rows.max() >= n_r or cols.min() < 0 or cols.max() >= n_c:
        raise ValueError(f"sparse index out of range for shape {shape}")
    if n_r >= 2**31 or n_c >= 2**31 or rows.shape[0] >= 2**31:
        raise ValueError("sparse operand exceeds int32 indexing")
    order = np.argsort(rows, kind="stable")
    counts = np.bincount(rows, minlength=n_r)
    rowptr = np.zeros(n_r + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    return HostCSR(rowptr.astype(np.int32), cols[order].astype(np.int32),
                   values[order].astype(np.float32), (n_r, n_c))


def is_identity(coords, values, shape) -> bool:
    """True when a feature feed is the identity (featureless nodes, main.py:186-193): then
    X·W ≡ W exactly and the T2 SpMM is skipped."""
    n_r, n_c = int(shape[0]), int(shape[1])
    coords = np.asarray(coords)
    values = np.asarray(values)
    if n_r != n_c or coords.shape[0] != n_r:
        return False
    idx = np.arange(n_r)
    return bool(np.array_equal(coords[:, 0], idx) and np.array_equal(coords[:, 1], idx)
                and np.all(values == 1))


@dataclass
class StackedCSR:
    """K relations of one (i,j) group with a common shape, stacked: relation k's row r is
    rowptr[k*n_rows + r] .. rowptr[k*n_rows + r + 1] into col/val (global offsets)."""

    rowptr: np.ndarray
    col: np.ndarray
    val: np.ndarray
    n_rows: int
    n_cols: int
    n_rels: int
    rel_nnz: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))

    @property
    def nnz(self) -> int:
        return int(self.col.shape[0])


def stack_relations(csrs: Sequence[HostCSR]) -> StackedCSR:
    if not csrs:
        raise ValueError("empty relation group")
    n_r, n_c = csrs[0].shape
    for c in csrs:
        if c.shape != (n_r, n_c):
            raise ValueError("all relations of a group must share one shape")
    nnz = [c.nnz for c in csrs]
    total = int(np.sum(nnz))
    if total >= 2**31:
        raise ValueError("group exceeds int32 nonzero offsets")
    rowptr = np.empty(len(csrs) * n_r + 1, np.int64)
    off = 0
    for k, c in enumerate(csrs):
        rowptr[k * n_r:(k + 1) * n_r] = c.rowptr[:-1].astype(np.int64) + off
        off += c.nnz
    rowptr[-1] = off
    col = np.concatenate([c.col for c in csrs]) if total else np.zeros(0, np.int32)
    val = np.concatenate([c.val for c in csrs]) if total else np.zeros(0, np.float32)
    return StackedCSR(rowptr.astype(np.int32), col.astype(np.int32), val.astype(np.float32),
                      n_r, n_c, len(csrs), np.asarray(nnz, np.int64))


@dataclass
class MergedCSR:
    """A group's relations in the chunk-merged layout of dg_rel_group (decagon_hip.h):
    for chunk c and row r the nonzeros of every relation of the chunk, contiguous, at
    [rowptr[c*n_rows + r], rowptr[c*n_rows + r + 1]); vcol = k_x * n_cols + col where k_x is
    the relation's slab in the relation-stacked dense operand."""

    rowptr: np.ndarray
    vcol: np.ndarray
    val: np.ndarray
    n_rows: int
    n_cols: int
    n_chunks: int
    chunk: int
    x_rows: int

    @property
    def nnz(self) -> int:
        return int(self.vcol.shape[0])


def merge_chunks(csrs: Sequence[HostCSR], slabs: Sequence[int], chunk: int, n_slabs: int) -> MergedCSR:
    """Build the chunk-merged layout.  `csrs` are the (local) relations in order, `slabs[k]`
    the slab of relation k in the stacked operand (its global relation index), `chunk`
    relations per chunk, `n_slabs` slabs in the operand.  Inside a (chunk, row) range the
    nonzeros run relation by relation, each relation's in-row (feed) order kept."""
    if not csrs:
        raise ValueError("empty relation group")
    n_r, n_c = csrs[0].shape
    K = len(csrs)
    chunk = max(1, min(int(chunk), K))
    n_chunks = -(-K // chunk)
    counts = np.zeros(n_chunks * n_r, np.int64)
    for k, c in enumerate(csrs):
        if c.shape != (n_r, n_c):
            raise ValueError("all relations of a group must share one shape")
        counts[(k // chunk) * n_r:(k // chunk + 1) * n_r] += np.diff(c.rowptr.astype(np.int64))
    total = int(counts.sum())
    if total >= 2**31 or n_slabs * n_c >= 2**31:
        raise ValueError("group exceeds int32 indexing")
    rowptr = np.zeros(n_chunks * n_r + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    vcol = np.empty(total, np.int32)
    val = np.empty(total, np.float32)
    fill = rowptr[:-1].copy()  # next free position of each (chunk, row) range
    for k, c in enumerate(csrs):
        cb = (k // chunk) * n_r
        lens = np.diff(c.rowptr.astype(np.int64))
        if c.nnz == 0:
            continue
        starts = fill[cb:cb + n_r]
        # destination of each nonzero: its row's next free slot + its rank within the row
        rows = np.repeat(np.arange(n_r), lens)
        rank = np.arange(c.nnz, dtype=np.int64) - np.repeat(c.rowptr[:-1].astype(np.int64), lens)
        dst = starts[rows] + rank
        vcol[dst] = int(slabs[k]) * n_c + c.col
        val[dst] = c.val
        fill[cb:cb + n_r] += lens
    return MergedCSR(rowptr.astype(np.int32), vcol, val, n_r, n_c, n_chunks, chunk, n_slabs * n_c)


@dataclass
class StagedLayout:
    """Device layout of a group for dg_spmm_staged_f32 (include/decagon_hip.h).

    Per relation, rows longer than a segment length L are split into virtual rows of at most
    L consecutive nonzeros (L the smallest that leaves at most `lanes` virtual rows); the
    virtual rows are sorted by length (descending, stable) and the nonzeros stored
    diagonal-major — the m-th nonzero of every virtual row that has one, in sorted order — so
    thread i of a workgroup owns sorted virtual row i and a wave's pairs at diagonal m are
    one contiguous run.

      pairs [nnz + 1, 2] int32   (column, fp32 value bits), relations back to back, + 1 pad pair
      jm    int32                per relation at jmoff[k]: [n_virt, n_rounds, 0, 0]
                                 (n_rounds = most segments of a row), vinfo[n_virt] =
                                 row | seg << 10 | len << 16 per sorted virtual row,
                                 doff[maxlen + 1] (absolute pair offset of diagonal m)
    """

    pairs: np.ndarray
    jm: np.ndarray
    jmoff: np.ndarray
    n_rows: int
    n_cols: int
    nnz: int


def _segment_length(lens: np.ndarray, lanes: int) -> int:
    """Smallest L with sum(ceil(lens / L)) <= lanes."""
    nnz = int(lens.sum())
    L = max(1, -(-nnz // lanes))
    while int((-(-lens // L)).sum()) > lanes:
        L += 1
    return L


def staged_layout(csrs: Sequence[HostCSR], order: Optional[Callable] = None,
                  lanes: int = 1024, split: bool = True) -> StagedLayout:
    """Build the staged layout of relations `csrs` (all one shape, local columns) with at
    most `lanes` virtual rows per relation (split=False: one virtual row per nonempty row).
    `order(csr, perm) -> rank` places each nonzero of a (virtual-row) CSR on a diagonal
    (default: feed order); the device path passes the library's bank-conflict-avoiding
    order (kernels.staged_order)."""
    if not csrs:
        raise ValueError("empty relation group")
    n_r, n_c = csrs[0].shape
    if n_r >= 1024 or n_c > 1024 or lanes > 1024:
        raise ValueError("staged groups need n_rows < 1024, n_cols <= 1024")
    total = int(sum(c.nnz for c in csrs))
    if total + 1 >= 2**31:
        raise ValueError("group exceeds int32 indexing")
    pairs = np.zeros((total + 1, 2), np.int32)
    jm_parts, jmoff = [], [0]
    base = 0
    for c in csrs:
        if c.shape != (n_r, n_c):
            raise ValueError("all relations of a group must share one shape")
        lens = np.diff(c.rowptr.astype(np.int64))
        L = (_segment_length(lens, lanes) if split else int(lens.max())) if c.nnz else 1
        nseg = -(-lens // L)                                   # segments per row (0: empty row)
        vrow = np.repeat(np.arange(n_r), nseg)                 # virtual row -> row
        vseg = np.arange(len(vrow)) - np.repeat(np.cumsum(nseg) - nseg, nseg)
        vstart = c.rowptr[:-1].astype(np.int64)[vrow] + vseg * L
        vlen = np.minimum(L, lens[vrow] - vseg * L)
        n_v = len(vrow)
        vrowptr = np.zeros(n_v + 1, np.int64)
        np.cumsum(vlen, out=vrowptr[1:])                       # virtual CSR = same nonzero order
        perm = np.argsort(-vlen, kind="stable")
        rl = vlen[perm]
        maxlen = int(rl[0]) if n_v else 0
        cnt = n_v - np.cumsum(np.bincount(rl, minlength=maxlen + 1))[:maxlen]
        doff = np.empty(maxlen + 1, np.int64)
        doff[0] = base
        np.cumsum(cnt, out=doff[1:])
        doff[1:] += base
        if c.nnz:
            inv = np.empty(n_v, np.int64)
            inv[perm] = np.arange(n_v)
            vr = np.repeat(np.arange(n_v), vlen)
            if order is None:
                rank = np.arange(c.nnz, dtype=np.int64) - vrowptr[:-1][vr]
            else:
                vcsr = HostCSR(vrowptr.astype(np.int32), c.col, c.val, (n_v, n_c))
                rank = np.asarray(order(vcsr, perm), np.int64)
            dst = doff[rank] + inv[vr]
            pairs[dst, 0] = c.col
            pairs[dst, 1] = np.ascontiguousarray(c.val, np.float32).view(np.int32)
        rounds = int(nseg.max()) if n_r else 0
        vinfo = vrow[perm] | (vseg[perm] << 10) | (rl << 16)
        seg = np.concatenate([[n_v, rounds, 0, 0], vinfo, doff]).astype(np.int64)
        pad = (-len(seg)) % 4
        jm_parts.append(np.concatenate([seg.astype(np.int32), np.zeros(pad, np.int32)]))
        jmoff.append(jmoff[-1] + len(seg) + pad)
        base += c.nnz
    return StagedLayout(pairs, np.concatenate(jm_parts) if jm_parts else np.zeros(0, np.int32),
                        np.asarray(jmoff, np.int32), n_r, n_c, total)
