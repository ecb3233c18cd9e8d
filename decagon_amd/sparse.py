"""Host-side sparse formats at the drop-in boundary.

The reference feeds every adjacency matrix as a COO tuple `(coords[nnz,2], values[nnz],
shape)` (decagon/utility/preprocessing.py:20-26, decagon/deep/minibatch.py:259-267) into a
`tf.sparse_placeholder(tf.float32)` (main.py:103-104).  Here those tuples are converted
once to CSR (rows ascending, the order of the nonzeros inside a row preserved — TF's
SparseTensorDenseMatMul visits nonzeros in feed order) and uploaded; the values are cast
float64 -> float32 exactly as the placeholder's dtype does.
"""
from __future__ import annotations

import os
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


def chunk_segments(csrs: Sequence[HostCSR], m: MergedCSR) -> np.ndarray:
    """Segment starts of merge_chunks' layout (dg_spmm_seg_f32): int32 [n_chunks·n_rows·chunk],
    entry (c·n_rows + r)·chunk + t = the first nonzero of relation c·chunk + t in row r's range
    of chunk c (relations run one after another inside the range; relation slots past the last
    relation are empty segments at the range's end)."""
    n_r, ch, nc = m.n_rows, m.chunk, m.n_chunks
    seg = np.empty((nc, n_r, ch), np.int64)
    start = m.rowptr[:-1].astype(np.int64).reshape(nc, n_r).copy()
    for t in range(ch):
        seg[:, :, t] = start
        for c in range(nc):
            k = c * ch + t
            if k < len(csrs):
                start[c] += np.diff(csrs[k].rowptr.astype(np.int64))
    return seg.reshape(-1).astype(np.int32)


def merge_windows(csrs: Sequence[HostCSR], slabs: Sequence[int], n_windows: int, n_slabs: int) -> MergedCSR:
    """The chunk-merged layout with COLUMN-WINDOW chunks: chunk w holds, for every row, the
    nonzeros of every relation whose column lies in window w (columns split into n_windows
    equal ranges), relation by relation, each relation's in-row order kept.  The partial
    sums of a row over the windows add up to the row's full sum.  Launched in partial mode,
    the XCD-contiguous item map puts each window on its own XCDs, so the operand rows a
    window gathers stay in those XCDs' L2 (large square groups such as PPI)."""
    if not csrs:
        raise ValueError("empty relation group")
    n_r, n_c = csrs[0].shape
    n_windows = max(1, int(n_windows))
    edges = np.linspace(0, n_c, n_windows + 1).astype(np.int64)
    keys, vcols, vals = [], [], []
    for k, c in enumerate(csrs):
        if c.shape != (n_r, n_c):
            raise ValueError("all relations of a group must share one shape")
        lens = np.diff(c.rowptr.astype(np.int64))
        rows = np.repeat(np.arange(n_r, dtype=np.int64), lens)
        win = np.searchsorted(edges, c.col.astype(np.int64), side="right") - 1
        keys.append(win * n_r + rows)
        vcols.append(int(slabs[k]) * n_c + c.col.astype(np.int64))
        vals.append(c.val)
    key = np.concatenate(keys) if keys else np.zeros(0, np.int64)
    total = key.shape[0]
    if total >= 2**31 or n_slabs * n_c >= 2**31:
        raise ValueError("group exceeds int32 indexing")
    order = np.argsort(key, kind="stable")  # stable: relation order, then in-row order
    counts = np.bincount(key, minlength=n_windows * n_r)
    rowptr = np.zeros(n_windows * n_r + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    vcol = np.concatenate(vcols)[order].astype(np.int32) if total else np.zeros(0, np.int32)
    val = np.concatenate(vals)[order].astype(np.float32) if total else np.zeros(0, np.float32)
    return MergedCSR(rowptr.astype(np.int32), vcol, val, n_r, n_c, n_windows, len(csrs), n_slabs * n_c)


@dataclass
class StagedLayout:
    """Device layout of a group for dg_spmm_staged_f32 (include/decagon_hip.h).

    Per relation, a row of len nonzeros becomes a group of S = ceil(len / L) virtual rows of
    equal length ceil(len / S) (the last padded with zero pairs: column n_cols, value 0), S <= 8,
    L the smallest segment length leaving at most `lanes` virtual rows.  Virtual rows are
    sorted by length (descending) with each group on consecutive lanes of one 64-lane wave
    (dummy lanes — all zero pairs — pad where a group would straddle a wave boundary).  Lane
    l = 64w + j owns virtual row l; wave w's pairs are a dense block [rlw_w][64] (rlw_w = its
    longest lane rounded up to a multiple of 4, holes filled with zero pairs), so the pair of
    lane j at diagonal m sits at woff_w + 64m + j and the kernel loads it with no table or test.
    A group's segments are summed within the wave in lane order.

      pairs [n_pairs, 2] int32   (column, fp32 value bits), relations and waves back to back;
                                 holes read one of sixteen zero columns (n_cols + z, value 0)
      jm    int32                per relation at jmoff[k]: [n_waves, largest group, 0, 0],
                                 (then STAGED_JM_SPARE zeros ending the array)
                                 woff[16] (absolute pair offset of each wave's block),
                                 rlw[16] (diagonals per wave, 0 past n_waves),
                                 vinfo[64 n_waves] = row | seg << 10 | (group size - 1) << 13 |
                                 len << 16 (row 1023: dummy lane)
    """

    pairs: np.ndarray
    jm: np.ndarray
    jmoff: np.ndarray
    n_rows: int
    n_cols: int
    nnz: int

    @property
    def jm_len(self) -> int:
        """Ints in jm: the relation tables plus STAGED_JM_SPARE zeros (the kernel reads every
        lane's vinfo slot unconditionally)."""
        return len(self.jm)


STAGED_MAX_GROUP = 8     # segments per row (3 bits of vinfo)
STAGED_DUMMY_ROW = 1023  # vinfo row of a dummy (padding) lane
STAGED_JM_SPARE = 1024   # zero ints ending jm


def _group_sizes(lens: np.ndarray, L: int) -> np.ndarray:
    """Segments per row for segment length at most L: a power of two (1, 2, 4 or 8), so the
    kernel combines a group's segments by a DPP shift tree inside one 16-lane row."""
    need = np.maximum(1, -(-lens // L))
    return (1 << np.ceil(np.log2(need)).astype(np.int64)).astype(np.int64)


def _segment_length(lens: np.ndarray, lanes: int) -> int:
    """Smallest L >= ceil(max / 8) leaving sum(group sizes) virtual rows, with room for the
    alignment padding of groups, within `lanes`."""
    nnz = int(lens.sum())
    L = max(1, -(-nnz // lanes), -(-int(lens.max()) // STAGED_MAX_GROUP))
    budget = lanes - (STAGED_MAX_GROUP - 1) * (-(-lanes // 64))
    nz = lens[lens > 0]
    floor = len(nz)
    while int(_group_sizes(nz, L).sum()) > max(budget, floor):
        L += 1
    return L


def _place_groups(glen: np.ndarray, gsize: np.ndarray, lanes: int) -> List[Tuple[int, int]]:
    """Lane order of groups: descending length, each group of size S (a power of two)
    starting at a lane that is a multiple of S — so it sits inside one 64-lane wave and one
    16-lane DPP row.  Returns [(group index, or -1 for a dummy lane, length)] in lane order — a
    dummy pads up to the next aligned lane where no single of that length is left to do so."""
    order = np.lexsort((-gsize, -glen))     # by length desc, then bigger groups first
    out: List[Tuple[int, int]] = []
    pos, i, n = 0, 0, len(order)
    while i < n:
        ln = int(glen[order[i]])
        j = i
        while j < n and glen[order[j]] == ln:
            j += 1
        multi = [int(g) for g in order[i:j] if gsize[g] > 1]
        single = [int(g) for g in order[i:j] if gsize[g] == 1]
        for g in multi:
            while pos % int(gsize[g]):
                out.append((single.pop() if single else -1, ln))
                pos += 1
            out.append((g, ln))
            pos += int(gsize[g])
        for g in single:
            out.append((g, ln))
            pos += 1
        i = j
    if pos > lanes:
        raise ValueError("staged layout needs more than %d lanes" % lanes)
    return out


def staged_layout(csrs: Sequence[HostCSR], block: Optional[Callable] = None,
                  lanes: int = 1024, split: bool = True) -> StagedLayout:
    """Build the staged layout of relations `csrs` (all one shape, local columns) with at
    most `lanes` virtual rows per relation (split=False: one virtual row per nonempty row).
    `block(lrowptr, lcol, lval, rlw, n_cols) -> pairs` fills a relation's pair block from its
    lanes (a CSR over virtual rows) and the waves' diagonals; the device path passes the
    library's bank-conflict-avoiding builder (kernels.staged_block: each nonzero's diagonal,
    each hole's zero column).  Default: feed order, holes on column n_cols."""
    if not csrs:
        raise ValueError("empty relation group")
    n_r, n_c = csrs[0].shape
    if n_r >= STAGED_DUMMY_ROW or n_c > 1024 or lanes > 1024:
        raise ValueError("staged groups need n_rows < 1023, n_cols <= 1024")
    pairs_parts, jm_parts, jmoff = [], [], [0]
    base = 0
    # the block builder (C, GIL released) runs on a thread pool while the lanes of the next
    # relations are laid out here
    pool = None
    if block is not None and len(csrs) > 1:
        from concurrent.futures import ThreadPoolExecutor
        pool = ThreadPoolExecutor(max_workers=max(1, min(16, len(os.sched_getaffinity(0)))))
    for c in csrs:
        if c.shape != (n_r, n_c):
            raise ValueError("all relations of a group must share one shape")
        lens = np.diff(c.rowptr.astype(np.int64))
        rows_nz = np.nonzero(lens)[0]
        if len(rows_nz) > lanes:
            raise ValueError("more nonempty rows than lanes")
        L = (_segment_length(lens, lanes) if split else int(lens.max())) if len(rows_nz) else 1
        while True:
            S = _group_sizes(lens[rows_nz], L)                # group size per nonempty row
            E = -(-lens[rows_nz] // S)                        # segment length (padded)
            try:
                placed = _place_groups(E, S, lanes)
                break
            except ValueError:                                # boundary padding overflowed
                L += 1
        # lanes in order: row, segment, group size, length, first real nonzero, real count
        lrow, lseg, lgs, llen, lst, lcnt = [], [], [], [], [], []
        for g, ln in placed:
            if g < 0:
                lrow.append(STAGED_DUMMY_ROW); lseg.append(0); lgs.append(1)
                llen.append(ln); lst.append(0); lcnt.append(0)
                continue
            r, sz = int(rows_nz[g]), int(S[g])
            r0, total_r = int(c.rowptr[r]), int(lens[r])
            for q in range(sz):
                lrow.append(r); lseg.append(q); lgs.append(sz); llen.append(ln)
                lst.append(r0 + q * ln); lcnt.append(max(0, min(ln, total_r - q * ln)))
        n_v = len(lrow)
        n_w = -(-n_v // 64)
        pad_l = n_w * 64 - n_v                                # dummy lanes ending the last wave
        llen = np.asarray(llen + [0] * pad_l, np.int64)
        lcnt = np.asarray(lcnt + [0] * pad_l, np.int64)
        lrow = lrow + [STAGED_DUMMY_ROW] * pad_l
        lseg = lseg + [0] * pad_l
        lgs = lgs + [1] * pad_l
        # wave w: a dense [rlw_w][64] block of pairs, rlw_w = its longest lane rounded up to 4
        rlw = ((llen[::64] + 3) // 4 * 4) if n_w else np.zeros(0, np.int64)
        woff = np.zeros(16, np.int64)
        woff[:n_w] = base + np.concatenate([[0], np.cumsum(rlw * 64)[:-1]]) if n_w else 0
        n_pairs = int(rlw.sum()) * 64
        # the lanes' real nonzeros as a CSR over lanes (each a contiguous piece of its row)
        n_l = n_w * 64
        vrowptr = np.zeros(n_l + 1, np.int64)
        np.cumsum(lcnt, out=vrowptr[1:])
        vr = np.repeat(np.arange(n_l), lcnt)
        src = np.repeat(np.asarray(lst + [0] * pad_l, np.int64), lcnt) + (np.arange(len(vr)) - vrowptr[:-1][vr])
        vcol = np.ascontiguousarray(c.col[src], np.int32)
        vval = np.ascontiguousarray(np.asarray(c.val, np.float32)[src])
        if block is not None and n_w:
            args = (vrowptr, vcol, vval, rlw, n_c)
            rel_pairs = pool.submit(block, *args) if pool is not None else block(*args)
        else:
            rel_pairs = np.zeros((n_pairs, 2), np.int32)
            rel_pairs[:, 0] = n_c  # padding: the zero column, value 0
            if c.nnz:
                rank = np.arange(len(src), dtype=np.int64) - vrowptr[:-1][vr]
                dst = woff[vr >> 6] - base + rank * 64 + (vr & 63)
                rel_pairs[dst, 0] = vcol
                rel_pairs[dst, 1] = vval.view(np.int32)
        pairs_parts.append(rel_pairs)
        big = int(max(lgs)) if n_v else 1
        # per wave: diagonals (low 16 bits) and its largest group (bits 16+): a wave whose
        # rows are all unsplit skips the segment combine
        gs_w = np.asarray(lgs, np.int64).reshape(n_w, 64).max(axis=1) if n_w else np.zeros(0, np.int64)
        rl16 = np.zeros(16, np.int64)
        rl16[:n_w] = rlw | (gs_w << 16)
        vinfo = (np.asarray(lrow, np.int64) | (np.asarray(lseg, np.int64) << 10)
                 | ((np.asarray(lgs, np.int64) - 1) << 13) | (llen << 16))
        seg = np.concatenate([[n_w, big, 0, 0], woff, rl16, vinfo]).astype(np.int64)
        jm_parts.append(seg.astype(np.int32))
        jmoff.append(jmoff[-1] + len(seg))
        base += n_pairs
    for k, part in enumerate(pairs_parts):
        if hasattr(part, "result"):  # a block still being built
            pairs_parts[k] = np.asarray(part.result(), np.int32).reshape(-1, 2)
    if pool is not None:
        pool.shutdown()
    if base >= 2**31:
        raise ValueError("group exceeds int32 indexing")
    # at least one 4-diagonal block: waves without pairs read block 0 unconditionally
    pairs = np.concatenate(pairs_parts) if base else np.zeros((256, 2), np.int32)
    if not base:
        pairs[:, 0] = n_c
    jm = np.concatenate(jm_parts + [np.zeros(STAGED_JM_SPARE, np.int32)])
    return StagedLayout(pairs, jm,
                        np.asarray(jmoff, np.int32), n_r, n_c, int(sum(c.nnz for c in csrs)))
