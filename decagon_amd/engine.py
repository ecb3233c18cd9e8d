"""Device-resident relation graph and the fused two-layer GCN forward plan.

The reference rebuilds the full-graph forward inside every `sess.run` and re-feeds every
COO adjacency from the host each step (decagon/deep/minibatch.py:259-267, main.py:315).
Here the adjacencies are converted once to the chunk-merged CSR of dg_rel_group and uploaded
(`DeviceGraph`), all buffers are allocated once (`ForwardPlan`), and one forward is a fixed
sequence of launches — capturable into a hipGraph.  Per layer, per node type i:

  fused   (every group (i,j) is one chunk, single GPU)   dg_gcn_fused_f32
          Σ_k Â_k·X_k, l2norm per group, Σ_j, relu            layers.py:90-93, model.py:74-75
          (+ layer 1: the next layer's P_k = H1_i·W2_k)        layers.py:113
  partial (many relations, or sharded)                   dg_spmm_groups_f32 + dg_gcn_epilogue_f32
  projections not fused                                  dg_gemm_f32, all groups in one launch

With a relation shard (multi-GPU, sharding.py) each rank runs its relations only, writes or
reduces its chunk partials into one pre-normalisation sum per group, all-reduces those sums
(RCCL) and runs the same epilogue: the normalisation must follow the full Σ_k
(layers.py:92-93).  Every relation-indexed buffer (W1, the projections P, sparse-feature
products X·W1) is indexed by the GLOBAL relation id, so one merged layout serves both layers.
"""
from __future__ import annotations

import heapq
import math
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import kernels
from ._lib import DG_EPI_L2NORM, DG_EPI_RELU, DG_MAX_GROUPS
from .sparse import HostCSR, MergedCSR, chunk_segments, merge_chunks, merge_windows, staged_layout
from .tuning import knob

EdgeType = Tuple[int, int]


# LDS-staged groups (staged.hip): many relations over a column space narrow enough that one
# relation's 16-float column slice and the output rows' accumulators fit LDS.
STAGED_MIN_RELS = knob("DG_STAGED_MIN_RELS", 32)
STAGED_MAX_COLS = 1024
STAGED_MAX_ROWS = 1022
STAGED_BINS = knob("DG_STAGED_BINS", 128)


def drop_tag(layer: int, group: int) -> int:
    """The dropout mask stream of (layer, edge-type index): layer 1 masks rows of the
    relation-stacked W1 of the group, layer 2 masks elements of H1_j per relation."""
    return (layer << 16) | group


def stageable(n_rels: int, n_rows: int, n_cols: int) -> bool:
    return (knob("DG_STAGED", True) and n_rels >= STAGED_MIN_RELS
            and 0 < n_cols <= STAGED_MAX_COLS and 0 < n_rows <= STAGED_MAX_ROWS
            and kernels.staged_lds_bytes(n_rows, n_cols) <= kernels.STAGED_LDS_BYTES)


STAGED_TARGET_BLOCKS = knob("DG_STAGED_BLOCKS", 256)  # one round: a workgroup per CU

# Large groups whose relations fit one chunk (PPI: 2 x 19,085^2) are laid out in column
# windows (sparse.merge_windows): each window's gathers stay in its XCDs' L2.  Measured on
# config P's PPI (scripts/exp_window.py): d=64 63.6 us merged -> 40.0 us with 2 windows
# (+5.6 us epilogue); 4 windows 40.8, 8 windows 53.7 (the window partials start to cost).
# A rank's row block of such a group at N = 8 (2,386 protein rows) is windowed too, in twice
# as many windows (its launch is short of waves, not of L2): config P's N = 8 rank share
# (--simulate-world 8, max over ranks) 110.7 us without windows, 106.5 with 2, 106.0 with 4,
# 109.9 with 8 (round 5).
WINDOW_MIN_ROWS = knob("DG_WINDOW_MIN_ROWS", 1024)
WINDOW_FULL_ROWS = 4096  # below this many rows: 2 x N_WINDOWS windows
N_WINDOWS = knob("DG_WINDOWS", 2)
# node types with at most this many rows finish in the fused row-per-workgroup kernel; larger
# ones run partial mode + epilogue (one wave per row keeps more gathers in flight)
FUSED_MAX_ROWS = knob("DG_FUSED_MAX_ROWS", 4096)
# a layer's gather-bound launch beside its LDS-bound staged launch on a second stream: no gain
# measured (config P step 494.8 us concurrent vs 496.5 sequential; the staged kernel slows by
# what the other saves) and the fork / join cost ~10 us of idle GPU each at small per-rank
# shares (8-GPU rehearsal), so one stream by default
CONCURRENT_LAUNCHES = knob("DG_CONCURRENT", False)
# layer 2 of staged groups makes its slabs H1_j·W2_k on the MFMA inside the SpMM kernel
STAGED_PROJ = knob("DG_STAGED_PROJ", True)
# one-GPU plans whose node types all fit dg_gcn_fused_seg_f32 (config S) use it, layer 2
# reassociated; DG_FUSED_SEG=0 keeps dg_gcn_fused_f32 with the projection epilogue + P
FUSED_SEG = knob("DG_FUSED_SEG", True)
# config S's N-GPU rank share (seg mode): each row of the rank's block finished by one
# dg_gcn_fused_seg_f32 workgroup, one wave per relation of the row's N relation sets
# (DG_SEG_FUSED=0, or more relations a row: dg_spmm_seg_f32 partials + the epilogue launch)
SEG_FUSED = knob("DG_SEG_FUSED", True)
# ... when a row has at most 16 relations (one wave each: N <= 2 for config S).  A form whose 16
# waves looped over more relations measured 25.2 µs a rank share at N = 4 (seg + epilogue 25.1)
# and 35.6 at N = 8 (25.6), so it was not kept
SEG_FUSED_MAX_ITEMS = 16
# fused-seg and seg launches (config S on one GPU and its N-GPU row blocks) through their
# wave-table forms, dg_gcn_fused_tab_f32 / dg_spmm_seg_tab_f32 (host-built: each wave's segment
# bounds, gather base and finishing roles precomputed, its first pairs at a fixed slot; bitwise
# the same rows): config S's step 18.14 -> 15.56 us at 200 steps (round 5)
WAVE_TABLE = knob("DG_WAVE_TABLE", True)
# the wave-table fused launches deal each row's pairs over every wave slot of its workgroup
# (PreparedFusedTab balance, round 6) instead of one wave per relation: 0 never, 1 layer 1 only
# (d_in == d_out), 2 both layers
TAB_BALANCE = knob("DG_TAB_BALANCE", 1)
STAGED_FIRST = knob("DG_STAGED_FIRST", True)
# sharded forward plans: layer 2 of the non-staged groups reassociated over the rank's own rows
# and relations, Σ_k (Â_k·H1_j)·W2_k in dg_spmm_seg_f32, instead of every rank projecting all of
# H1_j·W2_k (config P's PPI: 19,085 rows x 2 relations, 9.4 µs on every rank at N = 8)
REASSOC_ROWS = knob("DG_REASSOC_ROWS", True)
# sharded forward plans: layer 1 of the row-split, non-windowed, non-staged groups in
# dg_spmm_seg_f32 (one wave per (row, relation), its segment's pairs in one load) instead of
# dg_spmm_groups_f32 (one wave per two (chunk, row) items): a rank's short row block (config P
# at N = 8: 2,386 protein rows, the PPI's two relations in one chunk) keeps more waves in flight.
# Off: at P's N = 8 share it took 3-5 us off seven ranks (107.1-108.0 -> 102.7-104.1 us) but
# added 1.7 us to the slowest (rank 4, 110.6 -> 112.3: a wave per (row, relation) walks a hub
# row's long segment alone), so the max over ranks got worse
SEG_ROWS_L1 = knob("DG_SEG_ROWS_L1", False)


def _epilogue(targets, d: int, flags: int, peer=None, push=None):
    """An epilogue launch in its row-table form when the targets allow it (WAVE_TABLE), else
    dg_gcn_epilogue_multi_f32 / _peer_f32 — bitwise the same rows either way."""
    if WAVE_TABLE:
        try:
            return kernels.PreparedEpilogueTab(targets, d, flags, peer=peer, push=push)
        except ValueError:
            pass
    return kernels.PreparedEpilogueMulti(targets, d, flags, peer=peer, push=push)


# staged groups in variable-size output chunks (dg_staged_group.chunk_start): the relations are
# dealt LPT into about STAGED_TARGET_BLOCKS / 4 chunks (a 64-wide layer's), each split LPT in two
# for a 32-wide layer — instead of fixed runs of snake-binned relations, which at a rank's share
# (config P at N = 8: ~241 relations, 4 a chunk) put a 43 k-nonzero relation beside three others
STAGED_VAR = knob("DG_STAGED_VAR", True)


def _lpt_bins(costs: np.ndarray, items: np.ndarray, n_bins: int, cap: int) -> List[List[int]]:
    """items dealt largest first to the least-loaded bin that has room (< cap items); ties to the
    lower bin index (deterministic).  Every bin gets an item when len(items) >= n_bins."""
    order = items[np.argsort(-costs[items], kind="stable")]
    bins: List[List[int]] = [[] for _ in range(n_bins)]
    heap = [(0.0, b) for b in range(n_bins)]
    for it in order:
        full = []
        while True:
            load, b = heapq.heappop(heap)
            if len(bins[b]) < cap:
                break
            full.append((load, b))
        bins[b].append(int(it))
        heapq.heappush(heap, (load + float(costs[it]), b))
        for f in full:
            heapq.heappush(heap, f)
    return bins


def staged_var_chunks(costs: Sequence[float], n_top: int, split: int = 2, cap: int = 64):
    """Variable output chunks of a staged group: (device order of the relations, top-level chunk
    starts, sub-chunk starts).  The relations are dealt LPT into n_top chunks of <= cap, each
    chunk's relations LPT into <= split sub-chunks; the device order lists the chunks heaviest,
    lightest, second heaviest, ... (so runs of two merge evenly), sub-chunk by sub-chunk."""
    c = np.asarray(costs, np.float64)
    n = len(c)
    n_top = max(1, min(n_top, n))
    if n > n_top * cap:
        raise ValueError("more relations than chunks x cap")
    top = _lpt_bins(c, np.arange(n), n_top, cap)
    loads = np.array([c[b].sum() for b in top])
    by = list(np.argsort(-loads, kind="stable"))
    seq = []
    while by:
        seq.append(by.pop(0))
        if by:
            seq.append(by.pop())
    order, tops, subs = [], [0], [0]
    for b in seq:
        items = np.asarray(top[b], np.int64)
        for sb in _lpt_bins(c, items, min(split, len(items)), cap):
            order += sb
            subs.append(len(order))
        tops.append(len(order))
    return np.asarray(order, np.int64), np.asarray(tops, np.int32), np.asarray(subs, np.int32)


# ... and a relation costing more than STAGED_PIECE x a chunk's mean (a 32-wide layer's chunks are
# halves) is cut by rows into pieces of at most that (each piece its own staged "relation" reading
# the same slab): config P's N = 8 rank share holds 58 k-nonzero relations against chunks of ~45 k
STAGED_PIECE = knob("DG_STAGED_PIECE", 0.5)


def staged_pieces(loc: Sequence[HostCSR], costs: Sequence[float], n_top: int, frac: float):
    """Row pieces of the relations that cost more than frac x sum(costs) / n_top: a list of
    (relation index, HostCSR) — whole relations as themselves, heavy ones as pieces of consecutive
    rows of about equal nonzeros, at most that cost each (every row in exactly one piece, so a
    row's sum over a relation is the same arithmetic)."""
    mean = float(sum(costs)) / max(1, n_top)
    out = []
    for i, (c, cost) in enumerate(zip(loc, costs)):
        n_p = int(math.ceil(cost / (frac * mean))) if frac > 0 and cost > frac * mean else 1
        if n_p <= 1:
            out.append((i, c))
            continue
        rp = c.rowptr.astype(np.int64)
        cuts = np.searchsorted(rp, np.arange(1, n_p) * (c.nnz / n_p), side="left")
        bounds = np.unique(np.concatenate([[0], np.clip(cuts, 0, c.shape[0]), [c.shape[0]]]))
        for ra, rb in zip(bounds[:-1], bounds[1:]):
            p0, p1 = int(rp[ra]), int(rp[rb])
            if p1 == p0:
                continue
            prow = (np.clip(rp, p0, p1) - p0).astype(np.int32)
            out.append((i, HostCSR(prow, c.col[p0:p1], c.val[p0:p1], tuple(c.shape))))
    return out


def staged_chunk_starts(grp, d: int) -> Optional[np.ndarray]:
    """The variable output chunks of a staged group for a layer of width d (None: fixed runs of
    staged_out_chunk relations): the sub-chunks when the layer wants at least twice the top-level
    chunks of workgroups' worth (STAGED_TARGET_BLOCKS / slices), the top-level chunks when it
    wants at least as many, else runs of consecutive top-level chunks (heavy-light pairs)."""
    if grp.var_chunks is None:
        return None
    tops, subs = grp.var_chunks
    want = max(1, STAGED_TARGET_BLOCKS // -(-d // 16))
    n_top = len(tops) - 1
    if want >= 2 * n_top and len(subs) - 1 <= kernels.STAGED_MAX_CHUNKS:
        return subs
    if want >= n_top:
        return tops
    f = -(-n_top // want)
    st = tops[::f] if (n_top % f == 0) else np.concatenate([tops[::f], tops[-1:]])
    if np.diff(st).max() > 64:
        return None
    return st.astype(np.int32)


def _staged_n(grp) -> int:
    """Relations of a staged group's layout (row pieces counted one by one)."""
    lay = getattr(grp, "layout", None)
    return lay.n_rels if lay is not None else grp.n_rels


def staged_out_chunk(grp, d: int) -> int:
    """Relations per output chunk of a staged group for a layer of width d: a multiple of the
    group's snake-bin size (so chunks stay balanced) giving about STAGED_TARGET_BLOCKS
    workgroups of (chunk, 16-float slice) — one round on the chip, one LDS-full workgroup per CU.
    (With variable chunks, staged_chunk_starts: the largest chunk.)"""
    st = staged_chunk_starts(grp, d)
    if st is not None:
        return int(np.diff(st).max())
    n_slices = -(-d // 16)
    want = max(1, STAGED_TARGET_BLOCKS // n_slices)        # output chunks
    per = max(1, -(-_staged_n(grp) // want))
    oc = grp.out_chunk * max(1, -(-per // grp.out_chunk))
    return min(oc, 64)


# a staged relation's cost in "nonzeros": its nonzeros plus the per-relation overhead (slab
# copy, tables, barrier) of the staged kernel
STAGED_REL_OVERHEAD = 1500


def snake_bins(costs: Sequence[float], bin_size: int, max_swaps: int = 4000) -> np.ndarray:
    """An order of the items in which every run of `bin_size` consecutive items has about
    the same total cost (a staged launch's output chunk is one or more such runs).  The
    relation sizes are Zipf-skewed (P: 7.5 k - 58 k nonzeros), so dealing in snake order
    leaves the bin with the largest relation 10-50 % over the mean, and that bin's workgroup
    sets the launch time.  Here: rounds of n_bins items (largest first), each round's items
    to the bins in increasing load order; then pairwise swaps between the heaviest bin and
    any other that lower the heaviest load, until none does (deterministic).  Bins are
    emitted heaviest-with-lightest so that runs of two bins balance as well."""
    n = len(costs)
    n_bins = max(1, -(-n // bin_size))
    c = np.asarray(costs, np.float64)
    order = np.argsort(-c, kind="stable")
    B = np.full((n_bins, bin_size), -1, np.int64)     # item ids per bin (-1: empty slot)
    cap = np.full(n_bins, bin_size, np.int64)
    cap[-1] = n - (n_bins - 1) * bin_size               # only the last bin may be short
    fill = np.zeros(n_bins, np.int64)
    load = np.zeros(n_bins)
    r0 = 0
    while r0 < n:
        open_ = np.nonzero(fill < cap)[0]
        items = order[r0:r0 + len(open_)]
        tgt = open_[np.argsort(load[open_], kind="stable")[:len(items)]]
        B[tgt, fill[tgt]] = items
        fill[tgt] += 1
        load[tgt] += c[items]
        r0 += len(items)
    cost = np.where(B >= 0, c[np.maximum(B, 0)], np.nan)
    for _ in range(max_swaps):
        h = int(np.argmax(load))
        ch = cost[h]                                    # [bs]
        d = ch[None, :, None] - cost[:, None, :]        # [bins, bs_h, bs_l]: swap h's i with l's j
        with np.errstate(invalid="ignore"):
            new_max = np.maximum(load[h] - d, load[:, None, None] + d)
            gain = np.where((d > 0) & np.isfinite(d), load[h] - new_max, -np.inf)
        gain[h] = -np.inf
        k = int(np.argmax(gain))
        if not gain.flat[k] > 1e-9:
            break
        l, i, j = np.unravel_index(k, gain.shape)
        dd = d[l, i, j]
        B[h, i], B[l, j] = B[l, j], B[h, i]
        cost[h, i], cost[l, j] = cost[l, j], cost[h, i]
        load[h] -= dd
        load[l] += dd
    full = n_bins - 1 if cap[-1] < bin_size else n_bins
    by = list(np.argsort(-load[:full], kind="stable"))
    seq = []
    while by:
        seq.append(by.pop(0))
        if by:
            seq.append(by.pop())
    seq += list(range(full, n_bins))                     # the short bin last
    out = [int(i) for b in seq for i in B[b] if i >= 0]
    return np.asarray(out, np.int64)


def _tab_balance(d_in: int, d_out: int) -> bool:
    """TAB_BALANCE's choice for a wave-table fused launch (layer 1: d_in == d_out)."""
    return TAB_BALANCE >= 2 or (TAB_BALANCE == 1 and d_in == d_out)


def _tab_groups_fit(tgts, d: int) -> bool:
    """The wave-table fused form finishes a row in one wave, one lane set of d/4 lanes per group
    (PreparedFusedTab): at most 64 / (d/4) groups a target; otherwise the fused-seg form."""
    return all(len(gs) <= 64 // (d // 4) for _, _, gs, _ in tgts)


def choose_chunk(n_rels: int, n_rows: int, nnz: int, d: int, target_waves: int = 32768) -> int:
    """Relations per chunk.  Partials cost 8·d bytes per (chunk, row) against ≈8 bytes per
    nonzero of CSR reads; keep them under a quarter of it, but keep at least `target_waves`
    waves (one per (chunk, row)) to fill 256 CUs when the group is big.  Small groups end
    up as one chunk, which is what lets the fused kernel finish the layer."""
    if n_rels <= 1 or n_rows == 0:
        return max(1, n_rels)
    avg = nnz / float(n_rels * n_rows)
    chunk_traffic = max(1, math.ceil(4.0 * d / max(avg, 1e-9)))
    chunk_par = max(1, (n_rels * n_rows) // target_waves)
    chunk = chunk_par if chunk_traffic <= chunk_par else chunk_traffic
    return int(min(max(1, chunk), n_rels))


def row_slice(c: HostCSR, a: int, b: int) -> HostCSR:
    """Rows [a, b) of a CSR relation (a row-split rank's block), columns unchanged."""
    p0, p1 = int(c.rowptr[a]), int(c.rowptr[b])
    return HostCSR((c.rowptr[a:b + 1] - p0).astype(np.int32), c.col[p0:p1], c.val[p0:p1], (b - a, c.shape[1]))


@dataclass
class DeviceGroup:
    """One (i,j) group's (local) relations on the device, chunk-merged."""

    edge_type: EdgeType
    n_rows: int
    n_cols: int
    K: int                         # relations of the group in the whole graph (slab count)
    rel_ids: np.ndarray            # global relation id of each local relation
    chunk: int
    n_chunks: int
    rowptr: torch.Tensor
    vcol: torch.Tensor
    val: torch.Tensor
    nnz: int
    vcol_max: int
    rel_map: Optional[torch.Tensor] = None   # device rel_ids, when not 0..K-1
    staged: bool = False           # runs through dg_spmm_staged_f32 (layout: chunk = 1)
    out_chunk: int = 1             # staged: snake-bin size (a layer's output chunk is a multiple)
    # staged, variable chunks (STAGED_VAR): (top-level chunk starts, sub-chunk starts), device order
    var_chunks: Optional[Tuple[np.ndarray, np.ndarray]] = None
    # staged, heavy relations in row pieces (staged_pieces): the layout's slab per piece (global
    # relation id; the layout then lists pieces, not rel_ids' relations); None: rel_map
    staged_slab: Optional[torch.Tensor] = None
    layout: Optional["kernels.StagedDevice"] = None  # staged: the diagonal-major layout
    host: Optional[List[HostCSR]] = None  # the local relations (host CSR), device order
    seg: Optional[torch.Tensor] = None    # dg_spmm_seg_f32's segment starts (sparse.chunk_segments)
    # a windowed row-split group's second layout for the reassociated layer 2 (all its relations
    # in one chunk, with segment starts): (rowptr, vcol, val, seg, chunk, n_chunks, vcol_max)
    seg2: Optional[tuple] = None

    @property
    def n_rels(self) -> int:
        return int(self.rel_ids.shape[0])


class DeviceGraph:
    """Every (i,j) group's relations, chunk-merged and uploaded once.

    adj[(i,j)] lists the K_ij relations (HostCSR, or None for relations another rank owns);
    `local` restricts each group to a subset (a rank's shard); `chunk` overrides the
    relations-per-chunk policy (an int for every group, or a dict per edge type)."""

    def __init__(self, edge_types: Dict[EdgeType, int], adj: Dict[EdgeType, Sequence[Optional[HostCSR]]],
                 device: torch.device, local: Optional[Dict[EdgeType, Sequence[int]]] = None,
                 chunk=None, target_waves: int = 32768, d_policy: int = 64,
                 row_block: Optional[Dict[int, Tuple[int, int, int]]] = None, segments: bool = True):
        """segments: also upload each chunk-merged group's segment starts (sparse.chunk_segments)
        for dg_spmm_seg_f32 — groups of at most 16 relations per chunk."""
        self.edge_types = dict(edge_types)
        self.device = device
        self.groups: Dict[EdgeType, DeviceGroup] = {}
        self.n_nodes: Dict[int, int] = {}
        self.sharded = local is not None
        # row-split node types (sharding.py): this rank holds rows [a, b) of every relation
        # into them; their groups' output rows are local row indices
        self.row_block = dict(row_block or {})
        for et, K in self.edge_types.items():
            rels = list(adj[et])
            if len(rels) != K:
                raise ValueError(f"edge type {et}: {len(rels)} matrices fed, {K} expected")
            known = [r for r in rels if r is not None]
            if not known:
                raise ValueError(f"edge type {et}: no relation given")
            n_r, n_c = known[0].shape
            for t, n in ((et[0], n_r), (et[1], n_c)):
                if self.n_nodes.setdefault(t, n) != n:
                    raise ValueError(f"node type {t}: inconsistent sizes {self.n_nodes[t]} vs {n}")
            ids = np.arange(K, dtype=np.int32) if local is None else np.asarray(local[et], np.int32)
            if any(rels[k] is None for k in ids):
                raise ValueError(f"edge type {et}: a local relation was not given")
            loc = [rels[k] for k in ids]
            if et[0] in self.row_block:
                a, b, _ = self.row_block[et[0]]
                loc = [row_slice(c, a, b) for c in loc]
                n_r = b - a
            nnz = int(sum(c.nnz for c in loc))
            ch = chunk.get(et) if isinstance(chunk, dict) else chunk
            staged = ch is None and stageable(len(loc), n_r, n_c)
            out_chunk = 1
            if staged:
                # one chunk per relation; output chunks of out_chunk relations with balanced
                # nonzero counts (relation sizes are Zipf-skewed)
                out_chunk = max(1, -(-len(loc) // STAGED_BINS))
                costs = [c.nnz + STAGED_REL_OVERHEAD for c in loc]
                var, pieces = None, None
                n_top = max(1, STAGED_TARGET_BLOCKS // -(-d_policy // 16))
                if STAGED_VAR:
                    pieces = staged_pieces(loc, costs, n_top, STAGED_PIECE)
                    if len(pieces) == len(loc):
                        pieces = None
                n_v = len(pieces) if pieces is not None else len(loc)
                if STAGED_VAR and n_v <= 65535 and n_v <= 64 * n_top:
                    vcosts = costs if pieces is None else [c.nnz + STAGED_REL_OVERHEAD for _, c in pieces]
                    perm, tops, subs = staged_var_chunks(vcosts, n_top)
                    var = (tops, subs)
                else:
                    pieces = None
                    perm = snake_bins(costs, out_chunk)
                if pieces is None:
                    ids = ids[perm]
                    loc = [loc[i] for i in perm]
                    stage_loc, stage_slab = loc, None
                else:  # the pieces in device order; the group's relations keep their order
                    stage_loc = [pieces[i][1] for i in perm]
                    stage_slab = ids[np.asarray([pieces[i][0] for i in perm], np.int64)].astype(np.int32)
                ch = 1
            if ch is None:
                ch = choose_chunk(len(loc), n_r, nnz, d_policy, target_waves)
            windows = (not staged and loc and ch >= len(loc) and n_r >= WINDOW_MIN_ROWS
                       and N_WINDOWS > 1 and (chunk is None))
            if windows:
                m = merge_windows(loc, ids, N_WINDOWS if n_r >= WINDOW_FULL_ROWS else 2 * N_WINDOWS, K)
            elif loc:
                m = merge_chunks(loc, ids, ch, K)
            else:
                m = MergedCSR(np.zeros(n_r + 1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32),
                              n_r, n_c, 1, 1, K * n_c)
            g = DeviceGroup(
                et, n_r, n_c, K, ids, m.chunk, m.n_chunks,
                torch.from_numpy(m.rowptr).to(device), torch.from_numpy(m.vcol).to(device),
                torch.from_numpy(m.val).to(device), m.nnz,
                int(m.vcol.max()) if m.nnz else -1)
            if ids.size and not np.array_equal(ids, np.arange(K)):
                g.rel_map = torch.from_numpy(ids).to(device)
            g.staged, g.out_chunk = staged, out_chunk
            if staged:
                g.var_chunks = var
                if stage_slab is not None:
                    g.staged_slab = torch.from_numpy(stage_slab).to(device)
            g.host = loc  # local relations in device order (the backward builds Âᵀ from them)
            if segments and loc and not staged and not windows and m.chunk <= 16:
                g.seg = torch.from_numpy(chunk_segments(loc, m)).to(device)
            elif windows and et[0] in self.row_block and len(loc) <= 16 and REASSOC_ROWS:
                # (sharded: layer 2 of this group reassociated over the rank's rows, ForwardPlan)
                m2 = merge_chunks(loc, ids, len(loc), K)
                up = lambda a: torch.from_numpy(a).to(device)  # noqa: E731
                g.seg2 = (up(m2.rowptr), up(m2.vcol), up(m2.val), up(chunk_segments(loc, m2)), m2.chunk, m2.n_chunks,
                          int(m2.vcol.max()) if m2.nnz else -1)
            if staged:
                lay = staged_layout(stage_loc, kernels.staged_block,
                                    lanes=knob("DG_STAGED_LANES", 1024),
                                    split=knob("DG_STAGED_SPLIT", True))
                g.layout = kernels.StagedDevice.upload(lay, device)
            self.groups[et] = g

    @property
    def total_nnz(self) -> int:
        return sum(g.nnz for g in self.groups.values())


@dataclass
class LayerWeights:
    """Weight stacks of one layer: per (i,j) group a tensor [K, d_in, d_out] (device)."""

    stacks: Dict[EdgeType, torch.Tensor]


class ForwardPlan:
    """All buffers and prepared launches of one two-layer forward on one device."""

    # a fused launch projects a row onto at most this many layer-2 relations (VALU epilogue);
    # beyond it the batched MFMA GEMM is used
    FUSED_PROJ_MAX_RELS = knob("DG_FUSED_PROJ_MAX", 64)

    def __init__(self, dgraph: DeviceGraph, features: Dict[int, Optional[HostCSR]],
                 w1: LayerWeights, w2: LayerWeights, h1: int, h2: int,
                 allreduce: Optional[Callable[[torch.Tensor], None]] = None, keep_sums: bool = False,
                 dropout: Optional[Tuple[float, torch.Tensor]] = None, shard=None):
        self.g = dgraph
        self.h1, self.h2 = h1, h2
        # multi-GPU (sharding.RelationShard): the collectives joining the ranks' shares —
        # all-reduce of the relation-sharded node types' sums, all-gather of the row-split
        # node types' finished row blocks
        self.shard = shard
        if shard is not None:
            allreduce = shard.allreduce
        self.allreduce = allreduce
        self.row_block = dict(dgraph.row_block)
        self.world = shard.world_size if shard is not None else 1
        self.allgather = shard.allgather if shard is not None else None
        if self.row_block and (shard is None or shard.row_block != self.row_block
                               or (self.allgather is None and getattr(shard, "peer", None) is None)):
            raise ValueError("a row-split device graph needs its RelationShard (with an all-gather or a peer exchange)")
        if shard is not None and allreduce is None:
            raise ValueError("a RelationShard needs its all-reduce")
        # dropout (training): (keep probability, device state {seed, step}); every forward
        # draws new masks (the step advances first), the backward reuses them
        # (sharded: a relation's masks are keyed by its GLOBAL id, so every rank — and one GPU —
        # masks it identically; each rank masks its own relations only)
        self.keep, self.drop_state = 1.0, None
        if dropout is not None and float(dropout[0]) < 1.0:
            self.keep, self.drop_state = float(dropout[0]), dropout[1]
        # flat mode: every group's pre-normalisation sum S_ij lands in one flat buffer per
        # layer (all-reduced when sharded; kept for the backward when training), and one fused
        # launch over dense-rows groups (DG_GROUP_DENSE_ROWS) finishes every node type from it
        self.flat_mode = allreduce is not None or keep_sums
        self.keep_sums = keep_sums
        self.sums_mode = False  # set below: partial mode whose epilogue also writes each S_ij
        self.launch_groups: Dict[int, List[EdgeType]] = {}  # id(SpMM launch) -> its groups
        dev = dgraph.device
        f32 = dict(device=dev, dtype=torch.float32)
        self.edge_types = list(dgraph.edge_types)
        self.targets: Dict[int, List[EdgeType]] = {}
        for et in self.edge_types:
            self.targets.setdefault(et[0], []).append(et)
        if any(len(v) > DG_MAX_GROUPS for v in self.targets.values()):
            raise ValueError(f"more than {DG_MAX_GROUPS} edge types into one node type")
        if keep_sums and allreduce is None:
            # one GPU, training: when no node type would take the fused path anyway (config P),
            # keep the partial-mode layers and let their one epilogue launch also write every
            # group's pre-normalisation sum S_ij — no flat reduces, no finishing launch
            self.flat_mode = False
            if not self._fused_targets():
                self.sums_mode = True
            else:
                self.flat_mode = True
        n = dgraph.n_nodes
        # config S's weak scaling (RelationShard.weak_sets form "seg"): every node type row-split,
        # its groups in dg_spmm_seg_f32 (one wave per (row, relation), one chunk per relation
        # set) + the epilogue, and layer 2 reassociated, Σ_k (Â_k·H1_j)·W2_k — no projection
        # GEMM over every relation on every rank (forward only: the backward keeps the sums)
        self.seg_mode = (shard is not None and getattr(shard, "seg_rows", False) and not keep_sums
                         and self.drop_state is None and h1 == 64 and h2 == 32
                         and all(et[0] in self.row_block for et in self.edge_types)
                         and all(g.seg is not None or not g.n_rels for g in dgraph.groups.values()))
        # (otherwise such a shard runs the same chunks in dg_spmm_groups_f32 + the epilogue,
        # with the projection GEMM)

        # ---- layer-1 dense operand: W1 (identity features) or X_j·W1_k (sparse features) ----
        self._pre: List[Callable[[], None]] = []
        x1: Dict[EdgeType, torch.Tensor] = {}
        self.et_index = {et: n for n, et in enumerate(self.edge_types)}
        if self.drop_state is not None:
            self._pre.append(lambda st=self.drop_state: kernels.dropout_advance(st))
        for et in self.edge_types:
            i, j = et
            grp = dgraph.groups[et]
            W = w1.stacks[et]
            K, F, dh = W.shape
            if dh != h1 or K != grp.K:
                raise ValueError(f"layer-1 weights of {et} are {tuple(W.shape)}, expected ({grp.K}, *, {h1})")
            fj = features.get(j)
            if fj is None:  # identity features: X_j·W_k ≡ W_k (bit-exact), no kernel
                if F != n[j]:
                    raise ValueError(f"identity features of type {j} need {n[j]} weight rows, got {F}")
                x1[et] = W
                if self.drop_state is not None:
                    # dropout_sparse on the identity (layers.py:87-88): relation k's operand is W1_k
                    # with rows kept / scaled by 1/keep — a masked copy of the stack per forward
                    # (sharded: of the local relations' slabs only, at their global positions)
                    xd = torch.empty_like(W)
                    t = drop_tag(1, self.et_index[et])
                    if grp.rel_map is None:
                        self._pre.append(lambda W=W, xd=xd, t=t: kernels.dropout_rows(W, xd, self.drop_state, t,
                                                                                      self.keep))
                    elif grp.n_rels:
                        self._pre.append(lambda W=W, xd=xd, t=t, m=grp.rel_map, F=F, mx=int(grp.rel_ids.max()):
                                         kernels.dropout_rows_map(W, xd, m, F, self.drop_state, t, self.keep, True,
                                                                  True, rel_map_max=mx))
                    x1[et] = xd
                continue
            if fj.shape[0] != n[j] or fj.shape[1] != F:
                raise ValueError(f"features of type {j} have shape {fj.shape}, weights expect (*, {F})")
            # X_j·W1_k for every relation k of the group (global slabs; sharded ranks compute
            # all of them — sparse features are small next to the adjacency): one copy of X_j's
            # pattern shared by the K chunks, chunk k reading W1_k; with dropout, chunk k masks
            # X_j's values with its own draw (dropout_sparse per relation, layers.py:23-31, :88)
            xw = torch.empty((K, n[j], h1), **f32)
            drop = (None if self.drop_state is None
                    else (self.drop_state, drop_tag(1, self.et_index[et]), self.keep))
            spec = kernels.RelGroupSpec(torch.from_numpy(fj.rowptr).to(dev), torch.from_numpy(fj.col).to(dev),
                                        torch.from_numpy(fj.val).to(dev), W, xw, n[j], K, h1, F,
                                        vcol_max=int(fj.col.max()) if fj.nnz else -1, shared=True, drop=drop)
            self._pre.append(kernels.PreparedSpmm([spec], h1))
            x1[et] = xw

        # row-split node types: the full output rows live in a buffer padded to world × block
        # rows (this rank finishes its block in place, the all-gather fills the rest)
        # (keyed by node type and layer: h1 == h2 must not share a buffer).  Every such buffer
        # is carved from ONE exchange region with the same layout on every rank, which a peer
        # exchange (peer.py) maps into every peer
        self._pad: Dict[Tuple[int, int], torch.Tensor] = {}
        self.xregion: Optional[torch.Tensor] = None
        self.peer = None
        split_nodes = [i for i in self.targets if i in self.row_block]
        # the peer all-reduce (config P's drug rows, peer mode "fused"): the relation-sharded
        # groups' pre-normalisation sums of layer L live in `world` slots of the region, slot r
        # written by rank r's epilogue launch into every rank's copy; the finishing launch adds
        # the slots in rank order (dense-rows groups with n_chunks = world) — no RCCL all-reduce
        pc = getattr(shard, "peer", None)
        self.peer_reduce = (pc is not None and pc.mode == "fused" and self.flat_mode and not keep_sums
                            and self.drop_state is None and bool(split_nodes) and not self.seg_mode
                            and not self._fused_targets() and self._peer_reduce_fits(dgraph, split_nodes))
        self._red_slots: Dict[Tuple[int, EdgeType], torch.Tensor] = {}  # (layer, et) -> [world, n_i, d] view
        if split_nodes:
            layout, off = {}, 0
            for layer, d in ((1, h1), (2, h2)):
                for i in split_nodes:
                    nb = self.world * self.row_block[i][2] * d
                    layout[i, layer] = (off, nb, d)
                    off += -(-nb // 64) * 64  # 256-byte aligned
            red_layout = {}
            if self.peer_reduce:
                for layer, d in ((1, h1), (2, h2)):
                    red = [et for et in self.edge_types if et[0] not in self.row_block]
                    per = sum(n[et[0]] * d for et in red)  # one slot: every group's rows, in order
                    per = -(-per // 64) * 64
                    o2 = 0
                    for et in red:
                        red_layout[layer, et] = (off, o2, per, n[et[0]], d)
                        o2 += n[et[0]] * d
                    off += self.world * per
            # zeros: a slot no rank ever pushes (a group without relations on that rank) reads as
            # zeros forever
            if pc is not None and pc.region_kind:  # (uncached by default: peer.PeerConfig)
                from .peer import device_tensor

                self.xregion = device_tensor(max(off, 64), pc.region_kind, dev)
            else:
                self.xregion = torch.zeros(max(off, 64), **f32)
            for (i, layer), (o, nb, d) in layout.items():
                self._pad[i, layer] = self.xregion[o:o + nb].view(-1, d)
            for key, (base, o2, per, rows, d) in red_layout.items():
                self._red_slots[key] = torch.as_strided(self.xregion, (self.world, rows, d), (per, d, 1),
                                                        base + o2)
            if pc is not None:
                from .peer import PeerExchange

                self.peer = PeerExchange(self.xregion, shard.rank, self.world, pc)

        def out_buf(i, d, layer):
            if i not in self.row_block:
                return torch.empty((n[i], d), **f32)
            return self._pad[i, layer][:n[i]]

        self.hidden1 = {i: out_buf(i, h1, 1) for i in self.targets}
        self.embeddings = {i: out_buf(i, h2, 2) for i in self.targets}

        # ---- layer-2 projection buffers P_k = H1_j·W2_k (global slabs) ----
        # staged groups make their slabs H1_j·W2_k in the layer-2 kernel itself
        # (dg_spmm_staged_proj_f32): no P buffer, no GEMM for them (64-wide H1, no dropout)
        self.staged_proj = {et for et in self.edge_types
                            if dgraph.groups[et].staged and dgraph.groups[et].n_rels and h1 == 64
                            and self.drop_state is None and STAGED_PROJ}
        # one GPU (config S): every node type finished by dg_gcn_fused_seg_f32 — one workgroup
        # per row, one wave per relation — with layer 2 reassociated (no projection in layer 1,
        # no GEMM), when every group is one chunk of <= 16 relations per row in total
        self.fused_seg = (FUSED_SEG and not self.flat_mode and not self.row_block and self.drop_state is None
                          and h1 == 64 and h2 == 32
                          and all(g.seg is not None and g.n_chunks == 1 and g.chunk == g.n_rels >= 1
                                  and not g.staged for g in dgraph.groups.values())
                          and all(sum(dgraph.groups[et].n_rels for et in ets) <= 16
                                  for ets in self.targets.values()))
        self.seg_proj = {et for et in self.edge_types
                         if (self.seg_mode or self.fused_seg) and dgraph.groups[et].n_rels and h1 == 64 and h2 == 32}
        # sharded forward plans: every other non-staged group's layer 2 reassociated as well, over
        # the rank's own rows / relations (config P: PPI in its one-chunk layout, (0,1), (1,0)),
        # so no rank runs a projection GEMM over all of H1 (REASSOC_ROWS)
        self.seg_proj |= {et for et in self.edge_types
                          if REASSOC_ROWS and shard is not None and not keep_sums and self.drop_state is None
                          and h1 == 64 and h2 == 32 and dgraph.groups[et].n_rels and not dgraph.groups[et].staged
                          and (dgraph.groups[et].seg is not None or dgraph.groups[et].seg2 is not None)}
        self.seg_l1 = {et for et in self.edge_types
                       if SEG_ROWS_L1 and shard is not None and not self.seg_mode and not keep_sums
                       and self.drop_state is None and h1 in (32, 64) and et[0] in self.row_block
                       and dgraph.groups[et].n_rels and not dgraph.groups[et].staged
                       and dgraph.groups[et].seg is not None}
        self.proj: Dict[EdgeType, torch.Tensor] = {}
        for et in self.edge_types:
            grp = dgraph.groups[et]
            K, din, dout = w2.stacks[et].shape
            if din != h1 or dout != h2 or K != grp.K:
                raise ValueError(f"layer-2 weights of {et} are {(K, din, dout)}, expected ({grp.K}, {h1}, {h2})")
            if et[1] not in self.hidden1:
                raise ValueError(f"node type {et[1]} has no incoming edge type; layer 2 needs hidden1[{et[1]}]")
            if et not in self.staged_proj and et not in self.seg_proj:
                self.proj[et] = torch.empty((K, n[et[1]], h2), **f32)

        # a second stream: a layer's gather-bound launch (dg_spmm_groups_f32) runs beside its
        # LDS-bound staged launch (dg_spmm_staged_f32) — different units, no data dependence
        self.side_stream = (torch.cuda.Stream(dev) if dev.type == "cuda" and CONCURRENT_LAUNCHES else None)

        # ---- layer 1 (+ the layer-2 projections of rows it finishes) ----
        self.fused = list(self.targets) if self.fused_seg else self._fused_targets()
        rels_from: Dict[int, int] = {}
        for et in self.edge_types:
            rels_from[et[1]] = rels_from.get(et[1], 0) + dgraph.groups[et].n_rels
        # layer-1 rows finished by a fused launch (the SpMM one, or — sharded — the one that
        # finishes the all-reduced sums) project themselves onto the layer-2 relations
        finished = (set(self.targets) - set(self.row_block)) if self.flat_mode else set(self.fused)
        proj_fused = [et for et in self.edge_types
                      if dgraph.groups[et].n_rels and et[1] in finished and et not in self.staged_proj
                      and et not in self.seg_proj
                      and rels_from[et[1]] <= self.FUSED_PROJ_MAX_RELS and self.drop_state is None]
        if len(proj_fused) > DG_MAX_GROUPS:
            proj_fused = []
        projs = []
        for et in proj_fused:
            grp = dgraph.groups[et]
            projs.append((et[1], kernels.ProjSpec(
                w2.stacks[et], self.proj[et], grp.n_rels, -1, rel_map=grp.rel_map,
                rel_map_max=int(grp.rel_ids.max()) if grp.rel_map is not None else None)))
        self._layer1 = self._build_layer(x1, h1, True, f32, projs)

        # ---- layer 2: remaining projections in one batched MFMA GEMM launch, then SpMM ----
        gemms, drops = [], []
        self.hdrop: Dict[EdgeType, torch.Tensor] = {}
        for et in self.edge_types:
            grp = dgraph.groups[et]
            if not grp.n_rels or et in proj_fused or et in self.staged_proj or et in self.seg_proj:
                continue
            j = et[1]
            W = w2.stacks[et]
            if self.drop_state is not None:
                # tf.nn.dropout(H1_j) drawn per relation (layers.py:111-113): H_k = M_k∘H1_j/keep,
                # one slab per LOCAL relation in ascending relation id (the backward's dP order;
                # sharded: slab b is relation sorted_ids[b], its mask drawn under that global id),
                # projected into P's global slabs
                hd = torch.empty((grp.n_rels, n[j], h1), **f32)
                self.hdrop[et] = hd
                t = drop_tag(2, self.et_index[et])
                sids = np.sort(grp.rel_ids).astype(np.int32)
                smap = None if np.array_equal(sids, np.arange(grp.K)) else torch.from_numpy(sids).to(dev)
                if smap is None:
                    drops.append(lambda j=j, hd=hd, t=t: kernels.dropout_elems(self.hidden1[j], hd, self.drop_state,
                                                                               t, self.keep))
                else:
                    drops.append(lambda j=j, hd=hd, t=t, m=smap, mx=int(sids.max()): kernels.dropout_elems_map(
                        self.hidden1[j], hd, m, self.drop_state, t, self.keep, rel_map_max=mx))
                gemms.append(kernels.PreparedGemm(
                    hd, (n[j] * h1, h1, 1), W, (h1 * h2, h2, 1), self.proj[et], (n[j] * h2, h2, 1),
                    n[j], h2, h1, grp.n_rels, b_map=smap, b_batches=W.shape[0],
                    b_map_max=int(sids.max()) if smap is not None else None))
                continue
            gemms.append(kernels.PreparedGemm(
                self.hidden1[j], (0, h1, 1), W, (h1 * h2, h2, 1), self.proj[et], (n[j] * h2, h2, 1),
                n[j], h2, h1, grp.n_rels, b_map=grp.rel_map, b_batches=W.shape[0],
                b_map_max=int(grp.rel_ids.max()) if grp.rel_map is not None else None))
        self._gemm2 = drops + [kernels.PreparedGemmMulti(gemms[s:s + DG_MAX_GROUPS])
                               for s in range(0, len(gemms), DG_MAX_GROUPS)]
        self._layer2 = self._build_layer(self.proj, h2, False, f32,
                                         staged_proj={et: (self.hidden1[et[1]], w2.stacks[et])
                                                      for et in self.staged_proj},
                                         seg_w={et: (self.hidden1[et[1]], w2.stacks[et]) for et in self.seg_proj})

    # ------------------------------------------------------------------ layer builder
    def _fused_targets(self) -> List[int]:
        """Node types one dg_gcn_fused_f32 launch finishes: at most FUSED_MAX_ROWS (local) rows,
        every group one chunk (and not staged).  Sharded plans finish only row-split node types
        this way, when the shard asks for it (`fused_rows`: their rows are complete on this
        rank; relation-sharded ones need the all-reduce first), and the sharded backward takes
        none."""
        if self.flat_mode and (self.keep_sums or not self.row_block
                               or not getattr(self.shard, "fused_rows", False)):
            return []

        def rows(i):
            if i in self.row_block:
                return self.row_block[i][1] - self.row_block[i][0]
            return self.g.n_nodes[i]

        return [i for i, ets in self.targets.items()
                if (not self.flat_mode or i in self.row_block)
                and 0 < rows(i) <= FUSED_MAX_ROWS
                and all(self.g.groups[et].n_chunks == 1 and self.g.groups[et].n_rels > 0
                        and not self.g.groups[et].staged for et in ets)]

    def _spec(self, et, x: torch.Tensor, out, d) -> kernels.RelGroupSpec:
        grp = self.g.groups[et]
        return kernels.RelGroupSpec(grp.rowptr, grp.vcol, grp.val, x, out, grp.n_rows, grp.n_chunks, d,
                                    grp.K * grp.n_cols, vcol_max=grp.vcol_max)

    def _seg_spec(self, et, x: torch.Tensor, out=None, w=None) -> kernels.SegSpec:
        grp = self.g.groups[et]
        if grp.seg is None and grp.seg2 is not None:  # a windowed group's one-chunk layout
            rp, vc, vv, sg, ch, nc, vmax = grp.seg2
        else:
            rp, vc, vv, sg, ch, nc, vmax = grp.rowptr, grp.vcol, grp.val, grp.seg, grp.chunk, grp.n_chunks, grp.vcol_max
        return kernels.SegSpec(rp, sg, vc, vv, x, out, grp.n_rows, grp.n_cols, nc, ch, grp.n_rels, x.stride(-2),
                               grp.K * grp.n_cols, vcol_max=vmax, w=w, slab=grp.rel_map,
                               slab_max=int(grp.rel_ids.max()) if grp.n_rels else -1)

    def _seg_chunks(self, et) -> int:
        grp = self.g.groups[et]
        return grp.seg2[5] if (grp.seg is None and grp.seg2 is not None) else grp.n_chunks

    def _build_layer(self, xs: Dict[EdgeType, torch.Tensor], d, relu, f32, projs=(), staged_proj=None, seg_w=None):
        """Prepared launches of one layer: fused targets in one dg_gcn_fused_f32 launch; the
        other targets' groups in partial mode + epilogue — with, when sharded, the chunk
        reduce into the all-reduce buffer and the all-reduce before the epilogue."""
        g = self.g
        n = g.n_nodes
        outs = self.hidden1 if relu else self.embeddings
        launches: List[Callable[[], None]] = []
        fused_t = self.fused
        gathers = []
        if self.seg_mode and SEG_FUSED and all(sum(g.groups[et].n_rels for et in ets) <= SEG_FUSED_MAX_ITEMS
                                               for ets in self.targets.values()):
            # every node type row-split: one launch finishes this rank's row block of each
            # (its workgroups' waves loop over the N relation sets), then the all-gathers
            seg_w = seg_w or {}
            tgts = []
            for i in self.targets:
                a, b, blk = self.row_block[i]
                pad = self._pad[i, 1 if relu else 2]
                r0 = self.shard.rank * blk
                gathers.append((pad, pad[r0:r0 + blk]))
                tgts.append((pad[r0:r0 + (b - a)], b - a,
                             [self._seg_spec(et, seg_w[et][0], None, seg_w[et][1]) if et in seg_w
                              else self._seg_spec(et, xs[et]) for et in self.targets[i]], relu))
            fused_peer = self._peer_fused(relu)
            d_in = self.h1 if seg_w else d
            if WAVE_TABLE and d_in == 64 and (d == 64 or seg_w) and _tab_groups_fit(tgts, d):
                # (one wave per relation here: dealing the pairs of N = 2's 14-relation rows over
                # 16 wave slots measured 16.45 / 23.04 µs a rank against 16.39 / 22.65, RCCL no-op /
                # peer loopback, round 6)
                launches.append(kernels.PreparedFusedTab(tgts, d_in, d, peer=fused_peer, balance=False))  # (the wave-table form)
            else:
                launches.append(kernels.PreparedFusedSeg(tgts, d_in, d, peer=fused_peer))
            self.launch_groups[id(launches[-1])] = [et for i in self.targets for et in self.targets[i]]
            if fused_peer is not None:
                gathers = []  # the launch itself ends with the exchange
            return _Layer(launches, None, False, self.allreduce, [], [], {}, self.side_stream, None, (), gathers,
                          self.allgather, self._peer_gather_all(gathers, relu))
        if self.fused_seg:
            seg_w = seg_w or {}
            tgts = [(outs[i], n[i], [self._seg_spec(et, seg_w[et][0], None, seg_w[et][1]) if et in seg_w
                                     else self._seg_spec(et, xs[et]) for et in self.targets[i]], relu)
                    for i in fused_t]
            d_in = self.h1 if seg_w else d
            if WAVE_TABLE and d_in == 64 and (d == 64 or seg_w) and _tab_groups_fit(tgts, d):
                # the wave-table form: the same rows bitwise, fewer dependent loads a wave
                launches.append(kernels.PreparedFusedTab(tgts, d_in, d, balance=_tab_balance(d_in, d)))
            else:
                launches.append(kernels.PreparedFusedSeg(tgts, d_in, d))
            self.launch_groups[id(launches[-1])] = [et for i in fused_t for et in self.targets[i]]
        elif fused_t:
            # waves per group: small launches (latency-bound) split the densest row group's
            # batches of 64 over up to two waves; big launches have parallelism to spare
            avg = max(g.groups[et].nnz / max(1, g.groups[et].n_rows) for i in fused_t for et in self.targets[i])
            max_groups = max(len(self.targets[i]) for i in fused_t)
            rows = sum(g.groups[self.targets[i][0]].n_rows for i in fused_t)
            # (row blocks of N relation sets — config S's weak scaling — have N times longer
            # rows over 1/N of the rows: up to 16 waves per row there; measured at N = 8, rank
            # 0's layer 1: 27.0 µs at 2 waves per group)
            cap = 16 // max_groups if self.row_block else 2
            wpg = 1 if rows >= 4096 else int(max(1, min(cap, 16 // max_groups, math.ceil(avg / 64.0))))
            if knob("DG_WPG", 0):  # tuning override
                wpg = max(1, min(knob("DG_WPG", 0), 16 // max_groups))
            pspecs = []
            for tgt_node, pj in projs:
                if tgt_node in fused_t:  # (sharded: the finishing launch projects the others)
                    pj.target = fused_t.index(tgt_node)
                    pspecs.append(pj)
            tgts = []
            for i in fused_t:
                out, rows_i = outs[i], n[i]
                if i in self.row_block:
                    # a row-split node type (sharded): this rank's block, finished in place in the
                    # padded output, then all-gathered
                    a, b, blk = self.row_block[i]
                    pad = self._pad[i, 1 if relu else 2]
                    r0 = self.shard.rank * blk
                    out, rows_i = pad[r0:r0 + (b - a)], b - a
                    gathers.append((pad, pad[r0:r0 + blk]))
                tgts.append((out, rows_i, [self._spec(et, xs[et], None, d) for et in self.targets[i]], relu))
            launches.append(kernels.PreparedFused(tgts, d, pspecs, wpg))
            self.launch_groups[id(launches[-1])] = [et for i in fused_t for et in self.targets[i]]
        rest = [et for et in self.edge_types if et[0] not in fused_t]
        flags = DG_EPI_L2NORM | (DG_EPI_RELU if relu else 0)
        # row-split node types (sharded) not finished by the fused launch: their groups run in
        # partial mode over this rank's row block and one epilogue finishes the block before
        # the exchange
        split_t = [i for i in self.targets if i in self.row_block and i not in fused_t]
        red = [et for et in rest if et[0] not in self.row_block]
        flat, views, send, sviews = None, {}, None, {}
        layer_no = 1 if relu else 2
        # the peer all-reduce: each relation-sharded group's sum goes to this rank's slot (and
        # every peer's copy of it) from the epilogue launch; no flat buffer, no RCCL all-reduce
        peer_red = self.peer_reduce and bool(red) and bool(split_t)
        if peer_red:
            for et in red:
                sviews[et] = self._red_slots[layer_no, et][self.shard.rank]
        elif self.flat_mode and red:
            # flat (the reduced sums, read by the finishing launch and the backward) and, when
            # sharded, send (this rank's partial sums, written by its SpMM / reduces): the
            # all-reduce runs out of place, so the regions of groups without local relations
            # stay zero from allocation on — no per-step fill
            sizes = [g.groups[et].n_rows * d for et in red]
            flat = torch.zeros(int(sum(sizes)), **f32)
            send = torch.zeros_like(flat) if self.allreduce is not None else flat
            off = 0
            for et, sz in zip(red, sizes):
                views[et] = flat[off:off + sz]
                sviews[et] = send[off:off + sz]
                off += sz
        partials, specs, staged, reduces, segs = {}, [], [], [], []
        # outside seg mode: layer 2 reassociated (seg_w) and, in layer 1, the row-split groups of
        # SEG_ROWS_L1 — both in dg_spmm_seg_f32
        reassoc = (set(seg_w or {}) | (self.seg_l1 if relu else set())) if not self.seg_mode else set()
        for et in rest:
            grp = g.groups[et]
            cst = staged_chunk_starts(grp, d) if grp.staged else None
            n_out = ((len(cst) - 1 if cst is not None else -(-_staged_n(grp) // staged_out_chunk(grp, d)))
                     if grp.staged else grp.n_chunks)
            if et in reassoc:
                n_out = self._seg_chunks(et)
            if flat is not None and et in views and n_out == 1:
                part = sviews[et]  # single chunk: the SpMM writes the group sum in place
            else:
                part = torch.zeros((max(1, n_out), grp.n_rows, d), **f32)
                if flat is not None and et in views and grp.n_rels:
                    reduces.append(kernels.PreparedEpilogue([(part, n_out)], sviews[et], grp.n_rows, d, 0))
            partials[et] = (part, max(1, n_out))
            if not grp.n_rels:
                continue
            if grp.staged:
                sp = (staged_proj or {}).get(et)
                staged.append(kernels.StagedSpec(
                    grp.layout, grp.staged_slab if grp.staged_slab is not None else grp.rel_map, xs.get(et), part, staged_out_chunk(grp, d), d, grp.K * grp.n_cols,
                    slab_max=int(grp.rel_ids.max()), proj=sp, chunk_start=cst))
            elif self.seg_mode or et in reassoc:
                if et in (seg_w or {}):  # layer 2 reassociated: H1_j and W2's stack
                    segs.append(self._seg_spec(et, seg_w[et][0], part, seg_w[et][1]))
                else:
                    segs.append(self._seg_spec(et, xs[et], part))
            else:
                specs.append(self._spec(et, xs[et], part, d))
        spmm_ets = [et for et in rest if g.groups[et].n_rels and not g.groups[et].staged
                    and not (self.seg_mode or et in reassoc)]
        seg_ets = [et for et in rest if g.groups[et].n_rels and not g.groups[et].staged
                   and (self.seg_mode or et in reassoc)]
        if segs:
            d_in = self.h1 if seg_w else d
            for s in range(0, len(segs), DG_MAX_GROUPS):
                part = segs[s:s + DG_MAX_GROUPS]
                if WAVE_TABLE and kernels._tab_shape(d_in, d, part):
                    launches.append(kernels.PreparedSegTab(part, d_in, d))  # (the wave-table form)
                else:
                    launches.append(kernels.PreparedSeg(part, d_in, d))
                self.launch_groups[id(launches[-1])] = seg_ets[s:s + DG_MAX_GROUPS]
        staged_ets = [et for et in rest if g.groups[et].n_rels and g.groups[et].staged]
        for s in range(0, len(staged), DG_MAX_GROUPS):
            launches.append(kernels.PreparedStaged(staged[s:s + DG_MAX_GROUPS], d))
            self.launch_groups[id(launches[-1])] = staged_ets[s:s + DG_MAX_GROUPS]
        for s in range(0, len(specs), DG_MAX_GROUPS):
            launches.append(kernels.PreparedSpmm(specs[s:s + DG_MAX_GROUPS], d))
            self.launch_groups[id(launches[-1])] = spmm_ets[s:s + DG_MAX_GROUPS]
        need_zero = send is flat and flat is not None and any(g.groups[et].n_rels == 0 for et in red)
        epis, local_epis = [], []
        epi_peer = self._peer_fused(relu) if split_t else None
        if split_t:
            blocks = []
            for i in split_t:
                a, b, blk = self.row_block[i]
                pad = self._pad[i, 1 if relu else 2]
                r0 = self.shard.rank * blk
                parts = [partials[et] for et in self.targets[i]]
                if self.keep_sums:
                    # training: the epilogue also keeps each group's pre-normalisation sum S_ij over
                    # this rank's block rows (the backward's l2-norm gradient reads them)
                    for n_, et in enumerate(self.targets[i]):
                        views[et] = torch.empty((b - a) * d, **f32)
                        parts[n_] = (parts[n_][0], parts[n_][1], views[et])
                blocks.append((parts, pad[r0:r0 + (b - a)], b - a))
                if epi_peer is None:  # (else the epilogue launch itself ends with the exchange)
                    gathers.append((pad, pad[r0:r0 + blk]))
            n_push = len(blocks)
            # the relation-sharded node types' chunk reduces ride in the same launch: a target
            # whose groups write their pre-normalisation sums into the send buffer (its
            # finished rows go to a scratch buffer, unread) — one launch per layer instead of two
            if peer_red:
                # every relation-sharded group with local relations: its sum into this rank's
                # slot, pushed to every peer (the rest of the slot stays zero)
                red_t = [i for i in self.targets if i not in self.row_block
                         and any(g.groups[et].n_rels for et in self.targets[i])]
            else:
                red_t = [i for i in self.targets if i not in self.row_block
                         and any(et in views and g.groups[et].n_rels and partials[et][1] > 1
                                 for et in self.targets[i])]
            n_groups = sum(len(self.targets[i]) for i in split_t + red_t)
            fits = len(split_t) + len(red_t) <= 8 and n_groups <= DG_MAX_GROUPS
            # (__init__ enabled peer_red only where _peer_reduce_fits said these targets fit)
            assert fits or not peer_red
            if (reduces or peer_red) and fits:
                for i in red_t:
                    grp_parts = []
                    for et in self.targets[i]:
                        part, nc = partials[et][:2]
                        if peer_red:
                            grp_parts.append((part, nc, sviews[et] if g.groups[et].n_rels else None, True))
                            continue
                        reduced = et in views and g.groups[et].n_rels and nc > 1
                        grp_parts.append((part, nc, sviews[et] if reduced else None))
                    blocks.append((grp_parts, torch.empty((n[i], d), **f32), n[i]))
                reduces = []
            local_epis.append(_epilogue(blocks, d, flags, peer=epi_peer, push=[t < n_push for t in range(len(blocks))]))
        launches += reduces
        if peer_red:
            # the relation-sharded rows finished from the world slots, added in rank order by
            # the dense-rows groups of ONE fused launch (l2norm, Σ_j, relu, layer-1 projections)
            tl = [i for i in self.targets if i not in self.row_block]
            pspecs = []
            for tgt_node, pj in projs:
                pj.target = tl.index(tgt_node)
                pspecs.append(pj)

            def slots_spec(i, et):
                sl = self._red_slots[layer_no, et]
                per = sl.stride(0)
                x = torch.as_strided(self.xregion, ((self.world - 1) * per + n[i] * d,), (1,), sl.storage_offset())
                return kernels.RelGroupSpec(None, None, None, x, None, n[i], self.world, d, per // d, dense=True)

            epis.append(kernels.PreparedFused(
                [(outs[i], n[i], [slots_spec(i, et) for et in self.targets[i]], relu) for i in tl], d, pspecs, 1))
        elif flat is not None:
            # sharded: the all-reduced group sums S_ij are finished by ONE fused launch whose
            # groups are the dense rows S_ij[r] themselves (DG_GROUP_DENSE_ROWS), so the l2norm,
            # Σ_j, relu and (layer 1) the layer-2 projections of every node type run in one
            # kernel after the exchange
            tl = [i for i in self.targets if i not in self.row_block]
            pspecs = []
            for tgt_node, pj in projs:
                pj.target = tl.index(tgt_node)
                pspecs.append(pj)
            epis.append(kernels.PreparedFused(
                [(outs[i], n[i], [self._identity_spec(i, views[et], d) for et in self.targets[i]], relu)
                 for i in tl], d, pspecs, 1))
        elif not split_t:
            if self.sums_mode:  # training: the epilogue also writes each group's S_ij
                for et in rest:
                    views[et] = torch.empty(g.groups[et].n_rows * d, **f32)
                    partials[et] = partials[et] + (views[et],)
            # every partial-mode node type finishes in ONE launch (side by side, no stream fork)
            tl = [i for i in self.targets if i not in fused_t]
            # node types with the most chunk partials per row first: their long rows start early
            tl.sort(key=lambda i: -sum(partials[et][1] for et in self.targets[i]))
            if tl:
                epis.append(_epilogue([([partials[et] for et in self.targets[i]], outs[i], n[i]) for i in tl], d, flags))
        return _Layer(launches, flat, need_zero, self.allreduce, epis, fused_t, views, self.side_stream, send,
                      local_epis, gathers, self.allgather, self._peer_gather_all(gathers, relu))

    # ---- peer exchange (peer.py) ----
    def _peer_reduce_fits(self, dgraph, split_nodes) -> bool:
        """Whether the pushing epilogue launch can carry the peer all-reduce: the row-split node
        types plus every relation-sharded node type with local relations as targets of ONE
        dg_gcn_epilogue_peer_f32 launch (<= 8 targets, <= DG_MAX_GROUPS groups).  A larger graph
        keeps the flat buffer and the RCCL all-reduce instead (it used to raise)."""
        red_t = [i for i in self.targets if i not in self.row_block
                 and any(dgraph.groups[et].n_rels for et in self.targets[i])]
        t = list(split_nodes) + red_t
        return len(t) <= 8 and sum(len(self.targets[i]) for i in t) <= DG_MAX_GROUPS

    def _peer_fused(self, layer1: bool):
        """(PeerExchange, slot) for a finishing launch that pushes its rows and exchanges, or None."""
        if self.peer is None or self.peer.cfg.mode != "fused":
            return None
        from .peer import SLOT_FUSED

        return self.peer, SLOT_FUSED + (0 if layer1 else 1)

    def _peer_gather_all(self, gathers, layer1: bool):
        """With a peer exchange, the layer's remaining all-gathers as ONE stand-alone
        dg_peer_allgather launch (mode "kernel", or a finishing launch without a push form)."""
        if self.peer is None or not gathers:
            return None
        from .peer import SLOT_KERNEL

        return self.peer.allgather_fn([blk for _, blk in gathers], SLOT_KERNEL + (0 if layer1 else 1))

    def peer_probe(self):
        """bench.py: each layer's stand-alone peer exchange of this rank's blocks (slots
        SLOT_PROBE + layer - 1), to time beside whatever exchange the plan runs."""
        from .peer import SLOT_PROBE

        out = []
        for layer in (1, 2):
            blks = [self._pad[i, layer][self.shard.rank * self.row_block[i][2]:
                                        (self.shard.rank + 1) * self.row_block[i][2]]
                    for i in self.targets if i in self.row_block]
            if blks:
                out.append(self.peer.allgather_fn(blks, SLOT_PROBE + layer - 1))
        return out

    def _identity_spec(self, i: int, x: torch.Tensor, d: int) -> kernels.RelGroupSpec:
        """A group spec with no adjacency (DG_GROUP_DENSE_ROWS): the fused kernel reads the dense
        rows x[r] as the group sums."""
        n_i = self.g.n_nodes[i]
        return kernels.RelGroupSpec(None, None, None, x, None, n_i, 1, d, n_i, dense=True)

    def run_layer1(self) -> None:
        for p in self._pre:
            p()
        self._layer1.run()

    def run_layer2(self) -> None:
        for gm in self._gemm2:
            gm()
        self._layer2.run()

    def run(self) -> None:
        if self.peer is not None:
            self.peer.ensure_ok()  # a timed-out exchange found by an earlier check poisons the plan
        self.run_layer1()
        self.run_layer2()

    def phases(self) -> List[Tuple[str, Callable[[], None]]]:
        """The forward as alternating ("compute", fn) / ("exchange", fn) phases: the device
        launches between two collectives form one compute phase (capturable into one
        hipGraph), each layer's all-reduce of its pre-normalisation sums is an exchange."""
        out: List[Tuple[str, Callable[[], None]]] = []
        cur: List[Callable[[], None]] = []

        def close():
            if cur:
                fns = list(cur)
                out.append(("compute", lambda: [f() for f in fns]))
                cur.clear()

        cur.extend(self._pre)
        for layer, before in ((self._layer1, []), (self._layer2, self._gemm2)):
            cur.extend(before)
            if layer.need_zero:
                cur.append(layer.flat.zero_)
            cur.append(layer.run_spmm)
            cur.extend(layer.local_epilogues)
            if layer.has_exchange:
                close()
                out.append(("exchange", layer.exchange))
            cur.extend(layer.epilogues)
        close()
        return out

    def parallelism(self, backend: str = "nccl") -> str:
        return "1 GPU" if self.shard is None else self.shard.describe(backend)

    @property
    def spmm_launches(self):
        """(layer-1, layer-2) SpMM launches (fused or partial) — what the roofline times."""
        kinds = (kernels.PreparedSpmm, kernels.PreparedFused, kernels.PreparedStaged, kernels.PreparedSeg,
                 kernels.PreparedFusedSeg)
        pick = lambda L: [l for l in L.launches if isinstance(l, kinds)]
        return pick(self._layer1), pick(self._layer2)

    # ---- accounting (bench / DESIGN.md roofline) ----
    def _out_rows(self, i: int) -> int:
        """Rows of node type i this plan finishes (a row-split rank: its block)."""
        if i in self.row_block:
            return self.row_block[i][1] - self.row_block[i][0]
        return self.g.n_nodes[i]

    def group_bytes(self, et: EdgeType, d: int, fused: bool, layer: int = 1) -> int:
        """Algorithmic bytes of one group's SpMM: its CSR once (4 B per row of each
        relation + 8 B per nonzero), its dense operands once (4·d B per row of each X_k) and,
        in partial mode, its sum S_ij once (4·d B per output row)."""
        grp = self.g.groups[et]
        if not grp.n_rels:
            return 0
        tot = 4 * (grp.n_rels * grp.n_rows + 1) + 8 * grp.nnz
        if layer == 2 and (et in self.staged_proj or et in self.seg_proj):  # H1_j and W2 instead of P_k
            tot += 4 * self.h1 * (grp.n_cols + d * grp.n_rels)
        else:
            tot += 4 * d * grp.n_cols * grp.n_rels
        return tot if fused else tot + 4 * d * grp.n_rows

    def launch_bytes(self, launch, layer: int) -> int:
        """Algorithmic bytes of one SpMM launch of a layer (its groups; a fused launch also
        writes its targets' rows once, and in layer 1 reads W2 / writes P for its fused
        projections)."""
        L = self._layer1 if layer == 1 else self._layer2
        d = self.h1 if layer == 1 else self.h2
        ets = self.launch_groups.get(id(launch), [])
        fused = isinstance(launch, (kernels.PreparedFused, kernels.PreparedFusedSeg))
        tot = sum(self.group_bytes(et, d, fused, layer) for et in ets)
        if fused:
            tot += sum(4 * d * self._out_rows(i) for i in L.fused_targets)
            if layer == 1 and isinstance(launch, kernels.PreparedFused):
                for pj in launch._keep[2]:
                    K, din, dout = pj.w.shape
                    tot += 4 * pj.n_rels * (din * dout + pj.out.shape[1] * dout)
        return tot

    def layer_bytes(self, layer: int) -> int:
        """Algorithmic (compulsory) HBM bytes of one layer's SpMM launches: the CSR once
        (row pointers 4 B per row of each relation, vcol+val 8 B per nonzero), every distinct
        dense operand X_k once (4·d B per row of X_k), the output once — 4·d B per row of each
        group's sum S_ij in partial mode (chunk / window partials are the implementation's
        choice, not counted), per output row in fused mode — and, for layer 1, the fused
        projections' W2 reads and P writes."""
        L = self._layer1 if layer == 1 else self._layer2
        d = self.h1 if layer == 1 else self.h2
        tot = 0
        for et, grp in self.g.groups.items():
            if not grp.n_rels:
                continue
            tot += 4 * (grp.n_rels * grp.n_rows + 1) + 8 * grp.nnz
            if layer == 2 and (et in self.staged_proj or et in self.seg_proj):  # H1_j and W2 instead of P_k
                tot += 4 * self.h1 * (grp.n_cols + d * grp.n_rels)
            else:
                tot += 4 * d * grp.n_cols * grp.n_rels
            if et[0] not in L.fused_targets:
                tot += 4 * d * grp.n_rows
        for i in L.fused_targets:
            tot += 4 * d * self._out_rows(i)
        if layer == 1:
            for f in L.launches:
                if isinstance(f, kernels.PreparedFused):
                    for pj in f._keep[2]:
                        K, din, dout = pj.w.shape
                        rows = pj.out.shape[1]
                        tot += 4 * pj.n_rels * (din * dout + rows * dout)
        return tot


class _Layer:
    """The prepared launches of one layer and how to run them."""

    def __init__(self, launches, flat, need_zero, allreduce, epilogues, fused_targets, views=None,
                 side_stream=None, send=None, local_epilogues=(), gathers=(), allgather=None, gather_all=None):
        self.launches = launches
        self.side_stream = side_stream
        self.flat = flat
        self.send = flat if send is None else send  # this rank's partial sums (sharded: all-reduced into flat)
        self.views = views or {}  # flat mode: (i,j) -> that group's S_ij, [n_i * d]
        self.need_zero = need_zero
        self.allreduce = allreduce
        self.epilogues = epilogues
        self.fused_targets = fused_targets
        self.local_epilogues = list(local_epilogues)  # row-split blocks, finished before the exchange
        self.gathers = list(gathers)                  # (padded out, this rank's block) per node type
        self.allgather = allgather
        self.gather_all = gather_all                  # all gathers in one peer-exchange launch

    @property
    def has_exchange(self) -> bool:
        return (self.flat is not None and self.allreduce is not None) or bool(self.gathers)

    def exchange(self) -> None:
        """The layer's collectives: all-reduce of the relation-sharded sums, then the
        all-gather of the row-split blocks."""
        if self.flat is not None and self.allreduce is not None:
            self.allreduce(self.send, self.flat)
        if self.gather_all is not None:
            self.gather_all()
            return
        for out, blk in self.gathers:
            self.allgather(out, blk)

    def run(self) -> None:
        if self.need_zero:
            self.flat.zero_()  # groups without local relations contribute zeros
        self.run_spmm()
        for e in self.local_epilogues:
            e()
        if self.has_exchange:
            self.exchange()
        for e in self.epilogues:
            e()

    def run_spmm(self) -> None:
        """The layer's SpMM launches (and chunk reduces), as the forward runs them."""
        side = [l for l in self.launches if isinstance(l, kernels.PreparedSpmm)]
        main = [l for l in self.launches if not isinstance(l, kernels.PreparedSpmm)]
        if (self.side_stream is not None and side
                and any(isinstance(l, kernels.PreparedStaged) for l in main)):
            # fork: the gather-bound launches on the side stream, the LDS-bound staged ones
            # here; join before the chunk reduces / epilogues (graph-capturable)
            cur = torch.cuda.current_stream()
            self.side_stream.wait_stream(cur)
            if STAGED_FIRST:  # the LDS-full staged workgroups claim their CUs first
                for l in main:
                    if not isinstance(l, kernels.PreparedEpilogue):
                        l()
            with torch.cuda.stream(self.side_stream):
                for l in side:
                    l()
            if not STAGED_FIRST:
                for l in main:
                    if not isinstance(l, kernels.PreparedEpilogue):
                        l()
            cur.wait_stream(self.side_stream)
            for l in main:
                if isinstance(l, kernels.PreparedEpilogue):
                    l()
        else:
            for l in self.launches:
                l()
