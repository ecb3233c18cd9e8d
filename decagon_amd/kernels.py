"""Typed Python entry points over the C ABI (include/decagon_hip.h).

Every wrapper checks on the host, before launching, that the device buffers are large
enough for the indices the kernel will form (a bad shape must fail here, never fault on the
GPU), then launches on the current torch stream.  Launches are asynchronous and
graph-capturable; no wrapper synchronises.

The `Prepared*` classes hold the ctypes argument blocks of a fixed launch so that the hot
loop (engine.py) pays one ctypes call per kernel and nothing else.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .tuning import knob
from ._lib import (DgAdamSeg, DgEpiGroup, DgFusedTarget, DgGemmDesc, DgL2gGroup, DgProj, DgRelGroup,
                   DgStagedGroup, DgStagedProj, check)


def _stream_ptr(stream: Optional[torch.cuda.Stream] = None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream


def _dev(t: torch.Tensor, dtype: torch.dtype, what: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what}: expected a torch.Tensor, got {type(t).__name__}")
    if not t.is_cuda:
        raise ValueError(f"{what}: must be a device (HIP) tensor")
    if t.dtype != dtype:
        raise TypeError(f"{what}: dtype {t.dtype}, expected {dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{what}: must be contiguous")
    return t


# --------------------------------------------------------------------------------------
# SpMM over relation groups
# --------------------------------------------------------------------------------------
@dataclass
class RelGroupSpec:
    """One relation group in the chunk-merged layout of dg_rel_group (decagon_hip.h)."""

    rowptr: torch.Tensor          # int32 [n_chunks*n_rows + 1]
    vcol: torch.Tensor            # int32 [nnz] virtual columns (rows of x)
    val: torch.Tensor             # float32 [nnz]
    x: torch.Tensor               # float32, relation-stacked dense operand, row v at v*x_ld
    out: Optional[torch.Tensor]   # float32 [n_chunks, n_rows, d] (None in fused mode)
    n_rows: int
    n_chunks: int
    x_ld: int
    x_rows: int                   # rows of x the kernel may address (per chunk when shared)
    vcol_max: int = -1            # host-known max(vcol) (-1: no nonzeros)
    shared: bool = False          # DG_GROUP_SHARED_PATTERN: one CSR [n_rows] for every chunk, chunk c
                                  # reading x rows [c*x_rows, (c+1)*x_rows) (dg_spmm_groups_f32 only)
    drop: Optional[Tuple[torch.Tensor, int, float]] = None  # DG_GROUP_DROPOUT (shared only):
                                  # (device state {seed, step}, stream tag, keep) — chunk c scales
                                  # nonzero p by mask element c·nnz + (drop_index[p] or p)
    drop_index: Optional[torch.Tensor] = None
    dense: bool = False           # DG_GROUP_DENSE_ROWS (dg_gcn_fused_f32 only): row r of the sum
                                  # is x[r] — or, with n_chunks = S slots, Σ_c x[c·x_rows·x_ld + r]
                                  # in slot order; rowptr / vcol / val unused (may be None)

    def validate(self, d: int, need_out: bool = True) -> None:
        if self.dense:
            _dev(self.x, torch.float32, "x")
            if not 1 <= self.n_chunks <= _lib.DG_PEER_MAX or self.shared or self.drop is not None:
                raise ValueError("a dense-rows group has 1..8 slots, no shared pattern, no dropout")
            if self.x_ld < d or self.x_ld % 4:
                raise ValueError("x_ld must be >= d and a multiple of 4")
            last = (self.n_chunks - 1) * self.x_rows * self.x_ld + (self.n_rows - 1) * self.x_ld + d
            if self.x_rows < self.n_rows or (self.n_rows and self.x.numel() < last):
                raise ValueError("x smaller than the group's rows (slots)")
            return
        _dev(self.rowptr, torch.int32, "rowptr")
        _dev(self.vcol, torch.int32, "vcol")
        _dev(self.val, torch.float32, "val")
        _dev(self.x, torch.float32, "x")
        if need_out or self.out is not None:
            _dev(self.out, torch.float32, "out")
        if self.n_rows == 0:
            return
        if self.n_chunks < 1:
            raise ValueError("n_chunks must be >= 1")
        n_ptr = (self.n_rows if self.shared else self.n_chunks * self.n_rows) + 1
        if self.rowptr.numel() < n_ptr:
            raise ValueError(f"rowptr has {self.rowptr.numel()} entries, kernel reads {n_ptr}")
        if self.vcol.numel() != self.val.numel():
            raise ValueError("vcol/val length mismatch")
        if self.x_ld < d or self.x_ld % 4:
            raise ValueError("x_ld must be >= d and a multiple of 4")
        if self.vcol_max >= self.x_rows:
            raise ValueError(f"vcol reaches row {self.vcol_max} of a {self.x_rows}-row operand")
        slabs = self.n_chunks if self.shared else 1
        if self.x_rows > 0 and self.x.numel() < (slabs * self.x_rows - 1) * self.x_ld + d:
            raise ValueError(f"x has {self.x.numel()} elements, kernel may read {(slabs * self.x_rows - 1) * self.x_ld + d}")
        if self.x_rows * self.x_ld >= 2**31:
            raise ValueError("dense operand too large for 32-bit gather offsets")
        if need_out and self.out.numel() < self.n_chunks * self.n_rows * d:
            raise ValueError("out too small for [n_chunks, n_rows, d]")
        if self.drop is not None:
            state, _, keep = self.drop
            if not self.shared:
                raise ValueError("dropout masks apply to a shared pattern only")
            if not (isinstance(state, torch.Tensor) and state.is_cuda and state.dtype == torch.int64
                    and state.numel() >= 2):
                raise ValueError("dropout state: int64 device tensor {seed, step}")
            if not 0.0 < float(keep) <= 1.0:
                raise ValueError("keep must be in (0, 1]")
            if self.n_chunks * self.vcol.numel() >= 2**32:
                raise ValueError("dropout mask counter exceeds 32 bits")
            if self.drop_index is not None:
                _dev(self.drop_index, torch.int32, "drop_index")
                if self.drop_index.numel() != self.vcol.numel():
                    raise ValueError("drop_index must have one entry per nonzero")


def _fill_group(g, s: RelGroupSpec) -> None:
    if s.dense:
        g.rowptr = g.vcol = g.val = g.out = None
        g.x = s.x.data_ptr()
        g.x_ld, g.n_rows, g.n_chunks, g.x_rows = s.x_ld, s.n_rows, s.n_chunks, s.x_rows
        g.flags = _lib.DG_GROUP_DENSE_ROWS
        g.drop_state = g.drop_index = None
        return
    g.rowptr = s.rowptr.data_ptr()
    g.vcol = s.vcol.data_ptr() if s.vcol.numel() else None
    g.val = s.val.data_ptr() if s.val.numel() else None
    g.x = s.x.data_ptr()
    g.out = s.out.data_ptr() if s.out is not None else None
    g.x_ld = s.x_ld
    g.n_rows = s.n_rows
    g.n_chunks = s.n_chunks
    g.x_rows = s.x_rows
    g.flags = _lib.DG_GROUP_SHARED_PATTERN if s.shared else 0
    g.drop_state = None
    g.drop_index = None
    if s.drop is not None:
        state, tag, keep = s.drop
        g.flags |= _lib.DG_GROUP_DROPOUT
        g.drop_state = state.data_ptr()
        g.drop_tag = int(tag)
        g.drop_keep = float(keep)
        g.drop_stride = int(s.vcol.numel())
        g.drop_index = s.drop_index.data_ptr() if s.drop_index is not None else None


FUSED_RPB = 1  # spmm.hip kFusedRpb: rows per fused workgroup, at most
SPMM_LDS_MAX_ROWS = 160 * 1024 // 144  # dg_spmm_groups_lds_f32: operand rows staged in LDS


class PreparedSpmm:
    """A fixed dg_spmm_groups_f32 launch (descriptor block built once); lds=True: the
    dg_spmm_groups_lds_f32 form for small shared operands (x_rows <= SPMM_LDS_MAX_ROWS)."""

    def __init__(self, specs: Sequence[RelGroupSpec], d: int, lds: bool = False):
        if len(specs) > _lib.DG_MAX_GROUPS:
            raise ValueError(f"at most {_lib.DG_MAX_GROUPS} groups per launch")
        for s in specs:
            s.validate(d)
        self.specs = list(specs)  # keep tensors alive
        self.d = d
        arr = (DgRelGroup * max(1, len(specs)))()
        for i, s in enumerate(specs):
            g = arr[i]
            _fill_group(g, s)
        self._arr = arr
        self._n = len(specs)
        if lds and any(s.x_rows > SPMM_LDS_MAX_ROWS for s in specs):
            raise ValueError("dg_spmm_groups_lds_f32: operand too large for LDS")
        self._name = "dg_spmm_groups_lds_f32" if lds else "dg_spmm_groups_f32"
        self._fn = getattr(_lib.load(), self._name)

    def __call__(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        check(self._fn(self._arr, self._n, self.d, _stream_ptr(stream)), self._name)


@dataclass
class SegSpec:
    """One group of dg_spmm_seg_f32 (decagon_hip.h): the chunk-merged CSR, its segment starts
    (sparse.chunk_segments) and, for the reassociated layer 2, the weight stack w with each
    local relation's slab."""

    rowptr: torch.Tensor          # int32 [n_chunks*n_rows + 1]
    seg: torch.Tensor             # int32 [n_chunks*n_rows*chunk]
    vcol: torch.Tensor            # int32 [nnz]
    val: torch.Tensor             # float32 [nnz]
    x: torch.Tensor               # float32: stacked X (no w) or H [n_cols, x_ld]
    out: Optional[torch.Tensor]   # float32 [n_chunks, n_rows, d_out] (None in the fused form)
    n_rows: int
    n_cols: int
    n_chunks: int
    chunk: int
    n_rels: int
    x_ld: int
    x_rows: int                   # bound on vcol
    vcol_max: int = -1
    w: Optional[torch.Tensor] = None      # float32 [K, 64, 32]
    slab: Optional[torch.Tensor] = None   # int32 [n_rels] (None: relation k is slab k)
    slab_max: int = -1

    def validate(self, d_in: int, d_out: int, need_out: bool = True) -> None:
        for t, what in ((self.rowptr, "rowptr"), (self.seg, "seg"), (self.vcol, "vcol")):
            _dev(t, torch.int32, what)
        _dev(self.val, torch.float32, "val")
        _dev(self.x, torch.float32, "x")
        if need_out:
            _dev(self.out, torch.float32, "out")
        if not 1 <= self.chunk <= 16:
            raise ValueError("chunk must be in [1, 16]")
        if not (self.n_chunks - 1) * self.chunk < self.n_rels <= self.n_chunks * self.chunk:
            raise ValueError("every chunk must hold at least one relation")
        if self.rowptr.numel() < self.n_chunks * self.n_rows + 1:
            raise ValueError("rowptr too short")
        if self.seg.numel() < self.n_chunks * self.n_rows * self.chunk:
            raise ValueError("seg too short")
        if self.vcol.numel() != self.val.numel():
            raise ValueError("vcol/val length mismatch")
        if self.vcol_max >= self.x_rows:
            raise ValueError(f"vcol reaches row {self.vcol_max} of a {self.x_rows}-row operand")
        if self.x_ld < d_in or self.x_ld % 4:
            raise ValueError("x_ld must be >= d_in and a multiple of 4")
        if self.x_rows * self.x_ld >= 2**31:
            raise ValueError("dense operand too large for 32-bit gather offsets")
        if need_out and self.out.numel() < self.n_chunks * self.n_rows * d_out:
            raise ValueError("out too small for [n_chunks, n_rows, d_out]")
        if self.w is None:
            if self.n_rows and self.x_rows and self.x.numel() < (self.x_rows - 1) * self.x_ld + d_in:
                raise ValueError("x smaller than x_rows rows")
            return
        _dev(self.w, torch.float32, "w")
        K = self.w.shape[0]
        if tuple(self.w.shape[1:]) != (64, 32) or (d_in, d_out) != (64, 32):
            raise ValueError("the reassociated form takes a [K, 64, 32] stack (d_in 64, d_out 32)")
        if self.x_rows > K * self.n_cols:
            raise ValueError("vcol bound beyond the stack's slabs")
        if self.x.numel() < (self.n_cols - 1) * self.x_ld + 64:
            raise ValueError("H smaller than n_cols rows")
        if self.slab is not None:
            _dev(self.slab, torch.int32, "slab")
            if self.slab.numel() < self.n_rels or not 0 <= self.slab_max < K:
                raise ValueError("slab map must index inside w")
        elif self.n_rels > K:
            raise ValueError("n_rels > K")


def _seg_array(specs: Sequence[SegSpec], d_in: int, d_out: int, need_out: bool):
    if len(specs) > _lib.DG_MAX_GROUPS:
        raise ValueError(f"at most {_lib.DG_MAX_GROUPS} groups per launch")
    if len({s.w is None for s in specs}) > 1:
        raise ValueError("every group of a launch has a weight stack, or none")
    arr = (_lib.DgSegGroup * max(1, len(specs)))()
    for i, s in enumerate(specs):
        s.validate(d_in, d_out, need_out)
        g = arr[i]
        g.rowptr, g.seg = s.rowptr.data_ptr(), s.seg.data_ptr()
        g.vcol = s.vcol.data_ptr() if s.vcol.numel() else None
        g.val = s.val.data_ptr() if s.val.numel() else None
        g.slab = s.slab.data_ptr() if s.slab is not None else None
        g.x = s.x.data_ptr()
        g.out = s.out.data_ptr() if s.out is not None else None
        g.w = s.w.data_ptr() if s.w is not None else None
        g.x_ld, g.n_rows, g.n_cols, g.n_chunks = s.x_ld, s.n_rows, s.n_cols, s.n_chunks
        g.chunk, g.n_rels, g.x_rows = s.chunk, s.n_rels, s.x_rows
    return arr


class PreparedSeg:
    """A fixed dg_spmm_seg_f32 launch (every group with w, or none)."""

    def __init__(self, specs: Sequence[SegSpec], d_in: int, d_out: int):
        arr = _seg_array(specs, d_in, d_out, True)
        self.specs = list(specs)
        self._arr, self._n, self.d_in, self.d_out = arr, len(specs), d_in, d_out
        self._fn = _lib.load().dg_spmm_seg_f32

    def __call__(self, stream=None) -> None:
        check(self._fn(self._arr, self._n, self.d_in, self.d_out, _stream_ptr(stream)), "dg_spmm_seg_f32")


class PreparedFusedSeg:
    """A fixed dg_gcn_fused_seg_f32 launch: targets = [(out tensor, n_rows, [SegSpec], relu)],
    each output row finished by one workgroup, one wave per relation (at most 16 a row; groups
    chunk-merged, any chunks); with weight stacks (d_in 64 → d_out 32) the reassociated layer 2."""

    def __init__(self, targets, d_in: int, d_out: int, peer=None):
        """peer = (PeerExchange, slot): every target's `out` lies in the exchange region; the
        launch also pushes the rows to every peer and ends with the exchange
        (dg_gcn_fused_seg_peer_f32)."""
        specs, tarr = [], (DgFusedTarget * len(targets))()
        for t, (out, n_rows, gspecs, relu) in enumerate(targets):
            _dev(out, torch.float32, "out")
            if out.numel() < n_rows * d_out:
                raise ValueError("fused output too small")
            if sum(s.n_rels for s in gspecs) > 16:
                raise ValueError("at most 16 relations per target row")
            tarr[t].out, tarr[t].n_rows = out.data_ptr(), n_rows
            tarr[t].g_begin, tarr[t].g_count = len(specs), len(gspecs)
            tarr[t].flags = _lib.DG_EPI_RELU if relu else 0
            for s in gspecs:
                if s.n_rows != n_rows or s.n_rels < 1:
                    raise ValueError("fused seg groups: the target's rows, at least one relation")
                specs.append(s)
        if len(targets) > _lib.DG_MAX_GROUPS:
            raise ValueError(f"at most {_lib.DG_MAX_GROUPS} targets per launch")
        self._garr = _seg_array(specs, d_in, d_out, False)
        self._keep = (specs, [t[0] for t in targets])
        self._tarr, self._ng, self._nt, self.d_in, self.d_out = tarr, len(specs), len(targets), d_in, d_out
        self._xchg = None
        if peer is not None:
            ex, slot = peer
            for out, *_ in targets:
                ex.offset(out)  # raises unless inside the region
            self._xchg = ctypes.byref(ex.xchg(slot))
            self._keep = self._keep + (ex,)
            self._fn = _lib.load().dg_gcn_fused_seg_peer_f32
        else:
            self._fn = _lib.load().dg_gcn_fused_seg_f32

    def __call__(self, stream=None) -> None:
        if self._xchg is not None:
            check(self._fn(self._garr, self._ng, self._tarr, self._nt, self.d_in, self.d_out, self._xchg,
                           _stream_ptr(stream)), "dg_gcn_fused_seg_peer_f32")
            return
        check(self._fn(self._garr, self._ng, self._tarr, self._nt, self.d_in, self.d_out, _stream_ptr(stream)),
              "dg_gcn_fused_seg_f32")


class _WaveTable:
    """Host builder of a dg_wave_table (decagon_hip.h): per wave slot a 64-byte descriptor and
    the first S pairs of its segment (in the hand-out order of its gather form: pair m in lane
    16·(m & 3) + (m >> 2), stored compactly at (m & 3)·S/4 + (m >> 2)), the rest in batches of
    64 in an overflow array.  S (slot_pairs, round 6) is the smallest of 16 / 32 / 48 / 64
    holding the first batch of ≥ SLOT_COVER of the non-empty waves: a wave then fetches S·8 B
    where round 5 fetched 512 B whatever its length (a config-S wave holds 7–81 pairs)."""

    SLOT_COVER = 0.97

    DESC = np.dtype([("x", "<u8"), ("w", "<u8"), ("orow", "<u8"), ("cnt", "<i4"), ("x_ld", "<i4"), ("ovf", "<i4"),
                     ("role", "<u4"), ("wr", "<u4"), ("pad", "<i4", 5)])

    def __init__(self, specs: Sequence[SegSpec], n_slots: int, proj: bool):
        assert self.DESC.itemsize == 64
        self.specs, self.proj = list(specs), proj
        self.host = [(s.rowptr.cpu().numpy(), s.seg.cpu().numpy(), s.vcol.cpu().numpy(), s.val.cpu().numpy(),
                      None if s.slab is None else s.slab.cpu().numpy()) for s in specs]
        self.n_slots = n_slots
        self.pv: dict = {}  # wave slot -> its pairs [cnt, 2] (laid out at upload, once S is known)
        self.desc = np.zeros(n_slots, self.DESC)
        # entry of pair m within a batch: its lane in the DPP hand-out (both layers since round 6)
        m = np.arange(64)
        self.lane_of = 16 * (m & 3) + (m >> 2)

    def bounds(self, g: int, k: int, r: int) -> Tuple[int, int]:
        """[beg, end) of relation k's segment (of spec g) in row r."""
        s = self.specs[g]
        rowptr, seg = self.host[g][:2]
        c, t = divmod(k, s.chunk)
        si = (c * s.n_rows + r) * s.chunk + t
        beg = int(seg[si])
        end = int(seg[si + 1]) if t + 1 < s.chunk else int(rowptr[c * s.n_rows + r + 1])
        return beg, end

    def seg_len(self, g: int, k: int, r: int) -> int:
        beg, end = self.bounds(g, k, r)
        return end - beg

    def relation(self, i: int, g: int, k: int, r: int) -> None:
        """Wave slot i gathers relation k (of spec g) of row r."""
        beg, end = self.bounds(g, k, r)
        self.wave(i, g, r, [(k, 0, end - beg)])

    def wave(self, i: int, g: int, r: int, pieces) -> None:
        """Wave slot i gathers the pieces [(k, a, b)] of row r, in order: pairs a..b of relation
        k's segment (of spec g) — with a weight stack (layer 2 reassociated) one relation's only,
        since the wave multiplies its aggregate by that relation's W slab."""
        s = self.specs[g]
        vcol, val, slab = self.host[g][2:]
        d = self.desc
        vcs, vvs = [], []
        for k, a, b in pieces:
            beg, _ = self.bounds(g, k, r)
            vc = vcol[beg + a:beg + b].astype(np.int64)
            if self.proj:
                sl = int(slab[k]) if slab is not None else k
                vc = vc - sl * s.n_cols  # plain rows of H
                d["w"][i] = s.w.data_ptr() + sl * 64 * 32 * 4
            vcs.append(vc)
            vvs.append(val[beg + a:beg + b])
        if self.proj and len({k for k, _, _ in pieces}) > 1:
            raise ValueError("a reassociated wave gathers one relation")
        vc = np.concatenate(vcs) if vcs else np.zeros(0, np.int64)
        vv = np.concatenate(vvs) if vvs else np.zeros(0, np.float32)
        cnt = len(vc)
        d["x"][i], d["x_ld"][i], d["cnt"][i] = s.x.data_ptr(), s.x_ld, cnt
        self.pv[i] = np.stack([vc.astype(np.int32), vv.astype(np.float32).view(np.int32)], 1)

    def slot_pairs(self) -> int:
        fixed = knob("DG_TAB_SLOT", 0)  # (A/B: a fixed slot size; 0 = by SLOT_COVER)
        if fixed:
            if fixed not in (16, 32, 48, 64):
                raise ValueError("DG_TAB_SLOT: 16, 32, 48 or 64")
            return fixed
        cnts = np.array([len(p) for p in self.pv.values() if len(p)], np.int64)
        if not len(cnts):
            return 16
        need = float(np.quantile(cnts, self.SLOT_COVER))
        return next(S for S in (16, 32, 48, 64) if S >= need or S == 64)

    def layout(self, S: int):
        """(pairs [n_slots·S, 2], ovf [.., 2]) for first-batch slots of S pairs; sets desc.ovf."""
        pairs = np.zeros((self.n_slots * S, 2), np.int32)
        ovf: List[np.ndarray] = []
        n_ovf = 0
        m = np.arange(S)
        compact = (m & 3) * (S // 4) + (m >> 2)  # slot entry of pair m (its lane's row-major rank)
        for i, pv in self.pv.items():
            cnt = len(pv)
            m0 = min(cnt, S)
            pairs[i * S + compact[:m0]] = pv[:m0]
            if cnt > S:
                self.desc["ovf"][i] = n_ovf
                for q0 in range(S, cnt, 64):
                    blk = np.zeros((64, 2), np.int32)
                    n = min(64, cnt - q0)
                    blk[self.lane_of[:n]] = pv[q0:q0 + n]
                    ovf.append(blk)
                    n_ovf += 64
        return pairs, (np.concatenate(ovf) if ovf else np.zeros((64, 2), np.int32))

    def upload(self, owner, n_blocks: int, nw: int, stride: int, dev) -> "_lib.DgWaveTable":
        S = self.slot_pairs()
        pairs, ovf = self.layout(S)
        owner._pairs = torch.from_numpy(pairs).to(dev)
        owner._ovf = torch.from_numpy(ovf).to(dev)
        owner.slot_pairs = S
        raw = torch.from_numpy(self.desc.view(np.uint8).copy())
        owner._desc = torch.empty(raw.numel() + 64, dtype=torch.uint8, device=dev)
        off = (-owner._desc.data_ptr()) % 64  # 64-byte aligned descriptors
        owner._desc_v = owner._desc[off:off + raw.numel()]
        owner._desc_v.copy_(raw.to(dev))
        tab = _lib.DgWaveTable()
        tab.pairs, tab.ovf, tab.desc = owner._pairs.data_ptr(), owner._ovf.data_ptr(), owner._desc_v.data_ptr()
        tab.n_blocks, tab.nw, tab.nw_stride, tab.slot_pairs = n_blocks, nw, stride, S
        return tab


def _tab_shape(d_in: int, d_out: int, specs) -> bool:
    return d_in == 64 and (d_out == 64 or (d_out == 32 and all(s.w is not None for s in specs)))


class PreparedFusedTab(PreparedFusedSeg):
    """The same launch as PreparedFusedSeg (same targets, rows, waves and arithmetic: bitwise the
    same rows) through dg_gcn_fused_tab_f32: the wave table — each wave's 64-byte descriptor and
    its segment's first 64 pairs at a fixed slot — is built here once, on the host, from the
    chunk-merged CSR and segment starts of the specs (decagon_hip.h documents the layout).
    Shapes: d_in = d_out = 64, or 64 -> 32 with weight stacks.  peer = (PeerExchange, slot):
    the rows also go to every peer and the launch ends with the exchange
    (dg_gcn_fused_tab_peer_f32; PreparedFusedSeg's peer form, bitwise the same rows).

    balance (round 6): spread each row's pairs over every wave slot its workgroup gives the row
    instead of one wave per relation.  A relation segment of config S runs 7 to 81 pairs, and a
    workgroup waits for its slowest wave.  Layer 1 deals each group's pairs (its relations back
    to back: every pair gathers one row of the stacked operand) in contiguous slices over the
    group's waves, waves given to groups by their pairs; the reassociated layer 2 keeps one
    relation per wave (its W slab) and gives the spare slots to the longest segments.  The kernel
    and its finishing roles are unchanged — a group's normalising wave sums its waves' rows in
    order — so only the fp32 summation order within a group differs from the per-relation form."""

    def __init__(self, targets, d_in: int, d_out: int, peer=None, balance: bool = False):
        super().__init__(targets, d_in, d_out, peer=peer)
        specs = self._keep[0]
        if not _tab_shape(d_in, d_out, specs):
            raise ValueError("dg_gcn_fused_tab_f32: d_in = d_out = 64, or 64 -> 32 with weight stacks")
        proj = d_out != d_in
        if any(len(gs) > 64 // (d_out // 4) for _, _, gs, _ in targets):
            raise ValueError("dg_gcn_fused_tab_f32: at most 64 / (d_out / 4) groups a target (one lane set each)")
        waves_t = [sum(s.n_rels for s in gs) for _, _, gs, _ in targets]
        nw = max([1] + waves_t)
        stride = 8 if nw <= 8 else 16
        if balance:
            nw = stride  # every wave slot of a workgroup takes a share of its rows' pairs
        self.balance = balance
        plan = []  # (target, first row, rows per workgroup) per workgroup, in launch order
        for t, (_, n_rows, _, _) in enumerate(targets):
            rpb = min(nw // waves_t[t], 4)
            plan += [(t, r0, rpb) for r0 in range(0, n_rows, rpb)]
        tb = _WaveTable(specs, len(plan) * stride, proj)
        g_first = np.cumsum([0] + [len(gs) for _, _, gs, _ in targets])
        for b, (t, r0, rpb) in enumerate(plan):
            out, n_rows, gspecs, relu = targets[t]
            gc = len(gspecs)
            nr = [s.n_rels for s in gspecs]
            per_row = nw // rpb if balance else waves_t[t]  # wave slots of one row
            counts = [[1] * gc for _ in range(rpb)]  # waves per group, per row slot
            for slot in range(rpb):
                r = r0 + slot
                if r >= n_rows:
                    continue
                gs = [int(g_first[t]) + gl for gl in range(gc)]
                if balance:
                    waves = _balanced_waves(tb, gs, nr, r, per_row, proj)
                else:  # one wave per relation, groups in order
                    waves = [[[(k, 0, None)] for k in range(nr[gl])] for gl in range(gc)]
                counts[slot] = [len(wg) for wg in waves]
                w = slot * per_row
                for gl, wg in enumerate(waves):
                    for pieces in wg:
                        tb.wave(b * stride + w, gs[gl], r,
                                [(k, a, e if e is not None else tb.seg_len(gs[gl], k, r)) for k, a, e in pieces])
                        w += 1
            for w in range(nw):
                i = b * stride + w
                if w < rpb * gc:
                    s2, gg = divmod(w, gc)
                    gb = s2 * per_row + sum(counts[s2][:gg])
                    tb.desc["role"][i] = ((1 << 31) | ((s2 * DG_MAX_GROUPS_TAB + gg) << 16) | (counts[s2][gg] << 8)
                                          | gb)
                if w < rpb and r0 + w < n_rows:
                    tb.desc["orow"][i] = out.data_ptr() + (r0 + w) * d_out * 4
                    tb.desc["wr"][i] = gc | ((1 if relu else 0) << 8) | (w << 16)
                    tb.desc["pad"][i, 0] = (r0 + w) * d_out * 4  # (the peer form: row offset,
                    tb.desc["pad"][i, 1] = n_rows * d_out * 4     # target bytes)
                    # the row's finishing wave (round 6): each group's wave count − 1 in 4 bits,
                    # and the row slot's first wave
                    tb.desc["pad"][i, 2] = np.int32(np.uint32(sum((c - 1) << (4 * u)
                                                                  for u, c in enumerate(counts[w]))))
                    tb.desc["pad"][i, 3] = w * per_row
        if not plan and peer is not None:
            raise ValueError("dg_gcn_fused_tab_peer_f32: the exchange needs at least one row a rank")
        self._tab = tb.upload(self, len(plan), nw, stride, specs[0].x.device)
        self.n_blocks, self.nw = len(plan), nw
        if self._xchg is not None:
            self._tfn, self._tname = _lib.load().dg_gcn_fused_tab_peer_f32, "dg_gcn_fused_tab_peer_f32"
        else:
            self._tfn, self._tname = _lib.load().dg_gcn_fused_tab_f32, "dg_gcn_fused_tab_f32"

    def __call__(self, stream=None) -> None:
        if self._xchg is not None:
            check(self._tfn(ctypes.byref(self._tab), self.d_in, self.d_out, self._xchg, _stream_ptr(stream)),
                  self._tname)
        else:
            check(self._tfn(ctypes.byref(self._tab), self.d_in, self.d_out, _stream_ptr(stream)), self._tname)

    def seg_form(self, stream=None) -> None:
        """The same rows through dg_gcn_fused_seg_f32 (tests: bitwise equal unless balanced)."""
        PreparedFusedSeg.__call__(self, stream)


def _split_even(n: int, parts: int) -> List[Tuple[int, int]]:
    """[a, b) slices of n items over `parts` waves, the first n % parts one longer."""
    q, rem = divmod(n, parts)
    out, a = [], 0
    for p in range(parts):
        e = a + q + (1 if p < rem else 0)
        out.append((a, e))
        a = e
    return out


def _balanced_waves(tb: "_WaveTable", gs, nr, r: int, slots: int, proj: bool):
    """Row r's waves for PreparedFusedTab(balance=True): per group, a list of waves, each a list
    of pieces (relation k, first pair, end pair) of the relation's segment.  `slots` wave slots
    in all, at least one per group (per relation with weight stacks); the spare slots go, one at
    a time, to the job whose share per wave is the largest (ties: the first)."""
    if proj:  # jobs are relations: a reassociated wave multiplies by one relation's W slab
        jobs = [(gl, k) for gl in range(len(gs)) for k in range(nr[gl])]
        sizes = [tb.seg_len(gs[gl], k, r) for gl, k in jobs]
    else:  # jobs are groups: every pair of a group gathers one row of the stacked operand
        jobs = [(gl, None) for gl in range(len(gs))]
        sizes = [sum(tb.seg_len(gs[gl], k, r) for k in range(nr[gl])) for gl in range(len(gs))]
    if len(jobs) > slots:
        raise ValueError(f"{len(jobs)} jobs for {slots} wave slots")
    parts = [1] * len(jobs)
    for _ in range(slots - len(jobs)):
        j = max(range(len(jobs)), key=lambda x: (-(-sizes[x] // parts[x]), -x))
        if sizes[j] <= parts[j]:
            break  # no job left with more than one pair per wave
        parts[j] += 1
    waves = [[] for _ in gs]
    for (gl, k), n, p in zip(jobs, sizes, parts):
        if k is not None:
            waves[gl] += [[(k, a, e)] for a, e in _split_even(n, p)]
            continue
        # a group: its relations' segments back to back, cut into p contiguous slices
        lens = [tb.seg_len(gs[gl], kk, r) for kk in range(nr[gl])]
        starts = np.cumsum([0] + lens)
        for a, e in _split_even(n, p):
            pieces = []
            for kk in range(nr[gl]):
                lo, hi = max(a, starts[kk]), min(e, starts[kk + 1])
                if lo < hi:
                    pieces.append((kk, int(lo - starts[kk]), int(hi - starts[kk])))
            waves[gl].append(pieces)
    return waves


class PreparedSegTab(PreparedSeg):
    """The same launch as PreparedSeg (dg_spmm_seg_f32's workgroups in its XCD-contiguous item
    order, waves and chunk partials — bit for bit) through dg_spmm_seg_tab_f32, from a wave
    table built here once.  Shapes as PreparedFusedTab."""

    def __init__(self, specs: Sequence[SegSpec], d_in: int, d_out: int):
        super().__init__(specs, d_in, d_out)
        if not _tab_shape(d_in, d_out, specs):
            raise ValueError("dg_spmm_seg_tab_f32: d_in = d_out = 64, or 64 -> 32 with weight stacks")
        live = [g for g, s in enumerate(specs) if s.n_rows > 0 and s.n_rels > 0]
        nw = max([1] + [specs[g].chunk for g in live])
        stride = 8 if nw <= 8 else 16
        blocks = []  # (spec, chunk c, first row, rows per workgroup) or None (a dead workgroup)
        for g in live:
            s = specs[g]
            rpb = nw // s.chunk
            row_blocks = -(-s.n_rows // rpb)
            items = s.n_chunks * row_blocks
            n_blocks = 8 * (-(-items // 8))
            per = n_blocks >> 3
            for lb in range(n_blocks):
                item = (lb & 7) * per + (lb >> 3)
                blocks.append(None if item >= items else (g, item // row_blocks, (item % row_blocks) * rpb, rpb))
        tb = _WaveTable(specs, len(blocks) * stride, d_out != d_in)
        for b, blk in enumerate(blocks):
            if blk is None:
                continue
            g, c, r0, rpb = blk
            s = specs[g]
            for w in range(nw):
                i = b * stride + w
                slot, t = divmod(w, s.chunk)
                r = r0 + slot
                if not (slot < rpb and r < s.n_rows):
                    continue
                k = c * s.chunk + t
                if k < s.n_rels:
                    tb.relation(i, g, k, r)
                if t == 0:
                    tb.desc["orow"][i] = s.out.data_ptr() + (c * s.n_rows + r) * d_out * 4
                    tb.desc["role"][i] = s.chunk << 8
        self._tab = tb.upload(self, len(blocks), nw, stride, specs[0].x.device)
        self.n_blocks, self.nw = len(blocks), nw
        self._tfn = _lib.load().dg_spmm_seg_tab_f32

    def __call__(self, stream=None) -> None:
        check(self._tfn(ctypes.byref(self._tab), self.d_in, self.d_out, _stream_ptr(stream)), "dg_spmm_seg_tab_f32")

    def seg_form(self, stream=None) -> None:
        """The same partials through dg_spmm_seg_f32 (tests: bitwise equal)."""
        PreparedSeg.__call__(self, stream)


DG_MAX_GROUPS_TAB = 8  # nbuf groups per row slot in gcn_tab_kernel (DG_MAX_GROUPS)


@dataclass
class ProjSpec:
    """Projection epilogue of a fused launch: out[kk] = row · w[rel_map[kk] or kk]."""

    w: torch.Tensor                     # float32 [K, d, d_out]
    out: torch.Tensor                   # float32 [n_rels, n_rows, d_out]
    n_rels: int
    target: int                         # index into the fused launch's targets
    rel_map: Optional[torch.Tensor] = None
    rel_map_max: Optional[int] = None


class PreparedFused:
    """A fixed dg_gcn_fused_f32 launch.

    targets = [(out tensor, n_rows, [group specs], relu)], projs = [ProjSpec]."""

    def __init__(self, targets, d: int, projs: Sequence[ProjSpec] = (), waves_per_group: int = 1):
        specs, tarr = [], (DgFusedTarget * len(targets))()
        max_groups = 1
        for t, (out, n_rows, gspecs, relu) in enumerate(targets):
            _dev(out, torch.float32, "out")
            if out.numel() < n_rows * d:
                raise ValueError("fused output too small")
            tarr[t].out = out.data_ptr()
            tarr[t].n_rows = n_rows
            tarr[t].g_begin = len(specs)
            tarr[t].g_count = len(gspecs)
            tarr[t].flags = _lib.DG_EPI_RELU if relu else 0
            max_groups = max(max_groups, len(gspecs))
            for s in gspecs:
                if s.n_rows != n_rows:
                    raise ValueError("group rows != target rows")
                s.validate(d, need_out=False)
                specs.append(s)
        if len(specs) > _lib.DG_MAX_GROUPS or len(targets) > _lib.DG_MAX_GROUPS:
            raise ValueError(f"at most {_lib.DG_MAX_GROUPS} groups / targets per fused launch")
        if not 1 <= waves_per_group or max_groups * waves_per_group > 16:
            raise ValueError("groups x waves_per_group must be <= 16")
        if len(projs) > _lib.DG_MAX_GROUPS:
            raise ValueError(f"at most {_lib.DG_MAX_GROUPS} projections per fused launch")
        parr = (DgProj * max(1, len(projs)))()
        for i, pj in enumerate(projs):
            _dev(pj.w, torch.float32, "proj w")
            _dev(pj.out, torch.float32, "proj out")
            K, din, dout = pj.w.shape
            n_rows = targets[pj.target][1]
            if din != d or pj.out.numel() < pj.n_rels * n_rows * dout:
                raise ValueError("projection shapes do not match the fused layer")
            if pj.rel_map is not None:
                _dev(pj.rel_map, torch.int32, "proj rel_map")
                if pj.rel_map_max is None or not 0 <= pj.rel_map_max < K:
                    raise ValueError("proj rel_map_max must index inside w")
            elif pj.n_rels > K:
                raise ValueError("projection n_rels > K")
            parr[i].w = pj.w.data_ptr()
            parr[i].rel_map = pj.rel_map.data_ptr() if pj.rel_map is not None else None
            parr[i].out = pj.out.data_ptr()
            parr[i].n_rels = pj.n_rels
            parr[i].target = pj.target
            parr[i].d_out = dout
        garr = (DgRelGroup * len(specs))()
        for i, s in enumerate(specs):
            _fill_group(garr[i], s)
        self._keep = (specs, [t[0] for t in targets], list(projs))
        self._garr, self._tarr, self._parr = garr, tarr, parr
        self._ng, self._nt, self._np, self.d = len(specs), len(targets), len(projs), d
        self.wpg = waves_per_group
        self._max_groups = max_groups
        self._fn = _lib.load().dg_gcn_fused_f32

    def block_threads(self) -> int:
        """Waves per workgroup of this launch (dg_gcn_fused_f32's rows-per-workgroup rule)."""
        rpb = max(1, min(FUSED_RPB, 16 // (self._max_groups * self.wpg)))
        return rpb * self._max_groups * self.wpg

    def __call__(self, stream=None) -> None:
        check(self._fn(self._garr, self._ng, self._tarr, self._nt, self._parr if self._np else None, self._np,
                       self.wpg, self.d, _stream_ptr(stream)), "dg_gcn_fused_f32")


def staged_block(lrowptr: np.ndarray, lcol: np.ndarray, lval: np.ndarray, rlw: np.ndarray,
                 n_cols: int) -> np.ndarray:
    """One relation's pair block of the staged layout with the library's bank-conflict-avoiding
    diagonals and hole columns (dg_staged_block, host-only).  Lanes as a CSR over 64·waves
    virtual rows; returns pairs [sum(rlw)·64, 2] int32."""
    lrowptr = np.ascontiguousarray(lrowptr, np.int32)
    lcol = np.ascontiguousarray(lcol, np.int32)
    lval = np.ascontiguousarray(lval, np.float32)
    rlw = np.ascontiguousarray(rlw, np.int32)
    pairs = np.zeros((int(rlw.sum()) * 64, 2), np.int32)
    check(_lib.load().dg_staged_block(lrowptr.ctypes.data, lcol.ctypes.data, lval.ctypes.data, len(lrowptr) - 1,
                                      rlw.ctypes.data, n_cols, pairs.ctypes.data), "dg_staged_block")
    return pairs


@dataclass
class StagedDevice:
    """A StagedLayout (sparse.py) uploaded to the device."""

    pairs: torch.Tensor
    jm: torch.Tensor
    jmoff: torch.Tensor
    n_rows: int
    n_cols: int
    n_rels: int
    jm_len: int                   # ints in jm (tables + spare)
    jm_end: int                   # jmoff[n_rels]

    @classmethod
    def upload(cls, layout, device) -> "StagedDevice":
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        return cls(t(layout.pairs), t(layout.jm), t(layout.jmoff), layout.n_rows, layout.n_cols,
                   len(layout.jmoff) - 1, layout.jm_len, int(layout.jmoff[-1]))


STAGED_LDS_BYTES = 160 * 1024
STAGED_MAX_CHUNKS = _lib.DG_STAGED_MAX_CHUNKS
STAGED_JM_SPARE = 1024


def staged_lds_bytes(n_rows: int, n_cols: int) -> int:
    """LDS of one staged workgroup (mirrors dg_spmm_staged_f32): two slab buffers of n_cols + 16
    columns 80 B apart (the slab rows, then sixteen zero columns), 1 KiB of chunk tables,
    n_rows 64-byte accumulators (80-byte rows when LDS has room)."""
    return 2 * (n_cols + 16) * 80 + 1024 + n_rows * 64


@dataclass
class StagedSpec:
    """One group for dg_spmm_staged_f32."""

    layout: StagedDevice
    slab: Optional[torch.Tensor]  # int32 [n_rels] or None
    x: torch.Tensor
    out: torch.Tensor             # float32 [ceil(n_rels/out_chunk), n_rows, d]
    out_chunk: int
    x_ld: int
    x_rows: int
    slab_max: int = -1            # host-known max(slab) (or n_rels-1 without slab), for checks
    # (H [n_cols][64], W [K][64][d]): relation k's operand is H·W[slab(k)], made in the kernel
    # (dg_spmm_staged_proj_f32); x / x_ld / x_rows are then unused
    proj: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    # variable output chunks: host int32 [n_chunks + 1], chunk c = relations [cs[c], cs[c+1])
    # (out is then [n_chunks, n_rows, d]); None: runs of out_chunk relations
    chunk_start: Optional[np.ndarray] = None

    def n_out(self) -> int:
        if self.chunk_start is not None:
            return len(self.chunk_start) - 1
        return -(-self.layout.n_rels // self.out_chunk)

    def validate(self, d: int) -> None:
        L = self.layout
        for t, nm, dt in ((L.pairs, "pairs", torch.int32), (L.jm, "jm", torch.int32),
                          (L.jmoff, "jmoff", torch.int32), (self.out, "out", torch.float32)):
            _dev(t, dt, nm)
        if self.proj is None:
            _dev(self.x, torch.float32, "x")
        if L.pairs.data_ptr() % 16:
            raise ValueError("pairs must be 16-byte aligned")
        if not (0 < L.n_rows < 1023 and 0 < L.n_cols <= 1024):
            raise ValueError("staged groups need n_rows < 1023, n_cols <= 1024")
        if L.jm_len < L.jm_end + STAGED_JM_SPARE or L.jm.numel() < L.jm_len:
            raise ValueError("staged jm must end with 1024 spare ints")
        if staged_lds_bytes(L.n_rows, L.n_cols) > STAGED_LDS_BYTES:
            raise ValueError("staged group does not fit LDS (two slab buffers + accumulators)")
        if not 1 <= self.out_chunk <= 64:
            raise ValueError("staged out_chunk must be 1..64")
        if self.slab is not None:
            _dev(self.slab, torch.int32, "slab")
            if self.slab.numel() < L.n_rels:
                raise ValueError("slab shorter than n_rels")
        smax = self.slab_max if self.slab_max >= 0 else L.n_rels - 1
        if self.proj is not None:
            h, w = self.proj
            if not (isinstance(h, torch.Tensor) and h.is_cuda and h.dtype == torch.float32):
                raise ValueError("proj h: float32 device tensor required (rows may be padded)")
            _dev(w, torch.float32, "proj w")
            if h.dim() != 2 or h.shape[0] < L.n_cols or h.shape[1] != 64 or h.stride(1) != 1 or h.stride(0) % 4:
                raise ValueError("proj h must be [n_cols][64], rows 16-byte aligned")
            if w.dim() != 3 or tuple(w.shape[1:]) != (64, d) or not w.is_contiguous() or w.shape[0] <= smax:
                raise ValueError("proj w must be a contiguous [K][64][d] stack covering the slabs")
        else:
            if (smax + 1) * L.n_cols > self.x_rows or self.x.numel() < (self.x_rows - 1) * self.x_ld + d:
                raise ValueError("dense operand smaller than the slabs address")
            if self.x_rows * self.x_ld >= 2**31:
                raise ValueError("dense operand too large for 32-bit gather offsets")
        if self.chunk_start is not None:
            cs = np.asarray(self.chunk_start)
            if (cs.ndim != 1 or not 2 <= len(cs) <= STAGED_MAX_CHUNKS + 1 or cs[0] != 0 or cs[-1] != L.n_rels
                    or L.n_rels > 65535 or np.diff(cs).min() < 1 or np.diff(cs).max() > 64):
                raise ValueError("staged chunk_start: 0 = c_0 < ... < c_n = n_rels, 1..64 relations a chunk, "
                                 f"at most {STAGED_MAX_CHUNKS} chunks")
        n_out = self.n_out()
        if self.out.numel() < n_out * L.n_rows * d:
            raise ValueError("staged out too small")


class PreparedStaged:
    """A fixed dg_spmm_staged_f32 launch."""

    def __init__(self, specs: Sequence[StagedSpec], d: int):
        if not 1 <= len(specs) <= _lib.DG_MAX_GROUPS:
            raise ValueError(f"1..{_lib.DG_MAX_GROUPS} groups per launch")
        arr = (DgStagedGroup * len(specs))()
        proj = specs[0].proj is not None
        if any((s.proj is not None) != proj for s in specs):
            raise ValueError("a staged launch's groups are all projected or none")
        parr = (DgStagedProj * len(specs))() if proj else None
        cstarts = []
        for i, s in enumerate(specs):
            s.validate(d)
            L, g = s.layout, arr[i]
            g.pairs, g.jm, g.jmoff = L.pairs.data_ptr(), L.jm.data_ptr(), L.jmoff.data_ptr()
            g.slab = s.slab.data_ptr() if s.slab is not None else None
            g.x = s.x.data_ptr() if s.x is not None else None
            if proj:
                h, w = s.proj
                parr[i].h, parr[i].w, parr[i].h_ld, parr[i].din = h.data_ptr(), w.data_ptr(), h.stride(0), 64
            g.out = s.out.data_ptr()
            g.x_ld = s.x_ld
            g.n_rows, g.n_cols, g.n_rels = L.n_rows, L.n_cols, L.n_rels
            g.out_chunk, g.x_rows, g.jm_len = s.out_chunk, s.x_rows, L.jm_len
            if s.chunk_start is not None:
                cs = np.ascontiguousarray(s.chunk_start, np.int32)
                cstarts.append(cs)  # (read at each launch: kept alive with the launch)
                g.chunk_start, g.n_chunks = cs.ctypes.data, len(cs) - 1
        self._keep = list(specs) + cstarts
        self._arr, self._parr, self._n, self.d = arr, parr, len(specs), d
        lib = _lib.load()
        self._fn = lib.dg_spmm_staged_proj_f32 if proj else lib.dg_spmm_staged_f32

    def __call__(self, stream=None) -> None:
        if self._parr is not None:
            check(self._fn(self._arr, self._parr, self._n, self.d, _stream_ptr(stream)), "dg_spmm_staged_proj_f32")
        else:
            check(self._fn(self._arr, self._n, self.d, _stream_ptr(stream)), "dg_spmm_staged_f32")


def spmm_groups(specs: Sequence[RelGroupSpec], d: int, stream=None) -> None:
    PreparedSpmm(specs, d)(stream)


def spmm_csr(rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor, x: torch.Tensor,
             n_rows: int, out: Optional[torch.Tensor] = None, stream=None, beta: float = 0.0) -> torch.Tensor:
    """Y = A·X + beta·Y for one CSR relation (tf.sparse_tensor_dense_matmul, layers.py:90, :114),
    through dg_spmm_csr_f32.  beta = 1 adds the relation's product into a running sum (tf.add_n
    of layers.py:92 one relation at a time); beta = 0 overwrites out without reading it."""
    if x.dim() != 2:
        raise ValueError("x must be 2-D")
    if not np.isfinite(beta):
        raise ValueError("beta must be finite")
    x = x.contiguous()
    n_cols, d = x.shape
    if out is None:
        if beta != 0.0:
            raise ValueError("beta != 0 needs out (the running sum)")
        out = torch.empty((n_rows, d), device=x.device, dtype=torch.float32)
    vmax = int(col.max()) if col.numel() else -1
    spec = RelGroupSpec(rowptr, col, val, x, out, n_rows, 1, d, n_cols, vcol_max=vmax)
    spec.validate(d)
    if out.dim() != 2 or out.shape[0] < n_rows or out.shape[1] != d:
        raise ValueError("out must be [n_rows, d]")
    check(_lib.load().dg_spmm_csr_f32(rowptr.data_ptr(), col.data_ptr(), val.data_ptr(), n_rows, n_cols,
                                      x.data_ptr(), d, out.data_ptr(), d, d, ctypes.c_float(beta),
                                      _stream_ptr(stream)), "dg_spmm_csr_f32")
    return out


def rownorm_l2(x: torch.Tensor, out: Optional[torch.Tensor] = None, relu: bool = False,
               stream=None) -> torch.Tensor:
    """tf.nn.l2_normalize(x, dim=1) (layers.py:93, :117), then relu if asked (model.py:75), through
    dg_rownorm_l2_f32.  out may be x (in place)."""
    _dev(x, torch.float32, "x")
    if x.dim() != 2:
        raise ValueError("x must be 2-D")
    n_rows, d = x.shape
    if out is None:
        out = torch.empty_like(x)
    _dev(out, torch.float32, "out")
    if out.shape != x.shape:
        raise ValueError("out must have x's shape")
    flags = _lib.DG_EPI_RELU if relu else 0
    check(_lib.load().dg_rownorm_l2_f32(x.data_ptr(), out.data_ptr(), n_rows, d, flags, _stream_ptr(stream)),
          "dg_rownorm_l2_f32")
    return out


# --------------------------------------------------------------------------------------
# Epilogue
# --------------------------------------------------------------------------------------
class PreparedEpilogue:
    def __init__(self, partials: Sequence[Tuple[torch.Tensor, int]], out: torch.Tensor, n_rows: int,
                 d: int, flags: int):
        if not partials:
            raise ValueError("at least one group")
        if len(partials) > _lib.DG_MAX_GROUPS:
            raise ValueError(f"at most {_lib.DG_MAX_GROUPS} groups")
        _dev(out, torch.float32, "out")
        if out.numel() < n_rows * d:
            raise ValueError("out too small")
        arr = (DgEpiGroup * len(partials))()
        for i, (p, nc, *rest) in enumerate(partials):
            _dev(p, torch.float32, "partial")
            if p.numel() < nc * n_rows * d:
                raise ValueError("partial too small for [n_chunks, n_rows, d]")
            arr[i].partial = p.data_ptr()
            arr[i].n_chunks = nc
        self._keep = [p for p, *_ in partials] + [out]
        self._arr = arr
        self._args = (len(partials), out.data_ptr(), n_rows, d, flags)
        self._fn = _lib.load().dg_gcn_epilogue_f32

    def __call__(self, stream=None) -> None:
        n, o, r, d, f = self._args
        check(self._fn(self._arr, n, o, r, d, f, _stream_ptr(stream)), "dg_gcn_epilogue_f32")


class PreparedEpilogueMulti:
    """dg_gcn_epilogue_multi_f32: several node types' epilogues in one launch —
    targets = [(partials [(tensor, n_chunks[, sum_out[, push]])], out, n_rows)], one flag set;
    a group's optional sum_out [n_rows, d] receives its pre-normalisation sum S_ij (with a peer
    exchange and push: also every peer's copy of it — this rank's slot of the all-reduce)."""

    def __init__(self, targets: Sequence[Tuple[Sequence[Tuple[torch.Tensor, int]], torch.Tensor, int]], d: int,
                 flags: int, peer=None, push: Optional[Sequence[bool]] = None):
        """peer = (PeerExchange, slot): the targets flagged in `push` (their `out` inside the
        exchange region) also go to every peer, and the launch ends with the exchange
        (dg_gcn_epilogue_peer_f32)."""
        if not targets or len(targets) > 8:
            raise ValueError("1..8 targets per launch")
        if sum(len(p) for p, _, _ in targets) > _lib.DG_MAX_GROUPS:
            raise ValueError(f"at most {_lib.DG_MAX_GROUPS} groups over all targets")
        self._keep, self._garrs = [], []
        tarr = (_lib.DgEpiTarget * len(targets))()
        for t, (partials, out, n_rows) in enumerate(targets):
            if not partials:
                raise ValueError("at least one group per target")
            _dev(out, torch.float32, "out")
            if out.numel() < n_rows * d:
                raise ValueError("out too small")
            garr = (DgEpiGroup * len(partials))()
            for i, (p, nc, *so) in enumerate(partials):
                _dev(p, torch.float32, "partial")
                if p.numel() < nc * n_rows * d:
                    raise ValueError("partial too small for [n_chunks, n_rows, d]")
                garr[i].partial = p.data_ptr()
                garr[i].n_chunks = nc
                if so and so[0] is not None:  # the group's pre-normalisation sum S_ij
                    _dev(so[0], torch.float32, "sum_out")
                    if so[0].numel() < n_rows * d:
                        raise ValueError("sum_out too small for [n_rows, d]")
                    garr[i].sum_out = so[0].data_ptr()
                    self._keep.append(so[0])
                    if len(so) > 1 and so[1]:
                        if peer is None:
                            raise ValueError("a pushed sum needs a peer exchange")
                        peer[0].offset(so[0])  # raises unless inside the region
                        garr[i].group_flags = _lib.DG_EPI_PUSH
                self._keep.append(p)
            self._keep.append(out)
            self._garrs.append(garr)
            tarr[t].groups = ctypes.cast(garr, ctypes.POINTER(DgEpiGroup))
            tarr[t].n_groups = len(partials)
            tarr[t].out = out.data_ptr()
            tarr[t].n_rows = n_rows
            if peer is not None and (push is None or push[t]):
                peer[0].offset(out)  # raises unless inside the region
                tarr[t].target_flags = _lib.DG_EPI_PUSH
        self._tarr = tarr
        self._args = (len(targets), d, flags)
        self._xchg = None
        if peer is not None:
            self._xchg = ctypes.byref(peer[0].xchg(peer[1]))
            self._keep.append(peer[0])
            self._fn = _lib.load().dg_gcn_epilogue_peer_f32
        else:
            self._fn = _lib.load().dg_gcn_epilogue_multi_f32

    def __call__(self, stream=None) -> None:
        n, d, f = self._args
        if self._xchg is not None:
            check(self._fn(self._tarr, n, d, f, self._xchg, _stream_ptr(stream)), "dg_gcn_epilogue_peer_f32")
            return
        check(self._fn(self._tarr, n, d, f, _stream_ptr(stream)), "dg_gcn_epilogue_multi_f32")


class PreparedEpilogueTab(PreparedEpilogueMulti):
    """The same launch as PreparedEpilogueMulti (bitwise its rows) through
    dg_gcn_epilogue_tab_f32: one 64-byte descriptor per output row built here once (its
    target's output, each group's chunk-0 partial row and chunk count), so a wave issues all its
    partial loads at once.  Targets whose groups carry sum outputs, or more than four groups,
    are not supported (ValueError: use PreparedEpilogueMulti)."""

    DESC = np.dtype([("out", "<u8"), ("part", "<u8", 4), ("off", "<i4"), ("plane", "<i4"), ("n_chunks", "<u4"),
                     ("info", "<u4"), ("bytes", "<i4"), ("pad", "<i4")])

    def __init__(self, targets, d: int, flags: int, peer=None, push: Optional[Sequence[bool]] = None):
        if d not in (32, 64):
            raise ValueError("dg_gcn_epilogue_tab_f32: d = 32 or 64")
        for partials, _, _ in targets:
            if len(partials) > 4 or any(len(p) > 2 and p[2] is not None for p in partials) \
                    or any(p[1] > 255 for p in partials):
                raise ValueError("dg_gcn_epilogue_tab_f32: at most 4 groups a row, 255 chunks, no group sums")
        super().__init__(targets, d, flags, peer, push)
        assert self.DESC.itemsize == 64
        n = sum(nr for _, _, nr in targets)
        desc = np.zeros(n, self.DESC)
        i = 0
        for t, (partials, out, nr) in enumerate(targets):
            if nr == 0:
                continue
            rows = np.arange(nr, dtype=np.int64)
            sl = slice(i, i + nr)
            desc["out"][sl] = out.data_ptr()
            desc["off"][sl] = rows * d
            desc["plane"][sl] = nr * d
            desc["bytes"][sl] = nr * d * 4
            ncs = 0
            for g, (p, nc, *_) in enumerate(partials):
                desc["part"][sl, g] = p.data_ptr() + rows * d * 4
                ncs |= nc << (8 * g)
            desc["n_chunks"][sl] = ncs
            pushed = peer is not None and (push is None or push[t])
            desc["info"][sl] = len(partials) | ((1 if pushed else 0) << 8)
            i += nr
        dev = targets[0][1].device
        raw = torch.from_numpy(desc.view(np.uint8).copy())
        self._rows = torch.empty(raw.numel() + 64, dtype=torch.uint8, device=dev)
        off = (-self._rows.data_ptr()) % 64
        self._rows_v = self._rows[off:off + raw.numel()]
        self._rows_v.copy_(raw.to(dev))
        self._n_rows = n
        self._tfn = _lib.load().dg_gcn_epilogue_tab_f32

    def __call__(self, stream=None) -> None:
        _, d, f = self._args
        check(self._tfn(self._rows_v.data_ptr() if self._n_rows else None, self._n_rows, d, f, self._xchg,
                        _stream_ptr(stream)), "dg_gcn_epilogue_tab_f32")

    def multi_form(self, stream=None) -> None:
        """The same rows through dg_gcn_epilogue_multi_f32 / _peer_f32 (tests: bitwise equal)."""
        PreparedEpilogueMulti.__call__(self, stream)


def gcn_epilogue(partials, out, n_rows, d, flags, stream=None) -> None:
    PreparedEpilogue(partials, out, n_rows, d, flags)(stream)


# --------------------------------------------------------------------------------------
# GEMM
# --------------------------------------------------------------------------------------
class PreparedGemm:
    """C_b = diag(sc)·((A_b·diag(sa))·B_b) on the fp32 MFMA, batched and strided.

    a, b, c are given as (tensor, (bs, s0, s1)) with element strides; sizes m, n, k, batch.
    """

    def __init__(self, a: torch.Tensor, a_strides, b: torch.Tensor, b_strides, c: torch.Tensor,
                 c_strides, m: int, n: int, k: int, batch: int = 1,
                 sa: Optional[torch.Tensor] = None, sc: Optional[torch.Tensor] = None,
                 b_map: Optional[torch.Tensor] = None, b_batches: Optional[int] = None,
                 b_map_max: Optional[int] = None, reduce: int = 0,
                 drop: Optional[Tuple[torch.Tensor, int, float]] = None):
        for t, nm in ((a, "a"), (b, "b"), (c, "c")):
            if not (t.is_cuda and t.dtype == torch.float32):
                raise ValueError(f"{nm}: float32 device tensor required")

        def span(strides, d0, d1, nb=batch):
            bs, s0, s1 = strides
            return (nb - 1) * bs + (d0 - 1) * s0 + (d1 - 1) * s1 + 1

        nb_b = batch
        if b_map is not None:
            _dev(b_map, torch.int32, "b_map")
            nb_b = batch if b_batches is None else b_batches
            if b_map.numel() < batch or b_map_max is None or not (0 <= b_map_max < nb_b):
                raise ValueError("b_map must cover the batch and index inside b")
        if m and n and k and batch:
            if a.numel() < span(a_strides, m, k) or b.numel() < span(b_strides, k, n, nb_b):
                raise ValueError("gemm operand too small for its strides")
        if reduce < 0:
            raise ValueError("reduce must be >= 0")
        n_out = -(-batch // reduce) if reduce else nb_b
        if m and n and batch and c.numel() < span(c_strides, m, n, n_out):
            raise ValueError("gemm output too small for its strides")
        if sa is not None and (sa.numel() < k or sa.dtype != torch.float32 or not sa.is_cuda):
            raise ValueError("sa must be a float32 device vector of length k")
        if sc is not None and (sc.numel() < n or sc.dtype != torch.float32 or not sc.is_cuda):
            raise ValueError("sc must be a float32 device vector of length n")
        desc = DgGemmDesc()
        desc.a, desc.b, desc.c = a.data_ptr(), b.data_ptr(), c.data_ptr()
        desc.sa = sa.data_ptr() if sa is not None else None
        desc.sc = sc.data_ptr() if sc is not None else None
        desc.b_map = b_map.data_ptr() if b_map is not None else None
        desc.a_bs, desc.a_sm, desc.a_sk = a_strides
        desc.b_bs, desc.b_sk, desc.b_sn = b_strides
        desc.c_bs, desc.c_sm, desc.c_sn = c_strides
        desc.m, desc.n, desc.k, desc.batch = m, n, k, batch
        desc.reduce = reduce
        if drop is not None:  # (device state {seed, step}, stream tag, keep): masked batch-reduce
            state, tag, keep_p = drop
            if not reduce:
                raise ValueError("the dropout mask applies in batch-reduce mode")
            if state.dtype != torch.int64 or not state.is_cuda:
                raise ValueError("dropout state: int64 device tensor {seed, step}")
            if nb_b * m * n >= 2**32:
                raise ValueError("dropout mask indices are 32-bit: (mapped) batches·m·n < 2^32")
            desc.drop_state, desc.drop_tag, desc.drop_keep = state.data_ptr(), int(tag), float(keep_p)
        self._desc = desc
        self._keep = (a, b, c, sa, sc, b_map, drop)
        self._fn = _lib.load().dg_gemm_f32

    def __call__(self, stream=None) -> None:
        check(self._fn(ctypes.byref(self._desc), 1, _stream_ptr(stream)), "dg_gemm_f32")


class PreparedGemmMulti:
    """Several prepared GEMMs (≤ DG_MAX_GROUPS) in one dg_gemm_f32 launch."""

    def __init__(self, gemms: Sequence[PreparedGemm]):
        if not 1 <= len(gemms) <= _lib.DG_MAX_GROUPS:
            raise ValueError(f"1..{_lib.DG_MAX_GROUPS} GEMMs per launch")
        arr = (DgGemmDesc * len(gemms))()
        for i, g in enumerate(gemms):
            ctypes.memmove(ctypes.byref(arr[i]), ctypes.byref(g._desc), ctypes.sizeof(DgGemmDesc))
        self._keep = list(gemms)
        self._arr, self._n = arr, len(gemms)
        self._fn = _lib.load().dg_gemm_f32

    def __call__(self, stream=None) -> None:
        check(self._fn(self._arr, self._n, _stream_ptr(stream)), "dg_gemm_f32")


class PreparedGemmTN:
    """dg_gemm_tn_f32: c[b] = a[b]ᵀ·b_stack[b] for a [rows][M] shared (or [batch][rows][M]) and
    b_stack [batch][rows][N] (contiguous), c [batch][M][N]; rows split into ranges of about
    `rows_per_split` (0: enough to fill the chip)."""

    def __init__(self, a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, rows_per_split: int = 0):
        _dev(a, torch.float32, "a")
        _dev(b, torch.float32, "b")
        _dev(c, torch.float32, "c")
        batch, rb, N = b.shape
        if a.dim() == 3:
            if a.shape[0] != batch:
                raise ValueError("gemm_tn: batched a must have one matrix per batch")
            rows, M = a.shape[1], a.shape[2]
            a_bs = rows * M
        else:
            rows, M = a.shape
            a_bs = 0
        if rb != rows or tuple(c.shape) != (batch, M, N):
            raise ValueError("gemm_tn: shapes")
        if rows_per_split <= 0:  # enough workgroups to fill the chip, ranges of >= 64 rows
            self.n_split = max(1, min(-(-1024 // max(1, batch)), -(-rows // 64)))
        else:
            self.n_split = max(1, -(-rows // max(2, rows_per_split)))
        self.partial = (torch.empty((self.n_split, batch, M, N), device=a.device) if self.n_split > 1 else None)
        self._keep = (a, b, c)
        self._args = (a.data_ptr(), M, a_bs, b.data_ptr(), N, rows * N, c.data_ptr(), rows, M, N, batch, self.n_split,
                      self.partial.data_ptr() if self.partial is not None else None)
        self._fn = _lib.load().dg_gemm_tn_f32

    def __call__(self, stream=None) -> None:
        check(self._fn(*self._args, _stream_ptr(stream)), "dg_gemm_tn_f32")


def matmul(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
           sa: Optional[torch.Tensor] = None, sc: Optional[torch.Tensor] = None, stream=None):
    """out = diag-scaled a @ b for 2-D fp32 device tensors (any strides)."""
    m, k = a.shape
    k2, n = b.shape
    if k != k2:
        raise ValueError("inner dimensions differ")
    if out is None:
        out = torch.empty((m, n), device=a.device, dtype=torch.float32)
    PreparedGemm(a, (0, a.stride(0), a.stride(1)), b, (0, b.stride(0), b.stride(1)), out,
                 (0, out.stride(0), out.stride(1)), m, n, k, 1, sa, sc)(stream)
    return out


# --------------------------------------------------------------------------------------
# Decoder, losses, sampler
# --------------------------------------------------------------------------------------
def decoder_score(row_table: torch.Tensor, col_table: torch.Tensor, row_idx: torch.Tensor,
                  col_idx: torch.Tensor, G: torch.Tensor, l: Optional[torch.Tensor],
                  out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """out[p] = row_table[row_idx[p]]ᵀ · L · G · L · col_table[col_idx[p]]."""
    _dev(row_table, torch.float32, "row_table")
    _dev(col_table, torch.float32, "col_table")
    _dev(row_idx, torch.int32, "row_idx")
    _dev(col_idx, torch.int32, "col_idx")
    _dev(G, torch.float32, "G")
    d = G.shape[0]
    if G.shape != (d, d) or row_table.shape[1] != d or col_table.shape[1] != d:
        raise ValueError("decoder: d mismatch")
    n = row_idx.numel()
    if col_idx.numel() != n:
        raise ValueError("row_idx / col_idx length mismatch")
    if l is not None:
        _dev(l, torch.float32, "l")
        if l.numel() != d:
            raise ValueError("l must have d entries")
    if out is None:
        out = torch.empty(n, device=G.device, dtype=torch.float32)
    fn = _lib.load().dg_decoder_score_f32
    check(fn(row_table.data_ptr(), row_table.shape[1], col_table.data_ptr(), col_table.shape[1],
             row_idx.data_ptr(), col_idx.data_ptr(), n, G.data_ptr(),
             l.data_ptr() if l is not None else None, d, out.data_ptr(), _stream_ptr(stream)),
          "dg_decoder_score_f32")
    return out


def decoder_score_bf16(row_table: torch.Tensor, col_table: torch.Tensor, rows: torch.Tensor,
                       cols: torch.Tensor, G: torch.Tensor, l_table: Optional[torch.Tensor] = None,
                       rel: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                       stream=None, paired: bool = False) -> torch.Tensor:
    """bf16 DEDICOM scores of pairs (rows[p], cols[p]) of relations rel[p] (dg_decoder_score_bf16):
    uᵀ·D_k·G·D_k·v with bf16 tables / G / diagonals and fp32 accumulation (config 5).
    paired: the caller promises pair p and pair p + n/2 share the column and the relation (a
    positive and its negative); dg_decoder_score_bf16_paired contracts the shared side once,
    T = G·bf16(D_k∘v), and dots it with both rows (half the MFMA work; the bf16 operand rounding
    sits on D_k∘v instead of u∘D_k), reading cols and rel of the first half only."""
    n = rows.numel()
    if paired and (n % 2 or cols.numel() != n or (rel is not None and rel.numel() != n)):
        raise ValueError("paired scoring needs an even number of pairs, cols / rel of the same length")
    d = G.shape[0]
    for t, nm in ((row_table, "row_table"), (col_table, "col_table"), (G, "G")):
        _dev(t, torch.bfloat16, nm)
    if l_table is not None:
        _dev(l_table, torch.bfloat16, "l_table")
        if l_table.shape[-1] != d or l_table.stride(-1) != 1 or (l_table.dim() == 2 and l_table.stride(0) != d):
            raise ValueError("l_table must be a contiguous [n_rel, d] bf16 tensor")
    for t, nm in ((rows, "rows"), (cols, "cols")):
        _dev(t, torch.int32, nm)
    if rel is not None:
        _dev(rel, torch.int32, "rel")
    if G.shape != (d, d) or not G.is_contiguous():
        raise ValueError("G must be a contiguous d×d bf16 matrix")
    if row_table.shape[1] != d or col_table.shape[1] != d or row_table.stride(1) != 1 or col_table.stride(1) != 1:
        raise ValueError("tables must have d contiguous columns")
    if out is None:
        out = torch.empty(n, device=rows.device, dtype=torch.float32)
    if paired:
        name = "dg_decoder_score_bf16_paired"
        tabs = (row_table.data_ptr(), row_table.stride(0), row_table.shape[0], col_table.data_ptr(),
                col_table.stride(0), col_table.shape[0])
    else:
        name = "dg_decoder_score_bf16"
        tabs = (row_table.data_ptr(), row_table.stride(0), col_table.data_ptr(), col_table.stride(0))
    check(getattr(_lib.load(), name)(
        *tabs, rows.data_ptr(), cols.data_ptr(), rel.data_ptr() if rel is not None else None,
        n // 2 if paired else n, G.data_ptr(), l_table.data_ptr() if l_table is not None else None, d,
        out.data_ptr(), _stream_ptr(stream)), name)
    return out


def hinge_loss(pos: torch.Tensor, neg: torch.Tensor, margin: float,
               out: Optional[torch.Tensor] = None, stream=None,
               workspace: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Σ relu(neg − pos + margin) (optimizer.py:116-120): one workgroup, or — with a
    workspace of DG_HINGE_WS_BYTES (first word zero; hinge_workspace()) — up to 256."""
    _dev(pos, torch.float32, "pos")
    _dev(neg, torch.float32, "neg")
    if pos.numel() != neg.numel():
        raise ValueError("pos/neg length mismatch")
    if out is None:
        out = torch.empty(1, device=pos.device, dtype=torch.float32)
    if workspace is not None:
        if workspace.numel() * workspace.element_size() < _lib.DG_HINGE_WS_BYTES or not workspace.is_cuda:
            raise ValueError("hinge workspace too small")
        check(_lib.load().dg_hinge_loss_ws_f32(pos.data_ptr(), neg.data_ptr(), pos.numel(), float(margin),
                                                out.data_ptr(), workspace.data_ptr(), _stream_ptr(stream)),
              "dg_hinge_loss_ws_f32")
        return out
    check(_lib.load().dg_hinge_loss_f32(pos.data_ptr(), neg.data_ptr(), pos.numel(), float(margin),
                                         out.data_ptr(), _stream_ptr(stream)), "dg_hinge_loss_f32")
    return out


def hinge_workspace(device) -> torch.Tensor:
    return torch.zeros(_lib.DG_HINGE_WS_BYTES // 4, dtype=torch.int32, device=device)


def xent_loss(pos: torch.Tensor, neg: torch.Tensor, neg_weight: float,
              out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    _dev(pos, torch.float32, "pos")
    _dev(neg, torch.float32, "neg")
    if pos.numel() != neg.numel():
        raise ValueError("pos/neg length mismatch")
    if out is None:
        out = torch.empty(1, device=pos.device, dtype=torch.float32)
    check(_lib.load().dg_xent_loss_f32(pos.data_ptr(), neg.data_ptr(), pos.numel(), float(neg_weight),
                                        out.data_ptr(), _stream_ptr(stream)), "dg_xent_loss_f32")
    return out


def unigram_sample(table: torch.Tensor, n: int, seed: int, offset: int,
                   out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """n draws from an alias table (sampling.alias_table, uploaded as int32 [range, 2])."""
    _dev(table, torch.int32, "alias table")
    if table.dim() != 2 or table.shape[1] != 2:
        raise ValueError("alias table must be [range, 2]")
    if out is None:
        out = torch.empty(n, device=table.device, dtype=torch.int32)
    _dev(out, torch.int32, "out")
    if out.numel() < n:
        raise ValueError("out too small")
    check(_lib.load().dg_unigram_sample(table.data_ptr(), table.shape[0], n, seed & (2**64 - 1),
                                         offset & (2**64 - 1), out.data_ptr(), _stream_ptr(stream)),
          "dg_unigram_sample")
    return out


def unigram_sample_slots(table: torch.Tensor, slot0: int, batch: int, n: int, seed: int,
                         out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """n draws, draw i from the alias table of relation slot slot0 + i // batch (table: int32
    [n_slots, range, 2], one per GLOBAL slot; or a shared [range, 2]) — counter slot0·batch + i,
    so the draws do not depend on how slots are dealt to ranks (dg_unigram_sample_slots)."""
    _dev(table, torch.int32, "alias table")
    if table.dim() == 3 and table.shape[2] == 2 and table.is_contiguous():
        rng, stride = table.shape[1], table.shape[1]
        if slot0 + -(-n // batch) > table.shape[0]:
            raise ValueError("slot range outside the alias tables")
    elif table.dim() == 2 and table.shape[1] == 2:
        rng, stride = table.shape[0], 0
    else:
        raise ValueError("alias tables must be [n_slots, range, 2] (contiguous) or [range, 2]")
    if out is None:
        out = torch.empty(n, device=table.device, dtype=torch.int32)
    _dev(out, torch.int32, "out")
    if out.numel() < n:
        raise ValueError("out too small")
    check(_lib.load().dg_unigram_sample_slots(table.data_ptr(), rng, stride, slot0, batch, n, seed & (2**64 - 1),
                                               out.data_ptr(), _stream_ptr(stream)), "dg_unigram_sample_slots")
    return out


def slot_score_hinge_bf16(E_row: torch.Tensor, E_col: torch.Tensor, pos_rows: torch.Tensor, pos_cols: torch.Tensor,
                          table: torch.Tensor, slot0: int, n_slots: int, batch: int, seed: int, G: torch.Tensor,
                          D: torch.Tensor, margin: float, out: torch.Tensor, neg_rows: torch.Tensor,
                          loss: torch.Tensor, workspace: torch.Tensor, stream=None) -> None:
    """Config 5's step in one launch (dg_slot_score_hinge_bf16): local slots [0, n_slots) are
    relations slot0 .. slot0 + n_slots − 1; pos_rows / pos_cols hold their n = n_slots·batch
    positives (slot-major).  neg_rows ← each slot's alias draws (unigram_sample_slots' draws),
    out[:n] / out[n:] ← positive / negative scores (decoder_score_bf16(paired=True)), loss ←
    the hinge sum."""
    n = n_slots * batch
    for t, nm in ((E_row, "E_row"), (E_col, "E_col"), (G, "G"), (D, "D")):
        _dev(t, torch.bfloat16, nm)
    for t, nm in ((pos_rows, "pos_rows"), (pos_cols, "pos_cols"), (neg_rows, "neg_rows"), (table, "alias table")):
        _dev(t, torch.int32, nm)
    _dev(out, torch.float32, "out")
    _dev(loss, torch.float32, "loss")
    d = G.shape[0]
    if d != 256 or G.shape != (256, 256) or D.dim() != 2 or D.shape[1] != d or E_row.shape[1] != d \
            or E_col.shape[1] != d:
        raise ValueError("slot scorer: d = 256 tables, G and D rows")
    if table.dim() == 3 and table.shape[2] == 2:
        rng, stride = table.shape[1], table.shape[1]
        if slot0 + n_slots > table.shape[0]:
            raise ValueError("slot range outside the alias tables")
    elif table.dim() == 2 and table.shape[1] == 2:
        rng, stride = table.shape[0], 0
    else:
        raise ValueError("alias tables must be [n_slots, range, 2] or [range, 2]")
    if rng > E_row.shape[0] or slot0 + n_slots > D.shape[0]:
        raise ValueError("sampler range exceeds the row table, or slots exceed D")
    if pos_rows.numel() < n or pos_cols.numel() < n or neg_rows.numel() < n or out.numel() < 2 * n:
        raise ValueError("pairs / outputs shorter than n_slots·batch")
    if workspace.numel() * workspace.element_size() < _lib.DG_HINGE_WS_BYTES or not workspace.is_cuda:
        raise ValueError("hinge workspace too small")
    check(_lib.load().dg_slot_score_hinge_bf16(
        E_row.data_ptr(), E_row.stride(0), E_row.shape[0], E_col.data_ptr(), E_col.stride(0), E_col.shape[0],
        pos_rows.data_ptr(), pos_cols.data_ptr(),
        table.data_ptr(), rng, stride, slot0, n_slots, batch, seed & (2**64 - 1), G.data_ptr(), D.data_ptr(), d,
        float(margin), out.data_ptr(), neg_rows.data_ptr(), loss.data_ptr(), workspace.data_ptr(),
        _stream_ptr(stream)), "dg_slot_score_hinge_bf16")


def upload_alias(degrees, device) -> torch.Tensor:
    """The alias table of one degree vector, int32 [range, 2]; a list of degree vectors (one per
    relation) gives [n, range, 2] (every vector the same length)."""
    from .sampling import alias_table

    if isinstance(degrees, (list, tuple)) or (isinstance(degrees, np.ndarray) and degrees.ndim == 2):
        tabs = np.stack([alias_table(d) for d in degrees])
        return torch.from_numpy(tabs.view(np.int32)).to(device)
    return torch.from_numpy(alias_table(degrees).view(np.int32)).to(device)


class PreparedDecoderHinge:
    """dg_decoder_hinge_f32 on fixed buffers: sampled (or given) negatives, positive and
    negative scores of n pairs and the hinge loss, in one launch."""

    def __init__(self, row_table: torch.Tensor, col_table: torch.Tensor, rows: torch.Tensor,
                 cols: torch.Tensor, G: torch.Tensor, l: Optional[torch.Tensor], margin: float,
                 alias: Optional[torch.Tensor] = None, neg_rows: Optional[torch.Tensor] = None,
                 seed: int = 0, offset: int = 0):
        for t, nm, dt in ((row_table, "row_table", torch.float32), (col_table, "col_table", torch.float32),
                          (rows, "rows", torch.int32), (cols, "cols", torch.int32), (G, "G", torch.float32)):
            _dev(t, dt, nm)
        d = G.shape[0]
        n = rows.numel()
        if n < 1:
            raise ValueError("empty batch")
        if G.shape != (d, d) or row_table.shape[1] != d or col_table.shape[1] != d or cols.numel() != n:
            raise ValueError("decoder_hinge: shape mismatch")
        if l is not None:
            _dev(l, torch.float32, "l")
        if neg_rows is None:
            if alias is None:
                raise ValueError("need either negatives or a sampler alias table")
            _dev(alias, torch.int32, "alias")
            if alias.shape[0] > row_table.shape[0]:
                raise ValueError("sampler range exceeds the row table")
        else:
            _dev(neg_rows, torch.int32, "neg_rows")
        dev = G.device
        self.pos = torch.empty(n, device=dev)
        self.neg = torch.empty(n, device=dev)
        self.neg_rows = torch.empty(n, device=dev, dtype=torch.int32)
        self.loss = torch.empty(1, device=dev)
        self._ws = torch.zeros(4 + -(-n // 32), device=dev)  # ticket word + partials
        self._keep = (row_table, col_table, rows, cols, G, l, alias, neg_rows)
        self.seed, self.offset = seed, offset
        self._args = [row_table.data_ptr(), row_table.shape[1], col_table.data_ptr(), col_table.shape[1],
                      rows.data_ptr(), cols.data_ptr(), neg_rows.data_ptr() if neg_rows is not None else None,
                      alias.data_ptr() if alias is not None else None, alias.shape[0] if alias is not None else 0,
                      seed, offset, n, G.data_ptr(), l.data_ptr() if l is not None else None, d, float(margin),
                      self.pos.data_ptr(), self.neg.data_ptr(), self.neg_rows.data_ptr(), self.loss.data_ptr(),
                      self._ws.data_ptr()]
        self._fn = _lib.load().dg_decoder_hinge_f32

    def __call__(self, stream=None) -> None:
        a = list(self._args)
        a[9], a[10] = self.seed & (2**64 - 1), self.offset & (2**64 - 1)
        check(self._fn(*a, _stream_ptr(stream)), "dg_decoder_hinge_f32")


# --------------------------------------------------------------------------------------
# Training step (train.hip): decoder gradient, gather-gradient scatter, l2-norm backward, Adam
# --------------------------------------------------------------------------------------
class PreparedDecoderGrad:
    """dg_decoder_grad_f32 for one batch: row / column gradient rows of the n positive and n
    negative pairs, and the decoder parameter gradients dG = L·dM·L, dl, diag(dG) (each
    written only if its output tensor is given)."""

    def __init__(self, row_table, col_table, rows, cols, neg_rows, pos, neg, G, l, margin: float,
                 dG: Optional[torch.Tensor] = None, dl: Optional[torch.Tensor] = None,
                 dG_diag: Optional[torch.Tensor] = None):
        for t, nm, dt in ((row_table, "row_table", torch.float32), (col_table, "col_table", torch.float32),
                          (rows, "rows", torch.int32), (cols, "cols", torch.int32),
                          (neg_rows, "neg_rows", torch.int32), (pos, "pos", torch.float32),
                          (neg, "neg", torch.float32), (G, "G", torch.float32)):
            _dev(t, dt, nm)
        d = G.shape[0]
        n = rows.numel()
        if G.shape != (d, d) or row_table.shape[1] != d or col_table.shape[1] != d:
            raise ValueError("decoder_grad: shape mismatch")
        if cols.numel() != n or neg_rows.numel() != n or pos.numel() != n or neg.numel() != n:
            raise ValueError("decoder_grad: batch sizes differ")
        if l is not None:
            _dev(l, torch.float32, "l")
        if dl is not None and l is None:
            raise ValueError("dl needs a diagonal L")
        for t, nm, sz in ((dG, "dG", d * d), (dl, "dl", d), (dG_diag, "dG_diag", d)):
            if t is not None:
                _dev(t, torch.float32, nm)
                if t.numel() != sz:
                    raise ValueError(f"{nm} must have {sz} elements")
        dev = G.device
        self.grad_rows = torch.empty((2 * n, d), device=dev)
        self.grad_cols = torch.empty((n, d), device=dev)
        lib = _lib.load()
        nbytes = int(lib.dg_decoder_grad_workspace(n, d))
        self._ws = torch.empty(max(1, nbytes // 4), device=dev)
        self.row_idx = torch.empty(2 * n, device=dev, dtype=torch.int32)  # positives, then negatives
        self._rows, self._negs = rows, neg_rows
        self._keep = (row_table, col_table, rows, cols, neg_rows, pos, neg, G, l, dG, dl, dG_diag)
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        self._args = [row_table.data_ptr(), row_table.shape[1], col_table.data_ptr(), col_table.shape[1],
                      rows.data_ptr(), cols.data_ptr(), neg_rows.data_ptr(), n, pos.data_ptr(), neg.data_ptr(),
                      G.data_ptr(), ptr(l), d, float(margin), self.grad_rows.data_ptr(),
                      self.grad_cols.data_ptr(), ptr(dG), ptr(dl), ptr(dG_diag), self._ws.data_ptr(), nbytes]
        self._fn = lib.dg_decoder_grad_f32

    def __call__(self, stream=None) -> None:
        check(self._fn(*self._args, _stream_ptr(stream)), "dg_decoder_grad_f32")
        n = self._rows.numel()  # the scatter's row index list (negatives may be resampled per step)
        self.row_idx[:n].copy_(self._rows)
        self.row_idx[n:].copy_(self._negs)


def scatter_rows(idx: torch.Tensor, src: torch.Tensor, out: torch.Tensor, stream=None) -> None:
    """out[idx[q]] += Σ src[q'] over the occurrences q' of idx[q] (fixed order); indices
    outside out's rows update nothing (checked on the device: no host synchronisation, so
    the call is capturable)."""
    _dev(idx, torch.int32, "idx")
    _dev(src, torch.float32, "src")
    _dev(out, torch.float32, "out")
    n = idx.numel()
    if src.dim() != 2 or src.shape[0] != n or out.dim() != 2 or out.shape[1] != src.shape[1]:
        raise ValueError("scatter_rows: shapes")
    check(_lib.load().dg_scatter_rows_f32(idx.data_ptr(), n, src.data_ptr(), src.shape[1], out.data_ptr(),
                                          out.stride(0), out.shape[0], _stream_ptr(stream)), "dg_scatter_rows_f32")


class PreparedL2Grad:
    """dg_l2norm_grad_f32: ds_g = backward of l2_normalize(s_g) at dy (∘ [mask > 0]) for the
    groups (s_g, ds_g) of one node type."""

    def __init__(self, groups: Sequence[Tuple[torch.Tensor, torch.Tensor]], dy: torch.Tensor,
                 mask: Optional[torch.Tensor], n_rows: int, d: int):
        if not 1 <= len(groups) <= _lib.DG_MAX_GROUPS:
            raise ValueError("1..DG_MAX_GROUPS groups")
        for t, nm in [(dy, "dy")] + ([(mask, "mask")] if mask is not None else []):
            _dev(t, torch.float32, nm)
            if t.numel() < n_rows * d:
                raise ValueError(f"{nm} too small")
        arr = (DgL2gGroup * len(groups))()
        for i, (s_, ds) in enumerate(groups):
            _dev(s_, torch.float32, "s")
            _dev(ds, torch.float32, "ds")
            if s_.numel() < n_rows * d or ds.numel() < n_rows * d:
                raise ValueError("l2 grad group too small")
            arr[i].s, arr[i].ds = s_.data_ptr(), ds.data_ptr()
        self._arr, self._n = arr, len(groups)
        self._keep = (list(groups), dy, mask)
        self._args = (dy.data_ptr(), mask.data_ptr() if mask is not None else None, n_rows, d)
        self._fn = _lib.load().dg_l2norm_grad_f32

    def __call__(self, stream=None) -> None:
        check(self._fn(self._arr, self._n, *self._args, _stream_ptr(stream)), "dg_l2norm_grad_f32")


class PreparedAdam:
    """dg_adam_f32 over fixed (param, grad or None, m, v) segments (≤ DG_MAX_ADAM_SEGS per
    launch; more segments → several launches)."""

    def __init__(self, segs: Sequence[Tuple[torch.Tensor, Optional[torch.Tensor], torch.Tensor, torch.Tensor]]):
        self._arrs = []
        for s0 in range(0, len(segs), _lib.DG_MAX_ADAM_SEGS):
            chunk = segs[s0:s0 + _lib.DG_MAX_ADAM_SEGS]
            arr = (DgAdamSeg * len(chunk))()
            for i, (p, g, m, v) in enumerate(chunk):
                for t, nm in ((p, "param"), (m, "m"), (v, "v")) + (((g, "grad"),) if g is not None else ()):
                    _dev(t, torch.float32, nm)
                    if t.numel() != p.numel():
                        raise ValueError(f"adam {nm}: {t.numel()} elements, param has {p.numel()}")
                arr[i].param, arr[i].m, arr[i].v = p.data_ptr(), m.data_ptr(), v.data_ptr()
                arr[i].grad = g.data_ptr() if g is not None else None
                arr[i].n = p.numel()
            self._arrs.append((arr, len(chunk)))
        self._keep = list(segs)
        self._fn = _lib.load().dg_adam_f32

    def __call__(self, alpha: float, beta1: float, beta2: float, eps: float,
                 state: Optional[torch.Tensor] = None, stream=None) -> None:
        """alpha from the argument, or (state given: device float[3] {β1^t, β2^t, alpha}) from
        the device — the graph-capturable form."""
        sp = None
        if state is not None:
            _dev(state, torch.float32, "adam state")
            sp = state.data_ptr()
        for arr, n in self._arrs:
            check(self._fn(arr, n, alpha, beta1, beta2, eps, sp, _stream_ptr(stream)), "dg_adam_f32")


def adam_advance(state: torch.Tensor, lr: float, beta1: float, beta2: float, stream=None) -> None:
    """β1^t, β2^t ← ·β1, ·β2 and the next alpha, on the device (TF's _finish)."""
    _dev(state, torch.float32, "adam state")
    check(_lib.load().dg_adam_advance(state.data_ptr(), lr, beta1, beta2, _stream_ptr(stream)), "dg_adam_advance")


# --------------------------------------------------------------------------------------
# Dropout (dropout.hip)
# --------------------------------------------------------------------------------------
def _drop_state(state: torch.Tensor) -> None:
    if not (isinstance(state, torch.Tensor) and state.is_cuda and state.dtype == torch.int64
            and state.numel() >= 2):
        raise ValueError("dropout state must be an int64 device tensor {seed, step}")


def dropout_rows(inp: torch.Tensor, out: torch.Tensor, state: torch.Tensor, tag: int, keep: float,
                 stream=None) -> None:
    """out[r] = inp[r] · s(r) over the rows of a 2-D view (in place allowed)."""
    _dev(inp, torch.float32, "in")
    _dev(out, torch.float32, "out")
    _drop_state(state)
    d = inp.shape[-1]
    n = inp.numel() // d
    if out.numel() != inp.numel():
        raise ValueError("dropout_rows: shapes")
    check(_lib.load().dg_dropout_rows_f32(inp.data_ptr(), out.data_ptr(), n, d, state.data_ptr(), tag, keep,
                                          _stream_ptr(stream)), "dg_dropout_rows_f32")


def dropout_elems(src: torch.Tensor, out: torch.Tensor, state: torch.Tensor, tag: int, keep: float,
                  stream=None) -> None:
    """out[k] = src ∘ M_k / keep for k < out.shape[0] (src [n][d], out [K][n][d])."""
    _dev(src, torch.float32, "src")
    _dev(out, torch.float32, "out")
    _drop_state(state)
    K, n, d = out.shape
    if tuple(src.shape) != (n, d):
        raise ValueError("dropout_elems: shapes")
    check(_lib.load().dg_dropout_elems_f32(src.data_ptr(), out.data_ptr(), K, n, d, state.data_ptr(), tag, keep,
                                           _stream_ptr(stream)), "dg_dropout_elems_f32")


def _map_max(rel_map: torch.Tensor, rel_map_max: Optional[int]) -> int:
    """max(rel_map): host-known (plans pass it, so a captured step never syncs) or read once."""
    if not rel_map.numel():
        return -1
    return int(rel_map.max()) if rel_map_max is None else int(rel_map_max)


def dropout_rows_map(inp: torch.Tensor, out: torch.Tensor, rel_map: torch.Tensor, rows_per_slab: int,
                     state: torch.Tensor, tag: int, keep: float, in_global: bool, out_global: bool,
                     stream=None, rel_map_max: Optional[int] = None) -> None:
    """Row masks of a relation shard: local slab b (rows_per_slab rows) is global relation
    rel_map[b] and takes its mask bits; in / out addressed at global slabs (in_global /
    out_global) or local ones (dg_dropout_rows_map_f32).  The mask bit of a row is its global
    row index, 32-bit: (max(rel_map) + 1)·rows_per_slab must stay below 2^32, as the
    unmapped dg_dropout_rows_f32 requires of its rows."""
    _dev(inp, torch.float32, "in")
    _dev(out, torch.float32, "out")
    _dev(rel_map, torch.int32, "rel_map")
    _drop_state(state)
    d = inp.shape[-1]
    n_map = rel_map.numel()
    mx = _map_max(rel_map, rel_map_max)
    if (mx + 1) * rows_per_slab >= 0xFFFFFFFF:
        raise ValueError("dropout_rows_map: global row indices exceed the 32-bit mask counter")
    for t, glob in ((inp, in_global), (out, out_global)):
        slabs = t.numel() // (rows_per_slab * d) if rows_per_slab else 0
        need = (mx + 1) if (glob and n_map) else n_map
        if t.shape[-1] != d or slabs < need:
            raise ValueError("dropout_rows_map: operand too small for its slabs")
    check(_lib.load().dg_dropout_rows_map_f32(inp.data_ptr(), out.data_ptr(), rel_map.data_ptr(), n_map,
                                              rows_per_slab, d, (1 if in_global else 0) | (2 if out_global else 0),
                                              state.data_ptr(), tag, keep, _stream_ptr(stream)),
          "dg_dropout_rows_map_f32")


def dropout_elems_map(src: torch.Tensor, out: torch.Tensor, rel_map: torch.Tensor, state: torch.Tensor, tag: int,
                      keep: float, stream=None, rel_map_max: Optional[int] = None) -> None:
    """out[b] = src ∘ M_{rel_map[b]} / keep (src [n][d], out [K_local][n][d]): the per-relation
    tf.nn.dropout masks of a relation shard (dg_dropout_elems_map_f32).  Mask elements are
    rel_map[b]·n·d + r·d + f, 32-bit: (max(rel_map) + 1)·n·d must stay below 2^32, as the
    unmapped dg_dropout_elems_f32 requires of its K·n·d."""
    _dev(src, torch.float32, "src")
    _dev(out, torch.float32, "out")
    _dev(rel_map, torch.int32, "rel_map")
    _drop_state(state)
    K, n, d = out.shape
    if tuple(src.shape) != (n, d) or rel_map.numel() != K:
        raise ValueError("dropout_elems_map: shapes")
    if (_map_max(rel_map, rel_map_max) + 1) * n * d >= 0xFFFFFFFF:
        raise ValueError("dropout_elems_map: mask element indices exceed the 32-bit mask counter")
    check(_lib.load().dg_dropout_elems_map_f32(src.data_ptr(), out.data_ptr(), rel_map.data_ptr(), K, n, d,
                                               state.data_ptr(), tag, keep, _stream_ptr(stream)),
          "dg_dropout_elems_map_f32")


def dropout_advance(state: torch.Tensor, stream=None) -> None:
    _drop_state(state)
    check(_lib.load().dg_dropout_advance(state.data_ptr(), _stream_ptr(stream)), "dg_dropout_advance")
