"""ctypes binding of libdecagon_hip.so (include/decagon_hip.h).

This is the one place the Python layer touches native code.  There is no fallback: if the
library is missing or fails to load, importing the compute path raises, and every op of the
package fails loudly instead of silently running on the CPU.
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path
from ctypes import POINTER, c_float, c_int32, c_int64, c_uint64, c_void_p

from . import _build
from .tuning import knob

DG_OK = 0
DG_EINVAL = -1
DG_EALIGN = -2
DG_ETOOMANY = -3
DG_MAX_GROUPS = 8
DG_STAGED_MAX_CHUNKS = 128
DG_EPI_L2NORM = 1
DG_EPI_RELU = 2
DG_EPI_CHUNK_RELU = 4
ABI_VERSION = 38
DG_HINGE_WS_BYTES = 16 + 4 * 256  # decagon_hip.h
DG_RANK_LOGIT, DG_RANK_SIGMOID64, DG_RANK_SIGMOID32 = 0, 1, 2  # decagon_hip.h
DG_GROUP_SHARED_PATTERN = 1  # dg_rel_group.flags
DG_GROUP_DROPOUT = 2
DG_GROUP_DENSE_ROWS = 4  # dg_gcn_fused_f32 only: row r of the group's sum is x[r]
DG_MAX_ADAM_SEGS = 32
DG_PEER_MAX = 8  # peer exchange (decagon_hip.h)
DG_PEER_SLOTS = 8
DG_PEER_SUB_BASE, DG_PEER_SUB_STRIDE = 64, 16
DG_PEER_STATE_WORDS = DG_PEER_SUB_BASE + DG_PEER_SLOTS * 8 * DG_PEER_SUB_STRIDE
DG_PEER_ERROR_WORD = 2 * DG_PEER_SLOTS
DG_PEER_DIAG_BASE, DG_PEER_DIAG_WORDS, DG_PEER_SLOW_TICKS = 24, 18, 10000  # wait records (round 6)
DG_IPC_HANDLE_BYTES = 64
DG_EPI_PUSH = 1

_ERRS = {DG_EINVAL: "DG_EINVAL", DG_EALIGN: "DG_EALIGN", DG_ETOOMANY: "DG_ETOOMANY"}


class DgRelGroup(ctypes.Structure):
    _fields_ = [
        ("rowptr", c_void_p),
        ("vcol", c_void_p),
        ("val", c_void_p),
        ("x", c_void_p),
        ("out", c_void_p),
        ("x_ld", c_int64),
        ("n_rows", c_int32),
        ("n_chunks", c_int32),
        ("x_rows", c_int32),
        ("flags", c_int32),
        ("drop_tag", ctypes.c_uint32),
        ("drop_keep", c_float),
        ("drop_stride", c_int32),
        ("drop_state", c_void_p),
        ("drop_index", c_void_p),
    ]


class DgStagedGroup(ctypes.Structure):
    _fields_ = [
        ("pairs", c_void_p),
        ("jm", c_void_p),
        ("jmoff", c_void_p),
        ("slab", c_void_p),
        ("x", c_void_p),
        ("out", c_void_p),
        ("x_ld", c_int64),
        ("n_rows", c_int32),
        ("n_cols", c_int32),
        ("n_rels", c_int32),
        ("out_chunk", c_int32),
        ("x_rows", c_int32),
        ("jm_len", c_int32),
        ("chunk_start", c_void_p),   # HOST int32 [n_chunks + 1] or NULL (fixed out_chunk)
        ("n_chunks", c_int32),
        ("pad", c_int32),
    ]


class DgSegGroup(ctypes.Structure):
    _fields_ = [
        ("rowptr", c_void_p),
        ("seg", c_void_p),
        ("vcol", c_void_p),
        ("val", c_void_p),
        ("slab", c_void_p),
        ("x", c_void_p),
        ("w", c_void_p),
        ("out", c_void_p),
        ("x_ld", c_int64),
        ("n_rows", c_int32),
        ("n_cols", c_int32),
        ("n_chunks", c_int32),
        ("chunk", c_int32),
        ("n_rels", c_int32),
        ("x_rows", c_int32),
    ]


class DgTabDesc(ctypes.Structure):
    """dg_tab_desc: one wave's 64-byte descriptor (the wave-table fused launch)."""
    _fields_ = [("x", c_void_p), ("w", c_void_p), ("orow", c_void_p), ("cnt", c_int32), ("x_ld", c_int32),
                ("ovf", c_int32), ("role", ctypes.c_uint32), ("wr", ctypes.c_uint32), ("pad", c_int32 * 5)]


class DgWaveTable(ctypes.Structure):
    _fields_ = [("pairs", c_void_p), ("ovf", c_void_p), ("desc", c_void_p), ("n_blocks", c_int32),
                ("nw", c_int32), ("nw_stride", c_int32), ("slot_pairs", c_int32)]


class DgStagedProj(ctypes.Structure):
    _fields_ = [("h", c_void_p), ("w", c_void_p), ("h_ld", c_int64), ("din", c_int32), ("pad", c_int32)]


class DgProj(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("rel_map", c_void_p), ("out", c_void_p), ("n_rels", c_int32),
                ("target", c_int32), ("d_out", c_int32), ("reserved", c_int32)]


class DgFusedTarget(ctypes.Structure):
    _fields_ = [("out", c_void_p), ("n_rows", c_int32), ("g_begin", c_int32), ("g_count", c_int32),
                ("flags", c_int32)]


class DgEpiGroup(ctypes.Structure):
    _fields_ = [("partial", c_void_p), ("sum_out", c_void_p), ("n_chunks", c_int32), ("group_flags", c_int32)]


class DgEpiTarget(ctypes.Structure):
    _fields_ = [
        ("groups", POINTER(DgEpiGroup)),
        ("n_groups", c_int32),
        ("reserved0", c_int32),
        ("out", c_void_p),
        ("n_rows", c_int32),
        ("target_flags", c_int32),
        ("reserved", c_int32 * 2),
    ]


class DgPeerXchg(ctypes.Structure):
    _fields_ = [
        ("delta", c_int64 * DG_PEER_MAX),
        ("flags", c_void_p * DG_PEER_MAX),
        ("state", c_void_p),
        ("timeout_ticks", c_int64),
        ("rank", c_int32),
        ("world", c_int32),
        ("slot", c_int32),
        ("loopback", c_int32),
    ]


class DgGemmDesc(ctypes.Structure):
    _fields_ = [
        ("a", c_void_p),
        ("b", c_void_p),
        ("c", c_void_p),
        ("sa", c_void_p),
        ("sc", c_void_p),
        ("b_map", c_void_p),
        ("a_bs", c_int64),
        ("a_sm", c_int64),
        ("a_sk", c_int64),
        ("b_bs", c_int64),
        ("b_sk", c_int64),
        ("b_sn", c_int64),
        ("c_bs", c_int64),
        ("c_sm", c_int64),
        ("c_sn", c_int64),
        ("m", c_int32),
        ("n", c_int32),
        ("k", c_int32),
        ("batch", c_int32),
        ("reduce", c_int32),
        ("drop_tag", ctypes.c_uint32),
        ("drop_state", c_void_p),
        ("drop_keep", c_float),
        ("reserved", c_int32),
    ]


class DgL2gGroup(ctypes.Structure):
    _fields_ = [("s", c_void_p), ("ds", c_void_p)]


class DgAdamSeg(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("m", c_void_p), ("v", c_void_p), ("n", c_int64)]


# name -> (restype, argtypes); must match include/decagon_hip.h exactly.
SIGNATURES = {
    "dg_abi_version": (c_int32, []),
    "dg_spmm_groups_f32": (c_int32, [POINTER(DgRelGroup), c_int32, c_int32, c_void_p]),
    "dg_spmm_groups_lds_f32": (c_int32, [POINTER(DgRelGroup), c_int32, c_int32, c_void_p]),
    "dg_spmm_seg_f32": (c_int32, [POINTER(DgSegGroup), c_int32, c_int32, c_int32, c_void_p]),
    "dg_gcn_fused_seg_f32": (c_int32, [POINTER(DgSegGroup), c_int32, POINTER(DgFusedTarget), c_int32, c_int32,
                                       c_int32, c_void_p]),
    "dg_spmm_csr_f32": (
        c_int32,
        [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_int64, c_void_p, c_int64, c_int32,
         c_float, c_void_p],
    ),
    "dg_rownorm_l2_f32": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p]),
    "dg_gcn_fused_f32": (
        c_int32,
        [POINTER(DgRelGroup), c_int32, POINTER(DgFusedTarget), c_int32, POINTER(DgProj), c_int32, c_int32,
         c_int32, c_void_p],
    ),
    "dg_gcn_epilogue_multi_f32": (c_int32, [POINTER(DgEpiTarget), c_int32, c_int32, c_int32, c_void_p]),
    "dg_gcn_epilogue_peer_f32": (c_int32, [POINTER(DgEpiTarget), c_int32, c_int32, c_int32, POINTER(DgPeerXchg),
                                           c_void_p]),
    "dg_gcn_fused_tab_f32": (c_int32, [POINTER(DgWaveTable), c_int32, c_int32, c_void_p]),
    "dg_gcn_fused_tab_peer_f32": (c_int32, [POINTER(DgWaveTable), c_int32, c_int32, POINTER(DgPeerXchg), c_void_p]),
    "dg_spmm_seg_tab_f32": (c_int32, [POINTER(DgWaveTable), c_int32, c_int32, c_void_p]),
    "dg_gcn_epilogue_tab_f32": (c_int32, [c_void_p, c_int32, c_int32, c_int32, POINTER(DgPeerXchg), c_void_p]),
    "dg_gcn_fused_seg_peer_f32": (c_int32, [POINTER(DgSegGroup), c_int32, POINTER(DgFusedTarget), c_int32, c_int32,
                                            c_int32, POINTER(DgPeerXchg), c_void_p]),
    "dg_peer_alloc": (c_int32, [c_int64, c_int32, POINTER(c_void_p)]),
    "dg_peer_free": (c_int32, [c_void_p]),
    "dg_ipc_get_handle": (c_int32, [c_void_p, c_void_p, POINTER(c_int64)]),
    "dg_ipc_open": (c_int32, [c_void_p, POINTER(c_void_p)]),
    "dg_ipc_close": (c_int32, [c_void_p]),
    "dg_peer_read": (c_int32, [c_void_p, c_void_p, c_int64]),
    "dg_peer_allgather": (c_int32, [POINTER(DgPeerXchg), c_void_p, POINTER(c_int64), POINTER(c_int64), c_int32,
                                    c_void_p]),
    "dg_gcn_epilogue_f32": (
        c_int32,
        [POINTER(DgEpiGroup), c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    ),
    "dg_gemm_f32": (c_int32, [POINTER(DgGemmDesc), c_int32, c_void_p]),
    "dg_gemm_tn_f32": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_void_p, c_int32,
                                 c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "dg_dropout_rows_f32": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, ctypes.c_uint32, c_float,
                                      c_void_p]),
    "dg_dropout_elems_f32": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p,
                                       ctypes.c_uint32, c_float, c_void_p]),
    "dg_dropout_rows_map_f32": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_int32, c_int32, c_void_p,
                                          ctypes.c_uint32, ctypes.c_float, c_void_p]),
    "dg_dropout_elems_map_f32": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p,
                                           ctypes.c_uint32, ctypes.c_float, c_void_p]),
    "dg_dropout_advance": (c_int32, [c_void_p, c_void_p]),
    "dg_spmm_staged_f32": (c_int32, [POINTER(DgStagedGroup), c_int32, c_int32, c_void_p]),
    "dg_spmm_staged_proj_f32": (c_int32, [POINTER(DgStagedGroup), POINTER(DgStagedProj), c_int32, c_int32, c_void_p]),
    "dg_staged_block": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_void_p]),
    "dg_decoder_score_bf16": (c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p,
                                        c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "dg_slot_score_hinge_bf16": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_void_p, c_void_p,
                                           c_void_p, c_int32,
                                           c_int64, c_int32, c_int32, c_int32, c_uint64, c_void_p, c_void_p,
                                           c_int32, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "dg_decoder_score_bf16_paired": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64, c_void_p,
                                               c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                               c_void_p]),
    "dg_decoder_hinge_f32": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
         c_uint64, c_uint64, c_int32, c_void_p, c_void_p, c_int32, c_float, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p],
    ),
    "dg_decoder_score_f32": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
         c_int32, c_void_p, c_void_p],
    ),
    "dg_hinge_loss_f32": (c_int32, [c_void_p, c_void_p, c_int32, c_float, c_void_p, c_void_p]),
    "dg_hinge_loss_ws_f32": (c_int32, [c_void_p, c_void_p, c_int32, c_float, c_void_p, c_void_p, c_void_p]),
    "dg_xent_loss_f32": (c_int32, [c_void_p, c_void_p, c_int32, c_float, c_void_p, c_void_p]),
    "dg_decoder_grad_workspace": (c_int64, [c_int32, c_int32]),
    "dg_decoder_grad_f32": (
        c_int32,
        [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
         c_void_p, c_void_p, c_int32, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
         c_int64, c_void_p],
    ),
    "dg_scatter_rows_f32": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_int64, c_int32,
                                      c_void_p]),
    "dg_l2norm_grad_f32": (c_int32, [POINTER(DgL2gGroup), c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                     c_void_p]),
    "dg_adam_f32": (c_int32, [POINTER(DgAdamSeg), c_int32, c_float, c_float, c_float, c_float, c_void_p,
                              c_void_p]),
    "dg_adam_advance": (c_int32, [c_void_p, c_float, c_float, c_float, c_void_p]),
    "dg_rank_metrics_workspace": (c_int64, [c_int32]),
    "dg_rank_metrics_ex_workspace": (c_int64, [c_int32, c_int32]),
    "dg_rank_metrics_ex_f32": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                         c_int64, c_void_p]),
    "dg_rank_metrics_f32": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_int64,
                                      c_void_p]),
    "dg_unigram_sample_slots": (c_int32, [c_void_p, c_int32, c_int64, c_int32, c_int32, c_int32, ctypes.c_uint64,
                                          c_void_p, c_void_p]),
    "dg_unigram_sample": (
        c_int32,
        [c_void_p, c_int32, c_int32, c_uint64, c_uint64, c_void_p, c_void_p],
    ),
}

_LIB = None
_LOAD_LOCK = threading.Lock()  # staged_layout's thread pool may make the first call


class KernelError(RuntimeError):
    pass


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load (building first if needed and allowed) and type the native library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOAD_LOCK:
        if _LIB is None:
            _LIB = _load(build_if_missing)
    return _LIB


def _load(build_if_missing: bool) -> ctypes.CDLL:
    override = knob("DG_LIB", "")  # an instrumented build (scripts/staged_prof.py)
    path = Path(override) if override else _build.lib_path()
    if not override and (not path.exists() or (build_if_missing and _build.needs_build())):
        if not build_if_missing:
            raise ImportError(f"{path} missing: run __graft_entry__.build() or python -m decagon_amd._build")
        _build.build()
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    got = lib.dg_abi_version()
    if got != ABI_VERSION:
        raise ImportError(f"libdecagon_hip ABI {got} != expected {ABI_VERSION}; rebuild")
    return lib


def check(rc: int, what: str) -> None:
    if rc != DG_OK:
        name = _ERRS.get(rc, f"hipError_t {rc}")
        raise KernelError(f"{what} failed: {name}")
