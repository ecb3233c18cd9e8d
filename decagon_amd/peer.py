"""Peer-store exchange over xGMI: the sharded forward's all-gather of row-split blocks without
RCCL (csrc/peer.h has the device protocol, include/decagon_hip.h the C ABI).

Why: config S at N GPUs (weak scaling, sharding.RelationShard.weak_sets) exchanges two small
row blocks per step (29 KB + 14 KB per rank at N = 8).  An RCCL all-gather of that size costs
several µs of launch, handshake and per-hop latency; ≥ 6× at 8 GPUs leaves ≈ 2 µs for both
(DESIGN.md §6).  Here every rank's finishing kernel stores its finished rows straight into
every peer's copy of the output (IPC-mapped peer memory) and its last workgroup raises an
arrival flag at every peer and waits — bounded — for theirs, so the exchange costs no launch
of its own.

    region   one device tensor per rank holding every row-split output of the plan, the same
             layout on every rank (ForwardPlan carves the padded outputs from it); exported
             with hipIpcGetMemHandle and opened by every peer
    flags    one uncached block per rank ([DG_PEER_SLOTS][DG_PEER_MAX] words) that the peers
             write and only its owner polls
    state    this rank's per-slot {arrivals, epoch} and the error word (a torch int32 tensor)

Modes (PeerConfig.mode): "fused" — the row-split layer's finishing launch pushes and
exchanges (dg_gcn_epilogue_peer_f32 / dg_gcn_fused_seg_peer_f32), slots 0 and 1;
"kernel" — the layer's exchange is one stand-alone dg_peer_allgather launch, slots 2 and 3.
`loopback` is the one-GPU rehearsal: every "peer" copy is local scratch, and the last
workgroup raises every rank's flag itself, so one process times a rank's share with the
exchange's stores, arrivals, flags and polls in it (not the xGMI wire latency).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.utils.dlpack

from . import _lib
from ._lib import DgPeerXchg, check

TIMEOUT_S = 2.0          # a wait gives up (error word) after this long
_TICKS_PER_S = 100e6     # s_memrealtime: 100 MHz

SLOT_FUSED = 0           # + layer - 1
SLOT_KERNEL = 2          # + layer - 1
SLOT_PROBE = 4           # + layer - 1: bench.py's stand-alone exchange timing beside another mode


@dataclass
class PeerConfig:
    """How a RelationShard's row-split blocks are exchanged when not over RCCL.

    region_kind: the memory of the exchange region (dg_peer_alloc kinds): 0 coarse-grained
    device memory (a torch allocation), 1 fine-grained, 2 uncached (the default since round 6).
    Uncached, a row a peer stored over xGMI is read from memory by every later kernel of the
    receiving GPU — no line of it can be stale in an L2 that cached it before the peer rewrote
    it — and it measured no slower in loopback (config S at N = 8: 25.35 µs a rank against
    25.91 coarse-grained and 26.00 fine-grained; config P: 114.3 against 114.6 / 116.7;
    DESIGN §6)."""

    mode: str = "fused"                                       # "fused" | "kernel"
    gather: Optional[Callable[[object], List[object]]] = None  # all-gather of picklable objects
    loopback: bool = False
    timeout_s: float = TIMEOUT_S
    region_kind: int = 2

    def __post_init__(self):
        if self.mode not in ("fused", "kernel"):
            raise ValueError(f"unknown peer exchange mode {self.mode!r}")
        if not self.loopback and self.gather is None:
            raise ValueError("a peer exchange across processes needs an object all-gather")
        if self.region_kind not in (0, 1, 2):
            raise ValueError("region_kind: 0 (coarse-grained), 1 (fine-grained) or 2 (uncached)")


# ---- device memory of a given kind as a torch tensor (DLPack) ----
class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int), ("device_id", ctypes.c_int)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int), ("dtype", _DLDataType),
                ("shape", ctypes.POINTER(ctypes.c_int64)), ("strides", ctypes.POINTER(ctypes.c_int64)),
                ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(_DLManagedTensor))
_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p), ("deleter", _DELETER)]
_LIVE = {}  # id -> (managed struct, shape, deleter, pointer): alive until torch releases the tensor


def device_tensor(numel: int, kind: int, device: torch.device) -> torch.Tensor:
    """A zeroed float32 device tensor of `numel` elements in dg_peer_alloc memory of `kind`
    (0 coarse-grained, 1 fine-grained, 2 uncached), owned by torch: the memory is freed with
    dg_peer_free when the last view of the tensor is released."""
    lib = _lib.load()
    ptr = ctypes.c_void_p()
    check(lib.dg_peer_alloc(4 * max(1, numel), kind, ctypes.byref(ptr)), "dg_peer_alloc")
    shape = (ctypes.c_int64 * 1)(numel)
    m = _DLManagedTensor()
    key = id(m)

    def _free(_):
        ent = _LIVE.pop(key, None)
        if ent is not None:
            lib.dg_peer_free(ent[3])

    deleter = _DELETER(_free)
    m.dl_tensor.data = ptr.value
    m.dl_tensor.device = _DLDevice(10, device.index or 0)  # kDLROCM
    m.dl_tensor.ndim = 1
    m.dl_tensor.dtype = _DLDataType(2, 32, 1)  # kDLFloat, 32 bits
    m.dl_tensor.shape = shape
    m.dl_tensor.strides = None
    m.dl_tensor.byte_offset = 0
    m.deleter = deleter
    _LIVE[key] = (m, shape, deleter, ptr.value)
    pycapsule_new = ctypes.pythonapi.PyCapsule_New
    pycapsule_new.restype = ctypes.py_object
    pycapsule_new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    cap = pycapsule_new(ctypes.addressof(m), b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(cap)


def dist_gather(group=None) -> Callable[[object], List[object]]:
    """The object all-gather of torch.distributed's default (or given) group."""
    import torch.distributed as dist

    def _g(obj):
        out = [None] * dist.get_world_size(group)
        dist.all_gather_object(out, obj, group=group)
        return out

    return _g


class PeerExchange:
    """This rank's view of every rank's exchange region and flag block (collective: every
    rank constructs it at the same point, with regions of the same size and layout)."""

    def __init__(self, region: torch.Tensor, rank: int, world: int, cfg: PeerConfig):
        if not region.is_cuda or not region.is_contiguous():
            raise ValueError("the exchange region must be a contiguous device tensor")
        if region.data_ptr() % 16:
            raise ValueError("the exchange region must be 16-byte aligned")
        if not 1 <= world <= _lib.DG_PEER_MAX or not 0 <= rank < world:
            raise ValueError(f"peer exchange: rank {rank} of {world} (at most {_lib.DG_PEER_MAX} ranks)")
        self.lib = _lib.load()
        self.region, self.rank, self.world, self.cfg = region, rank, world, cfg
        self.nbytes = region.numel() * region.element_size()
        dev = region.device
        self.state = torch.zeros(_lib.DG_PEER_STATE_WORDS, dtype=torch.int32, device=dev)
        fp = ctypes.c_void_p()
        check(self.lib.dg_peer_alloc(4 * _lib.DG_PEER_SLOTS * _lib.DG_PEER_MAX, 2, ctypes.byref(fp)), "dg_peer_alloc")
        self._flags = fp.value
        self._opened: List[int] = []
        self._scratch: List[torch.Tensor] = []
        base = region.data_ptr()
        bases, flags = [0] * world, [0] * world
        if cfg.loopback:
            for p in range(world):
                if p == rank:
                    bases[p] = base
                else:  # (the peers' regions stand-ins: of the configured memory kind too)
                    self._scratch.append(torch.empty_like(region) if cfg.region_kind == 0
                                         else device_tensor(region.numel(), cfg.region_kind, dev))
                    bases[p] = self._scratch[-1].data_ptr()
                flags[p] = self._flags
        else:
            mine = (self._handle(base), self._handle(self._flags), self.nbytes)
            got = cfg.gather(mine)
            if len(got) != world:
                raise RuntimeError(f"peer exchange: {len(got)} ranks answered, {world} expected")
            for p, ((h, off), (hf, offf), nb) in enumerate(got):
                if nb != self.nbytes:
                    raise RuntimeError(f"peer exchange: rank {p}'s region is {nb} B, this rank's {self.nbytes} B")
                if p == rank:
                    bases[p], flags[p] = base, self._flags
                    continue
                bases[p] = self._open(h) + off
                flags[p] = self._open(hf) + offf
        self.bases, self.flags = bases, flags
        self.delta = [b - base for b in bases]
        if any(d % 16 for d in self.delta):
            raise RuntimeError("peer exchange: a peer region is not 16-byte aligned")
        self._descs = {}
        self.failed = 0  # the error word last read by check() (nonzero: the exchange is poisoned)

    # ---- IPC ----
    def _handle(self, ptr: int) -> Tuple[bytes, int]:
        h = (ctypes.c_char * _lib.DG_IPC_HANDLE_BYTES)()
        off = ctypes.c_int64()
        check(self.lib.dg_ipc_get_handle(ptr, h, ctypes.byref(off)), "dg_ipc_get_handle")
        return bytes(h), int(off.value)

    def _open(self, handle: bytes) -> int:
        h = (ctypes.c_char * _lib.DG_IPC_HANDLE_BYTES).from_buffer_copy(handle)
        p = ctypes.c_void_p()
        check(self.lib.dg_ipc_open(h, ctypes.byref(p)), "dg_ipc_open (hipIpcOpenMemHandle)")
        self._opened.append(p.value)
        return p.value

    # ---- descriptors ----
    def xchg(self, slot: int) -> DgPeerXchg:
        """The C descriptor of one exchange slot (kept alive by this object)."""
        if not 0 <= slot < _lib.DG_PEER_SLOTS:
            raise ValueError(f"slot {slot} out of range")
        d = self._descs.get(slot)
        if d is None:
            d = DgPeerXchg()
            for p in range(self.world):
                d.delta[p] = self.delta[p]
                d.flags[p] = self.flags[p]
            d.state = self.state.data_ptr()
            d.timeout_ticks = int(self.cfg.timeout_s * _TICKS_PER_S)
            d.rank, d.world, d.slot, d.loopback = self.rank, self.world, slot, int(self.cfg.loopback)
            self._descs[slot] = d
        return d

    def offset(self, t: torch.Tensor) -> int:
        """Byte offset of a tensor (view) inside the region."""
        off = t.data_ptr() - self.region.data_ptr()
        if off < 0 or off + t.numel() * t.element_size() > self.nbytes:
            raise ValueError("tensor is not inside the exchange region")
        return off

    def allgather_fn(self, blocks: Sequence[torch.Tensor], slot: int) -> Callable[[], None]:
        """A prepared stand-alone exchange of this rank's blocks (views of the region)."""
        n = len(blocks)
        if not 1 <= n <= _lib.DG_MAX_GROUPS:
            raise ValueError("1..8 blocks per exchange")
        offs = (ctypes.c_int64 * n)(*[self.offset(b) for b in blocks])
        sizes = (ctypes.c_int64 * n)(*[b.numel() * b.element_size() for b in blocks])
        x = self.xchg(slot)
        fn, reg = self.lib.dg_peer_allgather, self.region.data_ptr()
        keep = (offs, sizes, x, list(blocks))

        def run(stream=None):
            _ = keep
            s = torch.cuda.current_stream() if stream is None else stream
            check(fn(ctypes.byref(x), reg, offs, sizes, n, s.cuda_stream), "dg_peer_allgather")

        return run

    # ---- status ----
    def error(self) -> int:
        """The error word (0: every wait so far completed); synchronises the device."""
        torch.cuda.synchronize(self.region.device)
        return int(self.state[_lib.DG_PEER_ERROR_WORD].item())

    def flags_now(self) -> List[int]:
        """This rank's flag block as it stands now ([DG_PEER_SLOTS][DG_PEER_MAX] words; device
        synchronised first)."""
        torch.cuda.synchronize(self.region.device)
        n = _lib.DG_PEER_SLOTS * _lib.DG_PEER_MAX
        buf = (ctypes.c_uint32 * n)()
        check(self.lib.dg_peer_read(self._flags, buf, 4 * n), "dg_peer_read")
        return list(buf)

    def diagnostics(self) -> dict:
        """The device's wait records (decagon_hip.h, DG_PEER_DIAG_BASE): the slow completed
        waits (count, longest in µs) and, after a timeout, the timed-out wait — its slot, the
        epoch it expected, each source's flag word when it gave up and NOW, and the verdict per
        late source: "late" (its flag reached the expected epoch after the bound: a host or
        scheduling skew longer than the bound) or "never raised" (still short of it)."""
        st = [int(x) & 0xffffffff for x in self.state.cpu().tolist()]
        b = _lib.DG_PEER_DIAG_BASE
        out = {"slow_waits": st[b + 16], "slowest_wait_us": st[b + 17] / _TICKS_PER_S * 1e6,
               "error_word": st[_lib.DG_PEER_ERROR_WORD]}
        if not out["error_word"]:
            return out
        slot, want = st[b], st[b + 1]
        seen = st[b + 2:b + 2 + self.world]
        tick = lambda lo: (st[b + lo] | (st[b + lo + 1] << 32))  # noqa: E731
        now = self.flags_now()[slot * _lib.DG_PEER_MAX:slot * _lib.DG_PEER_MAX + self.world]
        late = {}
        for s_, (v, w) in enumerate(zip(seen, now)):
            if ((v - want) & 0xffffffff) >= 0x80000000:  # short of the expected epoch at the bound
                late[s_] = "late" if ((w - want) & 0xffffffff) < 0x80000000 else "never raised"
        out.update({"slot": slot, "expected_epoch": want, "flags_at_bound": seen, "flags_now": now,
                    "waited_us": (tick(12) - tick(10)) / _TICKS_PER_S * 1e6,
                    "raised_to_wait_us": (tick(10) - tick(14)) / _TICKS_PER_S * 1e6,
                    "wait_start_tick": tick(10), "late_sources": late})
        return out

    def check(self) -> None:
        """Raise if any wait so far timed out (synchronises the device).  A timed-out wait
        poisons the exchange on the device (csrc/peer.h: this rank then raises no flag and
        waits for none, so every peer's next wait times out too); here it poisons the host
        side: every later ensure_ok() — ForwardPlan.run's entry — raises as well.  The message
        carries the wait record (diagnostics()): which sources were late or never arrived."""
        e = self.error()
        if e:
            self.failed = e
            try:
                self.failed_diag = self.diagnostics()
            except Exception as exc:  # the record is an aid; the error stands without it
                self.failed_diag = {"unreadable": repr(exc)}
        self.ensure_ok()

    def ensure_ok(self) -> None:
        """Raise if an earlier check() found a timed-out wait (no device access)."""
        e = self.failed
        if e:
            raise RuntimeError(f"peer exchange timed out: slot {(e >> 8) & 0xff}, waiting for rank {e & 0xff} "
                               f"(error word {e:#x}); the exchange is poisoned, rebuild the plan; "
                               f"wait record: {getattr(self, 'failed_diag', None)}")

    def close(self) -> None:
        """Unmap the peers' regions and free the flag block (after the last exchange)."""
        if self.region.is_cuda:
            torch.cuda.synchronize(self.region.device)
        for p in self._opened:
            self.lib.dg_ipc_close(p)
        self._opened = []
        if self._flags:
            self.lib.dg_peer_free(self._flags)
            self._flags = 0
        self._scratch = []
