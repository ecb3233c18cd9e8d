"""RCCL communicator for the collectives inside the captured step (one process per GPU).

The per-layer exchange of the sharded forward (sharding.py: the all-reduce of the
relation-sharded pre-normalisation sums, the all-gather of the row-split blocks) and config
5's scalar-loss all-reduce are captured into the step's hipGraph together with the kernels.
They are issued straight to RCCL (the librccl.so PyTorch-ROCm ships) on the caller's current
stream, through a communicator of their own: a collective issued through torch.distributed's
ProcessGroupNCCL inside a capture leaves a work item whose event was recorded in the capturing
stream, and the process group's watchdog thread later queries that event and aborts the
process (hipErrorCapturedEvent) — observed on the one-GPU RCCL rehearsal, ROCm 7 / torch 2.10.
torch.distributed stays in charge of rendezvous, barriers and the eager timing reductions.

RCCL symbols used (nccl.h names): ncclGetUniqueId, ncclCommInitRank, ncclAllReduce,
ncclAllGather, ncclCommDestroy, ncclGetErrorString.
"""
from __future__ import annotations

import ctypes
from pathlib import Path
from typing import Callable, Optional, Tuple

import torch

_NCCL_FLOAT32 = 7  # ncclDataType_t
_NCCL_SUM = 0      # ncclRedOp_t


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_byte * 128)]


_LIB = None


def _lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        path = Path(torch.__file__).resolve().parent / "lib" / "librccl.so"
        lib = ctypes.CDLL(str(path))
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
        lib.ncclAllGather.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]
        lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        _LIB = lib
    return _LIB


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what}: RCCL error {rc} ({_lib().ncclGetErrorString(rc).decode()})")


class RcclComm:
    """One RCCL communicator over the ranks of the default torch.distributed group (the
    unique id travels through it); collectives run on torch's current stream, so they are
    captured into whatever hipGraph that stream is recording."""

    def __init__(self, rank: int, world: int):
        import torch.distributed as dist

        lib = _lib()
        uid = _UniqueId()
        if rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        box = [bytes(bytearray(uid.internal))]
        dist.broadcast_object_list(box, src=0)
        ctypes.memmove(ctypes.addressof(uid), box[0], 128)
        self.comm = ctypes.c_void_p()
        _check(lib.ncclCommInitRank(ctypes.byref(self.comm), world, uid, rank), "ncclCommInitRank")
        self.rank, self.world = rank, world

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def all_reduce(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> None:
        """Sum over the ranks of a contiguous fp32 device tensor, in place or into `out`."""
        out = t if out is None else out
        for x in (t, out):
            if x.dtype != torch.float32 or not x.is_contiguous() or not x.is_cuda:
                raise ValueError("RcclComm.all_reduce takes contiguous fp32 device tensors")
        if out.numel() != t.numel():
            raise ValueError("RcclComm.all_reduce: out must match t")
        _check(_lib().ncclAllReduce(t.data_ptr(), out.data_ptr(), t.numel(), _NCCL_FLOAT32, _NCCL_SUM,
                                    self.comm, self._stream()), "ncclAllReduce")

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """out = the ranks' equal blocks in rank order; `inp` may be this rank's block of `out`
        (in place, as RCCL allows)."""
        for x in (out, inp):
            if x.dtype != torch.float32 or not x.is_contiguous() or not x.is_cuda:
                raise ValueError("RcclComm.all_gather takes contiguous fp32 device tensors")
        if out.numel() != inp.numel() * self.world:
            raise ValueError("RcclComm.all_gather: out must hold world x inp elements")
        # in place: inp must be exactly this rank's block of out (RCCL reads it from there)
        lo, hi = out.data_ptr(), out.data_ptr() + 4 * out.numel()
        if lo <= inp.data_ptr() < hi and inp.data_ptr() != lo + 4 * self.rank * inp.numel():
            raise ValueError("RcclComm.all_gather: an in-place input must be this rank's block of out")
        _check(_lib().ncclAllGather(inp.data_ptr(), out.data_ptr(), inp.numel(), _NCCL_FLOAT32, self.comm,
                                    self._stream()), "ncclAllGather")

    def collectives(self) -> Tuple[Callable[..., None], Callable[[torch.Tensor, torch.Tensor], None]]:
        """(allreduce, allgather) with the signatures sharding.RelationShard takes."""
        return self.all_reduce, self.all_gather

    def destroy(self) -> None:
        if self.comm:
            _lib().ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()


_COMM: Optional[RcclComm] = None


def world_comm() -> RcclComm:
    """The process's RCCL communicator over the default group (created once, collectively)."""
    import torch.distributed as dist

    global _COMM
    if _COMM is None:
        _COMM = RcclComm(dist.get_rank(), dist.get_world_size())
    return _COMM
