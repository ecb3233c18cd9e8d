"""Session-side plumbing shared by layers, model and optimizer: parameter placement,
variable scopes, feed → device conversion with caching, and the standalone (single edge
type) layer forward.

Feed caching.  The reference re-feeds every adjacency tuple on every step
(minibatch.py:259-267).  A session caches the host CSR and the device copy of a fed sparse
value keyed by the identity of the objects fed — the arrays of a (coords, values, shape)
tuple, or the scipy matrix / SparseTensorValue itself — and keeps those objects referenced,
so a key cannot be recycled; re-feeding the same values — what every reference driver does —
costs nothing.  Fed numpy arrays are marked read-only when cached, so mutating one in place
fails loudly instead of leaving a stale device copy (feed a new array instead, or call
`Session.invalidate_feeds()`).  The caches are LRU-bounded by bytes (host: DG_FEED_CACHE_HOST_MB,
default 8 GiB; device graphs + plans: DG_FEED_CACHE_DEVICE_MB, default 64 GiB of the 288 GB),
so a driver that re-masks graphs every step (the active learners) cannot grow them without
bound.
"""
from __future__ import annotations

import contextlib
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp
import torch

from . import kernels
from ._lib import DG_EPI_CHUNK_RELU, DG_EPI_L2NORM
from .engine import DeviceGraph, DeviceGroup
from .graph import InvalidArgumentError, Node, RunContext
from .sparse import HostCSR, SparseTensorValue, as_coo_tuple, coo_to_csr, is_identity
from .tuning import knob

_scope: List[str] = []


def param_device() -> torch.device:
    """Parameters live on the HIP device when one is visible (always, on the GPU box).
    Without one they are allocated on the host so the model can be constructed and
    inspected, but nothing can run: Session() refuses to start without a device."""
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


@contextlib.contextmanager
def variable_scope(name: str):
    _scope.append(name)
    try:
        yield
    finally:
        _scope.pop()


def scoped(name: str) -> str:
    return "/".join(_scope + [name])


def as_device_f32(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        if not x.is_cuda:
            x = x.to("cuda")
        return x.to(torch.float32).contiguous()
    return torch.as_tensor(np.asarray(x, np.float32), device="cuda")


# ---------------------------------------------------------------- sparse feeds → device
class ByteLRU:
    """An LRU map bounded by the bytes of its entries.  Inserting past the cap evicts the
    least recently used entries (never the one just inserted); `on_evict(key, value)` runs
    for each evicted entry."""

    def __init__(self, cap_bytes: int, on_evict=None):
        self.cap = int(cap_bytes)
        self.on_evict = on_evict
        self._d: "OrderedDict[Any, Tuple[Any, int]]" = OrderedDict()
        self.bytes = 0

    def __len__(self) -> int:
        return len(self._d)

    def __contains__(self, key) -> bool:
        return key in self._d

    def get(self, key):
        hit = self._d.get(key)
        if hit is None:
            return None
        self._d.move_to_end(key)
        return hit[0]

    def put(self, key, value, nbytes: int) -> None:
        if key in self._d:
            self.bytes -= self._d.pop(key)[1]
        self._d[key] = (value, int(nbytes))
        self.bytes += int(nbytes)
        while self.bytes > self.cap and len(self._d) > 1:
            k, (v, nb) = self._d.popitem(last=False)
            self.bytes -= nb
            if self.on_evict is not None:
                self.on_evict(k, v)

    def add_bytes(self, key, nbytes: int) -> None:
        """Charge `nbytes` more to a cached entry (memory allocated for it after insertion),
        evicting least recently used entries past the cap as put() does."""
        hit = self._d.get(key)
        if hit is None:
            return
        self._d[key] = (hit[0], hit[1] + int(nbytes))
        self.bytes += int(nbytes)
        self._d.move_to_end(key)
        while self.bytes > self.cap and len(self._d) > 1:
            k, (v, nb) = self._d.popitem(last=False)
            self.bytes -= nb
            if self.on_evict is not None:
                self.on_evict(k, v)

    def pop(self, key) -> None:
        hit = self._d.pop(key, None)
        if hit is not None:
            self.bytes -= hit[1]

    def keys(self):
        return list(self._d.keys())


HOST_CACHE_BYTES = knob("DG_FEED_CACHE_HOST_MB", 8192) << 20
DEVICE_CACHE_BYTES = knob("DG_FEED_CACHE_DEVICE_MB", 65536) << 20


def _lru(ctx: RunContext, name: str) -> ByteLRU:
    caches = ctx.session.caches
    if name not in caches:
        if name == "dgraph":  # evicting a device graph also evicts the plans built on it
            def drop_plans(key, hit):
                plans = caches.get("plans")
                if plans is not None:
                    for pk in plans.keys():
                        if pk[2] == id(hit[1]):
                            plans.pop(pk)
            caches[name] = ByteLRU(DEVICE_CACHE_BYTES, drop_plans)
        else:
            caches[name] = ByteLRU(DEVICE_CACHE_BYTES if name == "plans" else HOST_CACHE_BYTES)
    return caches[name]


def _freeze(*objs) -> None:
    """Mark fed numpy arrays (and a scipy matrix's arrays) read-only: they are cached by
    identity, so an in-place change must fail instead of silently going stale."""
    for o in objs:
        if sp.issparse(o):
            for a in (getattr(o, "data", None), getattr(o, "indices", None), getattr(o, "indptr", None),
                      getattr(o, "row", None), getattr(o, "col", None)):
                if isinstance(a, np.ndarray):
                    a.flags.writeable = False
        elif isinstance(o, np.ndarray):
            o.flags.writeable = False


def _feed_key(value) -> Tuple:
    """Identity key of a fed sparse value: its (coords, values) objects — a tuple re-built
    each step around the same arrays still hits — or the scipy matrix / SparseTensorValue."""
    if sp.issparse(value):
        return ("sp", id(value)), (value,)
    if isinstance(value, SparseTensorValue):
        return (id(value.indices), id(value.values), tuple(int(x) for x in value.dense_shape)), \
            (value.indices, value.values)
    if isinstance(value, (tuple, list)) and len(value) == 3:
        return (id(value[0]), id(value[1]), tuple(int(x) for x in value[2])), (value[0], value[1])
    raise TypeError(f"cannot feed {type(value).__name__} to a sparse placeholder")


def _csr_bytes(c: Optional[HostCSR]) -> int:
    return 0 if c is None else int(c.rowptr.nbytes + c.col.nbytes + c.val.nbytes)


def host_csr(ctx: RunContext, node: Node) -> HostCSR:
    """CSR of a fed sparse value, cached per session by the identity of what was fed."""
    value = ctx.value(node)
    key, keep = _feed_key(value)
    cache = _lru(ctx, "host_csr")
    hit = cache.get(key)
    if hit is None:
        csr = coo_to_csr(*as_coo_tuple(value))
        _freeze(*keep)
        hit = (keep, csr)  # keep the fed objects referenced: ids stay valid
        cache.put(key, hit, _csr_bytes(csr))
    return hit[1]


def feature_csr(ctx: RunContext, node: Node):
    """None for identity features (X·W ≡ W), else a HostCSR."""
    value = ctx.value(node)
    key, keep = _feed_key(value)
    cache = _lru(ctx, "features")
    hit = cache.get(key)
    if hit is None:
        coo = as_coo_tuple(value)
        csr = None if is_identity(*coo) else coo_to_csr(*coo)
        _freeze(*keep)
        hit = (keep, csr)
        cache.put(key, hit, _csr_bytes(csr))
    return hit[1]


def _device_bytes(dg: DeviceGraph) -> int:
    tot = 0
    for g in dg.groups.values():
        for t in (g.rowptr, g.vcol, g.val, g.rel_map):
            if t is not None:
                tot += t.numel() * t.element_size()
        if g.layout is not None:
            tot += sum(t.numel() * t.element_size() for t in (g.layout.pairs, g.layout.jm, g.layout.jmoff))
    return tot


def device_graph(ctx: RunContext, edge_types: Dict[Tuple[int, int], int],
                 adj_nodes: Dict[Tuple[int, int], Sequence[Node]],
                 local: Optional[Dict] = None, chunk=None, row_block: Optional[Dict] = None) -> DeviceGraph:
    csrs = {et: [host_csr(ctx, n) for n in adj_nodes[et]] for et in edge_types}
    key = ("dgraph", tuple((et, tuple(id(c) for c in csrs[et])) for et in edge_types),
           None if local is None else tuple((et, tuple(v)) for et, v in local.items()), chunk,
           None if not row_block else tuple(sorted(row_block.items())))
    cache = _lru(ctx, "dgraph")
    hit = cache.get(key)
    if hit is None:
        dg = DeviceGraph(edge_types, csrs, ctx.session.device, local, chunk=chunk, row_block=row_block)
        hit = (csrs, dg)  # keep the host CSRs referenced: the key's ids stay valid
        cache.put(key, hit, _device_bytes(dg))
    return hit[1]


def plan_cache(ctx: RunContext) -> ByteLRU:
    """The session's ForwardPlan cache (keys: ("plan", model id, device-graph id, ...))."""
    return _lru(ctx, "plans")


def device_group(ctx: RunContext, nodes: Sequence[Node], chunk: Optional[int] = None) -> DeviceGroup:
    et = (0, 1)  # label only
    g = device_graph(ctx, {et: len(nodes)}, {et: list(nodes)}, chunk=chunk)
    return g.groups[et]


def invalidate(session) -> None:
    session.caches.clear()


# ---------------------------------------------------------------- standalone layer forward
def _conv(grp: DeviceGroup, x: torch.Tensor, d_out: int, per_rel_relu: bool) -> torch.Tensor:
    """l2norm(Σ_k act(Â_k·X_k)) for one group; per-relation relu needs one chunk per
    relation (the epilogue applies it to each chunk partial before the sum)."""
    dev = x.device
    if per_rel_relu and grp.n_chunks != grp.n_rels:
        raise ValueError("per-relation activation needs a one-relation-per-chunk layout")
    part = torch.empty((grp.n_chunks, grp.n_rows, d_out), device=dev, dtype=torch.float32)
    kernels.spmm_groups([kernels.RelGroupSpec(grp.rowptr, grp.vcol, grp.val, x, part, grp.n_rows, grp.n_chunks,
                                              d_out, grp.K * grp.n_cols, vcol_max=grp.vcol_max)], d_out)
    out = torch.empty((grp.n_rows, d_out), device=dev, dtype=torch.float32)
    flags = DG_EPI_L2NORM | (DG_EPI_CHUNK_RELU if per_rel_relu else 0)
    kernels.gcn_epilogue([(part, grp.n_chunks)], out, grp.n_rows, d_out, flags)
    return out


def gcn_layer(grp: DeviceGroup, W: torch.Tensor, feat: Optional[HostCSR], d_out: int,
              per_rel_relu: bool, drop=None) -> torch.Tensor:
    """GraphConvolutionSparseMulti._call (layers.py:85-94) for one edge type.  drop = (keep,
    device state {seed, step}, tag): dropout_sparse (layers.py:23-31, :88) drawn per relation —
    identity features: a row mask on each W_k; sparse features: a mask on X_j's values inside
    the shared-pattern SpMM (the ForwardPlan's masks, dropout.h)."""
    K, F, _ = W.shape
    dev = W.device
    if feat is None:
        if F != grp.n_cols:
            raise ValueError("identity features need one weight row per node")
        x = W
        if drop is not None:
            keep, state, tag = drop
            x = torch.empty_like(W)
            kernels.dropout_rows(W, x, state, tag, keep)
    else:
        x = torch.empty((K, feat.shape[0], d_out), device=dev, dtype=torch.float32)
        if drop is not None:
            keep, state, tag = drop
            spec = kernels.RelGroupSpec(torch.from_numpy(feat.rowptr).to(dev), torch.from_numpy(feat.col).to(dev),
                                        torch.from_numpy(feat.val).to(dev), W, x, feat.shape[0], K, d_out, F,
                                        vcol_max=int(feat.col.max()) if feat.nnz else -1, shared=True,
                                        drop=(state, tag, keep))
        else:
            from .sparse import merge_chunks

            fm = merge_chunks([feat] * K, np.arange(K), 1, K)
            spec = kernels.RelGroupSpec(torch.from_numpy(fm.rowptr).to(dev), torch.from_numpy(fm.vcol).to(dev),
                                        torch.from_numpy(fm.val).to(dev), W, x, feat.shape[0], K, d_out, K * F,
                                        vcol_max=int(fm.vcol.max()) if fm.nnz else -1)
        kernels.spmm_groups([spec], d_out)
    return _conv(grp, x, d_out, per_rel_relu)


def gcn_layer_dense(grp: DeviceGroup, W: torch.Tensor, h: torch.Tensor, d_out: int,
                    per_rel_relu: bool, drop=None) -> torch.Tensor:
    """GraphConvolutionMulti._call (layers.py:109-118) for one edge type.  drop = (keep, device
    state, tag): tf.nn.dropout of the inputs drawn per relation (layers.py:112) — an element mask
    M_k on H for each relation, then H∘M_k/keep · W_k."""
    K, d_in, _ = W.shape
    if h.shape != (grp.n_cols, d_in):
        raise ValueError(f"inputs shape {tuple(h.shape)} != ({grp.n_cols}, {d_in})")
    P = torch.empty((K, grp.n_cols, d_out), device=h.device, dtype=torch.float32)
    a, a_stride = h, 0
    if drop is not None:
        keep, state, tag = drop
        a = torch.empty((K, grp.n_cols, d_in), device=h.device, dtype=torch.float32)
        kernels.dropout_elems(h.contiguous(), a, state, tag, keep)
        a_stride = grp.n_cols * d_in
    kernels.PreparedGemm(a, (a_stride, d_in, 1), W, (d_in * d_out, d_out, 1), P, (grp.n_cols * d_out, d_out, 1),
                         grp.n_cols, d_out, d_in, K)()
    return _conv(grp, P, d_out, per_rel_relu)


# ---------------------------------------------------------------- decoders
def latent_operands(ctx: RunContext, g_kind: str, g_var, l_kind: str, l_var, d: int,
                    g_node: Optional[Node] = None, l_node: Optional[Node] = None):
    """(G dense d×d, l vector or None) for uᵀ·L·G·L·v (model.py:121-134).

    If the caller fed a latent matrix node, that value wins; a fed non-diagonal L is folded
    into G (uᵀ·L·G·L·v = uᵀ·(LGL)·v)."""
    dev = ctx.session.device
    cache = ctx.cache
    if g_node is not None and ctx.is_fed(g_node):
        G = as_device_f32(ctx.value(g_node))
    elif g_kind == "dense":
        G = g_var.tensor
    else:
        key = ("G", g_kind, id(g_var), d)
        if key not in cache:
            cache[key] = (torch.eye(d, device=dev) if g_kind == "eye" else torch.diag(g_var.tensor))
        G = cache[key]
    if l_node is not None and ctx.is_fed(l_node):
        L = np.asarray(ctx.value(l_node), np.float32)
        if np.count_nonzero(L - np.diag(np.diag(L))) == 0:
            return G.contiguous(), as_device_f32(np.diag(L).copy())
        Ld = as_device_f32(L)
        return kernels.matmul(kernels.matmul(Ld, G.contiguous()), Ld), None
    if l_kind == "eye":
        return G.contiguous(), None
    return G.contiguous(), l_var.tensor


def full_scores(rows: torch.Tensor, cols: torch.Tensor, G: torch.Tensor, l: Optional[torch.Tensor]):
    """rows·L·G·L·colsᵀ as two fp32 MFMA GEMMs (optimizer.py:87-106)."""
    T = kernels.matmul(rows, G, sa=l)                    # (rows∘l)·G
    colsT = cols.t()                                     # strided view, no copy
    return kernels.matmul(T, colsT, sa=l)                # ((…)∘l)·colsᵀ


def sigmoid_(x: torch.Tensor) -> torch.Tensor:
    return x.sigmoid_()
