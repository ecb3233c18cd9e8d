"""Session-side plumbing shared by layers, model and optimizer: parameter placement,
variable scopes, feed → device conversion with caching, and the standalone (single edge
type) layer forward.

Feed caching.  The reference re-feeds every adjacency tuple on every step
(minibatch.py:259-267).  A session caches the device copy of a fed sparse value keyed by the
identity of its numpy arrays (and keeps those arrays referenced, so the key cannot be
recycled); re-feeding the same tuples — what every reference driver does — costs nothing.
Feeds are treated as immutable: mutate a fed array in place and the cached device copy is
stale (call `Session.invalidate_feeds()`, or feed a new array).
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import kernels
from ._lib import DG_EPI_CHUNK_RELU, DG_EPI_L2NORM
from .engine import DeviceGraph, DeviceGroup
from .graph import InvalidArgumentError, Node, RunContext
from .sparse import HostCSR, as_coo_tuple, coo_to_csr, is_identity

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
def _feed_key(value) -> Tuple:
    c, v, s = as_coo_tuple(value)
    return (id(c), id(v), tuple(s)), (c, v, s)


def host_csr(ctx: RunContext, node: Node) -> HostCSR:
    """CSR of a fed sparse value, cached per session by array identity."""
    value = ctx.value(node)
    key, coo = _feed_key(value)
    cache = ctx.session.caches.setdefault("host_csr", {})
    hit = cache.get(key)
    if hit is None:
        hit = (coo, coo_to_csr(*coo))  # keep coo referenced: ids stay valid
        cache[key] = hit
    return hit[1]


def feature_csr(ctx: RunContext, node: Node):
    """None for identity features (X·W ≡ W), else a HostCSR."""
    value = ctx.value(node)
    key, coo = _feed_key(value)
    cache = ctx.session.caches.setdefault("features", {})
    hit = cache.get(key)
    if hit is None:
        hit = (coo, None if is_identity(*coo) else coo_to_csr(*coo))
        cache[key] = hit
    return hit[1]


def device_graph(ctx: RunContext, edge_types: Dict[Tuple[int, int], int],
                 adj_nodes: Dict[Tuple[int, int], Sequence[Node]],
                 local: Optional[Dict] = None, chunk=None, row_block: Optional[Dict] = None) -> DeviceGraph:
    csrs = {et: [host_csr(ctx, n) for n in adj_nodes[et]] for et in edge_types}
    key = ("dgraph", tuple((et, tuple(id(c) for c in csrs[et])) for et in edge_types),
           None if local is None else tuple((et, tuple(v)) for et, v in local.items()), chunk,
           None if not row_block else tuple(sorted(row_block.items())))
    cache = ctx.session.caches.setdefault("dgraph", {})
    hit = cache.get(key)
    if hit is None:
        hit = (csrs, DeviceGraph(edge_types, csrs, ctx.session.device, local, chunk=chunk, row_block=row_block))
        cache[key] = hit
    return hit[1]


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
              per_rel_relu: bool) -> torch.Tensor:
    """GraphConvolutionSparseMulti._call (layers.py:85-94) for one edge type."""
    K, F, _ = W.shape
    if feat is None:
        if F != grp.n_cols:
            raise ValueError("identity features need one weight row per node")
        x = W
    else:
        from .sparse import merge_chunks

        fm = merge_chunks([feat] * K, np.arange(K), 1, K)
        dev = W.device
        x = torch.empty((K, feat.shape[0], d_out), device=dev, dtype=torch.float32)
        kernels.spmm_groups([kernels.RelGroupSpec(
            torch.from_numpy(fm.rowptr).to(dev), torch.from_numpy(fm.vcol).to(dev),
            torch.from_numpy(fm.val).to(dev), W, x, feat.shape[0], K, d_out, K * F,
            vcol_max=int(fm.vcol.max()) if fm.nnz else -1)], d_out)
    return _conv(grp, x, d_out, per_rel_relu)


def gcn_layer_dense(grp: DeviceGroup, W: torch.Tensor, h: torch.Tensor, d_out: int,
                    per_rel_relu: bool) -> torch.Tensor:
    """GraphConvolutionMulti._call (layers.py:109-118) for one edge type."""
    K, d_in, _ = W.shape
    if h.shape != (grp.n_cols, d_in):
        raise ValueError(f"inputs shape {tuple(h.shape)} != ({grp.n_cols}, {d_in})")
    P = torch.empty((K, grp.n_cols, d_out), device=h.device, dtype=torch.float32)
    kernels.PreparedGemm(h, (0, d_in, 1), W, (d_in * d_out, d_out, 1), P, (grp.n_cols * d_out, d_out, 1),
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
