"""Device-resident relation graph and the fused two-layer GCN forward plan.

The reference rebuilds the full-graph forward inside every `sess.run` and re-feeds every
COO adjacency from the host each step (decagon/deep/minibatch.py:259-267, main.py:315).
Here the adjacencies are converted to stacked CSR and uploaded once (`DeviceGraph`), all
buffers are allocated once (`ForwardPlan`), and one forward is a fixed sequence of
launches — capturable into a hipGraph:

  layer 1   [dg_spmm_groups_f32  X_j·W_k for sparse features]          layers.py:89
            dg_spmm_groups_f32   Σ_k Â_k·X_k  over every (i,j) group    layers.py:90-92
            dg_gcn_epilogue_f32  l2norm, Σ_j, relu  per node type       layers.py:93, model.py:75
  layer 2   dg_gemm_f32          P_k = H1_j·W2_k, batched over k         layers.py:113
            dg_spmm_groups_f32   Σ_k Â_k·P_k                             layers.py:114-116
            dg_gcn_epilogue_f32  l2norm, Σ_j  per node type              layers.py:117, model.py:88

With a relation shard (multi-GPU, sharding.py) each rank runs its relations only, reduces
its chunk partials to one pre-normalisation sum per group, all-reduces those sums (RCCL)
and then runs the same epilogue: the normalisation must follow the full Σ_k
(layers.py:92-93).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import kernels
from ._lib import DG_EPI_L2NORM, DG_EPI_RELU, DG_MAX_GROUPS
from .sparse import HostCSR, StackedCSR, stack_relations

EdgeType = Tuple[int, int]


@dataclass
class DeviceGroup:
    """One (i,j) group's relations on the device (stacked CSR, local relation order)."""

    edge_type: EdgeType
    n_rows: int
    n_cols: int
    rel_ids: np.ndarray            # global relation index k of each local relation
    rowptr: torch.Tensor
    col: torch.Tensor
    val: torch.Tensor
    rel_nnz: np.ndarray
    rel_map: Optional[torch.Tensor] = None   # device copy of rel_ids when not 0..K-1

    @property
    def n_rels(self) -> int:
        return int(self.rel_ids.shape[0])

    @property
    def nnz(self) -> int:
        return int(self.col.numel())


class DeviceGraph:
    """Stacked CSR of every (i,j) group, uploaded once.

    `adj[(i,j)]` is the list of the K_ij relations (HostCSR) in k order; `local` optionally
    restricts each group to a subset of its relations (a rank's shard)."""

    def __init__(self, edge_types: Dict[EdgeType, int], adj: Dict[EdgeType, Sequence[HostCSR]],
                 device: torch.device, local: Optional[Dict[EdgeType, Sequence[int]]] = None):
        self.edge_types = dict(edge_types)
        self.device = device
        self.groups: Dict[EdgeType, DeviceGroup] = {}
        self.n_nodes: Dict[int, int] = {}
        for et, K in self.edge_types.items():
            rels = list(adj[et])
            if len(rels) != K:
                raise ValueError(f"edge type {et}: {len(rels)} matrices fed, {K} expected")
            known = [r for r in rels if r is not None]  # non-local relations may be None
            if not known:
                raise ValueError(f"edge type {et}: no relation given")
            n_r, n_c = known[0].shape
            for t, n in ((et[0], n_r), (et[1], n_c)):
                if self.n_nodes.setdefault(t, n) != n:
                    raise ValueError(f"node type {t}: inconsistent sizes {self.n_nodes[t]} vs {n}")
            ids = np.arange(K, dtype=np.int32) if local is None else np.asarray(local[et], np.int32)
            if any(rels[k] is None for k in ids):
                raise ValueError(f"edge type {et}: a local relation was not given")
            if ids.size:
                st = stack_relations([rels[k] for k in ids])
            else:
                st = StackedCSR(np.zeros(1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32),
                                n_r, n_c, 0, np.zeros(0, np.int64))
            g = DeviceGroup(
                et, n_r, n_c, ids,
                torch.from_numpy(st.rowptr).to(device),
                torch.from_numpy(st.col).to(device),
                torch.from_numpy(st.val).to(device),
                st.rel_nnz,
            )
            if ids.size and not np.array_equal(ids, np.arange(K)):
                g.rel_map = torch.from_numpy(ids).to(device)
            self.groups[et] = g

    @property
    def total_nnz(self) -> int:
        return sum(g.nnz for g in self.groups.values())


def choose_chunk(n_rels: int, n_rows: int, nnz: int, d: int, target_waves: int = 32768) -> int:
    """Relations per output chunk.  Partials cost 8·d bytes per (chunk,row) against
    ≈8·nnz_per_row·chunk bytes of CSR reads; keep them under a quarter of it, but keep at
    least `target_waves` waves (one per (chunk,row)) to fill 256 CUs when the group is big."""
    if n_rels <= 1 or n_rows == 0:
        return max(1, n_rels)
    avg = nnz / float(n_rels * n_rows)
    chunk_traffic = max(1, math.ceil(4.0 * d / max(avg, 1e-9)))
    chunk_par = max(1, (n_rels * n_rows) // target_waves)
    chunk = chunk_par if chunk_traffic <= chunk_par else chunk_traffic
    return int(min(max(1, chunk), n_rels))


@dataclass
class LayerWeights:
    """Weight stacks of one layer: per (i,j) group a tensor [K, d_in, d_out] (device)."""

    stacks: Dict[EdgeType, torch.Tensor]


class ForwardPlan:
    """All buffers and prepared launches of one two-layer forward on one device."""

    def __init__(self, dgraph: DeviceGraph, features: Dict[int, Optional[HostCSR]],
                 w1: LayerWeights, w2: LayerWeights, h1: int, h2: int,
                 allreduce: Optional[Callable[[torch.Tensor], None]] = None,
                 chunk_override: Optional[int] = None, target_waves: int = 32768):
        self.g = dgraph
        self.h1, self.h2 = h1, h2
        self.allreduce = allreduce
        dev = dgraph.device
        f32 = dict(device=dev, dtype=torch.float32)
        self.edge_types = list(dgraph.edge_types)
        self.targets: Dict[int, List[EdgeType]] = {}
        for et in self.edge_types:
            self.targets.setdefault(et[0], []).append(et)
        if any(len(v) > DG_MAX_GROUPS for v in self.targets.values()):
            raise ValueError(f"more than {DG_MAX_GROUPS} edge types into one node type")
        n = dgraph.n_nodes

        # ---- feature products X_j·W1_k (only for non-identity features) ----
        self._pre: List[Callable[[], None]] = []
        x1: Dict[EdgeType, Tuple[torch.Tensor, int, int, int]] = {}
        feat_dev: Dict[int, Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = {}
        for et in self.edge_types:
            i, j = et
            grp = dgraph.groups[et]
            W = w1.stacks[et]
            K, F, dh = W.shape
            if dh != h1:
                raise ValueError("layer-1 weight width != hidden1")
            fj = features.get(j)
            if fj is None:  # identity features: X_j·W_k ≡ W_k (bit-exact), no kernel
                if F != n[j]:
                    raise ValueError(f"identity features of type {j} need {n[j]} weight rows, got {F}")
                x1[et] = (W, F * h1, h1, K)
                continue
            if fj.shape[0] != n[j] or fj.shape[1] != F:
                raise ValueError(f"features of type {j} have shape {fj.shape}, weights expect (*, {F})")
            if j not in feat_dev:
                feat_dev[j] = tuple(torch.from_numpy(a).to(dev) for a in (fj.rowptr, fj.col, fj.val))
            rp, cl, vl = feat_dev[j]
            n_loc = grp.n_rels
            xw = torch.empty((max(1, n_loc), n[j], h1), **f32)
            if n_loc:
                spec = kernels.RelGroupSpec(rp, cl, vl, W, xw, n[j], F, n_loc, 1, F * h1, h1, 0,
                                            rel_map=grp.rel_map, x_rels=K,
                                            rel_map_max=int(grp.rel_ids.max()))
                self._pre.append(kernels.PreparedSpmm([spec], h1))
            x1[et] = (xw, n[j] * h1, h1, n_loc)  # local order already applied

        # ---- layer 1 SpMM ----
        self.partial1: Dict[EdgeType, Tuple[torch.Tensor, int]] = {}
        specs1 = []
        for et in self.edge_types:
            grp = dgraph.groups[et]
            xt, xs, xld, x_rels = x1[et]
            local_x = features.get(et[1]) is not None
            ch = chunk_override or choose_chunk(grp.n_rels, grp.n_rows, grp.nnz, h1, target_waves)
            nch = max(1, -(-grp.n_rels // ch)) if grp.n_rels else 1
            part = torch.zeros((nch, grp.n_rows, h1), **f32)
            self.partial1[et] = (part, nch)
            if grp.n_rels:
                specs1.append(kernels.RelGroupSpec(
                    grp.rowptr, grp.col, grp.val, xt, part, grp.n_rows, grp.n_cols, grp.n_rels, ch,
                    xs, xld, grp.n_rows,
                    rel_map=None if local_x else grp.rel_map, x_rels=x_rels,
                    rel_map_max=None if (local_x or grp.rel_map is None) else int(grp.rel_ids.max())))
        self._spmm1 = [kernels.PreparedSpmm(specs1[s:s + DG_MAX_GROUPS], h1)
                       for s in range(0, len(specs1), DG_MAX_GROUPS)]

        # ---- layer 2 projection + SpMM ----
        self.proj: Dict[EdgeType, torch.Tensor] = {}
        self.partial2: Dict[EdgeType, Tuple[torch.Tensor, int]] = {}
        self.hidden1 = {i: torch.empty((n[i], h1), **f32) for i in self.targets}
        self.embeddings = {i: torch.empty((n[i], h2), **f32) for i in self.targets}
        self._gemm2 = []
        specs2 = []
        for et in self.edge_types:
            i, j = et
            grp = dgraph.groups[et]
            W = w2.stacks[et]
            K, din, dout = W.shape
            if din != h1 or dout != h2:
                raise ValueError("layer-2 weight shape != (hidden1, hidden2)")
            if j not in self.hidden1:
                raise ValueError(f"node type {j} has no incoming edge type; layer 2 needs hidden1[{j}]")
            P = torch.empty((max(1, grp.n_rels), n[j], h2), **f32)
            self.proj[et] = P
            ch = chunk_override or choose_chunk(grp.n_rels, grp.n_rows, grp.nnz, h2, target_waves)
            nch = max(1, -(-grp.n_rels // ch)) if grp.n_rels else 1
            part = torch.zeros((nch, grp.n_rows, h2), **f32)
            self.partial2[et] = (part, nch)
            if not grp.n_rels:
                continue
            H = self.hidden1[j]
            self._gemm2.append(kernels.PreparedGemm(
                H, (0, h1, 1), W, (h1 * h2, h2, 1), P, (n[j] * h2, h2, 1),
                n[j], h2, h1, grp.n_rels, b_map=grp.rel_map, b_batches=K,
                b_map_max=int(grp.rel_ids.max()) if grp.rel_map is not None else None))
            specs2.append(kernels.RelGroupSpec(
                grp.rowptr, grp.col, grp.val, P, part, grp.n_rows, grp.n_cols, grp.n_rels, ch,
                n[j] * h2, h2, grp.n_rows))
        self._spmm2 = [kernels.PreparedSpmm(specs2[s:s + DG_MAX_GROUPS], h2)
                       for s in range(0, len(specs2), DG_MAX_GROUPS)]

        # ---- epilogues (and the cross-rank sum when sharded) ----
        self._epi1 = self._make_epilogue(self.partial1, self.hidden1, h1, DG_EPI_L2NORM | DG_EPI_RELU, f32)
        self._epi2 = self._make_epilogue(self.partial2, self.embeddings, h2, DG_EPI_L2NORM, f32)

    def _make_epilogue(self, partials, outs, d, flags, f32):
        """Returns (reduce_launches, flat_sum_buffer or None, epilogue_launches)."""
        n = self.g.n_nodes
        if self.allreduce is None:
            epis = [kernels.PreparedEpilogue([partials[et] for et in self.targets[i]], outs[i], n[i], d, flags)
                    for i in self.targets]
            return [], None, epis
        # sharded: per-group chunk reduce into one flat buffer, all-reduce, then epilogue
        sizes = [self.g.groups[et].n_rows * d for et in self.edge_types]
        flat = torch.zeros(int(sum(sizes)), **f32)
        views, off = {}, 0
        for et, sz in zip(self.edge_types, sizes):
            views[et] = flat[off:off + sz]
            off += sz
        reds = []
        for et in self.edge_types:
            if self.g.groups[et].n_rels:
                reds.append(kernels.PreparedEpilogue([partials[et]], views[et], self.g.groups[et].n_rows, d, 0))
        epis = [kernels.PreparedEpilogue([(views[et], 1) for et in self.targets[i]], outs[i], n[i], d, flags)
                for i in self.targets]
        return reds, flat, epis

    def _run_epilogue(self, epi) -> None:
        reds, flat, epis = epi
        if flat is not None:
            if len(reds) < len(self.edge_types):
                flat.zero_()  # groups without local relations contribute zeros
            for r in reds:
                r()
            self.allreduce(flat)
        for e in epis:
            e()

    def run_layer1(self) -> None:
        for p in self._pre:
            p()
        for s in self._spmm1:
            s()
        self._run_epilogue(self._epi1)

    def run_layer2(self) -> None:
        for gm in self._gemm2:
            gm()
        for s in self._spmm2:
            s()
        self._run_epilogue(self._epi2)

    def run(self) -> None:
        self.run_layer1()
        self.run_layer2()

    # ---- accounting (bench / DESIGN.md roofline) ----
    def layer_bytes(self, layer: int) -> int:
        """Algorithmic (compulsory) HBM bytes of one layer's SpMM launch: every CSR array
        once (rowptr 4 B/row/relation, col+val 8 B/nonzero), every distinct dense operand
        X_k once (4·d B per row), every partial written once (4·d B per row)."""
        d = self.h1 if layer == 1 else self.h2
        parts = self.partial1 if layer == 1 else self.partial2
        tot = 0
        for et, grp in self.g.groups.items():
            if not grp.n_rels:
                continue
            tot += 4 * (grp.n_rels * grp.n_rows + 1) + 8 * grp.nnz
            tot += 4 * d * grp.n_cols * grp.n_rels
            tot += 4 * d * grp.n_rows * parts[et][1]
        return tot
