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

        self.hidden1 = {i: torch.empty((n[i], h1), **f32) for i in self.targets}
        self.embeddings = {i: torch.empty((n[i], h2), **f32) for i in self.targets}

        # ---- layer-2 projection buffers P_k = H1_j·W2_k ----
        self.proj: Dict[EdgeType, torch.Tensor] = {}
        x2_specs = {}
        for et in self.edge_types:
            i, j = et
            grp = dgraph.groups[et]
            K, din, dout = w2.stacks[et].shape
            if din != h1 or dout != h2:
                raise ValueError("layer-2 weight shape != (hidden1, hidden2)")
            if j not in self.hidden1:
                raise ValueError(f"node type {j} has no incoming edge type; layer 2 needs hidden1[{j}]")
            P = torch.empty((max(1, grp.n_rels), n[j], h2), **f32)
            self.proj[et] = P
            x2_specs[et] = (P, n[j] * h2, h2, max(1, grp.n_rels), None)

        # ---- layer 1: Σ_k Â_k·X_k (+ epilogue, + the layer-2 projections of fused rows) ----
        x1_specs = {}
        for et in self.edge_types:
            grp = dgraph.groups[et]
            xt, xs, xld, x_rels = x1[et]
            local_x = features.get(et[1]) is not None
            x1_specs[et] = (xt, xs, xld, x_rels, None if local_x else grp.rel_map)
        fused1 = self._fused_targets(h1, chunk_override, target_waves)
        rels_from = {}
        for et in self.edge_types:
            rels_from[et[1]] = rels_from.get(et[1], 0) + dgraph.groups[et].n_rels
        proj_fused = [et for et in self.edge_types
                      if dgraph.groups[et].n_rels and et[1] in fused1
                      and rels_from[et[1]] <= self.FUSED_PROJ_MAX_RELS]
        if len(proj_fused) > DG_MAX_GROUPS:
            proj_fused = []
        projs = []
        for et in proj_fused:
            grp = dgraph.groups[et]
            projs.append((et[1], kernels.ProjSpec(
                w2.stacks[et], self.proj[et], grp.n_rels, -1, rel_map=grp.rel_map,
                rel_map_max=int(grp.rel_ids.max()) if grp.rel_map is not None else None)))
        self._layer1 = self._build_layer(x1_specs, h1, True, chunk_override, target_waves, f32, projs)

        # ---- layer 2: remaining projections as one batched MFMA GEMM launch, then SpMM ----
        gemms = []
        for et in self.edge_types:
            grp = dgraph.groups[et]
            if not grp.n_rels or et in proj_fused:
                continue
            j = et[1]
            W = w2.stacks[et]
            gemms.append(kernels.PreparedGemm(
                self.hidden1[j], (0, h1, 1), W, (h1 * h2, h2, 1), self.proj[et], (n[j] * h2, h2, 1),
                n[j], h2, h1, grp.n_rels, b_map=grp.rel_map, b_batches=W.shape[0],
                b_map_max=int(grp.rel_ids.max()) if grp.rel_map is not None else None))
        self._gemm2 = [kernels.PreparedGemmMulti(gemms[s:s + DG_MAX_GROUPS])
                       for s in range(0, len(gemms), DG_MAX_GROUPS)]
        self._layer2 = self._build_layer(x2_specs, h2, False, chunk_override, target_waves, f32)

    # a fused launch projects a row onto at most this many layer-2 relations (VALU epilogue);
    # beyond it the batched MFMA GEMM is used
    FUSED_PROJ_MAX_RELS = 64

    def _chunks(self, d, chunk_override, target_waves):
        chunk, nch = {}, {}
        for et in self.edge_types:
            grp = self.g.groups[et]
            c = chunk_override or choose_chunk(grp.n_rels, grp.n_rows, grp.nnz, d, target_waves)
            chunk[et] = max(1, min(c, max(1, grp.n_rels)))
            nch[et] = max(1, -(-grp.n_rels // chunk[et])) if grp.n_rels else 1
        return chunk, nch

    def _fused_targets(self, d, chunk_override, target_waves):
        if self.allreduce is not None:
            return []
        _, nch = self._chunks(d, chunk_override, target_waves)
        return [i for i, ets in self.targets.items()
                if all(nch[et] == 1 and self.g.groups[et].n_rels > 0 for et in ets)]

    # ------------------------------------------------------------------ layer builder
    def _build_layer(self, x_specs, d, relu, chunk_override, target_waves, f32, projs=()):
        """Prepared launches of one layer.  Per node type i: if every group (i, j) fits one
        chunk and no cross-rank sum is needed, the whole target runs in the fused kernel
        (SpMM + l2norm + Σ_j + relu, one launch for all such targets); otherwise its groups
        run in partial mode (chunked sums) followed by the epilogue — with, when sharded,
        the chunk reduce into the all-reduce buffer and the all-reduce before it."""
        g = self.g
        n = g.n_nodes
        outs = self.hidden1 if relu else self.embeddings
        chunk, nch = self._chunks(d, chunk_override, target_waves)

        def spec(et, out, ch):
            grp = g.groups[et]
            xt, xs, xld, x_rels, rmap = x_specs[et]
            return kernels.RelGroupSpec(
                grp.rowptr, grp.col, grp.val, xt, out, grp.n_rows, grp.n_cols, grp.n_rels, ch, xs, xld,
                grp.n_rows, rel_map=rmap, x_rels=x_rels,
                rel_map_max=int(grp.rel_ids.max()) if rmap is not None else None)

        fused_t = self._fused_targets(d, chunk_override, target_waves)
        launches: List[Callable[[], None]] = []
        if fused_t:
            # waves per group: one batch of 64 nonzeros per wave for the densest row group
            avg = max(g.groups[et].nnz / max(1, g.groups[et].n_rows) for i in fused_t for et in self.targets[i])
            max_groups = max(len(self.targets[i]) for i in fused_t)
            wpg = int(max(1, min(4, 16 // max_groups, math.ceil(avg / 64.0))))
            pspecs = []
            for tgt_node, pj in projs:
                pj.target = fused_t.index(tgt_node)
                pspecs.append(pj)
            launches.append(kernels.PreparedFused(
                [(outs[i], n[i], [spec(et, None, max(1, g.groups[et].n_rels)) for et in self.targets[i]], relu)
                 for i in fused_t], d, pspecs, wpg))
        rest = [et for et in self.edge_types if et[0] not in fused_t]
        flags = DG_EPI_L2NORM | (DG_EPI_RELU if relu else 0)
        flat, views = None, {}
        if self.allreduce is not None and rest:
            sizes = [g.groups[et].n_rows * d for et in rest]
            flat = torch.zeros(int(sum(sizes)), **f32)
            off = 0
            for et, sz in zip(rest, sizes):
                views[et] = flat[off:off + sz]
                off += sz
        partials, specs, reduces = {}, [], []
        for et in rest:
            grp = g.groups[et]
            if flat is not None and nch[et] == 1:
                part = views[et]  # single chunk: the SpMM writes the group sum in place
            else:
                part = torch.zeros((nch[et], grp.n_rows, d), **f32)
                if flat is not None and grp.n_rels:
                    reduces.append(kernels.PreparedEpilogue([(part, nch[et])], views[et], grp.n_rows, d, 0))
            partials[et] = (part, nch[et])
            if grp.n_rels:
                specs.append(spec(et, part, chunk[et]))
        launches += [kernels.PreparedSpmm(specs[s:s + DG_MAX_GROUPS], d)
                     for s in range(0, len(specs), DG_MAX_GROUPS)]
        launches += reduces
        need_zero = flat is not None and any(g.groups[et].n_rels == 0 for et in rest)
        epis = []
        for i in self.targets:
            if i in fused_t:
                continue
            src = [(views[et], 1) if flat is not None else partials[et] for et in self.targets[i]]
            epis.append(kernels.PreparedEpilogue(src, outs[i], n[i], d, flags))
        return _Layer(launches, flat, need_zero, self.allreduce, epis, chunk, nch, fused_t)

    def run_layer1(self) -> None:
        for p in self._pre:
            p()
        self._layer1.run()

    def run_layer2(self) -> None:
        for gm in self._gemm2:
            gm()
        self._layer2.run()

    def run(self) -> None:
        self.run_layer1()
        self.run_layer2()

    @property
    def spmm_launches(self):
        """(layer-1, layer-2) SpMM launches (fused or partial) — what the roofline times."""
        pick = lambda L: [l for l in L.launches if isinstance(l, (kernels.PreparedSpmm, kernels.PreparedFused))]
        return pick(self._layer1), pick(self._layer2)

    # ---- accounting (bench / DESIGN.md roofline) ----
    def layer_bytes(self, layer: int) -> int:
        """Algorithmic (compulsory) HBM bytes of one layer's SpMM launches: every CSR array
        once (rowptr 4 B per row per relation, col+val 8 B per nonzero), every distinct
        dense operand X_k once (4·d B per row of X_k), and the output once — 4·d B per row
        per chunk partial in partial mode, per output row in fused mode."""
        L = self._layer1 if layer == 1 else self._layer2
        d = self.h1 if layer == 1 else self.h2
        tot = 0
        for et, grp in self.g.groups.items():
            if not grp.n_rels:
                continue
            tot += 4 * (grp.n_rels * grp.n_rows + 1) + 8 * grp.nnz
            tot += 4 * d * grp.n_cols * grp.n_rels
            if et[0] not in L.fused_targets:
                tot += 4 * d * grp.n_rows * L.n_chunks[et]
        for i in L.fused_targets:
            tot += 4 * d * self.g.n_nodes[i]
        return tot


class _Layer:
    """The prepared launches of one layer and how to run them."""

    def __init__(self, launches, flat, need_zero, allreduce, epilogues, chunk, n_chunks, fused_targets):
        self.launches = launches
        self.flat = flat
        self.need_zero = need_zero
        self.allreduce = allreduce
        self.epilogues = epilogues
        self.chunk = chunk
        self.n_chunks = n_chunks
        self.fused_targets = fused_targets

    def run(self) -> None:
        if self.need_zero:
            self.flat.zero_()  # groups without local relations contribute zeros
        for l in self.launches:
            l()
        if self.flat is not None:
            self.allreduce(self.flat)
        for e in self.epilogues:
            e()
