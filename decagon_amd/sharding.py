"""Sharding the GCN forward across GPUs (one process per GPU, torch.distributed over
RCCL/xGMI).

The reference has no parallelism.  Every relation's Â_k·X_k is independent
until the per-(i,j) sum Σ_k, which must be complete before the row L2 normalisation
(decagon/deep/layers.py:92-93); after it, the layer's rows are independent.  Two ways to
split a node type's work follow from that, and a plan uses both:

  relation-sharded  (small node types: the 645 drugs)
      each rank owns a subset of the relations of every group into the node type (LPT over
      nonzero counts), writes
      its partial pre-normalisation sums S_ij into one flat buffer and the ranks all-reduce
      it (one RCCL all-reduce per layer); every rank then finishes those rows redundantly.
  row-split         (node types of >= ROW_SPLIT_MIN rows: the 19,085 proteins)
      each rank owns a contiguous block of the node type's rows for EVERY relation into it,
      so its S_ij rows are complete locally: it normalises and finishes its block, and the
      blocks are all-gathered (padded to equal size) into the full hidden1 / embeddings that
      the next layer's gathers and the decoder read.  Config S's weak scaling (N relation
      sets over the same nodes) row-splits every node type (RelationShard.weak_sets).

Per layer the exchange is therefore one all-reduce of the relation-sharded node types' sums
(config P: 2 × 645 × d floats) plus one all-gather of the row-split node types' finished
rows (19,085 × d floats in total) — not an all-reduce of the proteins' 2 × 19,085 × d sums,
which bounded round 1's relation-only sharding at ≈3× on 8 GPUs.

Weights are replicated (the largest stack, polypharmacy W1 of (1,1), is 318 MB — small
against 288 GB of HBM); kernels pick a rank's relations out of the full stack through the
relation map of dg_rel_group / dg_gemm_desc, without copies.
"""
from __future__ import annotations

import heapq
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from .tuning import knob

EdgeType = Tuple[int, int]

# node types with at least this many rows are row-split across ranks (the others are
# relation-sharded); config P's proteins (19,085) are, its drugs (645) and config S are not
ROW_SPLIT_MIN = 4096


def lpt_assign(costs: Sequence[float], world_size: int, start: Optional[Sequence[float]] = None) -> List[int]:
    """Longest-processing-time-first assignment of items to ranks (deterministic: ties by
    item index, then rank); `start` = each rank's load before the items."""
    order = sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i))
    heap = [(0.0 if start is None else float(start[r]), r) for r in range(world_size)]
    heapq.heapify(heap)
    owner = [0] * len(costs)
    for i in order:
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + float(costs[i]), r))
    return owner


# config P's relation dealing: a relation of a group that is not staged (the drug-target group,
# one relation) costs the rank holding it a launch tail beyond its nonzeros — measured 2.7-3.2 us a
# step on that rank at N = 8 (round 6) — charged in nonzeros of staged work, so LPT gives that
# rank fewer drug x drug relations
GROUP_TAIL = knob("DG_SHARD_GROUP_TAIL", 0)
# ... or such a group (fewer relations than ranks, not staged) dealt by output rows over every
# rank (RelationShard.dealt), so no rank carries its whole launch tail.  Off: config P at N = 8
# measured 98.4 / 96.7 µs max against 97.2 / 97.7 — every rank then pays the relation's row-chain
# tail (93.8-95.6 → 96.0-97.4), which is latency, not row count (round 6)
DEAL_ROWS = knob("DG_SHARD_DEAL_ROWS", False)


def row_block(n_rows: int, rank: int, world_size: int) -> Tuple[int, int, int]:
    """(first row, end row, padded block size) of `rank`'s block of a row-split node type:
    equal blocks of ceil(n / world) rows (the last one short), so the all-gather moves
    equal-sized pieces."""
    blk = -(-n_rows // world_size)
    a = min(n_rows, rank * blk)
    return a, min(n_rows, a + blk), blk


def slot_range(n_slots: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous, balanced block of relation slots of `rank` (config 5's scorer)."""
    base, extra = divmod(n_slots, world_size)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


@dataclass
class RelationShard:
    """This rank's share of the forward: the local relations of every group, the row blocks
    of the row-split node types, and the collectives that join the shares."""

    rank: int
    world_size: int
    local: Dict[EdgeType, List[int]]
    allreduce: Optional[Callable[..., None]] = None  # allreduce(t) in place, allreduce(t, out)
    loads: List[float] = field(default_factory=list)
    # node type -> (first row, end row, padded block) of this rank (row-split node types)
    row_block: Dict[int, Tuple[int, int, int]] = field(default_factory=dict)
    # allgather(out [world * blk, d], inp = out[rank * blk:(rank + 1) * blk]) — in place
    allgather: Optional[Callable[[torch.Tensor, torch.Tensor], None]] = None
    scheme: str = "relations LPT-sharded"  # how the relations were dealt (describe())
    # relations per chunk the plan should use per edge type (None: the plan's policy) — a
    # row-split plan whose blocks the fused kernel finishes needs one chunk per group
    chunks: Optional[Dict[EdgeType, int]] = None
    # row-split node types finished by the fused SpMM kernel over their row block (one chunk
    # per group; config S's weak scaling) instead of partial mode + an epilogue
    fused_rows: bool = False
    # row-split node types in dg_spmm_seg_f32 + the epilogue, layer 2 reassociated (config S's
    # weak scaling at N GPUs; `chunks` then holds the relations per set)
    seg_rows: bool = False
    # relation-sharded groups of fewer relations than ranks dealt by ROWS instead (split's
    # deal_rows): every rank holds each of their relations over its block [a, b) of output rows,
    # the other rows emptied (same shape; the all-reduce adds the blocks) — edge type -> (a, b)
    dealt: Dict[EdgeType, Tuple[int, int]] = field(default_factory=dict)
    # the row-split blocks exchanged by peer stores over xGMI instead of `allgather`
    # (peer.PeerConfig: the finishing launch pushes its rows and ends with the exchange, or a
    # stand-alone exchange launch); the all-reduce of relation-sharded sums stays `allreduce`
    peer: Optional[object] = None

    @staticmethod
    def lpt(edge_types: Dict[EdgeType, int], rel_cost: Dict[EdgeType, Sequence[float]], rank: int,
            world_size: int, allreduce=None) -> "RelationShard":
        """Every relation whole to one rank, LPT over its cost (no row split)."""
        items = [(et, k) for et in edge_types for k in range(edge_types[et])]
        costs = [float(rel_cost[et][k]) for et, k in items]
        owner = lpt_assign(costs, world_size)
        local: Dict[EdgeType, List[int]] = {et: [] for et in edge_types}
        loads = [0.0] * world_size
        for (et, k), r, c in zip(items, owner, costs):
            loads[r] += c
            if r == rank:
                local[et].append(k)
        return RelationShard(rank, world_size, local, allreduce, loads)

    @staticmethod
    def split(edge_types: Dict[EdgeType, int], n_nodes: Dict[int, int], rel_cost: Dict[EdgeType, Sequence[float]],
              rank: int, world_size: int, allreduce=None, allgather=None,
              row_split_min: int = ROW_SPLIT_MIN, deal_rows=()) -> "RelationShard":
        """Row-split the node types of >= row_split_min rows (every rank keeps all relations
        of the groups into them, on its row block); LPT the relations of the groups into the
        other node types, starting from the row-split work each rank already holds.  Groups in
        `deal_rows` (relation-sharded ones) are dealt by output rows instead: every rank holds
        all their relations over its row block (`dealt`)."""
        # (every rank must own at least one row of a row-split node type)
        rows = {t for t, n in n_nodes.items()
                if n >= row_split_min and (world_size - 1) * -(-n // world_size) < n}
        blocks = {t: row_block(n_nodes[t], rank, world_size) for t in rows}
        local: Dict[EdgeType, List[int]] = {}
        items, costs = [], []
        base = [0.0] * world_size
        dealt = {}
        for et, K in edge_types.items():
            if et[0] in rows or et in deal_rows:
                local[et] = list(range(K))
                share = sum(float(c) for c in rel_cost[et]) / world_size
                base = [b + share for b in base]
                if et[0] not in rows:
                    dealt[et] = row_block(n_nodes[et[0]], rank, world_size)[:2]
            else:
                local[et] = []
                for k in range(K):
                    items.append((et, k))
                    costs.append(float(rel_cost[et][k]))
        owner = lpt_assign(costs, world_size, base)
        loads = list(base)
        for (et, k), r, c in zip(items, owner, costs):
            loads[r] += c
            if r == rank:
                local[et].append(k)
        return RelationShard(rank, world_size, local, allreduce, loads, blocks, allgather, dealt=dealt)

    @staticmethod
    def polypharmacy(graph, rank: int, world_size: int, comm: bool = True, collectives=None) -> "RelationShard":
        """Config P's shard: proteins row-split, drug-target relations LPT on nonzeros.
        comm=False: no collectives (a one-GPU timing rehearsal of one rank's share);
        collectives = (allreduce, allgather) to use instead of torch.distributed's (the RCCL
        communicator of rccl.py for captured steps)."""
        from .engine import STAGED_REL_OVERHEAD, stageable

        # LPT cost of a relation: its nonzeros, + the staged kernel's per-relation overhead for a
        # staged group's, + GROUP_TAIL for any other group's (the latency tail its launch adds on
        # the rank that holds it)
        nnz, deal = {}, []
        for et, rels in graph.adj.items():
            n_r, n_c = graph.n_nodes[et[0]], graph.n_nodes[et[1]]
            staged = stageable(len(rels), n_r, n_c)
            extra = STAGED_REL_OVERHEAD if staged else GROUP_TAIL
            nnz[et] = [len(c[1]) + extra for c in rels]
            if DEAL_ROWS and not staged and len(rels) < world_size and n_r >= world_size:
                deal.append(et)  # (the drug-target relation: its rows over every rank)
        if not comm:
            ar, ag = _no_op_reduce, _no_op
        elif collectives is not None:
            ar, ag = collectives
        else:
            ar, ag = torch_allreduce(), torch_allgather()
        return RelationShard.split(graph.edge_types, graph.n_nodes, nnz, rank, world_size, ar, ag, deal_rows=deal)

    @staticmethod
    def weak_sets(edge_types: Dict[EdgeType, int], n_nodes: Dict[int, int], rank: int, world_size: int,
                  allreduce=None, allgather=None, form: Optional[str] = None) -> "RelationShard":
        """Config S's weak scaling (synthetic.replicate_sets): the graph holds world_size relation
        sets over the same nodes, set r at relations [r·K, (r+1)·K) of every group (K = the
        group's relations per set).  Every node type is row-split: each rank finishes its row
        block over every set's relations and the blocks are all-gathered — no all-reduce.
        form "seg" (default; DG_S_ROWS_FORM overrides): one chunk per relation set, the blocks in
        dg_spmm_seg_f32 (one wave per (row, relation), layer 2 reassociated so no rank projects
        every relation) + the epilogue; "fused": one chunk per group in dg_gcn_fused_f32 (one
        workgroup per row) with the layer-2 projection GEMM over every relation on every rank."""
        form = form or knob("DG_S_ROWS_FORM", "seg")
        if form not in ("seg", "fused"):
            raise ValueError(f"unknown weak-scaling form {form!r}")
        nnz = {et: [1.0] * K for et, K in edge_types.items()}
        sh = RelationShard.split(edge_types, n_nodes, nnz, rank, world_size, allreduce, allgather, row_split_min=1)
        if form == "seg":
            if any(K % world_size for K in edge_types.values()):
                raise ValueError("every group must hold world_size relation sets")
            # one relation set per chunk (two sets a chunk — half the partials a row's epilogue
            # adds, twice the waves a workgroup — measured the same: 24.35 vs 24.38 µs at N = 8)
            sh.chunks = {et: K // world_size for et, K in edge_types.items()}
            sh.seg_rows = True
        else:
            sh.chunks = dict(edge_types)
            sh.fused_rows = True
        sh.scheme = "one relation set per GPU"
        return sh

    def local_csr(self, csr: Dict[EdgeType, Sequence]) -> Dict[EdgeType, list]:
        """The graph's per-group relation lists with the relations of other ranks replaced by
        empty stand-ins of the same shape (never uploaded; they only carry the group's shape
        when this rank owns none of its relations), and a row-dealt group's relations cut to
        this rank's rows."""
        from .sparse import HostCSR

        def empty(c):
            return HostCSR(np.zeros(c.shape[0] + 1, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32),
                           tuple(c.shape))

        def rows(c, ab):  # rows [a, b) of c, the others emptied (same shape)
            a, b = ab
            rp = c.rowptr.astype(np.int64)
            p0, p1 = int(rp[a]), int(rp[b])
            return HostCSR((np.clip(rp, p0, p1) - p0).astype(np.int32), c.col[p0:p1], c.val[p0:p1], tuple(c.shape))

        out = {}
        for et, v in csr.items():
            mine = set(self.local[et])
            out[et] = [(rows(c, self.dealt[et]) if et in self.dealt else c) if k in mine else empty(c)
                       for k, c in enumerate(v)]
        return out

    def describe(self, backend: str = "nccl") -> str:
        lib = "RCCL" if backend == "nccl" else backend
        rs = ", ".join(f"node type {t} row-split" for t in sorted(self.row_block))
        shared = any(t not in self.row_block for et in self.local for t in [et[0]])
        if self.row_block and not shared:
            return f"x{self.world_size}: every node type row-split; {lib} all-gather of the finished rows per layer"
        return (f"x{self.world_size}: {self.scheme}" + (f", {rs}" if rs else "")
                + f"; {lib} all-reduce of the relation-sharded sums"
                + (" + all-gather of the row-split rows" if rs else "") + " per layer")


def _no_op(*_a) -> None:
    return None


def _no_op_reduce(t: torch.Tensor, out: Optional[torch.Tensor] = None) -> None:
    """The all-reduce of a one-rank timing rehearsal: out = t (the data path stays valid)."""
    if out is not None and out is not t:
        out.copy_(t)


def torch_allreduce(group=None) -> Callable[[torch.Tensor], None]:
    """Sum-all-reduce over the default (or given) process group — RCCL when the backend is
    'nccl' on ROCm, gloo on CPU tests."""
    import torch.distributed as dist

    def _ar(t: torch.Tensor, out: Optional[torch.Tensor] = None) -> None:
        """Sum over the ranks, in place, or into `out` (t unchanged)."""
        if out is not None and out is not t:
            out.copy_(t)
            t = out
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    return _ar


def torch_allgather(group=None) -> Callable[[torch.Tensor, torch.Tensor], None]:
    """In-place all-gather of equal row blocks: `inp` is this rank's block of `out`."""
    import torch.distributed as dist

    def _ag(out: torch.Tensor, inp: torch.Tensor) -> None:
        if out.is_cuda and dist.get_backend(group) == "gloo":
            # gloo (CPU tests, one-GPU multi-rank rehearsals): staged through host memory
            off = (inp.data_ptr() - out.data_ptr()) // out.element_size()
            flat = out.reshape(-1).cpu()
            dist.all_gather_into_tensor(flat, flat[off:off + inp.numel()].clone(), group=group)
            out.copy_(flat.view_as(out))
            return
        dist.all_gather_into_tensor(out, inp, group=group)

    return _ag
