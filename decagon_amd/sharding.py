"""Relation sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference has no parallelism.  The GCN forward shards naturally: every
relation's Â_k·X_k is independent until the per-(i,j) sum Σ_k, which must be complete
before the row L2 normalisation (decagon/deep/layers.py:92-93).  So each rank

  1. owns a subset of the relations of every group (LPT over nonzero counts, or whole
     relation sets — one set per GPU in the weak-scaling bench),
  2. runs the SpMM of its relations and reduces its chunk partials to one
     pre-normalisation sum S_ij per group,
  3. all-reduces the flat buffer of every S_ij (one RCCL all-reduce per layer: 2 per
     forward; the only collective on the data path),
  4. runs the epilogue (normalise, Σ_j, relu) redundantly — every rank ends with the full
     hidden1 / embeddings, which layer 2 and the decoder need.

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

EdgeType = Tuple[int, int]


def lpt_assign(costs: Sequence[float], world_size: int) -> List[int]:
    """Longest-processing-time-first assignment of items to ranks (deterministic: ties by
    item index, then rank)."""
    order = sorted(range(len(costs)), key=lambda i: (-float(costs[i]), i))
    heap = [(0.0, r) for r in range(world_size)]
    owner = [0] * len(costs)
    for i in order:
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + float(costs[i]), r))
    return owner


@dataclass
class RelationShard:
    """This rank's relations per group and the collective that sums group partials."""

    rank: int
    world_size: int
    local: Dict[EdgeType, List[int]]
    allreduce: Optional[Callable[[torch.Tensor], None]] = None
    loads: List[float] = field(default_factory=list)

    @staticmethod
    def lpt(edge_types: Dict[EdgeType, int], rel_cost: Dict[EdgeType, Sequence[float]], rank: int,
            world_size: int, allreduce=None) -> "RelationShard":
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
    def blocks(edge_types_per_rank: Dict[EdgeType, int], rank: int, world_size: int,
               allreduce=None) -> "RelationShard":
        """Weak scaling: the graph holds world_size relation sets; rank r owns set r, i.e.
        relations [r*K_ij, (r+1)*K_ij) of every group."""
        local = {et: list(range(rank * k, (rank + 1) * k)) for et, k in edge_types_per_rank.items()}
        return RelationShard(rank, world_size, local, allreduce)


def torch_allreduce(group=None) -> Callable[[torch.Tensor], None]:
    """Sum-all-reduce over the default (or given) process group — RCCL when the backend is
    'nccl' on ROCm, gloo on CPU tests."""
    import torch.distributed as dist

    def _ar(t: torch.Tensor) -> None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    return _ar
