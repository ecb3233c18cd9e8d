"""DecagonModel with the reference's constructor and attributes (decagon/deep/model.py).

Construction mirrors `_build` (model.py:64-137): the same layer objects (for variable
layout and names), the same `hidden1` / `embeddings` / `latent_inters` / `latent_varies`
attributes in the same edge-type order.  Evaluation differs: every layer of every edge type
runs through one fused ForwardPlan (engine.py) per uploaded graph — five to six HIP
launches per forward instead of one TF op per relation.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch

from . import runtime
from .engine import ForwardPlan, LayerWeights
from .flags import FLAGS
from .graph import Node, RunContext
from .layers import (BilinearDecoder, DEDICOMDecoder, DistMultDecoder, GraphConvolutionMulti,
                     GraphConvolutionSparseMulti, InnerProductDecoder, act_kind)


class Model:
    """model.py:12-44."""

    def __init__(self, **kwargs):
        allowed_kwargs = {"name", "logging"}
        for kwarg in kwargs.keys():
            assert kwarg in allowed_kwargs, "Invalid keyword argument: " + kwarg
        name = kwargs.get("name")
        if not name:
            name = self.__class__.__name__.lower()
        self.name = name
        self.logging = kwargs.get("logging", False)
        self.vars = {}

    def _build(self):
        raise NotImplementedError

    def build(self):
        with runtime.variable_scope(self.name):
            self._build()
        self.vars = {v.name: v for v in self._variables()}

    def _variables(self):
        return []

    def fit(self):
        pass

    def predict(self):
        pass


class _LatentNode(Node):
    """One entry of latent_inters / latent_varies: I, diag(vector) or a dense variable."""

    def __init__(self, name: str, kind: str, var, d: int):
        super().__init__(name)
        self.kind, self.var, self.d = kind, var, d

    def _compute(self, ctx: RunContext):
        dev = ctx.session.device
        if self.kind == "eye":
            return torch.eye(self.d, device=dev)
        if self.kind == "diag":
            return torch.diag(self.var.tensor)
        return self.var.tensor


class DecagonModel(Model):
    """model.py:47-137."""

    def __init__(self, placeholders, num_feat, nonzero_feat, edge_types, decoders, **kwargs):
        super().__init__(**kwargs)
        self.edge_types = edge_types
        self.num_edge_types = sum(self.edge_types.values())
        self.num_obj_types = max([i for i, _ in self.edge_types]) + 1
        self.decoders = decoders
        self.inputs = {i: placeholders["feat_%d" % i] for i, _ in self.edge_types}
        self.input_dim = num_feat
        self.nonzero_feat = nonzero_feat
        self.placeholders = placeholders
        self.dropout = placeholders["dropout"]
        self.adj_mats = {et: [placeholders["adj_mats_%d,%d,%d" % (et[0], et[1], k)] for k in range(n)]
                         for et, n in self.edge_types.items()}
        self.build()

    def _build(self):
        h1, h2 = int(FLAGS.hidden1), int(FLAGS.hidden2)
        self.h1, self.h2 = h1, h2
        self.layers1: Dict[Tuple[int, int], GraphConvolutionSparseMulti] = {}
        self.layers2: Dict[Tuple[int, int], GraphConvolutionMulti] = {}
        ident = lambda x: x  # noqa: E731  (model.py:71, :83)
        for i, j in self.edge_types:
            self.layers1[i, j] = GraphConvolutionSparseMulti(
                input_dim=self.input_dim, output_dim=h1, edge_type=(i, j),
                num_types=self.edge_types[i, j], adj_mats=self.adj_mats,
                nonzero_feat=self.nonzero_feat, act=ident, dropout=self.dropout,
                logging=self.logging)
        self.hidden1 = {}
        for i in dict.fromkeys(i for i, _ in self.edge_types):
            self.hidden1[i] = Node(f"{self.name}/hidden1_{i}",
                                   lambda ctx, i=i: self._forward(ctx).hidden1[i])
            self.hidden1[i].model = self
        for i, j in self.edge_types:
            self.layers2[i, j] = GraphConvolutionMulti(
                input_dim=h1, output_dim=h2, edge_type=(i, j),
                num_types=self.edge_types[i, j], adj_mats=self.adj_mats, act=ident,
                dropout=self.dropout, logging=self.logging)
        self.embeddings = [None] * self.num_obj_types
        for i in dict.fromkeys(i for i, _ in self.edge_types):
            self.embeddings[i] = Node(f"{self.name}/embeddings_{i}",
                                      lambda ctx, i=i: self._forward(ctx).embeddings[i])
            self.embeddings[i].model = self  # the optimizer's training step finds the model here

        self.edge_type2decoder = {}
        for i, j in self.edge_types:
            decoder = self.decoders[i, j]
            kw = dict(input_dim=h2, logging=self.logging, edge_type=(i, j),
                      num_types=self.edge_types[i, j], act=ident, dropout=self.dropout)
            if decoder == "innerproduct":
                self.edge_type2decoder[i, j] = InnerProductDecoder(**kw)
            elif decoder == "distmult":
                self.edge_type2decoder[i, j] = DistMultDecoder(**kw)
            elif decoder == "bilinear":
                self.edge_type2decoder[i, j] = BilinearDecoder(**kw)
            elif decoder == "dedicom":
                self.edge_type2decoder[i, j] = DEDICOMDecoder(**kw)
            else:
                raise ValueError("Unknown decoder type")

        self.latent_inters: List[_LatentNode] = []
        self.latent_varies: List[_LatentNode] = []
        self._latent_spec = []
        for edge_type in self.edge_types:
            dec = self.edge_type2decoder[edge_type]
            for k in range(self.edge_types[edge_type]):
                gk, gv, lk, lv = dec.latent(k)
                r = len(self.latent_inters)
                self.latent_inters.append(_LatentNode(f"{self.name}/latent_inter_{r}", gk, gv, h2))
                self.latent_varies.append(_LatentNode(f"{self.name}/latent_vary_{r}", lk, lv, h2))
                self._latent_spec.append((gk, gv, lk, lv))

    def _variables(self):
        out = []
        for lay in list(self.layers1.values()) + list(self.layers2.values()) + \
                list(self.edge_type2decoder.values()):
            out.extend(lay.vars.values())
        return out

    # ------------------------------------------------------------------ evaluation
    def weight_stacks(self):
        return (LayerWeights({et: l.weights_stack for et, l in self.layers1.items()}),
                LayerWeights({et: l.weights_stack for et, l in self.layers2.items()}))

    # the counter-based dropout masks (dropout.hip) of this model start from this seed
    dropout_seed = 20180701

    def dropout_state(self, ctx: RunContext) -> torch.Tensor:
        """The device dropout state {seed, step} of this model in the session (step = the
        number of forwards run with dropout so far)."""
        key = ("dropout_state", id(self))
        cache = ctx.session.caches
        if key not in cache:
            cache[key] = torch.tensor([self.dropout_seed, 0], dtype=torch.int64, device=ctx.session.device)
        return cache[key]

    def plan(self, ctx: RunContext, shard=None, training: bool = False, keep: float = 1.0) -> ForwardPlan:
        """The cached ForwardPlan for the adjacency/feature values fed in this run (training:
        the flat-mode plan that keeps every group's pre-normalisation sum for the backward;
        keep < 1: dropout, layers.py:87-88 and :112)."""
        local = None if shard is None else shard.local
        dg = runtime.device_graph(ctx, self.edge_types, self.adj_mats, local,
                                  row_block=None if shard is None else shard.row_block)
        feats = {j: runtime.feature_csr(ctx, self.inputs[j]) if j in self.inputs else None
                 for j in dg.n_nodes}
        key = ("plan", id(self), id(dg), tuple((j, id(f)) for j, f in feats.items()),
               None if shard is None else id(shard), training, keep)
        cache = runtime.plan_cache(ctx)
        hit = cache.get(key)
        if hit is None:
            for et in self.edge_types:
                if self.layers1[et].weights_stack.device != ctx.session.device:
                    raise RuntimeError("model parameters are not on the session's device "
                                       "(construct the model after a HIP device is visible)")
            w1, w2 = self.weight_stacks()
            before = torch.cuda.memory_allocated(ctx.session.device)
            p = ForwardPlan(dg, feats, w1, w2, self.h1, self.h2,
                            shard=shard, keep_sums=training,
                            dropout=(keep, self.dropout_state(ctx)) if keep < 1.0 else None)
            hit = (dg, feats, p)
            cache.put(key, hit, torch.cuda.memory_allocated(ctx.session.device) - before)
            p.cache_ref = (cache, key)  # later allocations for this plan (its TrainPlan) are charged to it
        return hit[2]

    def _forward(self, ctx: RunContext) -> ForwardPlan:
        key = ("forward", id(self))
        if key not in ctx.cache:
            d = float(ctx.value(self.dropout))
            if not 0.0 <= d < 1.0:
                raise ValueError(f"dropout rate {d} outside [0, 1)")
            p = self.plan(ctx, getattr(ctx.session, "shard", None), training=ctx.training, keep=1.0 - d)
            p.run()
            ctx.cache[key] = p
        return ctx.cache[key]
