"""DecagonOptimizer with the reference's constructor and attributes
(decagon/deep/optimizer.py:8-160).

Scores: the reference forms the B×B product row·L·G·L·colᵀ and keeps its diagonal
(optimizer.py:51-57, :63-85); here `outputs` / `neg_outputs` come from
dg_decoder_score_f32, which computes exactly the diagonal.  `preds` / `neg_preds` (the
full B×B matrices) and `predictions` (E_i·L·G·L·E_jᵀ, :87-106) are fp32-MFMA GEMMs.
Negatives are drawn on the device from the same distortion-0.75 unigram distribution as
tf.nn.fixed_unigram_candidate_sampler (:37-49); feeding `opt.neg_samples` injects them
(TF semantics: any tensor may be fed), which is how parity tests pin them.

`opt_op` (:108-114) runs the training step on the device: the forward in training mode, the
backward of the hinge cost (decagon_amd/train.py) and TF 1.8's Adam on every variable.
`grads_vars` returns (gradient, value) pairs of every variable, like compute_gradients.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from . import kernels, runtime, train
from .flags import FLAGS
from .graph import InvalidArgumentError, Node, Operation, RunContext


class _Sampler:
    """Per-relation device alias tables of degree^0.75 (built once per session)."""

    def __init__(self, degrees_list, device):
        self.tables = [kernels.upload_alias(deg, device) for deg in degrees_list]
        self.counter = 0


class DecagonOptimizer:
    def __init__(self, embeddings, latent_inters, latent_varies, degrees, edge_types,
                 edge_type2dim, placeholders, margin=0.1, neg_sample_weights=1., batch_size=100):
        self.embeddings = embeddings
        self.latent_inters = latent_inters
        self.latent_varies = latent_varies
        self.edge_types = edge_types
        self.degrees = degrees
        self.edge_type2dim = edge_type2dim
        self.obj_type2n = {i: self.edge_type2dim[i, j][0][0] for i, j in self.edge_types}
        self.margin = margin
        self.neg_sample_weights = neg_sample_weights
        self.batch_size = batch_size
        self.seed = 0

        self.placeholders = placeholders
        self.inputs = placeholders["batch"]
        self.batch_edge_type_idx = placeholders["batch_edge_type_idx"]
        self.batch_row_edge_type = placeholders["batch_row_edge_type"]
        self.batch_col_edge_type = placeholders["batch_col_edge_type"]

        # flat relation index r -> (i, j, k), in edge-type order (minibatch.py:45-54)
        self._rel_degrees = []
        self._rel_of = []
        for i, j in self.edge_types:
            for k in range(self.edge_types[i, j]):
                self._rel_of.append((i, j, k))
                self._rel_degrees.append(self.degrees[i][k])

        self.row_inputs = Node("optimizer/row_inputs", lambda ctx: self._batch(ctx)[:, 0])
        self.col_inputs = Node("optimizer/col_inputs", lambda ctx: self._batch(ctx)[:, 1])
        obj_type_n = [self.obj_type2n[i] for i in range(len(self.embeddings))]
        self.obj_type_lookup_start = np.cumsum([0] + obj_type_n[:-1])
        self.obj_type_lookup_end = np.cumsum(obj_type_n)

        # One fused launch (dg_decoder_hinge_f32) yields negatives, both score vectors and the
        # hinge loss; the reference's nodes are views of it.
        self._decode = Node("optimizer/decode", self._decode_fn)
        self.neg_samples = Node("optimizer/neg_samples", lambda ctx: ctx.value(self._decode)[3])
        self.outputs = Node("optimizer/outputs", lambda ctx: ctx.value(self._decode)[0])
        self.neg_outputs = Node("optimizer/neg_outputs", lambda ctx: ctx.value(self._decode)[1])
        self.preds = Node("optimizer/preds", lambda ctx: self._full(ctx, self.row_inputs))
        self.neg_preds = Node("optimizer/neg_preds", lambda ctx: self._full(ctx, self.neg_samples))
        self.predict()
        self._build()

    # ------------------------------------------------------------------ graph pieces
    def _batch(self, ctx: RunContext) -> np.ndarray:
        b = np.asarray(ctx.value(self.inputs))
        if b.ndim != 2 or b.shape[1] != 2:
            raise InvalidArgumentError(f"batch must be [B, 2], got {b.shape}")
        return b.astype(np.int32, copy=False)

    def _edge(self, ctx):
        e = int(np.asarray(ctx.value(self.batch_edge_type_idx)))
        rt = int(np.asarray(ctx.value(self.batch_row_edge_type)))
        ct = int(np.asarray(ctx.value(self.batch_col_edge_type)))
        if not 0 <= e < len(self._rel_of):
            raise InvalidArgumentError(f"batch_edge_type_idx {e} out of range")
        return e, rt, ct

    def _idx_dev(self, ctx, node: Node, n_max: int) -> torch.Tensor:
        v = ctx.value(node)
        if isinstance(v, torch.Tensor):
            t = v.to(device=ctx.session.device, dtype=torch.int32)
            if t.numel():
                lo, hi = int(t.min()), int(t.max())
                if lo < 0 or hi >= n_max:
                    raise InvalidArgumentError(f"{node.name}: index out of range [0, {n_max})")
            return t.contiguous()
        a = np.asarray(v).astype(np.int64).reshape(-1)
        if a.size and (a.min() < 0 or a.max() >= n_max):
            raise InvalidArgumentError(f"{node.name}: index out of range [0, {n_max})")
        return torch.from_numpy(a.astype(np.int32)).to(ctx.session.device)

    def _tables(self, ctx, rt, ct):
        row = runtime.as_device_f32(ctx.value(self.embeddings[rt]))
        col = runtime.as_device_f32(ctx.value(self.embeddings[ct]))
        return row, col

    def _latent(self, ctx, e):
        gi, gv = self.latent_inters[e], self.latent_varies[e]
        if hasattr(gi, "kind") and hasattr(gv, "kind"):  # DecagonModel's latent nodes
            return runtime.latent_operands(ctx, gi.kind, gi.var, gv.kind, gv.var, gi.d, gi, gv)
        # arbitrary user nodes: fold a dense L into G (uᵀ·L·G·L·v = uᵀ·(LGL)·v)
        G = runtime.as_device_f32(ctx.value(gi))
        L = runtime.as_device_f32(ctx.value(gv))
        return kernels.matmul(kernels.matmul(L, G), L), None

    def _sampler(self, ctx) -> _Sampler:
        key = ("sampler", id(self))
        cache = ctx.session.caches
        if key not in cache:
            cache[key] = _Sampler(self._rel_degrees, ctx.session.device)
        return cache[key]

    def _decode_fn(self, ctx: RunContext):
        """(pos scores, neg scores, hinge loss, negative rows) of the fed batch."""
        e, rt, ct = self._edge(ctx)
        row_t, col_t = self._tables(ctx, rt, ct)
        rows = self._idx_dev(ctx, self.row_inputs, row_t.shape[0])
        cols = self._idx_dev(ctx, self.col_inputs, col_t.shape[0])
        G, l = self._latent(ctx, e)
        if ctx.is_fed(self.neg_samples):
            negs = self._idx_dev(ctx, self.neg_samples, row_t.shape[0])
            if negs.numel() != rows.numel():
                raise InvalidArgumentError("neg_samples must have one entry per batch edge")
            op = kernels.PreparedDecoderHinge(row_t, col_t, rows, cols, G, l, self.margin, neg_rows=negs)
        else:
            s = self._sampler(ctx)
            if s.tables[e].shape[0] > row_t.shape[0]:
                raise InvalidArgumentError("degrees list longer than the row embedding table")
            op = kernels.PreparedDecoderHinge(row_t, col_t, rows, cols, G, l, self.margin, alias=s.tables[e],
                                              seed=self.seed, offset=s.counter)
            s.counter += rows.numel()
        op()
        return op.pos, op.neg, op.loss[0], op.neg_rows

    def _scores(self, ctx: RunContext, rows_node: Node) -> torch.Tensor:
        e, rt, ct = self._edge(ctx)
        row_t, col_t = self._tables(ctx, rt, ct)
        rows = self._idx_dev(ctx, rows_node, row_t.shape[0])
        cols = self._idx_dev(ctx, self.col_inputs, col_t.shape[0])
        if rows.numel() != cols.numel():
            raise InvalidArgumentError("row / column index counts differ")
        G, l = self._latent(ctx, e)
        return kernels.decoder_score(row_t, col_t, rows, cols, G, l)

    def _full(self, ctx: RunContext, rows_node: Node) -> torch.Tensor:
        e, rt, ct = self._edge(ctx)
        row_t, col_t = self._tables(ctx, rt, ct)
        rows = self._idx_dev(ctx, rows_node, row_t.shape[0]).long()
        cols = self._idx_dev(ctx, self.col_inputs, col_t.shape[0]).long()
        G, l = self._latent(ctx, e)
        return runtime.full_scores(row_t.index_select(0, rows).contiguous(),
                                   col_t.index_select(0, cols).contiguous(), G, l)

    def batch_predict(self, row_inputs, col_inputs):
        """optimizer.py:63-85 as a node: the full B×B score matrix."""
        return Node("optimizer/batch_predict", lambda ctx: self._full(ctx, row_inputs))

    def predict(self):
        """optimizer.py:87-106: predictions = E_i·L·G·L·E_jᵀ for the fed edge type."""
        def fn(ctx):
            e, rt, ct = self._edge(ctx)
            row_t, col_t = self._tables(ctx, rt, ct)
            G, l = self._latent(ctx, e)
            return runtime.full_scores(row_t, col_t, G, l)
        self.predictions = Node("optimizer/predictions", fn)

    def _build(self):
        self.cost = self._hinge_loss(self.outputs, self.neg_outputs)
        self.optimizer = "adam"  # tf.train.AdamOptimizer(learning_rate=FLAGS.learning_rate)
        self.opt_op = Operation("optimizer/opt_op", lambda ctx: self._train(ctx, apply=True), training=True)
        self.grads_vars = Node("optimizer/grads_vars", lambda ctx: self._train(ctx, apply=False))
        self.grads_vars.training = True

    # ------------------------------------------------------------------ training step
    def _model(self):
        for e in self.embeddings:
            m = getattr(e, "model", None)
            if m is not None:
                return m
        raise NotImplementedError("opt_op needs the embeddings of a DecagonModel")

    def _train_plan(self, ctx: RunContext, model):
        fwd = model._forward(ctx)
        # the backward plan lives on its forward plan: evicting the plan (runtime's LRU) drops both
        plans = fwd.__dict__.setdefault("_train_plans", {})
        if id(self) not in plans:
            feats = {j: runtime.feature_csr(ctx, model.inputs[j]) if j in model.inputs else None
                     for j in fwd.g.n_nodes}
            w1, w2 = model.weight_stacks()
            before = torch.cuda.memory_allocated(ctx.session.device)
            plans[id(self)] = train.TrainPlan(fwd, w1, w2, feats)
            ref = getattr(fwd, "cache_ref", None)
            if ref is not None:  # the backward's buffers count against the plan's LRU entry
                ref[0].add_bytes(ref[1], torch.cuda.memory_allocated(ctx.session.device) - before)
        return fwd, plans[id(self)]

    def _decoder_grads(self, ctx: RunContext, model, e: int, rt: int, ct: int):
        """Zeroed gradient buffers of every decoder, the batch relation's entries filled
        (TF's gather over the stacked latent lists gives the others dense zeros)."""
        key = ("dec_grads", id(self))
        cache = ctx.session.caches
        if key not in cache:
            cache[key] = {et: torch.zeros_like(d.flat) for et, d in model.edge_type2decoder.items()}
        grads = cache[key]
        for t in grads.values():
            t.zero_()
        i, j, k = self._rel_of[e]
        dec = model.edge_type2decoder[i, j]
        gflat = grads[i, j]

        def gview(var):
            off = (var.tensor.data_ptr() - dec.flat.data_ptr()) // 4
            return gflat[off:off + var.tensor.numel()]

        gk, gv, lk, lv = model._latent_spec[e]
        fed = ctx.is_fed(self.latent_inters[e]) or ctx.is_fed(self.latent_varies[e])
        out = {"dG": None, "dl": None, "dG_diag": None}
        if not fed:
            if gk == "dense":
                out["dG"] = gview(gv)
            elif gk == "diag":
                out["dG_diag"] = gview(gv)
            if lk == "diag":
                out["dl"] = gview(lv)
        return grads, out

    def _train(self, ctx: RunContext, apply: bool):
        """One training step (apply) or the gradients only (compute_gradients)."""
        if not ctx.training:
            raise RuntimeError("training ops must be fetched through Session.run")
        for nd in (self.outputs, self.neg_outputs, self.cost):
            if ctx.is_fed(nd):
                raise InvalidArgumentError(f"{nd.name} is fed: the cost's gradient does not reach the model")
        model = self._model()
        fwd, tp = self._train_plan(ctx, model)
        pos, neg, _, negs_dev = ctx.value(self._decode)
        e, rt, ct = self._edge(ctx)
        row_t, col_t = self._tables(ctx, rt, ct)
        rows = self._idx_dev(ctx, self.row_inputs, row_t.shape[0])
        cols = self._idx_dev(ctx, self.col_inputs, col_t.shape[0])
        negs = (self._idx_dev(ctx, self.neg_samples, row_t.shape[0]) if ctx.is_fed(self.neg_samples)
                else negs_dev)
        G, l = self._latent(ctx, e)
        dec_grads, outs = self._decoder_grads(ctx, model, e, rt, ct)
        if outs["dl"] is not None and l is None:
            raise RuntimeError("DEDICOM decoder without its diagonal")
        op = kernels.PreparedDecoderGrad(row_t, col_t, rows, cols, negs, pos, neg, G, l, self.margin, **outs)

        def decoder_grad(dE):
            op()
            kernels.scatter_rows(op.row_idx, op.grad_rows, dE[rt])
            kernels.scatter_rows(cols, op.grad_cols, dE[ct])

        tp.backward(decoder_grad)
        w1, w2 = model.weight_stacks()
        ets = list(model.edge_types)
        pairs = tp.adam_pairs(w1, w2)  # whole stacks (one GPU) or the local relations (sharded)
        params = [p for p, _ in pairs] + [model.edge_type2decoder[et].flat for et in ets]
        grads = [g for _, g in pairs] + [dec_grads[et] for et in ets]
        if not apply:
            # (sharded: every relation's gradient gathered from its owner rank, so every rank
            # returns the whole model's (gradient, variable) list, as compute_gradients does)
            gW1, gW2 = tp.full_grads()
            return self._grads_vars(model, gW1, gW2, dec_grads)
        # the Adam slots belong to the variables (session-wide); the prepared launch, which holds
        # this plan's gradient buffers, lives on the TrainPlan, so evicting the plan frees both
        key = ("adam", id(self))
        cache = ctx.session.caches
        if key not in cache:
            cache[key] = train.AdamState(params, lr=float(FLAGS.learning_rate))
        st = cache[key]
        prep = getattr(tp, "adam_prepared", None)
        if prep is None or prep[0] is not st:
            tp.adam_prepared = prep = (st, st.prepared(grads))
        st.apply(prep[1])
        return None

    def _grads_vars(self, model, gW1, gW2, dec_grads):
        """[(gradient, variable value)] in model.vars order (layers 1, layers 2, decoders);
        gW1 / gW2: every relation's gradient stack (TrainPlan.full_grads)."""
        out = []
        for et, lay in model.layers1.items():
            for k in range(lay.num_types):
                out.append((gW1[et][k], lay.vars["weights_%d" % k].tensor))
        for et, lay in model.layers2.items():
            for k in range(lay.num_types):
                out.append((gW2[et][k], lay.vars["weights_%d" % k].tensor))
        for et, dec in model.edge_type2decoder.items():
            for var in dec.vars.values():
                off = (var.tensor.data_ptr() - dec.flat.data_ptr()) // 4
                out.append((dec_grads[et][off:off + var.tensor.numel()].view(var.tensor.shape).clone(),
                            var.tensor.clone()))
        return [(g.clone(), v.clone()) for g, v in out]

    def _hinge_loss(self, aff, neg_aff):
        """optimizer.py:116-120: sum(relu(neg - (pos - margin)))."""
        def fn(ctx):
            if aff is self.outputs and neg_aff is self.neg_outputs and not (
                    ctx.is_fed(aff) or ctx.is_fed(neg_aff)):
                return ctx.value(self._decode)[2]  # computed by the fused decoder launch
            pos = runtime.as_device_f32(ctx.value(aff))
            neg = runtime.as_device_f32(ctx.value(neg_aff))
            return kernels.hinge_loss(pos, neg, self.margin)[0]
        return Node("optimizer/cost", fn)

    def _xent_loss(self, aff, neg_aff):
        """optimizer.py:122-127."""
        def fn(ctx):
            pos = runtime.as_device_f32(ctx.value(aff))
            neg = runtime.as_device_f32(ctx.value(neg_aff))
            return kernels.xent_loss(pos, neg, self.neg_sample_weights)[0]
        return Node("optimizer/xent_cost", fn)


def gather_cols(params, indices, name=None):
    """optimizer.py:130-160: gather columns of a 2-D array (host-side index plumbing)."""
    p = np.asarray(params)
    if p.ndim != 2:
        raise ValueError("'params' must be 2D.")
    idx = np.asarray(indices)
    if idx.ndim != 1:
        raise ValueError("'params' must be 1D.")
    return p[:, idx]
