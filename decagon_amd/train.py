"""The training step: backward of the hinge cost through both GCN layers, and TF 1.8's Adam.

Reference: `DecagonOptimizer._build` (decagon/deep/optimizer.py:108-114) —
`tf.train.AdamOptimizer(FLAGS.learning_rate).minimize(self.cost)` — driven by
`sess.run([opt.opt_op, opt.cost, ...])` (main.py:315, DecagonTrainer.py:90-102).  TF derives
the backward graph automatically; here it is written out over the forward's saved state:

  forward (ForwardPlan in flat mode)  S1_ij = Σ_k Â_k·W1_k,  H1_i = relu(Σ_j l2n(S1_ij))
                                      S2_ij = Σ_k Â_k·(H1_j·W2_k),  E_i = Σ_j l2n(S2_ij)
  decoder + gathers                   dE_i (dg_decoder_grad_f32 + dg_scatter_rows_f32)
  layer 2                             dS2_ij = l2n'(S2_ij)·dE_i            dg_l2norm_grad_f32
                                      dP_ijk = Â_kᵀ·dS2_ij                 dg_spmm_groups_f32 (Âᵀ)
                                      dW2_ijk = H1_jᵀ·dP_ijk               dg_gemm_tn_f32
                                      dH1_j = Σ_ik dP_ijk·W2_ijkᵀ          dg_gemm_f32 (batch-reduce)
                                                                           + dg_gcn_epilogue_f32
  layer 1                             dS1_ij = l2n'(S1_ij)·(dH1_i∘[H1_i>0]) dg_l2norm_grad_f32
                                      dW1_ijk = Â_kᵀ·dS1_ij                dg_spmm_groups_f32 (Âᵀ)
  Adam (every variable, every step)   dg_adam_f32

Âᵀ of every relation is built once on the host from the uploaded CSR and stored as a
relation-chunked CSR whose virtual columns index the shared operand dS_ij directly, so the
transposed SpMM writes dP / dW1 straight in the weight-stack layout [K][n_j][d].

Relation-sharded training (N GPUs, sharding.RelationShard.lpt: every relation whole on one
rank, the forward in flat mode with its two all-reduces): a relation's weights are used only
by the rank that owns it, so that rank alone computes their gradients and applies Adam to
them — the gradient and Adam-slot stacks hold the LOCAL relations only ([K_local][…], in
ascending relation id), no weight gradient is exchanged and Adam's memory and time shard
with the relations.  The one extra collective is an all-reduce of dH1 (every node type's
rows, h1 wide) after the layer-2 backward, because dH1_j = Σ_ik dP_ijk·W2_ijkᵀ sums over
every rank's relations; the decoder and everything after the forward's all-reduces run
redundantly and identically on every rank.  With dropout every relation's masks are drawn
under its global id (dropout.hip's mapped forms), so each rank's forward and backward mask its
relations exactly as one GPU does.  Row-split node types (sharding.RelationShard.split) are
handled too: a rank holds rows [a, b) of every relation into the node type, so its l2-norm
gradient runs over its block (dE / dH1 rows a..b, the S_ij block sums its epilogue kept), its
Âᵀ·dS products are partial weight gradients summed by one all-reduce per such relation stack
after the backward (PPI: 9.8 MB), and every rank applies the same Adam step to those weights;
their dH1 contributions join the existing dH1 all-reduce.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import kernels
from ._lib import DG_MAX_GROUPS
from .engine import ForwardPlan, LayerWeights, drop_tag
from .sparse import HostCSR, merge_chunks
from .tuning import knob

EdgeType = Tuple[int, int]

BETA1, BETA2, EPSILON = 0.9, 0.999, 1e-8  # tf.train.AdamOptimizer defaults


def transpose_csr(c: HostCSR, with_perm: bool = False):
    """Âᵀ in CSR (rows = Â's columns, each row's nonzeros in ascending Â-row order);
    with_perm: also each transposed nonzero's position in Â (int32)."""
    n_r, n_c = c.shape
    lens = np.diff(c.rowptr.astype(np.int64))
    rows = np.repeat(np.arange(n_r, dtype=np.int64), lens)
    cols = c.col.astype(np.int64)
    order = np.lexsort((rows, cols))
    counts = np.bincount(cols, minlength=n_c)
    rowptr = np.zeros(n_c + 1, np.int64)
    np.cumsum(counts, out=rowptr[1:])
    t = HostCSR(rowptr.astype(np.int32), rows[order].astype(np.int32), c.val[order].astype(np.float32),
                (n_c, n_r))
    return (t, order.astype(np.int32)) if with_perm else t


def adam_alpha(lr: float, t: int, beta1: float = BETA1, beta2: float = BETA2) -> float:
    """lr·sqrt(1 − β2^t)/(1 − β1^t) in float32, with the beta powers kept as float32
    variables multiplied once per step — as TF 1.8's Adam computes it."""
    f = np.float32
    b1p, b2p = f(beta1), f(beta2)
    for _ in range(t - 1):
        b1p, b2p = f(b1p * f(beta1)), f(b2p * f(beta2))
    return float(f(f(lr) * np.sqrt(f(1) - b2p) / (f(1) - b1p)))


class AdamState:
    """m / v slots of a list of parameters (zeros at creation, as TF's slots) and the beta
    powers + alpha on the device ({β1^t, β2^t, alpha}, advanced after every update), so a
    whole training step is capturable into one hipGraph."""

    def __init__(self, params: Sequence[torch.Tensor], lr: float = 0.001):
        self.params = list(params)
        self.lr = float(lr)
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        dev = self.params[0].device if self.params else torch.device("cuda")
        self.state = torch.tensor([BETA1, BETA2, adam_alpha(self.lr, 1)], dtype=torch.float32, device=dev)

    def prepared(self, grads: Sequence[Optional[torch.Tensor]]) -> kernels.PreparedAdam:
        return kernels.PreparedAdam([(p, g, m, v) for p, g, m, v in zip(self.params, grads, self.m, self.v)])

    def apply(self, prepared: kernels.PreparedAdam) -> None:
        """One ApplyAdam over every segment, then the beta powers / alpha advance."""
        prepared(0.0, BETA1, BETA2, EPSILON, state=self.state)
        kernels.adam_advance(self.state, self.lr, BETA1, BETA2)


class TrainPlan:
    """Buffers and prepared launches of one backward over a flat-mode ForwardPlan."""

    def __init__(self, fwd: ForwardPlan, w1: LayerWeights, w2: LayerWeights,
                 features: Dict[int, Optional[HostCSR]]):
        if not fwd.keep_sums:
            raise NotImplementedError("training runs over a ForwardPlan(keep_sums=True)")
        self.sharded = fwd.allreduce is not None
        self.allreduce = fwd.allreduce
        # with dropout (fwd.drop_state), the backward reuses the forward's masks: the draws of the
        # forward's step, regenerated from the same counter-based hash (dropout.hip)
        # sparse features X_j (mono side effects): layer 1's weight gradient is X_jᵀ·(Â_kᵀ·dS1)
        # per relation, a second transposed SpMM over the same K chunks the forward used
        g = fwd.g
        self.fwd = fwd
        dev = g.device
        f32 = dict(device=dev, dtype=torch.float32)
        h1, h2 = fwd.h1, fwd.h2
        n = g.n_nodes
        self.h1, self.h2 = h1, h2
        ets = fwd.edge_types
        self.dE = {i: torch.zeros((n[i], h2), **f32) for i in fwd.targets}
        srcs = sorted({et[1] for et in ets})
        # dH1 of every node type in one flat buffer (sharded: all-reduced after the layer-2 backward)
        self._dH1_flat = torch.zeros(sum(n[j] for j in n) * h1, **f32)
        self.dH1, off = {}, 0
        for j in sorted(n):
            self.dH1[j] = self._dH1_flat[off:off + n[j] * h1].view(n[j], h1)
            off += n[j] * h1
        self.local_ids: Dict[EdgeType, np.ndarray] = {}  # global ids of gW*[et]'s rows
        # row-split node types (sharding.RelationShard.split): this rank holds rows [a, b) of every
        # relation into them, so its Âᵀ·dS products over those rows are PARTIAL weight
        # gradients — all-reduced after the backward (every rank then applies the same Adam step)
        rb = dict(fwd.row_block)
        dealt = set(getattr(fwd.shard, "dealt", None) or ())
        self._dealt = dealt
        rows_of = lambda i: (rb[i][1] - rb[i][0]) if i in rb else n[i]  # noqa: E731
        self._rowsplit_grads: List[torch.Tensor] = []
        self.gW1: Dict[EdgeType, torch.Tensor] = {}
        self.gW2: Dict[EdgeType, torch.Tensor] = {}
        specs2, specs1, gemm_w2, gemm_h1 = [], [], [], []
        self._w1_drop = []
        self._feat_specs: List[kernels.RelGroupSpec] = []
        runs: Dict[int, List[Tuple[torch.Tensor, int]]] = {j: [] for j in srcs}
        self._dS1, self._dS2 = {}, {}
        for et in ets:
            i, j = et
            grp = g.groups[et]
            if grp.host is None or (grp.n_rels != grp.K and not self.sharded):
                raise NotImplementedError("training needs every relation of a group on this device")
            order = np.argsort(grp.rel_ids, kind="stable")
            ids = np.asarray(grp.rel_ids, np.int64)[order]
            self.local_ids[et] = ids
            K = len(ids)  # local relations (all K_ij on one GPU)
            # sharded: local relation c (ascending id) is global relation ids[c] — the batch map of
            # the W2 reads and of the dropout masks
            idmap = None if np.array_equal(ids, np.arange(grp.K)) else torch.from_numpy(ids.astype(np.int32)).to(dev)
            if K == 0:  # another rank owns every relation of the group: no local gradient
                self.gW1[et] = torch.zeros((0, n[j] if features.get(j) is None else int(features[j].shape[1]), h1), **f32)
                self.gW2[et] = torch.zeros((0, h1, h2), **f32)
                # (the layer's l2-norm backward still writes the group's dS: nothing reads it)
                self._dS1[et] = torch.zeros((n[i], h1), **f32)
                self._dS2[et] = torch.zeros((n[i], h2), **f32)
                continue
            rels = [transpose_csr(grp.host[p]) for p in order]
            m = merge_chunks(rels, [0] * K, 1, 1)  # chunk k = local relation k; vcol = Â row (into dS)
            rp, vc, vv = (torch.from_numpy(m.rowptr).to(dev), torch.from_numpy(m.vcol).to(dev),
                          torch.from_numpy(m.val).to(dev))
            vmax = int(m.vcol.max()) if m.nnz else -1
            dS2 = torch.zeros((rows_of(i), h2), **f32)
            dS1 = torch.zeros((rows_of(i), h1), **f32)
            dP = torch.zeros((K, n[j], h2), **f32)
            self._dS1[et], self._dS2[et] = dS1, dS2
            self.gW2[et] = torch.zeros((K,) + tuple(w2.stacks[et].shape[1:]), **f32)
            fj = features.get(j)
            F = n[j] if fj is None else int(fj.shape[1])
            self.gW1[et] = torch.zeros((K, F, h1), **f32)
            if tuple(w1.stacks[et].shape) != (grp.K, F, h1):
                raise ValueError(f"layer-1 weights of {et} are {tuple(w1.stacks[et].shape)}, expected ({grp.K}, {F}, {h1})")
            # Âᵀ·dS1 per relation: the weight gradient itself (identity features), or the
            # operand of X_jᵀ·(·) (sparse features)
            g1 = self.gW1[et] if fj is None else torch.zeros((K, n[j], h1), **f32)
            specs2.append(kernels.RelGroupSpec(rp, vc, vv, dS2, dP, n[j], K, h2, rows_of(i), vcol_max=vmax))
            specs1.append(kernels.RelGroupSpec(rp, vc, vv, dS1, g1, n[j], K, h1, rows_of(i), vcol_max=vmax))
            if i in rb or et in dealt:  # (row-dealt groups: partial over this rank's rows too)
                self._rowsplit_grads += [self.gW1[et], self.gW2[et]]
            if fj is not None:  # X_jᵀ's pattern shared by the K chunks, chunk k reading G_k
                xt, perm = transpose_csr(fj, with_perm=True)
                drop = None
                if fwd.drop_state is not None:  # the forward's per-relation masks of X_j's values
                    drop = (fwd.drop_state, drop_tag(1, fwd.et_index[et]), fwd.keep)
                self._feat_specs.append(kernels.RelGroupSpec(
                    torch.from_numpy(xt.rowptr).to(dev), torch.from_numpy(xt.col).to(dev),
                    torch.from_numpy(xt.val).to(dev), g1, self.gW1[et], F, K, h1, n[j],
                    vcol_max=int(xt.col.max()) if xt.nnz else -1, shared=True, drop=drop,
                    drop_index=torch.from_numpy(perm).to(dev) if drop is not None else None))
            # dW2_k = H_kᵀ·dP_k with H_k = H1_j (or its per-relation dropout draw), the reduction
            # over the n_j rows split for long ones
            H = fwd.hdrop.get(et, fwd.hidden1[j])
            gemm_w2.append(kernels.PreparedGemmTN(H, dP, self.gW2[et]))
            # dH1_j partials = Σ_k M_k∘(dP_k·W2_kᵀ) over runs of R relations: B(c, m) = W2_k[m][c]
            # (M_k: layer 2's dropout mask of relation k, when dropout is on)
            R = K if K <= 64 else knob("DG_REDUCE_RUN", 16)
            n_runs = -(-K // R)
            part = torch.zeros((n_runs, n[j], h1), **f32)
            drop = ((fwd.drop_state, drop_tag(2, fwd.et_index[et]), fwd.keep) if fwd.drop_state is not None
                    else None)
            W2 = w2.stacks[et]  # (sharded: read at the local relations' global slabs)
            gemm_h1.append(kernels.PreparedGemm(dP, (n[j] * h2, h2, 1), W2, (h1 * h2, 1, h2), part,
                                                (n[j] * h1, h1, 1), n[j], h1, h2, K, reduce=R, drop=drop,
                                                b_map=idmap, b_batches=grp.K,
                                                b_map_max=int(ids.max()) if idmap is not None else None))
            if fwd.drop_state is not None and fj is None:  # dW1 rows through layer 1's row masks
                tg = drop_tag(1, fwd.et_index[et])
                if idmap is None:
                    self._w1_drop.append(lambda g=self.gW1[et], tg=tg:
                                         kernels.dropout_rows(g, g, fwd.drop_state, tg, fwd.keep))
                else:
                    self._w1_drop.append(lambda g=self.gW1[et], tg=tg, m=idmap, F=F, mx=int(ids.max()):
                                         kernels.dropout_rows_map(g, g, m, F, fwd.drop_state, tg, fwd.keep, False,
                                                                  False, rel_map_max=mx))
            runs[j].append((part, n_runs))
        chunked = lambda xs: [xs[s:s + DG_MAX_GROUPS] for s in range(0, len(xs), DG_MAX_GROUPS)]  # noqa: E731
        # Âᵀ·dS: operands small enough for LDS (the drug side) take the LDS-staged form
        small = lambda s: s.x_rows <= kernels.SPMM_LDS_MAX_ROWS  # noqa: E731
        self._spmm2, self._spmm1 = [], []
        for specs, d, out in ((specs2, h2, self._spmm2), (specs1, h1, self._spmm1)):
            for lds in (True, False):
                sel = [s for s in specs if small(s) == lds]
                out += [kernels.PreparedSpmm(c, d, lds=lds) for c in chunked(sel)]
        self._feat = [kernels.PreparedSpmm(c, h1) for c in chunked(self._feat_specs)]
        self._gemm_w2 = gemm_w2
        self._gemm_h1 = [kernels.PreparedGemmMulti(c) for c in chunked(gemm_h1)]
        self._epi_h1 = []
        for j, lst in runs.items():
            if not lst:  # no local relation reads H1_j: its (zeroed) dH1 rows come from the all-reduce
                continue
            if len(lst) > DG_MAX_GROUPS:
                raise ValueError(f"more than {DG_MAX_GROUPS} edge types out of node type {j}")
            self._epi_h1.append(kernels.PreparedEpilogue(lst, self.dH1[j], n[j], h1, 0))
        L1, L2 = fwd._layer1, fwd._layer2
        self._l2g2, self._l2g1 = [], []
        for i, tets in fwd.targets.items():
            a, b = (rb[i][0], rb[i][1]) if i in rb else (0, n[i])  # (row-split: this rank's block)
            self._l2g2.append(kernels.PreparedL2Grad([(L2.views[et], self._dS2[et]) for et in tets],
                                                     self.dE[i][a:b], None, b - a, h2))
            dy = self.dH1[i][a:b]  # zero when no layer-2 relation reads H1_i
            self._l2g1.append(kernels.PreparedL2Grad([(L1.views[et], self._dS1[et]) for et in tets],
                                                     dy, fwd.hidden1[i][a:b], b - a, h1))

    def backward(self, decoder_grad) -> None:
        """dE ← decoder_grad(dE) (it adds the decoder's row gradients into the zeroed dE),
        then both layers' backward into gW2 / gW1."""
        for t in self.dE.values():
            t.zero_()
        if self.sharded:
            self._dH1_flat.zero_()  # node types without local layer-2 relations add zeros
        decoder_grad(self.dE)
        for l in self._l2g2:
            l()
        for s in self._spmm2:
            s()
        for gm in self._gemm_w2:
            gm()
        for gm in self._gemm_h1:
            gm()
        for e in self._epi_h1:
            e()
        if self.sharded:
            self.allreduce(self._dH1_flat)  # dH1_j = Σ over every rank's relations
        for l in self._l2g1:
            l()
        for s in self._spmm1:
            s()
        for s in self._feat:
            s()
        for f in self._w1_drop:
            f()
        for gr in self._rowsplit_grads:  # row-split groups: Σ over the ranks' row blocks
            self.allreduce(gr)

    def full_grads(self) -> Tuple[Dict[EdgeType, torch.Tensor], Dict[EdgeType, torch.Tensor]]:
        """Every relation's W1 / W2 gradient as full [K, ...] stacks, on every rank — what
        compute_gradients returns for the whole model (optimizer.py:114).  One GPU: the stacks
        themselves.  Sharded: a relation-sharded group's relation k lives on its owner rank
        only, so the local slices are placed at their global ids in zero stacks and the stacks
        of every such group are summed over the ranks in ONE all-reduce (exactly one rank owns
        each relation: the sum is a gather, bit-exact); a row-split group's stacks are already
        complete and equal on every rank (all-reduced by the backward) and are copied."""
        if not self.sharded:
            return self.gW1, self.gW2
        rb = self.fwd.row_block
        shapes, sizes = [], []
        for name, grads in (("w1", self.gW1), ("w2", self.gW2)):
            for et in self.fwd.edge_types:
                if et[0] in rb or et in self._dealt:
                    continue
                K = self.fwd.g.groups[et].K
                shapes.append((name, et, (K,) + tuple(grads[et].shape[1:])))
                sizes.append(int(np.prod(shapes[-1][2])))
        dev = self.fwd.g.device
        flat = torch.zeros(int(sum(sizes)), dtype=torch.float32, device=dev)
        out = {"w1": {}, "w2": {}}
        off = 0
        for (name, et, shape), sz in zip(shapes, sizes):
            full = flat[off:off + sz].view(shape)
            off += sz
            ids = self.local_ids[et]
            if len(ids):
                full[torch.from_numpy(ids).to(dev)] = (self.gW1 if name == "w1" else self.gW2)[et]
            out[name][et] = full
        if flat.numel():
            self.allreduce(flat)
        for name, grads in (("w1", self.gW1), ("w2", self.gW2)):
            for et in self.fwd.edge_types:
                if et[0] in rb or et in self._dealt:
                    out[name][et] = grads[et].clone()
        return out["w1"], out["w2"]

    def adam_pairs(self, w1: LayerWeights, w2: LayerWeights) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        """(parameter, gradient) of every GCN weight this plan updates: whole stacks on one GPU;
        the local relations' slices, one pair per relation, when sharded."""
        out = []
        for stacks, grads in ((w1.stacks, self.gW1), (w2.stacks, self.gW2)):
            for et in self.fwd.edge_types:
                ids = self.local_ids[et]
                if len(ids) == stacks[et].shape[0]:
                    out.append((stacks[et], grads[et]))
                else:
                    out += [(stacks[et][int(k)], grads[et][c]) for c, k in enumerate(ids)]
        return out
