"""Layer classes with the reference's constructor signatures and variable layout
(decagon/deep/layers.py:12-213).

In the reference each layer's `_call` emits one TF op per relation.  Here a layer owns its
weights as one device stack [K, d_in, d_out] (the per-relation `vars['weights_%d']` are
views of it), and `DecagonModel` runs all layers of a model through the fused plan in
engine.py.  Calling a layer on its own (`layer(inputs)`) still works and returns a lazily
evaluated node that runs the same HIP kernels for that one edge type.

Activations are classified by probing (`act_kind`): identity (`lambda x: x`, what
DecagonModel passes, model.py:71/83/99/...) and relu are supported on the device path.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from . import inits, kernels, runtime
from ._lib import DG_EPI_CHUNK_RELU, DG_EPI_L2NORM
from .graph import InvalidArgumentError, Node, Variable

# global unique layer ID dictionary for layer name assignment (layers.py:9-20)
_LAYER_UIDS: Dict[str, int] = {}


def get_layer_uid(layer_name: str = "") -> int:
    _LAYER_UIDS[layer_name] = _LAYER_UIDS.get(layer_name, 0) + 1
    return _LAYER_UIDS[layer_name]


def relu(x):
    """tf.nn.relu on torch / numpy values (an activation marker the kernels recognise)."""
    if isinstance(x, torch.Tensor):
        return torch.clamp_min(x, 0)
    return np.maximum(x, 0)


def sigmoid(x):
    if isinstance(x, torch.Tensor):
        return torch.sigmoid(x)
    return 1.0 / (1.0 + np.exp(-np.asarray(x)))


def act_kind(act) -> str:
    """'identity' | 'relu' | 'sigmoid' for a callable activation, by probing it."""
    probe = torch.tensor([-1.5, 0.0, 2.0])
    try:
        out = act(probe)
    except Exception as e:  # pragma: no cover - exotic activations
        raise ValueError(f"unsupported activation {act!r}: {e}") from e
    if out is probe:
        return "identity"
    out = torch.as_tensor(out, dtype=torch.float32)
    if torch.equal(out, probe):
        return "identity"
    if torch.equal(out, torch.tensor([0.0, 0.0, 2.0])):
        return "relu"
    if torch.allclose(out, torch.sigmoid(probe)):
        return "sigmoid"
    raise ValueError(f"unsupported activation {act!r} (identity, relu or sigmoid)")


def dropout_sparse(x, keep_prob, num_nonzero_elems, seed: int = 0, step: int = 0, tag: int = 0):
    """layers.py:23-31 on a host COO tuple (coords, values, shape): each of the
    num_nonzero_elems values kept with probability keep_prob and scaled by 1/keep_prob,
    dropped ones removed (tf.sparse_retain).  The draw is the device's counter-based stream
    (dropout.h: element e of stream `tag` at (seed, step)) — TF's RNG is not reproducible.
    Inside a model, the per-relation masks are drawn on the device by the SpMM that computes
    X_j·W_k (DG_GROUP_DROPOUT); this standalone form is for callers of the layer API."""
    kp = float(keep_prob)
    if kp == 1.0:
        return x
    from .sparse import as_coo_tuple

    coords, vals, shape = as_coo_tuple(x)
    n = int(num_nonzero_elems)
    if n != len(vals):
        raise ValueError(f"num_nonzero_elems {n} != {len(vals)} values")
    scale = _drop_scale_host(seed, step, tag, n, kp)
    keep = scale != 0
    return coords[keep], (np.asarray(vals, np.float32)[keep] * scale[keep]).astype(np.float32), shape


def _drop_scale_host(seed: int, step: int, tag: int, n: int, keep: float) -> np.ndarray:
    """dropout.h's mask stream on the host (the same bits the kernels draw)."""
    def lowbias32(x):
        x = np.asarray(x, np.uint32)
        x = x ^ (x >> np.uint32(16))
        x = (x * np.uint32(0x7FEB352D)).astype(np.uint32)
        x = x ^ (x >> np.uint32(15))
        x = (x * np.uint32(0x846CA68B)).astype(np.uint32)
        return x ^ (x >> np.uint32(16))
    with np.errstate(over="ignore"):
        k1 = lowbias32(np.uint32(seed & 0xFFFFFFFF) ^ np.uint32((tag * 0x9E3779B9) & 0xFFFFFFFF))
        key = lowbias32(k1 ^ np.uint32((((seed >> 32) & 0xFFFFFFFF) + step * 0x85EBCA6B) & 0xFFFFFFFF))
        h = lowbias32(key ^ np.arange(n, dtype=np.uint32))
    thr = np.uint32(np.float32(keep) * np.float32(16777216.0))
    return np.where((h >> np.uint32(8)) < thr, np.float32(1.0) / np.float32(keep), np.float32(0)).astype(np.float32)


class MultiLayer:
    """Base layer (layers.py:34-67): name assignment, kwargs check, `vars` dict."""

    def __init__(self, edge_type=(), num_types=-1, **kwargs):
        self.edge_type = edge_type
        self.num_types = num_types
        allowed_kwargs = {"name", "logging"}
        for kwarg in kwargs.keys():
            assert kwarg in allowed_kwargs, "Invalid keyword argument: " + kwarg
        name = kwargs.get("name")
        if not name:
            layer = self.__class__.__name__.lower()
            name = layer + "_" + str(get_layer_uid(layer))
        self.name = name
        self.vars: Dict[str, Variable] = {}
        self.logging = kwargs.get("logging", False)
        self.issparse = False

    def _scope(self) -> str:
        return runtime.scoped(f"{self.name}_vars")

    def _call(self, inputs):
        return inputs

    def __call__(self, inputs):
        return self._call(inputs)


def _glorot_stack(k: int, d_in: int, d_out: int) -> torch.Tensor:
    arr = np.stack([inits.glorot_array(d_in, d_out) for _ in range(k)]) if k else \
        np.zeros((0, d_in, d_out), np.float32)
    return torch.from_numpy(arr).to(runtime.param_device())


def _dropout(ctx, layer, tag: int):
    """(keep, device state, tag) for a layer called on its own with dropout > 0, else None: the
    counter-based masks of dropout.h from the layer's own state {seed, step} in the session,
    advanced once per run, so every run draws new masks (TF's RNG stream itself is not
    reproducible; the distribution is: kept with probability keep, scaled by 1/keep)."""
    v = ctx.value(layer.dropout) if isinstance(layer.dropout, Node) else layer.dropout
    rate = float(v)
    if rate == 0.0:
        return None
    if not 0.0 < rate < 1.0:
        raise ValueError(f"dropout rate {rate} outside [0, 1)")
    key = ("layer_dropout_state", id(layer))
    cache = ctx.session.caches
    if key not in cache:
        cache[key] = torch.tensor([layer.dropout_seed, 0], dtype=torch.int64, device=ctx.session.device)
    state = cache[key]
    kernels.dropout_advance(state)
    return 1.0 - rate, state, tag


def _check_dropout(ctx, dropout) -> None:
    v = ctx.value(dropout) if isinstance(dropout, Node) else dropout
    if float(v) != 0.0:
        raise NotImplementedError("a decoder's _call with dropout > 0 (dead code in the reference, SURVEY §0.4)")


class _GraphConvBase(MultiLayer):
    dropout_seed = 20180702  # the standalone layer's dropout masks (a model's start at 20180701)

    def _make_weights(self, d_in: int, d_out: int) -> None:
        self.weights_stack = _glorot_stack(self.num_types, d_in, d_out)
        scope = self._scope()
        for k in range(self.num_types):
            self.vars["weights_%d" % k] = Variable(self.weights_stack[k], f"{scope}/weights_{k}:0",
                                                   initializer=lambda: inits.glorot_array(d_in, d_out))

    def _adj_group(self, ctx, per_rel: bool):
        """Upload (cached) this layer's adjacency feeds as one device group: one chunk for
        the whole group, or one per relation when the activation precedes add_n."""
        nodes = self.adj_mats[self.edge_type]
        return runtime.device_group(ctx, nodes, chunk=1 if per_rel else len(nodes))


class GraphConvolutionSparseMulti(_GraphConvBase):
    """Graph convolution on sparse features (layers.py:70-94):
    l2norm_rows( Σ_k act(Â_k · (X_j · W_k)) )."""

    def __init__(self, input_dim, output_dim, adj_mats, nonzero_feat, dropout=0., act=relu, **kwargs):
        super().__init__(**kwargs)
        self.dropout = dropout
        self.adj_mats = adj_mats
        self.act = act
        self.issparse = True
        self.nonzero_feat = nonzero_feat
        self.input_dim = input_dim
        self.output_dim = output_dim
        self._make_weights(input_dim[self.edge_type[1]], output_dim)

    def _call(self, inputs):
        kind = act_kind(self.act)
        if kind == "sigmoid":
            raise NotImplementedError("sigmoid activation inside a GCN layer is not on the HIP path")

        def fn(ctx):
            drop = _dropout(ctx, self, 1 << 16)
            grp = self._adj_group(ctx, kind == "relu")
            feat = runtime.feature_csr(ctx, inputs)
            return runtime.gcn_layer(grp, self.weights_stack, feat, self.output_dim, kind == "relu", drop)

        return Node(f"{self.name}/out", fn)


class GraphConvolutionMulti(_GraphConvBase):
    """Graph convolution on dense inputs (layers.py:97-118):
    l2norm_rows( Σ_k act(Â_k · (H_j · W_k)) )."""

    def __init__(self, input_dim, output_dim, adj_mats, dropout=0., act=relu, **kwargs):
        super().__init__(**kwargs)
        self.adj_mats = adj_mats
        self.dropout = dropout
        self.act = act
        self.input_dim = input_dim
        self.output_dim = output_dim
        self._make_weights(input_dim, output_dim)

    def _call(self, inputs):
        kind = act_kind(self.act)
        if kind == "sigmoid":
            raise NotImplementedError("sigmoid activation inside a GCN layer is not on the HIP path")

        def fn(ctx):
            drop = _dropout(ctx, self, 2 << 16)
            grp = self._adj_group(ctx, kind == "relu")
            h = ctx.value(inputs)
            h = runtime.as_device_f32(h)
            return runtime.gcn_layer_dense(grp, self.weights_stack, h, self.output_dim, kind == "relu", drop)

        return Node(f"{self.name}/out", fn)


class _DecoderBase(MultiLayer):
    """Decoders own parameters; DecagonModel reads them into latent_inters/latent_varies
    (model.py:116-137).  `_call` (dead code in the reference, §0.4 of SURVEY) is provided:
    it returns per-relation full score matrices act(row·L·G·L·colᵀ)."""

    def __init__(self, input_dim, dropout=0., act=sigmoid, **kwargs):
        super().__init__(**kwargs)
        self.dropout = dropout
        self.act = act
        self.input_dim = input_dim

    def _make_vars(self, init_fns) -> None:
        """All of the decoder's variables as views of ONE flat device buffer (`self.flat`),
        each starting 16-byte aligned — so the optimizer updates a decoder in one segment.
        init_fns: name -> initializer (drawn once here, again by global_variables_initializer)."""
        arrays = {name: fn() for name, fn in init_fns.items()}
        offs, off = {}, 0
        for name, a in arrays.items():
            offs[name] = off
            off += -(-int(np.asarray(a).size) // 4) * 4
        self.flat = torch.zeros(off, dtype=torch.float32, device=runtime.param_device())
        for name, a in arrays.items():
            a = np.ascontiguousarray(a, np.float32)
            view = self.flat[offs[name]:offs[name] + a.size].view(a.shape)
            view.copy_(torch.from_numpy(a))
            self.vars[name] = Variable(view, f"{self._scope()}/{name}:0", initializer=init_fns[name])

    def latent(self, k: int):
        """(G kind, G variable or None, L kind, L variable or None) for relation k."""
        raise NotImplementedError

    def _call(self, inputs):
        i, j = self.edge_type
        kind = act_kind(self.act)
        outs = []
        for k in range(self.num_types):
            def fn(ctx, k=k):
                _check_dropout(ctx, self.dropout)
                rows = runtime.as_device_f32(ctx.value(inputs[i]))
                cols = runtime.as_device_f32(ctx.value(inputs[j]))
                G, l = runtime.latent_operands(ctx, *self.latent(k), d=self.input_dim)
                rec = runtime.full_scores(rows, cols, G, l)
                if kind == "sigmoid":
                    rec = runtime.sigmoid_(rec)
                elif kind == "relu":
                    rec.clamp_min_(0)
                return rec
            outs.append(Node(f"{self.name}/rec_{k}", fn))
        return outs


class DEDICOMDecoder(_DecoderBase):
    """layers.py:121-147: global R (d×d) + per-relation diagonal D_k."""

    def __init__(self, input_dim, dropout=0., act=sigmoid, **kwargs):
        super().__init__(input_dim, dropout, act, **kwargs)
        d = input_dim
        fns = {"global_interaction": lambda: inits.glorot_array(d, d)}
        for k in range(self.num_types):
            fns["local_variation_%d" % k] = lambda: inits.glorot_array(d, 1).reshape(-1)
        self._make_vars(fns)

    def latent(self, k):
        return "dense", self.vars["global_interaction"], "diag", self.vars["local_variation_%d" % k]


class DistMultDecoder(_DecoderBase):
    """layers.py:150-172: G = diag(r_k), L = I."""

    def __init__(self, input_dim, dropout=0., act=sigmoid, **kwargs):
        super().__init__(input_dim, dropout, act, **kwargs)
        d = input_dim
        self._make_vars({"relation_%d" % k: (lambda: inits.glorot_array(d, 1).reshape(-1))
                         for k in range(self.num_types)})

    def latent(self, k):
        return "diag", self.vars["relation_%d" % k], "eye", None


class BilinearDecoder(_DecoderBase):
    """layers.py:175-195: G = M_k (d×d), L = I."""

    def __init__(self, input_dim, dropout=0., act=sigmoid, **kwargs):
        super().__init__(input_dim, dropout, act, **kwargs)
        d = input_dim
        self._make_vars({"relation_%d" % k: (lambda: inits.glorot_array(d, d))
                         for k in range(self.num_types)})

    def latent(self, k):
        return "dense", self.vars["relation_%d" % k], "eye", None


class InnerProductDecoder(_DecoderBase):
    """layers.py:198-213: G = I, L = I (no parameters)."""

    def __init__(self, input_dim, dropout=0., act=sigmoid, **kwargs):
        super().__init__(input_dim, dropout, act, **kwargs)
        self._make_vars({})

    def latent(self, k):
        return "eye", None, "eye", None
