"""The TF1-style surface the reference's callers use: placeholders, variables, lazily
evaluated tensors and `Session.run(fetches, feed_dict)`.

Callers of the reference build placeholders (main.py:93-108, DecagonDataSet.py:84-120),
construct `DecagonModel` / `DecagonOptimizer` once, then call
`sess.run([opt.opt_op, opt.cost, opt.batch_edge_type_idx], feed_dict)` (main.py:315,
DecagonTrainer.py:90-102) or `sess.run(opt.predictions, feed_dict)` (main.py:49,
DecagonAccuracyEvaluator.py:122).  Here a `Node` is a named, lazily evaluated value; a run
evaluates each requested node at most once (memoised in a `RunContext`), on the device,
and converts the fetched values to numpy with one synchronisation at the end.  As in TF,
any node — not only a placeholder — may be fed, which overrides its computation.
"""
from __future__ import annotations

import contextlib
import itertools
import weakref
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch

_ids = itertools.count()


class InvalidArgumentError(ValueError):
    """Raised like tf.errors.InvalidArgumentError (e.g. an unfed placeholder)."""


class Node:
    """A lazily evaluated value (the analogue of a tf.Tensor)."""

    def __init__(self, name: str, fn: Optional[Callable[["RunContext"], Any]] = None):
        self.name = name
        self._fn = fn
        self._id = next(_ids)

    def __repr__(self) -> str:
        return f"<{type(self).__name__} {self.name}>"

    def _compute(self, ctx: "RunContext") -> Any:
        if self._fn is None:
            raise InvalidArgumentError(f"{self.name} has no value")
        return self._fn(ctx)


class Operation(Node):
    """A node fetched for its side effect; fetching it yields None (like tf.Operation).
    `training` marks a training op: a run that fetches one evaluates the whole forward in
    training mode (the plan that keeps what the backward needs)."""

    def __init__(self, name: str, fn=None, training: bool = False):
        super().__init__(name, fn)
        self.training = training


class Placeholder(Node):
    def __init__(self, dtype=None, shape=None, name: Optional[str] = None, sparse: bool = False,
                 default: Any = None, has_default: bool = False):
        super().__init__(name or f"Placeholder_{next(_ids)}")
        self.dtype = dtype
        self.shape = shape
        self.sparse = sparse
        self.default = default
        self.has_default = has_default

    def _compute(self, ctx: "RunContext") -> Any:
        if self.has_default:
            return self.default
        raise InvalidArgumentError(
            f"You must feed a value for placeholder tensor '{self.name}'")


def placeholder(dtype=None, shape=None, name=None) -> Placeholder:
    return Placeholder(dtype, shape, name)


def sparse_placeholder(dtype=None, shape=None, name=None) -> Placeholder:
    return Placeholder(dtype, shape, name, sparse=True)


def placeholder_with_default(value, shape=None, name=None) -> Placeholder:
    return Placeholder(None, shape, name, default=value, has_default=True)


class Graph:
    """tf.Graph: here only the owner of a variable collection (TF's GLOBAL_VARIABLES), so that
    global_variables() / global_variables_initializer() cover the variables of one graph, not
    every model the process ever built.  Variables join the default graph at creation."""

    def __init__(self):
        self._variables: list = []  # weak references, in creation order

    @contextlib.contextmanager
    def as_default(self):
        global _DEFAULT
        prev, _DEFAULT = _DEFAULT, self
        try:
            yield self
        finally:
            _DEFAULT = prev


_DEFAULT = Graph()


def get_default_graph() -> Graph:
    return _DEFAULT


def reset_default_graph() -> None:
    """tf.reset_default_graph: later variables go to a fresh graph."""
    global _DEFAULT
    _DEFAULT = Graph()


class Variable(Node):
    """A device-resident parameter.  `value` is a view into a weight stack owned by the
    model, so loading a new value never moves the buffer the kernels were prepared with.
    `initializer` draws a fresh value (host numpy) — what global_variables_initializer runs."""

    def __init__(self, tensor: torch.Tensor, name: str, initializer: Optional[Callable[[], Any]] = None):
        super().__init__(name)
        self.tensor = tensor
        self.initializer = initializer
        _DEFAULT._variables.append(weakref.ref(self))

    @property
    def shape(self):
        return tuple(self.tensor.shape)

    def _compute(self, ctx: "RunContext") -> Any:
        return self.tensor

    def load(self, value, session=None) -> None:
        """tf.Variable.load: assign a new value (same shape)."""
        v = torch.as_tensor(np.asarray(value, dtype=np.float32))
        if tuple(v.shape) != self.shape:
            raise ValueError(f"{self.name}: shape {tuple(v.shape)} != {self.shape}")
        with torch.no_grad():
            self.tensor.copy_(v.to(self.tensor.device))

    def eval(self, session=None) -> np.ndarray:
        return self.tensor.detach().cpu().numpy()


class RunContext:
    def __init__(self, session: "Session", feeds: Dict[Node, Any], training: bool = False):
        self.session = session
        self.feeds = feeds
        self.cache: Dict[Any, Any] = {}
        self.training = training

    def is_fed(self, node: Node) -> bool:
        return node in self.feeds

    def value(self, node: Node) -> Any:
        """Evaluate a node (memoised per run); a fed node returns its feed."""
        if node in self.feeds:
            return self.feeds[node]
        key = ("node", node._id)
        if key not in self.cache:
            self.cache[key] = node._compute(self)
        return self.cache[key]


def _to_numpy(v: Any) -> Any:
    if v is None:
        return None
    if isinstance(v, torch.Tensor):
        return v.detach().cpu().numpy()
    if isinstance(v, (list, tuple)):
        return type(v)(_to_numpy(x) for x in v)
    if isinstance(v, (int, float, bool)):
        return np.asarray(v)[()]
    return v


class Session:
    """tf.Session stand-in.  `config` is accepted and ignored (thread pools are irrelevant:
    the work runs on the device).  The session owns the device caches (uploaded graphs,
    forward plans) of the models it runs."""

    def __init__(self, target: str = "", graph=None, config=None, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("decagon_amd.Session needs a HIP device (MI355X); none visible")
        self.device = (torch.device("cuda", torch.cuda.current_device()) if device is None
                       else torch.device(device))
        self.caches: Dict[Any, Any] = {}
        self._closed = False

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self) -> None:
        self.caches.clear()
        self._closed = True

    def invalidate_feeds(self) -> None:
        """Forget every cached feed conversion, device graph and plan (after changing a fed
        array's contents in place — which the read-only marking otherwise refuses)."""
        for name in ("host_csr", "features", "dgraph", "plans"):
            self.caches.pop(name, None)

    def reset_optimizer_slots(self) -> None:
        """Drop the optimizer state this session holds (Adam m / v / beta powers): the next
        opt_op starts from step 1, as after TF's variable initializer."""
        for key in [k for k in self.caches if isinstance(k, tuple) and k and k[0] == "adam"]:
            del self.caches[key]

    def run(self, fetches, feed_dict: Optional[Dict] = None):
        if self._closed:
            raise RuntimeError("Attempted to use a closed Session.")
        feeds = dict(feed_dict or {})
        for k in feeds:
            if not isinstance(k, Node):
                raise TypeError(f"feed_dict key {k!r} is not a graph node")

        def any_training(f) -> bool:
            if isinstance(f, Node):
                return bool(getattr(f, "training", False))
            if isinstance(f, dict):
                return any(any_training(v) for v in f.values())
            if isinstance(f, (list, tuple)):
                return any(any_training(x) for x in f)
            return False

        ctx = RunContext(self, feeds, training=any_training(fetches))

        def ev(f):
            if f is None:
                return None
            if isinstance(f, Operation):
                ctx.value(f)
                return None
            if isinstance(f, Node):
                return ctx.value(f)
            if isinstance(f, dict):
                return {k: ev(v) for k, v in f.items()}
            if isinstance(f, (list, tuple)):
                return type(f)(ev(x) for x in f)
            raise TypeError(f"cannot fetch {type(f).__name__}")

        out = ev(fetches)
        torch.cuda.current_stream().synchronize()
        # a sharded plan's peer exchange: a timed-out wait raises here, at this run's
        # synchronisation, not silently in a later step (PeerExchange.check)
        for v in list(ctx.cache.values()):
            peer = getattr(v, "peer", None)
            if peer is not None:
                peer.check()

        def conv(v):
            if isinstance(v, dict):
                return {k: conv(x) for k, x in v.items()}
            if isinstance(v, list):
                return [conv(x) for x in v]
            if isinstance(v, tuple):
                return tuple(conv(x) for x in v)
            return _to_numpy(v)

        return conv(out)


# dtype names accepted by placeholder() (the reference passes tf.int32 / tf.float32,
# main.py:93-106); only used for documentation, values are converted at feed time
int32 = "int32"
float32 = "float32"


@contextlib.contextmanager
def name_scope(name: str):
    """tf.name_scope (main.py:268): a naming scope; node names are not part of the contract."""
    yield name


def global_variables() -> list:
    """The default graph's live Variables, in creation order (tf.global_variables)."""
    reg = _DEFAULT._variables
    live = [r() for r in reg]
    reg[:] = [r for r, v in zip(list(reg), live) if v is not None]
    return [v for v in live if v is not None]


def global_variables_initializer() -> Operation:
    """tf.global_variables_initializer (main.py:286, DecagonTrainer.py:49): running it
    re-draws the variables of the default graph that existed when it was created — as TF's
    op groups the initializers of the collection at creation — from their initializers
    (glorot, inits.py:5-12 — in place, so the prepared kernels keep their buffers), and resets
    the optimizer slots the session holds (Adam's m, v and beta powers are TF variables too).
    Variables are also initialised at construction, so a model is usable without running it."""
    refs = [weakref.ref(v) for v in global_variables()]

    def fn(ctx):
        for r in refs:
            v = r()
            if v is not None and v.initializer is not None:
                v.load(v.initializer())
        ctx.session.reset_optimizer_slots()
        return None
    return Operation("init", fn)
