"""decagon_amd — MI355X-native Decagon GCN forward and edge decoders.

Drop-in for the TF1 hot path of jrectorb/decagon (decagon/deep/layers.py, model.py,
optimizer.py): the same DecagonModel / DecagonOptimizer surface over hand-written gfx950
HIP kernels (libdecagon_hip.so, C ABI in include/decagon_hip.h).  See DESIGN.md.
"""
from __future__ import annotations

__version__ = "0.1.0"

from . import flags  # noqa: F401
from .flags import FLAGS  # noqa: F401
from .graph import (Graph, InvalidArgumentError, Node, Operation, Placeholder, Session, Variable,  # noqa: F401
                    float32, get_default_graph, global_variables, global_variables_initializer, int32,
                    name_scope, placeholder, reset_default_graph,
                    placeholder_with_default, sparse_placeholder)
from .inits import set_random_seed  # noqa: F401
from .layers import (BilinearDecoder, DEDICOMDecoder, DistMultDecoder,  # noqa: F401
                     GraphConvolutionMulti, GraphConvolutionSparseMulti, InnerProductDecoder,
                     MultiLayer, dropout_sparse, get_layer_uid, relu, sigmoid)
from .model import DecagonModel, Model  # noqa: F401
from .optimizer import DecagonOptimizer, gather_cols  # noqa: F401
from .sparse import SparseTensorValue, preprocess_graph, sparse_to_tuple  # noqa: F401


def construct_placeholders(edge_types):
    """The placeholder dict of main.py:93-108 / DecagonDataSet.py:84-120."""
    ph = {
        "batch": placeholder("int32", name="batch"),
        "batch_edge_type_idx": placeholder("int32", shape=(), name="batch_edge_type_idx"),
        "batch_row_edge_type": placeholder("int32", shape=(), name="batch_row_edge_type"),
        "batch_col_edge_type": placeholder("int32", shape=(), name="batch_col_edge_type"),
        "degrees": placeholder("int32", name="degrees"),
        "dropout": placeholder_with_default(0.0, shape=(), name="dropout"),
    }
    ph.update({"adj_mats_%d,%d,%d" % (i, j, k): sparse_placeholder("float32", name="adj_mats_%d,%d,%d" % (i, j, k))
               for i, j in edge_types for k in range(edge_types[i, j])})
    ph.update({"feat_%d" % i: sparse_placeholder("float32", name="feat_%d" % i) for i, _ in edge_types})
    return ph


def library_path():
    from ._build import lib_path
    return lib_path()
