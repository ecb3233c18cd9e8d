"""Parameter initialisers (decagon/deep/inits.py:5-24).

Draws happen once on the host from a seeded generator and are uploaded; the values are
then owned by device weight stacks.  `set_random_seed` plays tf.set_random_seed's role.
"""
from __future__ import annotations

import numpy as np

_rng = np.random.default_rng(0)


def set_random_seed(seed: int) -> None:
    global _rng
    _rng = np.random.default_rng(seed)


def glorot_array(input_dim: int, output_dim: int) -> np.ndarray:
    """U(-r, r), r = sqrt(6 / (in + out))  (weight_variable_glorot, inits.py:5-12)."""
    r = np.sqrt(6.0 / (input_dim + output_dim))
    return _rng.uniform(-r, r, size=(input_dim, output_dim)).astype(np.float32)


def zeros_array(input_dim: int, output_dim: int) -> np.ndarray:
    return np.zeros((input_dim, output_dim), np.float32)


def ones_array(input_dim: int, output_dim: int) -> np.ndarray:
    return np.ones((input_dim, output_dim), np.float32)
