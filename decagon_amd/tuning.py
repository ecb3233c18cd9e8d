"""Plan-construction policy knobs: the one place the package reads its DG_* environment.

The C ABI (include/decagon_hip.h) reads no environment: every kernel choice is an argument.
Above it, the plan builders (engine.py, sharding.py, scorer.py, train.py, runtime.py) pick
layouts and launch forms by measured policy — window counts, staged binning, which launch form
finishes a row block — and a handful of those policies can be overridden for A/B runs through
DG_* variables.  Every such read goes through `knob`, which records the name, default and value
read, so `overrides()` lists exactly the knobs that differed from their defaults in this
process; bench.py prints that on its JSON line, so a measured number always says which
non-default policy it ran (an empty object: the shipped defaults).  tests/test_cpu_host.py
checks that no other module of the package reads DG_* variables directly.
"""
from __future__ import annotations

import os
from typing import Dict, Tuple, TypeVar, Union

T = TypeVar("T", bool, int, float, str)

# name -> (default, last value read)
_READ: Dict[str, Tuple[Union[bool, int, float, str], Union[bool, int, float, str]]] = {}
_FALSE = frozenset({"0", "false", "no", "off"})
_TRUE = frozenset({"1", "true", "yes", "on"})


def knob(name: str, default: T) -> T:
    """The value of DG_* variable `name` (its type is `default`'s; a bool knob takes
    0/false/no/off or 1/true/yes/on, case-insensitive, and raises ValueError on anything else),
    or `default` when unset.  Read at the call, so a knob consulted
    per plan follows the environment of that moment (tests set them with monkeypatch)."""
    if not name.startswith("DG_"):
        raise ValueError(f"tuning knobs are DG_* variables, got {name!r}")
    raw = os.environ.get(name)
    if raw is None:
        val = default
    elif isinstance(default, bool):
        low = raw.strip().lower()
        if low in _FALSE:
            val = False
        elif low in _TRUE:
            val = True
        else:
            raise ValueError(f"{name}={raw!r}: a switch takes one of {sorted(_FALSE | _TRUE)}")
    else:
        val = type(default)(raw)
    _READ[name] = (default, val)
    return val


def overrides() -> Dict[str, Union[bool, int, float, str]]:
    """The knobs read so far whose value differed from the default."""
    return {k: v for k, (d, v) in sorted(_READ.items()) if v != d}


def read() -> Dict[str, Tuple[Union[bool, int, float, str], Union[bool, int, float, str]]]:
    """Every knob read so far: name -> (default, value)."""
    return dict(_READ)
