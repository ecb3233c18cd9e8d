"""`tf.app.flags` stand-in: the model reads FLAGS.hidden1 / hidden2 / learning_rate inside
its constructors (decagon/deep/model.py:68, :80-81, :95; decagon/deep/optimizer.py:111),
and drivers define them with DEFINE_* (main.py:227-238, DecagonDataSet.py:122-165).

Defaults are main.py's values so that a model built without a driver matches config S.
"""
from __future__ import annotations

from typing import Any, Dict


class _FlagValues:
    def __init__(self) -> None:
        object.__setattr__(self, "_values", {})
        object.__setattr__(self, "_help", {})

    def __getattr__(self, name: str) -> Any:
        vals: Dict[str, Any] = object.__getattribute__(self, "_values")
        if name in vals:
            return vals[name]
        raise AttributeError(f"flag {name!r} is not defined")

    def __setattr__(self, name: str, value: Any) -> None:
        self._values[name] = value

    def __contains__(self, name: str) -> bool:
        return name in self._values

    def _define(self, name: str, default: Any, help_str: str, cast) -> None:
        if name in self._values and name in self._help:
            raise ValueError(f"flag {name!r} already defined")  # as absl does
        self._values[name] = cast(default) if default is not None else None
        self._help[name] = help_str

    def flag_values_dict(self) -> Dict[str, Any]:
        return dict(self._values)


FLAGS = _FlagValues()


def DEFINE_integer(name, default, help_str=""):
    FLAGS._define(name, default, help_str, int)


def DEFINE_float(name, default, help_str=""):
    FLAGS._define(name, default, help_str, float)


def DEFINE_boolean(name, default, help_str=""):
    FLAGS._define(name, default, help_str, bool)


def DEFINE_string(name, default, help_str=""):
    FLAGS._define(name, default, help_str, str)


DEFINE_bool = DEFINE_boolean

# main.py:229-238 defaults (not "defined" yet, so drivers may DEFINE_* them again)
for _k, _v in dict(neg_sample_size=1, learning_rate=0.001, epochs=50, hidden1=64, hidden2=32,
                   weight_decay=0.0, dropout=0.1, max_margin=0.1, batch_size=512, bias=True).items():
    FLAGS._values[_k] = _v
