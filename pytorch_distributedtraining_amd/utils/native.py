"""Access to the native host runtime (``_pdt_runtime``, pybind11/C++; see csrc/runtime/runtime.cpp)."""
from __future__ import annotations

import importlib

_rt = None
_err = None


def runtime():
    """The ``_pdt_runtime`` module, building it in-tree on first use if needed (None if impossible)."""
    global _rt, _err
    if _rt is not None:
        return _rt
    try:
        _rt = importlib.import_module("pytorch_distributedtraining_amd._pdt_runtime")
    except ImportError as e:
        try:
            from .. import _build

            _build.build_runtime()
            _rt = importlib.import_module("pytorch_distributedtraining_amd._pdt_runtime")
        except Exception as e2:  # pragma: no cover
            _err = (e, e2)
            return None
    return _rt


def require_runtime():
    rt = runtime()
    if rt is None:
        raise RuntimeError(f"native runtime _pdt_runtime unavailable: {_err}")
    return rt
