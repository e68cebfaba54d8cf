"""Access to the native host runtime (``_pdt_runtime``, pybind11/C++; see csrc/runtime/runtime.cpp)."""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

_rt = None
_err = None


def runtime():
    """The ``_pdt_runtime`` module, building it in-tree on first use if needed (None if impossible)."""
    global _rt, _err
    if _rt is not None:
        return _rt
    alt = os.environ.get("PDT_RUNTIME_DIR")
    if alt:       # an out-of-tree build (e.g. the ASan/UBSan one of tests/test_sanitizers_cpu.py), loaded loudly
        from .. import _build
        path = os.path.join(alt, os.path.basename(_build.runtime_ext_path()))
        spec = importlib.util.spec_from_file_location("pytorch_distributedtraining_amd._pdt_runtime", path)
        if spec is None or not os.path.exists(path):
            raise RuntimeError(f"PDT_RUNTIME_DIR={alt}: no runtime module at {path}")
        _rt = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(_rt)
        sys.modules["pytorch_distributedtraining_amd._pdt_runtime"] = _rt
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
