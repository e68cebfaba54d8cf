"""The ctypes signatures in ops/_lib.py must match the C declarations of every exported kernel entry
point (a mismatch corrupts arguments silently on the GPU)."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ctypes_signatures_match_hip_sources():
    from pytorch_distributedtraining_amd.ops._lib import _SIGS
    src = "".join(open(f).read() for f in glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    decl = {m.group(1): len([a for a in m.group(2).split(",") if a.strip()])
            for m in re.finditer(r"PDT_API (?:int|int64_t|long long) (pdt_\w+)\(([^)]*)\)", src, re.S)}
    assert set(decl) == set(_SIGS), (set(decl) ^ set(_SIGS))
    for k, v in _SIGS.items():
        assert decl[k] == len(v), f"{k}: C has {decl[k]} args, ctypes {len(v)}"
    from pytorch_distributedtraining_amd.ops._lib import _RET64
    wide = set(re.findall(r"PDT_API (?:int64_t|long long) (pdt_\w+)\(", src))
    assert wide == set(_RET64), wide ^ set(_RET64)     # 64-bit returns need a c_int64 restype
