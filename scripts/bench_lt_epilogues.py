#!/usr/bin/env python
"""Which hipBLASLt epilogue / type / transpose combinations have algorithms on this GPU (gfx950).
Result of the round-2 probe (profiles/r2_hipblaslt_epilogue_probe.txt): bias / gelu_bias / bgrada / bgradb
yes; gelu_aux_bias / dgelu / dgelu_bgrad no -- so the MLP keeps its hand GELU kernels and only the bias
gradients move into the weight-gradient GEMMs."""
import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops import _lib  # noqa: E402

torch.cuda.init()
lib = _lib.require()
names = {0: "none", 1: "bias", 2: "gelu_aux_bias", 3: "dgelu_bgrad", 4: "gelu_bias", 5: "dgelu", 6: "bgradb",
         7: "bgrada"}
m, n, k = 2048, 6144, 32768
for epi, tr, bdt in itertools.product((0, 6, 7, 2, 3), (0, 1, 2, 3), (1, 0)):
    r = lib.pdt_lt_probe(epi, tr, m, n, k, 1, bdt, 1)
    print(f"{names[epi]:14s} transA={tr & 1} transB={tr >> 1} bias={'bf16' if bdt else 'f32'} -> {r}", flush=True)
