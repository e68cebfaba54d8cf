#!/usr/bin/env python
"""Run the hand weight-gradient GEMM on the GPT-2 1.3B fc1 shape a few times (rocprofv3 PMC target)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributedtraining_amd.ops.linear import hip_wgrad  # noqa: E402

dy = torch.randn(65536, 8192, device="cuda", dtype=torch.bfloat16)
x = torch.randn(65536, 2048, device="cuda", dtype=torch.bfloat16)
for _ in range(int(os.environ.get("ITERS", "4"))):
    hip_wgrad(dy, x, splits=1)
torch.cuda.synchronize()
print("ok")
