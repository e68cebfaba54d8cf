#!/usr/bin/env python
"""World 1 vs world 2 (two ranks sharing cuda:0 over gloo) FSDP state after 3 steps of GPT-2 tiny: per parameter
the max |diff| and the count of elements outside tests/test_gpu_multiproc.py's tolerance."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dist_utils import run_workers  # noqa: E402
from test_gpu_multiproc import _train_fsdp  # noqa: E402

if __name__ == "__main__":
    strategy = sys.argv[1] if len(sys.argv) > 1 else "full_shard"
    (l1, sd1), = run_workers(_train_fsdp, 1, 3, strategy)
    (l2, sd2), _ = run_workers(_train_fsdp, 2, 3, strategy)
    print("fold", os.environ.get("PDT_FOLD_PROJ_BIAS", "1"), strategy, "losses", l1, l2)
    for k in sd1:
        d = (sd1[k] - sd2[k]).abs()
        bad = (d > 3e-3 + 3e-2 * sd2[k].abs()).sum().item()
        print(f"{k:40s} max|d|={d.max().item():.2e} bad={bad}/{d.numel()}")
