#!/usr/bin/env python
"""Per-kernel PMC summary of rocprofv3 --pmc runs (one directory per counter pass) for the hand kernels."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

KEYS = ("fa_", "win_attn", "bn_", "norm_", "adamw")


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            full = r.get("Kernel_Name", "?")
            m = re.search(r"((?:fa_|win_attn|bn_|norm_|adamw)\w*)(<[^()]*>)?", full)
            if m:
                acc[(m.group(1) + (m.group(2) or ""))[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    out = sys.argv[1]
    merged = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(out, "pmc_*"))):
        for k, cs in load(d).items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
    for k in sorted(merged):
        c = merged[k]
        line = [k]
        if c.get("SQ_BUSY_CYCLES") and c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            line.append(f"MFMA_busy/SQ_busy={c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1.0, c['SQ_BUSY_CYCLES']):.3f}")
        if c.get("SQ_INSTS_LDS"):
            line.append(f"LDS_bank_conflict_cycles/LDS_inst={c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_INSTS_LDS']:.3f}")
        if c.get("SQ_WAVE_CYCLES"):
            line.append(f"wait_any={c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']:.2f} "
                        f"issue_stall={c.get('SQ_WAIT_INST_ANY', 0) / c['SQ_WAVE_CYCLES']:.2f} "
                        f"active={c.get('SQ_ACTIVE_INST_ANY', 0) / c['SQ_WAVE_CYCLES']:.2f}")
        line.append("raw=" + ", ".join(f"{n}={v:.3g}" for n, v in sorted(c.items())))
        print(" | ".join(line))


if __name__ == "__main__":
    main()
