#!/usr/bin/env python
"""Per-kernel PMC summary of rocprofv3 --pmc runs (one directory per counter pass) for the hand kernels.

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128): the MFMA counter sums busy cycles
(32 per v_mfma_f32_32x32x16_bf16) over all 1,024 SIMDs, while rocprofv3 reports GRBM_GUI_ACTIVE summed over
the 8 XCDs -- so GRBM/8 is the kernel's cycle count and 1,024 x GRBM/8 = 128 x GRBM the SIMD-cycles
available (MI355X_MICROARCH.md, "s_memtime tick vs SQ PMC units" and "DVFS give-back").  A value of 1.0
means every SIMD issued MFMAs back to back for the whole dispatch.

    python scripts/summarize_pmc.py gpurun_out                # pmc_* pass directories
    python scripts/summarize_pmc.py --from-summary old.txt    # re-derive from a summary's raw= fields
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

KEYS = ("fa_", "win_attn", "bn_", "norm_", "adamw", "swin_mlp", "fp8_cast", "wgrad_kernel", "gemm_kernel", "Cijk")


def load(d):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            full = r.get("Kernel_Name", "?")
            m = re.search(r"((?:fa_|win_attn|bn_|norm_|adamw|swin_mlp|fp8_cast|wgrad_kernel|gemm_kernel|gemm_asm|Custom_Cijk|Cijk)\w*)(<[^()]*>)?", full)
            if m:
                acc[(m.group(1) + (m.group(2) or ""))[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


SIMD_CYCLES_PER_GRBM = 128     # 1,024 SIMDs / 8 XCDs (GRBM_GUI_ACTIVE is summed over the XCDs)


def derived(c):
    out = []
    if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
        out.append(f"MFMA_util={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (SIMD_CYCLES_PER_GRBM * c['GRBM_GUI_ACTIVE']):.3f}")
    if c.get("SQ_INSTS_MFMA") and c.get("SQ_INSTS_VALU") is not None:
        out.append(f"VALU_per_MFMA={(c['SQ_INSTS_VALU'] - c['SQ_INSTS_MFMA']) / c['SQ_INSTS_MFMA']:.2f}")
    if c.get("SQ_INSTS_MFMA") and c.get("SQ_INSTS_LDS") is not None:
        out.append(f"LDS_per_MFMA={c['SQ_INSTS_LDS'] / c['SQ_INSTS_MFMA']:.2f}")
    return out


def from_summary(path):
    for ln in open(path):
        if "raw=" not in ln:
            continue
        name = ln.split(" | ")[0]
        raw = dict(kv.split("=") for kv in ln.split("raw=")[1].strip().split(", "))
        c = {k: float(v) for k, v in raw.items()}
        print(" | ".join([name] + derived(c) + [f"raw=MFMA_BUSY={c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0):.3g}, "
                                                 f"GRBM_GUI_ACTIVE={c.get('GRBM_GUI_ACTIVE', 0):.3g}"]))


def main():
    if sys.argv[1] == "--from-summary":
        return from_summary(sys.argv[2])
    out = sys.argv[1]
    merged = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(out, "pmc_*"))):
        for k, cs in load(d).items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
    for k in sorted(merged):
        c = merged[k]
        line = [k]
        line.extend(derived(c))
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
