#!/usr/bin/env python
"""Communication / compute overlap from a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

For every trace file (one per process: run rocprofv3 with ``-o %pid%_name`` when several ranks are traced)
it reports the busy time of communication
kernels (xGMI collectives: names containing ``xgmi``; RCCL: ``ncclDevKernel`` / ``rccl``), the busy time of
compute kernels (everything else), which queues/streams each class ran on, and how much communication time
ran while a compute kernel of the same process was also running (interval intersection).

    python scripts/trace_overlap.py gpurun_out/prof_x2/*_kernel_trace.csv
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict


def _union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _measure(iv):
    return sum(b - a for a, b in iv)


def _intersect(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def is_comm(name: str) -> bool:
    n = name.lower()
    return "xgmi" in n or "nccl" in n or "rccl" in n


def analyse(path):
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(lambda: {"comm": [], "compute": [], "cq": set(), "kq": set(), "gemm": []})
    for r in rows:
        if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
            continue
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = per[path]
        q = (r["Queue_Id"], r["Stream_Id"])
        if is_comm(r["Kernel_Name"]):
            d["comm"].append((t0, t1))
            d["cq"].add(q)
        else:
            d["compute"].append((t0, t1))
            d["kq"].add(q)
            if r["Kernel_Name"].startswith("Cijk") or "gemm" in r["Kernel_Name"].lower():
                d["gemm"].append((t0, t1))
    out = []
    for tid, d in per.items():
        if not d["comm"]:
            continue
        c, k, g = _union(d["comm"]), _union(d["compute"]), _union(d["gemm"])
        out.append({"trace": tid, "comm_kernels": len(d["comm"]), "comm_busy_ms": _measure(c) / 1e6,
                    "compute_busy_ms": _measure(k) / 1e6, "comm_under_compute_ms": _intersect(c, k) / 1e6,
                    "comm_under_gemm_ms": _intersect(c, g) / 1e6,
                    "comm_queues": sorted(d["cq"]), "compute_queues": sorted(d["kq"])})
    return out


def main():
    for rec in (r for p in sys.argv[1:] for r in analyse(p)):
        frac = rec["comm_under_compute_ms"] / rec["comm_busy_ms"] if rec["comm_busy_ms"] else 0.0
        print(f"{rec['trace']}: {rec['comm_kernels']} comm kernels, comm busy "
              f"{rec['comm_busy_ms']:.2f} ms, compute busy {rec['compute_busy_ms']:.2f} ms, comm concurrent with "
              f"compute {rec['comm_under_compute_ms']:.2f} ms ({100 * frac:.1f} %), with GEMMs "
              f"{rec['comm_under_gemm_ms']:.2f} ms; comm queues {rec['comm_queues']} vs compute queues "
              f"{rec['compute_queues']}")


if __name__ == "__main__":
    main()
