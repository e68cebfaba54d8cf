#!/usr/bin/env python
"""Kernel statistics from a rocprofv3 rocpd database (the default output of `rocprofv3 --kernel-trace` on
ROCm 7.x: <name>_results.db, SQLite).

Writes the rocprofv3 kernel_stats.csv columns (Name, Calls, TotalDurationNs, AverageNs, Percentage) and,
with --step-kernel, restricts the table to the timed window of a bench run: from the end of the
`--skip`-th dispatch of the once-per-step kernel (e.g. the fused AdamW) to the end of its last dispatch,
so warm-up, model construction and teardown are excluded; durations are then also reported per step.

  python scripts/prof_db_stats.py gpurun_out/prof_r3/flagship_results.db --step-kernel adamw_mt_kernel \
      --skip 2 -o profiles/r3_gpt2_1.3b_fsdp1_mb96_kernel_stats.csv
"""
import argparse
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = re.sub(r"\s+", " ", name)
    return name if len(name) <= 240 else name[:237] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("-o", "--out", default="-")
    ap.add_argument("--step-kernel", default="")
    ap.add_argument("--skip", type=int, default=0, help="once-per-step dispatches to skip (warm-up steps)")
    ap.add_argument("--top", type=int, default=0)
    ap.add_argument("--gaps", type=int, default=0, help="also report idle time between dispatches (N largest)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    lo, hi, steps = None, None, None
    if a.step_kernel:
        marks = [r for r in rows if a.step_kernel in r[0]]
        if len(marks) <= a.skip:
            sys.exit(f"only {len(marks)} dispatches of {a.step_kernel}")
        lo, hi = marks[a.skip - 1][2] if a.skip else rows[0][1] - 1, marks[-1][2]
        steps = len(marks) - a.skip
        rows = [r for r in rows if lo < r[1] and r[2] <= hi]
    agg = {}
    for name, _s, _e, d in rows:
        e = agg.setdefault(name, [0, 0])
        e[0] += 1
        e[1] += d
    total = sum(v[1] for v in agg.values())
    out = sys.stdout if a.out == "-" else open(a.out, "w", newline="")
    w = csv.writer(out)
    hdr = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"]
    if steps:
        hdr += ["Steps", "MsPerStep"]
    w.writerow(hdr)
    items = sorted(agg.items(), key=lambda kv: -kv[1][1])
    if a.top:
        items = items[:a.top]
    for name, (n, d) in items:
        row = [short(name), n, d, round(d / n, 1), round(100.0 * d / total, 3)]
        if steps:
            row += [steps, round(d / steps / 1e6, 3)]
        w.writerow(row)
    if steps:
        span = (hi - lo) / 1e6
        print(f"# window {span:.1f} ms over {steps} steps = {span / steps:.1f} ms/step; kernel time "
              f"{total / 1e6 / steps:.1f} ms/step", file=sys.stderr)
    if a.gaps:
        # idle time between consecutive dispatches (one stream: the next kernel starts after the previous ends)
        gaps, last_end, last_name = [], None, None
        for name, st, en, _d in rows:
            if last_end is not None and st > last_end:
                gaps.append((st - last_end, last_name, name))
            if last_end is None or en > last_end:
                last_end, last_name = en, name
        tot = sum(g[0] for g in gaps)
        print(f"# idle between dispatches: {tot / 1e6 / max(steps or 1, 1):.2f} ms/step over {len(gaps)} gaps",
              file=sys.stderr)
        for g, before, after in sorted(gaps, reverse=True)[:a.gaps]:
            print(f"#   {g / 1e3:9.1f} us  after {short(before)[:70]}  before {short(after)[:70]}", file=sys.stderr)


if __name__ == "__main__":
    main()
