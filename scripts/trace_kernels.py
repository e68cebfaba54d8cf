"""Summarise a rocprofv3 kernel trace: per (kernel, grid) call count and average duration.

    python scripts/trace_kernels.py gpurun_out/prof/bench_kernel_trace.csv [--match Cijk] [--top 40]
        [--marker adamw_mt_kernel --last 3]

--marker / --last: steady state only -- the kernels after the (last + 1)-th-from-last call of the marker kernel
(one per training step: the optimizer), i.e. the last `last` steps, with times also given per step.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per = 1
    if a.marker and a.last > 0:
        marks = [r for r in rows if a.marker in r["Kernel_Name"]]
        if len(marks) <= a.last:
            raise SystemExit(f"only {len(marks)} {a.marker} calls: cannot isolate the last {a.last} steps")
        t0 = int(marks[-a.last - 1]["End_Timestamp"])
        t1 = int(marks[-1]["End_Timestamp"])
        rows = [r for r in rows if t0 < int(r["Start_Timestamp"]) <= t1]
        per = a.last
        print(f"steady state: last {a.last} steps, {(t1 - t0) / 1e6 / a.last:.2f} ms wall per step (marker to marker)")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        name = r["Kernel_Name"]
        if a.match and a.match not in name:
            continue
        key = (name[:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[key][0] += 1
        agg[key][1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"kernel time: {tot / 1e3 / per:.2f} ms per step")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t/1e3:9.2f} ms {t/1e3/per:8.2f} ms/step {100*t/tot:5.1f}% n={n:5d} avg={t/n:9.1f}us grid={k[1]}x{k[2]}x{k[3]} "
              f"wg={k[4]} {k[0]}")


if __name__ == "__main__":
    main()
