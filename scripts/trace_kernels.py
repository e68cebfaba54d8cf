"""Summarise a rocprofv3 kernel trace: per (kernel, grid) call count and average duration.

    python scripts/trace_kernels.py gpurun_out/prof/bench_kernel_trace.csv [--match Cijk] [--top 40]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
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
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t/1e3:9.2f} ms {100*t/tot:5.1f}% n={n:5d} avg={t/n:9.1f}us grid={k[1]}x{k[2]}x{k[3]} "
              f"wg={k[4]} {k[0]}")


if __name__ == "__main__":
    main()
