"""Full names of the torch (at::native) kernels in the steady state of a rocprofv3 kernel trace, with per-step time,
call count and grid -- to find which framework op launches them.

    python scripts/trace_torch_kernels.py run_kernel_trace.csv --marker adamw_mt_kernel --last 2
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="adamw_mt_kernel")
    ap.add_argument("--last", type=int, default=2)
    ap.add_argument("--match", default="at::native", help="substring a kernel name must contain ('' = all)")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--width", type=int, default=400, help="kernel-name characters kept (groups by that prefix)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [r for r in rows if a.marker in r["Kernel_Name"]]
    t0, t1 = int(marks[-a.last - 1]["End_Timestamp"]), int(marks[-1]["End_Timestamp"])
    rows = [r for r in rows if t0 < int(r["Start_Timestamp"]) <= t1]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        if a.match not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"][:a.width], r["Grid_Size_X"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(t for _, t in agg.values())
    span = (t1 - t0) / 1e6
    print(f"matched kernels: {tot / a.last / 1e3:.3f} ms/step busy of {span / a.last:.3f} ms/step wall")
    for (name, g), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / a.last / 1e3:7.3f} ms/step n/step={n / a.last:6.1f} grid={g} {name}")


if __name__ == "__main__":
    main()
