"""Summarise a rocprofv3 --kernel-trace run (CSV dir or rocpd .db): per-kernel time per step and,
for the GEMM kernels, per launch-grid breakdown.  Usage:
    python tools/prof_summary.py <prof_dir> <n_dispatch_steps> [--gemm] > profiles/<name>.txt
n_dispatch_steps = warmup + timed steps of the profiled bench run (all dispatches are counted).
"""
import collections
import csv
import glob
import os
import sqlite3
import sys


def load(d):
    rows = []
    dbs = glob.glob(os.path.join(d, "*.db"))
    if dbs:
        c = sqlite3.connect(dbs[0])
        for name, start, end, gx, gy, gz in c.execute("select name, start, end, grid_x, grid_y, grid_z from kernels"):
            rows.append((name, int(end) - int(start), (gx, gy, gz)))
        return rows
    for f in glob.glob(os.path.join(d, "*kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                         (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])))
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    rows = load(d)
    tot = collections.defaultdict(lambda: [0, 0])
    # the bench's ~200 ms head-start spin before its eager GEMM timing is not part of a step
    rows = [r for r in rows if "spin_kernel" not in r[0]]
    for name, dur, _ in rows:
        t = tot[short(name)]
        t[0] += 1
        t[1] += dur
    total = sum(v[1] for v in tot.values())
    print(f"# rocprofv3 kernel-trace summary of {d} ({steps} steps)")
    print(f"# total kernel time per step: {total / steps / 1e6:.3f} ms")
    print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10} {'avg us':>9}  kernel")
    for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{t / steps / 1e6:9.3f} {100 * t / total:6.2f} {n / steps:10.1f} {t / n / 1e3:9.1f}  {k}")
    # the bench's roofline kernel: every instantiation of the MFMA GEMM family together
    fam = [(n, t) for k, (n, t) in tot.items() if "gemm_glds_kernel" in k]
    red = [(n, t) for k, (n, t) in tot.items() if "splitk_reduce" in k]
    if fam:
        n = sum(f[0] for f in fam)
        t = sum(f[1] for f in fam)
        tr = sum(f[1] for f in red)
        print(f"# family gemm_glds_kernel<*>: {n / steps:.1f} launches/step, {t / steps / 1e6:.3f} ms/step, "
              f"avg {t / n / 1e3:.1f} us per launch; + split-K reductions {tr / steps / 1e6:.3f} ms/step")
    if "--gemm" in sys.argv:
        g = collections.defaultdict(lambda: [0, 0])
        for name, dur, grid in rows:
            if "gemm" in name:
                k = (short(name), grid)
                g[k][0] += 1
                g[k][1] += dur
        print("\n# GEMM launches by (kernel, grid)")
        for (k, grid), (n, t) in sorted(g.items(), key=lambda kv: -kv[1][1])[:40]:
            print(f"{t / steps / 1e6:9.3f} ms/step {n / steps:6.1f}/step avg {t / n / 1e3:8.1f} us  {k} grid={grid}")


if __name__ == "__main__":
    main()
