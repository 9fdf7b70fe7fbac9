"""Per-shape GEMM device time of one eager training step from a rocprofv3 kernel trace (no host gaps).

tools/gemm_profile.py --order ORDER.tsv records the profiled step's GEMM launches in launch order with
HIP events around each; for small GEMMs those events also time the host's launch latency (the GPU idles
between the two events while ctypes prepares the launch).  Run the same command under
`rocprofv3 --kernel-trace --output-format csv -d DIR`, then
    python tools/gemm_shapes_trace.py DIR ORDER.tsv > profiles/<name>.txt
maps the last gemm_glds_kernel dispatches of the trace onto the launches (conv2_dgrad: 4 dispatches, one
per parity class) and charges each split-K reduction to the GEMM dispatched before it."""
import ast
import collections
import csv
import glob
import os
import sys


def main():
    d, order = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    launches = []
    for line in open(order):
        fl, ev_ms, key = line.rstrip("\n").split("\t")
        launches.append((float(fl), float(ev_ms), ast.literal_eval(key)))
    need = sum(4 if k[-1] in ("conv2_dgrad", "conv2_dgrad_c1fold") else 1 for _, _, k in launches)
    # GEMM dispatches, each with the split-K reduction(s) that follow it
    gem = []
    for s, e, name in rows:
        if "gemm_glds_kernel" in name:
            gem.append([e - s])
        elif "splitk_reduce" in name and gem:
            gem[-1].append(e - s)
    if len(gem) < need:
        sys.exit(f"trace holds {len(gem)} GEMM dispatches, the order file needs {need}")
    gem = gem[len(gem) - need:]
    shapes = collections.OrderedDict()
    i = 0
    for fl, ev_ms, key in launches:
        k = 4 if key[-1] in ("conv2_dgrad", "conv2_dgrad_c1fold") else 1
        ns = sum(sum(g) for g in gem[i:i + k])
        nk = sum(g[0] for g in gem[i:i + k])
        i += k
        s = shapes.setdefault(key, [0, 0.0, 0.0, 0.0, 0.0])
        s[0] += 1
        s[1] += ns / 1e6
        s[2] += nk / 1e6
        s[3] += ev_ms
        s[4] += fl
    tot_dev = sum(v[1] for v in shapes.values())
    tot_fl = sum(v[4] for v in shapes.values())
    print(f"# {len(launches)} GEMM launches ({need} dispatches) of one eager step: device {tot_dev:.2f} ms incl. "
          f"split-K reductions, {tot_fl / tot_dev / 1e9:.1f} TFLOP/s; HIP-event sum {sum(v[3] for v in shapes.values()):.2f} ms")
    print(f"{'shape (mode_a, mode_b, M, N, K, batch)':48s} {'n':>4} {'device ms':>10} {'kernel ms':>10} "
          f"{'event ms':>9} {'TF/s dev':>9}")
    for key, (n, dev, ker, ev, fl) in sorted(shapes.items(), key=lambda kv: -kv[1][1]):
        print(f"{str(key):48s} {n:4d} {dev:10.3f} {ker:10.3f} {ev:9.3f} {fl / dev / 1e9:9.1f}")


if __name__ == "__main__":
    main()
