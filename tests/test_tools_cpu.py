"""Measurement tooling on CPU: tools/gemm_shapes_trace.py maps a kernel trace's GEMM dispatches onto the
launch-order record of tools/gemm_profile.py (conv2_dgrad = 4 dispatches, split-K reductions charged to
the GEMM before them, only the trace's last dispatches used)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(tmp_path, rows):
    d = tmp_path / "prof"
    d.mkdir()
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 0
        for name, dur in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur})
            t += dur + 10
    return d


def test_gemm_shapes_trace_maps_dispatches(tmp_path):
    g = "void espg::gemm_glds_kernel<0, 1, 128, false, 8, 3, 128>(espg::GemmArgs)"
    rows = [(g, 999_000),  # a warm-up step's dispatch: not part of the profiled step
            (g, 10_000), ("splitk_reduce4_kernel(espg::GemmArgs)", 4_000),
            ("ln_fwd_kernel<4>", 7_000),
            (g, 1_000), (g, 2_000), (g, 3_000), (g, 4_000),
            (g, 20_000)]
    d = _trace(tmp_path, rows)
    order = tmp_path / "order.tsv"
    order.write_text("2000000\t0.02\t(0, 1, 100, 100, 100, 1, 'bp')\n"
                     "8000000\t0.012\t(4, 1, 1000, 64, 576, 1, 'conv2_dgrad')\n"
                     "2000000\t0.03\t(0, 1, 100, 100, 100, 1, 'bp')\n")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gemm_shapes_trace.py"), str(d), str(order)],
                         capture_output=True, text=True, check=True).stdout
    lines = {ln.split(")")[0] + ")": ln for ln in out.splitlines() if ln.startswith("(")}
    bp = lines["(0, 1, 100, 100, 100, 1, 'bp')"].split()
    cv = lines["(4, 1, 1000, 64, 576, 1, 'conv2_dgrad')"].split()
    # (0,1,...): two launches, device = 10 + 4 (reduction) + 20 us, kernel = 30 us, events 0.05 ms
    assert bp[-5] == "2" and float(bp[-4]) == 0.034 and float(bp[-3]) == 0.030 and float(bp[-2]) == 0.05
    # conv2_dgrad: one launch of 4 class dispatches, 1 + 2 + 3 + 4 us
    assert cv[-5] == "1" and float(cv[-4]) == 0.010 and float(cv[-3]) == 0.010
    assert "12 dispatches" not in out and "(6 dispatches)" in out
