"""K-sweep of the MFMA GEMM at a fixed M x N (per-tile vs per-slab cost)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.gemm_bench import run  # noqa: E402

if __name__ == "__main__":
    M, N = int(sys.argv[1]), int(sys.argv[2])
    modes = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (0, 1)
    for k in (64, 128, 256, 512, 1024, 2048):
        ms, tf = run(modes[0], modes[1], M, N, k, 1)
        print(f"M={M} N={N} K={k:5d}  {ms * 1e3:8.1f} us  {tf:6.1f} TF/s", flush=True)
