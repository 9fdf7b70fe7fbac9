"""Prototype split-once bf16x6 GEMM (tools/x6_proto.hip -> tools/libx6proto.so) against the
library's esp_gemm_f32 on the same operands: accuracy vs fp64 and time per launch.
Usage: python tools/x6_proto_bench.py"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from espnet_slurp_amd import kernels as K  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libx6proto.so"))
lib.x6_gemm.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_int] * 2 + \
    [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def case(M, N, Kk, ma, mb):
    g = torch.Generator().manual_seed(M + N + Kk)
    A = torch.randn(M, Kk, generator=g)
    B = torch.randn(Kk, N, generator=g)
    Ad = (A if ma == 0 else A.t().contiguous()).cuda()
    Bd = (B.t().contiguous() if mb == 0 else B).cuda()
    C1 = torch.empty(M, N, device="cuda")
    C2 = torch.empty(M, N, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def proto():
        lib.x6_gemm(M, N, Kk, Ad.data_ptr(), Ad.stride(0), ma, Bd.data_ptr(), Bd.stride(0), mb, C1.data_ptr(), N, st)

    def libg():
        K.gemm(M, N, Kk, Ad, Bd, C2, mode_a=ma, lda=Ad.stride(0), mode_b=mb, ldb=Bd.stride(0), ldc=N)

    t1 = timed(proto)
    t2 = timed(libg)
    ref = A.double() @ B.double()
    den = A.double().abs() @ B.double().abs()
    e1 = ((C1.cpu().double() - ref).abs() / den).max().item()
    e2 = ((C2.cpu().double() - ref).abs() / den).max().item()
    fl = 2.0 * M * N * Kk
    print(f"M={M:6d} N={N:5d} K={Kk:6d} ({ma},{mb})  proto {t1 * 1e3:8.1f} us {fl / t1 / 1e9:6.1f} TF/s err {e1:.2e}"
          f"   lib {t2 * 1e3:8.1f} us {fl / t2 / 1e9:6.1f} TF/s err {e2:.2e}", flush=True)


def main():
    torch.cuda.init()
    for M, N, Kk, ma, mb in [(47872, 1024, 256, 0, 0), (47872, 256, 1024, 0, 0), (47872, 1024, 256, 0, 1),
                             (47872, 256, 1024, 0, 1), (4096, 4096, 4096, 0, 0), (4096, 4096, 4096, 1, 1),
                             (4096, 4096, 4096, 0, 1), (4096, 4096, 4096, 1, 0), (1000, 300, 80, 0, 0),
                             (1000, 300, 80, 1, 1), (132, 260, 48, 0, 1), (132, 260, 48, 1, 0), (47872, 512, 256, 0, 0), (1024, 256, 47872, 1, 1)]:
        case(M, N, Kk, ma, mb)


if __name__ == "__main__":
    main()
