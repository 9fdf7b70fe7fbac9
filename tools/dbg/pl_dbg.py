import os, sys
sys.path.insert(0, os.getcwd())
import torch
from espnet_slurp_amd import kernels as K
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
for (Bn, H, T, dk, Tp) in [(1, 1, 128, 64, 128)]:
    D = H * dk
    P = torch.randn(H * Bn * T * Tp, generator=g).to(dev)
    V = torch.randn(Bn * T, 3 * D, generator=g).to(dev)
    C = torch.empty(Bn * T, D, device=dev)
    K.gemm(T, dk, T, P, V, C, mode_a=K.KC, lda=Tp, mode_b=K.RC, ldb=3 * D, ldc=D, b_off=2 * D, batch=H * Bn,
           nb2=Bn, sa=(Bn * T * Tp, T * Tp), sb=(dk, T * 3 * D), sc=(dk, T * D))
    Cp = K.Planes(Bn * T, D, dev)
    Cp.buf.fill_(0)
    K.gemm(T, dk, T, P, V, Cp, mode_a=K.KC, lda=Tp, mode_b=K.RC, ldb=3 * D, ldc=D, b_off=2 * D, batch=H * Bn,
           nb2=Bn, sa=(Bn * T * Tp, T * Tp), sb=(dk, T * 3 * D), sc=(dk, T * D))
    torch.cuda.synchronize()
    pl = Cp.buf.view(3, Bn * T, D).float()
    print("C[0,:6]", C[0, :6].tolist())
    for p in range(3):
        print("plane", p, pl[p, 0, :6].tolist(), "nonzero", int((pl[p] != 0).sum()))
    ref = K.Planes.of(C)
    rp = ref.buf.view(3, Bn * T, D).float()
    for p in range(3):
        print("ref plane", p, rp[p, 0, :6].tolist())
    # search where the planes went: does plane0 match C bf16 elsewhere?
    hi = C.to(torch.bfloat16).float()
    print("hi==bf16(C)", bool(torch.equal(pl[0], hi)), "max|pl0-C|", float((pl[0] - C).abs().max()))
    Cp2 = K.Planes(Bn * T, D, dev)
    Cp2.buf.fill_(0)
    A = torch.randn(300, 128, generator=g).to(dev)
    B = torch.randn(128, 64, generator=g).to(dev)
    C2 = torch.empty(300, 64, device=dev)
    K.gemm(300, 64, 128, A, B, C2, mode_a=K.KC, lda=128, mode_b=K.RC, ldb=64, ldc=64)
    C3 = K.Planes(300, 64, dev)
    K.gemm(300, 64, 128, A, B, C3, mode_a=K.KC, lda=128, mode_b=K.RC, ldb=64, ldc=64)
    torch.cuda.synchronize()
    print("unbatched KCxRC planes ok", bool(torch.equal(C3.float(), C2)), float((C3.float() - C2).abs().max()))
