"""Time the rel-pos MHA block (forward and explicit backward, C2 shape B=128, T'=374, D=256,
H=4, attention dropout 0.1) on the flash path vs the materialised-probability path, latest and
legacy.  usage: python tools/flash_bench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from espnet_slurp_amd import kernels as K  # noqa: E402
from espnet_slurp_amd.asr.encoder.abs_encoder import pos_table  # noqa: E402
from espnet_slurp_amd.blocks import RelPositionMultiHeadedAttention, Seeds  # noqa: E402
from espnet_slurp_amd.flat import FlatParams  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    T, D, H = 374, 256, 4
    klen = torch.full((B,), T, dtype=torch.int32, device=dev)
    x = torch.randn(B * T, D, device=dev)
    res = torch.randn(B * T, D, device=dev)
    dout = torch.randn(B * T, D, device=dev)
    for legacy in (False, True):
        pos = pos_table("legacy" if legacy else "latest", T, D, dev)
        for flash in (True, False):
            K.FLASH_ATTN = flash
            torch.manual_seed(0)
            mod = RelPositionMultiHeadedAttention(H, D, 0.1, legacy).to(dev)
            mod.flat = FlatParams(mod, dev)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            tf = tb = 0.0
            n = 10
            for it in range(n + 2):
                ev[0].record()
                out, c = mod.fwd(x, res, pos, klen, B, T, 0.0, Seeds(it), True)
                ev[1].record()
                mod.bwd(c, dout)
                ev[2].record()
                torch.cuda.synchronize()
                if it >= 2:
                    tf += ev[0].elapsed_time(ev[1])
                    tb += ev[1].elapsed_time(ev[2])
            print(f"{'legacy' if legacy else 'latest'} {'flash' if flash else 'materialised'}: fwd {tf / n:.3f} ms"
                  f"  bwd {tb / n:.3f} ms  (block incl. projections)", flush=True)


if __name__ == "__main__":
    main()
