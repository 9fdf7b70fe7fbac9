"""Count Conv2dSubsampling ReLU decisions where the GPU's fp32 pre-activation and the fp64
reference's fall on different sides of 0 (full-size C2 fixture input)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oracle import espnet_cpu as O  # noqa: E402
from tests.helpers import build_model, c2_cfg, load_seeded  # noqa: E402
from espnet_slurp_amd.blocks import Seeds  # noqa: E402

dev = torch.device("cuda:0")
cfg = c2_cfg("latest")
m = build_model(cfg, dev)
load_seeded(m, cfg, 42)
P = O.deterministic_params(cfg, 42, torch.float64)
speech, slen, text, tlen = O.synthetic_batch(2, 1500, 80, 600, [1500, 1337], [40, 27], 43)
x = O.utterance_mvn(speech.double(), slen)
emb = m.encoder.embed
with torch.no_grad():
    _, c = emb.fwd(x.float().to(dev).contiguous(), 16.0, 0.0, Seeds(1), False)
    torch.cuda.synchronize()
    z1 = torch.relu(torch.nn.functional.conv2d(x[:, None], P["encoder.embed.conv.0.weight"],
                                               P["encoder.embed.conv.0.bias"], stride=2))  # (B, D, T1, F1)
    z2 = torch.nn.functional.conv2d(z1, P["encoder.embed.conv.2.weight"], P["encoder.embed.conv.2.bias"], stride=2)
    g1 = c.z1.view(c.B, c.T1, c.F1, -1).permute(0, 3, 1, 2).double().cpu()
    g2 = c.z2.view(c.B, c.T2, c.F2, -1).permute(0, 3, 1, 2).double().cpu()
print("z1 (post-ReLU): zero-mask flips", int(((g1 > 0) != (z1 > 0)).sum()), "of", z1.numel(),
      "max|err|", float((g1 - z1).abs().max()))
print("z2 (post-ReLU): zero-mask flips", int(((g2 > 0) != (z2 > 0)).sum()), "of", z2.numel(),
      "max|err| on positives", float(((g2 - torch.relu(z2)).abs()).max()))
