"""GPU grads vs the fp64 oracle and vs the reference fp32 fixture, per tensor."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import espnet_cpu as O  # noqa: E402
from tests.helpers import build_model, golden, load_seeded, rel_err, small_cfg  # noqa: E402

for name, rp in (("model_small_legacy", "legacy"), ("model_small_latest", "latest")):
    g = golden(name)
    cfg = small_cfg(rp)
    dev = torch.device("cuda:0")
    m = build_model(cfg, dev)
    load_seeded(m, cfg, int(g["seed"]))
    m.train()
    loss, st, _ = m(torch.from_numpy(g["speech"]).to(dev), torch.from_numpy(g["speech_lengths"]),
                    torch.from_numpy(g["text"]), torch.from_numpy(g["text_lengths"]))
    loss.backward()
    P = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k)
         for k, v in O.deterministic_params(cfg, int(g["seed"]), torch.float64).items()}
    l64, _, _ = O.asr_forward(P, torch.from_numpy(g["speech"]).double(), torch.from_numpy(g["speech_lengths"]),
                              torch.from_numpy(g["text"]), torch.from_numpy(g["text_lengths"]), cfg, bn_state={})
    l64.backward()
    print(name, "loss gpu", loss.item(), "ref32", float(g["loss"]), "f64", l64.item())
    rows = []
    for n, p in m.named_parameters():
        r64 = P[n].grad.numpy()
        rows.append((rel_err(p.grad.cpu().numpy(), r64), rel_err(g["grad/" + n], r64), n))
    rows.sort()
    for r in rows[-10:]:
        print(f"  gpu-vs-f64 {r[0]:.2e}  ref32-vs-f64 {r[1]:.2e}  {r[2]}")
