"""Full-size gradient diagnostics: per tensor, the GPU's slice / norm error against the fp64
reference next to the reference's own fp32 error (fixtures of make_golden.py fullgrad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import espnet_cpu as O  # noqa: E402
from tests.helpers import build_model, c2_cfg, golden, load_seeded  # noqa: E402

dev = torch.device("cuda:0")
for rel in sys.argv[1:] or ["latest"]:
    g = golden(f"fullsize_c2_grad_{rel}")
    cfg = c2_cfg(rel)
    m = build_model(cfg, dev)
    load_seeded(m, cfg, int(g["seed"]))
    speech, slen, text, tlen = O.synthetic_batch(2, 1500, 80, 600, list(g["lens"]), list(g["ulens"]), int(g["seed"]) + 1)
    m.train()
    loss, st, _ = m(speech.to(dev), slen, text, tlen)
    loss.backward()
    torch.cuda.synchronize()
    print(rel, "loss", loss.item(), "f32", float(g["loss_f32"]), "f64", float(g["loss_f64"]))
    rows = []
    scale = max(float(g["gmax_f64/" + n]) for n, _ in m.named_parameters())
    for n, p in m.named_parameters():
        if float(g["gmax_f64/" + n]) < 1e-6 * scale:
            continue
        got = p.grad.detach().double().reshape(-1).cpu()
        gm = float(g["gmax_f64/" + n])
        s = got[torch.from_numpy(g["gidx/" + n])].numpy()
        es = float(np.abs(s - g["gs_f64/" + n]).max()) / gm
        er = float(np.abs(g["gs_f32/" + n] - g["gs_f64/" + n]).max()) / gm
        gn64 = float(g["gn_f64/" + n])
        en = abs(float(got.norm()) - gn64) / gn64
        enr = abs(float(g["gn_f32/" + n]) - gn64) / gn64
        rows.append((es, er, en, enr, n))
    ratios = [r[0] / max(r[1], 1e-9) for r in rows]
    print(f"  median slice err gpu {np.median([r[0] for r in rows]):.2e} ref32 {np.median([r[1] for r in rows]):.2e}"
          f"  median ratio {np.median(ratios):.2f}")
    for r in sorted(rows)[-12:]:
        print(f"  slice gpu {r[0]:.2e} ref {r[1]:.2e} | norm gpu {r[2]:.2e} ref {r[3]:.2e}  {r[4]}")
