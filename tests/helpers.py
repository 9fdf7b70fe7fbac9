"""Shared test helpers: build the espnet_slurp_amd model for an oracle ModelCfg, load the
oracle's seeded parameters, fixture loading and tolerance checks."""
import os

import numpy as np
import torch

from oracle import espnet_cpu as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def token_list(V):
    return ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]


def small_cfg(rel_pos_type="latest", D=64, blocks=2, V=32):
    return O.ModelCfg(vocab_size=V,
                      enc=O.EncCfg(output_size=D, attention_heads=4, linear_units=128, num_blocks=blocks,
                                   rel_pos_type=rel_pos_type),
                      dec=O.DecCfg(attention_heads=4, linear_units=128, num_blocks=2), ctc_weight=0.3, lsm_weight=0.1)


def c1_cfg():
    return O.ModelCfg(vocab_size=30, enc=O.EncCfg(kind="transformer", output_size=256, attention_heads=4,
                                                   linear_units=1024, num_blocks=4), dec=None, ctc_weight=1.0)


def c2_cfg(rel_pos_type="latest", blocks=12):
    return O.ModelCfg(vocab_size=600, enc=O.EncCfg(output_size=256, attention_heads=4, linear_units=1024,
                                                    num_blocks=blocks, rel_pos_type=rel_pos_type),
                      dec=O.DecCfg(attention_heads=4, linear_units=2048, num_blocks=6))


def build_model(cfg: O.ModelCfg, device, specaug=None, dropout=None, frontend=None):
    from espnet_slurp_amd.asr.ctc import CTC
    from espnet_slurp_amd.asr.decoder.transformer_decoder import TransformerDecoder
    from espnet_slurp_amd.asr.encoder.conformer_encoder import ConformerEncoder
    from espnet_slurp_amd.asr.encoder.transformer_encoder import TransformerEncoder
    from espnet_slurp_amd.asr.espnet_model import ESPnetASRModel
    from espnet_slurp_amd.layers.utterance_mvn import UtteranceMVN
    e = cfg.enc
    p = e.dropout_rate if dropout is None else dropout
    if e.kind == "conformer":
        enc = ConformerEncoder(input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
                               linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=p,
                               positional_dropout_rate=p, attention_dropout_rate=p, macaron_style=e.macaron_style,
                               rel_pos_type=e.rel_pos_type, use_cnn_module=e.use_cnn_module,
                               cnn_module_kernel=e.cnn_module_kernel)
    else:
        enc = TransformerEncoder(input_size=e.input_size, output_size=e.output_size, attention_heads=e.attention_heads,
                                 linear_units=e.linear_units, num_blocks=e.num_blocks, dropout_rate=p,
                                 positional_dropout_rate=p, attention_dropout_rate=p)
    dec = None
    if cfg.dec is not None and cfg.ctc_weight != 1.0:
        d = cfg.dec
        dec = TransformerDecoder(vocab_size=cfg.vocab_size, encoder_output_size=e.output_size,
                                 attention_heads=d.attention_heads, linear_units=d.linear_units,
                                 num_blocks=d.num_blocks, dropout_rate=p, positional_dropout_rate=p,
                                 self_attention_dropout_rate=p, src_attention_dropout_rate=p)
    ctc = CTC(odim=cfg.vocab_size, encoder_output_size=e.output_size)
    m = ESPnetASRModel(vocab_size=cfg.vocab_size, token_list=token_list(cfg.vocab_size), frontend=frontend,
                       specaug=specaug, normalize=UtteranceMVN(), preencoder=None, encoder=enc, postencoder=None,
                       decoder=dec, ctc=ctc, joint_network=None, ctc_weight=cfg.ctc_weight,
                       lsm_weight=cfg.lsm_weight, length_normalized_loss=cfg.length_normalized_loss,
                       report_cer=False, report_wer=False)
    m = m.to(device)
    m.flatten()
    return m


def load_seeded(model, cfg, seed):
    P = O.deterministic_params(cfg, seed)
    missing, unexpected = model.load_state_dict(P, strict=True)
    return P


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))
