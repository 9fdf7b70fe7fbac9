"""ESPnetSLUModel (espnet2/slu/espnet_model.py:36-440) without post-decoder: the ASR model with
fixed sos/eos = V-1, blank 0, the reference's constructor kwargs and an ignored transcript."""
import pytest
import torch

from tests.helpers import small_cfg, token_list


def _parts(cfg):
    from espnet_slurp_amd.asr.ctc import CTC
    from espnet_slurp_amd.asr.decoder.transformer_decoder import TransformerDecoder
    from espnet_slurp_amd.asr.encoder.conformer_encoder import ConformerEncoder
    from espnet_slurp_amd.layers.utterance_mvn import UtteranceMVN
    e, d = cfg.enc, cfg.dec
    enc = ConformerEncoder(input_size=80, output_size=e.output_size, attention_heads=e.attention_heads,
                           linear_units=e.linear_units, num_blocks=e.num_blocks, rel_pos_type="latest",
                           macaron_style=True, use_cnn_module=True, cnn_module_kernel=31, dropout_rate=0.0,
                           positional_dropout_rate=0.0, attention_dropout_rate=0.0)
    dec = TransformerDecoder(vocab_size=cfg.vocab_size, encoder_output_size=e.output_size,
                             attention_heads=d.attention_heads, linear_units=d.linear_units, num_blocks=d.num_blocks,
                             dropout_rate=0.0, positional_dropout_rate=0.0, self_attention_dropout_rate=0.0,
                             src_attention_dropout_rate=0.0)
    return dict(frontend=None, specaug=None, normalize=UtteranceMVN(), preencoder=None, encoder=enc,
                postencoder=None, decoder=dec, ctc=CTC(odim=cfg.vocab_size, encoder_output_size=e.output_size),
                joint_network=None)


def test_slu_model_matches_asr_layout():
    from espnet_slurp_amd.asr.espnet_model import ESPnetASRModel
    from espnet_slurp_amd.slu.espnet_model import ESPnetSLUModel
    cfg = small_cfg("latest")
    V = cfg.vocab_size
    torch.manual_seed(0)
    slu = ESPnetSLUModel(vocab_size=V, token_list=token_list(V), transcript_token_list=["a", "b"], ctc_weight=0.3,
                         lsm_weight=0.1, **_parts(cfg))
    asr = ESPnetASRModel(vocab_size=V, token_list=token_list(V), ctc_weight=0.3, lsm_weight=0.1, **_parts(cfg))
    assert slu.sos == slu.eos == V - 1 and slu.blank_id == 0
    assert {k: tuple(v.shape) for k, v in slu.state_dict().items()} == \
        {k: tuple(v.shape) for k, v in asr.state_dict().items()}
    with pytest.raises(NotImplementedError):
        ESPnetSLUModel(vocab_size=V, token_list=token_list(V), postdecoder=object(), **_parts(cfg))
