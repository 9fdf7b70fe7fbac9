"""ESPnetSLUModel (espnet2/slu/espnet_model.py:36-440) for the SLURP intent / entity recipes
that train it WITHOUT a post-decoder or deliberation encoder (egs2/slurp_entity conformer
configs): then the SLU model is the ASR model — same encoder, CTC + attention losses over the
semantic token sequence, sos = eos = vocab_size - 1, blank = 0 (slu/espnet_model.py:72-76) —
plus an ignored `transcript` input.  The BERT post-decoder and the deliberation encoder are
Hugging Face modules outside this build: passing them raises NotImplementedError.
"""
from typing import List, Optional, Tuple, Union

from ..asr.espnet_model import ESPnetASRModel


class ESPnetSLUModel(ESPnetASRModel):
    def __init__(self, vocab_size: int, token_list: Union[Tuple[str, ...], List[str]], frontend, specaug, normalize,
                 preencoder, encoder, postencoder, decoder, ctc, joint_network=None, postdecoder=None,
                 deliberationencoder=None, transcript_token_list: Optional[Union[Tuple[str, ...], List[str]]] = None,
                 ctc_weight: float = 0.5, interctc_weight: float = 0.0, ignore_id: int = -1, lsm_weight: float = 0.0,
                 length_normalized_loss: bool = False, report_cer: bool = True, report_wer: bool = True,
                 sym_space: str = "<space>", sym_blank: str = "<blank>", extract_feats_in_collect_stats: bool = True,
                 two_pass: bool = False, pre_postencoder_norm: bool = False):
        if postdecoder is not None or deliberationencoder is not None or two_pass:
            raise NotImplementedError("ESPnetSLUModel: post-decoder / deliberation encoder / two_pass "
                                      "(Hugging Face modules) are outside this build")
        super().__init__(vocab_size=vocab_size, token_list=token_list, frontend=frontend, specaug=specaug,
                         normalize=normalize, preencoder=preencoder, encoder=encoder, postencoder=postencoder,
                         decoder=decoder, ctc=ctc, joint_network=joint_network, ctc_weight=ctc_weight,
                         interctc_weight=interctc_weight, ignore_id=ignore_id, lsm_weight=lsm_weight,
                         length_normalized_loss=length_normalized_loss, report_cer=report_cer, report_wer=report_wer,
                         sym_space=sym_space, sym_blank=sym_blank,
                         extract_feats_in_collect_stats=extract_feats_in_collect_stats)
        # slu/espnet_model.py:72-76: fixed ids, not looked up in the token list
        self.blank_id = 0
        self.sos = vocab_size - 1
        self.eos = vocab_size - 1
        self.transcript_token_list = list(transcript_token_list) if transcript_token_list is not None else None
        self.two_pass = two_pass
        self.pre_postencoder_norm = pre_postencoder_norm

    def forward(self, speech, speech_lengths, text, text_lengths, transcript=None, transcript_lengths=None, **kwargs):
        return super().forward(speech, speech_lengths, text, text_lengths, **kwargs)

    def encode(self, speech, speech_lengths, transcript_pad=None, transcript_pad_lens=None, **kwargs):
        return super().encode(speech, speech_lengths, **kwargs)
