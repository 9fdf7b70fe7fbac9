"""Speech2Text (espnet2/bin/asr_inference.py:52-470, ASR attention/CTC path): speech -> n-best
(text, tokens, token ids, hypothesis).  Encoder in eval mode (BatchNorm running statistics,
no dropout / SpecAug) on the HIP kernels, then the joint CTC/attention BeamSearch of
asr/beam_search.py with the reference's weights: decoder 1 - ctc_weight, ctc ctc_weight,
length_bonus penalty; pre-beam on the "full" scores unless ctc_weight == 1.0.
Tokenizers: "bpe" (sentencepiece model file, as the SLURP recipes use) and "char";
ids2tokens by the model's token_list.  LM / n-gram / transducer / streaming are out of scope.
"""
from typing import List, Optional, Tuple, Union

import numpy as np
import torch

from ..asr.beam_search import BeamSearch, CTCPrefixScorer, DecoderScorer, Hypothesis, LengthBonus


class CharTokenizer:
    def __init__(self, space_symbol: str = "<space>"):
        self.space_symbol = space_symbol

    def tokens2text(self, tokens):
        return "".join(tokens).replace(self.space_symbol, " ")


class SentencepiecesTokenizer:
    def __init__(self, model: str):
        import sentencepiece as spm
        self.sp = spm.SentencePieceProcessor()
        self.sp.load(str(model))

    def tokens2text(self, tokens):
        return self.sp.DecodePieces(list(tokens))


class Speech2Text:
    def __init__(self, asr_model, token_list: Optional[List[str]] = None, beam_size: int = 20,
                 ctc_weight: float = 0.5, penalty: float = 0.0, nbest: int = 1, maxlenratio: float = 0.0,
                 minlenratio: float = 0.0, token_type: Optional[str] = None, bpemodel: Optional[str] = None):
        asr_model.eval()
        self.asr_model = asr_model
        self.device = asr_model.flat.flat.device
        self.token_list = list(token_list if token_list is not None else asr_model.token_list)
        decoder = asr_model.decoder
        scorers = dict(decoder=DecoderScorer(decoder) if decoder is not None else None,
                       ctc=CTCPrefixScorer(asr_model.ctc, eos=asr_model.eos, blank=asr_model.blank_id),
                       length_bonus=LengthBonus())
        weights = dict(decoder=1.0 - ctc_weight, ctc=ctc_weight, length_bonus=penalty)
        self.beam_search = BeamSearch(scorers=scorers, weights=weights, beam_size=beam_size,
                                      vocab_size=len(self.token_list), sos=asr_model.sos, eos=asr_model.eos,
                                      token_list=self.token_list,
                                      pre_beam_score_key=None if ctc_weight == 1.0 else "full")
        self.maxlenratio, self.minlenratio, self.nbest = maxlenratio, minlenratio, nbest
        if token_type == "bpe":
            self.tokenizer = SentencepiecesTokenizer(bpemodel)
        elif token_type == "char":
            self.tokenizer = CharTokenizer()
        else:
            self.tokenizer = None

    @torch.no_grad()
    def encode(self, speech: Union[torch.Tensor, np.ndarray]) -> torch.Tensor:
        if isinstance(speech, np.ndarray):
            speech = torch.tensor(speech)
        speech = speech.unsqueeze(0).to(torch.float32).to(self.device)
        lengths = torch.tensor([speech.shape[1]], dtype=torch.int64)
        enc, _ = self.asr_model.encode(speech, lengths, sl_cpu=lengths)
        return enc[0]

    @torch.no_grad()
    def __call__(self, speech: Union[torch.Tensor, np.ndarray]) -> List[Tuple[Optional[str], List[str], List[int],
                                                                                Hypothesis]]:
        enc = self.encode(speech)
        hyps = self.beam_search.forward(enc, self.maxlenratio, self.minlenratio)[: self.nbest]
        out = []
        for h in hyps:
            token_int = [t for t in h.yseq[1:-1].tolist() if t != 0]
            token = [self.token_list[i] for i in token_int]
            text = self.tokenizer.tokens2text(token) if self.tokenizer is not None else None
            out.append((text, token, token_int, h))
        return out
