"""ASRTask subset: the espnet2 plugin registries and build_model (espnet2/tasks/asr.py:83-188,
439-562) so egs2/slurp* YAML `encoder:`/`decoder:`/`specaug:`/`normalize:`/`model_conf:`
sections drop in unchanged.  `ClassChoices.get_class` keeps the reference's error
behaviour (ValueError on unknown names, espnet2/train/class_choices.py:63-77)."""
from __future__ import annotations

import argparse
from typing import Dict, Optional, Type

import torch

from ..asr.ctc import CTC
from ..asr.decoder.transformer_decoder import TransformerDecoder
from ..asr.encoder.conformer_encoder import ConformerEncoder
from ..asr.encoder.transformer_encoder import TransformerEncoder
from ..asr.espnet_model import ESPnetASRModel
from ..asr.specaug.specaug import SpecAug
from ..asr.frontend.default import DefaultFrontend
from ..layers.global_mvn import GlobalMVN
from ..layers.utterance_mvn import UtteranceMVN
from ..torch_utils.initialize import initialize


class ClassChoices:
    def __init__(self, name: str, classes: Dict[str, Type], type_check=None, default: Optional[str] = None,
                 optional: bool = False):
        self.name = name
        self.base_type = type_check
        self.classes = {k.lower(): v for k, v in classes.items()}
        if "none" in self.classes or "nil" in self.classes or "null" in self.classes:
            raise ValueError('"none", "nil", and "null" are reserved.')
        self.default = default
        self.optional = optional

    def choices(self):
        return list(self.classes) + (["none"] if self.optional else [])

    def get_class(self, name: Optional[str]) -> Optional[type]:
        if name is None or (self.optional and name.lower() in ("none", "null", "nil")):
            return None
        if name.lower() in self.classes:
            return self.classes[name.lower()]
        raise ValueError(f"--{self.name} must be one of {self.choices()}: --{self.name} {name.lower()}")


frontend_choices = ClassChoices("frontend", dict(default=DefaultFrontend), default="default")
specaug_choices = ClassChoices("specaug", dict(specaug=SpecAug), default=None, optional=True)
normalize_choices = ClassChoices("normalize", dict(global_mvn=GlobalMVN, utterance_mvn=UtteranceMVN),
                                 default="utterance_mvn", optional=True)
model_choices = ClassChoices("model", dict(espnet=ESPnetASRModel), default="espnet")
encoder_choices = ClassChoices("encoder", dict(conformer=ConformerEncoder, transformer=TransformerEncoder),
                               default="rnn")
decoder_choices = ClassChoices("decoder", dict(transformer=TransformerDecoder), default="rnn", optional=True)


def build_model(args: argparse.Namespace, device="cuda") -> ESPnetASRModel:
    """ASRTask.build_model (asr.py:439-562) for the fbank (--input_size) path.

    args needs: token_list (a list or a token file path, as asr.py:441-450), input_size,
    specaug/_conf, normalize/_conf, encoder/_conf, decoder/_conf, ctc_conf, model_conf, init
    (the resolved config.yaml fields)."""
    if isinstance(args.token_list, str):
        with open(args.token_list, encoding="utf-8") as f:
            token_list = [line.rstrip() for line in f]
        args.token_list = list(token_list)  # "portable", as the reference does
    elif isinstance(args.token_list, (tuple, list)):
        token_list = list(args.token_list)
    else:
        raise RuntimeError("token_list must be str or list")
    for opt in ("preencoder", "postencoder"):
        if getattr(args, opt, None) is not None:
            raise NotImplementedError(f"--{opt}: not on the Conformer CTC/attention hot path")
    if getattr(args, "decoder", None) == "transducer":
        raise NotImplementedError("--decoder transducer: not on the CTC/attention hot path")
    vocab_size = len(token_list)
    if getattr(args, "input_size", None) is None:  # extract features in the model (asr.py:459-468)
        frontend = frontend_choices.get_class(getattr(args, "frontend", "default"))(
            **(getattr(args, "frontend_conf", None) or {}))
        input_size = frontend.output_size()
    else:  # features from the data loader
        args.frontend, args.frontend_conf = None, {}
        frontend = None
        input_size = args.input_size
    specaug_cls = specaug_choices.get_class(getattr(args, "specaug", None))
    specaug = specaug_cls(**(getattr(args, "specaug_conf", None) or {})) if specaug_cls else None
    norm_cls = normalize_choices.get_class(getattr(args, "normalize", "utterance_mvn"))
    normalize = norm_cls(**(getattr(args, "normalize_conf", None) or {})) if norm_cls else None
    encoder = encoder_choices.get_class(args.encoder)(input_size=input_size, **(args.encoder_conf or {}))
    dec_cls = decoder_choices.get_class(getattr(args, "decoder", None))
    decoder = dec_cls(vocab_size=vocab_size, encoder_output_size=encoder.output_size(),
                      **(getattr(args, "decoder_conf", None) or {})) if dec_cls else None
    ctc = CTC(odim=vocab_size, encoder_output_size=encoder.output_size(), **(getattr(args, "ctc_conf", None) or {}))
    model_cls = model_choices.get_class(getattr(args, "model", "espnet"))
    model = model_cls(vocab_size=vocab_size, frontend=frontend, specaug=specaug, normalize=normalize, preencoder=None,
                      encoder=encoder, postencoder=None, decoder=decoder, ctc=ctc, joint_network=None,
                      token_list=token_list, **(getattr(args, "model_conf", None) or {}))
    if getattr(args, "init", None) is not None:  # asr.py:556-557
        initialize(model, args.init)
    model = model.to(device)
    model.flatten()
    return model
