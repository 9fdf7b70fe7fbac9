"""ESPnetASRModel — drop-in for espnet2/asr/espnet_model.py:36-297 (CTC/attention hybrid).

forward(speech, speech_lengths, text, text_lengths) -> (loss[1], stats, weight[1]) exactly
like the reference (stat keys loss_ctc / loss_att / acc / loss, plus cer/wer = None).
The step runs as two autograd nodes whose backward passes are explicit kernel sequences:
  EncoderFn (asr/encoder/abs_encoder.py): SpecAug/MVN'd fbank -> encoder output hs
  HeadsFn (below): CTC branch + decoder branch + label-smoothing loss, fused loss
    gradients (computed in the forward, scaled by grad_output in the backward), one dhs.
Parameter gradients are written into the flat gradient buffer (flat.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple, Union

import torch
from torch import nn

from .. import kernels as K
from ..blocks import Linear, Seeds, empty
from ..flat import FlatParams
from .encoder.abs_encoder import draw_seed
from .error_calculator import ErrorCalculator


class AbsESPnetModel(nn.Module):
    """espnet2/train/abs_espnet_model.py:7-40."""

    def forward(self, **batch):
        raise NotImplementedError

    def collect_feats(self, **batch):
        raise NotImplementedError


def add_sos_eos(ys_pad_cpu: torch.Tensor, ys_lens_cpu: torch.Tensor, sos: int, eos: int, ignore_id: int):
    """add_sos_eos.py:12-31 on the host (integer bookkeeping): ys_in padded with eos,
    ys_out padded with ignore_id."""
    B = ys_pad_cpu.shape[0]
    ys = [ys_pad_cpu[i][ys_pad_cpu[i] != ignore_id] for i in range(B)]
    L = max(int(y.numel()) for y in ys) + 1
    ys_in = torch.full((B, L), eos, dtype=torch.long)
    ys_out = torch.full((B, L), ignore_id, dtype=torch.long)
    for i, y in enumerate(ys):
        n = int(y.numel())
        ys_in[i, 0] = sos
        ys_in[i, 1:n + 1] = y
        ys_out[i, :n] = y
        ys_out[i, n] = eos
    return ys_in, ys_out, torch.tensor([int(y.numel()) + 1 for y in ys], dtype=torch.long)


class HeadsFn(torch.autograd.Function):
    """CTC + attention-decoder losses of one batch; backward returns d loss / d hs."""

    @staticmethod
    def forward(ctx, hs, anchor, model, prep, seed):
        out4, state = model._heads_forward(hs, prep, Seeds(seed), True)
        ctx.model = model
        ctx.state = state
        loss = out4[3:4].clone()
        others = out4[0:3].clone()
        ctx.mark_non_differentiable(others)
        return loss, others

    @staticmethod
    def backward(ctx, g_loss, g_others):
        dhs = ctx.model._heads_backward(ctx.state, g_loss.contiguous())
        ctx.state = None
        return dhs, None, None, None, None


class Prepared(dict):
    """Host-side bookkeeping of one batch (lengths, sos/eos targets, SpecAug draws, dropout
    seeds) and its device-resident copies.  Everything the kernels read per step lives in
    `dev` (device tensors), so a captured HIP graph is re-targeted at a new batch of the same
    shapes by copying the new host values into the same device tensors (`copy_into`)."""
    __getattr__ = dict.__getitem__

    def to_device(self, device):
        self["dev"] = {k: K.h2d(v, device) for k, v in self["host"].items()}
        return self

    def copy_into(self, other: "Prepared"):
        """Write this batch's host values into another Prepared's device tensors (same shapes)."""
        for k, v in self["host"].items():
            d = other["dev"][k]
            assert d.shape == v.shape, (k, d.shape, v.shape)
            d.copy_(v.pin_memory(), non_blocking=True)


class ESPnetASRModel(AbsESPnetModel):
    def __init__(self, vocab_size: int, token_list: Union[Tuple[str, ...], List[str]], frontend, specaug,
                 normalize, preencoder, encoder, postencoder, decoder, ctc, joint_network=None,
                 ctc_weight: float = 0.5, interctc_weight: float = 0.0, ignore_id: int = -1,
                 lsm_weight: float = 0.0, length_normalized_loss: bool = False, report_cer: bool = True,
                 report_wer: bool = True, sym_space: str = "<space>", sym_blank: str = "<blank>",
                 sym_sos: str = "<sos/eos>", sym_eos: str = "<sos/eos>", extract_feats_in_collect_stats: bool = True,
                 lang_token_id: int = -1):
        assert 0.0 <= ctc_weight <= 1.0, ctc_weight
        super().__init__()
        if preencoder is not None or postencoder is not None or joint_network is not None:
            raise NotImplementedError("pre-/post-encoder/transducer are not on the hot path")
        if frontend is not None and not hasattr(frontend, "apply_prepared"):
            raise NotImplementedError("frontend: only the native DefaultFrontend (frontend: default)")
        if lang_token_id != -1:
            raise NotImplementedError("lang_token_id")
        assert 0.0 <= interctc_weight < 1.0, interctc_weight  # espnet_model.py:71
        self.blank_id = token_list.index(sym_blank)
        self.sos = token_list.index(sym_sos) if sym_sos in token_list else vocab_size - 1
        self.eos = token_list.index(sym_eos) if sym_eos in token_list else vocab_size - 1
        self.vocab_size = vocab_size
        self.ignore_id = ignore_id
        self.ctc_weight = ctc_weight
        self.interctc_weight = interctc_weight
        self.token_list = list(token_list).copy()
        self.frontend = frontend
        self.specaug = specaug
        self.normalize = normalize
        self.preencoder = preencoder
        self.postencoder = postencoder
        self.encoder = encoder
        if getattr(encoder, "interctc_use_conditioning", False):  # espnet_model.py:96-101
            encoder.conditioning_layer = Linear(vocab_size, encoder.output_size())
        self.decoder = None if ctc_weight == 1.0 else decoder
        self.ctc = None if ctc_weight == 0.0 else ctc
        self.lsm_weight = lsm_weight
        self.length_normalized_loss = length_normalized_loss
        # eval-mode cer_ctc / cer / wer (espnet_model.py:152-154, 515-540)
        self.error_calculator = (ErrorCalculator(token_list, sym_space, sym_blank, report_cer, report_wer)
                                 if report_cer or report_wer else None)
        self.extract_feats_in_collect_stats = extract_feats_in_collect_stats
        self.flat: Optional[FlatParams] = None
        if self.blank_id != 0:
            raise NotImplementedError("blank must be token 0 (torch CTCLoss default used by espnet2)")

    # ------------------------------------------------------------------ setup
    def flatten(self, device=None) -> FlatParams:
        """Move parameters into one flat HBM buffer (+ flat grads).  Call once, after .to(device)."""
        device = device or next(self.parameters()).device
        self.flat = FlatParams(self, device)
        for m in (self.encoder, self.decoder):
            if m is not None and hasattr(m, "attach_flat"):
                m.attach_flat(self.flat)
        return self.flat

    # ------------------------------------------------------------------ heads
    def _inter_request(self, prep: "Prepared", want_grad: bool):
        """Intermediate CTC (espnet_model.py:222-245, conformer_encoder.py:333-350): the request the encoder
        fills in its forward -- the shared CTC module, the targets, and the gradient scale of each branch,
        ctc_weight * interctc_weight / (n_layers * B) (loss = ctc_weight ((1 - w) loss_ctc + w mean_l
        loss_interctc_l) + (1 - ctc_weight) loss_att).  None when the model has no intermediate branch."""
        idx = getattr(self.encoder, "interctc_layer_idx", None)
        cond = getattr(self.encoder, "conditioning_layer", None) is not None
        if not idx or self.ctc is None or (self.interctc_weight == 0.0 and not cond):
            prep["inter"] = None
            return None
        d = prep.dev
        inter = dict(ctc=self.ctc, hlens=d["hlens"], ys=d["ys"], tlens=d["tlens"], Umax=prep.Umax,
                     gscale=self.ctc_weight * self.interctc_weight / (len(idx) * prep.B), want_grad=want_grad,
                     weighted=self.interctc_weight != 0.0, nll=[], grads=[], stats={})
        prep["inter"] = inter
        return inter

    def _heads_forward(self, hs, prep: "Prepared", seeds: Seeds, want_grad: bool):
        B, T, D = hs.shape
        dev = hs.device
        hs2d = hs.reshape(B * T, D)
        d = prep.dev
        hlens_i32 = d["hlens"]
        state = {"hs2d": hs2d, "B": B, "T": T}
        nll = grad_ctc = None
        inter = prep.get("inter")
        # (the encoder's intermediate branches also add ctc_lo gradient in its backward: the ctc module-done
        # hook waits for them, _heads_backward)
        state["inter_any"] = inter is not None
        if inter is not None and not inter["weighted"]:  # self-conditioning only: no intermediate loss
            inter = None
        w_ic = self.interctc_weight if inter else 0.0
        if self.ctc is not None:
            nll, grad_ctc, _ = self.ctc.loss_and_grad(hs2d, B, T, hlens_i32, d["ys"], d["tlens"], prep.Umax,
                                                      self.ctc_weight * (1.0 - w_ic) / B, want_grad=want_grad)
            state["grad_ctc"] = grad_ctc
        nll_main = nll
        if inter:
            # loss_ctc of the loss = (1 - w) loss_ctc + w mean_l loss_interctc_l, each utterance's inf zeroed in
            # its own CTC first (zero_infinity, ctc.py:44-45); the reported loss_ctc stays the main branch's
            zi = self.ctc.zero_infinity
            z = (lambda v: torch.where(torch.isinf(v), torch.zeros_like(v), v)) if zi else (lambda v: v)
            comb = z(nll) * (1.0 - w_ic)
            for idx, nl in inter["nll"]:
                comb = comb + z(nl) * (w_ic / len(inter["nll"]))
                inter["stats"][f"loss_interctc_layer{idx}"] = (z(nl).sum() / B).float().view(1)
            state["loss_ctc_main"] = (z(nll).sum() / B).float().view(1)
            state["inter"] = inter
            nll = comb
        row_loss = row_stat = None
        R = 0
        # length_normalized_loss: the denominator is this batch's target count, taken on device
        # by esp_reduce_losses (denom 0) and applied to the decoder gradient in the backward
        ln = self.length_normalized_loss
        denom = 0.0 if ln else prep.denom
        if self.decoder is not None:
            R = B * prep.L
            logits, dsaved = self.decoder.run_forward(hs, hlens_i32, d["ys_in"], d["ys_in_lens"], seeds, self.training)
            V = self.vocab_size
            grad_att = empty(R, V, like=hs) if want_grad else None
            row_loss = torch.empty(R, dtype=torch.float64, device=dev)
            row_stat = torch.empty(2 * R, dtype=torch.int32, device=dev)
            K.label_smoothing(logits, d["ys_out"], V, self.ignore_id, self.lsm_weight,
                              (1.0 - self.ctc_weight) / (1.0 if ln else denom), grad_att, row_loss, row_stat)
            state["grad_att"] = grad_att
            state["dec"] = dsaved
            if not self.training and self.error_calculator is not None:
                prep["eval_logits"] = logits  # eval-mode cer / wer read the decoder argmax (_error_rates)
        out4 = empty(5, like=hs)
        K.reduce_losses(nll, B, self.ctc.zero_infinity if self.ctc is not None else True, row_loss, row_stat, R,
                        denom, self.ctc_weight, out4)
        if ln and self.decoder is not None:
            state["inv_denom"] = out4[4:5]
        if inter:  # out4[0] (the stats' loss_ctc): the main branch's, the loss out4[3] already has the mix
            out4[0:1].copy_(state["loss_ctc_main"])
        return out4, state

    def _heads_backward(self, state, g_loss, hook=None):
        hs2d = state["hs2d"]
        dhs = torch.zeros_like(hs2d) if self.ctc is None else torch.empty_like(hs2d)
        hook = hook or getattr(self, "_grad_hook", None)
        if self.ctc is not None:
            g = state["grad_ctc"]
            K.scale_by_dev(g, g_loss)
            self.ctc.backward_from_logits(g, hs2d, dhs)
            inter = state.get("inter")
            if inter:  # the intermediate branches' loss gradients, applied in the encoder backward (which hooks ctc)
                for gi in inter["grads"]:
                    K.scale_by_dev(gi, g_loss)
            if hook is not None and not state.get("inter_any"):
                hook(self.ctc)
        if self.decoder is not None:
            g = state["grad_att"]
            if state.get("inv_denom") is not None:
                K.scale_by_dev(g, state["inv_denom"])
            K.scale_by_dev(g, g_loss)
            self.decoder.run_backward(state["dec"], g, dhs, hook)
        return dhs.view(state["B"], state["T"], -1)

    # ------------------------------------------------------------------ forward
    def prepare(self, speech_lengths: torch.Tensor, text: torch.Tensor, text_lengths: torch.Tensor, T_in: int,
                F_in: int, specaug_draws: Optional[dict] = None, t_bucket: Optional[int] = None,
                u_bucket: Optional[int] = None) -> Prepared:
        """All host-side work of a step (espnet_model.py:169-297 before any kernel): lengths,
        the target slice, add_sos_eos, SpecAug draws (CPU generator, as time_warp.py), the
        dropout seeds.  Returns host tensors; `.to_device()` moves them (pinned, async).

        t_bucket / u_bucket (HIP-graph trainer, length buckets): pad the frame axis to t_bucket
        frames and the target axis to u_bucket tokens (ys padded with ignore_id, ys_in with eos,
        ys_out with ignore_id: one decoder row more per token of padding, all ignored).  Every
        length-derived quantity (SpecAug draws, encoder lengths, the valid frame count
        `tvalid` the convolution module bounds itself with) is still taken from this batch's
        own padded length, so the step computes what the reference computes on it."""
        assert text_lengths.dim() == 1, text_lengths.shape
        B = int(speech_lengths.shape[0])
        text = text.detach().cpu().clone()
        text[text == -1] = self.ignore_id
        sl_cpu = speech_lengths.detach().cpu()
        tl_cpu = text_lengths.detach().cpu()
        text_cpu = text[:, : int(tl_cpu.max())].contiguous()
        host = {}
        n_samples = 0
        if self.frontend is not None:  # _extract_feats: speech[:, :max(len)] -> frames (host-side lengths)
            n_samples = min(T_in, int(sl_cpu.max()))
            host["wav_lens"] = sl_cpu.to(torch.int32)
            T = self.frontend.num_frames(n_samples)
            sl_cpu = self.frontend.output_lengths(sl_cpu)
            F_in = self.frontend.output_size()
        else:
            T = min(T_in, int(sl_cpu.max()))
        host.update({"lens": sl_cpu.to(torch.int32), "weight": torch.tensor([B], dtype=torch.long)})
        if self.specaug is not None and self.training:
            draws = specaug_draws if specaug_draws is not None else self.specaug.draw(B, T, F_in, sl_cpu.tolist())
            for k, v in draws.items():
                host["sa_" + k] = v.to(torch.int32)
        host["hlens"] = self.encoder.output_lengths(sl_cpu, T).to(torch.int32)
        T_true = T
        if t_bucket is not None:
            assert t_bucket >= T, (t_bucket, T)
            T = int(t_bucket)
            if self.frontend is not None:
                # raw samples padded to the frame bucket's sample count; the STFT's centre padding
                # still reflects at this batch's own sample count (device nvalid)
                host["nvalid"] = torch.tensor([n_samples], dtype=torch.int32)
                n_samples = self.frontend.samples_for_frames(T)
                assert n_samples <= T_in, (n_samples, T_in)
            # valid frames after Conv2dSubsampling of the batch's own padded length
            host["tvalid"] = torch.tensor([self.encoder.embed.out_frames(T_true)], dtype=torch.int32)
        if u_bucket is not None and u_bucket > text_cpu.shape[1]:
            pad = torch.full((B, int(u_bucket) - text_cpu.shape[1]), self.ignore_id, dtype=text_cpu.dtype)
            text_cpu = torch.cat([text_cpu, pad], 1)
        prep = Prepared(B=B, T=T, T_true=T_true, Umax=int(text_cpu.shape[1]), denom=float(B), L=0, host=host,
                        enc_seed=draw_seed(), heads_seed=draw_seed(), sl_cpu=sl_cpu, n_samples=n_samples,
                        ys_pad_cpu=text_cpu)
        if self.ctc is not None:
            host["ys"] = text_cpu
            host["tlens"] = tl_cpu.to(torch.int32)
        if self.decoder is not None:
            ys_in, ys_out, ys_in_lens = add_sos_eos(text_cpu, tl_cpu, self.sos, self.eos, self.ignore_id)
            if u_bucket is not None and ys_in.shape[1] < int(u_bucket) + 1:
                extra = int(u_bucket) + 1 - ys_in.shape[1]
                ys_in = torch.cat([ys_in, torch.full((B, extra), self.eos, dtype=ys_in.dtype)], 1)
                ys_out = torch.cat([ys_out, torch.full((B, extra), self.ignore_id, dtype=ys_out.dtype)], 1)
            prep["L"] = int(ys_in.shape[1])
            host["ys_in"], host["ys_out"] = ys_in, ys_out
            host["ys_in_lens"] = ys_in_lens.to(torch.int32)
        return prep

    def forward_prepared(self, speech: torch.Tensor, prep: Prepared):
        """The step's device work from a prepared batch: no host->device traffic and no host
        synchronisation, so the forward + backward can be captured as one HIP graph."""
        d = prep.dev
        if self.frontend is not None:  # raw samples -> log-mel on device (one kernel)
            feats = self.frontend.apply_prepared(speech, d["wav_lens"], prep.n_samples, d.get("nvalid"))
        else:
            feats = speech[:, : prep.T].contiguous().float()
        if self.specaug is not None and self.training:
            draws = {k[3:]: v for k, v in d.items() if k.startswith("sa_")}
            feats = self.specaug.apply_prepared(feats, d["lens"], draws)
        if self.normalize is not None:
            feats = self.normalize.apply_prepared(feats, d["lens"])
        grad_on = torch.is_grad_enabled() and next(iter(self.parameters())).requires_grad
        inter = self._inter_request(prep, grad_on)
        encoder_out = self.encoder.forward_prepared(feats, prep.sl_cpu, d["hlens"], prep.enc_seed, d.get("tvalid"),
                                                    **({"inter": inter} if inter else {}))
        anchor = next(p for p in (self.ctc or self.decoder).parameters())
        if torch.is_grad_enabled() and anchor.requires_grad:
            loss, others = HeadsFn.apply(encoder_out, anchor, self, prep, prep.heads_seed)
        else:
            out4, _ = self._heads_forward(encoder_out, prep, Seeds(prep.heads_seed), False)
            loss, others = out4[3:4], out4[0:3]
        stats = dict(
            loss_ctc=others[0:1].detach() if self.ctc is not None else None,
            cer_ctc=None,
            loss_att=others[1:2].detach() if self.decoder is not None else None,
            acc=others[2:3].detach() if self.decoder is not None else None,
            cer=None, wer=None,
            loss=loss.detach(),
        )
        if inter:
            stats.update({k: v.detach() for k, v in inter["stats"].items()})
        if not self.training and self.error_calculator is not None:
            stats.update(self._error_rates(encoder_out, prep))
        return loss, stats, d["weight"]

    def forward_explicit(self, speech: torch.Tensor, prep: Prepared):
        """forward_prepared without autograd nodes, for a caller that runs the backward itself
        (backward_explicit) on its own thread: the segmented HIP-graph capture of the
        data-parallel step ends and begins captures inside the module-done hook, which the
        autograd engine would call from its device thread.  Same kernels, same order."""
        d = prep.dev
        with torch.no_grad():
            if self.frontend is not None:
                feats = self.frontend.apply_prepared(speech, d["wav_lens"], prep.n_samples, d.get("nvalid"))
            else:
                feats = speech[:, : prep.T].contiguous().float()
            if self.specaug is not None and self.training:
                draws = {k[3:]: v for k, v in d.items() if k.startswith("sa_")}
                feats = self.specaug.apply_prepared(feats, d["lens"], draws)
            if self.normalize is not None:
                feats = self.normalize.apply_prepared(feats, d["lens"])
            enc = self.encoder
            inter = self._inter_request(prep, True)
            hs, _olens, saved = enc.run_forward(feats, prep.sl_cpu, Seeds(prep.enc_seed), enc.training, klen=d["hlens"],
                                                tvalid=d.get("tvalid"), **({"inter": inter} if inter else {}))
            out4, state = self._heads_forward(hs, prep, Seeds(prep.heads_seed), True)
        loss, others = out4[3:4], out4[0:3]
        stats = dict(
            loss_ctc=others[0:1] if self.ctc is not None else None,
            cer_ctc=None,
            loss_att=others[1:2] if self.decoder is not None else None,
            acc=others[2:3] if self.decoder is not None else None,
            cer=None, wer=None,
            loss=loss,
        )
        if inter:
            stats.update(inter["stats"])
        return loss, stats, d["weight"], (saved, state)

    def backward_explicit(self, ctx, g_loss: torch.Tensor, hook=None):
        """The backward of forward_explicit for d loss = g_loss (a device scalar): heads, then
        encoder (HeadsFn.backward + EncoderFn.backward), `hook(module)` at each module done."""
        saved, state = ctx
        dhs = self._heads_backward(state, g_loss, hook)
        self.encoder.run_backward(saved, dhs.contiguous(), hook)

    def _error_rates(self, encoder_out, prep) -> Dict[str, Optional[torch.Tensor]]:
        """Eval-mode error rates (espnet_model.py:515-521, 536-539): greedy CTC and decoder
        argmaxes on device, then the reference's host-side string edit distances."""
        dev = encoder_out.device
        as_t = lambda v: None if v is None else torch.tensor([v], dtype=torch.float32, device=dev)
        out = {}
        ys_pad = prep.ys_pad_cpu
        if self.ctc is not None:
            ys_hat = self.ctc.argmax(encoder_out).cpu()
            out["cer_ctc"] = as_t(self.error_calculator(ys_hat, ys_pad, is_ctc=True))
        if self.decoder is not None:
            R = prep.B * prep.L
            am = torch.empty(R, dtype=torch.int64, device=dev)
            K.argmax(prep.pop("eval_logits"), am, R, self.vocab_size)
            cer, wer = self.error_calculator(am.view(prep.B, prep.L).cpu(), ys_pad)
            out["cer"], out["wer"] = as_t(cer), as_t(wer)
        return out

    def forward(self, speech: torch.Tensor, speech_lengths: torch.Tensor, text: torch.Tensor,
                text_lengths: torch.Tensor, specaug_draws: Optional[dict] = None, **kwargs):
        assert text_lengths.dim() == 1, text_lengths.shape
        assert speech.shape[0] == speech_lengths.shape[0] == text.shape[0] == text_lengths.shape[0], (
            speech.shape, speech_lengths.shape, text.shape, text_lengths.shape)
        assert self.flat is not None, "call model.flatten() after moving the model to the GPU"
        if torch.is_grad_enabled():
            self.flat.ensure_grads()  # after a torch optimizer's zero_grad(set_to_none=True)
        text[text == -1] = self.ignore_id  # the reference mutates the batch (espnet_model.py:196)
        F_in = speech.shape[2] if speech.dim() == 3 else 0
        prep = self.prepare(speech_lengths, text, text_lengths, speech.shape[1], F_in, specaug_draws)
        prep.to_device(speech.device)
        return self.forward_prepared(speech, prep)

    def encode(self, speech: torch.Tensor, speech_lengths: torch.Tensor, sl_cpu: Optional[torch.Tensor] = None,
               specaug_draws: Optional[dict] = None):
        """espnet_model.py:319-377 (frontend=None: feats = speech[:, :max_len])."""
        if sl_cpu is None:
            sl_cpu = speech_lengths.detach().cpu()
        if self.frontend is not None:
            feats, feats_lengths = self.frontend(speech, sl_cpu)
        else:
            feats = speech[:, : int(sl_cpu.max())].contiguous().float()
            feats_lengths = sl_cpu
        if self.specaug is not None and self.training:
            feats, _ = self.specaug(feats, feats_lengths, draws=specaug_draws)
        if self.normalize is not None:
            feats, _ = self.normalize(feats, feats_lengths)
        return self.encoder(feats, feats_lengths)[:2]

    def collect_feats(self, speech, speech_lengths, text, text_lengths, **kwargs) -> Dict[str, torch.Tensor]:
        if self.frontend is not None and self.extract_feats_in_collect_stats:
            feats, flens = self.frontend(speech, speech_lengths)
            return {"feats": feats, "feats_lengths": flens}
        return {"feats": speech[:, : int(speech_lengths.max())], "feats_lengths": speech_lengths}
