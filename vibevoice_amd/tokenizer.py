"""The standalone σ-VAE tokenizer API callers reach through the model
(`model.model.acoustic_tokenizer.decode(latents, cache=..., sample_indices=...,
use_cache=True)`, `model.model.semantic_tokenizer.encode(audio, ...)`,
`VibeVoiceTokenizerStreamingCache`; reference
vibevoice/modular/modular_vibevoice_tokenizer.py:193-256, 955-1000, 1081-1108,
1171-1175), on the HIP engine.

The reference keeps each conv layer's streaming context in a Python dict keyed
by (layer, sample index).  Here the context of every layer of a sample lives on
the device, in one codec slot of an engine context (the per-slot ConvBuf
history that generate() uses); a VibeVoiceTokenizerStreamingCache maps the
caller's sample indices to slots.  The views run on their own engine context
over the model's packed weights (no second copy), so standalone calls never
touch the slots of a running generate().  Frames are decoded / encoded one per
call (vv_codec_decode / vv_codec_encode); a causal streaming conv stack gives
the same output frame by frame as over the whole sequence.
"""
import weakref
from dataclasses import dataclass
from typing import Optional, Union

import torch

from .engine import Engine


@dataclass
class VibeVoiceTokenizerEncoderOutput:
    """modular_vibevoice_tokenizer.py:955-1000 (same fields and sampling rules)."""
    mean: torch.Tensor
    std: Optional[Union[float, torch.Tensor]] = None

    def sample(self, dist_type="fix"):
        if dist_type == "fix":
            x = self.mean + self.std * torch.randn_like(self.mean)
            return x, self.std
        if dist_type == "gaussian":
            value = self.std / 0.8
            std = torch.randn(self.mean.size(0), device=self.mean.device, dtype=self.mean.dtype) * value
            while std.dim() < self.mean.dim():
                std = std.unsqueeze(-1)
            return self.mean + std * torch.randn_like(self.mean), std
        return self.mean, self.std

    def kl(self):
        return torch.nn.functional.mse_loss(self.mean, torch.zeros_like(self.mean), reduction="none")

    def mode(self):
        return self.mean


class VibeVoiceTokenizerStreamingCache:
    """Streaming state of a set of samples (modular_vibevoice_tokenizer.py:193-256).

    `cache` maps (net, sample index) -> codec slot; the conv contexts of all
    layers of that slot live on the device.  set_to_zero / clear act on whole
    samples (all layers), as generate() uses them (:557-560)."""

    def __init__(self):
        self.cache = {}
        self._pool = None

    def _bind(self, pool):
        if self._pool is None:
            self._pool = pool
            weakref.finalize(self, pool.release_all, self.cache)
        elif self._pool is not pool:
            raise ValueError("a VibeVoiceTokenizerStreamingCache serves one model")

    def set_to_zero(self, sample_indices):
        if self._pool is not None:
            self._pool.zero(self.cache, [int(i) for i in torch.as_tensor(sample_indices).reshape(-1).tolist()])

    def clear(self, layer_id=None, sample_indices=None):
        """Drop the state of the given samples (all of them when None).  The
        reference can clear one conv layer; here a sample's layers move
        together, so `layer_id` only selects which samples' entries exist."""
        if self._pool is None:
            return
        idx = None if sample_indices is None else {int(i) for i in torch.as_tensor(sample_indices).reshape(-1)}
        self._pool.release(self.cache, idx)


class _SlotPool:
    """Codec slots of the tokenizer views' engine context."""

    def __init__(self, model, n_slots):
        self.model = model
        self.n = n_slots
        self.free = {0: list(range(n_slots)), 1: list(range(n_slots))}   # per net: 0 decoder, 1 semantic encoder
        self._eng = None

    @property
    def eng(self):
        if self._eng is None:
            m = self.model.engine
            # same TP coordinates as the owner: its packed LM weights are this rank's shards
            # (no communicator: the views only run the replicated codec / connectors)
            # (persistent="follow": this codec context runs the owner's one-launch
            # kernels -- bit-identical to its codec step -- without registering, so
            # it never demotes the owner's context)
            self._eng = Engine(self.model.config, None, m.device, max_batch=self.n, max_ctx=64, packed=m.w,
                               tp_rank=m.tp_rank, tp_size=m.tp_size, tp_head=m.tp_head, persistent="follow")
        return self._eng

    def _i32(self, xs):
        return torch.tensor(xs, dtype=torch.int32, device=self.eng.device)

    def take(self, net, k):
        if len(self.free[net]) < k:
            raise RuntimeError(f"tokenizer streaming slots exhausted ({self.n}); clear() finished caches")
        got, self.free[net] = self.free[net][:k], self.free[net][k:]
        self.eng.codec_reset_net(net, self._i32(got))          # a new sample starts from zero context
        return got

    def give(self, net, slots):
        self.free[net].extend(slots)

    def slots(self, cache, net, sample_indices):
        idx = [int(i) for i in sample_indices]
        new = [i for i in idx if (net, i) not in cache.cache]
        for i, s in zip(new, self.take(net, len(new))):
            cache.cache[(net, i)] = s
        return self._i32([cache.cache[(net, i)] for i in idx])

    def zero(self, cache_dict, idx):
        for net in (0, 1):
            s = [cache_dict[(net, i)] for i in idx if (net, i) in cache_dict]
            if s:
                self.eng.codec_reset_net(net, self._i32(s))

    def release(self, cache_dict, idx=None):
        for key in [k for k in cache_dict if idx is None or k[1] in idx]:
            self.give(key[0], [cache_dict.pop(key)])

    def release_all(self, cache_dict):
        self.release(cache_dict)


class _TokenizerView:
    def __init__(self, model, pool, tcfg):
        self._m = model
        self._pool = pool
        self.config = tcfg
        self.fix_std = tcfg.fix_std
        self.std_dist_type = tcfg.std_dist_type

    @property
    def device(self):
        return self._m.device

    @property
    def dtype(self):
        return torch.bfloat16

    def _slots(self, net, n, cache, sample_indices, use_cache):
        """(slots, temporary?) for n samples."""
        if use_cache and cache is not None:
            cache._bind(self._pool)
            idx = range(n) if sample_indices is None else torch.as_tensor(sample_indices).reshape(-1).tolist()
            return self._pool.slots(cache, net, idx), None
        tmp = self._pool.take(net, n)
        return self._pool._i32(tmp), tmp


class AcousticTokenizer(_TokenizerView):
    """`model.model.acoustic_tokenizer` (VibeVoiceAcousticTokenizerModel, :1002-1120)."""

    def encode(self, audio, cache=None, sample_indices=None, use_cache=False, debug=False):
        """Non-streaming encode of whole clips (the voice-prompt path, :1081-1085):
        audio [n, 1, L] or [n, L] -> mean [n, ceil(L / hop), vae_dim]."""
        if use_cache:
            raise NotImplementedError("streaming acoustic encoding is not on the generate() path; "
                                      "encode whole clips (use_cache=False)")
        a = audio.reshape(audio.shape[0], -1).to(self.device, torch.bfloat16).contiguous()
        return VibeVoiceTokenizerEncoderOutput(mean=self._m.engine.acoustic_encode(a), std=self.fix_std)

    def sampling(self, encoder_output, dist_type=None):
        dist_type = dist_type or self.std_dist_type
        if dist_type not in ("fix", "gaussian"):
            raise ValueError(f"Unsupported dist_type: {dist_type}, expected 'fix' or 'gaussian'")
        return encoder_output.sample(dist_type=dist_type)

    @torch.no_grad()
    def decode(self, latents, cache=None, sample_indices=None, use_cache=False, debug=False):
        """latents [n, vae_dim, T] or [n, T, vae_dim] (the decoder input: the
        caller has already applied latent / scaling - bias, :651) -> audio
        [n, 1, T * hop] bf16.  use_cache with a cache streams from the cached
        state of each sample index (and updates it); otherwise from zero
        state (the non-streaming decode of the sequence)."""
        eng = self._pool.eng
        D = self.config.vae_dim
        z = latents if latents.shape[1] == D else latents.permute(0, 2, 1)
        n, _, T = z.shape
        z = z.to(self.device, torch.bfloat16)
        slots, tmp = self._slots(0, n, cache, sample_indices, use_cache)
        hop = self._m.engine.hop
        out = torch.empty(n, 1, T * hop, dtype=torch.bfloat16, device=self.device)
        frame = torch.empty(n, hop, dtype=torch.bfloat16, device=self.device)
        try:
            for t in range(T):
                eng.codec_decode(slots, z[:, :, t].contiguous(), frame)
                out[:, 0, t * hop:(t + 1) * hop] = frame
        finally:
            if tmp is not None:
                self._pool.give(0, tmp)
        return out


class SemanticTokenizer(_TokenizerView):
    """`model.model.semantic_tokenizer` (VibeVoiceSemanticTokenizerModel, :1123-1186)."""

    @torch.no_grad()
    def encode(self, audio, cache=None, sample_indices=None, use_cache=False, debug=False):
        """audio [n, 1, L] -> output with mean [n, ceil(L / hop), semantic_dim].
        Whole frames (as generate() feeds them, :673-679) stream frame by frame
        through the per-slot state (from zero state without a cache) — the same
        kernels as the fused loop step.  Without a cache, a clip that ends in a
        partial frame takes the non-streaming encoder (vv_semantic_encode), which
        right-pads every strided conv's input to whole strides as the reference's
        non-streaming path does (:127-133, :393-408; golden G5).  A partial frame
        WITH a streaming cache raises (the reference's streaming convs carry the
        remainder in their cache; generate() never feeds one)."""
        eng = self._pool.eng
        a = audio.reshape(audio.shape[0], -1).to(self.device, torch.bfloat16)
        n, L = a.shape
        hop = self._m.engine.hop
        if L % hop:
            if use_cache and cache is not None:
                raise ValueError(f"streaming semantic encode takes whole {hop}-sample frames (got {L} samples)")
            return VibeVoiceTokenizerEncoderOutput(mean=self._m.engine.semantic_encode(a.contiguous()))
        slots, tmp = self._slots(1, n, cache, sample_indices, use_cache)
        S = self._m.config.semantic_vae_dim
        mean = torch.empty(n, L // hop, S, dtype=torch.bfloat16, device=self.device)
        feat = torch.empty(n, S, dtype=torch.bfloat16, device=self.device)
        try:
            for t in range(L // hop):
                eng.codec_encode(slots, a[:, t * hop:(t + 1) * hop].contiguous(), feat)
                mean[:, t] = feat
        finally:
            if tmp is not None:
                self._pool.give(1, tmp)
        return VibeVoiceTokenizerEncoderOutput(mean=mean)

    def sampling(self, encoder_output, dist_type=None):
        return encoder_output.sample(dist_type="none")


class Connector:
    """`model.model.acoustic_connector` / `semantic_connector` (SpeechConnector,
    modeling_vibevoice.py:58-69): rows [..., din] -> [..., H] on the engine."""

    def __init__(self, model, which):
        self._m, self._which = model, which

    @torch.no_grad()
    def __call__(self, x):
        lead = x.shape[:-1]
        y = self._m.engine.connector(self._which, x.reshape(-1, x.shape[-1]).to(self._m.device, torch.bfloat16))
        return y.reshape(*lead, y.shape[-1])
