"""Streaming σ-VAE codec: acoustic decoder and (semantic/acoustic) encoder (oracle).

Restates vibevoice/modular/modular_vibevoice_tokenizer.py in functional form:
  ConvRMSNorm            :77-91   (fp32 normalise over channels, cast, x weight)
  SConv1d streaming      :327-382 (cat(cache, x) -> conv, cache = last ctx inputs,
                                   ctx = (k-1)*d - (s-1), zero-initialised)
  SConv1d non-streaming  :384-418 (causal left pad + extra right pad, pad_mode constant)
  SConvTranspose1d       :478-549 (cat(history, x) -> convT -> trim right k-s ->
                                   keep last T*s; history = last k-1 inputs)
  Block1D streaming body :925-944 / :787-804
  TokenizerDecoder       :816-951,  TokenizerEncoder :687-813
  decoder depths = reversed(encoder depths) (:1024-1028); encoder ratios reversed (:701).
`sd` holds the tokenizer's state dict (keys relative to
`model.acoustic_tokenizer.` / `model.semantic_tokenizer.`).  Streaming state is a
dict {layer_key: tensor[n_slots, C, ctx]} indexed by sample slot, the same
per-(layer, sample) contents as VibeVoiceTokenizerStreamingCache (:193-256).
"""
import math

import torch
import torch.nn.functional as F


def parse_depths(d):
    return [int(x) for x in d.split("-")] if isinstance(d, str) else list(d)


def codec_dims(tcfg, part):
    """Static layout of the decoder ("decoder") or encoder ("encoder")."""
    enc_depths = parse_depths(tcfg["encoder_depths"])
    if part == "decoder":
        dd = tcfg.get("decoder_depths")
        depths = parse_depths(dd) if dd is not None else list(reversed(enc_depths))
        ratios = list(tcfg.get("decoder_ratios") or tcfg["encoder_ratios"])
        nf = tcfg.get("decoder_n_filters", 32)
        chans = [nf * 2 ** (len(depths) - 1 - i) for i in range(len(depths))]
    else:
        depths = enc_depths
        ratios = list(reversed(tcfg["encoder_ratios"]))
        nf = tcfg.get("encoder_n_filters", 32)
        chans = [nf * 2 ** i for i in range(len(depths))]
    return dict(depths=depths, ratios=ratios, chans=chans, vae_dim=tcfg["vae_dim"],
                channels=tcfg.get("channels", 1), eps=tcfg.get("layernorm_eps", 1e-5),
                disable_last_norm=tcfg.get("disable_last_norm", True))


def conv_rms_norm(x, w, eps):
    """ConvRMSNorm (:77-91) on [B, C, T]."""
    y = x.transpose(1, 2)
    o = y.float()
    o = (o * torch.rsqrt(o.pow(2).mean(-1, keepdim=True) + eps)).type_as(y)
    if w is not None:
        o = o * w
    return o.transpose(1, 2)


class StreamState:
    """Per-(layer, slot) conv context, zero at first use (:337-346)."""

    def __init__(self, n_slots):
        self.n = n_slots
        self.buf = {}

    def get(self, key, slots, C, ctx, like):
        if key not in self.buf:
            self.buf[key] = torch.zeros(self.n, C, ctx, dtype=like.dtype, device=like.device)
        return self.buf[key][slots]

    def put(self, key, slots, val):
        self.buf[key][slots] = val

    def zero(self, slots):
        """VibeVoiceTokenizerStreamingCache.set_to_zero (:234-241)."""
        for v in self.buf.values():
            v[slots] = 0


def sconv(x, w, b, stride, state, key, slots, streaming):
    k = w.shape[-1]
    ctx = (k - 1) - (stride - 1)
    if streaming:
        hist = state.get(key, slots, x.shape[1], ctx, x)
        xin = torch.cat([hist, x], dim=2)
        if ctx > 0:
            state.put(key, slots, xin[:, :, xin.shape[2] - ctx:])
        return F.conv1d(xin, w, b, stride=stride)
    L = x.shape[-1]                                                     # :127-133, :398-403
    nfr = (L - k + ctx) / stride + 1
    extra = (math.ceil(nfr) - 1) * stride + (k - ctx) - L
    return F.conv1d(F.pad(x, (ctx, extra)), w, b, stride=stride)


def sconvtr(x, w, b, stride, state, key, slots, streaming):
    k = w.shape[-1]
    pad_total = k - stride
    T = x.shape[-1]
    if not streaming:
        y = F.conv_transpose1d(x, w, b, stride=stride)
        return y[..., : y.shape[-1] - pad_total]
    # history of up to k-1 previous inputs; a zero history gives the same
    # kept samples as the reference's empty first-chunk history (:522-533)
    hist = state.get(key, slots, x.shape[1], k - 1, x)
    full = torch.cat([hist, x], dim=2)
    y = F.conv_transpose1d(full, w, b, stride=stride)
    y = y[..., : y.shape[-1] - pad_total]
    state.put(key, slots, full[:, :, full.shape[2] - (k - 1):])
    return y[..., y.shape[-1] - T * stride:]


def block(sd, p, x, eps, state, slots, streaming):
    """Block1D streaming body (:925-944)."""
    r = x
    h = conv_rms_norm(x, sd.get(p + "norm.weight"), eps)
    h = sconv(h, sd[p + "mixer.conv.conv.conv.weight"], sd.get(p + "mixer.conv.conv.conv.bias"), 1,
              state, p + "mixer", slots, streaming)
    x = r + h * sd[p + "gamma"].unsqueeze(-1)
    r = x
    h = conv_rms_norm(x, sd.get(p + "ffn_norm.weight"), eps).permute(0, 2, 1)
    h = F.linear(F.gelu(F.linear(h, sd[p + "ffn.linear1.weight"], sd.get(p + "ffn.linear1.bias"))),
                 sd[p + "ffn.linear2.weight"], sd.get(p + "ffn.linear2.bias")).permute(0, 2, 1)
    return r + h * sd[p + "ffn_gamma"].unsqueeze(-1)


def _depthwise(sd, p):
    """depthwise conv weights are [C, 1, k]: F.conv1d needs groups=C."""
    return sd[p + "mixer.conv.conv.conv.weight"].shape[1] == 1


def decode(sd, dims, z, state=None, slots=None, streaming=True):
    """TokenizerDecoder.forward (:914-951): z [n, vae_dim, T] -> audio [n, 1, T*hop]."""
    if slots is None:
        slots = torch.arange(z.shape[0])
    x = sconv(z, sd["decoder.upsample_layers.0.0.conv.conv.weight"],
              sd.get("decoder.upsample_layers.0.0.conv.conv.bias"), 1, state, "dec.stem", slots, streaming)
    for i, depth in enumerate(dims["depths"]):
        if i > 0:
            q = f"decoder.upsample_layers.{i}.0.convtr.convtr."
            x = sconvtr(x, sd[q + "weight"], sd.get(q + "bias"), dims["ratios"][i - 1], state, f"dec.up{i}",
                        slots, streaming)
        for j in range(depth):
            x = _block_dw(sd, f"decoder.stages.{i}.{j}.", x, dims["eps"], state, slots, streaming)
    return sconv(x, sd["decoder.head.conv.conv.weight"], sd.get("decoder.head.conv.conv.bias"), 1,
                 state, "dec.head", slots, streaming)


def encode(sd, dims, audio, state=None, slots=None, streaming=True):
    """TokenizerEncoder.forward (:776-813): audio [n, 1, L] -> mean [n, T, vae_dim] (:1085)."""
    if slots is None:
        slots = torch.arange(audio.shape[0])
    x = audio
    for i, depth in enumerate(dims["depths"]):
        q = f"encoder.downsample_layers.{i}.0.conv.conv."
        stride = 1 if i == 0 else dims["ratios"][i - 1]
        x = sconv(x, sd[q + "weight"], sd.get(q + "bias"), stride, state, f"enc.down{i}", slots, streaming)
        for j in range(depth):
            x = _block_dw(sd, f"encoder.stages.{i}.{j}.", x, dims["eps"], state, slots, streaming)
    x = sconv(x, sd["encoder.head.conv.conv.weight"], sd.get("encoder.head.conv.conv.bias"), 1,
              state, "enc.head", slots, streaming)
    return x.permute(0, 2, 1)


def _block_dw(sd, p, x, eps, state, slots, streaming):
    if not _depthwise(sd, p):
        return block(sd, p, x, eps, state, slots, streaming)
    r = x
    h = conv_rms_norm(x, sd.get(p + "norm.weight"), eps)
    w, b = sd[p + "mixer.conv.conv.conv.weight"], sd.get(p + "mixer.conv.conv.conv.bias")
    k = w.shape[-1]
    if streaming:
        hist = state.get(p + "mixer", slots, h.shape[1], k - 1, h)
        hin = torch.cat([hist, h], dim=2)
        state.put(p + "mixer", slots, hin[:, :, hin.shape[2] - (k - 1):])
    else:
        hin = F.pad(h, (k - 1, 0))
    h = F.conv1d(hin, w, b, groups=w.shape[0])
    x = r + h * sd[p + "gamma"].unsqueeze(-1)
    r = x
    h = conv_rms_norm(x, sd.get(p + "ffn_norm.weight"), eps).permute(0, 2, 1)
    h = F.linear(F.gelu(F.linear(h, sd[p + "ffn.linear1.weight"], sd.get(p + "ffn.linear1.bias"))),
                 sd[p + "ffn.linear2.weight"], sd.get(p + "ffn.linear2.bias")).permute(0, 2, 1)
    return r + h * sd[p + "ffn_gamma"].unsqueeze(-1)
