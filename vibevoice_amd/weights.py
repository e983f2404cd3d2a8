"""Weights: the reference's checkpoint names -> engine names + layouts.

Checkpoint names are those of VibeVoiceForConditionalGenerationInference's
state dict (modeling_vibevoice.py:107-142,
modeling_vibevoice_inference.py:77-80).  `pack()` turns them into the
layouts the HIP kernels consume (vibevoice_amd/csrc/gemm.hip header):

  * q/k/v projections concatenated -> one [(nh+2nkv)d, H] GEMM (+ bias)
  * gate/up interleaved in blocks of 8 rows -> one GEMM with a SiLU*up epilogue
  * all adaLN modulation matrices of the head stacked -> one GEMM per step
  * causal conv [Co, Ci, k] -> [Co, k*Ci]  (channels-last im2col row order)
  * ConvTranspose [Ci, Co, 2r] -> 2-tap [r*Co, 2*Ci] (history row, current row)

`synthetic_state_dict()` builds seeded random weights at the reference's
shapes (no checkpoints are reachable offline).
"""
import math

import torch

from .config import VibeVoiceConfig

LM = "model.language_model."
HEAD = "model.prediction_head."


def codec_channels(cfg: VibeVoiceConfig, part, which="acoustic"):
    t = cfg.acoustic_tokenizer_config if which == "acoustic" else cfg.semantic_tokenizer_config
    n = len(cfg.enc_depths)
    if part == "decoder":
        nf = t.decoder_n_filters
        return [nf * 2 ** (n - 1 - i) for i in range(n)]
    nf = t.encoder_n_filters
    return [nf * 2 ** i for i in range(n)]


def _codec_shapes(cfg, prefix, part, which):
    """(name, shape) of one conv stack, in the reference's naming."""
    chans = codec_channels(cfg, part, which)
    t = cfg.acoustic_tokenizer_config if which == "acoustic" else cfg.semantic_tokenizer_config
    out = []
    n = len(chans)
    if part == "decoder":
        depths, ratios = cfg.dec_depths, cfg.ratios
        out.append((f"{prefix}decoder.upsample_layers.0.0.conv.conv", [chans[0], t.vae_dim, 7], chans[0]))
        for i in range(1, n):
            r = ratios[i - 1]
            out.append((f"{prefix}decoder.upsample_layers.{i}.0.convtr.convtr", [chans[i - 1], chans[i], 2 * r],
                        chans[i]))
        stages = "decoder.stages"
        out.append((f"{prefix}decoder.head.conv.conv", [1, chans[-1], 7], 1))
    else:
        depths, ratios = cfg.enc_depths, list(reversed(cfg.ratios))
        out.append((f"{prefix}encoder.downsample_layers.0.0.conv.conv", [chans[0], 1, 7], chans[0]))
        for i in range(1, n):
            r = ratios[i - 1]
            out.append((f"{prefix}encoder.downsample_layers.{i}.0.conv.conv", [chans[i], chans[i - 1], 2 * r],
                        chans[i]))
        stages = "encoder.stages"
        out.append((f"{prefix}encoder.head.conv.conv", [t.vae_dim, chans[-1], 7], t.vae_dim))
    blocks = []
    for i, dep in enumerate(depths):
        C = chans[i]
        for j in range(dep):
            blocks.append((f"{prefix}{stages}.{i}.{j}.", C))
    return out, blocks


def synthetic_state_dict(cfg: VibeVoiceConfig, seed=0, device="cpu", dtype=torch.bfloat16, mode="bench",
                         with_acoustic_encoder=True):
    """Seeded random weights with the reference's names and shapes.

    mode="bench": the reference's own init scales (std 0.02 linears,
    layer-scale gamma 1e-6, zero biases) so activations behave like an
    untrained model.  mode="test": larger, fan-in-scaled weights, random
    norms / gammas / biases so every term of every kernel is exercised.
    """
    meta = torch.device(device).type == "meta"     # shapes only (no data: byte accounting, layout tests)
    g = None if meta else torch.Generator(device=device).manual_seed(seed)
    sd = {}
    test = mode == "test"

    def rnd(shape, std):
        if meta:
            return torch.empty(shape, device=device, dtype=dtype)
        return (torch.randn(shape, generator=g, device=device, dtype=torch.float32) * std).to(dtype)

    def lin(name, shape, bias=None):
        std = (1.0 / math.sqrt(shape[1] if len(shape) == 2 else shape[1] * shape[2])) if test else 0.02
        sd[name + ".weight"] = rnd(shape, std)
        if bias is not None:
            sd[name + ".bias"] = rnd([bias], 0.1) if test else torch.zeros(bias, device=device, dtype=dtype)

    def norm(name, n):
        sd[name] = (1.0 + rnd([n], 0.1).float()).to(dtype) if test else torch.ones(n, device=device, dtype=dtype)

    lm = cfg.decoder_config
    H, nh, nkv = lm.hidden_size, lm.num_attention_heads, lm.num_key_value_heads
    d = lm.get("head_dim") or H // nh
    I, V = lm.intermediate_size, lm.vocab_size
    sd[LM + "embed_tokens.weight"] = rnd([V, H], 0.02 if not test else 1.0)
    for i in range(lm.num_hidden_layers):
        p = f"{LM}layers.{i}."
        lin(p + "self_attn.q_proj", [nh * d, H], nh * d)
        lin(p + "self_attn.k_proj", [nkv * d, H], nkv * d)
        lin(p + "self_attn.v_proj", [nkv * d, H], nkv * d)
        lin(p + "self_attn.o_proj", [H, nh * d])
        lin(p + "mlp.gate_proj", [I, H])
        lin(p + "mlp.up_proj", [I, H])
        lin(p + "mlp.down_proj", [H, I])
        norm(p + "input_layernorm.weight", H)
        norm(p + "post_attention_layernorm.weight", H)
    norm(LM + "norm.weight", H)
    if cfg.tie_word_embeddings:
        sd["lm_head.weight"] = sd[LM + "embed_tokens.weight"]
    else:
        lin("lm_head", [V, H])

    hc = cfg.diffusion_head_config
    Hh, F, Dl = hc.hidden_size, int(hc.hidden_size * hc.head_ffn_ratio), hc.latent_size
    lin(HEAD + "noisy_images_proj", [Hh, Dl])
    lin(HEAD + "cond_proj", [Hh, Hh])
    lin(HEAD + "t_embedder.mlp.0", [Hh, 256])
    lin(HEAD + "t_embedder.mlp.2", [Hh, Hh])
    for i in range(hc.head_layers):
        p = f"{HEAD}layers.{i}."
        lin(p + "ffn.gate_proj", [F, Hh])
        lin(p + "ffn.up_proj", [F, Hh])
        lin(p + "ffn.down_proj", [Hh, F])
        norm(p + "norm.weight", Hh)
        lin(p + "adaLN_modulation.1", [3 * Hh, Hh])
    lin(HEAD + "final_layer.linear", [Dl, Hh])
    lin(HEAD + "final_layer.adaLN_modulation.1", [2 * Hh, Hh])

    for name, din in (("acoustic", cfg.acoustic_vae_dim), ("semantic", cfg.semantic_vae_dim)):
        p = f"model.{name}_connector."
        lin(p + "fc1", [H, din], H)
        norm(p + "norm.weight", H)
        lin(p + "fc2", [H, H], H)
    sd["model.speech_scaling_factor"] = torch.tensor(0.2 if not test else 0.75, device=device).to(dtype)
    sd["model.speech_bias_factor"] = torch.tensor(-0.05 if not test else 0.1, device=device).to(dtype)

    parts = [("model.acoustic_tokenizer.", "decoder", "acoustic"), ("model.semantic_tokenizer.", "encoder", "semantic")]
    if with_acoustic_encoder:
        parts.append(("model.acoustic_tokenizer.", "encoder", "acoustic"))
    wi = cfg.acoustic_tokenizer_config.weight_init_value
    ls = cfg.acoustic_tokenizer_config.layer_scale_init_value
    for prefix, part, which in parts:
        convs, blocks = _codec_shapes(cfg, prefix, part, which)
        for name, shape, nb in convs:
            if test:
                fan = shape[0] * shape[2] if "convtr" in name else shape[1] * shape[2]
                sd[name + ".weight"] = rnd(shape, 1.0 / math.sqrt(fan) * (2.0 if "convtr" in name else 1.0))
                sd[name + ".bias"] = rnd([nb], 0.05)
            else:
                sd[name + ".weight"] = rnd(shape, wi)
                sd[name + ".bias"] = torch.zeros(nb, device=device, dtype=dtype)
        for p, C in blocks:
            norm(p + "norm.weight", C)
            norm(p + "ffn_norm.weight", C)
            if test:
                sd[p + "mixer.conv.conv.conv.weight"] = rnd([C, 1, 7], 0.4)
                sd[p + "mixer.conv.conv.conv.bias"] = rnd([C], 0.05)
                sd[p + "gamma"] = rnd([C], 0.3)
                sd[p + "ffn_gamma"] = rnd([C], 0.3)
            else:
                sd[p + "mixer.conv.conv.conv.weight"] = rnd([C, 1, 7], wi)
                sd[p + "mixer.conv.conv.conv.bias"] = torch.zeros(C, device=device, dtype=dtype)
                sd[p + "gamma"] = torch.full([C], ls, device=device).to(dtype)
                sd[p + "ffn_gamma"] = torch.full([C], ls, device=device).to(dtype)
            if test:
                sd[p + "ffn.linear1.weight"] = rnd([4 * C, C], 1.0 / math.sqrt(C))
                sd[p + "ffn.linear1.bias"] = rnd([4 * C], 0.05)
                sd[p + "ffn.linear2.weight"] = rnd([C, 4 * C], 1.0 / math.sqrt(4 * C))
                sd[p + "ffn.linear2.bias"] = rnd([C], 0.05)
            else:
                sd[p + "ffn.linear1.weight"] = rnd([4 * C, C], wi)
                sd[p + "ffn.linear1.bias"] = torch.zeros(4 * C, device=device, dtype=dtype)
                sd[p + "ffn.linear2.weight"] = rnd([C, 4 * C], wi)
                sd[p + "ffn.linear2.bias"] = torch.zeros(C, device=device, dtype=dtype)
    return sd


# ------------------------------------------------------------------ packing
def _gu(gate, up):
    """Interleave gate/up rows in blocks of 8 (EPI_SILU_MUL tile layout)."""
    I, H = gate.shape
    assert I % 8 == 0
    return torch.stack([gate.reshape(I // 8, 8, H), up.reshape(I // 8, 8, H)], dim=1).reshape(2 * I, H)


def mfma_pack(w):
    """[N, K] -> the same shape in MFMA-fragment order (csrc/gemm.hip header):
    block (tile t, chunk c) of 16 rows x 32 columns is 1 KB contiguous, lane l
    holding W[16t + (l & 15)][32c + 8(l >> 4) .. +7]."""
    N, K = w.shape
    assert N % 16 == 0 and K % 32 == 0, (N, K)
    return w.reshape(N // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(N, K)


def mfma_unpack(w):
    N, K = w.shape
    return w.reshape(N // 16, K // 32, 4, 16, 8).permute(0, 3, 1, 2, 4).contiguous().reshape(N, K)


def is_gemm_weight(name):
    """Engine weights consumed by the MFMA GEMM / GEMV kernels (MFMA-packed)."""
    if not name.endswith("_w") or name.endswith(".dw_w"):
        return False
    return name not in ("dec.head_w", "sem.stem_w", "aenc.stem_w")


def _rope_pack(x, nheads, d=128):
    """Reorder q or k projection rows (or bias) so each 16-row MFMA tile holds
    8 rotary pairs: tile t of a head = dims [8t, 8t+8) then [d/2+8t, d/2+8t+8)
    (EPI_ROPE layout, csrc/gemm.hip)."""
    rest = x.shape[1:]
    y = x.reshape(nheads, 2, d // 16, 8, *rest).transpose(1, 2)
    return y.reshape(nheads * d, *rest)


def _conv_rows(w):
    """[Co, Ci, k] -> [Co, k*Ci], element (co, j*Ci + ci) = w[co, ci, j]."""
    Co, Ci, k = w.shape
    return w.permute(0, 2, 1).reshape(Co, k * Ci)


def _convtr_2tap(w, b, r):
    """[Ci, Co, 2r] -> [r*Co, 2*Ci]: row (j*Co + co) = [w[:, co, j+r] (history) | w[:, co, j] (current)]."""
    Ci, Co, k = w.shape
    assert k == 2 * r
    wp = w.permute(2, 1, 0)  # [k, Co, Ci]
    packed = torch.cat([wp[r:], wp[:r]], dim=2).reshape(r * Co, 2 * Ci)
    return packed, b.repeat(r)


def rope_inv_freq(theta, d):
    """Qwen2RotaryEmbedding default inv_freq (transformers modeling_qwen2.py:69-86), fp32."""
    return 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.int64).to(dtype=torch.float) / d))


def tp_check(cfg: VibeVoiceConfig, tp_size):
    """Where the backbone shards cleanly: whole kv heads per
    rank (1.5B: 2 kv heads -> TP <= 2; Large: 4 -> TP <= 4)."""
    lm = cfg.decoder_config
    nh, nkv, inter = lm.num_attention_heads, lm.num_key_value_heads, lm.intermediate_size
    if nkv % tp_size or nh % tp_size or inter % (16 * tp_size):
        raise ValueError(f"TP={tp_size} does not shard {nh} q / {nkv} kv heads / intermediate {inter} cleanly")


def head_tp_check(cfg: VibeVoiceConfig, tp_size):
    """The diffusion head's FFN splits into whole 32-column chunks per rank
    (the row-parallel down projection's K; Large: 10,752 / 4 = 2,688 = 84 x 32)."""
    hc = cfg.diffusion_head_config
    F = int(hc.hidden_size * hc.head_ffn_ratio)
    if F % (32 * tp_size):
        raise ValueError(f"TP={tp_size} does not shard the diffusion head FFN ({F}) into 32-column chunks")


def head_tp_default(cfg: VibeVoiceConfig, tp_size):
    """Shard the head when its per-step weights cannot stay in the 256 MB
    Infinity Cache (VibeVoice-Large: 925 MB per step, streamed by every
    replicated rank); the 1.5B head (170 MB, cache-resident) stays replicated."""
    hc = cfg.diffusion_head_config
    F = int(hc.hidden_size * hc.head_ffn_ratio)
    return tp_size > 1 and hc.head_layers * 3 * F * hc.hidden_size * 2 > (192 << 20)


def pack(sd, cfg: VibeVoiceConfig, device, with_acoustic_encoder=True, tp_rank=0, tp_size=1, tp_head=False):
    """Reference state dict -> {engine name: contiguous device tensor}.

    The diffusion head's FFN is packed once, in the GEMV layout (gate|up tiles of
    8 gate + 8 up rows, MFMA-packed): k_head_m16 at 2 <= 2n <= 16 rows and the
    GEMV pair beyond read the same copy.

    tp_size > 1: this rank's Megatron shard of the Qwen2 layers
    (configuration_vibevoice.py:175-183): q/k/v rows of its heads and
    gate/up rows of its intermediate slice (column-parallel), the matching
    o_proj / down_proj input columns (row-parallel).  Embedding, norms,
    lm_head, diffusion head, codec and connectors are replicated, except with
    tp_head: the diffusion head's FFN then splits the same way (gate|up rows of
    the rank's hidden columns, the matching down_proj input columns; SURVEY.md
    §8e)."""
    dt = torch.bfloat16
    tp_check(cfg, tp_size)

    def t(x):
        return x.to(device=device, dtype=dt).contiguous()

    out = {}
    lm = cfg.decoder_config
    H, nh = lm.hidden_size, lm.num_attention_heads
    d = lm.get("head_dim") or H // nh
    out["lm.embed"] = t(sd[LM + "embed_tokens.weight"])
    out["lm.lm_head"] = t(sd["lm_head.weight"]) if "lm_head.weight" in sd else out["lm.embed"]
    out["lm.norm"] = t(sd[LM + "norm.weight"])
    out["lm.inv_freq"] = rope_inv_freq(lm.rope_theta, d).to(device)
    for i in range(lm.num_hidden_layers):
        p = f"{LM}layers.{i}."
        e = f"lm.{i}."
        out[e + "in_norm"] = t(sd[p + "input_layernorm.weight"])
        out[e + "post_norm"] = t(sd[p + "post_attention_layernorm.weight"])
        nkv = lm.num_key_value_heads
        nhl, nkvl, il = nh // tp_size, nkv // tp_size, lm.intermediate_size // tp_size
        qs = slice(tp_rank * nhl * d, (tp_rank + 1) * nhl * d)
        ks = slice(tp_rank * nkvl * d, (tp_rank + 1) * nkvl * d)
        fs = slice(tp_rank * il, (tp_rank + 1) * il)
        q, k, v = (sd[p + f"self_attn.{x}_proj.weight"] for x in "qkv")
        qb, kb, vb = (sd[p + f"self_attn.{x}_proj.bias"] for x in "qkv")
        out[e + "qkv_w"] = t(torch.cat([_rope_pack(q[qs], nhl, d), _rope_pack(k[ks], nkvl, d), v[ks]], 0))
        out[e + "qkv_b"] = t(torch.cat([_rope_pack(qb[qs], nhl, d), _rope_pack(kb[ks], nkvl, d), vb[ks]], 0))
        out[e + "o_w"] = t(sd[p + "self_attn.o_proj.weight"][:, qs])
        out[e + "gu_w"] = t(_gu(sd[p + "mlp.gate_proj.weight"][fs], sd[p + "mlp.up_proj.weight"][fs]))
        out[e + "down_w"] = t(sd[p + "mlp.down_proj.weight"][:, fs])

    hc = cfg.diffusion_head_config
    out["head.noisy_w"] = t(sd[HEAD + "noisy_images_proj.weight"])
    out["head.cond_w"] = t(sd[HEAD + "cond_proj.weight"])
    out["head.t0_w"] = t(sd[HEAD + "t_embedder.mlp.0.weight"])
    out["head.t2_w"] = t(sd[HEAD + "t_embedder.mlp.2.weight"])
    ada = [sd[f"{HEAD}layers.{i}.adaLN_modulation.1.weight"] for i in range(hc.head_layers)]
    ada.append(sd[HEAD + "final_layer.adaLN_modulation.1.weight"])
    out["head.ada_w"] = t(torch.cat(ada, 0))
    hF = int(hc.hidden_size * hc.head_ffn_ratio)
    if tp_head and tp_size > 1:
        head_tp_check(cfg, tp_size)
        hl = hF // tp_size
        hs = slice(tp_rank * hl, (tp_rank + 1) * hl)
    else:
        hs = slice(0, hF)
    for i in range(hc.head_layers):
        p = f"{HEAD}layers.{i}."
        out[f"head.{i}.norm"] = t(sd[p + "norm.weight"])
        out[f"head.{i}.gu_w"] = t(_gu(sd[p + "ffn.gate_proj.weight"][hs], sd[p + "ffn.up_proj.weight"][hs]))
        out[f"head.{i}.down_w"] = t(sd[p + "ffn.down_proj.weight"][:, hs])
    out["head.final_w"] = t(sd[HEAD + "final_layer.linear.weight"])

    for src, dst in (("acoustic", "ac"), ("semantic", "se")):
        p = f"model.{src}_connector."
        out[f"conn.{dst}.fc1_w"] = t(sd[p + "fc1.weight"])
        out[f"conn.{dst}.fc1_b"] = t(sd[p + "fc1.bias"])
        out[f"conn.{dst}.norm"] = t(sd[p + "norm.weight"])
        out[f"conn.{dst}.fc2_w"] = t(sd[p + "fc2.weight"])
        out[f"conn.{dst}.fc2_b"] = t(sd[p + "fc2.bias"])
    out["speech_scaling_factor"] = t(sd["model.speech_scaling_factor"].reshape(()))
    out["speech_bias_factor"] = t(sd["model.speech_bias_factor"].reshape(()))

    nets = [("dec", "model.acoustic_tokenizer.", "decoder", "acoustic"),
            ("sem", "model.semantic_tokenizer.", "encoder", "semantic")]
    if with_acoustic_encoder and "model.acoustic_tokenizer.encoder.head.conv.conv.weight" in sd:
        nets.append(("aenc", "model.acoustic_tokenizer.", "encoder", "acoustic"))
    for e, prefix, part, which in nets:
        chans = codec_channels(cfg, part, which)
        n = len(chans)
        if part == "decoder":
            w = sd[prefix + "decoder.upsample_layers.0.0.conv.conv.weight"]
            out[e + ".stem_w"] = t(_conv_rows(w))
            out[e + ".stem_b"] = t(sd[prefix + "decoder.upsample_layers.0.0.conv.conv.bias"])
            for i in range(1, n):
                q = f"{prefix}decoder.upsample_layers.{i}.0.convtr.convtr."
                pw, pb = _convtr_2tap(sd[q + "weight"], sd[q + "bias"], cfg.ratios[i - 1])
                out[f"{e}.tr{i}_w"], out[f"{e}.tr{i}_b"] = t(pw), t(pb)
            hw = sd[prefix + "decoder.head.conv.conv.weight"]
            out[e + ".head_w"] = t(hw[0].t())
            out[e + ".head_b"] = t(sd[prefix + "decoder.head.conv.conv.bias"])
            depths, st = cfg.dec_depths, "decoder.stages"
        else:
            w = sd[prefix + "encoder.downsample_layers.0.0.conv.conv.weight"]
            out[e + ".stem_w"] = t(w.reshape(w.shape[0], w.shape[2]))
            out[e + ".stem_b"] = t(sd[prefix + "encoder.downsample_layers.0.0.conv.conv.bias"])
            for i in range(1, n):
                q = f"{prefix}encoder.downsample_layers.{i}.0.conv.conv."
                out[f"{e}.tr{i}_w"] = t(_conv_rows(sd[q + "weight"]))
                out[f"{e}.tr{i}_b"] = t(sd[q + "bias"])
            out[e + ".head_w"] = t(_conv_rows(sd[prefix + "encoder.head.conv.conv.weight"]))
            out[e + ".head_b"] = t(sd[prefix + "encoder.head.conv.conv.bias"])
            depths, st = cfg.enc_depths, "encoder.stages"
        for i, dep in enumerate(depths):
            for j in range(dep):
                p = f"{prefix}{st}.{i}.{j}."
                b = f"{e}.s{i}.b{j}."
                C = chans[i]
                out[b + "norm"] = t(sd[p + "norm.weight"])
                out[b + "ffn_norm"] = t(sd[p + "ffn_norm.weight"])
                out[b + "dw_w"] = t(sd[p + "mixer.conv.conv.conv.weight"].reshape(C, 7))
                out[b + "dw_b"] = t(sd[p + "mixer.conv.conv.conv.bias"])
                out[b + "gamma"] = t(sd[p + "gamma"])
                out[b + "ffn_gamma"] = t(sd[p + "ffn_gamma"])
                out[b + "fc1_w"] = t(sd[p + "ffn.linear1.weight"])
                out[b + "fc1_b"] = t(sd[p + "ffn.linear1.bias"])
                out[b + "fc2_w"] = t(sd[p + "ffn.linear2.weight"])
                out[b + "fc2_b"] = t(sd[p + "ffn.linear2.bias"])
    for k in list(out):
        if is_gemm_weight(k):
            out[k] = mfma_pack(out[k])
    return out


def write_synthetic_checkpoint(path, cfg: VibeVoiceConfig, seed=0, mode="bench", shard_bytes=2 << 30,
                               tokenizer_dir=None, speech_tok_compress_ratio=None, state_dict=None):
    """An offline stand-in for a HF checkpoint directory:
    config.json + `model-0000i-of-0000n.safetensors` shards with the reference's
    state-dict names + `model.safetensors.index.json` (metadata.total_size and
    the tensor -> shard weight_map a HF loader reads), so
    `from_pretrained(path)` and the demos' `--model_path` run without network.
    The lm_head is left out when the top-level `tie_word_embeddings` ties it to
    the embedding — the flag the reference's tie_weights reads
    (modeling_vibevoice_inference.py:120-129) and synthetic_state_dict uses.
    Stale shards / index of an earlier write are removed first (the loader
    would otherwise mix them in).  `tokenizer_dir`: also write the
    preprocessor_config.json VibeVoiceProcessor.from_pretrained(path) reads,
    naming that local Qwen2-style tokenizer (vibevoice_processor.py:67-105).
    `state_dict`: write these tensors instead of synthetic_state_dict(cfg, seed).
    Returns the shard file names."""
    import json
    import os
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    for f in os.listdir(path):
        if f.endswith(".safetensors") or f == "model.safetensors.index.json":
            os.remove(os.path.join(path, f))
    sd = state_dict if state_dict is not None else synthetic_state_dict(cfg, seed=seed, device="cpu", mode=mode)
    emb = sd[LM + "embed_tokens.weight"]
    drop_head = cfg.tie_word_embeddings or sd.get("lm_head.weight") is emb
    names = sorted(k for k in sd if not (drop_head and k == "lm_head.weight"))
    shards, cur, size = [], [], 0
    for k in names:
        nb = sd[k].numel() * sd[k].element_size()
        if cur and size + nb > shard_bytes:
            shards.append(cur)
            cur, size = [], 0
        cur.append(k)
        size += nb
    shards.append(cur)
    files = [f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors" for i in range(len(shards))]
    weight_map, total = {}, 0
    for f, part in zip(files, shards):
        save_file({k: sd[k].contiguous() for k in part}, os.path.join(path, f), metadata={"format": "pt"})
        for k in part:
            weight_map[k] = f
            total += sd[k].numel() * sd[k].element_size()
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as fh:
        json.dump({"metadata": {"total_size": total}, "weight_map": weight_map}, fh, indent=2)
    with open(os.path.join(path, "config.json"), "w") as fh:
        json.dump(cfg.to_dict(), fh, indent=2)
    if tokenizer_dir is not None:
        pc = {"processor_class": "VibeVoiceProcessor",
              "speech_tok_compress_ratio": int(speech_tok_compress_ratio or cfg.hop), "db_normalize": True,
              "audio_processor": {"feature_extractor_type": "VibeVoiceTokenizerProcessor", "sampling_rate": 24000,
                                  "normalize_audio": True, "target_dB_FS": -25, "eps": 1e-6},
              "language_model_pretrained_name": os.path.abspath(tokenizer_dir)}
        with open(os.path.join(path, "preprocessor_config.json"), "w") as fh:
            json.dump(pc, fh, indent=2)
    return files


if __name__ == "__main__":      # python -m vibevoice_amd.weights <dir> [1.5B|Large] [seed]
    import sys
    _dir, _name = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "1.5B")
    _seed = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    print("\n".join(write_synthetic_checkpoint(_dir, VibeVoiceConfig.builtin(_name), seed=_seed)))
