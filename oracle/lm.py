"""Qwen2 decoder with a compacted per-row KV cache (oracle).

Restates the Qwen2 arithmetic the reference calls through
`VibeVoiceModel.forward` (vibevoice/modular/modeling_vibevoice.py:169-209 ->
transformers Qwen2Model, pinned 4.51.3 at pyproject.toml:22; restated from the
5.15.0 source, whose decode math is identical: modeling_qwen2.py:35-252):
  RMSNorm fp32 (eps 1e-6), bias-QKV, RoPE (theta from config, fp32 cos/sin cast
  to the activation dtype), GQA softmax(qK^T/sqrt(d)) in fp32 -> cast, SwiGLU MLP.
Positions: the reference derives position_ids = cumsum(attention_mask)-1
(HF 4.51.3 prepare_inputs_for_generation), so a row's position equals the
number of unmasked cache entries before it; a cache that keeps only the
unmasked entries (in order) therefore reproduces the reference exactly
(SURVEY.md §8a rows a3, a7).  `sd` holds `model.language_model.*` keys.
"""
import torch
import torch.nn.functional as F


def rms(x, w, eps):
    h = x.to(torch.float32)
    h = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
    return w * h.to(x.dtype)


def rope_cos_sin(pos, head_dim, theta, dtype):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float, device=pos.device) / head_dim))
    f = pos.float()[:, None] * inv[None, :]
    emb = torch.cat([f, f], dim=-1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def _rot(x):
    h = x.shape[-1] // 2
    return torch.cat([-x[..., h:], x[..., :h]], dim=-1)


class RowKV:
    """Compacted KV of one LM row: per layer K,V [n_kv, len, d]."""

    def __init__(self, n_layers):
        self.k = [None] * n_layers
        self.v = [None] * n_layers

    def length(self):
        return 0 if self.k[0] is None else self.k[0].shape[1]

    def truncate(self, n):
        for i in range(len(self.k)):
            if self.k[i] is not None:
                self.k[i] = self.k[i][:, :n]
                self.v[i] = self.v[i][:, :n]


def forward_rows(sd, cfg, x, kvs, commit=True):
    """Run T new tokens for each of R rows.

    x: [R, T, H] input embeddings; kvs: list of RowKV (len R).  Row r's new
    tokens take positions len_r .. len_r+T-1 and attend causally to the cache
    plus themselves.  Returns the final-norm hidden states [R, T, H].
    If commit is False the caches are left unchanged.
    """
    H = cfg["hidden_size"]
    nh, nkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    d = cfg.get("head_dim") or H // nh
    eps, theta = cfg["rms_norm_eps"], cfg["rope_theta"]
    R, T, _ = x.shape
    h = x
    new_kv = [([None] * cfg["num_hidden_layers"], [None] * cfg["num_hidden_layers"]) for _ in range(R)]
    for li in range(cfg["num_hidden_layers"]):
        p = f"layers.{li}."
        a = rms(h, sd[p + "input_layernorm.weight"], eps)
        q = F.linear(a, sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.q_proj.bias"])
        k = F.linear(a, sd[p + "self_attn.k_proj.weight"], sd[p + "self_attn.k_proj.bias"])
        v = F.linear(a, sd[p + "self_attn.v_proj.weight"], sd[p + "self_attn.v_proj.bias"])
        outs = []
        for r in range(R):
            L0 = kvs[r].length()
            pos = torch.arange(L0, L0 + T, device=x.device)
            cos, sin = rope_cos_sin(pos, d, theta, x.dtype)
            qr = q[r].view(T, nh, d).transpose(0, 1)
            kr = k[r].view(T, nkv, d).transpose(0, 1)
            vr = v[r].view(T, nkv, d).transpose(0, 1)
            qr = qr * cos + _rot(qr) * sin
            kr = kr * cos + _rot(kr) * sin
            kc = kr if kvs[r].k[li] is None else torch.cat([kvs[r].k[li], kr], dim=1)
            vc = vr if kvs[r].v[li] is None else torch.cat([kvs[r].v[li], vr], dim=1)
            new_kv[r][0][li], new_kv[r][1][li] = kc, vc
            rep = nh // nkv
            kk = kc.repeat_interleave(rep, dim=0)
            vv = vc.repeat_interleave(rep, dim=0)
            s = torch.matmul(qr, kk.transpose(1, 2)) * d ** -0.5
            mask = torch.full((T, kc.shape[1]), float("-inf"), device=x.device)
            mask = torch.triu(mask, diagonal=L0 + 1)
            pw = F.softmax(s.float() + mask, dim=-1).to(x.dtype)
            outs.append(torch.matmul(pw, vv).transpose(0, 1).reshape(T, nh * d))
        o = F.linear(torch.stack(outs), sd[p + "self_attn.o_proj.weight"])
        h = h + o
        a = rms(h, sd[p + "post_attention_layernorm.weight"], eps)
        m = F.linear(F.silu(F.linear(a, sd[p + "mlp.gate_proj.weight"])) * F.linear(a, sd[p + "mlp.up_proj.weight"]),
                     sd[p + "mlp.down_proj.weight"])
        h = h + m
    if commit:
        for r in range(R):
            kvs[r].k, kvs[r].v = new_kv[r]
    return rms(h, sd["norm.weight"], eps)


def forward_rows_masked(sd, cfg, x, kvs, masks):
    """One new token per row with an explicit attention mask, the way the
    reference runs its negative stream (DynamicCache + attention_mask,
    modeling_vibevoice_inference.py:591-604).

    masks[r]: bool [len_r + 1] over (existing cache entries, the new token).
    The new token's position is cumsum(mask)[-1] - 1 (HF 4.51.3
    prepare_inputs_for_generation); its K/V are always appended.
    """
    H = cfg["hidden_size"]
    nh, nkv = cfg["num_attention_heads"], cfg["num_key_value_heads"]
    d = cfg.get("head_dim") or H // nh
    eps, theta = cfg["rms_norm_eps"], cfg["rope_theta"]
    R = x.shape[0]
    h = x
    for li in range(cfg["num_hidden_layers"]):
        p = f"layers.{li}."
        a = rms(h, sd[p + "input_layernorm.weight"], eps)
        q = F.linear(a, sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.q_proj.bias"])
        k = F.linear(a, sd[p + "self_attn.k_proj.weight"], sd[p + "self_attn.k_proj.bias"])
        v = F.linear(a, sd[p + "self_attn.v_proj.weight"], sd[p + "self_attn.v_proj.bias"])
        outs = []
        for r in range(R):
            m = masks[r]
            pos = torch.tensor([int(m.long().sum()) - 1], device=x.device)
            cos, sin = rope_cos_sin(pos, d, theta, x.dtype)
            qr = q[r].view(1, nh, d).transpose(0, 1)
            kr = k[r].view(1, nkv, d).transpose(0, 1)
            vr = v[r].view(1, nkv, d).transpose(0, 1)
            qr = qr * cos + _rot(qr) * sin
            kr = kr * cos + _rot(kr) * sin
            kc = kr if kvs[r].k[li] is None else torch.cat([kvs[r].k[li], kr], dim=1)
            vc = vr if kvs[r].v[li] is None else torch.cat([kvs[r].v[li], vr], dim=1)
            kvs[r].k[li], kvs[r].v[li] = kc, vc
            rep = nh // nkv
            kk = kc.repeat_interleave(rep, dim=0)
            vv = vc.repeat_interleave(rep, dim=0)
            s = torch.matmul(qr, kk.transpose(1, 2)) * d ** -0.5
            bias = torch.zeros(kc.shape[1], device=x.device)
            bias[~m.to(x.device)] = float("-inf")
            pw = F.softmax(s.float() + bias, dim=-1).to(x.dtype)
            outs.append(torch.matmul(pw, vv).transpose(0, 1).reshape(1, nh * d))
        o = F.linear(torch.stack(outs), sd[p + "self_attn.o_proj.weight"])
        h = h + o
        a = rms(h, sd[p + "post_attention_layernorm.weight"], eps)
        h = h + F.linear(F.silu(F.linear(a, sd[p + "mlp.gate_proj.weight"])) * F.linear(a, sd[p + "mlp.up_proj.weight"]),
                         sd[p + "mlp.down_proj.weight"])
    return rms(h, sd["norm.weight"], eps)
