"""Tensor-parallel weight sharding (weights.pack, CPU): the ranks' shards of
every Qwen2 layer tile the TP=1 packing exactly once — q/k/v/bias rows per
head, gate/up rows per intermediate slice, o/down input columns — and shapes
that do not shard cleanly are rejected."""
import pytest
import torch

from tiny import tiny_config
from vibevoice_amd.weights import mfma_unpack, pack, synthetic_state_dict, tp_check


def _unrope(x, nheads, d=128):
    rest = x.shape[1:]
    return x.reshape(nheads, d // 16, 2, 8, *rest).transpose(1, 2).reshape(nheads * d, *rest)


def _ungu(w):
    n2, H = w.shape
    y = w.reshape(n2 // 16, 2, 8, H)
    return y[:, 0].reshape(-1, H), y[:, 1].reshape(-1, H)


@pytest.mark.parametrize("tp", [2, 4])
def test_shards_tile_the_layer(tp):
    cfg = tiny_config(hidden=256, layers=1, heads=8, kv_heads=4, inter=512)
    sd = synthetic_state_dict(cfg, seed=3, device="cpu", mode="test", with_acoustic_encoder=False)
    ref = pack(sd, cfg, "cpu")
    shards = [pack(sd, cfg, "cpu", tp_rank=r, tp_size=tp) for r in range(tp)]
    nh, nkv, d = 8, 4, 128
    p = "model.language_model.layers.0."

    def qkv(w, nhl, nkvl):
        w = mfma_unpack(w) if w.dim() == 2 else w
        q, k, v = w[:nhl * d], w[nhl * d:(nhl + nkvl) * d], w[(nhl + nkvl) * d:]
        return _unrope(q, nhl), _unrope(k, nkvl), v

    q = torch.cat([qkv(s_["lm.0.qkv_w"], nh // tp, nkv // tp)[0] for s_ in shards])
    k = torch.cat([qkv(s_["lm.0.qkv_w"], nh // tp, nkv // tp)[1] for s_ in shards])
    v = torch.cat([qkv(s_["lm.0.qkv_w"], nh // tp, nkv // tp)[2] for s_ in shards])
    assert torch.equal(q, sd[p + "self_attn.q_proj.weight"])
    assert torch.equal(k, sd[p + "self_attn.k_proj.weight"])
    assert torch.equal(v, sd[p + "self_attn.v_proj.weight"])
    qb = torch.cat([qkv(s_["lm.0.qkv_b"], nh // tp, nkv // tp)[0] for s_ in shards])
    assert torch.equal(qb, sd[p + "self_attn.q_proj.bias"])
    o = torch.cat([mfma_unpack(s_["lm.0.o_w"]) for s_ in shards], 1)
    assert torch.equal(o, sd[p + "self_attn.o_proj.weight"])
    gates, ups = zip(*[_ungu(mfma_unpack(s_["lm.0.gu_w"])) for s_ in shards])
    assert torch.equal(torch.cat(gates), sd[p + "mlp.gate_proj.weight"])
    assert torch.equal(torch.cat(ups), sd[p + "mlp.up_proj.weight"])
    down = torch.cat([mfma_unpack(s_["lm.0.down_w"]) for s_ in shards], 1)
    assert torch.equal(down, sd[p + "mlp.down_proj.weight"])
    # everything outside the backbone layers is replicated
    for name in ("lm.embed", "lm.norm", "head.ada_w", "dec.stem_w", "conn.ac.fc1_w"):
        for s_ in shards:
            assert torch.equal(s_[name], ref[name]), name


def test_unclean_shards_rejected():
    cfg = tiny_config(hidden=256, layers=1, heads=2, kv_heads=2, inter=512)
    tp_check(cfg, 2)
    with pytest.raises(ValueError):
        tp_check(cfg, 4)
