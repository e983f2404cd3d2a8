"""Weight layouts the fused diffusion-head FFN layer streams (csrc/head_ffn.hip),
host side only: weights.py's head_ffn_pack order is the one the kernel indexes
(workgroup w, chunk step i, thread t = rho * 16 + kap, 8 columns), it inverts,
and pack() emits the fused layer's streams exactly for the shape the kernel is
instantiated for (unsharded 1.5B head: H 1,536, F 4,608)."""
import torch

from tiny import tiny_config
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.weights import (HEAD_FFN_SHAPE, head_ffn_pack, head_ffn_unpack, head_layout_for, pack,
                                   synthetic_state_dict)


def test_head_ffn_pack_order_and_inverse():
    g = torch.Generator().manual_seed(3)
    H, F = HEAD_FFN_SHAPE
    gate = torch.randn(F, H, generator=g)
    up = torch.randn(F, H, generator=g)
    p = head_ffn_pack(gate, up)
    assert p.shape == (2 * F, H)
    G, HPW, KS, CPT, NT = 256, F // 256, 16, H // 8 // 16, 2 * (F // 256) * 16
    flat = p.reshape(-1)
    for (w, i, t, e) in [(0, 0, 0, 0), (5, 7, 123, 3), (255, 11, 575, 7), (100, 3, 17, 1)]:
        rho, kap = divmod(t, KS)
        u, which = divmod(rho, 2)
        src = gate if which == 0 else up
        assert flat[((w * CPT + i) * NT + t) * 8 + e] == src[w * HPW + u, (i * KS + kap) * 8 + e]
    g2, u2 = head_ffn_unpack(p)
    assert torch.equal(g2, gate) and torch.equal(u2, up)


def test_pack_emits_fused_streams_for_the_instantiated_shape():
    cfg = tiny_config(hidden=1536, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=1, device="cpu", mode="test", with_acoustic_encoder=False)
    w = pack(sd, cfg, "cpu", with_acoustic_encoder=False)
    P = "model.prediction_head.layers.0.ffn."
    assert torch.equal(w["head.0.dn_rows"], sd[P + "down_proj.weight"].t().contiguous().bfloat16())
    gate, up = head_ffn_unpack(w["head.0.gu_rows"])
    assert torch.equal(gate, sd[P + "gate_proj.weight"].bfloat16()) and torch.equal(up, sd[P + "up_proj.weight"].bfloat16())
    # a sharded head (F / 2 per rank) or another width has no fused streams
    w2 = pack(sd, cfg, "cpu", with_acoustic_encoder=False, tp_rank=0, tp_size=2, tp_head=True)
    assert "head.0.gu_rows" not in w2 and "head.0.dn_rows" not in w2
    small = tiny_config()
    ws = pack(synthetic_state_dict(small, seed=1, device="cpu", mode="test", with_acoustic_encoder=False), small, "cpu",
              with_acoustic_encoder=False)
    assert not any(k.endswith(("gu_rows", "dn_rows")) for k in ws)


def test_one_head_layout_resident():
    """an engine packs ONE copy of the head FFN -- by default
    the GEMV layout at every batch size (k_head_m16 runs 2 <= 2n <= 16 rows from
    it, faster at B = 1 than the persistent loop on the fused streams), the
    fused streams when asked -- and "both" only for tests switching paths on one
    engine.  1.5B: 170 MB saved."""
    cfg = VibeVoiceConfig.builtin("1.5B")
    assert head_layout_for(cfg, 1) == "gemv" and head_layout_for(cfg, 2) == "gemv"   # k_head_m16 at 2n <= 16
    assert head_layout_for(cfg, 3) == "gemv" and head_layout_for(cfg, 8) == "gemv"
    assert head_layout_for(cfg, 1, tp_size=2, tp_head=True) == "gemv"          # sharded width
    assert head_layout_for(VibeVoiceConfig.builtin("Large"), 1) == "gemv"
    sd = synthetic_state_dict(cfg, device="meta")
    sizes = {}
    for layout in ("fused", "gemv", "both"):
        w = pack(sd, cfg, "meta", head_layout=layout)
        has_f = all(f"head.{i}.gu_rows" in w and f"head.{i}.dn_rows" in w for i in range(4))
        has_g = all(f"head.{i}.gu_w" in w and f"head.{i}.down_w" in w for i in range(4))
        assert (has_f, has_g) == {"fused": (True, False), "gemv": (False, True), "both": (True, True)}[layout]
        sizes[layout] = sum(t.numel() * t.element_size() for t in w.values())
    ffn = 4 * 3 * 4608 * 1536 * 2
    assert sizes["both"] - sizes["fused"] == ffn and sizes["both"] - sizes["gemv"] == ffn
