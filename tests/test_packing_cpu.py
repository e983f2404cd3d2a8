"""Weight layouts of the diffusion head's FFN, host side only: pack() emits ONE
copy (the GEMV layout: gate|up interleaved in blocks of 8 rows, then
MFMA-fragment packed) that k_head_m16 (2 <= 2n <= 16 rows) and the GEMV pair
beyond both read, for the unsharded and the TP-sharded head."""
import torch

from tiny import tiny_config
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.weights import mfma_pack, mfma_unpack, pack, synthetic_state_dict


def test_mfma_pack_inverse_and_fragment_order():
    g = torch.Generator().manual_seed(3)
    w = torch.randn(64, 96, generator=g)
    p = mfma_pack(w)
    assert torch.equal(mfma_unpack(p), w)
    flat = p.reshape(-1)
    # block (tile t, chunk c) = 1 KB; lane l holds W[16t + (l & 15)][32c + 8(l >> 4) .. +7]
    for t, c, l, e in [(0, 0, 0, 0), (3, 2, 63, 7), (1, 1, 17, 3)]:
        assert flat[((t * 3 + c) * 64 + l) * 8 + e] == w[16 * t + (l & 15), 32 * c + 8 * (l >> 4) + e]


def test_one_head_layout_resident():
    """one copy of the head FFN, in the GEMV
    layout, at every batch size and sharding (the fused layer's streams and
    their kernels were removed in round 6)."""
    cfg = tiny_config(hidden=1536, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=1, device="cpu", mode="test", with_acoustic_encoder=False)
    for kw in ({}, {"tp_rank": 1, "tp_size": 2, "tp_head": True}):
        w = pack(sd, cfg, "cpu", with_acoustic_encoder=False, **kw)
        assert not any(k.endswith(("gu_rows", "dn_rows")) for k in w)
        P = "model.prediction_head.layers.0.ffn."
        F = sd[P + "gate_proj.weight"].shape[0]
        hs = slice(F // 2, F) if kw else slice(0, F)
        gu = w["head.0.gu_w"].float()
        gate = sd[P + "gate_proj.weight"][hs].bfloat16().float()
        up = sd[P + "up_proj.weight"][hs].bfloat16().float()
        n = gate.shape[0]
        inter = torch.stack([gate.reshape(n // 8, 8, -1), up.reshape(n // 8, 8, -1)], 1).reshape(2 * n, -1)
        assert torch.equal(mfma_unpack(gu), inter)      # every GEMM weight is MFMA-packed
    big = VibeVoiceConfig.builtin("1.5B")
    wm = pack(synthetic_state_dict(big, device="meta"), big, "meta")
    ffn = sum(t.numel() * t.element_size() for k, t in wm.items() if k.startswith("head.") and
              k.endswith((".gu_w", ".down_w")))
    assert ffn == 4 * 3 * 4608 * 1536 * 2     # 170 MB, once

