"""bench.py's algorithmic bytes per token, host only, on
shape-only (meta) weights of the real 1.5B model: every weight role is counted
once, in the layout the loop reads at that batch, and the stacked adaLN matrix
once per token (its one batched GEMM covers all S <= 16 steps' modulations,
engine.cpp head_mods).  Round 4's line counted a second head layout (+1.7 GB
per token) and the adaLN matrix S times (+0.6 GB)."""
import pytest
import torch

import bench
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.weights import pack, synthetic_state_dict


@pytest.fixture(scope="module")
def packed_1p5b():
    cfg = VibeVoiceConfig.builtin("1.5B")
    return cfg, pack(synthetic_state_dict(cfg, device="meta"), cfg, "meta")


def _nbytes(w, pred):
    return sum(t.numel() * t.element_size() for k, t in w.items() if pred(k))


def test_bytes_per_token_1p5b_b1_s10(packed_1p5b):
    cfg, w = packed_1p5b
    H, F, L = 1536, 4608, 4
    wb = bench.weight_bytes(w, B=1, S=10)
    assert wb["head_layout"].startswith("GEMV")
    # per diffusion step: 4 x (gate|up + down + norm) + noisy + final projections
    assert wb["head_step"] == L * (3 * F * H * 2 + H * 2) + 2 * 64 * H * 2
    # per token: cond_proj + the stacked adaLN matrix ((3L + 2) H x H) once
    assert wb["head_token"] == H * H * 2 + (3 * L + 2) * H * H * 2
    assert wb["lm"] == _nbytes(w, lambda k: k.startswith("lm.") and k not in ("lm.embed", "lm.lm_head", "lm.inv_freq"))
    bpt = bench.bytes_per_token(wb, cfg, B=1, S=10, ctx_pos=0, ctx_neg=0)
    assert bpt == 5_780_906_562 + 2 * 28_672   # weights + the two appended KV rows
    # at the bench's context (~900 positive / ~780 negative cached positions) it is ~5.83 GB
    assert 5.82e9 < bench.bytes_per_token(wb, cfg, 1, 10, 900, 780) < 5.84e9


def test_each_head_role_counted_once(packed_1p5b):
    cfg, w = packed_1p5b
    ffn = _nbytes(w, lambda k: k.startswith("head.") and k.endswith((".gu_w", ".down_w")))
    wb1, wb8 = bench.weight_bytes(w, B=1, S=10), bench.weight_bytes(w, B=8, S=10)
    assert wb1["head_step"] == wb8["head_step"]            # the same roles at either batch
    assert wb1["head_step"] < 2 * ffn                      # each role once
    assert wb8["head_layout"].startswith("GEMV")
    # S > 16: the adaLN GEMM runs once per 16 steps
    assert bench.weight_bytes(w, B=1, S=20)["head_token"] - wb1["head_token"] == 14 * 1536 * 1536 * 2


def test_roof_refuses_fractions_above_one():
    bad = bench.roof("k", "s", 42_479_616, 0.18e-6)
    assert bad["frac"] is None and "error" in bad
    ok = bench.roof("k", "s", 42_479_616, 15.8e-6)
    assert 0.33 < ok["frac"] < 0.34 and "error" not in ok
    assert torch.isfinite(torch.tensor(ok["achieved"]))
