"""Diffusion head + CFG DPM-Solver++ sampling on the GPU (vv_diffusion_sample).

Pinned two ways:
  * against the reference's own sample_speech_tokens output (committed golden
    tests/golden/g2_head.npz, bf16 model, H=128, S=5 and 10, cfg 1.3);
  * against the CPU oracle at the real 1.5B head shapes (H=1536) on seeded
    weights.
Tolerance (bf16 model; the reference's GPU path rounds at the same points but
accumulates GEMMs in a different order): rel L2 error of the latent < 2e-2,
cosine > 0.999.
"""
import pytest
import torch

from golden_io import load, t, weights
from gpu_util import cos, rel_err
from oracle import head as ohead
from tiny import tiny_config
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _collect_engines():
    """Engines of earlier tests / modules that are garbage but not yet collected
    still count as live contexts registered for the grid-waiting kernels
    (engine.cpp hl_register: they run only for a device's sole such context)."""
    import gc
    gc.collect()
    yield


def engine_with_head(cfg, head_sd, seed=0, max_batch=4):
    sd = synthetic_state_dict(cfg, seed=seed, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in head_sd.items():
        sd["model.prediction_head." + k] = v
    return Engine(cfg, sd, dev, max_batch=max_batch, max_ctx=256), sd


@pytest.mark.parametrize("S", [5, 10])
def test_head_vs_reference_golden(S):
    z = load("g2_head.npz")
    cfg = tiny_config()
    eng, _ = engine_with_head(cfg, weights(z, dtype=torch.bfloat16))
    eng.set_steps(S)
    pos = t(z, f"sst_pos_bf16_{S}", torch.bfloat16).to(dev)
    neg = t(z, f"sst_neg_bf16_{S}", torch.bfloat16).to(dev)
    n = pos.shape[0]
    x = t(z, f"sst_noise_{S}_bf16").to(torch.bfloat16)[:n].to(dev).contiguous()
    eng.diffusion_sample(pos, neg, x, 1.3)
    torch.cuda.synchronize()
    ref = t(z, f"sst_out_bf16_{S}")
    err, c = rel_err(x, ref), cos(x, ref)
    print(f"S={S} rel_err={err:.3e} cos={c:.6f}")
    assert err < 2e-2 and c > 0.999


def real_head_sd(g):
    from vibevoice_amd.config import VibeVoiceConfig
    cfg = VibeVoiceConfig.builtin("1.5B")
    hc = cfg.diffusion_head_config
    H, F = hc.hidden_size, int(hc.hidden_size * hc.head_ffn_ratio)
    sd = {}

    def r(*s, std):
        return (torch.randn(*s, generator=g) * std).bfloat16()
    sd["noisy_images_proj.weight"] = r(H, 64, std=0.125)
    sd["cond_proj.weight"] = r(H, H, std=H ** -0.5)
    sd["t_embedder.mlp.0.weight"] = r(H, 256, std=0.0625)
    sd["t_embedder.mlp.2.weight"] = r(H, H, std=H ** -0.5)
    for i in range(hc.head_layers):
        p = f"layers.{i}."
        sd[p + "ffn.gate_proj.weight"] = r(F, H, std=H ** -0.5)
        sd[p + "ffn.up_proj.weight"] = r(F, H, std=H ** -0.5)
        sd[p + "ffn.down_proj.weight"] = r(H, F, std=F ** -0.5)
        sd[p + "norm.weight"] = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
        sd[p + "adaLN_modulation.1.weight"] = r(3 * H, H, std=0.5 * H ** -0.5)
    sd["final_layer.linear.weight"] = r(64, H, std=H ** -0.5)
    sd["final_layer.adaLN_modulation.1.weight"] = r(2 * H, H, std=0.5 * H ** -0.5)
    return sd, hc, H


@pytest.mark.parametrize("n", [1, 3])
def test_head_sde_vs_oracle(n):
    """sde-dpmsolver++ (gradio_demo.py:114-118) at the real head shapes: the
    per-step fp32 noise is given to both; the oracle's SDE scheduler is pinned
    bit-exact to the reference (tests/golden/g1_sde_scheduler.npz)."""
    from vibevoice_amd.schedule import Schedule
    g = torch.Generator().manual_seed(12)
    sd, hc, H = real_head_sd(g)
    tiny = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    eng, _ = engine_with_head(tiny, sd)
    eng.set_schedule(Schedule.from_config(eng.schedule.config, algorithm_type="sde-dpmsolver++",
                                          beta_schedule="squaredcos_cap_v2"))
    S = 10
    eng.set_steps(S)
    pos = (torch.randn(n, H, generator=g)).bfloat16()
    neg = (torch.randn(n, H, generator=g)).bfloat16()
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    z = torch.randn(S, 2 * n, 64, generator=g)
    x = noise[:n].to(dev).contiguous()
    eng.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3, sde_noise=z.to(dev))
    torch.cuda.synchronize()
    ref = ohead.sample_speech_tokens(sd, pos, neg, noise, S, 1.3, hc.head_layers, sde_noise=z)
    err, c = rel_err(x, ref), cos(x, ref)
    print(f"SDE n={n} rel_err={err:.3e} cos={c:.6f}")
    assert err < 2e-2 and c > 0.999


@pytest.mark.parametrize("m16", [1, 0])
@pytest.mark.parametrize("n", [1, 2, 3])
def test_head_real_shape_vs_oracle(n, m16):
    """2n <= 16 rows run each FFN layer as one k_head_m16 launch by default;
    m16=0 forces the gate|up + down GEMV launches."""
    from vibevoice_amd import _lib
    from vibevoice_amd.config import VibeVoiceConfig
    _lib.lib().vv_head_m16(m16)
    cfg = VibeVoiceConfig.builtin("1.5B")
    hc = cfg.diffusion_head_config
    g = torch.Generator().manual_seed(11)
    H, F = hc.hidden_size, int(hc.hidden_size * hc.head_ffn_ratio)
    sd = {}

    def r(*s, std):
        return (torch.randn(*s, generator=g) * std).bfloat16()
    sd["noisy_images_proj.weight"] = r(H, 64, std=0.125)
    sd["cond_proj.weight"] = r(H, H, std=H ** -0.5)
    sd["t_embedder.mlp.0.weight"] = r(H, 256, std=0.0625)
    sd["t_embedder.mlp.2.weight"] = r(H, H, std=H ** -0.5)
    for i in range(hc.head_layers):
        p = f"layers.{i}."
        sd[p + "ffn.gate_proj.weight"] = r(F, H, std=H ** -0.5)
        sd[p + "ffn.up_proj.weight"] = r(F, H, std=H ** -0.5)
        sd[p + "ffn.down_proj.weight"] = r(H, F, std=F ** -0.5)
        sd[p + "norm.weight"] = (1 + 0.1 * torch.randn(H, generator=g)).bfloat16()
        sd[p + "adaLN_modulation.1.weight"] = r(3 * H, H, std=0.5 * H ** -0.5)
    sd["final_layer.linear.weight"] = r(64, H, std=H ** -0.5)
    sd["final_layer.adaLN_modulation.1.weight"] = r(2 * H, H, std=0.5 * H ** -0.5)
    # engine needs a whole model: tiny LM / codec at this hidden size are irrelevant here
    tiny = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    eng, _ = engine_with_head(tiny, sd)
    S = 10
    eng.set_steps(S)
    pos = r(n, H, std=1.0)
    neg = r(n, H, std=1.0)
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    x = noise[:n].to(dev).contiguous()
    try:
        eng.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3)
        torch.cuda.synchronize()
    finally:
        _lib.lib().vv_head_m16(1)
    eng.check_sync()
    ref = ohead.sample_speech_tokens(sd, pos, neg, noise, S, 1.3, hc.head_layers)
    err, c = rel_err(x, ref), cos(x, ref)
    print(f"n={n} m16={m16} rel_err={err:.3e} cos={c:.6f}")
    assert err < 2e-2 and c > 0.999


def test_one_launch_layer_only_for_the_devices_sole_context():
    """Two grid-waiting launches cannot be resident together (one workgroup per
    CU each): with a second registered context on the device, both take the
    GEMV launches; the first goes back to k_head_m16 when the second is
    destroyed, or when the second is switched off (vv_set_persistent: the
    standalone tokenizer API's codec context) -- graphs re-captured
    (vv_ws_epoch).  The GEMV path still matches the oracle."""
    from vibevoice_amd import _lib
    L = _lib.lib()
    g = torch.Generator().manual_seed(41)
    sd, hc, H = real_head_sd(g)
    tiny = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    a, _ = engine_with_head(tiny, sd)
    assert L.vv_head_m16_active(a.h, 1) == 1 and a.persistent_active()
    e0 = L.vv_ws_epoch()
    b, _ = engine_with_head(tiny, sd)
    assert L.vv_head_m16_active(a.h, 1) == 0 and L.vv_head_m16_active(b.h, 1) == 0
    assert L.vv_ws_epoch() != e0
    a.set_steps(10)
    pos = torch.randn(1, H, generator=g).bfloat16()
    neg = torch.randn(1, H, generator=g).bfloat16()
    noise = torch.randn(2, 64, generator=g).bfloat16()
    x = noise[:1].to(dev).contiguous()
    a.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3)
    torch.cuda.synchronize()
    ref = ohead.sample_speech_tokens(sd, pos, neg, noise, 10, 1.3, hc.head_layers)
    assert rel_err(x, ref) < 2e-2
    e1 = L.vv_ws_epoch()
    _lib.check(L.vv_set_persistent(b.h, 0), "set_persistent")
    assert L.vv_head_m16_active(a.h, 1) == 1 and not b.persistent_active() and L.vv_ws_epoch() != e1
    _lib.check(L.vv_set_persistent(b.h, 1), "set_persistent")
    assert L.vv_head_m16_active(a.h, 1) == 0
    b.close()
    assert L.vv_head_m16_active(a.h, 1) == 1
    a.close()
    # a context created with persistent=False never registers
    c = Engine(tiny, synthetic_state_dict(tiny, seed=0, device="cpu", mode="test", with_acoustic_encoder=False), dev,
               max_batch=1, max_ctx=64, persistent=False)
    assert not c.persistent_active() and L.vv_head_m16_active(c.h, 1) == 0
    # "follow" (the tokenizer API's codec context): runs the kernels while the
    # owner is the sole registered context, never demotes it
    f = Engine(tiny, synthetic_state_dict(tiny, seed=0, device="cpu", mode="test", with_acoustic_encoder=False), dev,
               max_batch=1, max_ctx=64, persistent="follow")
    assert not f.persistent_active()          # nobody registered
    o, _ = engine_with_head(tiny, sd)
    assert o.persistent_active() and f.persistent_active() and L.vv_head_m16_active(o.h, 1) == 1
    c.close()
    f.close()
    o.close()


@pytest.mark.parametrize("n", [1, 3, 8])
def test_head_m16_vs_oracle_and_gemv_pair(n):
    """configs[2]'s head (B = 8: 2n = 16 rows; n = 3, 1: 6, 2 rows, padded -- a
    GEMV-layout engine serving fewer samples): each FFN
    layer as ONE launch with one grid-wide hand-off (head_m16.hip: gate|up by
    MFMA over 2-3 tiles per workgroup, down over half a tile per two-tile
    workgroup) vs the oracle (rel < 2e-2, cosine > 0.999) and vs the
    gate|up + down GEMV launches (within bf16: the GEMM sums run in another
    order), the real 1.5B head shapes, S = 10, CFG 1.3; repeated calls and graph
    replays bitwise equal.  Layers l >= 1 build their A side distributed from the
    previous layer's row partials (default); the form that transforms the whole A
    side in every workgroup is checked the same way (its inverse RMS sums run in
    another order: within bf16 of it)."""
    from vibevoice_amd import _lib
    L = _lib.lib()
    g = torch.Generator().manual_seed(60 + n)
    sdh, hc, H = real_head_sd(g)
    cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in sdh.items():
        sd["model.prediction_head." + k] = v
    eng = Engine(cfg, sd, dev, max_batch=8, max_ctx=64)   # the GEMV layout (max_batch > 2)
    eng.set_steps(10)
    assert L.vv_head_m16_active(eng.h, n) == 1
    pos = torch.randn(n, H, generator=g).bfloat16()
    neg = torch.randn(n, H, generator=g).bfloat16()
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    ref = ohead.sample_speech_tokens(sdh, pos, neg, noise, 10, 1.3, hc.head_layers)
    outs = {}
    try:
        for mode, pre in ((1, 1), (0, 1), (1, 1), (1, 0)):
            L.vv_head_m16(mode)
            L.vv_head_m16_pre(pre)
            x = noise[:n].to(dev).contiguous()
            eng.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3)
            torch.cuda.synchronize()
            outs.setdefault(mode + 2 * (1 - pre), []).append(x.clone())
        L.vv_head_m16_pre(1)
        # graph replay of the one-launch layers (operands on the device before the capture)
        L.vv_head_m16(1)
        s = torch.cuda.Stream()
        pd, nd = pos.to(dev), neg.to(dev)
        xg = noise[:n].to(dev).contiguous()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            gr = torch.cuda.CUDAGraph()
            gr.capture_begin(capture_error_mode="thread_local")
            eng.diffusion_sample(pd, nd, xg, 1.3, stream=s)
            gr.capture_end()
        xg.copy_(noise[:n].to(dev))
        with torch.cuda.stream(s):
            gr.replay()
        torch.cuda.synchronize()
    finally:
        L.vv_head_m16(1)
        L.vv_head_m16_pre(1)
    eng.check_sync()
    m16, pair, whole = outs[1][0], outs[0][0], outs[3][0]
    e, ep, eb = rel_err(m16, ref), rel_err(pair, ref), rel_err(m16, pair)
    ew, ewd = rel_err(whole, ref), rel_err(m16, whole)
    print(f"head m16 n={n}: rel {e:.3e} vs oracle (GEMV pair {ep:.3e}, whole-A-side form {ew:.3e}), "
          f"{eb:.3e} vs the GEMV pair, {ewd:.3e} vs the whole-A-side form")
    assert torch.equal(m16, outs[1][1]) and torch.equal(m16, xg)
    assert e < 2e-2 and cos(m16, ref) > 0.999
    assert eb < 2e-2 and cos(m16, pair) > 0.999
    assert ew < 2e-2 and cos(whole, ref) > 0.999 and ewd < 2e-2


@pytest.mark.parametrize("n,S,sde", [(1, 10, False), (2, 5, False), (1, 7, True), (8, 10, False), (3, 5, True)])
def test_head_fin_one_launch_vs_oracle_and_gemv_pair(n, S, sde):
    """The step boundary (step s's final layer + CFG + DPM update, step s + 1's
    noisy projection) as ONE launch (head_fin.hip k_head_fin, 2n <= 4 rows: every
    workgroup computes the whole final layer, then its noisy tiles; latents, DPM
    history and state rows double-buffered over an even number of fused steps)
    at the 1.5B head shapes: vs the oracle (rel < 2e-2, cosine > 0.999), vs the
    two GEMV launches (within bf16: MFMA sums in another order), repeated runs
    bitwise equal.  S = 10: steps 1..8 fused; S = 5: 0..3; S = 7 with
    sde-dpmsolver++ noise: 0..5.  Above 4 rows (n = 3, 8) the noisy part is
    k_head_noisy16's arithmetic and also writes the row partials the next
    k_head_m16's distributed A side reads."""
    from vibevoice_amd import _lib
    from vibevoice_amd.schedule import Schedule
    L = _lib.lib()
    g = torch.Generator().manual_seed(31 + n + S)
    sd, hc, H = real_head_sd(g)
    tiny = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    eng, _ = engine_with_head(tiny, sd, max_batch=max(4, n))
    if sde:
        eng.set_schedule(Schedule.from_config(eng.schedule.config, algorithm_type="sde-dpmsolver++",
                                              beta_schedule="squaredcos_cap_v2"))
    eng.set_steps(S)
    assert L.vv_head_fin_active(eng.h, n) == 1
    pos = (torch.randn(n, H, generator=g)).bfloat16()
    neg = (torch.randn(n, H, generator=g)).bfloat16()
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    z = torch.randn(S, 2 * n, 64, generator=g) if sde else None
    outs = {}
    try:
        for on in (1, 0, 1):
            L.vv_head_fin(on)
            x = noise[:n].to(dev).contiguous()
            eng.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3, sde_noise=z.to(dev) if sde else None)
            torch.cuda.synchronize()
            outs.setdefault(on, []).append(x.clone())
    finally:
        L.vv_head_fin(1)
    eng.check_sync()
    ref = ohead.sample_speech_tokens(sd, pos, neg, noise, S, 1.3, hc.head_layers, sde_noise=z)
    one, pair = outs[1][0], outs[0][0]
    print(f"n={n} S={S} sde={sde}: one launch rel {rel_err(one, ref):.3e} vs oracle (GEMV pair "
          f"{rel_err(pair, ref):.3e}), {rel_err(one, pair):.3e} vs the pair")
    assert torch.equal(one, outs[1][1])
    assert rel_err(one, ref) < 2e-2 and cos(one, ref) > 0.999
    assert rel_err(one, pair) < 2e-2 and cos(one, pair) > 0.999
