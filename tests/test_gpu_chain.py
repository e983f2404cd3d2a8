"""Persistent GEMV chains (chain.hip): the diffusion head's S steps in one launch.

  * mirror mode (vv_chain_tune(2): the per-op kernels' launch plan) must be
    BIT-identical to the per-op launches -- the in-launch hand-offs (sc1 stores,
    sc1 loads, done counters, split tickets) then have nothing to hide behind;
  * the balanced plan (mode 1) re-splits K, so it differs from the per-op path
    by summation order only: deterministic run to run, rel L2 < 1e-2 against it;
  * no dependency wait gave up (vv_chain_error == 0).
The per-op reference runs with the fused head FFN layer and the one-launch
16-row layer switched off (they sum in a different order; tests/test_gpu_head.py
pins them).
Real VibeVoice-1.5B head shapes (H = 1536, FFN 4608, 4 layers), S = 10, CFG 1.3.
"""
import pytest
import torch

from gpu_util import cos, rel_err
from test_gpu_head import real_head_sd
from tiny import tiny_config
from vibevoice_amd import _lib
from vibevoice_amd.engine import Engine
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module")
def head_engine():
    g = torch.Generator().manual_seed(21)
    sd_head, hc, H = real_head_sd(g)
    cfg = tiny_config(hidden=H, layers=1, heads=12, kv_heads=2, inter=256)
    sd = synthetic_state_dict(cfg, seed=0, device="cpu", mode="test", with_acoustic_encoder=False)
    for k, v in sd_head.items():
        sd["model.prediction_head." + k] = v
    eng = Engine(cfg, sd, dev, max_batch=8, max_ctx=64)
    eng.set_steps(10)
    # the chain mirrors the per-op GEMV launches (gate|up, down); the fused FFN
    # layer (head_ffn.hip, the default at n <= 2) is a different summation order
    _lib.lib().vv_head_fused(0)
    _lib.lib().vv_head_m16(0)   # nor the one-launch layer at 4 < 2n <= 16 rows (head_m16.hip)
    yield eng, H, g
    _lib.lib().vv_chain_tune(0)
    _lib.lib().vv_head_fused(1)
    _lib.lib().vv_head_m16(1)


def run(eng, mode, pos, neg, noise, n, sde=None):
    _lib.lib().vv_chain_tune(mode)
    x = noise[:n].to(dev).contiguous()
    eng.diffusion_sample(pos.to(dev), neg.to(dev), x, 1.3, sde_noise=None if sde is None else sde.to(dev))
    torch.cuda.synchronize()
    assert _lib.lib().vv_chain_error(eng.h) == 0
    return x.cpu()


@pytest.mark.parametrize("n", [1, 2, 5, 8])
def test_head_chain_matches_per_op_launches(head_engine, n):
    eng, H, g = head_engine
    pos = torch.randn(n, H, generator=g).bfloat16()
    neg = torch.randn(n, H, generator=g).bfloat16()
    noise = torch.randn(2 * n, 64, generator=g).bfloat16()
    ref = run(eng, 0, pos, neg, noise, n)
    mir = run(eng, 2, pos, neg, noise, n)
    assert torch.equal(mir, ref), f"mirror chain differs: rel {rel_err(mir, ref):.3e}"
    bal = [run(eng, 1, pos, neg, noise, n) for _ in range(3)]
    assert torch.equal(bal[0], bal[1]) and torch.equal(bal[0], bal[2]), "balanced chain not deterministic"
    err, c = rel_err(bal[0], ref), cos(bal[0], ref)
    print(f"n={n} balanced vs per-op rel {err:.3e} cos {c:.6f}")
    assert err < 1e-2 and c > 0.9999


def test_head_chain_sde_binding(head_engine):
    """The per-call bindings (latents, per-step SDE noise, CFG scale) of the final op."""
    eng, H, g = head_engine
    from vibevoice_amd.schedule import Schedule
    base = eng.schedule
    eng.set_schedule(Schedule.from_config(base.config, algorithm_type="sde-dpmsolver++",
                                          beta_schedule="squaredcos_cap_v2"))
    eng.set_steps(10)
    try:
        n = 3
        pos = torch.randn(n, H, generator=g).bfloat16()
        neg = torch.randn(n, H, generator=g).bfloat16()
        noise = torch.randn(2 * n, 64, generator=g).bfloat16()
        z = torch.randn(10, 2 * n, 64, generator=g)
        ref = run(eng, 0, pos, neg, noise, n, sde=z)
        mir = run(eng, 2, pos, neg, noise, n, sde=z)
        assert torch.equal(mir, ref)
    finally:
        eng.set_schedule(base)
        eng.set_steps(10)
