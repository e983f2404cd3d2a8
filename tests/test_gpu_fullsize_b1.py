"""Full-size parity of the SHIPPED B = 1 path (configs[1] / configs[0]'s
workload) on the MI355X: a VibeVoice-1.5B model built as bench.py builds it
(max_batch 1) and alone on the device, so the loop runs the LM MLP block as one
k_lm_ffn launch, each diffusion-head FFN layer as one k_head_m16 launch (2
rows, whole A side) and the persistent codec stages (k_codec_stage /
k_codec_stage_s) -- asserted, not assumed.  The second case is the same model
with the grid-waiting kernels switched off (persistent=False: the GEMV
launches every shared-GPU deployment falls back to).
Teacher forcing against oracle/loop.py exactly as tests/test_gpu_fullsize.py
(whose shared max_batch-8 model runs two samples): per step and quantity, rel
L2 under the fixed bounds of tests/teacher.py and within 2.5x the bf16
reference's own deviation from fp32."""
import gc
import os

import pytest
import torch

from teacher import oracle_run, per_step_check, teacher_forced
from test_gpu_fullsize import IDS, SEED, STEPS, TK, D, E, S, X, _cpu_copy, _voice_noise
from vibevoice_amd import _lib
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.synthetic import synthetic_inputs
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", params=["default", "no_persistent"])
def m1(request):
    gc.collect()   # the persistent kernels run only for the device's sole registered context
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = VibeVoiceConfig.builtin("1.5B")
    sd_dev = synthetic_state_dict(cfg, seed=5, device=dev, mode="test")
    kw = {} if request.param == "default" else {"persistent": False}
    model = VibeVoiceForConditionalGenerationInference(cfg, sd_dev, dev, max_batch=1, max_ctx=1024, **kw)
    model.set_ddpm_inference_steps(STEPS)
    yield request.param, cfg, model, _cpu_copy(sd_dev)
    del model
    gc.collect()


@pytest.mark.parametrize("steps", [10, 5])
def test_teacher_forced_shipped_b1_path(m1, steps):
    layout, cfg, model, sd = m1
    L = _lib.lib()
    on = layout == "default"
    assert (L.vv_head_m16_active(model.engine.h, 1) == 1) == on, "k_head_m16"
    assert (L.vv_lm_ffn_active(model.engine.h, 2) == 1) == on, "k_lm_ffn"
    assert (L.vv_codec_stage_active(model.engine.h) == 1) == on, "k_codec_stage"
    inp = synthetic_inputs(batch=1, speakers=1, voice_seconds=3.0, text_tokens=64, seed=100)
    sched = [[D] * 6 + [E, S, D, D, X]]
    vn = _voice_noise(inp, cfg.acoustic_vae_dim)
    rec16, seqs, _, _ = oracle_run(sd, cfg, inp, sched, IDS, steps, vn, SEED, dtype=torch.bfloat16)
    sd32 = {k: v.float() for k, v in sd.items()}
    rec32, _, _, _ = oracle_run(sd32, cfg, inp, sched, IDS, steps, vn, SEED, dtype=torch.float32, teacher=rec16)
    model.set_ddpm_inference_steps(steps)
    try:
        got, sess = teacher_forced(model, inp, sched, rec16, TK, SEED)
    finally:
        model.set_ddpm_inference_steps(STEPS)
    assert len(got["latents"]) == len(rec16["latents"]) == 8
    assert torch.equal(sess.result().sequences, seqs)
    per_step_check(got, rec16, rec32, f"1.5B B=1 S={steps}, {layout} head layout + codec stages")
