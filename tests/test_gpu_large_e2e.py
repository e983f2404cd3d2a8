"""configs[3] as a whole model: VibeVoice-Large (28 Qwen2 layers at H 3584,
28 q / 4 kv heads, I 18,944, vocab 152,064; diffusion head H 3584 x 4 layers;
the real σ-VAE codec; acoustic / semantic connectors 64 -> 3584 and
128 -> 3584, modeling_vibevoice.py:58-69), a 4-speaker conversation prompt
(vibevoice_processor.py:246-304: four ragged voice clips through the acoustic
encoder, four script lines), teacher-forced against oracle/loop.py.

The oracle is the checker, run on the GPU with torch's own operators (a 7B
bf16 CPU loop would take the box minutes per step; test_gpu_large.py's 64K
check does the same), and cuDNN/MIOpen is switched off so its convolutions
are ATen's native im2col/depthwise kernels.  The product runs the same
synthetic weights through libvibevoice_hip.so.  Bounds: the fixed per-step
rel-L2 bounds of tests/teacher.py.
"""
import os
import types

import pytest
import torch

from gpu_util import cos, rel_err
from teacher import oracle_run, per_step_check, teacher_forced
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
TK = tokenizer_ids()
IDS = dict(eos=TK.eos_token_id, start=TK.speech_start_id, end=TK.speech_end_id, diffusion=TK.speech_diffusion_id)
D, E, S, X = IDS["diffusion"], IDS["end"], IDS["start"], IDS["eos"]
SEED = 4321
STEPS = 10


@pytest.fixture(scope="module")
def large():
    cfg = VibeVoiceConfig.builtin("Large")
    assert cfg.decoder_config.hidden_size == 3584 and cfg.decoder_config.num_hidden_layers == 28
    sd = synthetic_state_dict(cfg, seed=7, device=dev, mode="test")
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=1, max_ctx=1024)
    model.set_ddpm_inference_steps(STEPS)
    cudnn = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    yield types.SimpleNamespace(cfg=cfg, model=model, sd=sd)
    torch.backends.cudnn.enabled = cudnn


def _voice_noise(inp, D_lat, seed=11):
    nv, fr = inp["speech_masks"].shape
    g = torch.Generator().manual_seed(seed)
    return torch.randn(nv, generator=g), torch.randn(nv, fr, D_lat, generator=g)


def test_large_connectors_real_shape(large):
    """SpeechConnector x2 at H = 3584 (fc1 -> RMSNorm 1e-6 -> fc2) vs the
    oracle's, 40 rows each."""
    from oracle import loop as oloop
    g = torch.Generator(device=dev).manual_seed(3)
    eng = large.model.engine
    for which, p, din in ((0, "model.acoustic_connector.", 64), (1, "model.semantic_connector.", 128)):
        x = torch.randn(40, din, device=dev, generator=g).bfloat16()
        y = eng.connector(which, x)
        with torch.no_grad():
            ref = oloop.connector(large.sd, p, x)
        torch.cuda.synchronize()
        e = rel_err(y, ref)
        print(f"Large connector {which}: rel {e:.3e} cos {cos(y, ref):.6f}")
        assert y.shape == ref.shape == (40, 3584) and e < 1e-2


def test_teacher_forced_large_4_speakers(large):
    """A 4-speaker Large conversation: 28-layer prefill of the voice + script
    prompt, then diffusion steps with a speech_end / speech_start turn change
    (codec reset, negative-stream reset), eos.  Every step's hidden states,
    4 legal logits, latents, audio and connector embeddings within the fixed
    bounds."""
    inp = synthetic_inputs(batch=1, speakers=4, voice_seconds=[3.0, 2.2, 1.3, 2.7], text_tokens=64, seed=200)
    assert inp["speech_tensors"].shape[0] == 4
    sched = [[D, D, D, D, E, S, D, D, D, X]]
    vn = _voice_noise(inp, large.cfg.acoustic_vae_dim)
    print(f"Large prompt: {int(inp['attention_mask'].sum())} tokens, "
          f"{int(inp['speech_masks'].sum())} voice frames from 4 speakers")
    with torch.no_grad():
        rec16, seqs, _, _ = oracle_run(large.sd, large.cfg, inp, sched, IDS, STEPS, vn, SEED)
        sd32 = {k: v.float() for k, v in large.sd.items()}     # the bf16 reference's own deviation, for scale
        rec32, _, _, _ = oracle_run(sd32, large.cfg, inp, sched, IDS, STEPS, vn, SEED, dtype=torch.float32,
                                    teacher=rec16)
        del sd32
    got, sess = teacher_forced(large.model, inp, sched, rec16, TK, SEED)
    assert torch.equal(sess.result().sequences, seqs)
    per_step_check(got, rec16, rec32, "Large 4-speaker")


def test_large_tp4_group_28_layers(large):
    """configs[3]'s parallelism at full depth: the 28-layer Large backbone split
    over 4 ranks (Megatron split of configuration_vibevoice.py:175-183, whole KV
    heads per rank: 4 kv heads -> 1 per rank), driven as one group on this GPU
    (vv_lm_forward_group: an on-device sum stands in for the RCCL all-reduce)
    vs the TP = 1 engine: a 300-token prefill and 3 decode steps."""
    from vibevoice_amd.engine import Engine
    VALID = sorted(IDS.values())
    full = large.model.engine
    full.set_valid_ids(VALID)
    group = [Engine(large.cfg, large.sd, dev, max_batch=1, max_ctx=512, valid_ids=VALID, tp_rank=r, tp_size=4)
             for r in range(4)]
    i32 = dict(dtype=torch.int32, device=dev)
    g = torch.Generator(device=dev).manual_seed(12)
    N = 300
    x = torch.randn(N, 3584, device=dev, generator=g).bfloat16()
    args = (x, torch.zeros(N, **i32), torch.arange(N).to(**i32), torch.tensor([N - 1]).to(**i32))
    h1, l1 = full.lm_forward(*args)
    hg, lg = group[0].lm_forward_group(group[1:], *args)
    torch.cuda.synchronize()
    print(f"Large 28-layer TP=4 prefill: rel {rel_err(hg, h1):.3e} cos {cos(hg, h1):.6f}")
    assert rel_err(hg, h1) < 3e-2 and cos(hg, h1) > 0.999
    for s in range(3):
        step = torch.randn(1, 3584, device=dev, generator=g).bfloat16()
        a = (step, torch.zeros(1, **i32), torch.tensor([N + s]).to(**i32), torch.zeros(1, **i32))
        h1, l1 = full.lm_forward(*a)
        hg, lg = group[0].lm_forward_group(group[1:], *a)
        torch.cuda.synchronize()
        print(f"Large 28-layer TP=4 step {s}: rel {rel_err(hg, h1):.3e} cos {cos(hg, h1):.6f}")
        assert rel_err(hg, h1) < 3e-2 and cos(hg, h1) > 0.999
        assert torch.allclose(lg, l1, rtol=5e-2, atol=5e-2 * l1.abs().max().item())
    for e in group:
        e.close()
