"""Full-size parity on the MI355X: VibeVoice-1.5B (28 Qwen2 layers, H 1536,
12 q / 2 kv heads, I 8960; diffusion head H 1536 x 4 layers; the real 7-stage
σ-VAE codec, hop 3200) against oracle/loop.py, the CPU restatement pinned to
the reference's own generate() by golden G8.

Workloads (BASELINE.json configs[1] and configs[2]):
  * B = 1, one 3 s voice prompt (72,000 samples -> 23 latent frames through the
    real acoustic encoder), 10 diffusion steps, cfg 1.3;
  * B = 8 two-speaker dialogues, ragged voice clips (3.0 / 2.2 / 1.3 / 2.7 s)
    and ragged, left-padded scripts, forced schedules mixing speech_diffusion,
    speech_end (codec reset), speech_start (negative-stream reset), the skip
    correction and eos.
Weights: seeded synthetic, mode "test" (fan-in-scaled linears, random norms,
biases and layer-scale gammas, so every term of every kernel contributes).

Teacher forcing (the per-step check `north_star` names: acoustic-latent L2):
the oracle runs the loop in bf16 (the reference's GPU dtype) and records each
step's inputs.  The product loop is then driven with exactly those inputs —
the prompt embeddings, every step's next input embedding and, for the codec,
every step's latent — so each step's outputs (positive / negative hidden
states, the 4 legal logits, the diffusion latents, the audio chunk) measure
one step of arithmetic, not accumulated drift.  The reference's own bf16
error is measured the same way: the oracle in fp32, teacher-forced on the bf16
run.  Bound, per step and quantity: rel L2 < max(floor, 2 x that bf16
self-deviation), floors: hidden 2e-2, latents 2e-2, audio 2e-2.
Free-running (no forcing): token sequences equal, audio within
max(5e-2, 2 x the free-running bf16 self-deviation), as the tiny-config tests.
"""
import os
import types

import pytest
import torch

from gpu_util import cos, rel_err
from oracle import codec as ocodec
from oracle import loop as oloop
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
TK = tokenizer_ids()
IDS = dict(eos=TK.eos_token_id, start=TK.speech_start_id, end=TK.speech_end_id, diffusion=TK.speech_diffusion_id)
D, E, S, X = IDS["diffusion"], IDS["end"], IDS["start"], IDS["eos"]
FLOOR = dict(hpos=2e-2, hneg=2e-2, latents=2e-2, audio=2e-2)
STEPS = 10
SEED = 1234


def _cpu_copy(sd_dev):
    """CPU copy of a device state dict, keeping tied tensors tied."""
    out, seen = {}, {}
    for k, v in sd_dev.items():
        key = v.data_ptr()
        if key not in seen:
            seen[key] = v.cpu()
        out[k] = seen[key]
    return out


@pytest.fixture(scope="module")
def m15():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = VibeVoiceConfig.builtin("1.5B")
    sd_dev = synthetic_state_dict(cfg, seed=5, device=dev, mode="test")
    model = VibeVoiceForConditionalGenerationInference(cfg, sd_dev, dev, max_batch=8, max_ctx=1024)
    model.set_ddpm_inference_steps(STEPS)
    sd = _cpu_copy(sd_dev)
    return types.SimpleNamespace(cfg=cfg, model=model, sd=sd, sd32=None)


def _sd32(m):
    if m.sd32 is None:
        m.sd32 = {k: v.float() for k, v in m.sd.items()}
    return m.sd32


def _voice_noise(inp, D_lat, seed=9):
    nv, fr = inp["speech_masks"].shape
    g = torch.Generator().manual_seed(seed)
    return torch.randn(nv, generator=g), torch.randn(nv, fr, D_lat, generator=g)


def _oracle(m, inp, sched, vn, dtype=torch.bfloat16, teacher=None, max_new=None):
    rec = {}
    sd = m.sd if dtype == torch.bfloat16 else _sd32(m)
    torch.manual_seed(SEED)
    seqs, audio, reach = oloop.generate(sd, m.cfg, inp["input_ids"], inp["attention_mask"], IDS, ddpm_steps=STEPS,
                                        cfg_scale=1.3, forced=sched, dtype=dtype, record=rec, voice_noise=vn,
                                        teacher=teacher, max_new_tokens=max_new,
                                        speech_tensors=inp["speech_tensors"], speech_masks=inp["speech_masks"],
                                        speech_input_mask=inp["speech_input_mask"])
    return rec, seqs, audio, reach


def _teacher_forced(model, inp, sched, rec):
    """Drive the product loop with the oracle run's inputs (see module doc).
    Returns the per-step outputs the product computed."""
    B = inp["input_ids"].shape[0]
    got = dict(hpos=[], hneg=[], logits=[], latents=[], audio=[])
    pe = rec["prompt_embeds"].to(dev, torch.bfloat16)
    orig = model._prompt_embeds
    model._prompt_embeds = lambda *a, **k: pe.clone()
    try:
        torch.manual_seed(SEED)
        sess = model.generate_session(input_ids=inp["input_ids"], attention_mask=inp["attention_mask"], tokenizer=TK,
                                      cfg_scale=1.3, forced_tokens=sched, show_progress_bar=False,
                                      max_new_tokens=max(len(s) for s in sched) + 2)
    finally:
        model._prompt_embeds = orig
    post = sess._post_phase

    def hooked(n):
        k = sess.step_idx
        got["hpos"].append(sess.hid[:B].float().cpu())
        got["hneg"].append(sess.hid[B:].float().cpu())
        got["logits"].append(sess.logits_pin.clone()[:, sess.order])          # sorted ids, as the oracle records
        if n:
            got["latents"].append(sess.noise_dev[:n].float().cpu())
            sess.noise_dev[:n].copy_(rec["latents"][len(got["latents"]) - 1].to(dev, torch.bfloat16))
        post(n)
        if n:
            got["audio"].append(sess.audio_dev[:n].float().cpu())
        sess.x_in2[:B].copy_(rec["next_embeds"][k].to(dev, torch.bfloat16))
    sess._post_phase = hooked
    while sess.step():
        pass
    torch.cuda.synchronize()
    return got, sess


def _per_step_check(got, rec16, rec32, tag):
    """rel L2 per step and quantity vs the bf16 oracle; bound max(floor, 2 x
    the fp32-vs-bf16 deviation of the oracle on the same inputs)."""
    worst = {}
    fails = []
    dsteps = [k for k, d in enumerate(rec16["didx"]) if d.numel()]
    for q in ("hpos", "hneg", "latents", "audio"):
        for j in range(len(got[q]) if q in ("latents", "audio") else len(rec16["hpos"])):
            if q in ("latents", "audio"):
                r, r32 = rec16[q][j], rec32[q][j]
                g = got[q][j].reshape(r.shape)
            elif q == "hneg":
                if rec16["hneg"][j] is None or j not in dsteps:
                    continue
                rows = rec16["didx"][j]                 # the rows the head consumes
                g, r, r32 = got[q][j][rows], rec16[q][j][rows], rec32[q][j][rows]
            else:
                g, r, r32 = got[q][j], rec16[q][j], rec32[q][j]
            e, self_dev = rel_err(g, r), rel_err(r32, r)
            bound = max(FLOOR[q], 2 * self_dev)
            worst[q] = max(worst.get(q, (0, 0, 0)), (e, self_dev, bound))
            if not e < bound:
                fails.append(f"{q}[{j}] rel {e:.3e} >= {bound:.3e} (bf16 self-dev {self_dev:.3e})")
    for q, (e, sd_, b) in worst.items():
        print(f"{tag} {q}: worst rel {e:.3e} (bf16 reference self-deviation {sd_:.3e}, bound {b:.3e})")
    lg = max(rel_err(g, r) for g, r in zip(got["logits"], rec16["logits"]))
    print(f"{tag} logits(4 legal): worst rel {lg:.3e}")
    assert not fails, "\n".join(fails)


def test_acoustic_encoder_real_shape(m15):
    """The voice-prompt encoder at its real shape (modular_vibevoice_tokenizer.py
    :687-813, 1081-1085; ratios [2,2,4,5,5,8], depths 3-3-3-3-3-3-8, 32 -> 2048
    channels): a 3 s clip (72,000 samples -> 23 frames) and a ragged 1.3 s clip
    zero-padded beside it, vs the oracle's non-streaming encode in bf16; bound
    max(2e-2, 2 x the bf16 oracle's deviation from fp32)."""
    eng = m15.model.engine
    inp = synthetic_inputs(batch=2, speakers=1, voice_seconds=[3.0, 1.3], seed=3)
    audio = inp["speech_tensors"]
    assert audio.shape == (2, 72000)
    mean = eng.acoustic_encode(audio.to(dev, torch.bfloat16)).float().cpu()
    asd = {k[len("model.acoustic_tokenizer."):]: v for k, v in m15.sd.items()
           if k.startswith("model.acoustic_tokenizer.")}
    dims = ocodec.codec_dims(m15.cfg.acoustic_tokenizer_config, "encoder")
    ref = ocodec.encode(asd, dims, audio.to(torch.bfloat16).unsqueeze(1), None, None, streaming=False).float()
    ref32 = ocodec.encode({k: v.float() for k, v in asd.items()}, dims, audio.to(torch.bfloat16).float().unsqueeze(1),
                          None, None, streaming=False)
    assert mean.shape == ref.shape == (2, 23, 64), (mean.shape, ref.shape)
    for i in range(2):
        e, sdev = rel_err(mean[i], ref[i]), rel_err(ref32[i], ref[i])
        print(f"encoder clip {i}: rel {e:.3e} cos {cos(mean[i], ref[i]):.6f} (bf16 self-dev {sdev:.3e})")
        assert e < max(2e-2, 2 * sdev)


def test_prompt_embeds_real_shape(m15):
    """_process_speech_inputs + the splice at speech_input_mask
    (modeling_vibevoice_inference.py:150-177, 221-225) at 1.5B: encoder,
    gaussian sample (device draws replayed into the oracle), scaling, acoustic
    connector, scatter — two samples, ragged clips."""
    model = m15.model
    inp = synthetic_inputs(batch=2, speakers=1, voice_seconds=[3.0, 1.3], seed=4, text_jitter=8)
    torch.manual_seed(SEED)
    emb = model._prompt_embeds(inp["input_ids"].to(dev), inp["attention_mask"].to(dev), inp["speech_tensors"],
                               inp["speech_masks"], inp["speech_input_mask"]).float().cpu()
    nv, fr = inp["speech_masks"].shape
    torch.cuda.manual_seed(SEED)
    draw = torch.randn(nv, device=dev, dtype=torch.bfloat16).cpu()
    eps = torch.randn(nv, fr, m15.cfg.acoustic_vae_dim, device=dev, dtype=torch.bfloat16).cpu()
    rec = {}
    oloop.generate(m15.sd, m15.cfg, inp["input_ids"], inp["attention_mask"], IDS, ddpm_steps=STEPS, forced=[[X], [X]],
                   voice_noise=(draw, eps), record=rec, speech_tensors=inp["speech_tensors"],
                   speech_masks=inp["speech_masks"], speech_input_mask=inp["speech_input_mask"])
    ref = rec["prompt_embeds"].float()
    sim = inp["speech_input_mask"][inp["attention_mask"].bool()]
    assert emb.shape == ref.shape
    assert torch.equal(emb[~sim], ref[~sim])                      # text rows: plain embedding gathers
    e = rel_err(emb[sim], ref[sim])
    print(f"voice rows ({int(sim.sum())}): rel {e:.3e} cos {cos(emb[sim], ref[sim]):.6f}")
    assert e < 2e-2


def test_teacher_forced_1p5b_b1(m15):
    """configs[1]: B = 1, 3 s voice, S = 10, 6 diffusion steps then eos."""
    inp = synthetic_inputs(batch=1, speakers=1, voice_seconds=3.0, text_tokens=64, seed=100)
    sched = [[D] * 6 + [X]]
    vn = _voice_noise(inp, m15.cfg.acoustic_vae_dim)
    rec16, seqs, _, _ = _oracle(m15, inp, sched, vn)
    rec32, _, _, _ = _oracle(m15, inp, sched, vn, dtype=torch.float32, teacher=rec16)
    got, sess = _teacher_forced(m15.model, inp, sched, rec16)
    assert len(got["latents"]) == len(rec16["latents"]) == 6
    assert torch.equal(sess.result().sequences, seqs)
    _per_step_check(got, rec16, rec32, "1.5B B=1")


def test_teacher_forced_1p5b_b8_two_speakers(m15):
    """configs[2]: B = 8 two-speaker dialogues (16 ragged voice clips, ragged
    left-padded scripts), schedules with speech_end / speech_start / skip /
    early eos between diffusion steps."""
    inp = synthetic_inputs(batch=8, speakers=2, voice_seconds=[3.0, 2.2, 1.3, 2.7], text_tokens=64, seed=101,
                           text_jitter=12)
    sched = [
        [D] * 6 + [X],
        [D, D, E, S, D, D, X],
        [D, D, D, X],
        [S, D, D, D, D, D, X],
        [D, E, D, D, S, D, X],
        [D, D, D, D, E, S, D, X],
        [E, S, D, D, D, X],
        [D, D, S, D, D, D, X],
    ]
    vn = _voice_noise(inp, m15.cfg.acoustic_vae_dim)
    rec16, seqs, _, reach = _oracle(m15, inp, sched, vn)
    rec32, _, _, _ = _oracle(m15, inp, sched, vn, dtype=torch.float32, teacher=rec16)
    got, sess = _teacher_forced(m15.model, inp, sched, rec16)
    out = sess.result()
    assert torch.equal(out.sequences, seqs) and torch.equal(out.reach_max_step_sample.cpu(), reach)
    _per_step_check(got, rec16, rec32, "1.5B B=8 two-speaker")


def test_free_running_1p5b(m15):
    """No teacher forcing.  (1) Greedy, unforced, 8 steps from a 3 s voice
    prompt: the token sequence equals the oracle's.  (2) A forced 8-step
    diffusion run: audio within max(5e-2, 2 x the bf16 reference's own
    free-running deviation from fp32) — bf16 noise compounds through the
    autoregressive feedback."""
    model = m15.model
    inp = synthetic_inputs(batch=1, speakers=1, voice_seconds=3.0, text_tokens=64, seed=102)
    nv, fr = inp["speech_masks"].shape
    # (1) greedy token choice: the device's prefill draws replayed into the oracle
    torch.manual_seed(SEED)
    out = model.generate(**inp, tokenizer=TK, cfg_scale=1.3, max_new_tokens=8, show_progress_bar=False)
    torch.cuda.manual_seed(SEED)
    vn = (torch.randn(nv, device=dev, dtype=torch.bfloat16).cpu(),
          torch.randn(nv, fr, m15.cfg.acoustic_vae_dim, device=dev, dtype=torch.bfloat16).cpu())
    rec, seqs, _, _ = _oracle(m15, inp, None, vn, max_new=8)
    print("greedy tokens", (out.sequences[0, inp["input_ids"].shape[1]:] - 151640).tolist(),
          "oracle logit margins", [round(float(l.sort().values[0, -1] - l.sort().values[0, -2]), 2)
                                   for l in rec["logits"]])
    assert torch.equal(out.sequences, seqs)
    # (2) forced diffusion, free-running audio
    sched = [[D] * 8 + [X]]
    torch.manual_seed(SEED)
    out = model.generate(**inp, tokenizer=TK, cfg_scale=1.3, forced_tokens=sched, show_progress_bar=False)
    _, seqs16, a16, _ = _oracle(m15, inp, sched, vn)
    _, _, a32, _ = _oracle(m15, inp, sched, vn, dtype=torch.float32)
    assert torch.equal(out.sequences, seqs16)
    got, ref = out.speech_outputs[0], a16[0]
    assert got.shape == ref.shape == (1, 8 * 3200)
    e, c, noise = rel_err(got, ref), cos(got, ref), rel_err(ref, a32[0])
    print(f"1.5B free-running audio rel {e:.3e} cos {c:.6f} (bf16 reference vs fp32: {noise:.3e})")
    assert e < max(5e-2, 2 * noise)
