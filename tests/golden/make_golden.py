"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE.

Run in the build container only (needs /root/reference):
    python tests/golden/make_golden.py
Each fixture holds inputs, the reference's outputs and (tiny) weights, so the
oracle and the HIP path can be checked against the reference without the
reference being present (the GPU box has no /root/reference).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_harness  # noqa: E402

R = ref_harness.load()


def f32(t):
    return t.detach().to(torch.float32).cpu().numpy()


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print("wrote", path, sum(a.nbytes for a in arrays.values()) // 1024, "KiB raw")


def sd_arrays(module, prefix="w:"):
    """Weights are bf16-representable (randomize rounds them), stored as raw bf16 bits."""
    out = {}
    for k, v in module.state_dict().items():
        b = v.detach().to(torch.bfloat16)
        assert torch.equal(b.float(), v.detach().float()), k
        out[prefix + k] = b.view(torch.int16).numpy()
    return out


def randomize(module, seed, std=0.05):
    """Random weights everywhere (the reference zero-inits adaLN / final layers)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in module.named_parameters():
            if name.endswith("norm.weight") or name.endswith("gamma"):
                p.copy_(1.0 + 0.1 * torch.randn(p.shape, generator=g))
            else:
                p.copy_(std * torch.randn(p.shape, generator=g))
            p.copy_(p.to(torch.bfloat16).float())


# ---------------------------------------------------------------- G1-SDE scheduler
def g1_sde_scheduler():
    """sde-dpmsolver++ as gradio_demo.py:114-118 configures it (from_config with
    algorithm_type="sde-dpmsolver++", beta_schedule="squaredcos_cap_v2"); the
    per-step noise is passed as variance_noise so the trace is deterministic."""
    Sch = R["dpm"].DPMSolverMultistepScheduler
    out = {}
    for S in (1, 2, 5, 10, 20):
        # from_config(base.config, **overrides) == the constructor with the base
        # arguments plus the overrides (ConfigMixin; stubbed in the harness)
        s = Sch(num_train_timesteps=1000, beta_schedule="squaredcos_cap_v2", prediction_type="v_prediction",
                algorithm_type="sde-dpmsolver++")
        s.set_timesteps(S)
        out[f"sigmas_{S}"] = s.sigmas.numpy()
        for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            g = torch.Generator().manual_seed(200 + S)
            x = torch.randn(3, 64, generator=g).to(dt)
            vs = torch.randn(S, 3, 64, generator=g).to(dt)
            zs = torch.randn(S, 3, 64, generator=g)                     # fp32 (step() draws fp32 noise)
            s.set_timesteps(S)
            xs = []
            cur = x
            for i, t in enumerate(s.timesteps):
                cur = s.step(vs[i], t, cur, variance_noise=zs[i]).prev_sample
                xs.append(cur)
            out[f"x_{tag}_{S}"] = f32(x)
            out[f"v_{tag}_{S}"] = f32(vs)
            out[f"z_{tag}_{S}"] = f32(zs)
            out[f"trace_{tag}_{S}"] = f32(torch.stack(xs))
    save("g1_sde_scheduler.npz", **out)


# ---------------------------------------------------------------- G1 scheduler
def g1_scheduler():
    Sch = R["dpm"].DPMSolverMultistepScheduler
    out = {}
    for S in (1, 2, 5, 10, 20):
        s = Sch(num_train_timesteps=1000, beta_schedule="cosine", prediction_type="v_prediction")
        s.set_timesteps(S)
        out[f"timesteps_{S}"] = s.timesteps.numpy()
        out[f"sigmas_{S}"] = s.sigmas.numpy()
        out[f"t_bf16_{S}"] = f32(s.timesteps.to(torch.bfloat16))
        # a stepping trace on random model outputs, in fp32 and bf16
        for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            g = torch.Generator().manual_seed(100 + S)
            x = torch.randn(3, 64, generator=g).to(dt)
            vs = torch.randn(S, 3, 64, generator=g).to(dt)
            s.set_timesteps(S)
            xs = []
            cur = x
            for i, t in enumerate(s.timesteps):
                cur = s.step(vs[i], t, cur).prev_sample
                xs.append(cur)
            out[f"x_{tag}_{S}"] = f32(x)
            out[f"v_{tag}_{S}"] = f32(vs)
            out[f"trace_{tag}_{S}"] = f32(torch.stack(xs))
    save("g1_scheduler.npz", **out)


# ------------------------------------------------------------ G2/G3 diffusion head
def head_module(H):
    cfg = R["cfg"].VibeVoiceDiffusionHeadConfig(hidden_size=H, head_layers=4, head_ffn_ratio=3.0,
                                                rms_norm_eps=1e-5, latent_size=64)
    m = R["head"].VibeVoiceDiffusionHead(cfg)
    randomize(m, seed=H)
    return m.eval()


class _FakeInf:
    """Just enough of VibeVoiceForConditionalGenerationInference for the
    reference's own sample_speech_tokens (modeling_vibevoice_inference.py:712-725)."""

    def __init__(self, head, steps):
        self.model = type("M", (), {})()
        self.model.prediction_head = head
        self.model.noise_scheduler = R["dpm"].DPMSolverMultistepScheduler(
            num_train_timesteps=1000, beta_schedule="cosine", prediction_type="v_prediction")
        self.ddpm_inference_steps = steps
        self.config = type("C", (), {"acoustic_vae_dim": 64})()


def g2_g3_head():
    out = {}
    H = 128
    head = head_module(H)
    out.update(sd_arrays(head))
    g = torch.Generator().manual_seed(7)
    for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        m = head.to(dt)
        noisy = torch.randn(4, 64, generator=g).to(dt)
        t = torch.tensor([999., 999., 500., 500.]).to(dt)
        cond = torch.randn(4, H, generator=g).to(dt)
        with torch.no_grad():
            y = m(noisy, t, condition=cond)
        out[f"fwd_noisy_{tag}"], out[f"fwd_t_{tag}"] = f32(noisy), f32(t)
        out[f"fwd_cond_{tag}"], out[f"fwd_out_{tag}"] = f32(cond), f32(y)
        for S in (5, 10):
            n = 2
            pos = torch.randn(n, H, generator=g).to(dt)
            neg = torch.randn(n, H, generator=g).to(dt)
            fake = _FakeInf(m, S)
            torch.manual_seed(1234 + S)
            with torch.no_grad():
                lat = R["mvi"].VibeVoiceForConditionalGenerationInference.sample_speech_tokens(
                    fake, pos, neg, cfg_scale=1.3)
            torch.manual_seed(1234 + S)
            noise = torch.randn(2 * n, 64)        # the draw made inside (:716)
            out[f"sst_pos_{tag}_{S}"], out[f"sst_neg_{tag}_{S}"] = f32(pos), f32(neg)
            out[f"sst_noise_{S}_{tag}"] = noise.numpy()
            out[f"sst_out_{tag}_{S}"] = f32(lat)
    save("g2_head.npz", **out)


# ------------------------------------------------------------------ G4/G5 codec
def codec_cfgs():
    return {
        "small": dict(encoder_n_filters=8, decoder_n_filters=8, encoder_ratios=[2, 2],
                      encoder_depths="1-1-2", vae_dim=16),
        "hop3200": dict(encoder_n_filters=2, decoder_n_filters=2, encoder_ratios=[8, 5, 5, 4, 2, 2],
                        encoder_depths="1-1-1-1-1-1-1", vae_dim=16),
    }


def g4_g5_codec():
    out = {}
    C = R["cfg"]
    for name, kw in codec_cfgs().items():
        acfg = C.VibeVoiceAcousticTokenizerConfig(**kw)
        m = R["tok"].VibeVoiceAcousticTokenizerModel(acfg).eval()
        randomize(m, seed=len(name), std=0.2)
        out.update({f"{name}/{k}": v for k, v in sd_arrays(m).items()})
        hop = int(np.prod(kw["encoder_ratios"]))
        g = torch.Generator().manual_seed(11)
        for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            mm = m.to(dt)
            # streaming decode: 2 samples, 5 steps, sample 1 skips step 2, set_to_zero(0) after step 3
            B, steps = 2, 5
            z = torch.randn(steps, B, kw["vae_dim"], 1, generator=g).to(dt)
            cache = R["tok"].VibeVoiceTokenizerStreamingCache()
            outs = []
            sched = [[0, 1], [0, 1], [0], [0, 1], [0, 1]]
            for s in range(steps):
                idx = torch.tensor(sched[s])
                with torch.no_grad():
                    a = mm.decode(z[s, idx], cache=cache, sample_indices=idx, use_cache=True)
                full = torch.zeros(B, 1, hop, dtype=dt)
                full[idx] = a
                outs.append(full)
                if s == 2:
                    cache.set_to_zero(torch.tensor([0]))
            out[f"{name}/dec_z_{tag}"] = f32(z)
            out[f"{name}/dec_audio_{tag}"] = f32(torch.stack(outs))
            # non-streaming decode of 4 frames == streaming (KAT-3)
            zz = torch.randn(1, kw["vae_dim"], 4, generator=g).to(dt)
            with torch.no_grad():
                out[f"{name}/dec_ns_audio_{tag}"] = f32(mm.decode(zz))
            out[f"{name}/dec_ns_z_{tag}"] = f32(zz)
            # streaming encode of 3 frames of audio, 2 samples
            aud = (0.3 * torch.randn(3, B, 1, hop, generator=g)).to(dt)
            cache = R["tok"].VibeVoiceTokenizerStreamingCache()
            lats = []
            for s in range(3):
                idx = torch.arange(B)
                with torch.no_grad():
                    lats.append(mm.encode(aud[s], cache=cache, sample_indices=idx, use_cache=True).mean)
            out[f"{name}/enc_audio_{tag}"] = f32(aud)
            out[f"{name}/enc_mean_{tag}"] = f32(torch.stack(lats))
            # non-streaming encode of a length that is NOT a multiple of hop (voice prompt path)
            L = 2 * hop + hop // 2 + 3
            a2 = (0.3 * torch.randn(2, 1, L, generator=g)).to(dt)
            with torch.no_grad():
                out[f"{name}/enc_ns_mean_{tag}"] = f32(mm.encode(a2).mean)
            out[f"{name}/enc_ns_audio_{tag}"] = f32(a2)
    save("g4_codec.npz", **out)


# ------------------------------------------------- G5 semantic encoder (partial frames)
def g5_semantic():
    """The semantic tokenizer's own model (VibeVoiceSemanticTokenizerModel,
    modular_vibevoice_tokenizer.py:1118-1186): non-streaming encode of clips
    whose length is NOT a multiple of the hop, so every strided conv gets the
    reference's per-layer extra right padding (:127-133, :393-408); plus a
    whole-frame clip streamed frame by frame vs its non-streaming encode."""
    out = {}
    C = R["cfg"]
    kw = dict(encoder_n_filters=2, encoder_ratios=[8, 5, 5, 4, 2, 2], encoder_depths="1-1-1-1-1-1-1", vae_dim=16)
    scfg = C.VibeVoiceSemanticTokenizerConfig(**kw)
    m = R["tok"].VibeVoiceSemanticTokenizerModel(scfg).eval()
    randomize(m, seed=5, std=0.2)
    out.update(sd_arrays(m))
    hop = int(np.prod(kw["encoder_ratios"]))
    g = torch.Generator().manual_seed(12)
    for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        mm = m.to(dt)
        for L in (hop // 3, 2 * hop + hop // 2 + 3, 3 * hop - 1):   # < 1 frame, 2.5 frames, just short of 3
            a = (0.3 * torch.randn(2, 1, L, generator=g)).to(dt)
            with torch.no_grad():
                out[f"ns_mean_{L}_{tag}"] = f32(mm.encode(a).mean)
            out[f"ns_audio_{L}_{tag}"] = f32(a)
    save("g5_semantic.npz", **out)


# -------------------------------------------------------------- G6 connectors
def g6_connector():
    out = {}
    SC = R["mv"].SpeechConnector
    for din in (64, 128):
        m = SC(din, 256).eval()
        randomize(m, seed=din)
        out.update({f"{din}/{k}": v for k, v in sd_arrays(m).items()})
        g = torch.Generator().manual_seed(din)
        for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
            x = torch.randn(3, 1, din, generator=g).to(dt)
            with torch.no_grad():
                y = m.to(dt)(x)
            out[f"{din}/x_{tag}"], out[f"{din}/y_{tag}"] = f32(x), f32(y)
    save("g6_connector.npz", **out)


# ------------------------------------------------------------------ G7 Qwen2
def lm_cfg():
    from transformers import Qwen2Config
    return Qwen2Config(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=2,
                       num_key_value_heads=1, head_dim=128, rms_norm_eps=1e-6, rope_theta=1e6,
                       vocab_size=64, max_position_embeddings=4096, tie_word_embeddings=False,
                       attn_implementation="eager")


def g7_qwen2():
    from transformers import AutoModel
    from transformers.cache_utils import DynamicCache
    cfg = lm_cfg()
    out = {}
    torch.manual_seed(3)
    m = AutoModel.from_config(cfg).eval()
    randomize(m, seed=3, std=0.05)
    out.update(sd_arrays(m))
    g = torch.Generator().manual_seed(5)
    for dt, tag in ((torch.float32, "f32"), (torch.bfloat16, "bf16")):
        mm = m.to(dt)
        B, L = 2, 7
        pad = [0, 3]                      # sample 1 is left-padded by 3 (vibevoice_processor.py:351-353)
        mask = torch.ones(B, L, dtype=torch.long)
        mask[1, :pad[1]] = 0
        emb = torch.randn(B, L, 256, generator=g).to(dt)
        cache = DynamicCache()
        pos = (mask.cumsum(-1) - 1).masked_fill(mask == 0, 1)   # HF 4.51.3 prepare_inputs_for_generation
        with torch.no_grad():
            o = mm(inputs_embeds=emb, attention_mask=mask, position_ids=pos, past_key_values=cache,
                   use_cache=True)
        hs = [o.last_hidden_state[:, -1]]
        steps = torch.randn(3, B, 1, 256, generator=g).to(dt)
        for s in range(3):
            mask = torch.cat([mask, torch.ones(B, 1, dtype=torch.long)], dim=1)
            p = (mask.cumsum(-1) - 1)[:, -1:]
            with torch.no_grad():
                o = mm(inputs_embeds=steps[s], attention_mask=mask, position_ids=p, past_key_values=cache,
                       use_cache=True)
            hs.append(o.last_hidden_state[:, -1])
        out[f"emb_{tag}"], out[f"steps_{tag}"] = f32(emb), f32(steps)
        out[f"mask0"] = mask[:, :L].numpy()
        out[f"hidden_{tag}"] = f32(torch.stack(hs))
    save("g7_qwen2.npz", **out)


# ------------------------------------------------------- G8 generate() loop trace
G8_IDS = dict(eos=151643, start=151652, end=151653, diffusion=151654, pad=151655)
G8_SCHEDULES = [
    [151654, 151654, 151654, 151654, 151654, 151653, 151652, 151654, 151643],
    [151654, 151653, 151654, 151654, 151652, 151654, 151654, 151643],   # step 1: skip at the KV-shift boundary
]


def g8_loop():
    """The reference's own generate() (modeling_vibevoice_inference.py:327-710)
    run end to end on CPU in fp32 with the tiny config of tests/tiny.py and the
    seeded synthetic weights (vibevoice_amd.weights.synthetic_state_dict, seed
    21, mode "test"; the test regenerates them), B = 2 left-padded text prompts,
    forced token schedules (diffusion x k, speech_end, speech_start while the
    other sample diffuses, the skip correction incl. its KV-shift boundary case,
    eos), both refresh_negative modes, S = 5, cfg 1.3, torch.manual_seed(1234).
    HF-4.51.3 plumbing shims: ref_harness.install_generate_shims.  The prompt
    has no voice: the prefill's voice-encoder call (which generate() always
    makes, :470-476) gets a dummy one-frame clip (hop 4) masked out of every position, and
    the global RNG is restored around it so the diffusion noise stream is the
    one a voice-free prompt would draw.  A third run (refresh_negative) adds
    voice prompts: two clips scattered at speech_input_mask, encoder + gaussian
    sample on the global RNG + connector, all the reference's code."""
    import types
    sys.path.insert(0, os.path.dirname(HERE))
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from tiny import tiny_config, tiny_dict
    from vibevoice_amd.weights import synthetic_state_dict
    forced = []
    ref_harness.install_generate_shims(R["mvi"], forced)
    d = tiny_dict(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    d["torch_dtype"] = "float32"
    d["decoder_config"]["attn_implementation"] = "eager"
    rcfg = R["cfg"].VibeVoiceConfig(**d)
    cls = R["mvi"].VibeVoiceForConditionalGenerationInference
    torch.manual_seed(0)
    model = cls(rcfg).float().eval()
    sd = synthetic_state_dict(tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512), seed=21,
                              device="cpu", dtype=torch.float32, mode="test")
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    missing = [k for k in missing if not k.startswith("model.acoustic_tokenizer.encoder.") and k != "lm_head.weight"]
    assert not missing, missing
    assert torch.equal(model.lm_head.weight, sd["model.language_model.embed_tokens.weight"])
    model.set_ddpm_inference_steps(5)
    orig = cls._process_speech_inputs

    def voice_free(self, *a, **k):
        st = torch.get_rng_state()
        try:
            return orig(self, *a, **k)
        finally:
            torch.set_rng_state(st)
    cls._process_speech_inputs = voice_free
    tok = types.SimpleNamespace(speech_start_id=G8_IDS["start"], speech_end_id=G8_IDS["end"],
                                speech_diffusion_id=G8_IDS["diffusion"], eos_token_id=G8_IDS["eos"],
                                bos_token_id=None, pad_token_id=G8_IDS["pad"])
    g = torch.Generator().manual_seed(2)
    P = 10
    ids = torch.randint(0, 151000, (2, P), generator=g)
    mask = torch.ones(2, P, dtype=torch.long)
    mask[1, :3] = 0
    ids[1, :3] = G8_IDS["pad"]
    forced[:] = G8_SCHEDULES
    out = {"input_ids": ids.numpy(), "attention_mask": mask.numpy(),
           "schedules": np.array([s + [G8_IDS["eos"]] * (9 - len(s)) for s in G8_SCHEDULES]),
           "schedule_lens": np.array([len(s) for s in G8_SCHEDULES]),
           "sd_checksum": np.array([float(v.double().sum()) for v in sd.values()])}
    for refresh in (True, False):
        torch.manual_seed(1234)
        with torch.no_grad():
            o = model.generate(input_ids=ids, attention_mask=mask, tokenizer=tok, cfg_scale=1.3,
                               speech_tensors=torch.zeros(1, 4), speech_masks=torch.zeros(1, 1, dtype=torch.bool),
                               speech_input_mask=torch.zeros(2, P, dtype=torch.bool), refresh_negative=refresh,
                               show_progress_bar=False)
        tag = "refresh" if refresh else "norefresh"
        out[f"{tag}/sequences"] = o.sequences.numpy()
        out[f"{tag}/reach"] = o.reach_max_step_sample.numpy()
        for b, a in enumerate(o.speech_outputs):
            out[f"{tag}/audio{b}"] = f32(a)
    # per-sample length cap (:421-422, 543-553): max_length_times = 0.5 gives
    # max_steps 5 and caps of 5 / 3 steps (the left-padded sample has 7 tokens),
    # so sample 1 finishes with reach_max_step_sample while sample 0 diffuses on
    forced[:] = [[G8_IDS["diffusion"]] * 9, [G8_IDS["diffusion"]] * 9]
    torch.manual_seed(1234)
    with torch.no_grad():
        o = model.generate(input_ids=ids, attention_mask=mask, tokenizer=tok, cfg_scale=1.3,
                           speech_tensors=torch.zeros(1, 4), speech_masks=torch.zeros(1, 1, dtype=torch.bool),
                           speech_input_mask=torch.zeros(2, P, dtype=torch.bool), max_length_times=0.5,
                           show_progress_bar=False)
    out["cap/sequences"] = o.sequences.numpy()
    out["cap/reach"] = o.reach_max_step_sample.numpy()
    for b, a in enumerate(o.speech_outputs):
        out[f"cap/audio{b}"] = f32(a)
    forced[:] = G8_SCHEDULES
    cls._process_speech_inputs = orig
    # voice-prompt prefill (_process_speech_inputs, :150-163, gaussian sample on the
    # global RNG): clip 0 (5 frames) in sample 0, clip 1 (13 samples -> 4 frames,
    # zero-padded to 20) in sample 1 after its 3 pad positions
    vt = torch.zeros(2, 20)
    vt[0] = 0.3 * torch.randn(20, generator=g)
    vt[1, :13] = 0.3 * torch.randn(13, generator=g)
    vm = torch.zeros(2, 5, dtype=torch.bool)
    vm[0, :5] = True
    vm[1, :4] = True
    sim = torch.zeros(2, P, dtype=torch.bool)
    sim[0, 1:6] = True
    sim[1, 4:8] = True
    out.update({"voice/speech_tensors": f32(vt), "voice/speech_masks": vm.numpy(),
                "voice/speech_input_mask": sim.numpy()})
    torch.manual_seed(1234)
    with torch.no_grad():
        o = model.generate(input_ids=ids, attention_mask=mask, tokenizer=tok, cfg_scale=1.3, speech_tensors=vt,
                           speech_masks=vm, speech_input_mask=sim, refresh_negative=True, show_progress_bar=False)
    out["voice/sequences"] = o.sequences.numpy()
    out["voice/reach"] = o.reach_max_step_sample.numpy()
    for b, a in enumerate(o.speech_outputs):
        out[f"voice/audio{b}"] = f32(a)
    # do_sample=True (:502-505): no forced schedule; the reference draws
    # torch.multinomial over the constrained full-vocabulary probabilities and the
    # diffusion noise from the same global CPU generator, interleaved
    cls._process_speech_inputs = voice_free
    forced[:] = []
    # the tied embedding rows of the 4 control ids are scaled down so their logits
    # are O(1) and the draw is not a foregone conclusion (test weights give logits ~16)
    emb = model.model.language_model.embed_tokens.weight
    rows = [G8_IDS[k] for k in ("eos", "start", "end", "diffusion")]
    mats = [emb] if model.lm_head.weight is emb else [emb, model.lm_head.weight]   # tied: one tensor
    saved = [w.data[rows].clone() for w in mats]
    for w in mats:
        w.data[rows] *= SAMPLE_ROW_SCALE
    for seed in SAMPLE_SEEDS:
        torch.manual_seed(seed)
        with torch.no_grad():
            o = model.generate(input_ids=ids, attention_mask=mask, tokenizer=tok, cfg_scale=1.3,
                               speech_tensors=torch.zeros(1, 4), speech_masks=torch.zeros(1, 1, dtype=torch.bool),
                               speech_input_mask=torch.zeros(2, P, dtype=torch.bool), refresh_negative=True,
                               generation_config={"do_sample": True}, show_progress_bar=False)
        out[f"sample{seed}/sequences"] = o.sequences.numpy()
        out[f"sample{seed}/reach"] = o.reach_max_step_sample.numpy()
        for b, a in enumerate(o.speech_outputs):
            out[f"sample{seed}/audio{b}"] = f32(a) if a is not None else np.zeros(0, np.float32)
    for w, v in zip(mats, saved):
        w.data[rows] = v
    forced[:] = G8_SCHEDULES
    cls._process_speech_inputs = orig
    save("g8_loop.npz", **out)


SAMPLE_SEEDS = (1234, 77)
SAMPLE_ROW_SCALE = 0.05


# ---------------------------------------------------------------- G9 processor
PROC_SCRIPTS = [
    "Speaker 1: Hello there, welcome to the show.\nSpeaker 2: It's great to be here!\n\nSpeaker 1:   Fine, thanks.",
    "Speaker 0: Today we talk about podcasts.\nnot a speaker line\nSpeaker 0: How are you doing?",
]
PROC_JSON = '[{"speaker": "1", "text": " Hello there. "}, {"speaker": "x", "text": "skip"}, {"speaker": 2, "text": "Hi"}]'
PROC_TXT = "Speaker 2: first\nplain line here\n\nspeaker 3 :  third  \nSpeaker 4:\n"


def g9_processor():
    """VibeVoiceProcessor (vibevoice/processor/vibevoice_processor.py) with the
    reference's own VibeVoiceTextTokenizerFast over the tiny Qwen2-style
    vocabulary (tiny_tokenizer.py; the real Qwen2.5 files are not available
    offline): batches with ragged voice prompts (dBFS normalisation, frame
    counts, left padding), a single script, no voices, no padding, and the
    .json / .txt script converters."""
    import json
    import tempfile
    import tiny_tokenizer
    from vibevoice.processor.vibevoice_processor import VibeVoiceProcessor
    from vibevoice.processor.vibevoice_tokenizer_processor import VibeVoiceTokenizerProcessor
    from vibevoice.modular.modular_vibevoice_text_tokenizer import VibeVoiceTextTokenizerFast
    tok = VibeVoiceTextTokenizerFast.from_pretrained(tiny_tokenizer.DIR)
    proc = VibeVoiceProcessor(tokenizer=tok, audio_processor=VibeVoiceTokenizerProcessor())
    rng = np.random.default_rng(9)
    voices = [(0.3 * rng.standard_normal(n)).astype(np.float32) for n in (7000, 12345, 3200, 640)]
    voices[2][:10] = 4.0                                   # clips after normalisation: avoid_clipping path
    out = {f"voice{i}": v for i, v in enumerate(voices)}
    out["scripts"] = np.array(PROC_SCRIPTS)
    out["ids"] = np.array([tok.speech_start_id, tok.speech_end_id, tok.speech_diffusion_id, tok.eos_token_id,
                           tok.pad_id])
    cases = {
        "a": dict(text=PROC_SCRIPTS, voice_samples=[[voices[0], voices[1]], [voices[2]]], padding=True,
                  return_tensors="pt"),
        "b": dict(text=PROC_SCRIPTS[0], voice_samples=[voices[3], voices[1], voices[0]], return_tensors="pt"),
        "c": dict(text=PROC_SCRIPTS, padding=True, return_tensors="pt"),
    }
    for tag, kw in cases.items():
        be = proc(**kw)
        for k in ("input_ids", "attention_mask", "speech_input_mask", "speech_tensors", "speech_masks"):
            v = be.get(k)
            if v is not None:
                out[f"{tag}_{k}"] = v.numpy()
        out[f"{tag}_parsed"] = np.array(json.dumps(be["parsed_scripts"]))
        out[f"{tag}_speakers"] = np.array(json.dumps(be["all_speakers_list"]))
    be = proc(text=PROC_SCRIPTS, padding=False, return_tensors=None)            # ragged python lists
    out["d_lengths"] = np.array([len(x) for x in be["input_ids"]])
    out["d_input_ids"] = np.concatenate([np.array(x) for x in be["input_ids"]])
    out["d_attention_mask"] = np.concatenate([np.array(x) for x in be["attention_mask"]])
    with tempfile.TemporaryDirectory() as d:
        pj, pt = os.path.join(d, "s.json"), os.path.join(d, "s.txt")
        with open(pj, "w") as f:
            f.write(PROC_JSON)
        with open(pt, "w") as f:
            f.write(PROC_TXT)
        out["json_src"], out["txt_src"] = np.array(PROC_JSON), np.array(PROC_TXT)
        out["json_script"] = np.array(proc._convert_json_to_script(pj))
        out["txt_script"] = np.array(proc._convert_text_to_script(pt))
        be = proc(text=[pj, pt], padding=True, return_tensors="pt")
        out["e_input_ids"] = be["input_ids"].numpy()
    save("g9_processor.npz", **out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    if len(sys.argv) > 1:                        # regenerate selected fixtures: make_golden.py g1_sde_scheduler
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    g1_scheduler()
    g1_sde_scheduler()
    g2_g3_head()
    g4_g5_codec()
    g5_semantic()
    g6_connector()
    g7_qwen2()
    g8_loop()
