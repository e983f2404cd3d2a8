"""The CPU oracle (oracle/) against the reference's golden vectors.

Fixtures come from tests/golden/make_golden.py, which runs the reference's
own modules.  fp32 comparisons are tight; bf16 ones allow for the oracle's
different (but same-rounding-point) op grouping.
"""
import pytest
import torch

from golden_io import DT, load, t, weights
from oracle import codec, head, lm, scheduler


def close(a, b, rtol, atol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = max(1.0, b.abs().max().item())
    assert torch.allclose(a, b, rtol=rtol, atol=atol * scale), f"max abs err {err} (scale {scale})"


TOL = {"f32": (1e-5, 1e-5), "bf16": (2e-2, 2e-2)}


@pytest.mark.parametrize("S", [1, 2, 5, 10, 20])
def test_scheduler_tables(S):
    z = load("g1_scheduler.npz")
    s = scheduler.DPMSolverPP()
    s.set_timesteps(S)
    assert (s.timesteps.numpy() == z[f"timesteps_{S}"]).all()
    assert (s.sigmas.numpy() == z[f"sigmas_{S}"]).all()
    assert (s.timesteps.to(torch.bfloat16).float().numpy() == z[f"t_bf16_{S}"]).all()


@pytest.mark.parametrize("S", [1, 2, 5, 10, 20])
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_scheduler_step_trace_bitexact(S, tag):
    """x0 in the sample dtype, fp32 update, cast back: bit-exact vs the reference."""
    z = load("g1_scheduler.npz")
    s = scheduler.DPMSolverPP()
    s.set_timesteps(S)
    x = t(z, f"x_{tag}_{S}", DT[tag])
    vs = t(z, f"v_{tag}_{S}", DT[tag])
    ref = t(z, f"trace_{tag}_{S}")
    for i in range(S):
        x = s.step(vs[i], x)
        assert torch.equal(x.float(), ref[i]), f"step {i}"


@pytest.mark.parametrize("S", [1, 2, 5, 10, 20])
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_sde_scheduler_step_trace_bitexact(S, tag):
    """sde-dpmsolver++ (gradio_demo.py:114-118) with the reference's own per-step
    fp32 noise (variance_noise): bit-exact vs the reference."""
    z = load("g1_sde_scheduler.npz")
    s = scheduler.DPMSolverPP(algorithm_type="sde-dpmsolver++")
    s.set_timesteps(S)
    assert (s.sigmas.numpy() == z[f"sigmas_{S}"]).all()
    x = t(z, f"x_{tag}_{S}", DT[tag])
    vs = t(z, f"v_{tag}_{S}", DT[tag])
    zs = t(z, f"z_{tag}_{S}")
    ref = t(z, f"trace_{tag}_{S}")
    for i in range(S):
        x = s.step(vs[i], x, zs[i])
        assert torch.equal(x.float(), ref[i]), f"step {i}"


@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_head_forward(tag):
    z = load("g2_head.npz")
    sd = weights(z, dtype=DT[tag])
    y = head.head_forward(sd, t(z, f"fwd_noisy_{tag}", DT[tag]), t(z, f"fwd_t_{tag}", DT[tag]),
                          t(z, f"fwd_cond_{tag}", DT[tag]), n_layers=4)
    close(y, t(z, f"fwd_out_{tag}"), *TOL[tag])


@pytest.mark.parametrize("S", [5, 10])
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_sample_speech_tokens(S, tag):
    z = load("g2_head.npz")
    sd = weights(z, dtype=DT[tag])
    lat = head.sample_speech_tokens(sd, t(z, f"sst_pos_{tag}_{S}", DT[tag]), t(z, f"sst_neg_{tag}_{S}", DT[tag]),
                                    t(z, f"sst_noise_{S}_{tag}").to(DT[tag]), S, 1.3, n_layers=4)
    close(lat, t(z, f"sst_out_{tag}_{S}"), *TOL[tag])


CODEC = {"small": dict(encoder_n_filters=8, decoder_n_filters=8, encoder_ratios=[2, 2],
                       encoder_depths="1-1-2", vae_dim=16),
         "hop3200": dict(encoder_n_filters=2, decoder_n_filters=2, encoder_ratios=[8, 5, 5, 4, 2, 2],
                         encoder_depths="1-1-1-1-1-1-1", vae_dim=16)}


@pytest.mark.parametrize("name", list(CODEC))
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_codec_streaming_decode(name, tag):
    z = load("g4_codec.npz")
    sd = weights(z, prefix=f"{name}/w:", dtype=DT[tag])
    dims = codec.codec_dims(CODEC[name], "decoder")
    zs = t(z, f"{name}/dec_z_{tag}", DT[tag])
    ref = t(z, f"{name}/dec_audio_{tag}")
    st = codec.StreamState(2)
    sched = [[0, 1], [0, 1], [0], [0, 1], [0, 1]]
    for s in range(zs.shape[0]):
        idx = torch.tensor(sched[s])
        a = codec.decode(sd, dims, zs[s, idx], st, idx)
        close(a, ref[s, idx], *TOL[tag])
        if s == 2:
            st.zero(torch.tensor([0]))


@pytest.mark.parametrize("name", list(CODEC))
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_codec_nonstreaming_decode(name, tag):
    z = load("g4_codec.npz")
    sd = weights(z, prefix=f"{name}/w:", dtype=DT[tag])
    dims = codec.codec_dims(CODEC[name], "decoder")
    a = codec.decode(sd, dims, t(z, f"{name}/dec_ns_z_{tag}", DT[tag]), None, None, streaming=False)
    close(a, t(z, f"{name}/dec_ns_audio_{tag}"), *TOL[tag])
    if tag == "f32":   # KAT-3: streaming frame-by-frame == one-shot non-streaming
        st = codec.StreamState(1)
        zz = t(z, f"{name}/dec_ns_z_{tag}")
        parts = [codec.decode(sd, dims, zz[:, :, i:i + 1], st, torch.tensor([0])) for i in range(zz.shape[2])]
        close(torch.cat(parts, dim=-1), a, 1e-5, 1e-5)


@pytest.mark.parametrize("name", list(CODEC))
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_codec_encode(name, tag):
    z = load("g4_codec.npz")
    sd = weights(z, prefix=f"{name}/w:", dtype=DT[tag])
    dims = codec.codec_dims(CODEC[name], "encoder")
    aud = t(z, f"{name}/enc_audio_{tag}", DT[tag])
    ref = t(z, f"{name}/enc_mean_{tag}")
    st = codec.StreamState(2)
    for s in range(aud.shape[0]):
        m = codec.encode(sd, dims, aud[s], st, torch.arange(2))
        close(m, ref[s], *TOL[tag])
    m = codec.encode(sd, dims, t(z, f"{name}/enc_ns_audio_{tag}", DT[tag]), None, None, streaming=False)
    close(m, t(z, f"{name}/enc_ns_mean_{tag}"), *TOL[tag])


G5_CFG = CODEC["hop3200"]   # the same encoder shape, semantic model


@pytest.mark.parametrize("L", [1066, 8003, 9599])
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_semantic_encode_partial_frames(L, tag):
    """G5: the reference's VibeVoiceSemanticTokenizerModel, non-streaming encode
    of clips that end in a partial frame (each strided conv right-pads its input
    to whole strides, modular_vibevoice_tokenizer.py:127-133, 393-408) ->
    ceil(L / hop) frames; the oracle's non-streaming encoder."""
    z = load("g5_semantic.npz")
    sd = weights(z, prefix="w:", dtype=DT[tag])
    dims = codec.codec_dims(G5_CFG, "encoder")
    ref = t(z, f"ns_mean_{L}_{tag}")
    assert ref.shape[1] == -(-L // 3200)
    m = codec.encode(sd, dims, t(z, f"ns_audio_{L}_{tag}", DT[tag]), None, None, streaming=False)
    close(m, ref, *TOL[tag])


@pytest.mark.parametrize("din", [64, 128])
@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_connector(din, tag):
    z = load("g6_connector.npz")
    sd = weights(z, prefix=f"{din}/w:", dtype=DT[tag])
    x = t(z, f"{din}/x_{tag}", DT[tag])
    y = torch.nn.functional.linear(x, sd["fc1.weight"], sd["fc1.bias"])
    y = lm.rms(y, sd["norm.weight"], 1e-6)
    y = torch.nn.functional.linear(y, sd["fc2.weight"], sd["fc2.bias"])
    close(y, t(z, f"{din}/y_{tag}"), *TOL[tag])


LMCFG = dict(hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=2,
             num_key_value_heads=1, head_dim=128, rms_norm_eps=1e-6, rope_theta=1e6)


@pytest.mark.parametrize("tag", ["f32", "bf16"])
def test_qwen2_compacted_kv(tag):
    """Left-padded prefill + 3 decode steps == compacted per-row caches with
    positions = number of cached entries (cumsum(mask)-1)."""
    z = load("g7_qwen2.npz")
    sd = weights(z, dtype=DT[tag])
    emb = t(z, f"emb_{tag}", DT[tag])
    steps = t(z, f"steps_{tag}", DT[tag])
    mask = z["mask0"]
    ref = t(z, f"hidden_{tag}")
    kvs = [lm.RowKV(2) for _ in range(2)]
    last = []
    for r in range(2):
        keep = torch.from_numpy(mask[r]).bool()
        h = lm.forward_rows(sd, LMCFG, emb[r:r + 1, keep], kvs[r:r + 1])
        last.append(h[0, -1])
    close(torch.stack(last), ref[0], *TOL[tag])
    for s in range(steps.shape[0]):
        h = lm.forward_rows(sd, LMCFG, steps[s], kvs)
        close(h[:, -1], ref[s + 1], *TOL[tag])


@pytest.mark.parametrize("refresh,voice,cap", [(True, False, False), (False, False, False), (True, True, False),
                                               (True, False, True)])
def test_loop_trace_g8(refresh, voice, cap):
    """oracle/loop.py (the literal restatement of generate(),
    modeling_vibevoice_inference.py:327-710) vs the reference's own generate()
    run end to end in fp32 (G8, tests/golden/make_golden.py:g8_loop): same
    synthetic weights, B = 2 left-padded prompts, forced schedules through
    diffusion / speech_end / speech_start / the skip correction (incl. the
    KV-shift boundary case) / eos, with and without voice prompts.  Token sequences and reach flags equal; audio
    within fp32 op-order noise (rel L2 < 1e-4)."""
    from oracle import loop
    from tiny import tiny_config
    from vibevoice_amd.weights import synthetic_state_dict
    z = load("g8_loop.npz")
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=21, device="cpu", dtype=torch.float32, mode="test")
    chk = torch.tensor([float(v.double().sum()) for v in sd.values()], dtype=torch.float64)
    assert torch.allclose(chk, torch.from_numpy(z["sd_checksum"]), rtol=1e-12, atol=1e-9), "weights drifted"
    scheds = [list(map(int, s[:n])) for s, n in zip(z["schedules"], z["schedule_lens"])]
    ids = dict(eos=151643, start=151652, end=151653, diffusion=151654)
    kw = {}
    if voice:      # voice-prompt prefill (modeling_vibevoice_inference.py:150-163, 221-225)
        kw = {k: torch.from_numpy(z[f"voice/{k}"]) for k in ("speech_tensors", "speech_masks", "speech_input_mask")}
    if cap:        # per-sample length cap (:421-422, 543-553): all-diffusion, max_length_times 0.5
        scheds, kw = [[ids["diffusion"]] * 9] * 2, dict(max_length_times=0.5)
    torch.manual_seed(1234)
    seqs, audio, reach = loop.generate(sd, cfg, torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"]),
                                       ids, ddpm_steps=5, cfg_scale=1.3, forced=scheds, refresh_negative=refresh,
                                       dtype=torch.float32, **kw)
    tag = "cap" if cap else "voice" if voice else "refresh" if refresh else "norefresh"
    assert torch.equal(seqs, torch.from_numpy(z[f"{tag}/sequences"]))
    assert torch.equal(reach, torch.from_numpy(z[f"{tag}/reach"]))
    for b in range(2):
        ref = torch.from_numpy(z[f"{tag}/audio{b}"])
        assert audio[b].shape == ref.shape, (audio[b].shape, ref.shape)
        err = ((audio[b].float() - ref).norm() / ref.norm()).item()
        assert err < 1e-4, f"sample {b} audio rel L2 {err:.3e}"


G8_SAMPLE_ROWS = [151643, 151652, 151653, 151654]
G8_SAMPLE_ROW_SCALE = 0.05          # make_golden.py SAMPLE_ROW_SCALE


def g8_sample_weights(dtype=torch.float32):
    """G8's weights with the 4 control rows of the tied embedding / lm_head
    scaled as make_golden.py's do_sample runs scale them."""
    from tiny import tiny_config
    from vibevoice_amd.weights import synthetic_state_dict
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=21, device="cpu", dtype=torch.float32, mode="test")
    e = sd["model.language_model.embed_tokens.weight"].clone()
    e[G8_SAMPLE_ROWS] *= G8_SAMPLE_ROW_SCALE
    sd["model.language_model.embed_tokens.weight"] = sd["lm_head.weight"] = e
    return cfg, {k: v.to(dtype) for k, v in sd.items()}


@pytest.mark.parametrize("seed", [1234, 77])
def test_loop_do_sample_g8(seed):
    """do_sample=True (modeling_vibevoice_inference.py:502-505): the oracle's
    literal torch.multinomial over the constrained full-vocabulary
    probabilities on the global CPU generator, interleaved with the diffusion
    noise draws, vs the reference's own generate() (G8 sample runs: sampled
    speech_start / speech_end / diffusion / eos, a diffusion token at step 0).
    Sequences equal, audio within fp32 op-order noise."""
    from oracle import loop
    z = load("g8_loop.npz")
    cfg, sd = g8_sample_weights()
    ids = dict(eos=151643, start=151652, end=151653, diffusion=151654)
    torch.manual_seed(seed)
    seqs, audio, reach = loop.generate(sd, cfg, torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"]),
                                       ids, ddpm_steps=5, cfg_scale=1.3, do_sample=True, dtype=torch.float32)
    tag = f"sample{seed}"
    assert torch.equal(seqs, torch.from_numpy(z[f"{tag}/sequences"]))
    assert torch.equal(reach, torch.from_numpy(z[f"{tag}/reach"]))
    for b in range(2):
        ref = torch.from_numpy(z[f"{tag}/audio{b}"])
        if ref.numel() == 0:
            assert audio[b] is None
            continue
        assert audio[b].shape == ref.shape, (audio[b].shape, ref.shape)
        err = ((audio[b].float() - ref).norm() / ref.norm()).item()
        assert err < 1e-4, f"sample {b} audio rel L2 {err:.3e}"


def test_multinomial_is_argmax_over_exponential_draw():
    """The identity the product's sampling rests on (ATen's one-sample
    multinomial path): torch.multinomial(p, 1) == argmax(p / q) with q ~ Exp(1)
    drawn over the whole row from the same generator state, and only the
    nonzero-probability columns of q matter."""
    V, idx = 151936, [151643, 151652, 151653, 151654]
    for t in range(50):
        s = torch.full((3, V), float("-inf"))
        s[:, idx] = torch.randn(3, 4, generator=torch.Generator().manual_seed(t)) * 2
        p = torch.softmax(s, -1)
        torch.manual_seed(t)
        a = torch.multinomial(p, 1).squeeze(1)
        torch.manual_seed(t)
        q = torch.empty(3, V).exponential_(1)
        c = torch.tensor(idx)[(torch.softmax(s[:, idx], -1) / q[:, idx]).argmax(-1)]
        assert torch.equal(a, c)
