"""End-to-end generate() on the GPU vs the oracle's literal restatement of the
reference loop (oracle/loop.py: negative stream kept as cache + attention mask
with the reference's in-place reset / shift, modeling_vibevoice_inference.py:
563-580, 609-639).

B = 2 left-padded text prompts, forced token schedules that exercise:
diffusion steps for both samples, speech_end (codec reset), speech_start
(negative reset) while the other sample diffuses, the skip correction,
the reference's KV-shift boundary case (a sample with one committed negative
entry skipped at the next pass), and eos.  Both refresh_negative modes.
Tolerance: audio rel L2 < max(5e-2, 2 x the bf16 reference's own deviation from
the fp32 reference loop) and cosine > 0.995 (bf16 model: summation-order noise
compounds through the autoregressive feedback); token sequences equal.
"""
import types

import pytest
import torch

from gpu_util import cos, rel_err
from oracle import loop as oloop
from tiny import tiny_config
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
IDS = dict(eos=151643, start=151652, end=151653, diffusion=151654)
D, E, S, X = IDS["diffusion"], IDS["end"], IDS["start"], IDS["eos"]
TOK = types.SimpleNamespace(speech_start_id=S, speech_end_id=E, speech_diffusion_id=D, eos_token_id=X,
                            bos_token_id=None, pad_token_id=151655)

SCHEDULES = [
    [D, D, D, D, D, E, S, D, X],
    [D, E, D, D, S, D, D, X],   # step 1: skip with one committed entry (KV-shift boundary case)
]


@pytest.mark.parametrize("refresh_negative,prompt", [(True, 10), (False, 10), (True, 300)])
def test_generate_matches_reference_loop(refresh_negative, prompt):
    """prompt = 300: the 597-row prefill takes the prefill attention kernel
    (k_attn_pf, rows of two slots per launch) inside generate()."""
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=21, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=max(128, 3 * prompt + 8))
    model.set_ddpm_inference_steps(5)
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(0, 151000, (2, prompt), generator=g)
    mask = torch.ones(2, prompt, dtype=torch.long)
    mask[1, :3] = 0
    ids[1, :3] = TOK.pad_token_id
    torch.manual_seed(1234)
    out = model.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                         forced_tokens=SCHEDULES, refresh_negative=refresh_negative, show_progress_bar=False)
    torch.cuda.synchronize()
    torch.manual_seed(1234)
    rec = {}
    seqs, audio, reach = oloop.generate(sd, cfg, ids, mask, IDS, ddpm_steps=5, cfg_scale=1.3, forced=SCHEDULES,
                                        refresh_negative=refresh_negative, record=rec)
    # the reference loop in fp32: how far the bf16 reference itself is from exact arithmetic
    torch.manual_seed(1234)
    sd32 = {k: v.float() for k, v in sd.items()}
    _, audio32, _ = oloop.generate(sd32, cfg, ids, mask, IDS, ddpm_steps=5, cfg_scale=1.3, forced=SCHEDULES,
                                   refresh_negative=refresh_negative, dtype=torch.float32)
    assert torch.equal(out.sequences, seqs)
    assert torch.equal(out.reach_max_step_sample.cpu(), reach)
    for b in range(2):
        got, ref = out.speech_outputs[b], audio[b]
        assert got.shape == ref.shape, (got.shape, ref.shape)
        e, c = rel_err(got, ref), cos(got, ref)
        noise = rel_err(ref, audio32[b])
        print(f"sample {b} audio rel_err {e:.3e} cos {c:.6f} (bf16 reference vs fp32: {noise:.3e}) "
              f"samples {ref.shape[-1]}")
        # bf16 summation-order noise compounds through the autoregressive feedback;
        # the HIP path must stay within twice the reference's own bf16 deviation
        assert e < max(5e-2, 2 * noise) and c > 0.995


def test_generate_voice_prompt_matches_reference_loop():
    """Voice-prompt prefill inside generate() (_process_speech_inputs,
    modeling_vibevoice_inference.py:150-163, spliced at speech_input_mask,
    :221-225): the golden G8 inputs (two ragged clips, one per sample) through
    the HIP encoder / gaussian sample / connector / scatter vs oracle/loop.py,
    which G8 pins to the reference's own generate() with voices.  The two
    gaussian-sample draws are made on the device (as the reference does on a
    GPU) and replayed into the oracle; tolerance as above."""
    from golden_io import load
    z = load("g8_loop.npz")
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=21, device="cpu", mode="test", with_acoustic_encoder=True)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=128)
    model.set_ddpm_inference_steps(5)
    ids, mask = torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"])
    voice = {k: torch.from_numpy(z[f"voice/{k}"]) for k in ("speech_tensors", "speech_masks", "speech_input_mask")}
    torch.manual_seed(1234)                       # seeds the CPU and the device generators
    out = model.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3, forced_tokens=SCHEDULES,
                         show_progress_bar=False, **voice)
    torch.cuda.synchronize()
    nv, frames = voice["speech_masks"].shape
    torch.cuda.manual_seed(1234)                  # replay the prefill's two device draws
    draw = torch.randn(nv, device=dev, dtype=torch.bfloat16).cpu()
    eps = torch.randn(nv, frames, cfg.acoustic_vae_dim, device=dev, dtype=torch.bfloat16).cpu()
    res = []
    for s32 in (False, True):
        torch.manual_seed(1234)
        sdx = {k: v.float() for k, v in sd.items()} if s32 else sd
        res.append(oloop.generate(sdx, cfg, ids, mask, IDS, ddpm_steps=5, cfg_scale=1.3, forced=SCHEDULES,
                                  dtype=torch.float32 if s32 else torch.bfloat16, voice_noise=(draw, eps), **voice))
    (seqs, audio, reach), (_, audio32, _) = res
    assert torch.equal(out.sequences, seqs)
    assert torch.equal(out.reach_max_step_sample.cpu(), reach)
    for b in range(2):
        got, ref = out.speech_outputs[b], audio[b]
        assert got.shape == ref.shape, (got.shape, ref.shape)
        e, c, noise = rel_err(got, ref), cos(got, ref), rel_err(ref, audio32[b])
        print(f"voice sample {b} audio rel_err {e:.3e} cos {c:.6f} (bf16 reference vs fp32: {noise:.3e})")
        assert e < max(5e-2, 2 * noise) and c > 0.995


def test_generate_length_cap_matches_reference_loop():
    """Per-sample length caps (modeling_vibevoice_inference.py:421-422, 543-553):
    max_length_times = 0.5 on G8's ragged prompts (10 / 7 tokens) caps the
    loop at 5 steps and the left-padded sample at 3, which then finishes with
    reach_max_step_sample while the other diffuses on.  Sequences and reach
    flags equal the reference's own generate() (golden G8 "cap"); audio vs the
    oracle as above."""
    from golden_io import load
    z = load("g8_loop.npz")
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=21, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=128)
    model.set_ddpm_inference_steps(5)
    ids, mask = torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"])
    sched = [[D] * 9, [D] * 9]
    torch.manual_seed(1234)
    out = model.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3, forced_tokens=sched,
                         max_length_times=0.5, show_progress_bar=False)
    torch.cuda.synchronize()
    assert torch.equal(out.sequences, torch.from_numpy(z["cap/sequences"]))
    assert torch.equal(out.reach_max_step_sample.cpu(), torch.from_numpy(z["cap/reach"]))
    res = []
    for s32 in (False, True):
        torch.manual_seed(1234)
        sdx = {k: v.float() for k, v in sd.items()} if s32 else sd
        res.append(oloop.generate(sdx, cfg, ids, mask, IDS, ddpm_steps=5, cfg_scale=1.3, forced=sched,
                                  max_length_times=0.5, dtype=torch.float32 if s32 else torch.bfloat16))
    (_, audio, _), (_, audio32, _) = res
    for b in range(2):
        got, ref = out.speech_outputs[b], audio[b]
        assert got.shape == ref.shape == z[f"cap/audio{b}"].shape, (got.shape, ref.shape)
        e, c, noise = rel_err(got, ref), cos(got, ref), rel_err(ref, audio32[b])
        print(f"cap sample {b} audio rel_err {e:.3e} cos {c:.6f} (bf16 reference vs fp32: {noise:.3e})")
        assert e < max(5e-2, 2 * noise) and c > 0.995


def test_graph_replay_matches_eager():
    """The hipGraph-captured loop body replays exactly the eager kernel sequence."""
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=5, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=128)
    model.set_ddpm_inference_steps(5)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 151000, (2, 12), generator=g)
    mask = torch.ones(2, 12, dtype=torch.long)
    sched = [[D] * 6 + [E, S] + [D] * 4 + [X], [D] * 3 + [S] + [D] * 8 + [X]]
    outs = []
    for graphs in (False, True, True):
        torch.manual_seed(77)
        outs.append(model.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                                   forced_tokens=sched, use_graphs=graphs, show_progress_bar=False))
    assert len(model._graph_cache) >= 2
    for o in outs[1:]:
        assert torch.equal(o.sequences, outs[0].sequences)
        for b in range(2):
            assert torch.equal(o.speech_outputs[b].cpu(), outs[0].speech_outputs[b].cpu())


@pytest.mark.parametrize("graphs", [False, True])
def test_speculative_diffusion_is_exact(graphs):
    """The diffusion queued before the token readback (GenerateSession._speculate)
    changes nothing: sequences and audio equal the non-speculative loop bit for
    bit, through mispredictions (speech_end / speech_start / eos after a
    diffusion step: the CPU generator is restored and the right rows redone) and
    in an unforced greedy run."""
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=5, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=128)
    model.set_ddpm_inference_steps(5)
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 151000, (2, 12), generator=g)
    mask = torch.ones(2, 12, dtype=torch.long)
    sched = [[D] * 4 + [E, S] + [D] * 3 + [X], [S] + [D] * 2 + [E] + [D] * 5 + [X]]
    for forced in (sched, None):
        outs, misses, rng = [], [], []
        for spec in (False, True):
            torch.manual_seed(77)
            kw = dict(forced_tokens=forced) if forced else dict(max_new_tokens=12)
            sess = model.generate_session(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                                          use_graphs=graphs, speculate=spec, show_progress_bar=False, **kw)
            while sess.step():
                pass
            outs.append(sess.result())
            misses.append(sess.spec_miss)
            rng.append(torch.get_rng_state())      # same CPU-generator consumption
        assert torch.equal(rng[0], rng[1])
        a, b = outs
        assert torch.equal(a.sequences, b.sequences)
        for i in range(2):
            if a.speech_outputs[i] is None:
                assert b.speech_outputs[i] is None
            else:
                assert torch.equal(a.speech_outputs[i].cpu(), b.speech_outputs[i].cpu())
        if forced:
            assert misses[1] > 0      # the mispredict path ran


def test_graphs_recaptured_after_workspace_growth():
    """A second generate() with a longer prompt grows the LM workspace (its
    prefill has more rows); hipGraphs captured by the first call hold the old
    pointers and must be re-captured (vv_ws_epoch), not replayed: the second
    call equals the same call on the eager path."""
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=8, device="cpu", mode="test", with_acoustic_encoder=False)
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=256)
    model.set_ddpm_inference_steps(3)
    sched = [[D] * 6 + [X], [D] * 5 + [X]]

    def run(L, graphs):
        ids = torch.randint(0, 151000, (2, L), generator=torch.Generator().manual_seed(L))
        torch.manual_seed(77)
        return model.generate(input_ids=ids, attention_mask=torch.ones(2, L, dtype=torch.long), tokenizer=TOK,
                              cfg_scale=1.3, forced_tokens=sched, use_graphs=graphs, max_new_tokens=10,
                              show_progress_bar=False)
    run(6, True)                      # captures the loop-body graphs at a small workspace
    e0 = model._graph_epoch
    long_graph = run(120, True)       # 240 prefill rows: the workspace grows
    assert model._graph_epoch != e0
    long_eager = run(120, False)
    for b in range(2):
        assert torch.equal(long_graph.speech_outputs[b].cpu(), long_eager.speech_outputs[b].cpu())


def test_device_multinomial_is_argmax_over_exponential_draw():
    """On the ROCm device too, torch.multinomial(p, 1) (what the reference's GPU
    run calls, modeling_vibevoice_inference.py:505) equals argmax(p / q) over a
    [B, vocab] Exp(1) draw from the same device-generator state — the draw the
    product makes when do_sample=True."""
    V, idx = 151936, [151643, 151652, 151653, 151654]
    for t in range(20):
        s = torch.full((3, V), float("-inf"), device=dev)
        s[:, idx] = torch.randn(3, 4, generator=torch.Generator().manual_seed(t)).to(dev) * 2
        p = torch.softmax(s, -1)
        torch.cuda.manual_seed(t)
        a = torch.multinomial(p, 1).squeeze(1).cpu()
        torch.cuda.manual_seed(t)
        q = torch.empty(3, V, device=dev).exponential_(1)
        c = torch.tensor(idx)[(torch.softmax(s[:, idx], -1) / q[:, idx]).argmax(-1).cpu()]
        assert torch.equal(a, c)


@pytest.mark.parametrize("seed", [1234, 77])
def test_generate_do_sample_matches_reference_loop(seed):
    """generate(generation_config={"do_sample": True}) on G8's sampling weights
    (control rows scaled so the draws are live; oracle/loop.py is pinned to the
    reference's own sampled generate() by G8 "sample<seed>").  The product
    draws the multinomial's Exp(1) vector on the device generator, as the
    reference's GPU run does; the test replays those device draws into the
    oracle (sample_q) while the diffusion noise comes from the CPU generator in
    both.  Sequences equal; audio as in the forced tests."""
    from test_oracle_golden import g8_sample_weights
    from golden_io import load
    z = load("g8_loop.npz")
    cfg, sd32 = g8_sample_weights()
    sd = {k: v.to(torch.bfloat16) for k, v in sd32.items()}
    model = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=128)
    model.set_ddpm_inference_steps(5)
    ids, mask = torch.from_numpy(z["input_ids"]), torch.from_numpy(z["attention_mask"])
    torch.manual_seed(seed)
    out = model.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                         generation_config={"do_sample": True}, show_progress_bar=False)
    torch.cuda.synchronize()
    valid = sorted(IDS[k] for k in ("start", "end", "diffusion", "eos"))
    torch.cuda.manual_seed(seed)
    qs = [torch.empty(2, cfg.decoder_config.vocab_size, device=dev).exponential_(1)[:, valid].cpu()
          for _ in range(out.sequences.shape[1] - ids.shape[1])]
    res = []
    for s32 in (False, True):
        torch.manual_seed(seed)
        res.append(oloop.generate(sd32 if s32 else sd, cfg, ids, mask, IDS, ddpm_steps=5, cfg_scale=1.3,
                                  do_sample=True, sample_q=lambda k: qs[k],
                                  dtype=torch.float32 if s32 else torch.bfloat16))
    (seqs, audio, reach), (_, audio32, _) = res
    print("sampled", (out.sequences[:, ids.shape[1]:] - 151640).tolist())
    assert torch.equal(out.sequences, seqs)
    assert torch.equal(out.reach_max_step_sample.cpu(), reach)
    for b in range(2):
        got, ref = out.speech_outputs[b], audio[b]
        if ref is None:
            assert got is None
            continue
        assert got.shape == ref.shape, (got.shape, ref.shape)
        a32 = audio32[b]
        noise = rel_err(ref, a32) if a32 is not None and a32.shape == ref.shape else 0.0
        e, c = rel_err(got, ref), cos(got, ref)
        print(f"do_sample sample {b} audio rel_err {e:.3e} cos {c:.6f} (bf16 reference vs fp32: {noise:.3e})")
        assert e < max(5e-2, 2 * noise) and c > 0.995
