"""The reference's plugin surface around generate() (GPU):

* from_pretrained(<dir>) loads a HF-style checkpoint directory (config.json +
  sharded *.safetensors with the reference's state-dict names, untied lm_head
  dropped -> tied to the embedding as modeling_vibevoice_inference.py:120-129)
  and produces exactly what the in-memory state dict produces;
* audio_streamer: put() receives every chunk of speech_outputs per sample,
  end() is called for a finished sample, and — as in the reference
  (modeling_vibevoice_inference.py:443-447) — the loop stops at the next step
  once any streamer flag is set;
* stop_check_fn stops the loop and ends the streamer (:434-440);
* model.model.language_model.config._attn_implementation exists
  (demo/inference_from_file.py:315-316).
"""
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from tiny import tiny_config, tiny_dict
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.synthetic import tokenizer_ids
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
TOK = tokenizer_ids()
D, E, S, X = TOK.speech_diffusion_id, TOK.speech_end_id, TOK.speech_start_id, TOK.eos_token_id


class RecordingStreamer:
    """Duck-typed AudioStreamer (vibevoice/modular/streamer.py:13-76)."""

    def __init__(self, batch):
        self.chunks = [[] for _ in range(batch)]
        self.finished_flags = [False] * batch
        self.ended = []

    def put(self, audio_chunks, sample_indices):
        for i, idx in enumerate(sample_indices.tolist()):
            if not self.finished_flags[idx]:
                self.chunks[idx].append(audio_chunks[i].detach().cpu())

    def end(self, sample_indices=None):
        idx = range(len(self.finished_flags)) if sample_indices is None else sample_indices.tolist()
        for i in idx:
            if not self.finished_flags[i]:
                self.finished_flags[i] = True
                self.ended.append(i)


def _model(sd, cfg):
    m = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=128)
    m.set_ddpm_inference_steps(3)
    return m


def _inputs():
    g = torch.Generator().manual_seed(4)
    return torch.randint(0, 151000, (2, 12), generator=g), torch.ones(2, 12, dtype=torch.long)


def test_from_pretrained_checkpoint_dir(tmp_path):
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=9, device="cpu", mode="test", with_acoustic_encoder=True)
    names = sorted(k for k in sd if k != "lm_head.weight")           # tied: not saved
    half = len(names) // 2
    for i, part in enumerate((names[:half], names[half:])):
        save_file({k: sd[k].contiguous() for k in part}, os.path.join(tmp_path, f"model-0000{i + 1}-of-00002.safetensors"))
    with open(os.path.join(tmp_path, "config.json"), "w") as f:
        json.dump(tiny_dict(hidden=256, layers=2, heads=2, kv_heads=1, inter=512), f)
    a = VibeVoiceForConditionalGenerationInference.from_pretrained(str(tmp_path), torch_dtype=torch.bfloat16,
                                                                   device_map="cuda",
                                                                   attn_implementation="flash_attention_2",
                                                                   max_batch=2, max_ctx=128)
    assert a.model.language_model.config._attn_implementation == "flash_attention_2"
    b = _model(sd, cfg)
    a.set_ddpm_inference_steps(3)
    ids, mask = _inputs()
    sched = [[D, D, D, X], [D, D, E, X]]
    outs = []
    for m in (a, b):
        torch.manual_seed(5)
        outs.append(m.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                               forced_tokens=sched, show_progress_bar=False))
    assert torch.equal(outs[0].sequences, outs[1].sequences)
    for i in range(2):
        assert torch.equal(outs[0].speech_outputs[i].cpu(), outs[1].speech_outputs[i].cpu())


def test_streamer_and_stop_check():
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=10, device="cpu", mode="test", with_acoustic_encoder=False)
    m = _model(sd, cfg)
    ids, mask = _inputs()
    # sample 1 emits eos at step 2: the streamer ends it, the loop stops at step 3
    sched = [[D] * 8 + [X], [D, D, X]]
    st = RecordingStreamer(2)
    torch.manual_seed(6)
    out = m.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3, forced_tokens=sched,
                     audio_streamer=st, show_progress_bar=False)
    assert out.sequences.shape[1] == 12 + 3
    assert st.ended[0] == 1 and sorted(st.ended) == [0, 1]
    for b in range(2):
        got = torch.cat(st.chunks[b], dim=-1)
        assert torch.equal(got.reshape(-1), out.speech_outputs[b].cpu().reshape(-1))
    # external stop after 4 steps
    calls = {"n": 0}

    def stop():
        calls["n"] += 1
        return calls["n"] > 4
    st2 = RecordingStreamer(2)
    torch.manual_seed(6)
    out2 = m.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                      forced_tokens=[[D] * 8 + [X]] * 2, audio_streamer=st2, stop_check_fn=stop,
                      show_progress_bar=False)
    assert out2.sequences.shape[1] == 12 + 4
    assert sorted(st2.ended) == [0, 1]
    assert out2.speech_outputs[0].shape[-1] == 4 * m.engine.hop


def test_grid_wait_error_raises_before_audio_is_streamed():
    """A grid wait of a one-launch kernel that gave up (raised here by the
    diagnostic hook, as the kernel's bounded wait would) invalidates that step's
    latents: the error word is read back behind every diffusion step
    (vv_sync_error_async), and step() raises before that step's audio reaches
    the streamer -- chunks before it were streamed, none from it on."""
    from vibevoice_amd import _lib
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=10, device="cpu", mode="test", with_acoustic_encoder=False)
    m = _model(sd, cfg)
    ids, mask = _inputs()
    for end_with_result in (False, True):
        st = RecordingStreamer(2)
        torch.manual_seed(6)
        sess = m.generate_session(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                                  forced_tokens=[[D] * 8 + [X]] * 2, audio_streamer=st)
        assert sess.step() and sess.step() and sess.step()
        clean = [len(c) for c in st.chunks]
        assert clean == [2, 2]                    # steps 0, 1 streamed; step 2's chunk waits for its check
        _lib.check(_lib.lib().vv_diag_raise_sync_error(m.engine.h), "raise")
        assert sess.step()                        # step 3 diffuses behind the raised word; step 2's chunk goes out
        assert [len(c) for c in st.chunks] == [3, 3]
        with pytest.raises(RuntimeError, match="grid wait gave up"):
            sess.result() if end_with_result else sess.step()
        assert [len(c) for c in st.chunks] == [3, 3]          # step 3's chunk never reached the streamer
        assert not sess.step()                                # the session is over
        _assert_counters_consistent(m)                        # vv_sync_reset ran before the raise
        # the word was reset by its read-back: a fresh session runs clean
        st2 = RecordingStreamer(2)
        out = m.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                         forced_tokens=[[D, D, X]] * 2, audio_streamer=st2, show_progress_bar=False)
        assert [len(c) for c in st2.chunks] == [2, 2] and out.speech_outputs[0].shape[-1] == 2 * m.engine.hop


def _assert_counters_consistent(m):
    """vv_diag_sync_words: every shard line a multiple of 32 arrivals, every
    generation line a multiple of 8 -- the state between two launches.  The
    raise hook leaves shard 0 at +5 and the generations at +3, as a launch that
    gave up does; only vv_sync_reset makes them consistent again."""
    import ctypes
    from vibevoice_amd import _lib
    words = (ctypes.c_uint * 39)()
    _lib.check(_lib.lib().vv_diag_sync_words(m.engine.h, words), "sync_words")
    for fam in range(3):
        w = list(words[fam * 13:(fam + 1) * 13])
        assert all(v % 32 == 0 for v in w[:8]), (fam, w)
        assert w[11] % 8 == 0 and w[12] % 8 == 0, (fam, w)


def test_grid_wait_error_on_the_last_step_without_streamer():
    """with no streamer, a wait that gave up in the LAST diffusion
    step (no logits read-back after it) still raises -- result() drains the
    queued error-word copy -- and the counters it left part-advanced are reset,
    so the next generate() equals a run that never saw the error."""
    from vibevoice_amd import _lib
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=11, device="cpu", mode="test", with_acoustic_encoder=False)
    m = _model(sd, cfg)
    ids, mask = _inputs()
    sched = [[D, D, D, X]] * 2

    def run():
        torch.manual_seed(7)
        return m.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3, forced_tokens=sched,
                          show_progress_bar=False)
    clean = run()
    torch.manual_seed(7)
    sess = m.generate_session(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3,
                              forced_tokens=[[D] * 8 + [X]] * 2)
    assert sess.step() and sess.step()
    _lib.check(_lib.lib().vv_diag_raise_sync_error(m.engine.h), "raise")
    assert sess.step()                     # the last diffusion step before result(): no read-back after it
    with pytest.raises(RuntimeError, match="grid wait gave up"):
        sess.result()
    _assert_counters_consistent(m)
    again = run()
    assert torch.equal(clean.sequences, again.sequences)
    for b in range(2):
        assert torch.equal(clean.speech_outputs[b].cpu(), again.speech_outputs[b].cpu())


def test_noise_scheduler_swap_sde():
    """gradio_demo.py:114-119: model.model.noise_scheduler replaced through
    from_config(config, algorithm_type="sde-dpmsolver++",
    beta_schedule="squaredcos_cap_v2"), then set_ddpm_inference_steps.  The SDE
    noise comes from the device generator, so a seeded run is reproducible and
    graph replay equals the eager loop; the result differs from the ODE solver's."""
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    m = _model(synthetic_state_dict(cfg, seed=9, device="cpu", mode="test", with_acoustic_encoder=False), cfg)
    ids, mask = _inputs()
    sched = [[D] * 5 + [X]] * 2

    def run(graphs):
        torch.manual_seed(5)
        return m.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3, forced_tokens=sched,
                          use_graphs=graphs, show_progress_bar=False)
    ode = run(True)
    ns = m.model.noise_scheduler
    m.model.noise_scheduler = ns.from_config(ns.config, algorithm_type="sde-dpmsolver++",
                                             beta_schedule="squaredcos_cap_v2")
    m.set_ddpm_inference_steps(num_steps=5)
    assert m.model.noise_scheduler.config.algorithm_type == "sde-dpmsolver++"
    outs = [run(False), run(True), run(True)]
    for o in outs[1:]:
        for b in range(2):
            assert torch.equal(o.speech_outputs[b].cpu(), outs[0].speech_outputs[b].cpu())
    assert not torch.equal(outs[0].speech_outputs[0].cpu(), ode.speech_outputs[0].cpu())
    with pytest.raises(NotImplementedError):
        ns.from_config(ns.config, algorithm_type="dpmsolver")


def test_processor_to_generate_with_audio_streamer():
    """demo/inference_from_file.py's path end to end on a tiny model: the
    product VibeVoiceProcessor (tiny Qwen2-style vocabulary, voice prompts of
    ragged lengths; speech_tok_compress_ratio = the tiny codec's hop) -> the
    engine's generate() with the product AudioStreamer.  Every streamed chunk
    equals speech_outputs, sequences extend input_ids, and the voice latents
    change the result (the prefill splice is live)."""
    import numpy as np
    from vibevoice_amd.processor import VibeVoiceProcessor, VibeVoiceTextTokenizerFast
    from vibevoice_amd.streamer import AudioStreamer
    tok_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny_qwen_tokenizer")
    tk = VibeVoiceTextTokenizerFast.from_pretrained(tok_dir)
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=12, device="cpu", mode="test", with_acoustic_encoder=True)
    m = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=512)
    m.set_ddpm_inference_steps(3)
    proc = VibeVoiceProcessor(tokenizer=tk, speech_tok_compress_ratio=m.engine.hop)
    rng = np.random.default_rng(5)
    v = [(0.2 * rng.standard_normal(n)).astype(np.float32) for n in (37, 20)]
    scripts = ["Speaker 1: Hello there.\nSpeaker 2: Hi!", "Speaker 1: Fine, thanks."]
    inputs = proc(text=scripts, voice_samples=[[v[0], v[1]], [v[1]]], padding=True, return_tensors="pt")
    d = tk.speech_diffusion_id
    sched = [[d] * 4 + [tk.eos_token_id], [d] * 2 + [tk.speech_end_id, tk.eos_token_id]]

    def run(streamer, voices=True):
        kw = dict(inputs)
        if not voices:
            kw["speech_tensors"] = torch.zeros_like(kw["speech_tensors"])
        torch.manual_seed(7)
        return m.generate(**kw, tokenizer=tk, cfg_scale=1.3, forced_tokens=sched, audio_streamer=streamer,
                          generation_config={"do_sample": False}, show_progress_bar=False)
    st = AudioStreamer(batch_size=2)
    out = run(st)
    L = inputs["input_ids"].shape[1]
    assert torch.equal(out.sequences[:, :L], inputs["input_ids"])
    assert st.finished_flags == [True, True]
    for b, n in enumerate((4, 2)):
        chunks = list(st.get_stream(b))
        assert len(chunks) == n
        assert torch.equal(torch.cat(chunks, dim=-1).reshape(-1), out.speech_outputs[b].cpu().reshape(-1))
    silent = run(None, voices=False)
    assert not torch.equal(silent.speech_outputs[0].cpu(), out.speech_outputs[0].cpu())
