"""Two engines driven from two host threads at once.

SURVEY.md §8b's threading contract: the reference's Gradio demo serves
generate() from worker threads (demo/gradio_demo.py), so two model instances in
one process must not share launch plans, workspaces or capture state.  Here two
tiny models with different weights generate concurrently, each on its own
stream and host thread with its own diffusion-noise generator
(`generate(generator=...)`), while their loop bodies are captured into
hipGraphs (thread-local capture mode, one capture stream per model) and
replayed; each thread's output must be BIT-identical to the same call run
alone afterwards (which replays the graphs captured during the concurrent run).
"""
import threading
import types

import pytest
import torch

from tiny import tiny_config
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
from vibevoice_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
dev = "cuda"
IDS = dict(eos=151643, start=151652, end=151653, diffusion=151654)
D, E, S, X = IDS["diffusion"], IDS["end"], IDS["start"], IDS["eos"]
TOK = types.SimpleNamespace(speech_start_id=S, speech_end_id=E, speech_diffusion_id=D, eos_token_id=X,
                            bos_token_id=None, pad_token_id=151655)
SCHED = [[D] * 6 + [E, S, D, D, D, X], [D, D, D, E, S, D, D, D, D, X]]


def _model(seed):
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    sd = synthetic_state_dict(cfg, seed=seed, device="cpu", mode="test", with_acoustic_encoder=False)
    m = VibeVoiceForConditionalGenerationInference(cfg, sd, dev, max_batch=2, max_ctx=256)
    m.set_ddpm_inference_steps(5)
    return m


def _inputs(seed):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, 151000, (2, 40), generator=g)
    mask = torch.ones(2, 40, dtype=torch.long)
    mask[1, :5] = 0
    ids[1, :5] = TOK.pad_token_id
    return ids, mask


def _run(model, seed, stream):
    ids, mask = _inputs(seed)
    with torch.cuda.stream(stream):
        out = model.generate(input_ids=ids, attention_mask=mask, tokenizer=TOK, cfg_scale=1.3, forced_tokens=SCHED,
                             generator=torch.Generator().manual_seed(seed), show_progress_bar=False)
        stream.synchronize()
        return out.sequences.clone(), [a.clone().cpu() for a in out.speech_outputs]


def test_two_engines_two_threads_bit_identical_to_serial():
    models = [_model(31), _model(32)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    seeds = [101, 202]
    res, errs = [None, None], []
    start = threading.Barrier(2)

    def worker(i):
        try:
            start.wait()
            for _ in range(2):   # the second call replays the graphs the first captured
                res[i] = _run(models[i], seeds[i], streams[i])
        except Exception as e:   # surfaced below
            errs.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a generate() thread hung"
    if errs:
        raise errs[0]
    torch.cuda.synchronize()
    for i in range(2):
        seq, audio = _run(models[i], seeds[i], streams[i])
        assert torch.equal(seq, res[i][0])
        assert len(audio) == len(res[i][1]) == 2
        for b in range(2):
            assert audio[b].shape == res[i][1][b].shape and audio[b].numel() > 0
            assert torch.equal(audio[b], res[i][1][b]), f"model {i} sample {b}: concurrent run differs from serial"
        print(f"model {i}: concurrent == serial, bitwise ({seq.shape[1]} tokens, {audio[0].shape[-1]} samples)")
    # different weights / prompts: the two models really computed different things
    assert not torch.equal(res[0][1][0], res[1][1][0])
