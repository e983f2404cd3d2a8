"""Host-side time of one generate-loop step (bench.py's configuration): wraps the
session's phase methods and the logits / error-word event waits with
perf_counter, runs warm-up + 60 timed steps, prints the mean host time per
call and per step of each, and the step's wall time -- where the host, not the
GPU, sets the pace (a GPU idle gap in profiles/summarize.py's launch order).
usage: python tools/host_step_timing.py [B]"""
import collections
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    from vibevoice_amd import modeling_vibevoice_inference as mvi
    from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids
    acc = collections.defaultdict(lambda: [0, 0.0])
    on = [False]

    def wrap(obj, name, label=None):
        f = getattr(obj, name)

        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                if on[0]:
                    e = acc[label or name]
                    e[0] += 1
                    e[1] += time.perf_counter() - t
        setattr(obj, name, g)
    sess_cls = [c for c in vars(mvi).values() if isinstance(c, type) and hasattr(c, "_speculate")][0]
    for n in ("step", "_lm_phase", "_speculate", "_diff_phase", "_post_phase", "_push_controls", "_stage_diffusion",
              "_check_err", "_replay"):
        wrap(sess_cls, n)
    wrap(torch.cuda.Event, "synchronize", "Event.synchronize (logits / error word)")
    wrap(torch.cuda.CUDAGraph, "replay", "CUDAGraph.replay")
    total = 90
    inp = synthetic_inputs(batch=B, speakers=2 if B > 1 else 1, voice_seconds=3.0, text_tokens=64, seed=100)
    L = inp["input_ids"].shape[1]
    model = VibeVoiceForConditionalGenerationInference.from_pretrained(
        "synthetic:1.5B", device_map="cuda", synthetic_seed=0, max_batch=B, max_ctx=L + total + 8)
    model.set_ddpm_inference_steps(10)
    tk = tokenizer_ids()
    forced = [[tk.speech_diffusion_id] * total for _ in range(B)]
    sess = model.generate_session(**inp, tokenizer=tk, cfg_scale=1.3, generation_config={"do_sample": False},
                                  forced_tokens=forced, max_length_times=total / L + 1, max_new_tokens=total + 2)
    for _ in range(20):
        assert sess.step()
    torch.cuda.synchronize()
    on[0] = True
    K = 60
    t0 = time.perf_counter()
    for _ in range(K):
        assert sess.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    on[0] = False
    print(f"B={B}: wall per step {dt * 1e6:.0f} us")
    for k, (c, t) in sorted(acc.items(), key=lambda x: -x[1][1]):
        print(f"{k:45s} calls/step {c / K:5.2f}  us/call {t / c * 1e6:8.1f}  us/step {t / K * 1e6:8.1f}")


if __name__ == "__main__":
    main()
