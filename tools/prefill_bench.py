"""Prefill (time to first audio) on one MI355X: python tools/prefill_bench.py [L ...]

SURVEY.md §8f row 1.  Times GenerateSession creation -- the reference's first
loop iteration (modeling_vibevoice_inference.py:150-177 voice-prompt encode +
:222-225 scatter + the Qwen2 causal prefill of both streams) -- for a 3 s voice
prompt and a script of L text tokens, then prints one JSON line per L with the
prefill rate (prompt tokens / s) and the MFMA rate of the LM's prefill FLOPs
(2 * 1.31e9 per token for the projections + 4 * L^2 / 2 * 128 * heads * layers
for causal attention) against the 2.5 PFLOP/s dense bf16 peak."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = 2500.0   # MI355X dense bf16 (MI355X_MICROARCH.md)


def main():
    from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids

    lens = [int(x) for x in sys.argv[1:]] or [64, 1024, 4096, 16384]
    reps = int(os.environ.get("VV_PREFILL_REPS", "3"))
    model = VibeVoiceForConditionalGenerationInference.from_pretrained(
        "synthetic:1.5B", device_map="cuda:0", synthetic_seed=0, max_batch=1, max_ctx=max(lens) + 512)
    model.set_ddpm_inference_steps(10)
    tk = tokenizer_ids()
    cfg = model.config.decoder_config
    H, layers, nh = cfg.hidden_size, cfg.num_hidden_layers, cfg.num_attention_heads
    hd = H // nh
    kvh, inter = cfg.num_key_value_heads, cfg.intermediate_size
    lm_params = layers * (H * (H + 2 * kvh * hd) + H * H + 3 * H * inter)   # projections (lm_head: 1 row/stream)
    for T in lens:
        inp = synthetic_inputs(batch=1, speakers=1, voice_seconds=3.0, text_tokens=T, seed=7)
        L = inp["input_ids"].shape[1]
        times = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sess = model.generate_session(**inp, tokenizer=tk, cfg_scale=1.3, generation_config={"do_sample": False},
                                          forced_tokens=[[tk.speech_diffusion_id] * 4], max_new_tokens=4)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            del sess
        dt = min(times[1:])
        flops = 2.0 * lm_params * L + 4.0 * (L * (L + 1) / 2) * hd * nh * layers
        print(json.dumps({"prompt_tokens": L, "text_tokens": T, "prefill_ms": round(dt * 1e3, 3),
                          "prompt_tok_per_s": round(L / dt, 1),
                          "lm_tflops": round(flops / dt / 1e12, 2),
                          "mfma_frac_of_peak": round(flops / dt / 1e12 / PEAK_TFLOPS, 4),
                          "all_ms": [round(x * 1e3, 3) for x in times]}), flush=True)


if __name__ == "__main__":
    main()
