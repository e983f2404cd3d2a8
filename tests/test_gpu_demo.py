"""demo/inference_from_file.py's call sequence (:255-378) through the
reference's own import paths (`vibevoice.*`, :9-10), on a synthetic checkpoint
directory (tiny config; config.json + indexed safetensors shards +
preprocessor_config.json naming a local Qwen2-style tokenizer):

  script file -> VibeVoiceProcessor.from_pretrained(model_path)
  -> VibeVoiceForConditionalGenerationInference.from_pretrained(model_path,
       torch_dtype=bf16, device_map="cuda", attn_implementation="flash_attention_2")
  -> .eval(), .set_ddpm_inference_steps(num_steps=10), model.model.language_model.config._attn_implementation
  -> processor(text=[script], voice_samples=[wav paths], padding=True, return_tensors="pt",
               return_attention_mask=True), tensors moved to cuda
  -> generate(**inputs, max_new_tokens=None, cfg_scale=1.3, tokenizer=processor.tokenizer,
              generation_config={'do_sample': False}, verbose=True)   (free-running greedy)
  -> processor.save_audio(outputs.speech_outputs[0], output_path=...)

Written for this repository (the demo itself is not copied).  Checks the
plumbing: the WAV on disk equals speech_outputs[0], its length is hop x the
number of speech_diffusion tokens generated, sequences extend input_ids and
only the four legal ids are generated.

Random weights pick arbitrary control tokens (an unpatched tiny model never
chose speech_diffusion in 212 greedy steps), so the checkpoint is steered the
way a trained one behaves on a script: one residual coordinate j is held
large and positive (embedding column and both connectors' output bias), and
an untied lm_head reads it with +1 for speech_diffusion and -1 for the other
control ids, so greedy decoding emits speech until the length cap.
"""
import os

import numpy as np
import pytest
import torch


pytestmark = pytest.mark.gpu
TOK_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny_qwen_tokenizer")


def test_demo_call_sequence(tmp_path):
    from scipy.io import wavfile
    from vibevoice.modular.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    from vibevoice.processor.vibevoice_processor import VibeVoiceProcessor
    from vibevoice_amd.weights import write_synthetic_checkpoint

    from tiny import tiny_dict
    from vibevoice_amd.config import VibeVoiceConfig
    from vibevoice_amd.processor import VibeVoiceTextTokenizerFast
    from vibevoice_amd.weights import synthetic_state_dict

    model_path = str(tmp_path / "model")
    d = tiny_dict(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    d["tie_word_embeddings"] = False
    cfg = VibeVoiceConfig(d)
    sd = synthetic_state_dict(cfg, seed=31, device="cpu", mode="test")
    tk0 = VibeVoiceTextTokenizerFast.from_pretrained(TOK_DIR)
    j = 7
    sd["model.language_model.embed_tokens.weight"][:, j] = 50.0
    for c in ("acoustic", "semantic"):
        sd[f"model.{c}_connector.fc2.bias"][j] = 50.0
    head = sd["lm_head.weight"]
    for t in (tk0.speech_start_id, tk0.speech_end_id, tk0.eos_token_id):
        head[t, j] = -1.0
    head[tk0.speech_diffusion_id, j] = 1.0
    write_synthetic_checkpoint(model_path, cfg, shard_bytes=8 << 20, tokenizer_dir=TOK_DIR, state_dict=sd)
    rng = np.random.default_rng(3)
    voices = []
    for name, n in (("en-Alice_woman", 90), ("en-Carter_man", 57)):
        p = str(tmp_path / f"{name}.wav")
        wavfile.write(p, 24000, (0.1 * rng.standard_normal(n)).astype(np.float32))
        voices.append(p)
    txt = tmp_path / "2p_hello.txt"
    txt.write_text("Speaker 1: Hello there, welcome to the show.\nSpeaker 2: It's great to be here!\n")
    scripts = [ln for ln in txt.read_text().splitlines() if ln.strip()]
    full_script = "\n".join(scripts).replace("’", "'")

    processor = VibeVoiceProcessor.from_pretrained(model_path)
    model = VibeVoiceForConditionalGenerationInference.from_pretrained(
        model_path, torch_dtype=torch.bfloat16, device_map="cuda", attn_implementation="flash_attention_2")
    model.eval()
    model.set_ddpm_inference_steps(num_steps=10)
    assert model.model.language_model.config._attn_implementation == "flash_attention_2"
    inputs = processor(text=[full_script], voice_samples=[voices], padding=True, return_tensors="pt",
                       return_attention_mask=True)
    for k, v in inputs.items():
        if torch.is_tensor(v):
            inputs[k] = v.to("cuda")
    torch.manual_seed(42)
    outputs = model.generate(**inputs, max_new_tokens=None, cfg_scale=1.3, tokenizer=processor.tokenizer,
                             generation_config={"do_sample": False}, verbose=True)
    out_path = str(tmp_path / "outputs" / "2p_hello_generated.wav")
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    processor.save_audio(outputs.speech_outputs[0], output_path=out_path)

    tk = processor.tokenizer
    L = inputs["input_ids"].shape[1]
    seq = outputs.sequences
    assert torch.equal(seq[:, :L].cpu(), inputs["input_ids"].cpu())
    gen = seq[0, L:]
    legal = {tk.speech_start_id, tk.speech_end_id, tk.speech_diffusion_id, tk.eos_token_id}
    assert set(gen.tolist()) <= legal
    n_diff = int((gen == tk.speech_diffusion_id).sum())
    sr, wav = wavfile.read(out_path)
    assert sr == 24000
    assert n_diff > 0
    hop = model.engine.hop
    assert wav.shape[-1] == n_diff * hop == outputs.speech_outputs[0].shape[-1]
    assert np.array_equal(wav.reshape(-1), outputs.speech_outputs[0].float().cpu().numpy().reshape(-1))
    print(f"demo sequence: {gen.numel()} generated tokens, {n_diff} speech frames, {wav.shape[-1]} samples")
