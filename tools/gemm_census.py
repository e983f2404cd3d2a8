"""GEMM shape census of one steady-state generate step (B=1, 1.5B): runs the
session eagerly with VV_GEMM_LOG=1 and counts the launches between two step
markers.  usage: VV_GEMM_LOG=1 python tools/gemm_census.py 2> census.log"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vibevoice_amd.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference  # noqa: E402
from vibevoice_amd.synthetic import synthetic_inputs, tokenizer_ids  # noqa: E402

inp = synthetic_inputs(batch=1, speakers=1, voice_seconds=3.0, text_tokens=64, seed=100)
model = VibeVoiceForConditionalGenerationInference.from_pretrained("synthetic:1.5B", device_map="cuda",
                                                                   synthetic_seed=0, max_batch=1, max_ctx=512)
model.use_graphs = False
model.set_ddpm_inference_steps(10)
tk = tokenizer_ids()
sess = model.generate_session(**inp, tokenizer=tk, cfg_scale=1.3, generation_config={"do_sample": False},
                              forced_tokens=[[tk.speech_diffusion_id] * 8], max_new_tokens=8, use_graphs=False)
for i in range(3):
    torch.cuda.synchronize()
    sys.stderr.flush()
    os.write(2, f"=== step {i}\n".encode())
    sess.step()
torch.cuda.synchronize()
os.write(2, b"=== end\n")
