"""Offline checkpoint directory, CPU only: the synthetic
checkpoint writer produces HF-style sharded safetensors with the reference's
state-dict names (tied lm_head omitted, as the reference's checkpoints do,
modeling_vibevoice_inference.py:120-129), and the product loader reads it back
with the safe loader into exactly the in-memory state dict."""
import os

import torch

from tiny import tiny_config
from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.modeling_vibevoice_inference import load_state_dict
from vibevoice_amd.weights import synthetic_state_dict, write_synthetic_checkpoint


def test_synthetic_checkpoint_round_trip(tmp_path):
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    files = write_synthetic_checkpoint(str(tmp_path), cfg, seed=4, mode="test", shard_bytes=8 << 20)
    assert len(files) > 1 and all(os.path.exists(os.path.join(tmp_path, f)) for f in files)
    assert files[0] == f"model-00001-of-{len(files):05d}.safetensors"
    sd = synthetic_state_dict(cfg, seed=4, device="cpu", mode="test")
    got = load_state_dict(str(tmp_path))
    assert set(got) == set(sd) | {"lm_head.weight"}
    for k, v in sd.items():
        assert got[k].dtype == v.dtype and torch.equal(got[k], v), k
    assert torch.equal(got["lm_head.weight"], sd["model.language_model.embed_tokens.weight"])
    cfg2 = VibeVoiceConfig.from_json_file(os.path.join(tmp_path, "config.json"))
    assert cfg2.to_dict() == cfg.to_dict()
