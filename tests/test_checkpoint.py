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


def test_checkpoint_index_and_stale_shards(tmp_path):
    """model.safetensors.index.json names every tensor's shard (the HF loader's
    map); a rewrite with fewer shards removes the old ones, and the loader
    reads exactly the indexed files."""
    import json
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    many = write_synthetic_checkpoint(str(tmp_path), cfg, seed=4, mode="test", shard_bytes=4 << 20)
    few = write_synthetic_checkpoint(str(tmp_path), cfg, seed=5, mode="test", shard_bytes=1 << 30)
    assert len(many) > len(few) == 1
    assert sorted(f for f in os.listdir(tmp_path) if f.endswith(".safetensors")) == few
    with open(os.path.join(tmp_path, "model.safetensors.index.json")) as f:
        idx = json.load(f)
    sd = synthetic_state_dict(cfg, seed=5, device="cpu", mode="test")
    assert set(idx["weight_map"]) == set(sd) - {"lm_head.weight"}
    assert idx["metadata"]["total_size"] == sum(v.numel() * v.element_size() for k, v in sd.items()
                                                if k != "lm_head.weight")
    got = load_state_dict(str(tmp_path), cfg)
    for k, v in sd.items():
        assert torch.equal(got[k], v), k


def test_checkpoint_tie_rule_follows_top_level_flag(tmp_path):
    """The reference ties lm_head when the TOP-LEVEL tie_word_embeddings is
    set (PretrainedConfig default True), whatever decoder_config says
    (modeling_vibevoice_inference.py:120-129): a Large-style config
    (decoder tie false, top level absent) saves no lm_head; an explicit
    top-level false saves it and loads it back untied."""
    from tiny import tiny_dict
    d = tiny_dict(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    d["decoder_config"]["tie_word_embeddings"] = False
    cfg = VibeVoiceConfig(d)
    write_synthetic_checkpoint(str(tmp_path / "a"), cfg, seed=4, mode="test")
    got = load_state_dict(str(tmp_path / "a"), cfg)
    assert got["lm_head.weight"] is got["model.language_model.embed_tokens.weight"]
    d["tie_word_embeddings"] = False
    cfg2 = VibeVoiceConfig(d)
    write_synthetic_checkpoint(str(tmp_path / "b"), cfg2, seed=4, mode="test", shard_bytes=8 << 20)
    sd = synthetic_state_dict(cfg2, seed=4, device="cpu", mode="test")
    got = load_state_dict(str(tmp_path / "b"), cfg2)
    assert torch.equal(got["lm_head.weight"], sd["lm_head.weight"])
    assert not torch.equal(got["lm_head.weight"], got["model.language_model.embed_tokens.weight"])


def test_checkpoint_preprocessor_config(tmp_path):
    """tokenizer_dir= writes the preprocessor_config.json that
    VibeVoiceProcessor.from_pretrained(<model dir>) reads (the demo loads the
    processor from the model path, inference_from_file.py:256)."""
    from vibevoice.processor.vibevoice_processor import VibeVoiceProcessor
    tok_dir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tiny_qwen_tokenizer")
    cfg = tiny_config(hidden=256, layers=2, heads=2, kv_heads=1, inter=512)
    write_synthetic_checkpoint(str(tmp_path), cfg, seed=4, mode="test", tokenizer_dir=tok_dir)
    proc = VibeVoiceProcessor.from_pretrained(str(tmp_path))
    assert proc.speech_tok_compress_ratio == cfg.hop
    assert proc.tokenizer.speech_diffusion_id == proc.tokenizer.convert_tokens_to_ids("<|vision_pad|>")
