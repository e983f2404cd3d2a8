"""Reference path vibevoice/modular/modular_vibevoice_tokenizer.py: the
streaming cache and encoder-output types callers construct.  The tokenizer
models themselves are reached as `model.model.acoustic_tokenizer` /
`model.model.semantic_tokenizer` (views over the HIP engine)."""
from vibevoice_amd.tokenizer import VibeVoiceTokenizerEncoderOutput, VibeVoiceTokenizerStreamingCache  # noqa: F401

__all__ = ["VibeVoiceTokenizerStreamingCache", "VibeVoiceTokenizerEncoderOutput"]
