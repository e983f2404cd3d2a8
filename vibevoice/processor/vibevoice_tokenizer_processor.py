"""Reference path vibevoice/processor/vibevoice_tokenizer_processor.py."""
from vibevoice_amd.processor import AudioNormalizer, VibeVoiceTokenizerProcessor  # noqa: F401

__all__ = ["VibeVoiceTokenizerProcessor", "AudioNormalizer"]
