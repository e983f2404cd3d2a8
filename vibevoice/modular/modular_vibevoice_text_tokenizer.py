"""Reference path vibevoice/modular/modular_vibevoice_text_tokenizer.py."""
from vibevoice_amd.processor import VibeVoiceTextTokenizerFast  # noqa: F401

__all__ = ["VibeVoiceTextTokenizerFast"]
