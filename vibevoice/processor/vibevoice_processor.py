"""Reference path vibevoice/processor/vibevoice_processor.py."""
from vibevoice_amd.processor import VibeVoiceProcessor  # noqa: F401

__all__ = ["VibeVoiceProcessor"]
