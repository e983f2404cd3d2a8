"""Reference path vibevoice/modular/configuration_vibevoice.py (config.json schema)."""
from vibevoice_amd.config import VibeVoiceConfig  # noqa: F401

__all__ = ["VibeVoiceConfig"]
