"""vibevoice_amd — MI355X-native engine for VibeVoice's next-token-diffusion generate loop.

Public surface mirrors the reference (vibevoice/modular/modeling_vibevoice_inference.py):
    from vibevoice_amd import VibeVoiceForConditionalGenerationInference
"""
__all__ = ["VibeVoiceForConditionalGenerationInference", "VibeVoiceConfig"]


def __getattr__(name):
    if name == "VibeVoiceForConditionalGenerationInference":
        from .modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
        return VibeVoiceForConditionalGenerationInference
    if name == "VibeVoiceConfig":
        from .config import VibeVoiceConfig
        return VibeVoiceConfig
    raise AttributeError(name)
