"""vibevoice_amd — MI355X-native engine for VibeVoice's next-token-diffusion generate loop.

Public surface mirrors the reference (vibevoice/modular/modeling_vibevoice_inference.py,
vibevoice/processor/vibevoice_processor.py, vibevoice/modular/streamer.py):
    from vibevoice_amd import VibeVoiceForConditionalGenerationInference, VibeVoiceProcessor, AudioStreamer
"""
_LAZY = {
    "VibeVoiceForConditionalGenerationInference": ".modeling_vibevoice_inference",
    "VibeVoiceGenerationOutput": ".modeling_vibevoice_inference",
    "VibeVoiceConfig": ".config",
    "VibeVoiceProcessor": ".processor",
    "VibeVoiceTokenizerProcessor": ".processor",
    "VibeVoiceTextTokenizerFast": ".processor",
    "AudioStreamer": ".streamer",
    "AsyncAudioStreamer": ".streamer",
}
__all__ = list(_LAZY)


def __getattr__(name):
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module(_LAZY[name], __name__), name)
    raise AttributeError(name)
