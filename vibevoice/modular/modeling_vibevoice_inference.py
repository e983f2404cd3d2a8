"""Reference path vibevoice/modular/modeling_vibevoice_inference.py.

Same public names; the class registers itself with
`AutoModelForCausalLM` exactly as the reference does at import time (:728), so
`AutoModelForCausalLM.from_config(VibeVoiceConfig(...))` builds the HIP engine.
"""
from transformers import AutoModelForCausalLM

from vibevoice_amd.config import VibeVoiceConfig
from vibevoice_amd.modeling_vibevoice_inference import (  # noqa: F401
    VibeVoiceForConditionalGenerationInference,
    VibeVoiceGenerationOutput,
    VibeVoiceTokenConstraintProcessor,
)

AutoModelForCausalLM.register(VibeVoiceConfig, VibeVoiceForConditionalGenerationInference, exist_ok=True)

__all__ = ["VibeVoiceForConditionalGenerationInference"]
