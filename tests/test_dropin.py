"""The reference's import paths and plugin registration resolve to this
package (CPU: no engine is built).

demo/inference_from_file.py:9-10 and gradio_demo.py:23-26 import
`vibevoice.modular.modeling_vibevoice_inference`,
`vibevoice.processor.vibevoice_processor`,
`vibevoice.modular.configuration_vibevoice` and `vibevoice.modular.streamer`;
modeling_vibevoice_inference.py:728 registers the class with
AutoModelForCausalLM.  The demo's CPU / MPS / fp32 branches
(inference_from_file.py:258-303) must fail with an explicit error before any
device work — the product has no CPU path.
"""
import os

import pytest
import torch

import vibevoice_amd
from vibevoice_amd import modeling_vibevoice_inference as mvi_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_import_paths_resolve_to_product():
    from vibevoice.modular.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    from vibevoice.processor.vibevoice_processor import VibeVoiceProcessor
    from vibevoice.processor.vibevoice_tokenizer_processor import AudioNormalizer, VibeVoiceTokenizerProcessor
    from vibevoice.modular.configuration_vibevoice import VibeVoiceConfig
    from vibevoice.modular.streamer import AsyncAudioStreamer, AudioStreamer
    from vibevoice.modular.modular_vibevoice_text_tokenizer import VibeVoiceTextTokenizerFast
    from vibevoice.schedule.dpm_solver import DPMSolverMultistepScheduler
    import vibevoice
    assert os.path.dirname(vibevoice.__file__) == os.path.join(ROOT, "vibevoice")
    assert VibeVoiceForConditionalGenerationInference is vibevoice_amd.VibeVoiceForConditionalGenerationInference
    assert VibeVoiceProcessor is vibevoice_amd.VibeVoiceProcessor
    assert VibeVoiceTokenizerProcessor is vibevoice_amd.VibeVoiceTokenizerProcessor
    assert VibeVoiceConfig is vibevoice_amd.VibeVoiceConfig
    assert AudioStreamer is vibevoice_amd.AudioStreamer and AsyncAudioStreamer is vibevoice_amd.AsyncAudioStreamer
    assert VibeVoiceTextTokenizerFast is vibevoice_amd.VibeVoiceTextTokenizerFast
    assert callable(AudioNormalizer)
    s = DPMSolverMultistepScheduler()
    sde = s.from_config(s.config, algorithm_type="sde-dpmsolver++", beta_schedule="squaredcos_cap_v2")
    assert sde.sde


def test_auto_model_registration():
    from transformers import AutoModelForCausalLM
    from transformers.models.auto.auto_factory import _get_model_class
    from vibevoice.modular.modeling_vibevoice_inference import VibeVoiceForConditionalGenerationInference
    cfg = vibevoice_amd.VibeVoiceConfig.builtin("1.5B")
    assert type(cfg) in AutoModelForCausalLM._model_mapping
    assert _get_model_class(cfg, AutoModelForCausalLM._model_mapping) is VibeVoiceForConditionalGenerationInference
    # from_config dispatches to the class; on a GPU-less host it stops at the device check
    with pytest.raises(ValueError, match="ROCm GPU only"):
        AutoModelForCausalLM.from_config(cfg, device_map="cpu")


@pytest.mark.parametrize("device_map", ["cpu", "mps", None, {"": "cpu"}, {"a": "cuda:0", "b": "cuda:1"}, "disk"])
def test_cpu_device_map_refused(device_map):
    with pytest.raises(ValueError):
        mvi_amd.resolve_device(device_map)
    with pytest.raises(ValueError):
        mvi_amd.VibeVoiceForConditionalGenerationInference.from_pretrained(
            "synthetic:1.5B", torch_dtype=torch.bfloat16, device_map=device_map)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, "float32"])
def test_non_bf16_dtype_refused(dtype):
    with pytest.raises(ValueError, match="bfloat16"):
        mvi_amd.VibeVoiceForConditionalGenerationInference.from_pretrained(
            "synthetic:1.5B", torch_dtype=dtype, device_map="cuda")


def test_gpu_device_maps_accepted():
    for dm, idx in [("cuda:3", 3), (torch.device("cuda", 2), 2), (5, 5), ({"": "cuda:1"}, 1), ({"": 4}, 4)]:
        d = mvi_amd.resolve_device(dm)
        assert d.type == "cuda" and d.index == idx
    assert mvi_amd.resolve_device("cuda").type == "cuda"
    assert mvi_amd.resolve_device("auto").type == "cuda"
    assert mvi_amd.resolve_dtype(None) is torch.bfloat16 and mvi_amd.resolve_dtype("auto") is torch.bfloat16


def test_token_constraint_processor():
    from vibevoice.modular.modeling_vibevoice_inference import VibeVoiceTokenConstraintProcessor
    p = VibeVoiceTokenConstraintProcessor([3, 5])
    s = p(None, torch.zeros(2, 8))
    assert torch.isfinite(s[:, [3, 5]]).all() and torch.isinf(s[:, [0, 1, 2, 4, 6, 7]]).all()
