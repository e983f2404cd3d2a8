"""VibeVoice configuration (the reference's config.json schema).

Reads the same JSON as VibeVoiceConfig (vibevoice/modular/configuration_vibevoice.py:
164-241; vibevoice/configs/qwen2.5_{1.5b_64k,7b_32k}.json) and derives the static
dimensions the engine needs.
"""
import copy
import json
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))
CONFIG_DIR = os.path.join(HERE, "configs")

# Defaults of the sub-configs (configuration_vibevoice.py:13-162)
TOKENIZER_DEFAULTS = dict(channels=1, causal=True, vae_dim=64, fix_std=0.5, std_dist_type="gaussian",
                          mixer_layer="depthwise_conv", conv_norm="none", pad_mode="constant",
                          disable_last_norm=True, layernorm="RMSNorm", layernorm_eps=1e-5,
                          layernorm_elementwise_affine=True, conv_bias=True, layer_scale_init_value=1e-6,
                          weight_init_value=1e-2, encoder_n_filters=32, encoder_ratios=[8, 5, 5, 4, 2, 2],
                          encoder_depths="3-3-3-3-3-3-8", decoder_n_filters=32, decoder_ratios=None,
                          decoder_depths=None)
HEAD_DEFAULTS = dict(hidden_size=768, head_layers=4, head_ffn_ratio=3.0, rms_norm_eps=1e-5, latent_size=64,
                     prediction_type="v_prediction", ddpm_num_steps=1000, ddpm_num_inference_steps=20,
                     ddpm_beta_schedule="cosine")


def _depths(d):
    return [int(x) for x in d.split("-")] if isinstance(d, str) else list(d)


class VibeVoiceConfig:
    """Attribute view over the JSON dict, with the derived codec layout."""

    model_type = "vibevoice"     # configuration_vibevoice.py:165
    sub_configs = {}             # read by AutoModelForCausalLM.from_config (no text_config sub-config)

    def __init__(self, d):
        self.raw = copy.deepcopy(d)
        self.decoder_config = _Attr(d["decoder_config"])
        at = dict(TOKENIZER_DEFAULTS, **d.get("acoustic_tokenizer_config", {}))
        st = dict(TOKENIZER_DEFAULTS)
        st.update(vae_dim=128, fix_std=0, std_dist_type="none")
        st.update(d.get("semantic_tokenizer_config", {}))
        self.acoustic_tokenizer_config = _Attr(at)
        self.semantic_tokenizer_config = _Attr(st)
        self.diffusion_head_config = _Attr(dict(HEAD_DEFAULTS, **d.get("diffusion_head_config", {})))
        self.acoustic_vae_dim = at["vae_dim"]
        self.semantic_vae_dim = st["vae_dim"]
        self.torch_dtype = d.get("torch_dtype", "bfloat16")
        self.tie_word_embeddings = d.get("tie_word_embeddings", True)  # PretrainedConfig default

    # codec layout (modular_vibevoice_tokenizer.py:1017-1028, :701)
    @property
    def enc_depths(self):
        return _depths(self.acoustic_tokenizer_config.encoder_depths)

    @property
    def dec_depths(self):
        dd = self.acoustic_tokenizer_config.decoder_depths
        return _depths(dd) if dd is not None else list(reversed(self.enc_depths))

    @property
    def ratios(self):
        t = self.acoustic_tokenizer_config
        return list(t.decoder_ratios or t.encoder_ratios)

    @property
    def hop(self):
        return int(math.prod(self.ratios))

    def to_dict(self):
        return copy.deepcopy(self.raw)

    @classmethod
    def from_json_file(cls, path):
        with open(path) as f:
            return cls(json.load(f))

    @classmethod
    def builtin(cls, name):
        """'1.5B' or 'Large' (vibevoice/configs/*.json, copied as data)."""
        fn = {"1.5B": "qwen2.5_1.5b_64k.json", "Large": "qwen2.5_7b_32k.json"}[name]
        return cls.from_json_file(os.path.join(CONFIG_DIR, fn))


class _Attr(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v
