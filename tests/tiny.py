"""A small but structurally complete VibeVoice config for GPU tests.

LM hidden = diffusion-head hidden = 128 (the committed g2_head.npz golden's
width), 1 q / 1 kv head of 128, two layers; codec with hop 4 (ratios [2, 2]),
one block per stage, 32 filters so every conv maps onto the HIP GEMM shapes.
"""
import copy

from vibevoice_amd.config import VibeVoiceConfig


def tiny_dict(hidden=128, layers=2, heads=1, kv_heads=1, inter=384, vocab=151936, ratios=(2, 2),
              depths="1-1-1", nf=32):
    tok = dict(causal=True, channels=1, conv_bias=True, conv_norm="none", disable_last_norm=True,
               encoder_depths=depths, encoder_n_filters=nf, decoder_n_filters=nf, encoder_ratios=list(ratios),
               decoder_ratios=list(ratios), layer_scale_init_value=1e-6, layernorm="RMSNorm",
               layernorm_elementwise_affine=True, layernorm_eps=1e-5, mixer_layer="depthwise_conv",
               pad_mode="constant", weight_init_value=0.01)
    return {
        "acoustic_vae_dim": 64,
        "acoustic_tokenizer_config": dict(tok, vae_dim=64, fix_std=0.5, std_dist_type="gaussian"),
        "semantic_tokenizer_config": dict(tok, vae_dim=128, fix_std=0, std_dist_type="none"),
        "decoder_config": dict(hidden_size=hidden, intermediate_size=inter, num_hidden_layers=layers,
                               num_attention_heads=heads, num_key_value_heads=kv_heads, head_dim=128,
                               max_position_embeddings=4096, rms_norm_eps=1e-6, rope_theta=1e6,
                               vocab_size=vocab, tie_word_embeddings=True, model_type="qwen2"),
        "diffusion_head_config": dict(hidden_size=hidden, head_layers=4, head_ffn_ratio=3.0, rms_norm_eps=1e-5,
                                      latent_size=64, prediction_type="v_prediction", ddpm_num_steps=1000,
                                      ddpm_num_inference_steps=10, ddpm_beta_schedule="cosine"),
        "semantic_vae_dim": 128,
        "torch_dtype": "bfloat16",
    }


def tiny_config(**kw):
    return VibeVoiceConfig(copy.deepcopy(tiny_dict(**kw)))
