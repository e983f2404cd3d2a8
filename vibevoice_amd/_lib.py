"""ctypes binding of libvibevoice_hip.so (C ABI: include/vibevoice_hip.h).

The product path has no fallback: if the library is missing or fails to load,
every entry point raises.  Build it with `make -C vibevoice_amd/csrc` (or
`__graft_entry__.build()`).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvibevoice_hip.so")

VV_MAX_STAGES = 8


class VVConfig(ctypes.Structure):
    _fields_ = [
        ("hidden", ctypes.c_int), ("n_layers", ctypes.c_int), ("n_heads", ctypes.c_int),
        ("n_kv_heads", ctypes.c_int), ("head_dim", ctypes.c_int), ("intermediate", ctypes.c_int),
        ("rms_eps", ctypes.c_float), ("rope_theta", ctypes.c_float),
        ("head_layers", ctypes.c_int), ("head_ffn", ctypes.c_int), ("latent_dim", ctypes.c_int),
        ("head_eps", ctypes.c_float),
        ("n_stages", ctypes.c_int), ("ratios", ctypes.c_int * VV_MAX_STAGES),
        ("dec_depths", ctypes.c_int * VV_MAX_STAGES), ("enc_depths", ctypes.c_int * VV_MAX_STAGES),
        ("dec_n_filters", ctypes.c_int), ("sem_n_filters", ctypes.c_int), ("ac_enc_n_filters", ctypes.c_int),
        ("semantic_dim", ctypes.c_int), ("codec_eps", ctypes.c_float),
        ("max_batch", ctypes.c_int), ("max_ctx", ctypes.c_int),
    ]


# (name, restype, argtypes) of every exported entry point
P, I, F, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
EXPORTS = [
    ("vv_last_error", ctypes.c_char_p, []),
    ("vv_create", I, [ctypes.POINTER(VVConfig), I, ctypes.POINTER(P)]),
    ("vv_destroy", None, [P]),
    ("vv_bind_weight", I, [P, ctypes.c_char_p, P, ctypes.POINTER(I64), I]),
    ("vv_finalize", I, [P]),
    ("vv_set_valid_ids", I, [P, I, ctypes.POINTER(I)]),
    ("vv_set_schedule", I, [P, I, ctypes.POINTER(F), P, P]),
    ("vv_lm_forward", I, [P, I, P, I, P, P, I, I, P, P, P, P]),
    ("vv_kv_copy", I, [P, I, P, P, P, P]),
    ("vv_kv_synthetic", I, [P, I, P, I, I, ctypes.c_uint, P]),
    ("vv_tp_unique_id", I, [P, I]),
    ("vv_tp_init", I, [P, I, I, P]),
    ("vv_tp_null_collective", I, [I]),
    ("vv_lm_forward_group", I, [I, ctypes.POINTER(P), I, P, I, P, P, I, I, P, P, P, P]),
    ("vv_tp_shard_head", I, [P, I]),
    ("vv_diffusion_sample_group", I, [I, ctypes.POINTER(P), I, P, P, P, F, P, P]),
    ("vv_embed", I, [P, I, P, P, P]),
    ("vv_diffusion_sample", I, [P, I, P, P, P, F, P, P]),
    ("vv_codec_step", I, [P, I, P, P, P, P, P, P, P]),
    ("vv_codec_reset", I, [P, I, P, P]),
    ("vv_codec_decode", I, [P, I, P, P, P, P]),
    ("vv_codec_encode", I, [P, I, P, P, P, P]),
    ("vv_codec_reset_net", I, [P, I, I, P, P]),
    ("vv_acoustic_encode", I, [P, I, I, P, P, P]),
    ("vv_semantic_encode", I, [P, I, I, P, P, P]),
    ("vv_vae_features", I, [P, I, I, P, P, P, P, P]),
    ("vv_connector", I, [P, I, I, P, P, P]),
    ("vv_scatter_rows", I, [P, I, I, P, I64, P, P, I64, P]),
    ("vv_gemm_bf16", I, [I, I, I, P, I64, P, P, I, P, I64, P, P, P, P]),
    ("vv_rmsnorm_bf16", I, [I, I, P, I64, P, F, P, I64, P]),
    ("vv_gemm_bf16_norm", I, [I, I, I, P, I64, P, F, P, I, P, I64, P, P]),
    ("vv_attention_bf16", I, [I, I, I, P, P, P, I64, I64, P, P, I, P, P, P]),
    ("vv_ws_epoch", I, []),
    ("vv_gemv_tune", I, [I, I, I, I, I]),
    ("vv_gemv_tune_tpw", I, [I]),
    ("vv_gemv_tune_maxm", I, [I]),
    ("vv_gemv_tune_wide", I, [I]),
    ("vv_gemv_tune_lds", I, [I]),
    ("vv_gemv_tune_rw", I, [I]),
    ("vv_gemv_plan", I, [I, I, I, I, I, I, P]),
    ("vv_gemm_tune_big", I, [I]),
    ("vv_gemv_stamps", I, [P]),
    ("vv_attn_stamps", I, [P]),
    ("vv_attn_tune", I, [I, I]),
    ("vv_attn_prefill", I, [I]),
    ("vv_codec_mix_fusion", I, [I]),
    ("vv_codec_stage", I, [I]),
    ("vv_codec_tile", I, [I]),
    ("vv_codec_tile_stamps", I, [P]),
    ("vv_codec_wide", I, [I]),
    ("vv_codec_wide_over", I, [I]),
    ("vv_codec_wide_active", I, [P, I]),
    ("vv_codec_wide_stamps", I, [P]),
    ("vv_head_m16", I, [I]),
    ("vv_head_m16_active", I, [P, I]),
    ("vv_head_m16_stamps", I, [P]),
    ("vv_lm_ffn", I, [I]),
    ("vv_lm_ffn_active", I, [P, I]),
    ("vv_lm_ffn_stamps", I, [P]),
    ("vv_head_fin", I, [I]),
    ("vv_head_fin_active", I, [P, I]),
    ("vv_lm_attn", I, [I]),
    ("vv_lm_attn_active", I, [P, I, I]),
    ("vv_lm_attn_stamps", I, [P]),
    ("vv_lm_attn_replay", I, [P, I, P, P, P, I, I, P]),
    ("vv_lm_mlp_replay", I, [P, I, P, P, I, P]),
    ("vv_head_m16_pre", I, [I]),
    ("vv_attn_defer_max", I, [I]),
    ("vv_codec_stage_active", I, [P]),
    ("vv_codec_stage_stamps", I, [P, I]),
    ("vv_gemm_tune_apack", I, [I]),
    ("vv_gemv_tune_shape", I, [I, I, I, I, I, I, I]),
    ("vv_rope_table", I, [I]),
    ("vv_attn_defer", I, [I, I]),
    ("vv_attn_group", I, [I]),
    ("vv_attn_pass_plan", I, [I, I, I, I, I, ctypes.POINTER(I)]),
    ("vv_gemv_tune_bal", I, [I]),
    ("vv_head_layers_replay", I, [P, I, P, P, I, P]),
    ("vv_sync_error", I, [P]),
    ("vv_sync_error_async", I, [P, P, P]),
    ("vv_diag_raise_sync_error", I, [P]),
    ("vv_diag_sync_words", I, [P, P]),
    ("vv_sync_reset", I, [P]),
    ("vv_set_persistent", I, [P, I]),
    ("vv_persist_decision", I, [I, I, I, I, I, I]),
    ("vv_persistent_active", I, [P]),
    ("vv_norm_pack", I, [I]),
]

EPI = {"store": 0, "gelu": 1, "silu_mul": 2, "res": 3, "f32": 4}

_lib = None


def lib():
    """Load (once) and return the library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run `make -C vibevoice_amd/csrc` (HIP path has no fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in EXPORTS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what=""):
    if rc != 0:
        msg = lib().vv_last_error().decode(errors="replace")
        raise RuntimeError(f"libvibevoice_hip {what}: {msg}")
