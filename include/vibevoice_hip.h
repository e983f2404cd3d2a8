/*
 * vibevoice_hip.h — C ABI of libvibevoice_hip.so, the MI355X (gfx950) engine
 * behind VibeVoice's next-token-diffusion generate loop.
 *
 * The reference has no FFI: its hot path sits behind the Hugging Face plugin
 * surface (AutoModelForCausalLM.register + .generate(),
 * vibevoice/modular/modeling_vibevoice_inference.py:327-710, :728).  The Python
 * host in vibevoice_amd/ keeps that surface and calls these entry points for
 * every piece of arithmetic of the loop body:
 *
 *   vv_lm_forward        <- self(...) positive pass :483-486 and negative pass
 *                           :598-600 (Qwen2 decode, batched as one set of rows),
 *                           and the prompt prefill :468-486 / :222-238
 *   vv_diffusion_sample  <- sample_speech_tokens :712-725 (+ prediction_head,
 *                           modular_vibevoice_diffusion_head.py:254-280, and
 *                           DPMSolverMultistepScheduler.step, dpm_solver.py:935)
 *   vv_codec_step        <- acoustic_tokenizer.decode :651-658, semantic_tokenizer
 *                           .encode :673-679, acoustic/semantic connectors :682-687
 *   vv_codec_reset       <- acoustic_cache/semantic_cache.set_to_zero :557-560
 *   vv_codec_decode /    <- acoustic_tokenizer.decode / semantic_tokenizer.encode with a
 *   vv_codec_encode /       VibeVoiceTokenizerStreamingCache (modular_vibevoice_tokenizer.py
 *   vv_codec_reset_net      :1081-1108, :193-256), the standalone codec API
 *   vv_acoustic_encode   <- _process_speech_inputs encode :150-164 (voice prompt)
 *   vv_connector         <- SpeechConnector.forward (modeling_vibevoice.py:58-69)
 *
 * Conventions: all tensor arguments are caller-owned DEVICE pointers (bf16 =
 * 2-byte bfloat16, int = int32) with explicit sizes; weights are borrowed (the
 * caller keeps them alive).  Every call is asynchronous on the caller's stream.
 * Return value 0 = ok; otherwise vv_last_error() (thread-local) describes it.
 */
#ifndef VIBEVOICE_HIP_H
#define VIBEVOICE_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vv_ctx vv_ctx;
typedef void* vv_stream; /* hipStream_t */

#define VV_MAX_STAGES 8

typedef struct vv_config {
  /* Qwen2 decoder (vibevoice/configs/qwen2.5_1.5b_64k.json decoder_config) */
  int hidden, n_layers, n_heads, n_kv_heads, head_dim, intermediate;
  float rms_eps, rope_theta;
  /* diffusion head (diffusion_head_config) */
  int head_layers, head_ffn, latent_dim;
  float head_eps;
  /* σ-VAE codec (acoustic_tokenizer_config / semantic_tokenizer_config) */
  int n_stages;                    /* len(depths) */
  int ratios[VV_MAX_STAGES];       /* decoder order: [8,5,5,4,2,2] */
  int dec_depths[VV_MAX_STAGES];   /* [8,3,3,3,3,3,3] */
  int enc_depths[VV_MAX_STAGES];   /* [3,3,3,3,3,3,8] */
  int dec_n_filters, sem_n_filters, ac_enc_n_filters;
  int semantic_dim;                /* 128 */
  float codec_eps;
  /* capacity */
  int max_batch;                   /* samples (LM rows = 2 * max_batch) */
  int max_ctx;                     /* KV positions per LM row */
} vv_config;

const char* vv_last_error(void);
/* Counter of workspace reallocations (any ctx of the process).  A workspace
 * grows when a call needs more than any earlier one (e.g. a longer prefill);
 * device pointers captured into a hipGraph before that are stale, so a host
 * that replays graphs re-captures them when this value changes. */
int vv_ws_epoch(void);
int vv_create(const vv_config* cfg, int device, vv_ctx** out);
void vv_destroy(vv_ctx* ctx);

/* Borrow a device weight under an engine name (see vibevoice_amd/weights.py
 * for the name list and the packing applied to the reference's tensors). */
int vv_bind_weight(vv_ctx* ctx, const char* name, const void* dev_ptr, const int64_t* shape, int ndim);
/* Check every required weight is bound; allocate KV / codec state / workspaces. */
int vv_finalize(vv_ctx* ctx);

/* ids of the constrained vocabulary (speech_start, speech_end, diffusion, eos). */
int vv_set_valid_ids(vv_ctx* ctx, int n, const int* host_ids);

/* Diffusion schedule for `steps` steps.  coef: host float[steps * 8] =
 * {alpha_s, sigma_s, c_x, c_d0, c_d1, inv_r0, order, 0} per step; tfreq: device
 * bf16[steps, 256] sinusoidal timestep features. */
int vv_set_schedule(vv_ctx* ctx, int steps, const float* coef, const void* tfreq, vv_stream st);

/* Token rows through the Qwen2 decoder.  Token i reads embedding row
 * i % embed_rows of embeds (embed_rows <= 0: ntok), has KV slot slot[i] and
 * position pos[i]; its K/V are written at cache index pos[i] of that slot and
 * it attends to cache entries [0, pos[i]].  max_pos_p1 = 1 + max(pos).
 * For the nout rows listed in out_idx the final-norm hidden state is written to
 * hidden_out[nout, H] and the valid-id logits to logits_out[nout, n_valid]. */
int vv_lm_forward(vv_ctx* ctx, int ntok, const void* embeds, int embed_rows, const int* slot, const int* pos,
                  int max_pos_p1,
                  int nout, const int* out_idx, void* hidden_out, float* logits_out, vv_stream st);

/* Tensor parallelism of the Qwen2 backbone (Megatron split declared at
 * configuration_vibevoice.py:175-183: q/k/v/gate/up column-parallel, o/down
 * row-parallel).  The engine is created with its rank's LOCAL head /
 * intermediate counts and bound to its shard of the weights; the residual
 * stream is all-reduced (RCCL, sum, bf16, in place) after o_proj and down_proj,
 * rank 0 alone carrying the residual into the sum.
 *   vv_tp_unique_id: ncclGetUniqueId into out (returns its size)
 *   vv_tp_init:      rank / size; unique_id NULL = no communicator (a
 *                    single-process group driven by vv_lm_forward_group)
 *   vv_lm_forward_group: the ranks of one group on ONE device, interleaved
 *                    layer by layer with a device-side sum as the all-reduce
 *                    (tests / single-GPU emulation); outputs from rank 0. */
int vv_tp_unique_id(void* out, int nbytes);
int vv_tp_init(vv_ctx* ctx, int rank, int size, const void* unique_id);
int vv_lm_forward_group(int n, vv_ctx* const* ctxs, int ntok, const void* embeds, int embed_rows, const int* slot,
                        const int* pos, int max_pos_p1, int nout, const int* out_idx, void* hidden_out,
                        float* logits_out, vv_stream st);
/* Switch (benchmarks only): 1 = skip the RCCL all-reduces of communicator
 * engines (outputs wrong), so bench.py --tp can time an LM pass with and
 * without its 2 x n_layers collectives and report their share. */
int vv_tp_null_collective(int on);

/* Copy the K/V cache entry src[i] -> dst[i] of slot slots[i] (all layers). */
int vv_kv_copy(vv_ctx* ctx, int n, const int* slots, const int* src, const int* dst, vv_stream st);
/* Benchmarks only: fill the KV cache of `slots` at
 * positions [p0, p1) with deterministic pseudo-random values, so decode can be
 * timed at a long context without a long prefill.  Not a reference operation. */
int vv_kv_synthetic(vv_ctx* c, int n, const int* slots, int p0, int p1, unsigned seed, vv_stream stream);

/* embeds_out[i] = embed_tokens[ids[i]] */
int vv_embed(vv_ctx* ctx, int n, const int* ids, void* embeds_out, vv_stream st);

/* n samples: pos_h, neg_h [n, H] conditions; x_io [n, latent] holds the first n
 * rows of the noise draw on entry and the denoised latent on return.
 * sde_noise: NULL for the model's dpmsolver++; for sde-dpmsolver++ the fp32
 * per-step draws [steps][2n][latent] (step()'s randn, dpm_solver.py:985-987). */
int vv_diffusion_sample(vv_ctx* ctx, int n, const void* pos_h, const void* neg_h, void* x_io, float cfg_scale,
                        const float* sde_noise, vv_stream st);

/* One streaming codec step for n samples in codec slots slots[n]:
 * latent [n, latent] -> audio_out [n, hop]; semantic features -> sem_out
 * [n, semantic_dim] (may be NULL); acoustic_connector(latent) +
 * semantic_connector(sem) -> row embed_rows[i] of embeds_out [*, H]. */
int vv_codec_step(vv_ctx* ctx, int n, const int* slots, const void* latent, void* audio_out, void* sem_out,
                  void* embeds_out, const int* embed_rows, vv_stream st);
int vv_codec_reset(vv_ctx* ctx, int n, const int* slots, vv_stream st);

/* The standalone tokenizer API, one frame per call on codec slots slots[n]
 * (replaces acoustic_tokenizer.decode(latents, cache, sample_indices,
 * use_cache=True) and semantic_tokenizer.encode(audio, cache, ...),
 * modular_vibevoice_tokenizer.py:1081-1108, with VibeVoiceTokenizerStreamingCache
 * :193-256 as the per-slot state):
 *   vv_codec_decode: z [n, latent] (the decoder input, already scaled) -> audio_out [n, hop]
 *   vv_codec_encode: audio [n, hop] -> sem_out [n, semantic_dim]
 *   vv_codec_reset_net: set_to_zero of one net's state (0 = acoustic decoder,
 *                       1 = semantic encoder). */
int vv_codec_decode(vv_ctx* ctx, int n, const int* slots, const void* z, void* audio_out, vv_stream st);
int vv_codec_encode(vv_ctx* ctx, int n, const int* slots, const void* audio, void* sem_out, vv_stream st);
int vv_codec_reset_net(vv_ctx* ctx, int net, int n, const int* slots, vv_stream st);

/* Non-streaming acoustic encoder over nv voice prompts of L samples (zero
 * padded): audio [nv, L] bf16 -> mean_out [nv, ceil(L/hop), latent] bf16. */
int vv_acoustic_encode(vv_ctx* ctx, int nv, int L, const void* audio, void* mean_out, vv_stream st);

/* z = mean + std[v]*noise; feat = (z + bias) * scale   (rows = nv * frames) */
int vv_vae_features(vv_ctx* ctx, int nv, int frames, const void* mean, const void* stdv, const void* noise,
                    void* feat_out, vv_stream st);

/* which: 0 = acoustic connector (in = latent), 1 = semantic connector. */
int vv_connector(vv_ctx* ctx, int which, int n, const void* x, void* out, vv_stream st);

/* dst[idx[i]] = src[i] for bf16 rows of C elements (row strides in elements). */
int vv_scatter_rows(vv_ctx* ctx, int n, int C, const void* src, int64_t lds, const int* idx, void* dst,
                    int64_t ldd, vv_stream st);

/* Low-level kernel entry points (used by the parity tests).  W is [N, K] in the
 * MFMA-packed order of vibevoice_amd/weights.py:mfma_pack (csrc/gemm.hip). */
int vv_gemm_bf16(int M, int N, int K, const void* A, int64_t lda, const void* W, const void* bias, int epi,
                 void* Y, int64_t ldy, const void* res, const void* gamma, vv_ctx* ws_ctx, vv_stream st);
/* The same with the A operand RMS-normalised on load (x * rsqrt(mean(x^2) + eps),
 * bf16, times norm_w when not NULL): the fused input_layernorm / ConvRMSNorm
 * producer of the loop's GEMMs (no bias / residual epilogues). */
int vv_gemm_bf16_norm(int M, int N, int K, const void* A, int64_t lda, const void* norm_w, float eps, const void* W,
                      int epi, void* Y, int64_t ldy, vv_ctx* ws_ctx, vv_stream st);
/* GQA attention of nq query rows (q [nq, nh*128] bf16, RoPE applied) over a
 * caller-owned cache in the engine layout ([slot][kv_head][ctx][128], strides
 * in elements): row i attends keys [0, pos[i]] of slot slots[i] -> out
 * [nq, nh*128].  max_pos_p1 bounds pos + 1 (launch plan); ws_ctx supplies the
 * split-merge workspace.  (Kernel entry for tests / benchmarks.) */
int vv_attention_bf16(int nq, int nh, int nkv, const void* q, const void* k_cache, const void* v_cache,
                      int64_t s_slot, int64_t s_head, const int* slots, const int* pos, int max_pos_p1, void* out,
                      vv_ctx* ws_ctx, vv_stream st);
/* Tuning hook (benchmarks only): override the GEMV launch plan — waves per
 * workgroup, split-K workgroups, split-K hand-off form (0 fences, 1 sc1),
 * target waves per launch, weight chunks in flight per wave (2/4/8).
 * 0 / -1 restore the built-in plan. */
int vv_gemv_tune(int nw, int ks, int handoff, int target_waves, int u);
/* Tuning hook (benchmarks only): 16-row weight tiles per workgroup of the
 * M <= 16 GEMV (the waves split into tpw groups that share one staging of the
 * A rows); 0 restores the built-in plan. */
int vv_gemv_tune_tpw(int tpw);
/* Tuning hook (benchmarks only): GEMMs with more than m rows (m >= 16) use the
 * tiled MFMA kernel instead of the GEMV family; 0 restores the built-in 64. */
int vv_gemv_tune_maxm(int m);
/* Tuning hook (benchmarks only): 0 = the 16 < M <= 64 GEMVs with >= 256 tiles
 * use k_gemv (A fragments per tile) instead of k_gemvw (A held per K slice
 * across several tiles); 1 = built-in. */
int vv_gemv_tune_wide(int on);
/* Tuning hook (benchmarks only): the largest dynamic LDS (bytes) the M <= 16
 * GEMV may stage its A slice in before it falls back to per-wave A fragment
 * loads, up to 148 KiB (per-kernel opt-in above 64 KB); 0 = built-in (64 KB). */
int vv_gemv_tune_lds(int bytes);
/* Tuning hook (benchmarks only): fused-RMSNorm GEMVs with at least min_m rows
 * (and an eligible shape) stage whole A rows per wave (k_gemv1's RW form: the
 * norm applied in registers, one barrier); 0 restores the built-in 1; -1 = the
 * built-in without the LDS-DMA form for K = 3,584 adaLN rows; 99 = off. */
int vv_gemv_tune_rw(int min_m);
/* Host-only plan query (no device work; tests and tools): the kernel form and
 * launch plan the library uses for an M <= 16 GEMV (xf: 0 none, 1 RMSNorm, 2
 * SiLU-add; has_w / has_mod: norm weight, adaLN shift / scale present).
 * out[7] = {kernel (0 = A staged in LDS, 1 = A fragments from L2), waves, K
 * splits, weight chunks in flight, tiles per workgroup, norm prologue form
 * (0 item per thread, 1 row per wave, 2 row per wave + LDS-DMA rows), dynamic
 * LDS bytes}. Replaces nothing in the reference (the plan is this engine's). */
int vv_gemv_plan(int M, int N, int K, int xf, int has_w, int has_mod, int* out);
/* Tuning hook (benchmarks / tests): XF-free GEMMs with >= 256 rows,
 * N % 128 == 0, K % 64 == 0 and >= 256 such tiles (or >= 2^30 MACs) take the
 * LDS-staged 128 x 128 tile (k_gemm_big, the prefill projections) with 2 LDS
 * stages (-1 / 2 = built-in) or 1 stage (1); 0 = they stay on k_gemm;
 * + 4 = any tile count (tests). */
int vv_gemm_tune_big(int mode);
/* Diagnostic (benchmarks only): M <= 16 GEMV launches write 4 s_memrealtime
 * stamps per workgroup (start, A staged, weights streamed, epilogue stored) to
 * buf (uint64[grid * 4]); NULL turns it off. */
int vv_gemv_stamps(void* buf);
/* Diagnostic (benchmarks only): vv_attention_bf16 launches write 4 stamps per
 * workgroup (start, K/V/Q landed, keys done, output stored); NULL: off. */
int vv_attn_stamps(void* buf);
/* Tuning hook (benchmarks only): attention keys per split (multiple of 32;
 * 0 = built-in) and the largest split count merged inside the attention
 * kernel (more splits go to the separate merge pass; -1 = built-in). */
int vv_attn_tune(int chunk, int merge_in);
/* Tuning hook (benchmarks / tests): the attention kernel for many query rows
 * per slot (prompt prefill): -1 = built-in choice (>= 256 rows and >= 32 rows
 * per slot of the engine -> the 32-row-tile prefill kernel), 0 = always the
 * per-row decode kernel, 1 = always the prefill kernel. */
int vv_attn_prefill(int mode);
/* Switch (benchmarks / tests): persistent GEMV chains (chain.hip) -- the
 * diffusion head's S steps run as ONE launch of one workgroup per CU instead of
 * S x (2 + 2L) GEMV launches.  0 (default, -1) = per-op launches; 1 = chains
 * with the balanced work split; 2 = chains with the per-op launch plan mirrored
 * (bit-identical to 0, the hand-off test).  Measured slower than 0 on MI355X
 * (DESIGN.md "Persistent chains"), so off by default. */
int vv_chain_tune(int mode);
/* Tuning hook (benchmarks only): weight chunks per wave per load batch of the
 * chain kernel (4 or 8 = built-in). */
int vv_chain_tune_u(int u);
/* Diagnostic: nonzero (1 + op index) if a chain launch's dependency wait gave
 * up (a producer never signalled within ~200 ms); reading resets it. */
int vv_chain_error(vv_ctx* c);
/* Diagnostic (benchmarks only): chain launches write s_memrealtime stamps per
 * (workgroup, op): wait begun, inputs ready, op signalled (uint64[G][nops][4]);
 * NULL: off. */
int vv_chain_stamps(void* buf);
/* Diagnostic (benchmarks only): vv_gemm_bf16 reads A in MFMA-fragment order
 * (as the packed weights; the 256 x 256 tile only). */
int vv_gemm_tune_apack(int on);
/* Tuning hook (benchmarks only): override the GEMV plan (waves, K splits, chunks
 * in flight, tiles per workgroup) for one weight shape N x K at M <= mmax rows;
 * up to 8 overrides; N <= 0 clears them. */
int vv_gemv_tune_shape(int N, int K, int mmax, int nw, int ks, int u, int tpw);
/* Test switch: 1 (default) = the q|k|v RoPE epilogue reads the engine's
 * per-position bf16 cos / sin table; 0 = computes cosf / sinf inline
 * (bit-identical by construction). */
int vv_rope_table(int on);
/* Test switch: on = 1 (default, chunk 128): decode passes of <= 4 rows over up
 * to 8,192 keys run 2..8 key splits of >= `chunk` keys (multiple of 32) and
 * leave their partials to o_proj, which merges them while staging its A rows
 * (bit-identical to the same splits merged in the attention kernel); on = n >= 2:
 * passes of <= n rows (n <= 16); 0 = the attn_plan splits everywhere. */
int vv_attn_defer(int on, int chunk);
/* Test switch: 1 (default) = the A rows of the prefill's 256 x 256-tile GEMMs
 * are written MFMA-fragment-packed by their producers (RMSNorm rows for q|k|v
 * and gate|up, gate|up's SiLU*up rows for down); 0 = row-major.  Both give the
 * same bits. */
int vv_norm_pack(int on);
/* Test switch (bit mask, default 3): bit 0 folds each codec Block1D's mixer
 * (norm, depthwise conv, gamma residual, FFN norm) into its fc1 GEMV where
 * <= 16 rows fit (XF_MIX); bit 1 runs whole narrow-stage blocks (C <= 128) as
 * one k_block launch.  0 = separate k_mix + GEMM launches everywhere.  Every
 * mask gives the same bits. */
int vv_codec_mix_fusion(int mask);
int vv_rmsnorm_bf16(int M, int C, const void* x, int64_t ldx, const void* w, float eps, void* y, int64_t ldy,
                    vv_stream st);

#ifdef __cplusplus
}
#endif
#endif
