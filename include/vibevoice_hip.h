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
 *
 * Threading: one vv_ctx per model instance; distinct contexts may be driven
 * from distinct host threads concurrently (each on its own stream) -- every
 * launch plan is a pure function of the call's shapes, and no entry point of
 * this header reads or writes process-wide mutable state except the
 * workspace-epoch counter below (an atomic).  Kernel-level entry points,
 * tuning hooks, timing stamps and benchmark-only switches are NOT part of this
 * interface: they live in vibevoice_hip_diag.h.
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
/* The diffusion head split over the same ranks (SURVEY.md §8e's option for
 * VibeVoice-Large, whose 925 MB of per-step head weights would otherwise be
 * streamed by every rank): the engine was created with head_ffn = this rank's
 * 1/size of the FFN width and bound to its shard (gate|up rows of its hidden
 * columns, column-parallel; the matching down_proj input columns,
 * row-parallel); after each head layer the [2n, H] state is all-reduced
 * (RCCL, sum, bf16, in place; S x head_layers collectives per token), rank 0
 * alone carrying the residual.  adaLN, noisy / cond / final projections and the
 * DPM update stay replicated.
 *   vv_tp_shard_head: mark the engine's head as sharded (after vv_tp_init)
 *   vv_diffusion_sample_group: the group's ranks on ONE device, a device-side
 *                    sum as the all-reduce (tests / single-GPU emulation). */
int vv_tp_shard_head(vv_ctx* ctx, int on);
int vv_diffusion_sample_group(int n_ranks, vv_ctx* const* ctxs, int n, const void* pos_h, const void* neg_h,
                              void* x_io, float cfg_scale, const float* sde_noise, vv_stream st);
/* Copy the K/V cache entry src[i] -> dst[i] of slot slots[i] (all layers). */
int vv_kv_copy(vv_ctx* ctx, int n, const int* slots, const int* src, const int* dst, vv_stream st);
/* embeds_out[i] = embed_tokens[ids[i]] */
int vv_embed(vv_ctx* ctx, int n, const int* ids, void* embeds_out, vv_stream st);

/* n samples: pos_h, neg_h [n, H] conditions; x_io [n, latent] holds the first n
 * rows of the noise draw on entry and the denoised latent on return.
 * sde_noise: NULL for the model's dpmsolver++; for sde-dpmsolver++ the fp32
 * per-step draws [steps][2n][latent] (step()'s randn, dpm_solver.py:985-987). */
int vv_diffusion_sample(vv_ctx* ctx, int n, const void* pos_h, const void* neg_h, void* x_io, float cfg_scale,
                        const float* sde_noise, vv_stream st);
/* Grid-waiting kernels.  Where this context is the device's only one with them
 * enabled, the LM MLP block at B = 1 (k_lm_ffn), each diffusion-head FFN layer
 * at 2 <= 2n <= 16 rows (k_head_m16) and the codec's C = 2,048 / 1,024 stages
 * of one sample (k_codec_stage*) each run as ONE launch of one workgroup per CU
 * whose workgroups wait for each other inside the launch (bounded, ~200 ms;
 * the occupancy query must show the whole grid co-resident, else the GEMV
 * launches run).  If a wait ever gave up (workgroups not co-resident, e.g.
 * another process's kernels holding CUs), every output since is invalid:
 * vv_sync_error returns 1 (and resets the counters), else 0; it synchronises
 * the device.  vv_sync_error_async is its stream-ordered form: it enqueues on
 * st a copy of the error word into dst (4 bytes of pinned host or device
 * memory) and the word's reset, so a host that reads dst after an event
 * recorded behind it sees every launch queued before the call; a host that
 * reads 1 must call vv_sync_reset (synchronises; zeroes every wait counter of
 * the context) before launching again.  GenerateSession reads it with every
 * step's logits read-back and before the step's audio leaves for a streamer
 * (step() raises; no invalid chunk is put).
 * vv_set_persistent(ctx, 0) turns the grid-waiting kernels off for ctx (the
 * process default is on unless the environment sets VIBEVOICE_PERSISTENT=0):
 * for GPUs shared by several processes, whose contexts this library cannot
 * see.  vv_set_persistent(ctx, 2) ("follow"): ctx does not register, and runs
 * the kernels while exactly one context of the device is registered -- a second
 * context over the same model (the standalone tokenizer API's codec slots) then
 * computes with the owner's kernels, bit-identically, without demoting it; the
 * two must not launch concurrently on different streams. */
int vv_set_persistent(vv_ctx* ctx, int on);
/* 1 when ctx launches its grid-waiting kernels now (enabled, sole context). */
int vv_persistent_active(vv_ctx* ctx);
int vv_sync_reset(vv_ctx* ctx);
int vv_sync_error(vv_ctx* ctx);
int vv_sync_error_async(vv_ctx* ctx, void* dst, vv_stream st);

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

/* Non-streaming semantic encoder (semantic_tokenizer.encode(audio) without a
 * cache, modular_vibevoice_tokenizer.py:1171-1175; each strided conv right-pads
 * its input to whole strides, :127-133 / :393-408): audio [nv, L] bf16 ->
 * mean_out [nv, ceil(L/hop), semantic_dim] bf16; L need not be whole frames. */
int vv_semantic_encode(vv_ctx* ctx, int nv, int L, const void* audio, void* mean_out, vv_stream st);

/* z = mean + std[v]*noise; feat = (z + bias) * scale   (rows = nv * frames) */
int vv_vae_features(vv_ctx* ctx, int nv, int frames, const void* mean, const void* stdv, const void* noise,
                    void* feat_out, vv_stream st);

/* which: 0 = acoustic connector (in = latent), 1 = semantic connector. */
int vv_connector(vv_ctx* ctx, int which, int n, const void* x, void* out, vv_stream st);

/* dst[idx[i]] = src[i] for bf16 rows of C elements (row strides in elements). */
int vv_scatter_rows(vv_ctx* ctx, int n, int C, const void* src, int64_t lds, const int* idx, void* dst,
                    int64_t ldd, vv_stream st);

#ifdef __cplusplus
}
#endif
#endif
