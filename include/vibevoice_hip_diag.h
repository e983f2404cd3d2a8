/*
 * vibevoice_hip_diag.h — diagnostics of libvibevoice_hip.so: kernel-level entry
 * points (parity tests, benchmarks), launch-plan tuning hooks, per-workgroup
 * timing stamps and benchmark-only switches.  NOT the product interface
 * (include/vibevoice_hip.h is): nothing in vibevoice_amd/ calls these, and the
 * reference has nothing they replace.
 *
 * The hooks set PROCESS-WIDE state (std::atomic words read by every launch of
 * every context): set them only while no other thread is launching work, and
 * restore the built-in value (0 / -1 as documented) afterwards.  Tests use them
 * to pin alternative forms bit-identical to the default; tools/ uses them for
 * same-box A/B runs.
 */
#ifndef VIBEVOICE_HIP_DIAG_H
#define VIBEVOICE_HIP_DIAG_H
#include <stdint.h>

#include "vibevoice_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Switch (benchmarks only): 1 = skip the RCCL all-reduces of communicator
 * engines (outputs wrong), so bench.py --tp can time an LM pass with and
 * without its 2 x n_layers collectives and report their share. */
int vv_tp_null_collective(int on);

/* Benchmarks only: fill the KV cache of `slots` at
 * positions [p0, p1) with deterministic pseudo-random values, so decode can be
 * timed at a long context without a long prefill.  Not a reference operation. */
int vv_kv_synthetic(vv_ctx* c, int n, const int* slots, int p0, int p1, unsigned seed, vv_stream stream);

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
/* Diagnostic (benchmarks only): vv_gemm_bf16 reads A in MFMA-fragment order
 * (as the packed weights; the 256 x 256 tile only). */
int vv_gemm_tune_apack(int on);
/* Tuning hook (benchmarks only): override the GEMV plan (waves, K splits, chunks
 * in flight, tiles per workgroup) for one weight shape N x K at M <= mmax rows;
 * up to 8 overrides; N <= 0 clears them. */
/* Test / A-B switch: 1 (default) = at 4 < 2n <= 16 rows each head FFN layer
 * is one launch with one grid-wide hand-off (head_m16.hip; within bf16 of the
 * GEMV pair, not bitwise) while ctx is the device's only registered context;
 * 0 = gate|up + down GEMV launches. */
int vv_head_m16(int on);
/* Test query: 1 when a head layer of n samples on ctx would run head_m16 now. */
int vv_head_m16_active(vv_ctx* ctx, int n);
/* Diagnostic: per-workgroup s_memrealtime stamps of every head_m16 launch into
 * buf ([256][16] u64, overwritten per launch; NULL = off). */
int vv_head_m16_stamps(void* buf);
/* Diagnostic switch: the LM MLP block at decode with <= 2 rows as one launch
 * (lm_ffn.hip; 1, default) or the gate|up + down GEMV pair (0); and whether
 * the one-launch block applies to this context at ntok rows. */
int vv_lm_ffn(int on);
int vv_lm_ffn_active(vv_ctx* ctx, int ntok);
/* Diagnostic: k_lm_ffn16 launches write per-workgroup phase stamps ([256][16]
 * u64, overwritten per launch; NULL = off). */
int vv_lm_ffn_stamps(void* buf);
/* Diagnostic switch: the LM attention half at decode (input_layernorm .. o_proj
 * + residual, <= 16 rows, contexts <= 4,096 keys) as one launch (lm_attn.hip;
 * 1, default) or the q|k|v, attention and o_proj launches (0); whether it applies
 * to this context at ntok rows over max_pos_p1 keys; and per-workgroup phase
 * stamps of its launches ([256][16] u64, overwritten per launch; NULL = off). */
/* Diagnostic switch: the diffusion head's step boundary (final layer + DPM of
 * step s, noisy projection of step s + 1) as one launch at 2n <= 4 rows
 * (head_fin.hip; 1, default) or the two GEMV launches (0); and whether it
 * applies to this context at n samples. */
int vv_head_fin(int on);
int vv_head_fin_active(vv_ctx* ctx, int n);
int vv_lm_attn(int on);
int vv_lm_attn_active(vv_ctx* ctx, int ntok, int max_pos_p1);
int vv_lm_attn_stamps(void* buf);
/* Diagnostic (bench.py): `reps` passes over the LM layers' attention halves alone
 * on ntok decode rows (embeds [ntok][H] as layer 0's input, slots / positions as
 * for vv_lm_forward). */
int vv_lm_attn_replay(vv_ctx* ctx, int ntok, const void* embeds, const int* slot, const int* pos, int max_pos_p1,
                      int reps, vv_stream stream);
/* Diagnostic (bench.py): `reps` passes over the LM layers' MLP blocks alone on
 * ntok decode rows (hidden [ntok][H] in place, act [ntok][I] scratch). */
int vv_lm_mlp_replay(vv_ctx* ctx, int ntok, void* hidden, void* act, int reps, vv_stream stream);
/* Diagnostic switch: head layers l >= 1 at 4 < 2n <= 16 rows build their A side
 * distributed from the previous layer's row partials (1, default) or transform
 * it whole in every workgroup (0). */
int vv_head_m16_pre(int on);
/* Diagnostic (bench.py): the head's condition rows and step-0 modulations for
 * n samples, then `reps` passes over its FFN layers alone (the kernels the loop
 * runs for them at this n), asynchronously on st. */
int vv_head_layers_replay(vv_ctx* ctx, int n, const void* pos_h, const void* neg_h, int reps, vv_stream st);
/* Test hook: raise the engine's grid-wait error word as a wait that gave up
 * would, and leave its wait counters part-advanced as such a launch does
 * (synchronises the device first). */
int vv_diag_raise_sync_error(vv_ctx* ctx);
/* Test hook: word 0 of the 13 counter lines of each wait family (head, codec
 * stage, LM MLP) into out[39]; consistent between launches when every shard
 * line (0-7) is a multiple of 32 and every generation line a multiple of 8. */
int vv_diag_sync_words(vv_ctx* ctx, unsigned* out);
/* The rule every grid-waiting launch applies (kernels.h persist_resident + the
 * context half): 1 when a grid of `grid` one-per-CU workgroups with the
 * occupancy query's blocks_per_cu on `cus` CUs and `scratch_bytes` of scratch
 * is resident, the context has the kernels enabled and it is the device's only
 * registered context.  Pure function (no device work). */
int vv_persist_decision(int blocks_per_cu, int cus, int scratch_bytes, int grid, int contexts_on_device, int enabled);
/* A/B / test switch: 1 (default) = each narrow codec stage (C <= 128) as ONE
 * launch (codec_tile.hip: transition conv + 3 Block1Ds [+ head conv], halo
 * recomputed per workgroup); 0 = one k_block launch per Block1D + the
 * transition GEMMs. */
int vv_codec_tile(int on);
/* Diagnostic: the tile launches record per-workgroup s_memrealtime phase stamps
 * ([n][tiles][16] u64 at buf + 4096 x (3 x net + stage), net 0 = decoder, 1 =
 * encoder; stage 0..2 in run order); NULL = off. */
int vv_codec_tile_stamps(void* buf);
/* A/B / test switch: 1 (default) = each wide codec stage (C = 256 / 512) as ONE
 * launch of workgroup clusters (codec_wide.hip) where the grid-waiting kernels
 * run; 0 = k_mix + fc1 / fc2 GEMMs per Block1D.  _active: whether a codec step
 * of n samples on ctx runs them now.  _stamps: per-workgroup phase stamps
 * ([n][tiles x S][16] u64 at buf + 8192 x (2 x net + (C == 512))); NULL = off. */
int vv_codec_wide(int on);
/* Diagnostic: wide-stage grids past one resident wave (1: clusters complete in
 * dispatch order; slower at B = 8 than the GEMM path) or only grids resident at
 * once (0, default). */
int vv_codec_wide_over(int on);
int vv_codec_wide_active(vv_ctx* ctx, int n);
int vv_codec_wide_stamps(void* buf);
/* A/B switch: 1 (default) = the balanced many-tile GEMV plan at M >= 8 (one
 * workgroup per CU, 4-5 weight tiles each); 0 = ntile / 8 workgroups. */
int vv_gemv_tune_bal(int on);
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
/* Test / A-B switch: the longest key split (keys) of the deferred-merge plan
 * above; a context needing longer splits takes the grouped plan below.
 * <= 0 restores the built-in 1,024. */
int vv_attn_defer_max(int keys);
/* Test switch: 1 (default) = decode passes of <= 16 rows over more than 8,192
 * keys run up to 120 splits of >= 256 keys merged in <= 8 groups by each
 * group's last-arriving workgroup, o_proj merging the groups; n >= 2: at most
 * n (<= 128) such splits; 0 = 1,024-key splits merged by k_attn_merge. */
int vv_attn_group(int on);
/* The decode attention's plan for a pass of ntok rows over max_pos_p1 keys,
 * host logic only (CPU tests): out = {prefill, nsplit, chunk, defer, group,
 * ngroups}. */
int vv_attn_pass_plan(int ntok, int lm_slots, int head_dim, int n_kv, int max_pos_p1, int* out);
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
/* Test / A-B switch: 1 (default) = a codec stage of Block1Ds at T = 1 and one
 * sample (the acoustic decoder's first, the semantic encoder's last) runs as
 * one persistent launch (codec_stage.hip) while ctx is the device's only
 * context registered for persistent kernels; 0 = one launch per GEMV. */
int vv_codec_stage(int on);
/* Test query: 1 when a one-sample codec step on ctx would run the acoustic
 * decoder's first stage as the persistent launch now. */
int vv_codec_stage_active(vv_ctx* ctx);
/* Diagnostic: the acoustic decoder's persistent launch of stage `stage`
 * records per-workgroup s_memrealtime stamps into buf ([256][64] u64;
 * nullptr: off). */
int vv_codec_stage_stamps(void* buf, int stage);
int vv_rmsnorm_bf16(int M, int C, const void* x, int64_t ldx, const void* w, float eps, void* y, int64_t ldy,
                    vv_stream st);

#ifdef __cplusplus
}
#endif
#endif
