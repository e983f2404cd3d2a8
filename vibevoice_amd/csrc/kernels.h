// Kernel argument structs and host launchers shared by the .hip kernel files
// and the engine (engine.cpp).  See each kernel for the reference it follows.
#pragma once
#include "common.h"

struct DpmCoef {
  float cfg;
  float alpha_s, sigma_s;  // x0 = alpha_s * x - sigma_s * v          (bf16 ops)
  float c_x, c_d0, c_d1, inv_r0;
  int order;               // 1: x' = c_x x - bf16(c_d0 x0)
                           // 2: x' = c_x x - bf16(c_d0 x0) - bf16(c_d1 bf16(inv_r0 bf16(x0 - m1)))
  float c_n;               // sde-dpmsolver++: + c_n * noise (fp32), added last (dpm_solver.py:680-686, 785-793)
};

struct KVLayout {
  bf16* k;
  bf16* v;
  long long s_layer, s_slot, s_head;  // elements; s_ctx = d
  int d, max_ctx;
};

// A-operand transform (XF_*).  XF_NORM: inverse RMS of each A row over K, then
// bf16(bf16(x * inv) * w) (w optional) and optionally the adaLN modulate
// bf16(bf16(y * bf16(1 + scale)) + shift) with shift/scale read from `mod` rows.
struct ATransform {
  int kind;
  float eps;
  const bf16* w;
  const bf16* mod;
  long long mod_ld;
  int shift_off, scale_off;
  const bf16* vec;      // XF_SILU_ADD
  // XF_MIX: the codec Block1D front half of k_mix computed in the GEMV prologue
  // (A rows = the x rows of M/T samples x T steps; w = mixer norm weight)
  int T, ctx;
  bf16* buf;             // conv history buffer (slot stride buf_sB), rows ctx + t written
  long long buf_sB;
  const int* slots;
  const bf16 *dw_w, *dw_b, *gamma, *ffn_w;
  bf16* y;               // residual rows y (fc2's residual), [M][K]
  // XF_ATTN_MERGE: o_proj's A rows = the decode attention output, merged here
  // from the key splits' (m, l, o) partials that k_attn left (AttnArgs::defer)
  const float* part_o;   // [M][nh][nsplit][128]
  const float* part_ml;  // [M][nh][nsplit][2]
  const int* qpos;       // [M] query position (row m attends keys 0..qpos[m])
  int nsplit, chunk;     // the attention launch's plan (row_chunk)
};

struct RopeEpi {         // EPI_ROPE
  int nh, nkv, layer, pad_;
  bf16* q_out;           // [M][nh*d]
  const int* slots;      // [M] KV slot of row
  const int* pos;        // [M] position == cache index written
  const float* inv_freq; // [d/2]
  const bf16* cs_tab;    // [max_ctx][cos d/2 | sin d/2] = bf16(cos / sin(pos * inv_freq)), or nullptr
  KVLayout kv;
};

struct DpmEpi {          // EPI_CFG_DPM
  int n, pad_;
  DpmCoef k;
  bf16* x;               // [n][N] latent, updated in place
  bf16* m1;              // [n][N] previous x0 (2nd-order history)
  const float* noise;    // [n][N] this step's SDE noise rows, or nullptr (ODE)
};

struct GemmArgs {
  int M, N, K;
  int ksplit;
  int handoff;            // split-K hand-off form (gemm.hip: splitk_handoff)
  int tpw;                // k_gemv1: 16-row weight tiles per workgroup (set by launch_gemm)
  RowMap a;
  const bf16* w;
  long long ldw;
  EpiArgs epi;
  ATransform xf;
  RopeEpi rope;
  DpmEpi dpm;
  float* ws;
  unsigned* counters;
  unsigned long long* stamps;  // diagnostic builds only: 4 s_memrealtime stamps per workgroup
  int keep;               // weights re-read soon (diffusion head): default cache policy, not nt
  int apack;              // k_gemm_xl: A rows in MFMA-fragment order (blocks (row tile, chunk) of 1 KB, as W)
};

struct NormArgs {
  int M, C;
  float eps;
  int has_mod;
  RowMap in, out;
  const bf16* w;
  const bf16* mod;      // row m: mod + m * mod_ld
  long long mod_ld;
  int shift_off, scale_off;
  int pack;             // 1: out.base receives the rows in MFMA-fragment order (16-row tiles x
                        // 32-column chunks of 1 KB, weights.py mfma_pack), the A layout
                        // k_gemm_xl stages with one contiguous 1 KB load per block
};

struct DwArgs {
  int M, C, T, K;    // rows (groups*T), channels, rows per group, kernel size
  RowMap buf;        // row t of group -> buffer row t (conv window rows t .. t+K-1)
  RowMap x;
  const bf16* w;     // [C, K]
  const bf16* b;     // [C]
  const bf16* gamma; // [C]
};

// Block1D mixer + FFN pre-norm, fused (elementwise.hip: k_mix)
struct MixArgs {
  int n, T, C, R;          // samples, rows per sample, channels, rows per workgroup
  float eps;
  int ctx;                 // history rows in front of the conv buffer (k - 1)
  const bf16* x;           // residual in  [n][T][C]
  bf16* y;                 // residual out [n][T][C]
  bf16* a;                 // ffn_norm(y)  [n][T][C]
  bf16* buf;               // conv buffer, slot s at buf + s * buf_sB: rows [ctx + t] = norm(x)[t]
  long long buf_sB;
  const int* slots;
  const bf16* norm_w;      // [C]
  const bf16* dw_w;        // [C][7]
  const bf16* dw_b;        // [C]
  const bf16* gamma;       // [C]
  const bf16* ffn_norm_w;  // [C]
};

// a whole codec Block1D in one launch (codec_block.hip, C <= 128)
struct BlockArgs {
  MixArgs mix;             // front half; mix.y / mix.a unused
  const bf16 *w1, *b1;     // fc1 [4C][C] MFMA-packed, bias [4C]
  const bf16 *w2, *b2;     // fc2 [C][4C] MFMA-packed, bias [C]
  const bf16* g2;          // ffn_gamma [C]
  RowMap out;              // block output rows (row = sample * T + t)
  bf16 *dbg_a, *dbg_h;     // diagnostics (tools/block_check.hip): fc1 input / hidden rows, or nullptr
};

struct Conv1Args {
  int M, C, K;
  RowMap buf;
  const bf16* w;   // [K][C]  (re-packed from [1, C, K])
  const bf16* b;   // [1]
  RowMap out, out2;
};

struct ConvIn1Args {
  int M, C, K;
  RowMap buf;      // 1 channel, sT = 1
  const bf16* w;   // [C, K]
  const bf16* b;   // [C]
  RowMap out;
};

struct RollDesc {
  bf16* base;
  long long sB;   // elements per slot
  int ctx, T, C, pad_;
};




struct AttnArgs {
  int nq, nh, nkv, layer, nsplit;
  int chunk;            // keys per split (multiple of 32)
  int merge;            // set by launch_attn: 1 = splits merged by k_attn_merge
  float scale;
  const bf16* q;        // [nq][nh*d]
  bf16* out;            // [nq][nh*d]
  const int* slots;
  const int* pos;        // [nq] position of the query; it attends keys [0, pos]
  KVLayout kv;
  float* part_o;        // [nq][nh][nsplit][d]
  float* part_ml;       // [nq][nh][nsplit][2]
  unsigned* counters;   // [nq * nkv] split tickets (zero between launches)
  unsigned long long* stamps;   // diagnostics only (tools/attn_stamps.py): 4 stamps per workgroup
  int prefill;          // 1: k_attn_pf (query rows in runs sharing a slot; no splits), see attn_use_prefill
  int defer;            // 1: every active split writes its partial, the consumer (o_proj, XF_ATTN_MERGE) merges
  int group;            // > 0 (long contexts): splits merge in groups of `group` consecutive splits -- the
                        // last-arriving workgroup of a group merges its partials into part_o2 / part_ml2
                        // ([nq][nh][ngroups][d] / [..][2]), which the consumer merges (XF_ATTN_MERGE)
  int ngroups;
  float* part_o2;
  float* part_ml2;
};

// out_r = sum_r in_r for every r (single-process tensor-parallel group)
struct SumRows {
  int n, pad_;
  bf16* p[8];
};


// ---- the one-launch kernels with grid-wide waits (persist_dev.h): k_head_m16,
// k_lm_ffn, k_codec_stage*.  Residency rule: every workgroup of the grid must be
// resident at once -- the occupancy query's blocks per CU times the device's CUs
// covers the grid, and no scratch (a wave waiting for a scratch slot is not
// resident).  The engine also requires the context to be the device's only
// registered one and the kernels switched on (vv_persist_decision).
inline bool persist_resident(int blocks_per_cu, int cus, long long scratch_bytes, int grid) {
  return scratch_bytes == 0 && blocks_per_cu >= 1 && (long long)blocks_per_cu * cus >= grid;
}
// the occupancy query of kernel k (nt threads, lds bytes of dynamic LDS) -> persist_resident
bool persist_resident_kernel(const void* k, int nt, int lds, int grid);

// ---- one head FFN layer at 2 <= 2n <= 16 rows in one launch (head_m16.hip), GEMV layout weights
struct HeadM16Args {
  const bf16* x;            // [R][H] state rows (ld ldx), read before the grid wait
  bf16* out;                // [R][H] (ld ldx): x + gate * ffn (in place: out == x)
  const bf16* mod;          // adaLN rows [R][ldmod]: shift / scale / gate at the offsets
  long long ldx, ldmod;
  int shift_off, scale_off, gate_off, R;
  float eps;
  int pad_;
  const bf16* nw;           // RMSNorm weight [H]
  const bf16* gu;           // gate|up, MFMA-packed [2F][H] (EPI_SILU_MUL pairing)
  const bf16* dn;           // down, MFMA-packed [H][F]
  bf16* act;                // [16][F] SiLU(gate) * up rows (workspace, written through)
  unsigned* sync;           // the head's wait lines: shards 0-7, this kernel's generation at line 12
  unsigned* err;            // set to 1 when the grid wait gave up
  unsigned long long* stamps;   // diagnostics (tools/head_m16_stamps.py): [G][16] s_memrealtime, or nullptr
  int a_first;              // 1: every wave's A-side DMA issued before any weight load (a barrier between)
  int late_down;            // 1 (default): the down weights issued after SiLU * up (during the hand-off); 0: after the gate|up products
  // the distributed A side (DESIGN.md "B = 8 head layer"): every launch's epilogue
  // writes per (row, owner) sums of squares of the rows it produced into ssp
  // [16][192]; with pre = 1 a launch builds the transformed A side from them --
  // each owner its 8 columns into xt [16][H], one grid wait, then every
  // workgroup DMAs xt (48 KB) instead of the raw rows, shift and scale (144 KB)
  float* ssp;               // nullptr: no partials written (and pre must be 0)
  bf16* xt;
  int pre;
};
bool head_m16_fits(int H, int F, int R);
int launch_head_m16(const HeadM16Args& a, hipStream_t st);
// x = noisy_images_proj(latents) at 2 <= R <= 16 rows (rows m and m + n read
// latent row m % n) with the row partial sums of squares k_head_m16's
// distributed A side reads for layer 0 (head_m16.hip)
struct HeadNoisyArgs {
  const bf16* lat;   // [n][D] latents
  const bf16* w;     // noisy_images_proj [H][D], MFMA-packed
  bf16* x;           // [R][ldx] state rows
  float* ssp;        // [16][192]
  int n, R, D, ldx;
};
int launch_head_noisy16(const HeadNoisyArgs& a, hipStream_t st);

// ---- the diffusion head's step boundary at 2n <= 16 rows in one launch (head_fin.hip):
// step s's final layer + CFG + DPM update, then step s+1's noisy projection
struct HeadFinArgs {
  int n, R;                 // samples, rows (2n: [cond n | uncond n])
  float eps;
  int shift_off, scale_off; // the final adaLN's shift / scale in the mod rows
  long long ldmod;
  const bf16* x;            // [R][H] state rows after the last FFN layer (read)
  const bf16* mod;          // adaLN rows [R][ldmod]
  const bf16* fw;           // final_layer.linear [D][H], MFMA-packed
  DpmCoef k;
  const bf16* lat;          // [n][D] latents (read)
  bf16* lat_out;            // [n][D] updated latents (written by workgroup 0)
  const bf16* m1;           // [n][D] DPM history (read)
  bf16* m1_out;             // [n][D] (written by workgroup 0)
  const float* noise;       // [R][D] sde-dpmsolver++ draw of this step, or nullptr
  const bf16* nw;           // noisy_images_proj [H][D], MFMA-packed
  bf16* xo;                 // [R][H] the next step's state rows = noisy(updated latents)
  float* ssp;               // R > 4: [16][192] row partial sums of squares (k_head_m16's distributed A side), or nullptr
};
bool head_fin_fits(int H, int D, int R);
int launch_head_fin(const HeadFinArgs& a, hipStream_t st);

// ---- one LM MLP block at decode (R <= 2 rows) in one launch (lm_ffn.hip), GEMV layout weights
struct LmFfnArgs {
  const bf16* x;     // [R][ldx] hidden rows (read: the A side and the residual)
  bf16* out;         // [R][ldx] (may alias x)
  int ldx, R;
  float eps;
  const bf16* nw;    // post_attention_layernorm weight [H]
  const bf16* gu;    // gate|up [2F][H], MFMA-packed (8 gate + 8 up rows per tile)
  const bf16* dn;    // down [H][F], MFMA-packed
  bf16* act;         // [R][F] SiLU(gate) * up, the hand-off rows
  unsigned* sync;    // shards 0-7, generation at line 11 (k_lm_ffn) / 12 (k_lm_ffn16); k_lm_ffn16's
                     // column-group tickets at word 13 x 32
  unsigned* err;     // set to 1 when the grid wait gave up
  float* slab;       // k_lm_ffn16: [48 column groups][4 hidden ranges][16][32] fp32 partials of down
  unsigned long long* stamps;   // diagnostics: [256][16] s_memrealtime per phase, or nullptr
};
bool lm_ffn_fits(int H, int F, int R);
int launch_lm_ffn(const LmFfnArgs& a, hipStream_t st);
// the same block at 3 <= R <= 16 rows (k_lm_ffn16: down split by hidden range too, per-group tickets)
bool lm_ffn16_fits(int H, int F, int R);
int launch_lm_ffn16(const LmFfnArgs& a, hipStream_t st);

// ---- the LM attention half at decode in one launch (lm_attn.hip): input_layernorm
// -> q|k|v + RoPE + KV append -> attention -> o_proj + residual, R <= 16 rows of
// the 1.5B shapes, contexts <= LA_MAX_KEYS keys
constexpr int LA_MAX_KEYS = 4096;
struct LmAttnArgs {
  GemmArgs qkv;      // the q|k|v projection as launch_gemm would run it: M = R, a = the A rows,
                     // w = qkv_w, epi = EPI_ROPE (+ bias), rope = q_out / KV cache / pos / slots
  const bf16* nw;    // input_layernorm weight [H]
  float eps, scale;  // RMSNorm eps, 1 / sqrt(head_dim)
  int R, pad_;
  const bf16* ow;    // o_proj [H][H], MFMA-packed
  RowMap res, out;   // residual rows (read) and output rows (written): x + o_proj(attention)
  bf16* att;         // [R][H] merged attention rows (the o_proj hand-off, written through)
  float* part;       // [units][6 * 128 + 12] per-unit (O, m, l) partials
  unsigned* sync;    // shards 0-7, this kernel's generation at line 15
  unsigned* err;     // set to 1 when a grid wait gave up
  unsigned long long* stamps;   // diagnostics: [256][16] s_memrealtime per phase, or nullptr
  int variant;              // bits (all set by default; vv_lm_attn bits 1..3 clear them, A/B): 1 = A
                            // and attention rows of the R rows only (not 16); 2 = o_proj weights
                            // issued after the first wait, not at entry; 4 = o_proj's residual
                            // operand loaded at entry
};
bool lm_attn_fits(int H, int nh, int nkv, int d, int R, int keys);
size_t lm_attn_part_floats(int R, int keys);
int launch_lm_attn(const LmAttnArgs& a, int keys, hipStream_t st);

// A whole codec stage of Block1Ds for one sample in ONE persistent launch
// (codec_stage.hip): C = 2,048 at T = 1, C = 1,024 at T = 2 or 8.
struct CodecStageBlock {
  const bf16 *norm, *dw_w, *dw_b, *gamma, *ffn_norm;   // mixer norm, depthwise conv [C][7] + bias, layer scale, FFN norm
  const bf16 *fc1_w, *fc1_b, *fc2_w, *fc2_b, *ffn_gamma;   // MFMA-packed fc1 [4C][C], fc2 [C][4C]
  bf16* mix;                // the block's conv buffer (history rows 0 .. ctx-1, new row ctx)
  long long mix_sB;         // elements per slot
};
struct CodecStageArgs {
  int depth, ctx;
  int C, M;                 // channels; rows = T (one sample)
  float eps;
  const int* slots;         // [1]: the sample's slot
  const bf16* x;            // [M][C] stage input rows
  bf16* xe;                 // [M][C] block outputs between blocks (written through)
  bf16* h;                  // [M][4C] hidden rows (written through)
  RowMap out;               // the last block's output rows
  CodecStageBlock b[8];
  unsigned* sync;           // 12 lines of 32 words (shards 0-7, generation 11)
  unsigned* err;            // set to 1 when a grid wait gave up
  unsigned long long* stamps;   // diagnostics: [G][64] s_memrealtime per phase, or nullptr
  int pubfirst;             // C = 2,048 weight-stream issue (codec_stage.hip): 0 = a block's whole
                            // stream at the previous block's end (round 5); 1 = the same after the
                            // output and arrival; 2 = after the wait; 3..5 = in four halves at the
                            // phase points, at most 6 / 10 / 14 loads in flight per wave (default 5)
};
bool codec_stage_fits(int C, int T, int n, int depth);
int launch_codec_stage(const CodecStageArgs& a, hipStream_t st);

// A whole narrow codec stage (C = 128 / 64 / 32) in ONE launch, halo recomputed
// per workgroup (codec_tile.hip): the transition conv that feeds it, its three
// Block1Ds and (decoder) the head conv.
enum { CT_PRE_NONE = 0, CT_PRE_CONVT = 1, CT_PRE_SCONV = 2, CT_PRE_STEM = 3 };
enum { CT_POST_NONE = 0, CT_POST_HEAD = 1 };
struct CodecTileBlock {
  const bf16 *norm, *dw_w, *dw_b, *gamma, *ffn_norm;      // mixer norm, depthwise conv [C][7] + bias, layer scale, FFN norm
  const bf16 *fc1_w, *fc1_b, *fc2_w, *fc2_b, *ffn_gamma;  // MFMA-packed fc1 [4C][C], fc2 [C][4C]
  bf16* mix;                // the block's conv buffer (6 history rows, then this frame's rows)
  long long mix_sB;         // elements per slot
};
struct CodecTileArgs {
  int n, T, depth;          // samples, rows per sample (the stage's), blocks (3)
  float eps;
  const int* slots;         // [n] codec slots
  const bf16* x;            // CT_PRE_NONE: stage input rows [n][T][C]
  const bf16* pre_buf;      // the transition's input ConvBuf (history rows first), by slot
  long long pre_sB;
  const bf16* pre_w;        // convT [2C][4C] / sconv [C][2C] MFMA-packed; stem [C][7]
  const bf16* pre_b;        // convT [2C] (repeated per phase) / sconv, stem [C]
  CodecTileBlock b[3];
  RowMap out;               // CT_POST_NONE: stage output rows (row = sample * T + t)
  const bf16* head_w;       // CT_POST_HEAD: [7][C], bias [1]
  const bf16* head_b;
  bf16* head_buf;           // the head conv's ConvBuf (6 history rows | T rows)
  long long head_sB;
  RowMap audio, audio2;     // audio rows (row = sample * T + t); audio2 optional
  unsigned long long* stamps;   // diagnostics: [n][tiles][16] s_memrealtime per phase, or nullptr
};
bool codec_tile_fits(int C, int pre, int post, int depth, int ctx);
int launch_codec_tile(const CodecTileArgs& a, int C, int pre, int post, hipStream_t st);

// A whole wide codec stage (C = 256 / 512) in ONE launch (codec_wide.hip): a
// cluster of C / 32 workgroups per 16-row time tile, each owning 128 hidden
// units; partials reduce-scattered and block outputs all-gathered inside the
// cluster (write-through hand-offs, bounded cluster-wide waits).
struct CodecWideArgs {
  int n, T, depth;
  float eps;
  const int* slots;
  const bf16* x;            // stage input rows [n][T][C]
  CodecTileBlock b[3];
  RowMap out;               // stage output rows (row = sample * T + t)
  unsigned* sync;           // one 32-word line per cluster (n x tiles), monotonic counters
  unsigned* err;            // set to 1 when a wait gave up
  float* slab;              // [n x tiles][S][40][C] fp32 partials
  bf16* xbuf;               // [n x tiles][40][C] block outputs
  unsigned long long* stamps;   // diagnostics: [n][tiles x S][16] s_memrealtime, or nullptr
};
bool codec_wide_fits(int C, int T, int n, int depth, int ctx);
size_t codec_wide_slab_floats(int C, int T, int n);
size_t codec_wide_xbuf_elems(int C, int T, int n);
int launch_codec_wide(const CodecWideArgs& a, int C, hipStream_t st);
// 1: grids past one resident wave run too (clusters complete in dispatch order); 0 (default): whole grid resident
void codec_wide_oversubscribe(int on);

size_t gemv_mix_lds(int M, int T, int C);
int launch_gemm(GemmArgs a, hipStream_t st);
int launch_sum_rows(SumRows s, long long count, hipStream_t st);
int launch_rmsnorm(NormArgs a, hipStream_t st);
int launch_dwconv(DwArgs a, hipStream_t st);
int launch_mix(MixArgs a, hipStream_t st);
size_t block_lds(int R, int C);   // 0: k_block does not apply
int launch_block(BlockArgs b, hipStream_t st);
int launch_conv_cout1(Conv1Args a, hipStream_t st);
int launch_conv_cin1(ConvIn1Args a, hipStream_t st);
int launch_roll(const RollDesc* d, int nd, const int* slots, int ns, int mode, hipStream_t st);
int launch_latent_to_dec(int n, int D, const bf16* lat, const bf16* s, const bf16* b, RowMap out, hipStream_t st);
int launch_vae_features(int rows, int D, int frames, const bf16* mean, const bf16* stdv, const bf16* noise,
                        const bf16* s, const bf16* b, bf16* out, hipStream_t st);
int launch_head_cond(int steps, int R, int H, const bf16* condp, const bf16* temb, bf16* out, hipStream_t st);
int launch_silu(int n, const bf16* x, bf16* y, hipStream_t st);
// true: launch_gemm would run this (XF-free) GEMM on the 256 x 256 tile
bool gemm_uses_xl(const GemmArgs& a);
int launch_rope_table(int npos, const float* inv_freq, bf16* tab, hipStream_t st);
int launch_cfg_dpm(int n, int D, DpmCoef k, const bf16* eps, bf16* x, bf16* m1, const float* noise, hipStream_t st);
int launch_gather_rows(int n, int C, const bf16* src, long long lds, const int* idx, RowMap dst, hipStream_t st);
int launch_copy_rows1(int n, int C, const bf16* src, long long lds, RowMap dst, hipStream_t st);
int attn_plan(int nq, int nkv, int max_len, int* chunk);
// true: nq query rows over at most nslots distinct slots take the prefill
// kernel (k_attn_pf: 32-row tiles share K/V; no split workspace)
bool attn_use_prefill(int nq, int nslots);
int launch_attn(AttnArgs a, hipStream_t st);
int launch_kv_fill(KVLayout kv, int n_layers, int nkv, int n, const int* slots, int p0, int p1, unsigned seed,
                   hipStream_t st);
int launch_kv_copy(KVLayout kv, int n_layers, int nkv, int n, const int* slots, const int* src, const int* dst,
                   hipStream_t st);
int launch_final_head(int R, int H, const bf16* h, const int* idx, const bf16* norm_w, float eps, bf16* hidden_out,
                      const bf16* W, const int* ids, int nid, float* logits, hipStream_t st);
int launch_lmhead_ids(int R, int H, const bf16* h, long long ldh, const bf16* W, const int* ids, int nid, float* out,
                      hipStream_t st);

// RowMap helpers (host)
static inline RowMap rowmap(const void* base, long long sT, int T = 1 << 30, long long sB = 0,
                            const int* idx = nullptr) {
  RowMap r;
  r.base = const_cast<void*>(base);
  r.sB = sB;
  r.sT = sT;
  r.T = T;
  r.pad_ = 0;
  r.idx = idx;
  return r;
}
