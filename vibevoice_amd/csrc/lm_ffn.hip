// One Qwen2 MLP block of the LM at decode (R = 2 rows: B = 1's positive and
// negative streams) in ONE launch of 256 workgroups with one grid-wide hand-off,
// reading the GEMV layout the LM binds (weights.py mfma_pack: gate|up [2I][H] in
// 16-row tiles of 8 gate + 8 up rows, down [H][I]):
//   x <- x + down(SiLU(gate_proj(a)) * up_proj(a)),  a = RMSNorm(x) * w
// (post_attention_layernorm + Qwen2MLP + residual, modeling_vibevoice.py:169-209
// via transformers' Qwen2DecoderLayer).
//
// Why (DESIGN.md "LM MLP in one launch"): as two GEMV launches the block took
// 13.5 + 11.6 us per layer at B = 1 (the down GEMV reaches 192 CUs at 2.4 TB/s).
// The decomposition is head_m16.hip's at I = 8,960:
//   * gate|up: the 192 down owners stream 4 of the 1,120 tiles each into
//     registers, the other 64 workgroups 5 or 6 (the 5th and 6th into LDS by
//     DMA), so no CU carries more than 332 KB (non-temporal: read once per token); the 8 waves split K (6 of the 48 k-blocks each),
//     MFMA 16x16x32 over the 2 rows (padded to 16), partial tiles summed in a
//     fixed order; SiLU * up -> the act columns, written through;
//   * one grid wait (the act rows gathered: 2 x 8,960 bf16);
//   * down: the 192 workgroups w % 4 != 3 own 8 output columns (half a 16-row
//     down tile over all 8,960 k, 140 KB: 18 k-blocks per wave in registers, 17
//     by DMA into LDS, only this workgroup's 8 rows of each block); issued after
//     SiLU * up so they stream through the hand-off; MFMA; residual.
// Arithmetic: xform<XF_NORM>'s rounding points (norm weight, no modulation), the
// residual as epi_row8's EPI_RES; the GEMM sums are fp32 MFMA sums in another
// order than the GEMV kernels' (tests/test_gpu_lm.py: within bf16 of them).
#include "persist_dev.h"

namespace lf {
constexpr int H = 1536, F = 8960, G = pk::G, RMAX = 2;
constexpr int NTC = 512, NT = NTC + 64;   // 8 compute waves + the control wave
constexpr int KC1 = H / 32, KC2 = F / 32; // 48 / 280 k-blocks
constexpr int T1 = 2 * F / 16;            // 1,120 gate|up tiles
constexpr int KPW1 = KC1 / 8, KPW2 = KC2 / 8;   // 6 / 35 k-blocks per compute wave
constexpr int NREG1 = 4;                  // gate|up tiles in registers (24 chunks per wave); up to 2 more in LDS
constexpr int NREG2 = 18, NLDS2 = KPW2 - NREG2; // down k-blocks per wave in registers / in LDS (17)
constexpr int SLOT2 = 18;                 // LDS down slots per wave (17 + 1 padding: DMA pairs)
constexpr int NCH = H / 8;                // 192 chunks per row
constexpr int XST = H + 8, AST = F + 8;   // padded LDS row strides (MFMA A reads)
constexpr int XS = 0, XS_B = RMAX * XST * 2;
constexpr int NW = XS + XS_B, NW_B = H * 2;
constexpr int WT = NW + NW_B, WT_B = 2 * KC1 * 1024;        // gate|up tiles 3, 4 (96 KB); then the down blocks
constexpr int RED1 = WT + WT_B, RED1_B = 6 * 8 * 256 * 4;    // gate|up partial tiles; then the act rows
constexpr int SM = RED1 + RED1_B, SM_B = 256;                // ok, inv, SiLU*up values, x columns
constexpr int TOTAL = SM + SM_B;
constexpr int DN2 = WT, RED2 = WT + 8 * SLOT2 * 512;        // phase B: down blocks [8][18][256] bf16 | partials [8][256]
static_assert(TOTAL <= 160 * 1024 && XS_B % 16 == 0 && NW % 16 == 0 && WT % 16 == 0, "lm ffn LDS");
static_assert(RMAX * AST * 2 <= RED1_B && RED2 + 8 * 256 * 4 <= WT + WT_B, "lm ffn phase-B LDS");
static_assert(4 * 4 + RMAX * 4 + 6 * RMAX * 8 * 2 + RMAX * 8 * 2 <= SM_B, "lm ffn small region");
}  // namespace lf

__global__ void __launch_bounds__(lf::NT) k_lm_ffn(LmFfnArgs a) {
  using namespace lf;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + XS);
  bf16* nw_s = (bf16*)(smem + NW);
  bf16* wt_s = (bf16*)(smem + WT);
  float* red1 = (float*)(smem + RED1);
  bf16* act_s = (bf16*)(smem + RED1);          // phase B: [R][AST]
  bf16* dn_s = (bf16*)(smem + DN2);            // phase B: [8 waves][18][256]
  float* red2 = (float*)(smem + RED2);
  unsigned* ok_s = (unsigned*)(smem + SM);
  float* inv_s = (float*)(smem + SM + 16);     // [RMAX]
  bf16* su_s = (bf16*)(smem + SM + 16 + RMAX * 4);   // [6][RMAX][8]
  bf16* xraw_s = su_s + 6 * RMAX * 8;                 // [RMAX][8] this workgroup's columns of x

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool ctl = wave == NTC / 64;
  const int w = blockIdx.x, lane = threadIdx.x & 63, R = a.R;
  // the 192 down owners (w % 4 != 3) stream 4 gate|up tiles each (tiles [0, 768));
  // the other 64 the remaining 352 (5 or 6 each): per CU 332 KB (owner: 4 tiles
  // + 140 KB of down) or 240-288 KB, against 380 KB when owners took 5
  // XCD-balanced (workgroup w runs on XCD w % 8): in each group of 32 workgroups,
  // rows (w >> 3) & 3 = 0..2 are owners and row 3 the others, so every XCD holds
  // 24 owners and 8 others; the others' 5 / 6 tiles alternate by group, so every
  // XCD streams the same bytes (with owner = w % 4 != 3 all 64 others, the
  // heaviest gate|up streams, sat on XCDs 3 and 7)
  const int grp = w >> 5, sub = (w >> 3) & 3;
  const bool owner = sub != 3;
  const int d = grp * 24 + sub * 8 + (w & 7);                       // down columns [8d, 8d + 8)
  const int u = grp * 8 + (w & 7);                                  // the others: u = 16 q + r
  const int t0 = owner ? 4 * d : 768 + 88 * (u >> 4) + ((u & 15) < 8 ? 5 * (u & 15) : 40 + 6 * ((u & 15) - 8));
  const int nt = owner ? 4 : 5 + ((u >> 3) & 1);                    // 4, or 5 / 6
  const int nlds = nt - NREG1;                                      // tiles in LDS (0, 1, 2; uniform)
  const int col0 = 8 * d;
  unsigned g0 = 0;
  if (ctl) __builtin_amdgcn_s_setprio(3);
  if (ctl) g0 = __hip_atomic_load((hl_gu32*)(a.sync + 11 * pk::LINE), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;
  // diagnostics (k_lm_ffn16's numbering): 0 start, 1 A side in LDS, 2 normalised, 3 gate|up
  // products, 4 SiLU * up, 5 hand-off released, 6 act rows + down weights landed, 9 end
  auto stamp = [&](int k) {
    if (a.stamps && threadIdx.x == 0) a.stamps[w * 16 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  auto issue_dn_lds = [&]() {
    // k-blocks [+18, +35) of the down weights by DMA into LDS slot wave, only
    // this workgroup's 8 rows of each 1 KB block (512 B: lanes 0-31 block b,
    // 32-63 block b + 1; the last pair's second block is padding)
    const int ln = hl_vopaque(lane);
    const bf16* dw = hl_opaque(a.dn) + (long long)(d >> 1) * KC2 * 512;
    const int p = ln & 31, L = 16 * (p >> 3) + 8 * (d & 1) + (p & 7);   // compact position p <- packed lane L
#pragma unroll
    for (int q = 0; q < SLOT2 / 2; ++q) {
      int kb = NREG2 + 2 * q + (ln >> 5);
      kb = kb < KPW2 ? kb : KPW2 - 1;
      hl_dma16<false, true>(dn_s + (wave * SLOT2 + 2 * q) * 256, dw + (long long)(wave * KPW2 + kb) * 512 + L * 8);
    }
  };

  bf16x8 wb[NREG1 * KPW1];
  if (ctl && owner && lane < R) hl_dma16<false>(xraw_s, hl_opaque(a.x) + (long long)lane * a.ldx + col0);
  if (!ctl) {
    const int ln = hl_vopaque(lane);
    // the A side first (row `wave`, wave 0 also the norm weight), then the
    // register tiles, then the LDS tiles: the norm waits only for the A side
    if (wave < R)
#pragma unroll
      for (int i = 0; i < NCH / 64; ++i)
        hl_dma16<false>(xs + wave * XST + i * 512, hl_opaque(a.x) + (long long)wave * a.ldx + (i * 64 + ln) * 8);
    if (wave == 0)
#pragma unroll
      for (int i = 0; i < NCH / 64; ++i) hl_dma16<false>(nw_s + i * 512, hl_opaque(a.nw) + (i * 64 + ln) * 8);
    const bf16* gw = hl_opaque(a.gu) + (long long)t0 * KC1 * 512 + ln * 8;
#pragma unroll
    for (int j = 0; j < NREG1; ++j)
#pragma unroll
      for (int kk = 0; kk < KPW1; ++kk) wb[j * KPW1 + kk] = hl_ldnt(gw + ((long long)j * KC1 + wave * KPW1 + kk) * 512);
    // tiles 4 and 5 into LDS (uniform per workgroup: 0, 1 or 2 of them)
    for (int j = 0; j < nlds; ++j)
#pragma unroll
      for (int kk = 0; kk < KPW1; ++kk)
        hl_dma16<false, true>(wt_s + (j * KC1 + wave * KPW1 + kk) * 512,
                              gw + ((long long)(NREG1 + j) * KC1 + wave * KPW1 + kk) * 512);
    // this wave's A-side DMA landed (the 24 register loads + 6 nlds DMAs behind it may fly)
    if (nlds == 0) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (nlds == 1) asm volatile("s_waitcnt vmcnt(30)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the x columns landed
  }
  __syncthreads();
  stamp(1);
  for (int m = wave; m < R; m += NT / 64) {   // inverse RMS in k_rmsnorm's order
    const int ln = hl_vopaque(lane);
    float ss = 0.f;
    for (int c = ln; c < NCH; c += 64) {
      const bf16x8 v = *(const bf16x8*)(xs + m * XST + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
    }
    ss = wave_sum(ss);
    if (ln == 0) inv_s[m] = rsqrtf(ss / (float)H + a.eps);
  }
  __syncthreads();
  for (int e = hl_vopaque((int)threadIdx.x); e < R * NCH; e += NT) {   // xform<XF_NORM> (norm weight only), in place
    const int m = e / NCH, c = e - m * NCH;
    const bf16x8 xv = *(const bf16x8*)(xs + m * XST + c * 8), wv = *(const bf16x8*)(nw_s + c * 8);
    const float inv = inv_s[m];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = tobf(rb(rb(bf(xv[j]) * inv) * bf(wv[j])));
    *(bf16x8*)(xs + m * XST + c * 8) = o;
  }
  __syncthreads();
  stamp(2);
  if (!ctl) {   // gate|up: D[row][tile row] over this wave's 6 k-blocks, per tile (rows >= R: never read)
    const int ln = hl_vopaque(lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the LDS tiles (and the register tiles)
    f32x4 acc[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW1; ++kk) {
      const int kc = wave * KPW1 + kk;
      const bf16x8 av = *(const bf16x8*)(xs + (ln & 15) * XST + kc * 32 + 8 * (ln >> 4));
#pragma unroll
      for (int j = 0; j < NREG1; ++j) acc[j] = mfma16(av, wb[j * KPW1 + kk], acc[j]);
#pragma unroll
      for (int j = 0; j < 2; ++j)   // (unfilled slots: products never stored)
        acc[NREG1 + j] = mfma16(av, *(const bf16x8*)(wt_s + (j * KC1 + kc) * 512 + ln * 8), acc[NREG1 + j]);
    }
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j < nt) *(f32x4*)(red1 + (j * 8 + wave) * 256 + ln * 4) = acc[j];
  }
  __syncthreads();
  stamp(3);
  for (int e = hl_vopaque((int)threadIdx.x); e < nt * R * 8; e += NT) {   // SiLU(gate) * up (epi_silu8)
    const int j = e / (R * 8), r = e - j * (R * 8), m = r >> 3, c = r & 7;
    float g = 0.f, u = 0.f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      g += red1[(j * 8 + v) * 256 + (c + 16 * (m >> 2)) * 4 + (m & 3)];
      u += red1[(j * 8 + v) * 256 + (c + 8 + 16 * (m >> 2)) * 4 + (m & 3)];
    }
    su_s[(j * RMAX + m) * 8 + c] = tobf(rb(silu_f(rb(g))) * rb(u));
  }
  __syncthreads();
  stamp(4);
  // (A/B, tools/lm_ffn16_stamps.py 2: the LDS half of the down weights issued at
  // entry, 18.3 -> 20.3 us; k_lm_ffn16's order -- act stores and the arrival
  // ahead of the down weights, the poll after them -- 19.0 us: at 2 rows the
  // stream, not the hand-off, sets the time, and both left HBM idle longer)
  if (!ctl && owner) {
    // the down weights, in flight through the hand-off: k-blocks [35 wave,
    // +18) into the registers (lanes of the other half tile read one line:
    // unconditional loads), [+18, +35) by DMA into LDS slot wave, only this
    // workgroup's 8 rows of each 1 KB block (512 B: lanes 0-31 block b, 32-63
    // block b + 1; the last pair's second block is padding)
    const int ln = hl_vopaque(lane);
    const bf16* dw = hl_opaque(a.dn) + (long long)(d >> 1) * KC2 * 512;
    const bool mine = ((ln & 15) >> 3) == (d & 1);
#pragma unroll
    for (int kk = 0; kk < NREG2; ++kk)
      wb[kk] = hl_ldnt(mine ? dw + (long long)(wave * KPW2 + kk) * 512 + ln * 8 : dw);
    issue_dn_lds();
  }
  if (ctl) {   // act[m][8 (t0 + j) .. + 8], written through
    for (int q = lane; q < nt * R * 2; q += 64) {
      const int j = q / (R * 2), r = q - j * R * 2, m = r >> 1, half = r & 1;
      MemWT::st8(hl_opaque(a.act) + (long long)m * F + 8 * (t0 + j) + 4 * half,
                 *(const bf16x4*)(su_s + (j * RMAX + m) * 8 + 4 * half));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) ok_s[0] = hl_grid_wait_gen(a.sync, 11, g0, 1, w, a.err) ? 1u : 0u;
  }
  __syncthreads();
  stamp(5);
  if (!ok_s[0] || !owner) return;
  // ================= down: act rows -> 8 output columns, residual
  if (!ctl) {
    const bf16* ap = hl_opaque(a.act);
    const int ln = hl_vopaque(lane);
    for (int q = wave; q < R * 18; q += NTC / 64) {   // row m, 64-chunk block i (1,120 chunks: 17.5 blocks)
      const int m = q / 18, i = q - m * 18, c = i * 64 + ln;
      if (c < F / 8) hl_dma16<true>(act_s + m * AST + i * 512, ap + (long long)m * F + c * 8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the act rows, the down registers and the LDS blocks
  }
  __syncthreads();
  stamp(6);
  if (!ctl) {
    const int ln = hl_vopaque(lane);
    const int p = (ln >> 4) * 8 + (ln & 7);   // this lane's compact position (the other half tile's lanes: garbage, never stored)
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    // A rows >= R read row R - 1 again (D row m depends on A row m only: never
    // stored); unconditional reads in groups of 5 ahead of their MFMAs (a guarded
    // read per k-block serialised 35 LDS round trips with the MFMAs: ~1.9 us)
    const bf16* ab = act_s + min(ln & 15, R - 1) * AST + wave * KPW2 * 32 + 8 * (ln >> 4);
#pragma unroll
    for (int k0 = 0; k0 < KPW2; k0 += 5) {
      bf16x8 av[5], wv[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        av[i] = *(const bf16x8*)(ab + (k0 + i) * 32);
        if (k0 + i >= NREG2) wv[i] = *(const bf16x8*)(dn_s + (wave * SLOT2 + k0 + i - NREG2) * 256 + p * 8);
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) acc = mfma16(av[i], k0 + i < NREG2 ? wb[k0 + i] : wv[i], acc);
    }
    *(f32x4*)(red2 + wave * 256 + ln * 4) = acc;
  }
  __syncthreads();
  if (threadIdx.x < RMAX * 8) {   // epi_row8's EPI_RES (no bias, no gamma); rows m < R
    const int m = threadIdx.x >> 3, c = threadIdx.x & 7;
    if (m < R) {
      const int n = c + 8 * (d & 1);   // the tile row of column col0 + c
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += red2[v * 256 + (n + 16 * (m >> 2)) * 4 + (m & 3)];
      a.out[(long long)m * a.ldx + col0 + c] = tobf(bf(xraw_s[m * 8 + c]) + rb(s));
    }
  }
  stamp(9);
}

bool lm_ffn_fits(int H, int F, int R) {
  if (H != lf::H || F != lf::F || R < 1 || R > lf::RMAX) return false;
  static const bool ok = persist_resident_kernel((const void*)k_lm_ffn, lf::NT, lf::TOTAL, lf::G);
  return ok;
}

int launch_lm_ffn(const LmFfnArgs& a, hipStream_t st) {
  if (!lm_ffn_fits(lf::H, lf::F, a.R) || a.ldx < lf::H) return 3;
  hipLaunchKernelGGL(k_lm_ffn, dim3(lf::G), dim3(lf::NT), lf::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ============================================================================
// The same block at 3 <= R <= 16 rows (B = 8: 16 rows), one launch of 256
// workgroups, one grid-wide hand-off (DESIGN.md §8's sizing):
//   * gate|up: the 192 down owners stream 4 of the 16-row tiles each, the other
//     64 workgroups the remaining 352 (5 or 6), into registers (12 compute
//     waves, wave v = tile slot v / 2 over k-blocks [24 (v % 2), + 24)): at most
//     452 KB per CU (stamps: both phases run at the per-CU ingest rate, so the
//     owners' down phase must not sit on top of a 5th tile); the whole 16-row A side
//     (48 KB) by LDS DMA, RMSNorm'd in place (xform<XF_NORM>'s rounding); MFMA;
//     the two K halves summed in order; SiLU * up -> the act columns, written
//     through;
//   * one grid wait;
//   * down, split by K as well as by columns (at 16 rows a column owner would
//     need all 287 KB of act rows): workgroups w < 192 own column group w / 4
//     (32 outputs = 2 tiles) over hidden range w % 4 (2,240 units: 72 KB of act
//     rows by DMA, 140 KB of weights into registers, issued through the
//     hand-off); the [16][32] fp32 partial goes to a slab, and the group's 4th
//     arrival (a per-group ticket, no second grid wait) sums the 4 partials in
//     range order + the residual -> out.
// Arithmetic as k_lm_ffn (another summation order than the GEMV pair).
namespace lf16 {
constexpr int H = 1536, F = 8960, G = pk::G, RMAX = 16;
constexpr int NWC = 12, NTC = NWC * 64, NT = NTC + 64;   // 12 compute waves + the control wave
constexpr int KC1 = H / 32, KC2 = F / 32;                // 48 / 280 k-blocks
constexpr int T1 = 2 * F / 16;                           // 1,120 gate|up tiles
constexpr int KH1 = KC1 / 2;                             // 24 k-blocks per wave (a tile's K half)
constexpr int NG = H / 32, NR = 4, KR = KC2 / NR;        // 48 column groups, 4 hidden ranges of 70 k-blocks
constexpr int KW2 = KR / 5;                              // 14 k-blocks per wave (5 waves per output tile)
constexpr int NCH = H / 8;                               // 192 chunks per row
constexpr int XST = H + 8, AST = KR * 32 + 8;            // padded LDS row strides
constexpr int XS = 0, XS_B = (RMAX * AST * 2 + 15) / 16 * 16;   // A rows (phase A) / act rows (phase B)
constexpr int NW = XS + XS_B, NW_B = H * 2;
constexpr int RED = NW + NW_B, RED_B = 6 * 2 * 256 * 4;  // [6 tiles][2 halves] / [2 tiles][5 K parts] f32x4 tiles
constexpr int SU = RED + RED_B, SU_B = 6 * RMAX * 8 * 2;
constexpr int SM = SU + SU_B, SM_B = 128;                // ok, last, inv[16]
constexpr int TOTAL = SM + SM_B;
constexpr int TK = 13 * pk::LINE;                        // ticket words in the sync buffer (after the 13 counter lines)
static_assert(RMAX * XST * 2 <= XS_B && TOTAL <= 160 * 1024, "lm ffn16 LDS");
}  // namespace lf16

__global__ void __launch_bounds__(lf16::NT) k_lm_ffn16(LmFfnArgs a) {
  using namespace lf16;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + XS);       // phase A: [16][XST] A rows; phase B: [16][AST] act rows
  bf16* nw_s = (bf16*)(smem + NW);
  float* red = (float*)(smem + RED);
  bf16* su_s = (bf16*)(smem + SU);     // [5][16][8]
  unsigned* ok_s = (unsigned*)(smem + SM);
  float* inv_s = (float*)(smem + SM + 16);

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool ctl = wave == NWC;
  const int w = blockIdx.x, lane = threadIdx.x & 63, R = a.R;
  const bool owner = w < NR * NG;
  const int u = w - NR * NG;                                       // non-owner index (XCD u % 8)
  // 5 / 6 tiles alternating every 8 (by parity all 6-tile streams sat on the odd XCDs)
  const int t0 = owner ? 4 * w : 768 + 88 * (u >> 4) + ((u & 15) < 8 ? 5 * (u & 15) : 40 + 6 * ((u & 15) - 8));
  const int nt = owner ? 4 : 5 + ((u >> 3) & 1);                   // 4, or 5 / 6
  const int js = wave >> 1, kh = wave & 1;                         // this wave's tile slot / K half
  const bool busy1 = !ctl && js < nt;
  const int grp = w >> 2, rng = w & 3;                             // down: columns [32 grp, +32), k-blocks [70 rng, +70)
  unsigned g0 = 0;
  if (ctl) __builtin_amdgcn_s_setprio(3);
  if (ctl) g0 = __hip_atomic_load((hl_gu32*)(a.sync + 12 * pk::LINE), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;
  // diagnostics: 0 start, 1 A side in LDS, 2 A side normalised, 3 gate|up products, 4 SiLU * up,
  // 5 hand-off released, 6 act rows + down weights landed, 7 down products, 8 partial published, 9 end
  auto stamp = [&](int k) {
    if (a.stamps && threadIdx.x == 0) a.stamps[w * 16 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  bf16x8 wb[KH1];
  if (!ctl) {
    const int ln = hl_vopaque(lane);
    // the A side first (rows m >= R re-read row R - 1: their products are never stored), the norm weight
    for (int q = wave; q < RMAX * NCH / 64; q += NWC) {   // 64-chunk piece q: row q / 3, chunks (q % 3) * 64 ..
      const int m = q / 3, i = q - m * 3;
      hl_dma16<false>(xs + m * XST + i * 512, hl_opaque(a.x) + (long long)min(m, R - 1) * a.ldx + (i * 64 + ln) * 8);
    }
    if (wave < 3) hl_dma16<false>(nw_s + wave * 512, hl_opaque(a.nw) + (wave * 64 + ln) * 8);
    if (busy1) {
      const bf16* gw = hl_opaque(a.gu) + ((long long)(t0 + js) * KC1 + kh * KH1) * 512 + ln * 8;
#pragma unroll
      for (int kk = 0; kk < KH1; ++kk) wb[kk] = hl_ldnt(gw + (long long)kk * 512);
      asm volatile("s_waitcnt vmcnt(24)" ::: "memory");   // this wave's A-side DMA (the 24 weight loads may fly)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  stamp(1);
  for (int m = wave; m < RMAX; m += NT / 64) {   // inverse RMS in k_rmsnorm's order
    const int ln = hl_vopaque(lane);
    float ss = 0.f;
    for (int c = ln; c < NCH; c += 64) {
      const bf16x8 v = *(const bf16x8*)(xs + m * XST + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
    }
    ss = wave_sum(ss);
    if (ln == 0) inv_s[m] = rsqrtf(ss / (float)H + a.eps);
  }
  __syncthreads();
  for (int e = hl_vopaque((int)threadIdx.x); e < RMAX * NCH; e += NT) {   // xform<XF_NORM> (norm weight only), in place
    const int m = e / NCH, c = e - m * NCH;
    const bf16x8 xv = *(const bf16x8*)(xs + m * XST + c * 8), wv = *(const bf16x8*)(nw_s + c * 8);
    const float inv = inv_s[m];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = tobf(rb(rb(bf(xv[j]) * inv) * bf(wv[j])));
    *(bf16x8*)(xs + m * XST + c * 8) = o;
  }
  __syncthreads();
  stamp(2);
  if (busy1) {   // gate|up tile t0 + js over this wave's K half
    const int ln = hl_vopaque(lane);
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KH1; ++kk) {
      const int kc = kh * KH1 + kk;
      acc = mfma16(*(const bf16x8*)(xs + (ln & 15) * XST + kc * 32 + 8 * (ln >> 4)), wb[kk], acc);
    }
    *(f32x4*)(red + (js * 2 + kh) * 256 + ln * 4) = acc;
  }
  __syncthreads();
  stamp(3);
  for (int e = hl_vopaque((int)threadIdx.x); e < nt * RMAX * 8; e += NT) {   // SiLU(gate) * up (epi_silu8), halves in order
    const int j = e / (RMAX * 8), r = e - j * (RMAX * 8), m = r >> 3, c = r & 7;
    const int lg = (c + 16 * (m >> 2)) * 4 + (m & 3), lu = (c + 8 + 16 * (m >> 2)) * 4 + (m & 3);
    const float g = red[(j * 2) * 256 + lg] + red[(j * 2 + 1) * 256 + lg];
    const float u = red[(j * 2) * 256 + lu] + red[(j * 2 + 1) * 256 + lu];
    su_s[(j * RMAX + m) * 8 + c] = tobf(rb(silu_f(rb(g))) * rb(u));
  }
  __syncthreads();
  stamp(4);
  if (ctl) {   // act[m][8 (t0 + j) .. + 8] for rows m < R, written through, and the arrival: both
               // ahead of the down weights in this CU's memory queue (behind them they waited ~3 us)
    for (int q = lane; q < nt * RMAX * 2; q += 64) {
      const int j = q / (RMAX * 2), r = q - j * RMAX * 2, m = r >> 1, half = r & 1;
      if (m < R)
        MemWT::st8(hl_opaque(a.act) + (long long)m * F + 8 * (t0 + j) + 4 * half,
                   *(const bf16x4*)(su_s + (j * RMAX + m) * 8 + 4 * half));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) hl_arrive_gen(a.sync, 12, w);
  }
  __syncthreads();
  if (wave < 10 && owner) {
    // the down weights, in flight through the hand-off (issued after SiLU * up:
    // issued before it, their 14 loads per thread held the owners' arrival back
    // ~3.5 us): tile 2 grp + (v & 1), k-blocks [70 rng + 14 (v >> 1), + 14), into
    // the registers freed by gate|up
    const int ln = hl_vopaque(lane);
    const bf16* dw = hl_opaque(a.dn) + ((long long)(2 * grp + (wave & 1)) * KC2 + rng * KR + (wave >> 1) * KW2) * 512 + ln * 8;
#pragma unroll
    for (int kk = 0; kk < KW2; ++kk) wb[kk] = hl_ldnt(dw + (long long)kk * 512);
  }
  if (ctl && lane == 0) ok_s[0] = hl_poll_gen(a.sync, 12, g0, 1, a.err) ? 1u : 0u;
  __syncthreads();
  stamp(5);
  if (!ok_s[0] || !owner) return;
  // ================= down over this workgroup's hidden range -> an fp32 partial of 32 columns
  if (!ctl) {
    const bf16* ap = hl_opaque(a.act) + (long long)rng * KR * 32;
    const int ln = hl_vopaque(lane);
    for (int q = wave; q < RMAX * 5; q += NWC) {   // row m, 64-chunk piece i (280 chunks: 4.375 pieces)
      const int m = q / 5, i = q - m * 5, c = i * 64 + ln;
      if (c < KR * 4) hl_dma16<true>(xs + m * AST + i * 512, ap + (long long)min(m, R - 1) * F + c * 8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the act rows and the down registers
  }
  __syncthreads();
  stamp(6);
  if (wave < 10) {
    const int ln = hl_vopaque(lane);
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KW2; ++kk) {
      const int kc = (wave >> 1) * KW2 + kk;
      acc = mfma16(*(const bf16x8*)(xs + (ln & 15) * AST + kc * 32 + 8 * (ln >> 4)), wb[kk], acc);
    }
    *(f32x4*)(red + ((wave & 1) * 5 + (wave >> 1)) * 256 + ln * 4) = acc;
  }
  __syncthreads();
  stamp(7);
  float* slab = a.slab + ((long long)grp * NR + rng) * RMAX * 32;
  if (threadIdx.x < RMAX * 32) {   // partial [m][c32], the 5 K parts in order
    const int m = threadIdx.x >> 5, c32 = threadIdx.x & 31, tl = c32 >> 4, n = c32 & 15;
    const int l = (n + 16 * (m >> 2)) * 4 + (m & 3);
    float s = 0.f;
#pragma unroll
    for (int kp = 0; kp < 5; ++kp) s += red[(tl * 5 + kp) * 256 + l];
    MemWT::stf(slab + m * 32 + c32, s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((hl_gu32*)(a.sync + TK + grp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ok_s[1] = (t & 3) == 3 ? 1u : 0u;   // the group's 4th arrival of this launch sums it
  }
  __syncthreads();
  stamp(8);
  if (!ok_s[1] || threadIdx.x >= RMAX * 32) return;
  {
    const int m = threadIdx.x >> 5, c32 = threadIdx.x & 31, col = 32 * grp + c32;
    if (m < R) {
      const float* sg = a.slab + (long long)grp * NR * RMAX * 32 + m * 32 + c32;
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < NR; ++r) s += MemWT::ldf(sg + r * RMAX * 32);
      a.out[(long long)m * a.ldx + col] = tobf(bf(a.x[(long long)m * a.ldx + col]) + rb(s));
    }
  }
  stamp(9);
}

bool lm_ffn16_fits(int H, int F, int R) {
  if (H != lf16::H || F != lf16::F || R < 3 || R > lf16::RMAX) return false;
  static const bool ok = persist_resident_kernel((const void*)k_lm_ffn16, lf16::NT, lf16::TOTAL, lf16::G);
  return ok;
}

int launch_lm_ffn16(const LmFfnArgs& a, hipStream_t st) {
  if (!lm_ffn16_fits(lf16::H, lf16::F, a.R) || a.ldx < lf16::H || !a.slab) return 3;
  hipLaunchKernelGGL(k_lm_ffn16, dim3(lf16::G), dim3(lf16::NT), lf16::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
