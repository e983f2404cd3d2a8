// One diffusion-head FFN layer at 2 <= 2n <= 16 rows (configs[2]: B = 8 -> 16
// rows) in ONE launch of 256 workgroups with one grid-wide hand-off, reading
// the GEMV layout the engine binds at that batch (weights.py mfma_pack: gate|up
// [2F][H] in 16-row tiles of 8 gate + 8 up rows, down [H][F]):
//   x <- x + gate * down(SiLU(gate_proj(a)) * up_proj(a)),  a = modulate(norm(x))
// (HeadLayer / FeedForwardNetwork, modular_vibevoice_diffusion_head.py:96-161).
//
// Why (DESIGN.md "B = 8 head"): as two GEMV launches the layer took 13.2 + 11.8
// us at 16 rows (k_gemv1 gate|up with the 16-row norm / modulation prologue,
// k_gemv down at 0.15 of HBM).  The persistent head's split-K decomposition does
// not carry to 16 rows (a 96 KB fp32 partial per workgroup), so this kernel
// splits differently:
//   * gate|up: workgroup w owns tiles [9w/4, 9(w+1)/4) of the 576 (2 or 3:
//     16-24 hidden units), every row's A side (16 x 1,536, transformed once per
//     workgroup from LDS), MFMA 16x16x32 with the 8 compute waves splitting K
//     (6 of the 48 k-blocks each), the partial tiles summed in a fixed order;
//     SiLU * up -> its act columns, written through;
//   * one grid wait (the act rows gathered);
//   * down: the 192 two-tile workgroups each own 8 output columns (half of a
//     16-row down tile, 72 KB, loaded into registers right after the gate|up
//     products, so the stream runs through the wait), MFMA over all 4,608 k
//     with the act rows DMA'd into LDS; gated residual; plain stores (the
//     launch's end publishes them).
// Weights are read with the default cache policy: the head's 170 MB are read S
// times per token and stay in the Infinity Cache (gemv_dev.h ldw<KEEP>).
// Arithmetic: xform<XF_NORM>'s rounding points and k_rmsnorm's row order for
// the norm; the GEMM sums are fp32 MFMA sums in another order than the GEMV
// kernels', so the layer is within bf16 of the two-launch path, not bitwise
// (tests/test_gpu_head.py).
#include "persist_dev.h"

namespace hm {
constexpr int H = 1536, F = 4608, G = pk::G, RMAX = 16;
constexpr int NTC = 512, NT = NTC + 64;   // 8 compute waves + the control wave
constexpr int KC1 = H / 32, KC2 = F / 32; // 48 / 144 k-blocks
constexpr int T1 = 2 * F / 16;            // 576 gate|up tiles
constexpr int KPW1 = KC1 / 8, KPW2 = KC2 / 8;   // k-blocks per compute wave: 6 / 18
constexpr int NCH = H / 8;                // 192 chunks per state row
constexpr int NOWN = 192;                 // down-column owners (8 columns each) = ssp partials per row
constexpr int WB = 3 * KPW1 > KPW2 ? 3 * KPW1 : KPW2;   // weight registers per lane (18 chunks)
// LDS, phase A: xs | sh | sc (each [16][H] bf16) | nw [H] | small;   the gate|up
// partial tiles [3][8 waves][256] fp32 reuse sh after the transform.
// Phase B: act [16][F] bf16 over xs / sh / sc | the down partials [8 waves][256]
// fp32 after the small region.
// xs / act rows padded by 16 B: the MFMA A reads (lane l: row l & 15) of an
// unpadded 3,072 / 9,216 B row stride all hit the same 4 banks (16-way conflicts)
constexpr int XST = H + 8, AST = F + 8;
constexpr int XS = 0, SH = XS + RMAX * XST * 2, SC = SH + RMAX * H * 2, NW = SC + RMAX * H * 2;
constexpr int SM = NW + H * 2;
constexpr int SM_B = (4 + RMAX + 3 * RMAX * 8) * 4 + 2 * RMAX * 8 * 2;   // ok, inv, silu*up values, xraw / gate
// (the down partials go after the small region, which holds the x / gate values
// the epilogue reads)
constexpr int ACT = 0, RED2 = (SM + SM_B + 15) / 16 * 16;
constexpr int TOTAL = RED2 + 8 * 256 * 4;
static_assert(TOTAL <= 160 * 1024 && 3 * 8 * 256 * 4 <= RMAX * H * 2, "head m16 LDS");
static_assert(ACT + RMAX * AST * 2 <= SM, "the act rows stay clear of the small region");
}  // namespace hm

__global__ void __launch_bounds__(hm::NT) k_head_m16(HeadM16Args a) {
  using namespace hm;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + XS);
  bf16* sh_s = (bf16*)(smem + SH);
  bf16* sc_s = (bf16*)(smem + SC);
  bf16* nw_s = (bf16*)(smem + NW);
  float* red1 = (float*)(smem + SH);          // [3][8][256] after the transform
  float* sm = (float*)(smem + SM);
  unsigned* ok_s = (unsigned*)sm;
  float* inv_s = sm + 4;                       // [16]
  bf16* su_s = (bf16*)(inv_s + RMAX);          // [3][16][8] SiLU(gate) * up
  bf16* xraw_s = su_s + 3 * RMAX * 8;          // [16][8] this workgroup's down columns of x
  bf16* gate_s = xraw_s + RMAX * 8;            // [16][8] their adaLN gates
  bf16* act_s = (bf16*)(smem + ACT);           // phase B: [16][F]
  float* red2 = (float*)(smem + RED2);         // phase B: [8][256]

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool ctl = wave == NTC / 64;
  const int w = blockIdx.x, lane = threadIdx.x & 63, R = a.R;
  // XCD-balanced (workgroup w runs on XCD w % 8): in each group of 32 workgroups,
  // rows (w >> 3) & 3 = 0..2 own down columns and stream 2 gate|up tiles, row 3
  // streams 3, so every XCD holds 24 owners and 8 three-tile workgroups (with
  // owner = w % 4 != 3, all 64 three-tile streams sat on XCDs 3 and 7)
  const int sub = (w >> 3) & 3;
  const bool owner = sub != 3;                                    // the two-tile workgroups own down columns
  const int d = (w >> 5) * 24 + sub * 8 + (w & 7);                // down columns [8d, 8d + 8)
  const int u = (w >> 5) * 8 + (w & 7);                           // the three-tile workgroups 0..63
  const int t0 = owner ? 2 * d : 2 * NOWN + 3 * u, nt = owner ? 2 : 3;   // gate|up tiles
  const int col0 = 8 * d;
  unsigned g0 = 0;
  // diagnostics: 0 entry, 1 A side landed (wave 0), 2 row norms, 3 transform,
  // 4 gate|up partials in LDS, 5 SiLU * up, 6 hand-off released, 7 act rows in
  // LDS, 8 down partials in LDS, 9 end (owners); 10 A side landed (wave 7),
  // 11 gate / x columns landed (control wave), 12 / 13 wave 0's norm / transform
  // loop done (before the barrier)
  auto stamp = [&](int k, bool by_ctl) {
    if (a.stamps && threadIdx.x == (by_ctl ? NTC : 0)) a.stamps[w * 16 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0, true);
  if (ctl) __builtin_amdgcn_s_setprio(3);
  if (ctl) g0 = __hip_atomic_load((hl_gu32*)(a.sync + 12 * pk::LINE), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;

  bf16x8 wb[WB];
  // this workgroup's half down tile into the registers (in flight through the
  // hand-off); lanes of the other half of the tile feed only output columns this
  // workgroup does not store: they read one line instead (unconditional loads)
  auto down_chunk = [&](int kk) {
    const int ln = hl_vopaque(lane);
    const bf16* dw = hl_opaque(a.dn) + (long long)(d >> 1) * KC2 * 512 + ln * 8;
    const bool mine = ((ln & 15) >> 3) == (d & 1);
    return mine ? dw + (long long)(wave * KPW2 + kk) * 512 : dw - ln * 8;
  };
  auto load_down = [&]() {
#pragma unroll
    for (int kk = 0; kk < KPW2; ++kk) wb[kk] = hl_ld(down_chunk(kk));
  };
  if (ctl && owner && lane < R) {   // x and adaLN gate of this workgroup's down columns (LDS DMA, first in the queue)
    hl_dma16<false>(gate_s, hl_opaque(a.mod) + (long long)lane * a.ldmod + a.gate_off + col0);
    hl_dma16<false>(xraw_s, hl_opaque(a.x) + (long long)lane * a.ldx + col0);
  }
  if (a.pre && ctl && owner) {
    // this workgroup's slice of the A side: its 8 columns of shift / scale / norm
    // weight, and the previous launch's row partial sums of squares (into the
    // dead sh / sc regions; the raw x columns are xraw_s)
    const bf16* mp = hl_opaque(a.mod);
    if (lane < R) {
      hl_dma16<false>(sc_s, mp + (long long)lane * a.ldmod + a.scale_off + col0);
      hl_dma16<false>(sc_s + RMAX * 8, mp + (long long)lane * a.ldmod + a.shift_off + col0);
    }
    if (lane == 0) hl_dma16<false>(nw_s, hl_opaque(a.nw) + col0);
    const float* sp = hl_opaque((const float*)a.ssp);
    for (int i = 0; i * 64 < R * NOWN / 4; ++i)
      if (i * 64 + lane < R * NOWN / 4) hl_dma16<false>(sh_s + i * 512, sp + (i * 64 + lane) * 4);
  }
  if (!a.pre && !ctl) {
    // the A side first (rows wave, wave + 8: state, shift, scale; wave 0 also the
    // norm weight; LDS DMA), then this wave's k-blocks of each gate|up tile: the
    // DMA waits below count only the weight loads behind it
    const int ln = hl_vopaque(lane);
    const bf16* xp = hl_opaque(a.x);
    const bf16* mp = hl_opaque(a.mod);
    for (int m = wave; m < R; m += NTC / 64) {
#pragma unroll
      for (int i = 0; i < NCH / 64; ++i) {
        const int c = i * 64 + ln;
        hl_dma16<false>(xs + m * XST + i * 512, xp + (long long)m * a.ldx + c * 8);
        hl_dma16<false>(sh_s + m * H + i * 512, mp + (long long)m * a.ldmod + a.shift_off + c * 8);
        hl_dma16<false>(sc_s + m * H + i * 512, mp + (long long)m * a.ldmod + a.scale_off + c * 8);
      }
    }
    if (wave == 0)
#pragma unroll
      for (int i = 0; i < NCH / 64; ++i) hl_dma16<false>(nw_s + i * 512, hl_opaque(a.nw) + (i * 64 + ln) * 8);
  }
  if (a.a_first) __builtin_amdgcn_s_barrier();   // (uniform) the whole A side queued ahead of the weights
  if (!ctl) {
    // (every load unconditional: a guarded load compiles to a branch and a
    // vmcnt(0) at its join, which drained the whole queue here; a two-tile
    // workgroup's third set reads one line of tile t0 and is never stored)
    const bf16* gw = hl_opaque(a.gu) + (long long)t0 * KC1 * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int kk = 0; kk < KPW1; ++kk)
        wb[j * KPW1 + kk] = hl_ld(j < nt ? gw + ((long long)j * KC1 + wave * KPW1 + kk) * 512 : gw - lane * 8);
    if (!a.pre) {
      asm volatile("s_waitcnt vmcnt(18)" ::: "memory");   // this wave's A-side DMA landed (18 weight loads may fly)
      stamp(1, false);
      if (wave == NTC / 64 - 1 && a.stamps && lane == 0) a.stamps[w * 16 + 10] = __builtin_amdgcn_s_memrealtime();
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the gate / x columns (and the slice) landed
    stamp(11, true);
  }
  if (a.pre) {
    // the distributed transform: owner rows' inverse RMS from the 192 partials
    // (fixed order: 4 lanes per row, 48 partials each, then pairwise), its 8
    // columns modulated (xform<XF_NORM>'s rounding points) and written through
    if (ctl && owner) {
      const int m = lane >> 2, q = lane & 3;
      const float* ps = (const float*)sh_s + m * NOWN + q * (NOWN / 4);
      float ss = 0.f;
      for (int i = 0; i < NOWN / 4; ++i) ss += ps[i];
      ss += __shfl_xor(ss, 1);
      ss += __shfl_xor(ss, 2);
      const float inv = rsqrtf(ss / (float)H + a.eps);
      const float invm = __shfl(inv, 4 * (lane & 15));
      if (lane < R) {
        const bf16x8 xv = *(const bf16x8*)(xraw_s + lane * 8), wv = *(const bf16x8*)nw_s;
        const bf16x8 scv = *(const bf16x8*)(sc_s + lane * 8), shv = *(const bf16x8*)(sc_s + RMAX * 8 + lane * 8);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = rb(bf(xv[j]) * invm);
          t = rb(t * bf(wv[j]));
          t = rb(rb(t * rb(1.0f + bf(scv[j]))) + bf(shv[j]));
          o[j] = tobf(t);
        }
        bf16* dst = hl_opaque(a.xt) + (long long)lane * H + col0;
        MemWT::st8(dst, __builtin_shufflevector(o, o, 0, 1, 2, 3));
        MemWT::st8(dst + 4, __builtin_shufflevector(o, o, 4, 5, 6, 7));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (ctl && lane == 0) ok_s[1] = hl_grid_wait_gen(a.sync, 12, g0, 1, w, a.err) ? 1u : 0u;
    __syncthreads();
    stamp(2, true);
    if (!ok_s[1]) return;
    if (!ctl) {   // the transformed rows (rows >= R stay unset: their MFMA rows are never read)
      const bf16* xp = hl_opaque((const bf16*)a.xt);
      for (int b = wave; b < R * NCH / 64; b += NTC / 64) hl_dma16<true>(xs + (b / (NCH / 64)) * XST + (b % (NCH / 64)) * 512, xp + (b * 64 + lane) * 8);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    stamp(3, true);
  } else {
  __syncthreads();
  if (wave == 0 && a.stamps && lane == 0) a.stamps[w * 16 + 14] = __builtin_amdgcn_s_memrealtime();
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
  if (wave == 0 && a.stamps && lane == 0) a.stamps[w * 16 + 12] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  stamp(2, true);
  // xform<XF_NORM>, in place, rows < R (rows >= R stay unset: their MFMA rows are never read)
  for (int e = hl_vopaque((int)threadIdx.x); e < R * NCH; e += NT) {
    const int m = e / NCH, c = e - m * NCH;
    bf16x8 o;
    const bf16x8 xv = *(const bf16x8*)(xs + m * XST + c * 8), wv = *(const bf16x8*)(nw_s + c * 8);
    const bf16x8 shv = *(const bf16x8*)(sh_s + e * 8), scv = *(const bf16x8*)(sc_s + e * 8);
    const float inv = inv_s[m];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = rb(bf(xv[j]) * inv);
      t = rb(t * bf(wv[j]));
      t = rb(rb(t * rb(1.0f + bf(scv[j]))) + bf(shv[j]));
      o[j] = tobf(t);
    }
    *(bf16x8*)(xs + m * XST + c * 8) = o;
  }
  if (wave == 0 && a.stamps && lane == 0) a.stamps[w * 16 + 13] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  stamp(3, true);
  }
  if (!ctl) {   // gate|up: D[row][tile row] over this wave's 6 k-blocks, per tile
    const int ln = hl_vopaque(lane);
    f32x4 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW1; ++kk) {
      const int kc = wave * KPW1 + kk;
      const bf16x8 av = *(const bf16x8*)(xs + (ln & 15) * XST + kc * 32 + 8 * (ln >> 4));
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16(av, wb[j * KPW1 + kk], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < nt) *(f32x4*)(red1 + (j * 8 + wave) * 256 + ln * 4) = acc[j];
    if (owner && !a.late_down) load_down();   // (the earlier issue point: A/B)
  }
  __syncthreads();
  stamp(4, true);
  for (int e = hl_vopaque((int)threadIdx.x); e < nt * RMAX * 8; e += NT) {   // SiLU(gate) * up (epi_silu8)
    const int j = e / (RMAX * 8), r = e - j * (RMAX * 8), m = r >> 3, c = r & 7;
    // D[m][n]: lane (n + 16 * (m >> 2)), element m & 3
    float g = 0.f, u = 0.f;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      g += red1[(j * 8 + v) * 256 + (c + 16 * (m >> 2)) * 4 + (m & 3)];
      u += red1[(j * 8 + v) * 256 + (c + 8 + 16 * (m >> 2)) * 4 + (m & 3)];
    }
    su_s[e] = tobf(rb(silu_f(rb(g))) * rb(u));
  }
  __syncthreads();
  stamp(5, true);
  // the down weights, in flight through the hand-off (issued here rather than
  // after the gate|up products: the 144 loads per CU took the waves ~1 us to
  // issue, delaying SiLU * up and the arrival; DESIGN.md "B = 8 head layer")
  if (!ctl && owner && a.late_down) load_down();
  if (ctl) {   // act[m][8 (t0 + j) .. + 8], written through
    for (int q = lane; q < nt * R * 2; q += 64) {
      const int j = q / (R * 2), r = q - j * R * 2, m = r >> 1, half = r & 1;
      MemWT::st8(hl_opaque(a.act) + (long long)m * F + 8 * (t0 + j) + 4 * half,
                 *(const bf16x4*)(su_s + (j * RMAX + m) * 8 + 4 * half));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) ok_s[0] = hl_grid_wait_gen(a.sync, 12, g0, a.pre ? 2 : 1, w, a.err) ? 1u : 0u;
  }
  __syncthreads();
  stamp(6, true);
  if (!ok_s[0] || !owner) return;
  // ================= down: act rows -> 8 output columns, gated residual
  if (!ctl) {
    const int t = hl_vopaque((int)threadIdx.x);
    const bf16* ap = hl_opaque(a.act);
    for (int m = 0; m < R; ++m)
#pragma unroll
      for (int i = 0; i < F / 8 / NTC; ++i) {   // 576 chunks per row: (m, i) covers chunks [512 i, 512 i + 512) ...
        const int c = i * NTC + t;
        hl_dma16<true>(act_s + m * AST + (i * NTC + 64 * wave) * 8, ap + (long long)m * F + c * 8);
      }
    if (F / 8 % NTC) {   // the 64 chunks left per row (576 = 512 + 64): wave 0
      for (int m = 0; m < R; ++m)
        if (wave == 0) hl_dma16<true>(act_s + m * AST + (F / 8 / NTC) * NTC * 8, ap + (long long)m * F + ((F / 8 / NTC) * NTC + t) * 8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  stamp(7, true);
  if (!ctl) {
    const int ln = hl_vopaque(lane);
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    // A rows >= R read row R - 1 again (D row m depends on A row m only: never
    // stored); unconditional reads in groups of 6 ahead of their MFMAs (a guarded
    // read per k-block serialised ~35 LDS round trips with the MFMAs)
    const bf16* ab = act_s + min(ln & 15, R - 1) * AST + wave * KPW2 * 32 + 8 * (ln >> 4);
#pragma unroll
    for (int k0 = 0; k0 < KPW2; k0 += 6) {
      bf16x8 av[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) av[i] = *(const bf16x8*)(ab + (k0 + i) * 32);
#pragma unroll
      for (int i = 0; i < 6; ++i) acc = mfma16(av[i], wb[k0 + i], acc);
    }
    *(f32x4*)(red2 + wave * 256 + ln * 4) = acc;
  }
  __syncthreads();
  stamp(8, true);
  if (threadIdx.x < RMAX * 8) {   // epi_row8's EPI_RES with the adaLN gate; rows m < R
    const int m = threadIdx.x >> 3, c = threadIdx.x & 7;
    float q = 0.f;
    if (m < R) {
      const int n = c + 8 * (d & 1);   // the tile row of column col0 + c
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += red2[v * 256 + (n + 16 * (m >> 2)) * 4 + (m & 3)];
      const float y = rb(bf(gate_s[m * 8 + c]) * rb(s));
      const bf16 ov = tobf(bf(xraw_s[m * 8 + c]) + y);
      a.out[(long long)m * a.ldx + col0 + c] = ov;
      q = bf(ov) * bf(ov);
    }
    if (a.ssp) {   // the next launch's row partial sums of squares (8 columns, fixed pairwise order)
      q += __shfl_xor(q, 1);
      q += __shfl_xor(q, 2);
      q += __shfl_xor(q, 4);
      if (c == 0 && m < R) a.ssp[m * NOWN + d] = q;
    }
  }
  stamp(9, false);
}

// One workgroup per owner d (columns [8d, 8d + 8)), thread (row m = t >> 3,
// column c = t & 7): the K = 64 dot in k order (fp32 fmaf of exact bf16
// products), rounded to bf16 at the store; the row's sum of squares over the 8
// columns in k_head_m16's epilogue order.
__global__ void __launch_bounds__(128) k_head_noisy16(HeadNoisyArgs a) {
  using namespace hm;
  const int d = blockIdx.x, t = threadIdx.x, m = t >> 3, c = t & 7;
  const int j = 8 * d + c;
  float q = 0.f;
  if (m < a.R) {
    const bf16* lr = a.lat + (long long)(m % a.n) * a.D;
    float acc = 0.f;
    for (int k = 0; k < a.D; k += 8) {
      const bf16x8 wv = *(const bf16x8*)hl_packed(a.w, a.D, j, k), xv = *(const bf16x8*)(lr + k);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(bf(xv[e]), bf(wv[e]), acc);
    }
    const bf16 ov = tobf(acc);
    a.x[(long long)m * a.ldx + j] = ov;
    q = bf(ov) * bf(ov);
  }
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  q += __shfl_xor(q, 4);
  if (c == 0 && m < a.R) a.ssp[m * NOWN + d] = q;
}

int launch_head_noisy16(const HeadNoisyArgs& a, hipStream_t st) {
  if (a.R < 2 || a.R > hm::RMAX || a.D % 32 || a.ldx < hm::H) return 3;
  hipLaunchKernelGGL(k_head_noisy16, dim3(hm::NOWN), dim3(128), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

bool head_m16_fits(int H, int F, int R) {
  if (H != hm::H || F != hm::F || R < 2 || R > hm::RMAX) return false;
  static const bool ok = persist_resident_kernel((const void*)k_head_m16, hm::NT, hm::TOTAL, hm::G);
  return ok;
}

int launch_head_m16(const HeadM16Args& a, hipStream_t st) {
  if (!head_m16_fits(hm::H, hm::F, a.R)) return 3;
  hipLaunchKernelGGL(k_head_m16, dim3(hm::G), dim3(hm::NT), hm::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
