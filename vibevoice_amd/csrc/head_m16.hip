// One diffusion-head FFN layer at 4 < 2n <= 16 rows (configs[2]: B = 8 -> 16
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
constexpr int WB = 3 * KPW1 > KPW2 ? 3 * KPW1 : KPW2;   // weight registers per lane (18 chunks)
// LDS, phase A: xs | sh | sc (each [16][H] bf16) | nw [H] | small;   the gate|up
// partial tiles [3][8 waves][256] fp32 reuse sh after the transform.
// Phase B: act [16][F] bf16 over xs / sh / sc | the down partials [8 waves][256]
// fp32 after the small region.
constexpr int XS = 0, SH = XS + RMAX * H * 2, SC = SH + RMAX * H * 2, NW = SC + RMAX * H * 2;
constexpr int SM = NW + H * 2;
constexpr int SM_B = (4 + RMAX + 3 * RMAX * 8) * 4 + 2 * RMAX * 8 * 2;   // ok, inv, silu*up values, xraw / gate
// (the down partials go after the small region, which holds the x / gate values
// the epilogue reads)
constexpr int ACT = 0, RED2 = (SM + SM_B + 15) / 16 * 16;
constexpr int TOTAL = RED2 + 8 * 256 * 4;
static_assert(TOTAL <= 160 * 1024 && 3 * 8 * 256 * 4 <= RMAX * H * 2, "head m16 LDS");
static_assert(ACT + RMAX * F * 2 <= SM, "the act rows stay clear of the small region");
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
  const int t0 = (w * 9) >> 2, nt = (((w + 1) * 9) >> 2) - t0;   // gate|up tiles (2 or 3)
  const bool owner = (w & 3) != 3;                                // the two-tile workgroups own down columns
  const int d = 3 * (w >> 2) + (w & 3);                           // down columns [8d, 8d + 8)
  const int col0 = 8 * d;
  unsigned g0 = 0;
  if (ctl) __builtin_amdgcn_s_setprio(3);
  if (ctl) g0 = __hip_atomic_load((hl_gu32*)(a.sync + 12 * pk::LINE), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;

  bf16x8 wb[WB];
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  if (!ctl) {
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
        hl_dma16<false>(xs + m * H + i * 512, xp + (long long)m * a.ldx + c * 8);
        hl_dma16<false>(sh_s + m * H + i * 512, mp + (long long)m * a.ldmod + a.shift_off + c * 8);
        hl_dma16<false>(sc_s + m * H + i * 512, mp + (long long)m * a.ldmod + a.scale_off + c * 8);
      }
    }
    if (wave == 0)
#pragma unroll
      for (int i = 0; i < NCH / 64; ++i) hl_dma16<false>(nw_s + i * 512, hl_opaque(a.nw) + (i * 64 + ln) * 8);
    // (every load unconditional: a guarded load compiles to a branch and a
    // vmcnt(0) at its join, which drained the whole queue here; a two-tile
    // workgroup's third set reads one line of tile t0 and is never stored)
    const bf16* gw = hl_opaque(a.gu) + (long long)t0 * KC1 * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int kk = 0; kk < KPW1; ++kk)
        wb[j * KPW1 + kk] = hl_ld(j < nt ? gw + ((long long)j * KC1 + wave * KPW1 + kk) * 512 : gw - lane * 8);
    asm volatile("s_waitcnt vmcnt(18)" ::: "memory");   // this wave's A-side DMA landed (18 weight loads may fly)
  }
  if (ctl && owner && lane < R) {   // x and adaLN gate of this workgroup's down columns
    const bf16* xp = hl_opaque(a.x);
    const bf16* mp = hl_opaque(a.mod);
    *(bf16x8*)(gate_s + lane * 8) = hl_ld(mp + (long long)lane * a.ldmod + a.gate_off + col0);
    *(bf16x8*)(xraw_s + lane * 8) = hl_ld(xp + (long long)lane * a.ldx + col0);
  }
  __syncthreads();
  for (int m = wave; m < R; m += NT / 64) {   // inverse RMS in k_rmsnorm's order
    const int ln = hl_vopaque(lane);
    float ss = 0.f;
    for (int c = ln; c < NCH; c += 64) {
      const bf16x8 v = *(const bf16x8*)(xs + m * H + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
    }
    ss = wave_sum(ss);
    if (ln == 0) inv_s[m] = rsqrtf(ss / (float)H + a.eps);
  }
  __syncthreads();
  for (int e = hl_vopaque((int)threadIdx.x); e < RMAX * NCH; e += NT) {   // xform<XF_NORM>, in place; rows >= R zero
    const int m = e / NCH, c = e - m * NCH;
    bf16x8 o = zero8;
    if (m < R) {
      const bf16x8 xv = *(const bf16x8*)(xs + e * 8), wv = *(const bf16x8*)(nw_s + c * 8);
      const bf16x8 shv = *(const bf16x8*)(sh_s + e * 8), scv = *(const bf16x8*)(sc_s + e * 8);
      const float inv = inv_s[m];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = rb(bf(xv[j]) * inv);
        t = rb(t * bf(wv[j]));
        t = rb(rb(t * rb(1.0f + bf(scv[j]))) + bf(shv[j]));
        o[j] = tobf(t);
      }
    }
    *(bf16x8*)(xs + e * 8) = o;
  }
  __syncthreads();
  if (!ctl) {   // gate|up: D[row][tile row] over this wave's 6 k-blocks, per tile
    const int ln = hl_vopaque(lane);
    f32x4 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW1; ++kk) {
      const int kc = wave * KPW1 + kk;
      const bf16x8 av = *(const bf16x8*)(xs + (ln & 15) * H + kc * 32 + 8 * (ln >> 4));
#pragma unroll
      for (int j = 0; j < 3; ++j) acc[j] = mfma16(av, wb[j * KPW1 + kk], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j < nt) *(f32x4*)(red1 + (j * 8 + wave) * 256 + ln * 4) = acc[j];
    if (owner) {   // this workgroup's half down tile into the registers (in flight through the wait)
      // lanes of the other half of the tile feed only output columns this
      // workgroup does not store: they read one line instead (unconditional loads)
      const bf16* dw = hl_opaque(a.dn) + (long long)(d >> 1) * KC2 * 512 + ln * 8;
      const bool mine = ((ln & 15) >> 3) == (d & 1);
#pragma unroll
      for (int kk = 0; kk < KPW2; ++kk)
        wb[kk] = hl_ld(mine ? dw + (long long)(wave * KPW2 + kk) * 512 : dw - ln * 8);
    }
  }
  __syncthreads();
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
  if (ctl) {   // act[m][8 (t0 + j) .. + 8], written through
    for (int q = lane; q < nt * R * 2; q += 64) {
      const int j = q / (R * 2), r = q - j * R * 2, m = r >> 1, half = r & 1;
      MemWT::st8(hl_opaque(a.act) + (long long)m * F + 8 * (t0 + j) + 4 * half,
                 *(const bf16x4*)(su_s + (j * RMAX + m) * 8 + 4 * half));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) ok_s[0] = hl_grid_wait_gen(a.sync, 12, g0, 1, w, a.err) ? 1u : 0u;
  }
  __syncthreads();
  if (!ok_s[0] || !owner) return;
  // ================= down: act rows -> 8 output columns, gated residual
  if (!ctl) {
    const int t = hl_vopaque((int)threadIdx.x);
    const bf16* ap = hl_opaque(a.act);
    for (int m = 0; m < R; ++m)
#pragma unroll
      for (int i = 0; i < F / 8 / NTC; ++i) {   // 576 chunks per row: (m, i) covers chunks [512 i, 512 i + 512) ...
        const int c = i * NTC + t;
        hl_dma16<true>(act_s + m * F + (i * NTC + 64 * wave) * 8, ap + (long long)m * F + c * 8);
      }
    if (F / 8 % NTC) {   // the 64 chunks left per row (576 = 512 + 64): wave 0
      for (int m = 0; m < R; ++m)
        if (wave == 0) hl_dma16<true>(act_s + m * F + (F / 8 / NTC) * NTC * 8, ap + (long long)m * F + ((F / 8 / NTC) * NTC + t) * 8);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (!ctl) {
    const int ln = hl_vopaque(lane);
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW2; ++kk) {
      const int kc = wave * KPW2 + kk;
      const bf16x8 av = (ln & 15) < R ? *(const bf16x8*)(act_s + (ln & 15) * F + kc * 32 + 8 * (ln >> 4)) : zero8;
      acc = mfma16(av, wb[kk], acc);
    }
    *(f32x4*)(red2 + wave * 256 + ln * 4) = acc;
  }
  __syncthreads();
  if (threadIdx.x < RMAX * 8) {   // epi_row8's EPI_RES with the adaLN gate; rows m < R
    const int m = threadIdx.x >> 3, c = threadIdx.x & 7;
    if (m < R) {
      const int n = c + 8 * (d & 1);   // the tile row of column col0 + c
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v) s += red2[v * 256 + (n + 16 * (m >> 2)) * 4 + (m & 3)];
      const float y = rb(bf(gate_s[m * 8 + c]) * rb(s));
      a.out[(long long)m * a.ldx + col0 + c] = tobf(bf(xraw_s[m * 8 + c]) + y);
    }
  }
}

bool head_m16_fits(int H, int F, int R) {
  if (H != hm::H || F != hm::F || R <= 4 || R > hm::RMAX) return false;
  static const bool ok = [] {
    hipFuncAttributes fa{};
    int nb = 0, dev = 0, cus = 0;
    const void* k = (const void*)k_head_m16;
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, hm::TOTAL) != hipSuccess ||
        hipFuncGetAttributes(&fa, k) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, hm::NT, hm::TOTAL) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
    return fa.localSizeBytes == 0 && nb >= 1 && cus >= hm::G;
  }();
  return ok;
}

int launch_head_m16(const HeadM16Args& a, hipStream_t st) {
  if (!head_m16_fits(hm::H, hm::F, a.R)) return 3;
  hipLaunchKernelGGL(k_head_m16, dim3(hm::G), dim3(hm::NT), hm::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
