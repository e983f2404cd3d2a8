// The diffusion head's step boundary in ONE launch at 2n <= 16 rows (B <= 8):
// step s's final layer -> CFG + DPM-Solver++ update of the latents -> step
// s+1's noisy_images_proj of the new latents (prediction_head's FinalLayer and
// noisy_images_proj, modular_vibevoice_diffusion_head.py:254-280;
// sample_speech_tokens' CFG + DPMSolverMultistepScheduler.step,
// modeling_vibevoice_inference.py:712-725, dpm_solver.py:935-1022).
//
// Per op these were two GEMV launches per diffusion step, 7.1 us (final + DPM
// epilogue, 196 KB of weights over 4 tiles) and 5.2 us (noisy, 196 KB over 96
// tiles): round trips, not bytes.  Here 24 workgroups of 8 waves each compute
// the whole final layer (the 196 KB come from the Infinity Cache / L2: the head's
// weights stay resident across the S steps), so every workgroup holds the new
// latents without a hand-off, then its 4 noisy tiles.  Workgroup 0 writes the
// new latents and DPM history; the caller double-buffers them and the state
// rows (a launch reads lat / m1 / x and writes lat_out / m1_out / xo: no
// workgroup may overwrite what another has yet to read).
// Arithmetic: xform<XF_NORM>'s (no norm weight, adaLN modulate), epi_dpm's
// term for term, EPI_STORE for noisy; MFMA sums in another order than the GEMV
// kernels' (tests: within bf16 of them).
#include "persist_dev.h"

namespace hf {
constexpr int H = 1536, D = 64, RMAX = 16, NW = 8, NT = NW * 64;
constexpr int NOWN = 192;                       // k_head_m16's down owners (8 columns each)
constexpr int KC = H / 32, KPW = KC / NW;       // 48 k-blocks, 6 per wave
constexpr int TF = D / 16, TN = H / 16;         // 4 final tiles, 96 noisy tiles
constexpr int G = 24, TPG = TN / G;             // 24 workgroups x 4 noisy tiles
constexpr int XST = H + 8;
constexpr int XS = 0, XS_B = 16 * XST * 2;      // normalised rows (16: the MFMA's padded rows)
constexpr int SH = XS + XS_B, SH_B = RMAX * H * 2;
constexpr int SC = SH + SH_B, SC_B = RMAX * H * 2;
constexpr int RED = SH, RED_B = NW * TF * 256 * 4;   // over shift / scale once they are consumed
constexpr int LAT = SC + SC_B, LAT_B = 16 * D * 2;     // new latents, as noisy's B rows [16][64]
constexpr int SM = LAT + LAT_B, SM_B = 64;
constexpr int TOTAL = SM + SM_B;
static_assert(TOTAL <= 160 * 1024 && TPG * G == TN && RED_B <= SH_B + SC_B, "head fin geometry");
}  // namespace hf

__global__ void __launch_bounds__(hf::NT) k_head_fin(HeadFinArgs a) {
  using namespace hf;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + XS);
  bf16* sh_s = (bf16*)(smem + SH);
  bf16* sc_s = (bf16*)(smem + SC);
  float* red = (float*)(smem + RED);
  bf16* lat_s = (bf16*)(smem + LAT);
  float* inv_s = (float*)(smem + SM);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, w = blockIdx.x, R = a.R, n = a.n;
  const int r16 = lane & 15, g4 = lane >> 4;
  const int ln = hl_vopaque(lane);

  // ---- the A side (x rows, adaLN shift / scale) by LDS DMA, then the weights:
  // the final tiles' k-blocks [6 wave, + 6), this wave's noisy k-block
  // (the R rows only: rows >= R are zeroed by the modulate; loading 16 rows at
  // R = 2 queued 126 KB of redundant reads ahead of the weights)
  for (int q = wave; q < R * 3 * 3; q += NW) {   // (row, x | shift | scale, 64-chunk piece)
    const int m = q / 9, k = (q / 3) % 3, i = q % 3, mm = min(m, R - 1);
    const bf16* src = k == 0 ? a.x + (long long)mm * H
                             : a.mod + (long long)mm * a.ldmod + (k == 1 ? a.shift_off : a.scale_off);
    bf16* dst = k == 0 ? xs + m * XST : (k == 1 ? sh_s : sc_s) + m * H;
    hl_dma16<false>(dst + i * 512, src + (i * 64 + ln) * 8);
  }
  bf16x8 wf[TF][KPW], wn[2];
#pragma unroll
  for (int t = 0; t < TF; ++t)
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) wf[t][kk] = hl_ld(hl_opaque(a.fw) + ((long long)t * KC + wave * KPW + kk) * 512 + ln * 8);
  // noisy: wave v < 4 owns tile TPG w + v (both k-blocks)
  const int nt = TPG * w + (wave & 3);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) wn[kk] = hl_ld(hl_opaque(a.nw) + ((long long)nt * 2 + kk) * 512 + ln * 8);
  asm volatile("s_waitcnt vmcnt(26)" ::: "memory");   // this wave's A-side DMA (24 + 2 weight loads younger)
  __syncthreads();
  for (int m = wave; m < R; m += NW) {   // inverse RMS (row_inv's order)
    float ss = 0.f;
    for (int c = ln; c < H / 8; c += 64) {
      const bf16x8 v = *(const bf16x8*)(xs + m * XST + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
    }
    ss = wave_sum(ss);
    if (ln == 0) inv_s[m] = rsqrtf(ss / (float)H + a.eps);
  }
  __syncthreads();
  for (int e = hl_vopaque((int)threadIdx.x); e < 16 * (H / 8); e += NT) {   // xform<XF_NORM> (modulate), in place
    const int m = e / (H / 8), c = e - m * (H / 8);
    bf16x8 o;
    if (m < R) {
      const bf16x8 xv = *(const bf16x8*)(xs + m * XST + c * 8);
      const bf16x8 sh = *(const bf16x8*)(sh_s + m * H + c * 8), sc = *(const bf16x8*)(sc_s + m * H + c * 8);
      const float inv = inv_s[m];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = rb(bf(xv[j]) * inv);
        t = rb(rb(t * rb(1.0f + bf(sc[j]))) + bf(sh[j]));
        o[j] = tobf(t);
      }
    } else {
      o = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
    *(bf16x8*)(xs + m * XST + c * 8) = o;
  }
  __syncthreads();
  // ---- the final layer: D[n][m], A = the weight tile, B = the rows; 8 K slices -> LDS
#pragma unroll
  for (int t = 0; t < TF; ++t) {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int kc = wave * KPW + kk;
      acc = mfma16(wf[t][kk], *(const bf16x8*)(xs + r16 * XST + kc * 32 + 8 * g4), acc);
    }
    *(f32x4*)(red + ((wave * TF + t) * 64 + lane) * 4) = acc;
  }
  __syncthreads();
  if (wave < TF) {   // tile t = wave: the K slices in order, then epi_dpm (lane: row m = lane & 15, dims 16 t + 4 g + i)
    const int t = wave, n0 = 16 * t;
    float e[4], u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
#pragma unroll
      for (int v = 0; v < NW; ++v) s += red[((v * TF + t) * 64 + lane) * 4 + i];
      e[i] = rb(s);   // final_layer.linear output (bf16, no bias)
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = __shfl(e[i], (lane + n) & 63);
    if (r16 < n) {
      const DpmCoef& k = a.k;
      const long long off = (long long)r16 * D + n0 + 4 * g4;
      const bf16x4 xv = *(const bf16x4*)(a.lat + off);
      const bf16x4 mv = *(const bf16x4*)(a.m1 + off);
      bf16x4 xo, mo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float c = e[i], un = u[i];
        const float vv = rb(un + rb(k.cfg * rb(c - un)));
        const float xsv = bf(xv[i]);
        const float x0 = rb(rb(k.alpha_s * xsv) - rb(k.sigma_s * vv));
        float out = k.c_x * xsv - rb(k.c_d0 * x0);
        if (k.order == 2) {
          const float d1 = rb(k.inv_r0 * rb(x0 - bf(mv[i])));
          out = out - rb(k.c_d1 * d1);
        }
        if (a.noise) out = out + k.c_n * a.noise[off + i];
        xo[i] = tobf(out);
        mo[i] = tobf(x0);
      }
      // noisy's B rows: row m reads latent row m % n (rows m and m + n)
      for (int m = r16; m < 16; m += n) *(bf16x4*)(lat_s + m * D + n0 + 4 * g4) = m < R ? xo : (bf16x4){0, 0, 0, 0};
      if (w == 0) {   // (into the other buffers: every workgroup reads the old ones)
        *(bf16x4*)(a.lat_out + off) = xo;
        *(bf16x4*)(a.m1_out + off) = mo;
      }
    }
  }
  __syncthreads();
  // ---- noisy_images_proj of the new latents
  if (R > 4) {
    // k_head_noisy16's arithmetic (fp32 fmaf in k order, bf16 store) and its row
    // partial sums of squares per 8-column owner, which layer 0's distributed A
    // side reads: owners [8 TPG w, + 8 TPG), thread (owner, row m, column c)
    for (int t = threadIdx.x; t < 2 * TPG * 128; t += NT) {
      const int d = 2 * TPG * w + (t >> 7), m = (t & 127) >> 3, c = t & 7, j = 8 * d + c;
      float q = 0.f;
      if (m < R) {
        float acc = 0.f;
        for (int k = 0; k < D; k += 8) {
          const bf16x8 wv = *(const bf16x8*)hl_packed(a.nw, D, j, k), xv = *(const bf16x8*)(lat_s + m * D + k);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc = fmaf(bf(xv[e]), bf(wv[e]), acc);
        }
        const bf16 ov = tobf(acc);
        a.xo[(long long)m * H + j] = ov;
        q = bf(ov) * bf(ov);
      }
      q += __shfl_xor(q, 1);
      q += __shfl_xor(q, 2);
      q += __shfl_xor(q, 4);
      if (a.ssp && c == 0 && m < R) a.ssp[m * NOWN + d] = q;
    }
    return;
  }
  // 2n <= 4 rows: wave v < 4, tile TPG w + v, MFMA (EPI_STORE)
  if (wave < TPG) {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) acc = mfma16(wn[kk], *(const bf16x8*)(lat_s + r16 * D + kk * 32 + 8 * g4), acc);
    if (r16 < R) {
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = tobf(acc[i]);
      *(bf16x4*)(a.xo + (long long)r16 * H + 16 * nt + 4 * g4) = o;
    }
  }
}

bool head_fin_fits(int H, int D, int R) {
  static_assert(2 * hf::TPG * 8 * hf::G == hf::NOWN * 8, "owners x columns");
  return H == hf::H && D == hf::D && R >= 2 && R <= hf::RMAX;
}

int launch_head_fin(const HeadFinArgs& a, hipStream_t st) {
  if (!head_fin_fits(hf::H, hf::D, a.R) || 2 * a.n != a.R || a.x == a.xo || a.lat == a.lat_out || a.m1 == a.m1_out)
    return 3;
  static const bool attr =
      hipFuncSetAttribute((const void*)k_head_fin, hipFuncAttributeMaxDynamicSharedMemorySize, hf::TOTAL) == hipSuccess;
  if (!attr) return 2;
  hipLaunchKernelGGL(k_head_fin, dim3(hf::G), dim3(hf::NT), hf::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
