// σ-VAE codec Block1D (modular_vibevoice_tokenizer.py:667-684, streaming conv
// :327-382) on the streaming decode path:
//   n_t = ConvRMSNorm(x_t)                        -> conv buffer (next steps' history)
//   y_t = x_t + bf16(bf16(dwconv_k7(n)_t + b) * gamma)
//   a_t = ConvRMSNorm_ffn(y_t)
//   out_t = y_t + bf16(ffn_gamma * bf16(fc2(GELU(fc1(a_t)))))
//
//   k_mix   : the front half (n, y, a) for any C <= 2048; fc1 / fc2 then run as
//             GEMMs (gemm.hip), or fc1 takes the mix in its prologue (XF_MIX)
//   k_block : the whole block in one workgroup for the narrow stages
//             (C <= 128: T = 800 / 1600 / 3200 rows per frame), fc1 and fc2 by
//             MFMA with the weights read from L2 and the hidden rows in LDS.
//             Same arithmetic and summation order as k_mix + k_gemm (one fp32
//             accumulator per output, 32-wide K chunks in order): bit-identical.
#include "kernels.h"

// ---------------------------------------------------------------- front half
// A workgroup owns rows [t0, t0 + R) of one sample and all C channels; it
// recomputes the normalised rows of its 6-row halo itself (history rows t < 0
// come from the buffer), so no other workgroup's output is read: the residual
// stream ping-pongs between two buffers.  Rows are handled by groups of
// LPR = min(64, C/8) lanes, 8 channels per lane per chunk; row sums reduce with
// shuffles inside the group.  The launch sizes R so that R * C/8 == 256 conv
// items (one per thread), or R == T with fewer.
// LDS: nrm [R + ctx][C] | ybuf [R][C] | ssp [R + ctx][C/8] | inv [R + ctx].
// TO_LDS: fc1's input rows go to a_lds (row stride a_ld) instead of a.a, and y
// is not stored to a.y (k_block keeps the residual in ybuf).
DEV size_t mix_lds_bytes(int R, int ctx, int C) {
  return (size_t)(2 * R + ctx) * C * sizeof(bf16) + (size_t)(R + ctx) * (C / 8 + 1) * sizeof(float);
}

// Every global load is issued in the kernel's first batch: the per-channel
// operands, the QB row items per thread (branch-free, clamped addresses, so
// the waits are counted), then `issue` (k_block's fc1 / fc2 weights, biases and
// output slot) -- one exposed memory round trip before the LDS phases instead
// of one per phase.  The raw x rows the workgroup owns stay in ybuf for the
// gamma residual (they were re-read from global).  blockDim.x % n8 == 0 (host
// check), so a thread's channel chunk is the same in every loop: c2.
template <bool TO_LDS, int QB, typename Issue>
DEV void mix_rows(const MixArgs& a, unsigned char* smem, bf16* a_lds, int a_ld, Issue&& issue) {
  const int t0 = blockIdx.x * a.R, smp = blockIdx.y;
  const int C = a.C, n8 = C >> 3;
  const int rows = a.R + a.ctx;
  bf16* nrm = (bf16*)smem;                       // [rows][C] normalised inputs of the conv
  bf16* ybuf = nrm + (size_t)rows * C;           // [R][C] raw x rows, then y
  float* ssp = (float*)(ybuf + (size_t)a.R * C); // [rows][n8] partial sums of squares
  float* inv = ssp + (size_t)rows * n8;          // [rows] inverse RMS (x rows, then y rows)
  const bf16* X = a.x + (long long)smp * a.T * C;
  bf16* buf = a.buf + (long long)a.slots[smp] * a.buf_sB;
  const int LPR = n8 < 64 ? n8 : 64;
  const int gi = threadIdx.x / LPR, gl = threadIdx.x - gi * LPR, ng = blockDim.x / LPR;
  // ---- this thread's conv item (row i, chunk c2)
  const int e2 = threadIdx.x;
  const int i2 = e2 / n8, c2 = e2 - i2 * n8;
  const bool own = e2 < a.R * n8 && t0 + i2 < a.T;
  bf16x8 wk[7], bb, gv, wf, wn;
#pragma unroll
  for (int k = 0; k < 7; ++k) wk[k] = *(const bf16x8*)(a.dw_w + (size_t)c2 * 56 + k * 8);
  bb = *(const bf16x8*)(a.dw_b + c2 * 8);
  gv = *(const bf16x8*)(a.gamma + c2 * 8);
  wf = *(const bf16x8*)(a.ffn_norm_w + c2 * 8);
  wn = *(const bf16x8*)(a.norm_w + c2 * 8);
  // ---- phase 1: rows t0 - ctx .. t0 + R - 1 (history rows t < 0 are already
  // normalised in the buffer; halo rows t >= 0 are recomputed from x)
  // QB items per thread per batch: all loads first, then the LDS stores
  const bf16x8 z8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  const int nitem = rows * n8;
  for (int e0 = threadIdx.x, first = 1; e0 < nitem; e0 += QB * blockDim.x, first = 0) {
    bf16x8 v[QB];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int e = e0 + q * blockDim.x;
      const int ee = e < nitem ? e : e0;
      const int i = ee / n8, c = ee - i * n8;
      const int t = t0 - a.ctx + i;
      const bf16* src = t < 0 ? buf + (long long)(a.ctx + t) * C + c * 8 : X + (long long)min(t, a.T - 1) * C + c * 8;
      v[q] = *(const bf16x8*)src;
    }
    if (first) issue();
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int e = e0 + q * blockDim.x;
      if (e < nitem) {
        const int i = e / n8, c = e - i * n8;
        const int t = t0 - a.ctx + i;
        const bf16x8 vq = t < a.T ? v[q] : z8;
        *(bf16x8*)(nrm + i * C + c * 8) = vq;   // history: normalised; else raw, normalised below
        if (i >= a.ctx) *(bf16x8*)(ybuf + (i - a.ctx) * C + c * 8) = vq;
        float ss = 0.f;
        if (t >= 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += bf(vq[j]) * bf(vq[j]);
        }
        ssp[e] = ss;
      }
    }
  }
  __syncthreads();
  for (int i = gi; i < rows && gi < ng; i += ng) {   // row sums in a fixed order
    float ss = 0.f;
    for (int c = gl; c < n8; c += LPR) ss += ssp[i * n8 + c];
    ss = group_sum_n(ss, LPR);   // DPP / permlane (common.h), XF_MIX's wave_sum order at LPR 64
    if (gl == 0) inv[i] = rsqrtf(ss / (float)C + a.eps);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < rows * n8; e += blockDim.x) {
    const int i = e / n8, c = e - i * n8;
    const int t = t0 - a.ctx + i;
    if (t < 0 || t >= a.T) continue;
    const bf16x8 v = *(const bf16x8*)(nrm + i * C + c * 8);
    const float r = inv[i];
    bf16x8 o8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o8[j] = tobf(rb(rb(bf(v[j]) * r) * bf(wn[j])));
    *(bf16x8*)(nrm + i * C + c * 8) = o8;
    if (i >= a.ctx) *(bf16x8*)(buf + (long long)(a.ctx + t) * C + c * 8) = o8;
  }
  __syncthreads();
  // ---- phase 2: depthwise conv + gamma residual for the thread's item
  if (own) {
    const int t = t0 + i2;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const bf16x8 v = *(const bf16x8*)(nrm + (i2 + k) * C + c2 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = j * 7 + k;                 // tap k of channel 8 c2 + j
        acc[j] += bf(wk[f >> 3][f & 7]) * bf(v[j]);
      }
    }
    const bf16x8 xv = *(const bf16x8*)(ybuf + i2 * C + c2 * 8);   // raw x row (phase 1)
    bf16x8 y8;
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y8[j] = tobf(bf(xv[j]) + rb(rb(acc[j] + bf(bb[j])) * bf(gv[j])));
      ss += bf(y8[j]) * bf(y8[j]);
    }
    if (!TO_LDS) *(bf16x8*)(a.y + ((long long)smp * a.T + t) * C + c2 * 8) = y8;
    *(bf16x8*)(ybuf + i2 * C + c2 * 8) = y8;
    ssp[e2] = ss;
  }
  __syncthreads();
  for (int i = gi; i < a.R && gi < ng; i += ng) {
    float ss = 0.f;
    for (int c = gl; c < n8; c += LPR) ss += ssp[i * n8 + c];
    ss = group_sum_n(ss, LPR);
    if (gl == 0) inv[i] = rsqrtf(ss / (float)C + a.eps);
  }
  __syncthreads();
  // ---- FFN pre-norm -> fc1's input row
  if (own) {
    const int t = t0 + i2;
    const bf16x8 y8 = *(const bf16x8*)(ybuf + i2 * C + c2 * 8);
    const float r = inv[i2];
    bf16x8 o8;
#pragma unroll
    for (int j = 0; j < 8; ++j) o8[j] = tobf(rb(rb(bf(y8[j]) * r) * bf(wf[j])));
    if (TO_LDS) *(bf16x8*)(a_lds + i2 * a_ld + c2 * 8) = o8;
    else *(bf16x8*)(a.a + ((long long)smp * a.T + t) * C + c2 * 8) = o8;
  }
}

__global__ void __launch_bounds__(256) k_mix(MixArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mix_rows<false, 4>(a, smem, nullptr, 0, [] {});
}

// ---------------------------------------------------------------- whole block
// After mix_rows: fc1 tiles (16 hidden x 16 rows, one per wave at a time, K = C)
// -> bias, GELU -> hidden rows in LDS; fc2 tiles (16 channels x 16 rows,
// K = 4C) -> bias, ffn_gamma, + y -> out.  Weights are MFMA-packed (weights.py:
// 16 x 32 block = 1 KB) and shared by every workgroup of the launch through L2.
template <int C>
__global__ void __launch_bounds__(256) k_block(BlockArgs b) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int R = 2048 / C, H4 = 4 * C, MT = R / 16;   // rows per workgroup, hidden width, row tiles
  constexpr int a_ld = C + 8, h_ld = H4 + 8;             // +16 B per row against bank conflicts
  constexpr int NTW1 = C / 16, NK1 = C / 32;             // fc1: hidden tiles per wave, K chunks
  constexpr int NK2 = H4 / 32;                           // fc2: K chunks (8 tiles = 2 per wave)
  const MixArgs& a = b.mix;
  const size_t base = (mix_lds_bytes(R, a.ctx, C) + 15) & ~(size_t)15;
  bf16* alds = (bf16*)(smem + base);                     // [R][a_ld]
  bf16* hlds = alds + (size_t)R * a_ld;                  // [R][h_ld]
  const bf16* ybuf = (const bf16*)smem + (size_t)(R + a.ctx) * C;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int t0 = blockIdx.x * R, smp = blockIdx.y;

  // fc1's weights / biases, fc2's biases / gamma and the output row base go out
  // with the mixer's first loads (fc2's weights too while registers allow:
  // C <= 64; at C = 128 they are issued before fc1's MFMAs instead)
  constexpr bool W2_EARLY = C <= 64;
  bf16x8 wf[NTW1][NK1];
  bf16x4 bv1[NTW1];
  bf16x8 w2f[2][NK2];
  bf16x4 bv2[2], gm2[2];
  long long obase = 0;
  auto load_w2 = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = (2 * wave + j) / MT;
#pragma unroll
      for (int c = 0; c < NK2; ++c) w2f[j][c] = *(const bf16x8*)(b.w2 + ((long long)nt * NK2 + c) * 512 + lane * 8);
    }
  };
  auto issue = [&]() {
#pragma unroll
    for (int j = 0; j < NTW1; ++j)
#pragma unroll
      for (int c = 0; c < NK1; ++c)
        wf[j][c] = *(const bf16x8*)(b.w1 + ((long long)(wave * NTW1 + j) * NK1 + c) * 512 + lane * 8);
#pragma unroll
    for (int j = 0; j < NTW1; ++j) bv1[j] = *(const bf16x4*)(b.b1 + (wave * NTW1 + j) * 16 + 4 * g);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = ((2 * wave + j) / MT) * 16 + 4 * g;
      bv2[j] = *(const bf16x4*)(b.b2 + n);
      gm2[j] = *(const bf16x4*)(b.g2 + n);
    }
    obase = rm_off(b.out, smp * a.T);   // row t of this sample: + t * out.sT (host: out.T == T)
    if (W2_EARLY) load_w2();
  };

  mix_rows<true, 2>(a, smem, alds, a_ld, issue);
  if (!W2_EARLY) load_w2();
  __syncthreads();
  if (b.dbg_a)
    for (int e = threadIdx.x; e < R * C / 8; e += blockDim.x) {
      const int i = e / (C / 8), c = e - i * (C / 8);
      if (t0 + i < a.T)
        *(bf16x8*)(b.dbg_a + ((long long)smp * a.T + t0 + i) * C + c * 8) = *(const bf16x8*)(alds + i * a_ld + c * 8);
    }

  // ---- fc1 + GELU -> hidden rows (LDS): wave w owns hidden tiles w*NTW1 .. +NTW1
  {
#pragma unroll
    for (int j = 0; j < NTW1; ++j) {
      const int n = (wave * NTW1 + j) * 16 + 4 * g;
      const bf16x4 bv = bv1[j];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16* xrow = alds + (mt * 16 + r) * a_ld + 8 * g;
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < NK1; ++c) acc = mfma16(wf[j][c], *(const bf16x8*)(xrow + c * 32), acc);
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = tobf(gelu_f(rb(acc[i] + bf(bv[i]))));
        *(bf16x4*)(hlds + (mt * 16 + r) * h_ld + n) = o;
        if (b.dbg_h && t0 + mt * 16 + r < a.T)
          *(bf16x4*)(b.dbg_h + ((long long)smp * a.T + t0 + mt * 16 + r) * H4 + n) = o;
      }
    }
  }
  __syncthreads();
  // ---- fc2 + ffn_gamma + residual -> out: wave w owns tiles 2w, 2w + 1
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tt = 2 * wave + j, nt = tt / MT, mt = tt - nt * MT;
    const bf16* xrow = hlds + (mt * 16 + r) * h_ld + 8 * g;
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NK2; ++c) acc = mfma16(w2f[j][c], *(const bf16x8*)(xrow + c * 32), acc);
    const int m = mt * 16 + r, t = t0 + m;
    if (t >= a.T) continue;
    const int n = nt * 16 + 4 * g;
    const bf16x4 bv = bv2[j];
    const bf16x4 gm = gm2[j];
    const bf16x4 yv = *(const bf16x4*)(ybuf + m * C + n);
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = rb(bf(gm[i]) * rb(acc[i] + bf(bv[i])));
      o[i] = tobf(bf(yv[i]) + v);
    }
    *(bf16x4*)((bf16*)b.out.base + obase + (long long)t * b.out.sT + n) = o;
  }
}

// ================================================================ host launchers
static size_t mix_lds_host(int R, int ctx, int C) {
  return (size_t)(2 * R + ctx) * C * sizeof(bf16) + (size_t)(R + ctx) * (C / 8 + 1) * sizeof(float);
}

int launch_mix(MixArgs a, hipStream_t st) {
  if (a.n <= 0 || a.T <= 0) return 0;
  if (a.C % 8 || a.C > 2048 || 256 % (a.C / 8) || a.ctx != 6) return 1;   // mix_rows: 256 % n8 == 0
  if (a.R * (a.C / 8) != 256 && !(a.R == a.T && a.R * (a.C / 8) < 256)) return 1;   // one conv item per thread
  const size_t lds = mix_lds_host(a.R, a.ctx, a.C);
  if (lds > 65536) return 1;
  hipLaunchKernelGGL(k_mix, dim3((a.T + a.R - 1) / a.R, a.n), dim3(256), lds, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

size_t block_lds(int R, int C) {
  if (C < 32 || C > 128 || C % 32 || R % 16 || R * (C / 8) != 256) return 0;
  const size_t base = (mix_lds_host(R, 6, C) + 15) & ~(size_t)15;
  return base + (size_t)R * (C + 8) * sizeof(bf16) + (size_t)R * (4 * C + 8) * sizeof(bf16);
}

int launch_block(BlockArgs b, hipStream_t st) {
  const MixArgs& a = b.mix;
  if (a.n <= 0 || a.T <= 0) return 0;
  const size_t lds = block_lds(a.R, a.C);
  if (!lds || a.ctx != 6 || lds > 65536 || !b.w1 || !b.w2 || !b.b1 || !b.b2 || !b.g2 || b.out.T != a.T) return 1;
  const dim3 grid((a.T + a.R - 1) / a.R, a.n);
  switch (a.C) {
    case 32: hipLaunchKernelGGL(k_block<32>, grid, dim3(256), lds, st, b); break;
    case 64: hipLaunchKernelGGL(k_block<64>, grid, dim3(256), lds, st, b); break;
    case 128: hipLaunchKernelGGL(k_block<128>, grid, dim3(256), lds, st, b); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
