// Row-wise / element-wise kernels of the generate loop (bf16 storage, fp32 math).
// Each rounds to bf16 exactly where the reference's torch ops round (common.h).
#include "kernels.h"

// ---------------------------------------------------------------- RMSNorm
// y = bf16( bf16( x * rsqrt(mean(x^2) + eps) ) * w )                    (w optional)
// optional adaLN modulate (modular_vibevoice_diffusion_head.py:43-45, :160, :186):
// y = bf16( bf16( y * bf16(1 + scale) ) + shift ),  shift/scale rows of `mod`.
// References: Qwen2RMSNorm / LlamaRMSNorm (weight * x.to(dtype)), diffusion-head
// RMSNorm (:31-38), ConvRMSNorm (modular_vibevoice_tokenizer.py:77-91).

__global__ void __launch_bounds__(256) k_rmsnorm(NormArgs a) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const bf16* x = rm_bf(a.in, m);
  const int nch = a.C >> 3;
  float ss = 0.f;
  for (int c = lane; c < nch; c += 64) {
    bf16x8 v = *(const bf16x8*)(x + c * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)a.C + a.eps);
  bf16* y = a.pack ? (bf16*)a.out.base + (long long)(m >> 4) * a.C * 16 + (m & 15) * 8 : rm_bfw(a.out, m);
  const bf16* md = a.has_mod ? a.mod + (long long)m * a.mod_ld : nullptr;
  for (int c = lane; c < nch; c += 64) {
    bf16x8 v = *(const bf16x8*)(x + c * 8);
    bf16x8 wv, sh, sc;
    if (a.w) wv = *(const bf16x8*)(a.w + c * 8);
    if (md) {
      sh = *(const bf16x8*)(md + a.shift_off + c * 8);
      sc = *(const bf16x8*)(md + a.scale_off + c * 8);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = rb(bf(v[j]) * inv);
      if (a.w) t = rb(t * bf(wv[j]));
      if (md) t = rb(rb(t * rb(1.0f + bf(sc[j]))) + bf(sh[j]));
      o[j] = tobf(t);
    }
    // packed: columns 8c .. 8c+7 are chunk c >> 2, lane (m & 15) + 16 (c & 3) of the row's tile
    *(bf16x8*)(y + (a.pack ? (c >> 2) * 512 + (c & 3) * 128 : c * 8)) = o;
  }
}

// ---------------------------------------------------------------- depthwise causal conv k=7
// Block1D mixer (modular_vibevoice_tokenizer.py:925-933): buf holds, per sample
// slot, KCTX = k-1 history rows (the previous normalised inputs, zero at start)
// followed by this step's T normalised rows.  x is the residual stream (in place):
//   x = bf16( x + bf16( bf16(conv + b) * gamma ) )

__global__ void __launch_bounds__(256) k_dwconv(DwArgs a) {
  const int nch = a.C >> 3;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)a.M * nch) return;
  const int m = (int)(gid / nch), c8 = (int)(gid - (long long)m * nch) * 8;
  const bf16* brow = rm_bf(a.buf, m) + c8;
  float acc[8];
  bf16x8 bb = *(const bf16x8*)(a.b + c8);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int k = 0; k < a.K; ++k) {
    bf16x8 v = *(const bf16x8*)(brow + (long long)k * a.buf.sT);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf(a.w[(c8 + j) * a.K + k]) * bf(v[j]);
  }
  bf16* xp = rm_bfw(a.x, m) + c8;
  bf16x8 xv = *(const bf16x8*)xp;
  bf16x8 gv = *(const bf16x8*)(a.gamma + c8);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = tobf(bf(xv[j]) + rb(rb(acc[j] + bf(bb[j])) * bf(gv[j])));
  *(bf16x8*)xp = o;
}

// ---------------------------------------------------------------- conv C_out = 1 (decoder head)
// TokenizerDecoder.head (:912): SConv1d(C -> 1, k=7).  Writes the audio chunk to
// `out` and, when out2.base != nullptr, also into the semantic encoder's stem
// buffer (the audio chunk is the encoder's input, modeling_vibevoice_inference.py:673).

__global__ void __launch_bounds__(256) k_conv_cout1(Conv1Args a) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= a.M) return;
  const bf16* brow = rm_bf(a.buf, m);
  float acc = 0.f;
  for (int k = 0; k < a.K; ++k) {
    const bf16* r = brow + (long long)k * a.buf.sT;
    const bf16* wk = a.w + k * a.C;
    for (int c = 0; c < a.C; c += 8) {
      bf16x8 v = *(const bf16x8*)(r + c);
      bf16x8 wv = *(const bf16x8*)(wk + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += bf(wv[j]) * bf(v[j]);
    }
  }
  const bf16 y = tobf(acc + bf(a.b[0]));
  *rm_bfw(a.out, m) = y;
  if (a.out2.base) *rm_bfw(a.out2, m) = y;
}

// ---------------------------------------------------------------- conv C_in = 1 (encoder stem)
// TokenizerEncoder stem (:731-733): SConv1d(1 -> C, k=7) over the audio buffer.

__global__ void __launch_bounds__(256) k_conv_cin1(ConvIn1Args a) {
  const int nch = a.C >> 3;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)a.M * nch) return;
  const int m = (int)(gid / nch), c8 = (int)(gid - (long long)m * nch) * 8;
  const bf16* brow = rm_bf(a.buf, m);
  float xin[16];
  for (int k = 0; k < a.K; ++k) xin[k] = bf(brow[(long long)k * a.buf.sT]);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float acc = 0.f;
    for (int k = 0; k < a.K; ++k) acc += bf(a.w[(c8 + j) * a.K + k]) * xin[k];
    o[j] = tobf(acc + bf(a.b[c8 + j]));
  }
  *(bf16x8*)(rm_bfw(a.out, m) + c8) = o;
}

// ---------------------------------------------------------------- streaming-state roll / reset
// After a codec step every conv buffer keeps its last `ctx` rows as the next
// step's history (SConv1d._forward_streaming :364-380 / SConvTranspose1d :538-547):
// rows [T, T+ctx) -> [0, ctx).  mode 1 zeroes rows [0, ctx) instead
// (VibeVoiceTokenizerStreamingCache.set_to_zero, :234-241).

// Forward copy row by row is safe when the regions overlap (T < ctx): row i is
// read before any later iteration overwrites it.  8 channels per thread.
__global__ void __launch_bounds__(256) k_roll(const RollDesc* d, const int* slots, int mode) {
  const RollDesc r = d[blockIdx.x];
  const int slot = slots[blockIdx.y];
  bf16* base = r.base + (long long)slot * r.sB;
  const bf16x8 z8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  if ((r.C & 7) == 0) {
    const int n8 = r.C >> 3;
    for (int e = threadIdx.x; e < r.ctx * n8; e += blockDim.x) {
      const int i = e / n8, c = (e - i * n8) * 8;
      if (r.T >= r.ctx || mode == 1) {
        *(bf16x8*)(base + (long long)i * r.C + c) =
            mode == 0 ? *(const bf16x8*)(base + (long long)(r.T + i) * r.C + c) : z8;
      }
    }
    if (r.T >= r.ctx || mode == 1) return;
  }
  // narrow or overlapping buffers (T < ctx: the source rows overlap the
  // destination rows).  Up to ROLL_REGS rows: each thread loads all its rows
  // into registers first, then stores them, so the ctx loads are in flight
  // together (one memory round trip instead of ctx dependent ones).
  constexpr int ROLL_REGS = 16;
  if (r.ctx <= ROLL_REGS) {
    if ((r.C & 7) == 0) {
      const int n8 = r.C >> 3;
      for (int c = threadIdx.x; c < n8; c += blockDim.x) {
        bf16x8 v[ROLL_REGS];
#pragma unroll
        for (int i = 0; i < ROLL_REGS; ++i)
          if (i < r.ctx) v[i] = *(const bf16x8*)(base + (long long)(r.T + i) * r.C + c * 8);
#pragma unroll
        for (int i = 0; i < ROLL_REGS; ++i)
          if (i < r.ctx) *(bf16x8*)(base + (long long)i * r.C + c * 8) = v[i];
      }
    } else {
      for (int c = threadIdx.x; c < r.C; c += blockDim.x) {
        bf16 v[ROLL_REGS];
#pragma unroll
        for (int i = 0; i < ROLL_REGS; ++i)
          if (i < r.ctx) v[i] = mode == 0 ? base[(long long)(r.T + i) * r.C + c] : tobf(0.f);
#pragma unroll
        for (int i = 0; i < ROLL_REGS; ++i)
          if (i < r.ctx) base[(long long)i * r.C + c] = v[i];
      }
    }
    return;
  }
  // longer contexts: one thread per channel, rows in order
  for (int c = threadIdx.x; c < r.C; c += blockDim.x)
    for (int i = 0; i < r.ctx; ++i)
      base[(long long)i * r.C + c] = mode == 0 ? base[(long long)(r.T + i) * r.C + c] : tobf(0.f);
}

// ---------------------------------------------------------------- small element-wise ops
// latent -> decoder input (modeling_vibevoice_inference.py:651):
//   z = bf16( bf16(latent / scaling) - bias )
__global__ void k_latent_to_dec(int n, int D, const bf16* lat, const bf16* scale, const bf16* bias, RowMap out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * D) return;
  const int m = i / D, d = i - m * D;
  *(rm_bfw(out, m) + d) = tobf(rb(bf(lat[i]) / bf(scale[0])) - bf(bias[0]));
}

// voice-prompt latents (modeling_vibevoice_inference.py:155-159, tokenizer :981-989):
//   z = bf16(mean + bf16(std[v] * noise));  feat = bf16( bf16(z + bias) * scaling )
__global__ void k_vae_features(int rows, int D, int frames, const bf16* mean, const bf16* stdv, const bf16* noise,
                               const bf16* scale, const bf16* bias, bf16* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * D) return;
  const int v = (i / D) / frames;
  const float z = rb(bf(mean[i]) + rb(bf(stdv[v]) * bf(noise[i])));
  out[i] = tobf(rb(z + bf(bias[0])) * bf(scale[0]));
}

// diffusion-head conditioning for a run of diffusion steps at once
// (modular_vibevoice_diffusion_head.py:273-274, :154-155): the condition rows are
// step-invariant and the timesteps are fixed by the schedule, so the adaLN
// input of every step is known up front:
//   out[s * R + r] = bf16(silu(bf16(cond_proj(cond)[r] + t_emb[s])))
__global__ void k_head_cond(int steps, int R, int H, const bf16* condp, const bf16* temb, bf16* out) {
  const int h8 = H >> 3;
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)steps * R * h8) return;
  const int c8 = (int)(i % h8), row = (int)(i / h8), s = row / R, r = row - s * R;
  const bf16x8 cv = *(const bf16x8*)(condp + (long long)r * H + c8 * 8);
  const bf16x8 tv = *(const bf16x8*)(temb + (long long)s * H + c8 * 8);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = tobf(silu_f(rb(bf(cv[j]) + bf(tv[j]))));
  *(bf16x8*)(out + (long long)row * H + c8 * 8) = o;
}

__global__ void k_silu(int n, const bf16* x, bf16* y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = tobf(silu_f(bf(x[i])));
}

// CFG combine + DPM-Solver++ update on the n live rows (sample_speech_tokens
// :717-724; DPMSolverMultistepScheduler.step dpm_solver.py:935-1022).  eps rows
// [0, n) are the conditional and [n, 2n) the unconditional predictions.

__global__ void k_cfg_dpm(int n, int D, DpmCoef k, const bf16* eps, bf16* x, bf16* m1, const float* noise) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * D) return;
  const float c = bf(eps[i]), u = bf(eps[i + n * D]);
  const float v = rb(u + rb(k.cfg * rb(c - u)));
  const float xs = bf(x[i]);
  const float x0 = rb(rb(k.alpha_s * xs) - rb(k.sigma_s * v));
  float out = k.c_x * xs - rb(k.c_d0 * x0);
  if (k.order == 2) {
    const float d1 = rb(k.inv_r0 * rb(x0 - bf(m1[i])));
    out = out - rb(k.c_d1 * d1);
  }
  if (noise) out = out + k.c_n * noise[i];
  x[i] = tobf(out);
  m1[i] = tobf(x0);
}

// gather bf16 rows: dst row i <- src row idx[i]  (embedding lookup, speech-frame scatter)
__global__ void k_gather_rows(int n, int C, const bf16* src, long long lds, const int* idx, RowMap dst) {
  const int nch = C >> 3;
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)n * nch) return;
  const int i = (int)(gid / nch), c8 = (int)(gid - (long long)i * nch) * 8;
  *(bf16x8*)(rm_bfw(dst, i) + c8) = *(const bf16x8*)(src + (long long)(idx ? idx[i] : i) * lds + c8);
}

// sum of the tensor-parallel partial residual streams, written back to every
// rank (the all-reduce of a single-process TP group; fp32 sum, one rounding)
__global__ void k_sum_rows(SumRows s, long long n8) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r = 0; r < s.n; ++r) {
    const bf16x8 v = *(const bf16x8*)(s.p[r] + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf(v[j]);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = tobf(acc[j]);
  for (int r = 0; r < s.n; ++r) *(bf16x8*)(s.p[r] + i * 8) = o;
}

// ================================================================ host launchers
int launch_sum_rows(SumRows s, long long count, hipStream_t st) {
  if (count % 8 || s.n < 1 || s.n > 8) return 1;
  const long long n8 = count / 8;
  hipLaunchKernelGGL(k_sum_rows, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, s, n8);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

static inline int nblk(long long n, int b) { return (int)((n + b - 1) / b); }

int launch_rmsnorm(NormArgs a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (a.C % 8) return 1;
  hipLaunchKernelGGL(k_rmsnorm, dim3(nblk(a.M, 4)), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_dwconv(DwArgs a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (a.C % 8) return 1;
  hipLaunchKernelGGL(k_dwconv, dim3(nblk((long long)a.M * (a.C / 8), 256)), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_conv_cout1(Conv1Args a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (a.C % 8) return 1;
  hipLaunchKernelGGL(k_conv_cout1, dim3(nblk(a.M, 256)), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_conv_cin1(ConvIn1Args a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (a.C % 8 || a.K > 16) return 1;
  hipLaunchKernelGGL(k_conv_cin1, dim3(nblk((long long)a.M * (a.C / 8), 256)), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_roll(const RollDesc* d, int nd, const int* slots, int ns, int mode, hipStream_t st) {
  if (nd <= 0 || ns <= 0) return 0;
  hipLaunchKernelGGL(k_roll, dim3(nd, ns), dim3(256), 0, st, d, slots, mode);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_latent_to_dec(int n, int D, const bf16* lat, const bf16* s, const bf16* b, RowMap out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_latent_to_dec, dim3(nblk(n * D, 256)), dim3(256), 0, st, n, D, lat, s, b, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_vae_features(int rows, int D, int frames, const bf16* mean, const bf16* stdv, const bf16* noise,
                        const bf16* s, const bf16* b, bf16* out, hipStream_t st) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(k_vae_features, dim3(nblk(rows * D, 256)), dim3(256), 0, st, rows, D, frames, mean, stdv,
                     noise, s, b, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_head_cond(int steps, int R, int H, const bf16* condp, const bf16* temb, bf16* out, hipStream_t st) {
  if (H % 8) return 1;
  hipLaunchKernelGGL(k_head_cond, dim3(nblk((long long)steps * R * (H / 8), 256)), dim3(256), 0, st, steps, R, H,
                     condp, temb, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_silu(int n, const bf16* x, bf16* y, hipStream_t st) {
  hipLaunchKernelGGL(k_silu, dim3(nblk(n, 256)), dim3(256), 0, st, n, x, y);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_cfg_dpm(int n, int D, DpmCoef k, const bf16* eps, bf16* x, bf16* m1, const float* noise, hipStream_t st) {
  hipLaunchKernelGGL(k_cfg_dpm, dim3(nblk(n * D, 256)), dim3(256), 0, st, n, D, k, eps, x, m1, noise);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
// element-wise row copy src row i -> dst row i, for destinations with no
// 16-byte alignment (an audio chunk into a conv buffer after its 6-row history)
__global__ void k_copy_rows1(int n, int C, const bf16* src, long long lds, RowMap dst) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)n * C) return;
  const int i = (int)(gid / C), c = (int)(gid - (long long)i * C);
  rm_bfw(dst, i)[c] = src[(long long)i * lds + c];
}
int launch_copy_rows1(int n, int C, const bf16* src, long long lds, RowMap dst, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_copy_rows1, dim3(nblk((long long)n * C, 256)), dim3(256), 0, st, n, C, src, lds, dst);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int launch_gather_rows(int n, int C, const bf16* src, long long lds, const int* idx, RowMap dst, hipStream_t st) {
  if (n <= 0) return 0;
  if (C % 8) return 1;
  hipLaunchKernelGGL(k_gather_rows, dim3(nblk((long long)n * (C / 8), 256)), dim3(256), 0, st, n, C, src, lds, idx,
                     dst);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// RoPE cos / sin table: tab[p][j] = bf16(cosf(p * inv_freq[j])), tab[p][64 + j] =
// bf16(sinf(...)) -- the same fp32 angle and rounding as the q|k|v epilogue's
// inline form (HF Qwen2RotaryEmbedding: fp32 angles, cos / sin cast to bf16,
// transformers modeling_qwen2.py:99-134), computed once per engine
__global__ void k_rope_table(int npos, const float* inv_freq, bf16* tab) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long long)npos * 64) return;
  const int p = (int)(e >> 6), j = (int)(e & 63);
  const float f = (float)p * inv_freq[j];
  tab[(long long)p * 128 + j] = tobf(cosf(f));
  tab[(long long)p * 128 + 64 + j] = tobf(sinf(f));
}

int launch_rope_table(int npos, const float* inv_freq, bf16* tab, hipStream_t st) {
  const long long n = (long long)npos * 64;
  hipLaunchKernelGGL(k_rope_table, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, npos, inv_freq, tab);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
