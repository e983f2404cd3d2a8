// Qwen2 attention for the generate loop: RoPE + KV append, GQA attention over a
// compacted per-row KV cache (split-K "flash decoding" + combine), restricted
// lm_head.  Reference: transformers Qwen2Attention / apply_rotary_pos_emb
// (modeling_qwen2.py:99-134, 150-173, 195-247) as called by VibeVoiceModel.forward
// (vibevoice/modular/modeling_vibevoice.py:169-209).
//
// KV cache layout (one buffer for K, one for V):  [layer][slot][kv_head][ctx][d]
// A row's cache holds only the entries its attention mask keeps, in order, so
// cache index == RoPE position.
#include "kernels.h"


// ---------------------------------------------------------------- RoPE + append
// qkv row: [q (nh*d) | k (nkv*d) | v (nkv*d)] (biases already added, bf16).
// q_embed = bf16(bf16(q*cos) + bf16(rotate_half(q)*sin)), cos/sin = bf16(fp32 cos/sin)

__global__ void __launch_bounds__(256) k_rope_kv(RopeArgs a) {
  const int i = blockIdx.x;
  const int d = a.kv.d, half = d >> 1;
  const bf16* row = a.qkv + (long long)i * a.ld_qkv;
  const int slot = a.slots[i], p = a.pos[i];
  const long long base = (long long)a.layer * a.kv.s_layer + (long long)slot * a.kv.s_slot + (long long)p * d;
  const int nrot = (a.nh + a.nkv) * half;
  for (int e = threadIdx.x; e < nrot; e += blockDim.x) {
    const int h = e / half, j = e - h * half;
    const float f = (float)p * a.inv_freq[j];
    const float cs = rb(cosf(f)), sn = rb(sinf(f));
    const float x1 = bf(row[h * d + j]), x2 = bf(row[h * d + j + half]);
    const bf16 o1 = tobf(rb(x1 * cs) + rb(-x2 * sn));
    const bf16 o2 = tobf(rb(x2 * cs) + rb(x1 * sn));
    if (h < a.nh) {
      a.q_out[(long long)i * a.nh * d + h * d + j] = o1;
      a.q_out[(long long)i * a.nh * d + h * d + j + half] = o2;
    } else {
      bf16* kp = a.kv.k + base + (long long)(h - a.nh) * a.kv.s_head;
      kp[j] = o1;
      kp[j + half] = o2;
    }
  }
  for (int e = threadIdx.x; e < a.nkv * d; e += blockDim.x) {
    const int h = e / d, j = e - h * d;
    a.kv.v[base + (long long)h * a.kv.s_head + j] = row[(a.nh + a.nkv) * d + e];
  }
}

// ---------------------------------------------------------------- attention
// Grid (query row x kv head, split); a workgroup of ATT_NW waves owns keys
// [k0, k1) of its split and hands each WAVE a contiguous sub-range, so short
// contexts need no cross-workgroup merge at all.  Inside a wave: lane = (key
// row kr = lane >> 4, dims dl = 8 * (lane & 15)); 8 keys per sub-chunk (2 per
// key row), K and V of the next sub-chunk prefetched; all G <= 8 query heads of
// the kv head share every K/V load (GQA).  Online softmax (running max / sum,
// fp32) per wave; the waves' (m, l, o) merge through LDS; with nsplit > 1 the
// splits' partials merge in the last-arriving workgroup (agent release /
// ticket / acquire, cdna_hip_programming.md Guideline 16).
constexpr int ATT_NW = 8;           // waves per workgroup (256 VGPRs each: G <= 8 heads fit)
constexpr int ATT_KEYS = 1024;      // keys per workgroup before the launch splits
constexpr int ATT_GMAX = 8;
constexpr int ATT_KC = 64;          // per-row split granularity

template <int G>
__global__ void __launch_bounds__(64 * ATT_NW) k_attn(AttnArgs a) {
  __shared__ float wm[ATT_NW][G], wl[ATT_NW][G];
  __shared__ float wo[ATT_NW][G][128];
  __shared__ float fm[G], fl[G];
  __shared__ unsigned last_flag;
  constexpr int d = 128;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int qi = blockIdx.x / a.nkv, kh = blockIdx.x - qi * a.nkv, split = blockIdx.y;
  const int len = a.pos[qi] + 1;
  // this row's split size: >= a.chunk, all nsplit splits cover len; splits past
  // the row's last key exit at once
  int chunk = (len + a.nsplit - 1) / a.nsplit;
  chunk = max(a.chunk, (chunk + ATT_KC - 1) / ATT_KC * ATT_KC);
  const int nact = (len + chunk - 1) / chunk;
  if (split >= nact) return;
  const int k0 = split * chunk;
  const int k1 = min(len, k0 + chunk);
  // this wave's keys
  const int per = (k1 - k0 + ATT_NW - 1) / ATT_NW;
  const int w0 = k0 + wave * per;
  const int w1 = min(k1, w0 + per);
  const long long cbase = (long long)a.layer * a.kv.s_layer + (long long)a.slots[qi] * a.kv.s_slot +
                          (long long)kh * a.kv.s_head;
  const bf16* K = a.kv.k + cbase;
  const bf16* V = a.kv.v + cbase;
  const int dl = (lane & 15) * 8, kr = lane >> 4;

  float qv[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const bf16x8 q8 = *(const bf16x8*)(a.q + (long long)qi * a.nh * d + (kh * G + h) * d + dl);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[h][e] = bf(q8[e]) * a.scale;
  }
  float o[G][8], m[G], l[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    m[h] = -INFINITY;
    l[h] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;
  }
  const bf16x8 z8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 kf[2], vf[2];
  auto load = [&](int c0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int key = c0 + kr + 4 * j;
      const bool ok = key < w1;
      kf[j] = ok ? *(const bf16x8*)(K + (long long)key * d + dl) : z8;
      vf[j] = ok ? *(const bf16x8*)(V + (long long)key * d + dl) : z8;
    }
  };
  if (w0 < w1) load(w0);
  for (int c0 = w0; c0 < w1; c0 += 8) {
    bf16x8 kc[2], vc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      kc[j] = kf[j];
      vc[j] = vf[j];
    }
    if (c0 + 8 < w1) load(c0 + 8);
    float sc[G][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float kx[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) kx[e] = bf(kc[j][e]);
      const bool ok = c0 + kr + 4 * j < w1;
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) s += qv[h][e] * kx[e];
        s += __shfl_xor(s, 8);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 1);
        sc[h][j] = ok ? s : -INFINITY;
      }
    }
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float mx = fmaxf(sc[h][0], sc[h][1]);
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      const float mnew = fmaxf(m[h], mx);
      const float al = __expf(m[h] - mnew);
      const float p0 = __expf(sc[h][0] - mnew), p1 = __expf(sc[h][1] - mnew);
      float ps = p0 + p1;
      ps += __shfl_xor(ps, 16);
      ps += __shfl_xor(ps, 32);
      l[h] = l[h] * al + ps;
      m[h] = mnew;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[h][e] = o[h][e] * al + p0 * bf(vc[0][e]) + p1 * bf(vc[1][e]);
    }
  }
  // this wave's (m, l, o): sum o over the 4 key rows (lanes +16, +32)
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = o[h][e];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      o[h][e] = v;
    }
  if (lane < 16) {
#pragma unroll
    for (int h = 0; h < G; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) wo[wave][h][dl + e] = o[h][e];
  }
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < G; ++h) {
      wm[wave][h] = m[h];
      wl[wave][h] = l[h];
    }
  }
  __syncthreads();
  // merge the waves: waves with no keys carry m = -inf, l = 0
  if (t < G) {
    float M = -INFINITY;
    for (int w = 0; w < ATT_NW; ++w) M = fmaxf(M, wm[w][t]);
    float L = 0.f;
    for (int w = 0; w < ATT_NW; ++w) L += wm[w][t] == -INFINITY ? 0.f : __expf(wm[w][t] - M) * wl[w][t];
    fm[t] = M;
    fl[t] = L;
  }
  __syncthreads();
  float res[(G * 128 + 64 * ATT_NW - 1) / (64 * ATT_NW)];
  int ne = 0;
  for (int e = t; e < G * d; e += 64 * ATT_NW, ++ne) {
    const int h = e / d, j = e - h * d;
    float s = 0.f;
    for (int w = 0; w < ATT_NW; ++w)
      if (wm[w][h] != -INFINITY) s += __expf(wm[w][h] - fm[h]) * wo[w][h][j];
    res[ne] = s;
  }
  if (nact == 1) {
    ne = 0;
    for (int e = t; e < G * d; e += 64 * ATT_NW, ++ne) {
      const int h = e / d, j = e - h * d;
      a.out[(long long)qi * a.nh * d + (kh * G + h) * d + j] = tobf(res[ne] / fl[h]);
    }
    return;
  }
  ne = 0;
  for (int e = t; e < G * d; e += 64 * ATT_NW, ++ne) {
    const int h = e / d, j = e - h * d;
    const long long pidx = ((long long)qi * a.nh + kh * G + h) * a.nsplit + split;
    a.part_o[pidx * d + j] = res[ne];
    if (j == 0) {
      a.part_ml[pidx * 2] = fm[h];
      a.part_ml[pidx * 2 + 1] = fl[h];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned* ctr = a.counters + blockIdx.x;
    const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = tk == (unsigned)(nact - 1);
    if (last_flag) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!last_flag) return;
  // merge the splits: out = sum_s e^{m_s - M} o_s / sum_s e^{m_s - M} l_s
  for (int e = t; e < G * d; e += 64 * ATT_NW) {
    const int h = e / d, j = e - h * d;
    const long long p0 = ((long long)qi * a.nh + kh * G + h) * a.nsplit;
    float M = -INFINITY;
    for (int s2 = 0; s2 < nact; ++s2) M = fmaxf(M, a.part_ml[(p0 + s2) * 2]);
    float num = 0.f, den = 0.f;
    for (int s2 = 0; s2 < nact; ++s2) {
      const float w = __expf(a.part_ml[(p0 + s2) * 2] - M);
      num += w * a.part_o[(p0 + s2) * d + j];
      den += w * a.part_ml[(p0 + s2) * 2 + 1];
    }
    a.out[(long long)qi * a.nh * d + (kh * G + h) * d + j] = tobf(num / den);
  }
}

// ---------------------------------------------------------------- restricted lm_head
// Only the valid control tokens can win the constrained argmax
// (VibeVoiceTokenConstraintProcessor, modeling_vibevoice_inference.py:54-67,
// :405-419, :494-507), so only those lm_head rows are computed:
//   logits[r][j] = bf16( h[r] . W[ids[j]] )   (bf16 Linear output, then .float())
__global__ void __launch_bounds__(256) k_lmhead_ids(int R, int H, const bf16* h, long long ldh, const bf16* W,
                                                    const int* ids, int nid, float* out) {
  const int r = blockIdx.x, j = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (j >= nid) return;
  const bf16* x = h + (long long)r * ldh;
  const bf16* w = W + (long long)ids[j] * H;
  float s = 0.f;
  for (int c = lane * 8; c < H; c += 512) {
    bf16x8 a = *(const bf16x8*)(x + c), b = *(const bf16x8*)(w + c);
#pragma unroll
    for (int t = 0; t < 8; ++t) s += bf(a[t]) * bf(b[t]);
  }
  s = wave_sum(s);
  if (lane == 0) out[r * nid + j] = rb(s);
}

// final norm + restricted lm_head over gathered rows: hidden_out[i] =
// Qwen2 norm(h[idx[i]]) (the last_hidden_state the diffusion head is conditioned
// on, modeling_vibevoice_inference.py:641-648), logits[i][j] = bf16(hidden . W[ids[j]]).
__global__ void __launch_bounds__(256) k_final_head(int H, const bf16* h, const int* idx, const bf16* norm_w,
                                                    float eps, bf16* hid, const bf16* W, const int* ids, int nid,
                                                    float* logits) {
  __shared__ float red[4][8];
  const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bf16* x = h + (long long)(idx ? idx[i] : i) * H;
  const int nch = H >> 3;
  // one workgroup per row, thread t owns elements [8t, 8t+8)
  float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float ss = 0.f;
  if (t < nch) {
    const bf16x8 x8 = *(const bf16x8*)(x + t * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = bf(x8[j]);
      ss += v[j] * v[j];
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wave][0] = ss;
  __syncthreads();
  ss = red[0][0] + red[1][0] + red[2][0] + red[3][0];
  const float inv = rsqrtf(ss / (float)H + eps);
  float part[4] = {0.f, 0.f, 0.f, 0.f};
  if (t < nch) {
    const bf16x8 w8 = *(const bf16x8*)(norm_w + t * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = rb(rb(v[j] * inv) * bf(w8[j]));
      o[j] = tobf(v[j]);
    }
    *(bf16x8*)(hid + (long long)i * H + t * 8) = o;
    for (int q = 0; q < nid; ++q) {
      const bf16x8 l8 = *(const bf16x8*)(W + (long long)ids[q] * H + t * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) part[q] += v[j] * bf(l8[j]);
    }
  }
  __syncthreads();
  for (int q = 0; q < nid; ++q) {
    const float s = wave_sum(part[q]);
    if (lane == 0) red[wave][1 + q] = s;
  }
  __syncthreads();
  if (t < nid) logits[i * nid + t] = rb(red[0][1 + t] + red[1][1 + t] + red[2][1 + t] + red[3][1 + t]);
}

// ================================================================ host launchers
int launch_final_head(int R, int H, const bf16* h, const int* idx, const bf16* norm_w, float eps, bf16* hidden_out,
                      const bf16* W, const int* ids, int nid, float* logits, hipStream_t st) {
  if (R <= 0) return 0;
  if (H % 8 || H / 8 > 256 || nid > 4 || (nid > 0 && (!W || !ids || !logits))) return 1;
  hipLaunchKernelGGL(k_final_head, dim3(R), dim3(256), 0, st, H, h, idx, norm_w, eps, hidden_out, W, ids, nid,
                     logits);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int launch_rope_kv(RopeArgs a, hipStream_t st) {
  if (a.R <= 0) return 0;
  if (a.kv.d != 128) return 1;
  hipLaunchKernelGGL(k_rope_kv, dim3(a.R), dim3(256), 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Launch plan for keys up to max_len: aim for ~1024 workgroups over
// (rows x kv heads x splits), never below 64 keys per split, at most 64
// splits (merge cost).  Each row then sizes its own splits from its length
// (k_attn), so a plan made for max_ctx serves every step of a captured graph.
// Launch plan for keys up to max_len: one workgroup per (row, kv head) takes up
// to ATT_KEYS keys (split over its 8 waves); longer contexts split the keys
// over workgroups (<= 64).  Each row sizes its own splits from its length
// (k_attn), so a plan made for max_ctx serves every step of a captured graph.
int attn_plan(int nq, int nkv, int max_len, int* chunk) {
  (void)nq;
  (void)nkv;
  int ns = (max_len + ATT_KEYS - 1) / ATT_KEYS;
  if (ns > 64) ns = 64;
  if (ns < 1) ns = 1;
  *chunk = ATT_KC;
  return ns;
}

int launch_attn(AttnArgs a, hipStream_t st) {
  if (a.nq <= 0) return 0;
  if (a.kv.d != 128 || a.nh % a.nkv || a.nh / a.nkv > ATT_GMAX || a.chunk % ATT_KC) return 1;
  if (a.nsplit > 1 && (!a.part_o || !a.part_ml || !a.counters)) return 1;
  dim3 grid(a.nq * a.nkv, a.nsplit);
  const dim3 blk(64 * ATT_NW);
  switch (a.nh / a.nkv) {
    case 1: hipLaunchKernelGGL(k_attn<1>, grid, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_attn<2>, grid, blk, 0, st, a); break;
    case 3: hipLaunchKernelGGL(k_attn<3>, grid, blk, 0, st, a); break;
    case 4: hipLaunchKernelGGL(k_attn<4>, grid, blk, 0, st, a); break;
    case 5: hipLaunchKernelGGL(k_attn<5>, grid, blk, 0, st, a); break;
    case 6: hipLaunchKernelGGL(k_attn<6>, grid, blk, 0, st, a); break;
    case 7: hipLaunchKernelGGL(k_attn<7>, grid, blk, 0, st, a); break;
    default: hipLaunchKernelGGL(k_attn<8>, grid, blk, 0, st, a); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int launch_lmhead_ids(int R, int H, const bf16* h, long long ldh, const bf16* W, const int* ids, int nid, float* out,
                      hipStream_t st) {
  if (R <= 0) return 0;
  if (H % 8 || nid > 4) return 1;
  hipLaunchKernelGGL(k_lmhead_ids, dim3(R), dim3(256), 0, st, R, H, h, ldh, W, ids, nid, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---------------------------------------------------------------- KV entry copy
// cache[slot][*][dst] = cache[slot][*][src] for every layer / kv head (K and V).
// Used for the reference's negative-stream shift whose KV boundary test
// (modeling_vibevoice_inference.py:628) differs from the mask's (:618): when
// it leaves the KV unshifted, the just-computed entry takes the place of the
// previous one.
__global__ void __launch_bounds__(256) k_kv_copy(KVLayout kv, int n_layers, int nkv, const int* slots,
                                                 const int* src, const int* dst) {
  const int i = blockIdx.x;
  const int d = kv.d;
  const int per = n_layers * nkv * d;
  for (int e = threadIdx.x; e < per; e += blockDim.x) {
    const int l = e / (nkv * d), r = e - l * nkv * d, h = r / d, j = r - h * d;
    const long long b = (long long)l * kv.s_layer + (long long)slots[i] * kv.s_slot + (long long)h * kv.s_head + j;
    kv.k[b + (long long)dst[i] * d] = kv.k[b + (long long)src[i] * d];
    kv.v[b + (long long)dst[i] * d] = kv.v[b + (long long)src[i] * d];
  }
}

int launch_kv_copy(KVLayout kv, int n_layers, int nkv, int n, const int* slots, const int* src, const int* dst,
                   hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_kv_copy, dim3(n), dim3(256), 0, st, kv, n_layers, nkv, slots, src, dst);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
