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
// Grid (query row x kv head, split).  A workgroup owns keys [k0, k1) of its
// split, walks them in 64-key sub-chunks with an online softmax (running max /
// sum per query head, fp32), and all ATT_GMAX <= 8 query heads of the kv head
// share each K/V load (GQA).  Thread t owns dims dl = 8*(t&15) and keys
// kr + 16j (kr = t>>4, j < 4) of a sub-chunk: 4 x 16-B K loads and 4 x 16-B V
// loads per thread, all issued together and the next sub-chunk prefetched.
// With nsplit > 1 every split stores (o, m, l) partials and the last arriver of
// the (row, kv head) group — agent-scope release / ticket / acquire
// (cdna_hip_programming.md Guideline 16) — merges them, so decode attention is
// one launch per layer.
constexpr int ATT_KC = 64;
constexpr int ATT_GMAX = 8;

template <int G>
__global__ void __launch_bounds__(256) k_attn(AttnArgs a) {
  __shared__ float sc[G][ATT_KC];
  __shared__ float red[4][G][128];
  __shared__ float mrun[G], lrun[G], alpha[G];
  __shared__ unsigned last_flag;
  constexpr int d = 128;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int qi = blockIdx.x / a.nkv, kh = blockIdx.x - qi * a.nkv, split = blockIdx.y;
  const int len = a.pos[qi] + 1;
  // this row's split size: >= a.chunk (the launch plan's floor), all nsplit
  // splits cover len; splits past the row's last key exit at once
  int chunk = (len + a.nsplit - 1) / a.nsplit;
  chunk = max(a.chunk, (chunk + ATT_KC - 1) / ATT_KC * ATT_KC);
  const int nact = (len + chunk - 1) / chunk;
  if (split >= nact) return;
  const int k0 = split * chunk;
  const int k1 = min(len, k0 + chunk);
  const long long cbase = (long long)a.layer * a.kv.s_layer + (long long)a.slots[qi] * a.kv.s_slot +
                          (long long)kh * a.kv.s_head;
  const bf16* K = a.kv.k + cbase;
  const bf16* V = a.kv.v + cbase;
  const int dl = (t & 15) * 8, kr = t >> 4;

  float qv[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    const bf16x8 q8 = *(const bf16x8*)(a.q + (long long)qi * a.nh * d + (kh * G + h) * d + dl);
#pragma unroll
    for (int e = 0; e < 8; ++e) qv[h][e] = bf(q8[e]) * a.scale;
  }
  float o[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[h][e] = 0.f;
  if (t < G) {
    mrun[t] = -INFINITY;
    lrun[t] = 0.f;
  }
  const bf16x8 z8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 kf[4], vf[4];
  auto load = [&](int c0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = c0 + kr + 16 * j;
      const bool ok = key < k1;
      kf[j] = ok ? *(const bf16x8*)(K + (long long)key * d + dl) : z8;
      vf[j] = ok ? *(const bf16x8*)(V + (long long)key * d + dl) : z8;
    }
  };
  if (k0 < k1) load(k0);
  for (int c0 = k0; c0 < k1; c0 += ATT_KC) {
    const int nk = min(ATT_KC, k1 - c0);
    bf16x8 kc[4], vc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      kc[j] = kf[j];
      vc[j] = vf[j];
    }
    if (c0 + ATT_KC < k1) load(c0 + ATT_KC);   // prefetch the next sub-chunk
    // scores s[h][key] = (q*scale) . k
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float kx[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) kx[e] = bf(kc[j][e]);
#pragma unroll
      for (int h = 0; h < G; ++h) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) s += qv[h][e] * kx[e];
        s += __shfl_xor(s, 8);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 1);
        if ((t & 15) == 0) sc[h][kr + 16 * j] = s;
      }
    }
    __syncthreads();
    // online softmax update, one wave per head
    for (int h = wave; h < G; h += 4) {
      const float s = lane < nk ? sc[h][lane] : -INFINITY;
      const float mnew = fmaxf(mrun[h], wave_max(s));
      const float p = lane < nk ? __expf(s - mnew) : 0.f;
      sc[h][lane] = p;
      const float sum = wave_sum(p);
      if (lane == 0) {
        const float al = __expf(mrun[h] - mnew);
        alpha[h] = al;
        lrun[h] = lrun[h] * al + sum;
        mrun[h] = mnew;
      }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float al = alpha[h];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[h][e] *= al;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kk = kr + 16 * j;
      if (kk < nk) {
        float vx[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) vx[e] = bf(vc[j][e]);
#pragma unroll
        for (int h = 0; h < G; ++h) {
          const float p = sc[h][kk];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[h][e] += p * vx[e];
        }
      }
    }
    __syncthreads();
  }
  // reduce the 16 key rows: 4 inside the wave (lanes +16, +32), 4 waves via LDS
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
      for (int e = 0; e < 8; ++e) red[wave][h][dl + e] = o[h][e];
  }
  __syncthreads();
  if (nact == 1) {
    for (int e = t; e < G * d; e += 256) {
      const int h = e / d, j = e - h * d;
      const float s = red[0][h][j] + red[1][h][j] + red[2][h][j] + red[3][h][j];
      a.out[(long long)qi * a.nh * d + (kh * G + h) * d + j] = tobf(s / lrun[h]);
    }
    return;
  }
  for (int e = t; e < G * d; e += 256) {
    const int h = e / d, j = e - h * d;
    const long long pidx = ((long long)qi * a.nh + kh * G + h) * a.nsplit + split;
    a.part_o[pidx * d + j] = red[0][h][j] + red[1][h][j] + red[2][h][j] + red[3][h][j];
    if (j == 0) {
      a.part_ml[pidx * 2] = mrun[h];
      a.part_ml[pidx * 2 + 1] = lrun[h];
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
  for (int e = t; e < G * d; e += 256) {
    const int h = e / d, j = e - h * d;
    const long long p0 = ((long long)qi * a.nh + kh * G + h) * a.nsplit;
    float M = -INFINITY;
    for (int s = 0; s < nact; ++s) M = fmaxf(M, a.part_ml[(p0 + s) * 2]);
    float num = 0.f, den = 0.f;
    for (int s = 0; s < nact; ++s) {
      const float m = a.part_ml[(p0 + s) * 2];
      const float w = __expf(m - M);
      num += w * a.part_o[(p0 + s) * d + j];
      den += w * a.part_ml[(p0 + s) * 2 + 1];
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

// ================================================================ host launchers
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
int attn_plan(int nq, int nkv, int max_len, int* chunk) {
  const int groups = nq * nkv;
  int want = 1024 / groups;
  if (want < 1) want = 1;
  int ns = (max_len + ATT_KC - 1) / ATT_KC;
  if (ns > want) ns = want;
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
  switch (a.nh / a.nkv) {
    case 1: hipLaunchKernelGGL(k_attn<1>, grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_attn<2>, grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL(k_attn<3>, grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL(k_attn<4>, grid, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL(k_attn<5>, grid, dim3(256), 0, st, a); break;
    case 6: hipLaunchKernelGGL(k_attn<6>, grid, dim3(256), 0, st, a); break;
    case 7: hipLaunchKernelGGL(k_attn<7>, grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(k_attn<8>, grid, dim3(256), 0, st, a); break;
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
