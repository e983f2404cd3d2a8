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
// One workgroup = (query row, kv head, key split).  Query row i attends to keys
// [0, len[i]) of cache slot slots[i].  softmax(q k^T / sqrt(d)) in fp32.
constexpr int ATT_CHUNK = 256;
constexpr int ATT_GMAX = 8;


__global__ void __launch_bounds__(256) k_attn(AttnArgs a) {
  __shared__ float sc[ATT_GMAX][ATT_CHUNK];
  __shared__ float ored[4][ATT_GMAX][128];
  __shared__ float mrow[ATT_GMAX], lrow[ATT_GMAX];
  const int d = 128;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int qi = blockIdx.x / a.nkv, kh = blockIdx.x - qi * a.nkv, split = blockIdx.y;
  const int G = a.nh / a.nkv;
  const int len = a.pos[qi] + 1;
  const int k0 = split * ATT_CHUNK;
  const int nk = min(ATT_CHUNK, len - k0);
  const long long cbase = (long long)a.layer * a.kv.s_layer + (long long)a.slots[qi] * a.kv.s_slot +
                          (long long)kh * a.kv.s_head;
  const bf16* K = a.kv.k + cbase;
  const bf16* V = a.kv.v + cbase;

  if (nk > 0) {
    // phase 1: scores; 16 lanes per key, 8 dims per lane
    const int sub = lane >> 4, dl = (lane & 15) * 8;
    float qv[ATT_GMAX][8];
#pragma unroll
    for (int h = 0; h < ATT_GMAX; ++h) {
      if (h >= G) break;
      bf16x8 t = *(const bf16x8*)(a.q + (long long)qi * a.nh * d + (kh * G + h) * d + dl);
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[h][j] = bf(t[j]);
    }
    for (int kk = wave * 4 + sub; kk < nk; kk += 16) {
      bf16x8 kv8 = *(const bf16x8*)(K + (long long)(k0 + kk) * d + dl);
      float kf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[j] = bf(kv8[j]);
#pragma unroll
      for (int h = 0; h < ATT_GMAX; ++h) {
        if (h >= G) break;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += qv[h][j] * kf[j];
        s += __shfl_xor(s, 8);
        s += __shfl_xor(s, 4);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 1);
        if ((lane & 15) == 0) sc[h][kk] = s * a.scale;
      }
    }
  }
  __syncthreads();
  // phase 2: per-head max / exp / sum over this chunk
  for (int h = wave; h < G; h += 4) {
    float mx = -INFINITY;
    for (int k = lane; k < nk; k += 64) mx = fmaxf(mx, sc[h][k]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int k = lane; k < nk; k += 64) {
      const float p = __expf(sc[h][k] - mx);
      sc[h][k] = p;
      sum += p;
    }
    sum = wave_sum(sum);
    if (lane == 0) { mrow[h] = mx; lrow[h] = sum; }
  }
  __syncthreads();
  // phase 3: o[h][dim] = sum_k p[h][k] v[k][dim]; lane owns dims 2l, 2l+1; waves split keys
  float o[ATT_GMAX][2];
#pragma unroll
  for (int h = 0; h < ATT_GMAX; ++h) o[h][0] = o[h][1] = 0.f;
  for (int k = wave; k < nk; k += 4) {
    const bf16* vr = V + (long long)(k0 + k) * d + 2 * lane;
    const float v0 = bf(vr[0]), v1 = bf(vr[1]);
#pragma unroll
    for (int h = 0; h < ATT_GMAX; ++h) {
      if (h >= G) break;
      const float p = sc[h][k];
      o[h][0] += p * v0;
      o[h][1] += p * v1;
    }
  }
#pragma unroll
  for (int h = 0; h < ATT_GMAX; ++h) {
    if (h >= G) break;
    ored[wave][h][2 * lane] = o[h][0];
    ored[wave][h][2 * lane + 1] = o[h][1];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * d; e += blockDim.x) {
    const int h = e / d, j = e - h * d;
    const float s = ored[0][h][j] + ored[1][h][j] + ored[2][h][j] + ored[3][h][j];
    const int hh = kh * G + h;
    if (a.nsplit == 1) {
      a.out[(long long)qi * a.nh * d + hh * d + j] = tobf(s / lrow[h]);
    } else {
      const long long pidx = ((long long)qi * a.nh + hh) * a.nsplit + split;
      a.part_o[pidx * d + j] = s;
      if (j == 0) {
        a.part_ml[pidx * 2] = nk > 0 ? mrow[h] : -INFINITY;
        a.part_ml[pidx * 2 + 1] = nk > 0 ? lrow[h] : 0.f;
      }
    }
  }
}

__global__ void __launch_bounds__(128) k_attn_combine(AttnArgs a) {
  const int qi = blockIdx.x / a.nh, hh = blockIdx.x - qi * a.nh;
  const int j = threadIdx.x;
  const long long p0 = ((long long)qi * a.nh + hh) * a.nsplit;
  float M = -INFINITY;
  for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.part_ml[(p0 + s) * 2]);
  float num = 0.f, den = 0.f;
  for (int s = 0; s < a.nsplit; ++s) {
    const float m = a.part_ml[(p0 + s) * 2];
    if (m == -INFINITY) continue;
    const float w = __expf(m - M);
    num += w * a.part_o[(p0 + s) * 128 + j];
    den += w * a.part_ml[(p0 + s) * 2 + 1];
  }
  a.out[(long long)qi * a.nh * 128 + hh * 128 + j] = tobf(num / den);
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

int attn_nsplit(int max_len) { return max_len <= ATT_CHUNK ? 1 : (max_len + ATT_CHUNK - 1) / ATT_CHUNK; }

int launch_attn(AttnArgs a, hipStream_t st) {
  if (a.nq <= 0) return 0;
  if (a.kv.d != 128 || a.nh % a.nkv || a.nh / a.nkv > ATT_GMAX) return 1;
  hipLaunchKernelGGL(k_attn, dim3(a.nq * a.nkv, a.nsplit), dim3(256), 0, st, a);
  if (a.nsplit > 1) hipLaunchKernelGGL(k_attn_combine, dim3(a.nq * a.nh), dim3(128), 0, st, a);
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
