// Qwen2 attention for the generate loop: RoPE + KV append, GQA attention over a
// compacted per-row KV cache (split-K "flash decoding" + combine), restricted
// lm_head.  Reference: transformers Qwen2Attention / apply_rotary_pos_emb
// (modeling_qwen2.py:99-134, 150-173, 195-247) as called by VibeVoiceModel.forward
// (vibevoice/modular/modeling_vibevoice.py:169-209).
//
// KV cache layout: K [layer][slot][kv_head][ctx][d]; V [layer][slot][kv_head]
// in blocks of 32 positions, each [d][32] (common.h v_off), so both MFMA
// operands of the kernel below (K as the key-column operand of Q.K^T, V as the
// key-row operand of P.V) are contiguous 16-byte loads, and a wave's V loads
// for one 32-key step are one 8 KB contiguous block.  A row's cache holds only the entries its
// attention mask keeps, in order, so cache index == RoPE position (SURVEY.md
// §8a rows a3, a7).
#include <atomic>
#include <type_traits>

#include "kernels.h"


// ---------------------------------------------------------------- attention
// Grid (query row x kv head, split); a workgroup of NW waves owns keys [k0, k1)
// of its split and hands each wave a contiguous sub-range, merged in LDS.  Per
// wave, 32 keys per step on the matrix cores (mfma 16x16x32 bf16):
//   S[16 heads x 16 keys] = Q[heads x 128] . K^T   (2 tiles, 4 MFMAs each; the
//       G <= 8 query heads of the kv head are the rows, padded to 16)
//   online softmax on S in registers (row = head spread over 16 lanes)
//   P (bf16, as the reference's eager path rounds it) -> per-wave LDS tile ->
//   O[heads x 128] += P[heads x 32 keys] . V[32 keys x 128] (8 MFMAs, V^T cache)
// K / V of the next step are prefetched while the current one computes.
//
// Splits: one CU takes in K/V at only ~20-30 GB/s (tools/attn_stamps.py: 4
// workgroups of 1,024 keys took 19 us), so long contexts are spread over up to
// ATT_SPLITS_MAX splits of >= ATT_CHUNK keys, 8 waves x 32 keys per step.  The
// splits' (m, l, O) merge in the last-arriving workgroup (write-through
// partials + one ticket, no fences) for <= ATT_MERGE_IN splits, else in
// k_attn_merge (one workgroup per query head and 64 dims: the partials of 256
// splits are 128 KB per head, too much for one CU).  Thinner splits at short
// contexts do not pay: the in-kernel merge costs ~6 us of dependent round
// trips (ticket, partial loads, store) and a merge launch ~4 us, against the
// 2-4 us the extra CUs save (plan sweep over 64-1024 keys per split x merge
// form, tools/ab_bench.py attn_tune: all within 1.5 % at B = 1 and 8).  At a
// 64K context 1,024-key splits (64 per row) beat 256-key splits (255): 4.47 vs
// 4.86 ms per step -- fewer partials to merge, each CU still streaming.
constexpr int ATT_GMAX = 8;
constexpr int ATT_KC = 32;            // per-row split granularity (one wave step)
constexpr int ATT_CHUNK = 1024;       // keys per split (8 waves x 4 steps of 32 keys)
constexpr int ATT_SPLITS_MAX = 256;
constexpr int ATT_MERGE_IN = 8;       // splits merged inside k_attn

// keys per split of a row with `len` keys: >= a.chunk, and all a.nsplit splits
// cover len (k_attn and k_attn_merge must agree)
DEV int row_chunk(const AttnArgs& a, int len) {
  const int c = (len + a.nsplit - 1) / a.nsplit;
  return max(a.chunk, (c + ATT_KC - 1) / ATT_KC * ATT_KC);
}

DEV f32x4 amfma(bf16x8 a, bf16x8 b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

// max / sum over the 16 lanes of a DPP row (one MFMA tile column group) with
// row-local DPP moves on the VALU: quad xor 1, quad xor 2, half-row mirror,
// row mirror (a butterfly: every lane ends with the whole row's value; each step
// adds a lane pair in both orders, so all lanes agree bit for bit).  Four
// __shfl_xor were four dependent ds_bpermute LDS round trips.
template <int CTRL>
DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
DEV float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
DEV float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}

DEV void astamp(const AttnArgs& a, int which) {
  if (a.stamps && threadIdx.x == 0) {
    unsigned long long* p = a.stamps + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * 4;
    p[which] = __builtin_amdgcn_s_memrealtime();
    // at entry, slot 3 also records where the workgroup runs (bit 62 marks it; a
    // storing workgroup overwrites it): XCC_ID << 32 | HW_ID (cu / sh / se fields)
    if (which == 0)
      p[3] = (1ull << 62) | ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
             __builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
}

template <int G, int NW>
__global__ void __launch_bounds__(64 * NW) k_attn(AttnArgs a) {
  __shared__ float wm[NW][G], wl[NW][G];
  __shared__ float wo[NW][G][128];
  __shared__ __attribute__((aligned(16))) bf16 pt[NW][16][32];
  __shared__ float fm[G], fl[G];
  __shared__ unsigned last_flag;
  constexpr int d = 128;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int r = lane & 15, g = lane >> 4;
  astamp(a, 0);
  // grid (split, row x kv head): consecutive workgroup ids -- which the
  // dispatcher deals round-robin over the 8 XCDs -- are consecutive splits of
  // one (row, kv head), so every XCD gets an equal share of each row's keys.
  // (With (row x kv head, split) a row's splits fell on id % 8 = the same 2
  // of 8 XCDs per kv head: at 65K keys B = 1 the long row's work ran on half
  // the chip while the short negative row's splits held the other half.)
  const int rk = blockIdx.y, split = blockIdx.x;
  const int qi = rk / a.nkv, kh = rk - qi * a.nkv;
  // the row's length, its KV slot and the Q fragments: all issued before any
  // is used, one memory round trip (the compiler sank the slot and Q loads
  // behind the early exit below, each a round trip of its own); the empty asm
  // makes len / slot live here, so their wait leaves the Q loads in flight
  const int pos_q = a.pos[qi];
  const int slot = a.slots[qi];
  // Q fragments (A operand): row = head r (zero past G), k = dims 32c + 8g .. +7;
  // the fp32 scores are scaled by 1/sqrt(d) after the MFMA
  bf16x8 qf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (r < G) {
      const bf16x8 q8 = *(const bf16x8*)(a.q + (long long)qi * a.nh * 128 + (kh * G + r) * 128 + 32 * c + 8 * g);
      qf[c] = q8;
    } else {
      qf[c] = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  asm volatile("" ::"v"(pos_q), "v"(slot));
  const int len = pos_q + 1;
  // this row's split size: >= a.chunk, all nsplit splits cover len; splits past
  // the row's last key exit at once
  const int chunk = row_chunk(a, len);
  const int nact = (len + chunk - 1) / chunk;
  if (split >= nact) return;
  const int k0 = split * chunk;
  const int k1 = min(len, k0 + chunk);
  // this wave's keys, in 32-key steps
  const int per = ((k1 - k0 + NW - 1) / NW + 31) / 32 * 32;
  const int w0 = k0 + wave * per;
  const int w1 = min(k1, w0 + per);
  const long long cbase = (long long)a.layer * a.kv.s_layer + (long long)slot * a.kv.s_slot +
                          (long long)kh * a.kv.s_head;
  const bf16* K = a.kv.k + cbase;             // [ctx][128]
  const bf16* VB = a.kv.v + cbase;            // 32-position blocks of [128][32] (v_off)
  const bf16x8 z8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};

  f32x4 o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m[i] = -INFINITY;
    l[i] = 0.f;
  }
  // K / V fragments of two 32-key steps in flight per wave (two register sets,
  // both issued before the first step computes): a 512-key split (65K context)
  // is 64 keys per wave, so all of a workgroup's K / V is requested at once
  bf16x8 kA[2][4], vA[8], kB[2][4], vB[8];
  // Loads are unconditional, from positions clamped into [0, w1): no branch
  // and no per-load wait.  (Guarded V loads followed by the tail mask compiled
  // to a branch + s_waitcnt vmcnt(0) after EACH of a step's 8 V loads -- eight
  // serialized memory round trips per step.)  Keys past w1 are masked where
  // their values are used: S to -inf (so P = 0) and V to 0 on the tail step
  // (the clamped rows hold other keys' values, and 0 x NaN would not vanish).
  auto load = [&](int c0, bf16x8 (&kf)[2][4], bf16x8 (&vf)[8]) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int key = min(c0 + 16 * tt + r, w1 - 1);   // B operand of S: col = key
#pragma unroll
      for (int c = 0; c < 4; ++c) kf[tt][c] = *(const bf16x8*)(K + (long long)key * d + 32 * c + 8 * g);
    }
    const int kb = min(c0 + 8 * g, (w1 - 1) & ~7);      // B operand of O: k = keys kb .. kb+7, col = dim
#pragma unroll
    for (int j = 0; j < 8; ++j) vf[j] = *(const bf16x8*)(VB + v_off(16 * j + r, kb));
  };
  if (w0 < w1) load(w0, kA, vA);
  if (w0 + 32 < w1) load(w0 + 32, kB, vB);
  if (a.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    astamp(a, 1);
  }
  auto step = [&](int c0, const bf16x8 (&kc)[2][4], bf16x8 (&vc)[8]) {   // vc is masked in place
    if (c0 + 32 > w1) {   // the wave's tail step (uniform): keys kb + e >= w1 contribute nothing
      const int kb = c0 + 8 * g;
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) vc[j][e] = kb + e < w1 ? vc[j][e] : (bf16)0.f;
    }
    // S tiles: lane holds S[head 4g+i][key c0 + 16tt + r]
    f32x4 sacc[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      sacc[tt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) sacc[tt] = amfma(qf[c], kc[tt][c], sacc[tt]);
    }
    float p[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s0 = c0 + r < w1 ? sacc[0][i] * a.scale : -INFINITY;
      float s1 = c0 + 16 + r < w1 ? sacc[1][i] * a.scale : -INFINITY;
      float mx = fmaxf(s0, s1);
      mx = row16_max(mx);
      const float mnew = fmaxf(m[i], mx);
      const float al = __expf(m[i] - mnew);
      p[0][i] = __expf(s0 - mnew);
      p[1][i] = __expf(s1 - mnew);
      float ps = p[0][i] + p[1][i];
      ps = row16_sum(ps);
      l[i] = l[i] * al + ps;
      m[i] = mnew;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j][i] *= al;
    }
    // P -> LDS [head][key] -> A operand (row = head r, k = keys 8g .. 8g+7)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 4; ++i) pt[wave][4 * g + i][16 * tt + r] = (bf16)p[tt][i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bf16x8 pa = *(const bf16x8*)&pt[wave][r][8 * g];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = amfma(pa, vc[j], o[j]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  for (int c0 = w0; c0 < w1; c0 += 64) {
    step(c0, kA, vA);
    if (c0 + 64 < w1) load(c0 + 64, kA, vA);
    if (c0 + 32 < w1) {
      step(c0 + 32, kB, vB);
      if (c0 + 96 < w1) load(c0 + 96, kB, vB);
    }
  }
  // this wave's (m, l, O): lane holds O[head 4g+i][dim 16j + r]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = 4 * g + i;
    if (h < G) {
#pragma unroll
      for (int j = 0; j < 8; ++j) wo[wave][h][16 * j + r] = o[j][i];
      if (r == 0) {
        wm[wave][h] = m[i];
        wl[wave][h] = l[i];
      }
    }
  }
  __syncthreads();
  astamp(a, 2);
  // merge the waves: waves with no keys carry m = -inf, l = 0
  if (t < G) {
    float M = -INFINITY;
    for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w][t]);
    float L = 0.f;
    for (int w = 0; w < NW; ++w) L += wm[w][t] == -INFINITY ? 0.f : __expf(wm[w][t] - M) * wl[w][t];
    fm[t] = M;
    fl[t] = L;
  }
  __syncthreads();
  constexpr int NE = (G * 128 + 64 * NW - 1) / (64 * NW);
  float res[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int e = t + q * 64 * NW;
    float sum = 0.f;
    if (e < G * d) {
      const int h = e / d, j = e - h * d;
      for (int w = 0; w < NW; ++w)
        if (wm[w][h] != -INFINITY) sum += __expf(wm[w][h] - fm[h]) * wo[w][h][j];
    }
    res[q] = sum;
  }
  if (nact == 1 && !a.defer && !a.group) {
#pragma unroll
    for (int q = 0; q < NE; ++q) {
      const int e = t + q * 64 * NW;
      if (e < G * d) {
        const int h = e / d, j = e - h * d;
        a.out[(long long)qi * a.nh * d + (kh * G + h) * d + j] = tobf(res[q] / fl[h]);
      }
    }
    if (a.stamps) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      astamp(a, 3);
    }
    return;
  }
  // partials: plain stores when k_attn_merge follows (the kernel boundary
  // publishes them); else write-through (sc1, agent-scope relaxed) stores, each
  // wave's vmcnt(0), a workgroup barrier and one ticket add; the last arriver
  // reads them with sc1 loads.  No release / acquire fence: an agent fence
  // writes back the XCD's whole L2 (MI355X_MICROARCH.md "publish-large", the
  // hand-off table's first row).
  const bool wt = !a.merge && !a.defer;   // group mode: write-through too (its last arriver reads them)
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int e = t + q * 64 * NW;
    if (e < G * d) {
      const int h = e / d, j = e - h * d;
      const long long pidx = ((long long)qi * a.nh + kh * G + h) * a.nsplit + split;
      if (wt) {
        __hip_atomic_store(a.part_o + pidx * d + j, res[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (j == 0) {
          __hip_atomic_store(a.part_ml + pidx * 2, fm[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.part_ml + pidx * 2 + 1, fl[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        a.part_o[pidx * d + j] = res[q];
        if (j == 0) {
          a.part_ml[pidx * 2] = fm[h];
          a.part_ml[pidx * 2 + 1] = fl[h];
        }
      }
    }
  }
  if (!wt) return;    // k_attn_merge or the consumer's merge (defer) runs next
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // group mode: splits [gs0, gs1) of this row's active ones form the group; its
  // last arriver merges them into the group partial
  const int gi = a.group ? split / a.group : 0;
  const int gs0 = a.group ? gi * a.group : 0, gs1 = a.group ? min(nact, gs0 + a.group) : nact;
  if (t == 0) {
    unsigned* ctr = a.counters + (a.group ? rk * a.ngroups + gi : rk);
    const unsigned tk = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = tk == (unsigned)(gs1 - gs0 - 1);
    if (last_flag) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last_flag) return;
  if (a.group) {
    // out = the group's (M, L, O): M = max m_s, L = sum e^{m_s - M} l_s, O = sum
    // e^{m_s - M} o_s in split order (the consumer divides by the merged L)
    auto ldg = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    constexpr int GMAX = 16;
    const int ng = gs1 - gs0;
    for (int e = t; e < G * d; e += 64 * NW) {
      const int h = e / d, j = e - h * d;
      const long long p0 = ((long long)qi * a.nh + kh * G + h) * a.nsplit + gs0;
      float mv[GMAX], lv[GMAX], ov[GMAX];
#pragma unroll
      for (int s2 = 0; s2 < GMAX; ++s2) {
        if (s2 < ng) {
          mv[s2] = ldg(a.part_ml + (p0 + s2) * 2);
          lv[s2] = ldg(a.part_ml + (p0 + s2) * 2 + 1);
          ov[s2] = ldg(a.part_o + (p0 + s2) * d + j);
        }
      }
      float M = -INFINITY;
#pragma unroll
      for (int s2 = 0; s2 < GMAX; ++s2)
        if (s2 < ng) M = fmaxf(M, mv[s2]);
      float num = 0.f, den = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < GMAX; ++s2) {
        if (s2 < ng) {
          const float w = __expf(mv[s2] - M);
          num += w * ov[s2];
          den += w * lv[s2];
        }
      }
      const long long q0 = ((long long)qi * a.nh + kh * G + h) * a.ngroups + gi;
      a.part_o2[q0 * d + j] = num;
      if (j == 0) {
        a.part_ml2[q0 * 2] = M;
        a.part_ml2[q0 * 2 + 1] = den;
      }
    }
    return;
  }
  // merge the splits: out = sum_s e^{m_s - M} o_s / sum_s e^{m_s - M} l_s
  auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int e = t; e < G * d; e += 64 * NW) {
    const int h = e / d, j = e - h * d;
    const long long p0 = ((long long)qi * a.nh + kh * G + h) * a.nsplit;
    float mv[ATT_MERGE_IN], lv[ATT_MERGE_IN], ov[ATT_MERGE_IN];
#pragma unroll
    for (int s2 = 0; s2 < ATT_MERGE_IN; ++s2) {
      if (s2 < nact) {
        mv[s2] = ld(a.part_ml + (p0 + s2) * 2);
        lv[s2] = ld(a.part_ml + (p0 + s2) * 2 + 1);
        ov[s2] = ld(a.part_o + (p0 + s2) * d + j);
      }
    }
    float M = -INFINITY;
#pragma unroll
    for (int s2 = 0; s2 < ATT_MERGE_IN; ++s2)
      if (s2 < nact) M = fmaxf(M, mv[s2]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < ATT_MERGE_IN; ++s2) {
      if (s2 < nact) {
        const float w = __expf(mv[s2] - M);
        num += w * ov[s2];
        den += w * lv[s2];
      }
    }
    a.out[(long long)qi * a.nh * d + (kh * G + h) * d + j] = tobf(num / den);
  }
  if (a.stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    astamp(a, 3);
  }
}

// Split merge for long contexts: out = sum_s e^{m_s - M} o_s / sum_s e^{m_s - M} l_s.
// Grid (row x query head, 2 halves of the 128 dims), 8 waves: wave w folds
// splits w, w + 8, ... (lane = dim), then the 8
// partial (M_w, num_w, den_w) combine in LDS in wave order.  (One thread per
// dim walking all 255 splits of a 64K context took 33 us: a chain of loads.)
__global__ void __launch_bounds__(512) k_attn_merge(AttnArgs a) {
  constexpr int d = 128, NWM = 8;
  __shared__ float sm[NWM], snum[NWM][64], sden[NWM];
  const int qi = blockIdx.x / a.nh, h = blockIdx.x - qi * a.nh;
  const int len = a.pos[qi] + 1;
  const int chunk = row_chunk(a, len);
  const int nact = (len + chunk - 1) / chunk;
  if (nact <= 1) return;                     // k_attn stored this row itself
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.y * 64 + lane;
  const long long p0 = ((long long)qi * a.nh + h) * a.nsplit;
  const float* ml = a.part_ml + p0 * 2;
  const float* o = a.part_o + p0 * d + j;
  // one online pass (running max, rescaled sums): the unrolled body's loads
  // do not depend on the accumulators, so 16 splits' loads are in flight at once
  float M = -INFINITY, num = 0.f, den = 0.f;
#pragma unroll 16
  for (int s2 = w; s2 < nact; s2 += NWM) {
    const float m = ml[s2 * 2], l = ml[s2 * 2 + 1], ov = o[(long long)s2 * d];
    const float Mn = fmaxf(M, m);
    const float sc = __expf(M - Mn), e = __expf(m - Mn);
    num = num * sc + e * ov;
    den = den * sc + e * l;
    M = Mn;
  }
  snum[w][lane] = num;
  if (lane == 0) {
    sm[w] = M;
    sden[w] = den;
  }
  __syncthreads();
  if (w == 0) {
    float Mt = -INFINITY;
#pragma unroll
    for (int v = 0; v < NWM; ++v) Mt = fmaxf(Mt, sm[v]);
    float nt = 0.f, dt = 0.f;
#pragma unroll
    for (int v = 0; v < NWM; ++v) {
      if (sm[v] == -INFINITY) continue;       // a wave with no split
      const float e = __expf(sm[v] - Mt);
      nt += e * snum[v][lane];
      dt += e * sden[v];
    }
    a.out[(long long)qi * a.nh * d + h * d + j] = tobf(nt / dt);
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
  // one workgroup per row; thread t owns 8-element chunks t, t + 256, ... (H <= 8192)
  float v[4][8];
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = t + 256 * q;
    if (c < nch) {
      const bf16x8 x8 = *(const bf16x8*)(x + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[q][j] = bf(x8[j]);
        ss += v[q][j] * v[q][j];
      }
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) red[wave][0] = ss;
  __syncthreads();
  ss = red[0][0] + red[1][0] + red[2][0] + red[3][0];
  const float inv = rsqrtf(ss / (float)H + eps);
  float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = t + 256 * q;
    if (c < nch) {
      const bf16x8 w8 = *(const bf16x8*)(norm_w + c * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[q][j] = rb(rb(v[q][j] * inv) * bf(w8[j]));
        o[j] = tobf(v[q][j]);
      }
      *(bf16x8*)(hid + (long long)i * H + c * 8) = o;
      for (int k = 0; k < nid; ++k) {
        const bf16x8 l8 = *(const bf16x8*)(W + (long long)ids[k] * H + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) part[k] += v[q][j] * bf(l8[j]);
      }
    }
  }
  __syncthreads();
  for (int k = 0; k < nid; ++k) {
    const float sk = wave_sum(part[k]);
    if (lane == 0) red[wave][1 + k] = sk;
  }
  __syncthreads();
  if (t < nid) logits[i * nid + t] = rb(red[0][1 + t] + red[1][1 + t] + red[2][1 + t] + red[3][1 + t]);
}

// ================================================================ host launchers
int launch_final_head(int R, int H, const bf16* h, const int* idx, const bf16* norm_w, float eps, bf16* hidden_out,
                      const bf16* W, const int* ids, int nid, float* logits, hipStream_t st) {
  if (R <= 0) return 0;
  if (H % 8 || H / 8 > 1024 || nid > 4 || (nid > 0 && (!W || !ids || !logits))) return 1;
  hipLaunchKernelGGL(k_final_head, dim3(R), dim3(256), 0, st, H, h, idx, norm_w, eps, hidden_out, W, ids, nid,
                     logits);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}


// ---------------------------------------------------------------- prefill attention
// The causal prefill of a prompt (the reference runs the
// whole prompt through Qwen2Model once, modeling_vibevoice_inference.py:484 at
// step 0): thousands of query rows over the same slot.  k_attn gives every row
// its own pass over its keys (K/V re-read per row, 6 of 16 MFMA rows used), so
// here a workgroup takes PF_Q = 32 consecutive query rows x the G query heads of
// one kv head (wave = head).  Per 32-key step the workgroup stages K and V once
// in LDS (16 one-KB blocks of 16-byte global_load_lds, already in MFMA fragment
// order, so every LDS read is a conflict-free lane-linear ds_read_b128), in a
// ring of PF_NS stages: later steps are in flight while the G waves compute s.  Per wave
// and step, on the matrix cores (mfma 16x16x32 bf16), transposed so P never
// leaves registers:
//   S^T[32 keys x 32 queries] = K . Q^T   (A = K rows, B = the wave's Q
//       fragments held for the whole kernel).  Row 4g+i of key tile kt is key
//       8g + 4kt + i (the K fragment gathers its rows in that order), so a lane
//       holds keys 8g .. 8g+7 of query column r
//   online softmax per query column (the 4 lanes r, r+16, r+32, r+48 hold its
//       keys: two xor-shuffles for the max; the sum stays per lane until the end)
//   O^T[128 dims x 32 queries] += V^T . P^T: the MFMA's k slots 8g .. 8g+7 are
//       the lane's own P values (bf16, as the reference's eager path rounds
//       them) and V^T's fragment is 16 contiguous bytes of a [dim][32 pos] V block.
// Rows of a tile may belong to different slots (sample boundaries, ragged
// prompts): the tile loops over its distinct slots, each pass masking the rows
// of other slots, so any (slot, pos) list is exact; runs of one slot cost one
// pass.  Keys > the row's position are masked (causal); the pass spans keys
// [0, max position of its rows].
constexpr int PF_Q = 32;
constexpr float PF_LAZY = 8.f;       // running-max slack (log2 units) before O is rescaled
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// 32-key steps per LDS stage (one barrier and one vmcnt wait per stage)
constexpr int PF_SUB = 2;
constexpr int PF_STAGE = PF_SUB * 16 * 512;   // bf16 elements per stage: per step 8 K + 8 V fragment blocks
// LDS stages: steps s+1 .. s+NS-2 in flight while step s computes, step
// s+NS-1 issued after the step's one barrier.  16K-token prefill (interleaved
// same-box runs, tools/ab_bench.py --prefill): NS 2 118.7 ms, NS 3 122.4, NS 4
// 122.4; the former two-barrier form with NS 2 124.6 ms
constexpr int PF_NS = 2;

// max / sum over lanes {l, l^16, l^32, l^48} (one query column of an MFMA
// tile): gfx950's v_permlane16_swap / v_permlane32_swap (VALU, a few cycles)
// instead of two ds_bpermute round trips.  With the value in both operands,
// the 16-swap yields rows (0,0,2,2) and (1,1,3,3), the 32-swap (0,1,0,1) and (2,3,2,3).
DEV float col_max(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
DEV float col_sum(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be constant)
DEV void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;   // conservative
  }
}

// QW = 16-query tiles per wave: 2 -> G waves (one per head); 1 -> 2G waves (a
// head's two tiles on two waves).  At G = 6 the 6-wave form leaves two SIMDs
// with one wave and two with two (the per-step barrier waits for the loaded
// ones), and 215 VGPRs allow no second workgroup; 12 waves of ~150 VGPRs fill
// every SIMD with three.
template <int G, int QW>
__global__ void __launch_bounds__(64 * G * 2 / QW) __attribute__((amdgpu_waves_per_eu(QW == 1 ? (G * 2 + 3) / 4 : (G >= 4 ? 2 : 1)))) k_attn_pf(AttnArgs a) {
  constexpr int d = 128;
  constexpr int NW = G * 2 / QW;             // waves
  constexpr int NI_MAX = (16 * PF_SUB + NW - 1) / NW;   // staging instructions per wave and stage
  // one LDS array (a second __shared__ object can make hipcc drain the
  // prefetch early, cdna_hip_programming.md §5 trap 4a): 2 stages + row table
  __shared__ __attribute__((aligned(16))) bf16 sm[PF_NS * PF_STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int ntile = (a.nq + PF_Q - 1) / PF_Q;
  const int q0 = (ntile - 1 - (int)blockIdx.x) * PF_Q;   // late (long) tiles first
  // the tile's row slots / positions come from global (uniform addresses: scalar
  // loads); an LDS table beside the 64 KB ring would not fit
  auto s_slot = [&](int j) { return q0 + j < a.nq ? a.slots[q0 + j] : -1; };
  auto s_pos = [&](int j) { return q0 + j < a.nq ? a.pos[q0 + j] : -1; };
  const int kh = blockIdx.y, h = kh * G + (QW == 2 ? wave : wave >> 1);
  const int qt0 = QW == 2 ? 0 : (wave & 1);   // the wave's first 16-query tile
  const bf16x8 z8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 qf[QW][4];   // B operand of S^T: column = query 16(qt0 + qt) + r, k = dims 32c + 8g .. +7
#pragma unroll
  for (int qt = 0; qt < QW; ++qt) {
    const int qi = q0 + 16 * (qt0 + qt) + r;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      qf[qt][c] = qi < a.nq ? *(const bf16x8*)(a.q + (long long)qi * a.nh * d + h * d + 32 * c + 8 * g) : z8;
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");   // no plain loads in flight beside the staging
  __syncthreads();
  int qslot[QW], qpos[QW];
#pragma unroll
  for (int qt = 0; qt < QW; ++qt) {
    qslot[qt] = s_slot(16 * (qt0 + qt) + r);
    qpos[qt] = s_pos(16 * (qt0 + qt) + r);
  }
  // this wave's staging blocks j = wave + NW * i: j < 8 K fragment (kt = j >> 2,
  // c = j & 3; lane row r' -> key 8(r' >> 2) + 4kt + (r' & 3)), j >= 8 V^T
  // fragment dt = j - 8 (dims 16dt + r', keys 8g' .. 8g'+7); both advance by
  // 128 elements per key
  const int ni = __builtin_amdgcn_readfirstlane((16 * PF_SUB - wave + NW - 1) / NW);   // wave-uniform: scalar branches in issue()
  int soff[NI_MAX];   // element offset in the step's 32-key K block / V block (< 4096)
#pragma unroll
  for (int i = 0; i < NI_MAX; ++i) {
    const int j = (wave + NW * i) & 15, sub = (wave + NW * i) >> 4;   // block j of step `sub` of the stage
    if (j < 8) {
      const int kt = j >> 2, c = j & 3;
      soff[i] = (sub * 32 + 8 * (r >> 2) + 4 * kt + (r & 3)) * d + 32 * c + 8 * g;
    } else {
      soff[i] = (int)v_off(16 * (j - 8) + r, sub * 32 + 8 * g);
    }
  }
  f32x4 o[8][QW];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt)
#pragma unroll
    for (int qt = 0; qt < QW; ++qt) o[dt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[QW], l[QW];
#pragma unroll
  for (int qt = 0; qt < QW; ++qt) {
    m[qt] = -INFINITY;
    l[qt] = 0.f;
  }
  const float sl2 = a.scale * 1.4426950408889634f;   // scores in log2 units
  unsigned valid = 0;
  for (int j = 0; j < PF_Q; ++j)
    if (s_slot(j) >= 0) valid |= 1u << j;
  unsigned done = 0;
  while (done != valid) {
    // one pass per distinct slot of the tile
    const int slot = s_slot(__builtin_ctz(valid & ~done));
    int kmax = 0, kmin = 1 << 30;
    unsigned seg = 0;
    for (int j = 0; j < PF_Q; ++j)
      if (s_slot(j) == slot) {
        seg |= 1u << j;
        kmax = max(kmax, s_pos(j));
        kmin = min(kmin, s_pos(j));
      }
    done |= seg;
    // steps whose keys every valid row of the tile attends need no mask (rows
    // past nq are never stored)
    const int kfull = seg == valid ? kmin + 1 : 0;
    const int nk = kmax + 1, nsteps = (nk + 32 * PF_SUB - 1) / (32 * PF_SUB);   // stages
    bool inq[QW];
#pragma unroll
    for (int qt = 0; qt < QW; ++qt) inq[qt] = qslot[qt] == slot;
    const long long cbase = (long long)a.layer * a.kv.s_layer + (long long)slot * a.kv.s_slot +
                            (long long)kh * a.kv.s_head;
    const bf16* K = a.kv.k + cbase;    // [ctx][128]
    const bf16* VB = a.kv.v + cbase;   // 32-position blocks of [128][32] (v_off)
    auto issue = [&](int step) {
      bf16* st = sm + (step % PF_NS) * PF_STAGE;
#pragma unroll
      for (int i = 0; i < NI_MAX; ++i)
        if (i < ni) {
          const bf16* src = (((wave + NW * i) & 15) >= 8 ? VB : K) + (long long)step * 32 * PF_SUB * d + soff[i];
          __builtin_amdgcn_global_load_lds((const void*)src,
                                           (__attribute__((address_space(3))) void*)(st + (wave + NW * i) * 512),
                                           16, 0, 0);
        }
    };
    for (int p = 0; p < PF_NS - 1 && p < nsteps; ++p) issue(p);
    for (int step = 0; step < nsteps; ++step) {
      // this wave's loads of `step` have landed (steps step + 1 .. step + NS - 2 stay in flight)
      if (PF_NS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (no runtime switch: n is always 0)
      else wait_vm(ni * min(PF_NS - 2, nsteps - 1 - step));
      // ONE barrier per step: every wave's loads of `step` are in LDS, and every
      // wave has finished reading step - 1, whose buffer takes step + NS - 1
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (step + PF_NS - 1 < nsteps) issue(step + PF_NS - 1);
#pragma unroll
      for (int sub = 0; sub < PF_SUB; ++sub) {
      const int k0 = (step * PF_SUB + sub) * 32;
      if (k0 >= nk) break;
      const bf16* st = sm + (step % PF_NS) * PF_STAGE + sub * 16 * 512;
      // all 8 K fragments, then the 16 S MFMAs (one LDS round trip, not one per key tile)
      bf16x8 kf[8];
#pragma unroll
      for (int f = 0; f < 8; ++f) kf[f] = *(const bf16x8*)(st + f * 512 + lane * 8);
      f32x4 s[2][QW];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int qt = 0; qt < QW; ++qt) {
          s[kt][qt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < 4; ++c) s[kt][qt] = amfma(kf[kt * 4 + c], qf[qt][c], s[kt][qt]);
        }
      // the V^T fragments do not depend on P: issued now, they land under the softmax
      // (read one at a time after it, each read's latency was exposed 8 times a step)
      bf16x8 vf[8];
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) vf[dt] = *(const bf16x8*)(st + (8 + dt) * 512 + lane * 8);
      __builtin_amdgcn_sched_barrier(0);
      // online softmax with a lazy running max: a column's m (log2 units) moves
      // only when a score exceeds it by > PF_LAZY, so P <= 2^PF_LAZY and the
      // O / l rescale (64 multiplies per column pair) runs only on the steps
      // where some column of the wave moved (a wave-uniform branch).  Steps every
      // row attends in full (all but the diagonal ones) skip the mask selects.
      const bool full = k0 + 32 <= kfull;
      float x[QW][2][4], al[QW];
      bool move[QW];
      if (full) {   // raw scores: the max commutes with the positive scale, exp2 takes fma(s, sl2, -m)
#pragma unroll
        for (int qt = 0; qt < QW; ++qt)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int i = 0; i < 4; ++i) x[qt][kt][i] = s[kt][qt][i];
      } else {
#pragma unroll
        for (int qt = 0; qt < QW; ++qt) {
          const bool in = inq[qt];
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int key = k0 + 8 * g + 4 * kt + i;
              x[qt][kt][i] = in && key <= qpos[qt] ? s[kt][qt][i] * sl2 : -INFINITY;
            }
        }
      }
      bool anymove = false;
#pragma unroll
      for (int qt = 0; qt < QW; ++qt) {
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 4; ++i) mx = fmaxf(mx, x[qt][kt][i]);
        mx = col_max(mx);
        if (full) mx *= sl2;
        move[qt] = mx > m[qt] + PF_LAZY;   // also the first live step (m = -inf); lanes of a column agree
        al[qt] = move[qt] ? exp2f(m[qt] - mx) : 1.f;
        if (move[qt]) m[qt] = mx;
        anymove |= move[qt];
      }
      if (__builtin_amdgcn_ballot_w64(anymove)) {
#pragma unroll
        for (int qt = 0; qt < QW; ++qt) {
          l[qt] *= al[qt];
#pragma unroll
          for (int dt = 0; dt < 8; ++dt) o[dt][qt] *= al[qt];
        }
      }
      bf16x8 pf[QW];
      // branch-free within a step: a column with no live key yet has every x =
      // -inf, so any finite reference gives p = 0; the raw v_exp_f32 (the libm
      // exp2f wraps it in a denormal-range fix-up, 5 VALU per value) flushes
      // results below 2^-126, far under a bf16 P's resolution next to the row's
      // max of 1..2^8.  Full steps: p = 2^fma(s, scale, -m) (one VALU less per score)
      auto probs = [&](auto full_c) {
#pragma unroll
        for (int qt = 0; qt < QW; ++qt) {
          const float mref = m[qt] != -INFINITY ? m[qt] : 0.f;
          float ps = 0.f;
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float e = decltype(full_c)::value ? __builtin_fmaf(x[qt][kt][i], sl2, -mref) : x[qt][kt][i] - mref;
              const float p = __builtin_amdgcn_exp2f(e);
              ps += p;
              pf[qt][4 * kt + i] = (bf16)p;
            }
          l[qt] += ps;
        }
      };
      if (full) probs(std::true_type{});
      else probs(std::false_type{});
      // the last step's V past the last key (unwritten cache) would meet P = 0:
      // zero it (0 * NaN) with a bit mask over the lane's keys 8g .. 8g+7
      if (k0 + 32 > nk) {
        const int lim = nk - k0 - 8 * g;
        u32x4 vm;
#pragma unroll
        for (int p2 = 0; p2 < 4; ++p2) vm[p2] = (2 * p2 < lim ? 0xFFFFu : 0u) | (2 * p2 + 1 < lim ? 0xFFFF0000u : 0u);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) vf[dt] = __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, vf[dt]) & vm);
      }
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int qt = 0; qt < QW; ++qt) o[dt][qt] = amfma(vf[dt], pf[qt], o[dt][qt]);
      }   // sub-step
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // the next pass restages every buffer
  }
  // lane holds O^T[dim 16dt + 4g + i][query 16qt + r]; l summed over the 4 lanes of the column
#pragma unroll
  for (int qt = 0; qt < QW; ++qt) {
    const float L = col_sum(l[qt]);
    const int qi = q0 + 16 * (qt0 + qt) + r;
    if (qi < a.nq) {
      const float inv = 1.f / L;
      bf16* op = a.out + (long long)qi * a.nh * d + h * d + 4 * g;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        bf16x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = tobf(o[dt][qt][i] * inv);
        *(bf16x4*)(op + 16 * dt) = v;
      }
    }
  }
}

static std::atomic<int> g_att_prefill{-1};   // diagnostic override (vv_attn_prefill): -1 auto, 0 never, 1 always
extern "C" int vv_attn_prefill(int mode) {
  g_att_prefill = mode < 0 ? -1 : mode > 0 ? 1 : 0;
  return 0;
}

// Tiles of 32 rows over at most nslots slots average <= 2 passes once
// nq >= 32 * nslots; decode steps (one row per slot) stay on k_attn.
bool attn_use_prefill(int nq, int nslots) {
  if (g_att_prefill >= 0) return g_att_prefill == 1;
  return nq >= 256 && nq >= PF_Q * nslots;
}

static int launch_attn_pf(const AttnArgs& a, hipStream_t st) {
  const dim3 grid((a.nq + PF_Q - 1) / PF_Q, a.nkv);
  // two waves per head (QW = 1) while that keeps <= 3 waves per SIMD (G <= 6)
  switch (a.nh / a.nkv) {
    case 1: hipLaunchKernelGGL((k_attn_pf<1, 1>), grid, dim3(128), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_attn_pf<2, 1>), grid, dim3(256), 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_attn_pf<3, 1>), grid, dim3(384), 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_attn_pf<4, 1>), grid, dim3(512), 0, st, a); break;
    case 5: hipLaunchKernelGGL((k_attn_pf<5, 1>), grid, dim3(640), 0, st, a); break;
    case 6: hipLaunchKernelGGL((k_attn_pf<6, 1>), grid, dim3(768), 0, st, a); break;
    case 7: hipLaunchKernelGGL((k_attn_pf<7, 2>), grid, dim3(448), 0, st, a); break;
    default: hipLaunchKernelGGL((k_attn_pf<8, 2>), grid, dim3(512), 0, st, a); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Launch plan for keys up to max_len: splits of ATT_CHUNK keys (at most
// ATT_SPLITS_MAX; beyond that the splits grow in ATT_CHUNK steps).  Each row
// sizes its own splits from its length (row_chunk), so a plan made for
// max_ctx serves every step of a captured graph.
static std::atomic<int> g_att_chunk{0}, g_att_merge_in{-1};   // diagnostic overrides (vv_attn_tune)
extern "C" int vv_attn_tune(int chunk, int merge_in) {
  if (chunk % ATT_KC) return 1;
  g_att_chunk = chunk;
  g_att_merge_in = merge_in;
  return 0;
}

int attn_plan(int nq, int nkv, int max_len, int* chunk) {
  (void)nq;
  (void)nkv;
  const int tc = g_att_chunk;
  int c = tc > 0 ? tc : ATT_CHUNK;
  int ns = (max_len + c - 1) / c;
  if (ns > ATT_SPLITS_MAX) {
    c = ((max_len + ATT_SPLITS_MAX - 1) / ATT_SPLITS_MAX + ATT_CHUNK - 1) / ATT_CHUNK * ATT_CHUNK;
    ns = (max_len + c - 1) / c;
  }
  if (ns < 1) ns = 1;
  *chunk = c;
  return ns;
}

template <int NW>
static void launch_attn_nw(const AttnArgs& a, dim3 grid, hipStream_t st) {
  const dim3 blk(64 * NW);
  switch (a.nh / a.nkv) {
    case 1: hipLaunchKernelGGL((k_attn<1, NW>), grid, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_attn<2, NW>), grid, blk, 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_attn<3, NW>), grid, blk, 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_attn<4, NW>), grid, blk, 0, st, a); break;
    case 5: hipLaunchKernelGGL((k_attn<5, NW>), grid, blk, 0, st, a); break;
    case 6: hipLaunchKernelGGL((k_attn<6, NW>), grid, blk, 0, st, a); break;
    case 7: hipLaunchKernelGGL((k_attn<7, NW>), grid, blk, 0, st, a); break;
    default: hipLaunchKernelGGL((k_attn<8, NW>), grid, blk, 0, st, a); break;
  }
}

int launch_attn(AttnArgs a, hipStream_t st) {
  if (a.nq <= 0) return 0;
  if (a.kv.d != 128 || a.nh % a.nkv || a.nh / a.nkv > ATT_GMAX) return 1;
  if (a.prefill) return launch_attn_pf(a, st);
  if (a.chunk % ATT_KC || a.nsplit > ATT_SPLITS_MAX) return 1;
  if ((a.nsplit > 1 || a.defer) && (!a.part_o || !a.part_ml || !a.counters)) return 1;
  if (a.defer && a.nsplit > ATT_MERGE_IN) return 1;
  if (a.group && (a.defer || a.group > 16 || a.ngroups > ATT_MERGE_IN || a.ngroups * a.group < a.nsplit ||
                  !a.part_o2 || !a.part_ml2 || (long long)a.nq * a.nkv * a.ngroups > 65536))
    return 1;
  const int mi = g_att_merge_in;
  a.merge = !a.defer && !a.group && a.nsplit > (mi >= 0 ? mi : ATT_MERGE_IN) ? 1 : 0;
  dim3 grid(a.nsplit, a.nq * a.nkv);
  const int nw = a.chunk >= 256 ? 8 : a.chunk >= 128 ? 4 : 2;   // 32 keys per wave step
  if (nw == 8) launch_attn_nw<8>(a, grid, st);
  else if (nw == 4) launch_attn_nw<4>(a, grid, st);
  else launch_attn_nw<2>(a, grid, st);
  if (a.merge) hipLaunchKernelGGL(k_attn_merge, dim3(a.nq * a.nh, 2), dim3(512), 0, st, a);
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
    const long long hb = b - j;                 // V: common.h v_off
    kv.v[hb + v_off(j, dst[i])] = kv.v[hb + v_off(j, src[i])];
  }
}

// Synthetic context (benchmarks only): K and V of every
// layer / kv head at positions [p0, p1) of the given slots get deterministic
// pseudo-random bf16 values in [-0.5, 0.5) (a hash of the element index), so a
// decode step can be timed attending ~64K keys without a 64K-token prefill.
__global__ void __launch_bounds__(256) k_kv_fill(KVLayout kv, int n_layers, int nkv, const int* slots, int p0, int p1,
                                                 unsigned seed) {
  const int span = p1 - p0;
  const long long per_head = (long long)span * kv.d;
  const long long total = per_head * n_layers * nkv;
  const int slot = slots[blockIdx.y];
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long lh = e / per_head, r = e - lh * per_head;
    const int layer = (int)(lh / nkv), h = (int)(lh - (long long)layer * nkv);
    const int pos = p0 + (int)(r / kv.d), j = (int)(r % kv.d);
    const long long base = (long long)layer * kv.s_layer + (long long)slot * kv.s_slot + (long long)h * kv.s_head;
    unsigned x = (unsigned)(e * 2654435761ull) ^ (seed + 0x9e3779b9u * (unsigned)slot);
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    kv.k[base + (long long)pos * kv.d + j] = tobf((float)(x & 0xffff) / 65536.f - 0.5f);
    kv.v[base + v_off(j, pos)] = tobf((float)(x >> 16) / 65536.f - 0.5f);
  }
}

int launch_kv_fill(KVLayout kv, int n_layers, int nkv, int n, const int* slots, int p0, int p1, unsigned seed,
                   hipStream_t st) {
  if (n <= 0 || p1 <= p0) return 0;
  if (p0 < 0 || p1 > kv.max_ctx) return 1;
  hipLaunchKernelGGL(k_kv_fill, dim3(2048, n), dim3(256), 0, st, kv, n_layers, nkv, slots, p0, p1, seed);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int launch_kv_copy(KVLayout kv, int n_layers, int nkv, int n, const int* slots, const int* src, const int* dst,
                   hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_kv_copy, dim3(n), dim3(256), 0, st, kv, n_layers, nkv, slots, src, dst);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
