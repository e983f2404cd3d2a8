// The LM attention half at decode in ONE launch (k_lm_attn): input_layernorm ->
// q|k|v projection (+bias) -> RoPE -> KV append -> GQA attention over the
// compacted per-row cache -> o_proj -> residual, for R <= 16 query rows of the
// 1.5B shapes (H 1,536, 12 q / 2 kv heads of 128) at contexts <= LA_MAX_KEYS.
// Reference: transformers Qwen2Attention (modeling_qwen2.py:99-134, 150-173,
// 195-247) as VibeVoiceModel.forward calls it per layer
// (vibevoice/modular/modeling_vibevoice.py:169-209) inside the generate loop
// (modeling_vibevoice_inference.py:483-486, 591-604).
//
// Per op this was three launches (k_gemv1 q|k|v with the RoPE / cache epilogue,
// k_attn with key splits, k_gemv1 o_proj merging the splits' partials): 7.5 +
// 6.5 + 7.4 us per layer at B = 1, ~11 MB of weights -- latency, not bytes.  Here
// 256 workgroups (one per CU) run four phases with three grid-wide waits:
//   1. workgroups 0..127 each own one 16-column q|k|v tile over all of K (48 KB
//      of weights in registers; the R A rows by LDS DMA, RMSNorm'd in place),
//      MFMA, the 8 waves' K slices summed in order, epi_rope's epilogue written
//      through (q rows; K rows and V columns into the cache).  Workgroups
//      128..223 meanwhile load their o_proj tile (48 KB) into registers, where it
//      stays until phase 4.
//   2. attention in units of (row, kv head, 32 keys), one wave each, dealt
//      round-robin over the 256 workgroups: S = Q.K^T and P.V on MFMA (k_attn's
//      step, the kv head's 6 query heads padded to 16 rows), the unit's
//      (m, l, O) partial written through.
//   3. one wave per (row, query head) merges its units' partials in unit order
//      (k_attn's merge formula) into the attention row, written through.
//   4. the o_proj workgroups DMA the attention rows, MFMA with the resident
//      weights, residual epilogue.
// Hand-offs: write-through (sc1) stores, each storing wave's vmcnt(0), a
// workgroup barrier, lane 0's arrival (persist_dev.h hl_grid_wait_gen); readers
// use sc1 / nt loads (L1-bypassing; MI355X_MICROARCH.md's hand-off table, first
// row).  Arithmetic: epi_rope's and k_attn's (scores scaled after the MFMA, P
// rounded to bf16 for P.V, l in fp32), the units merged as k_attn merges splits.
#include "persist_dev.h"

namespace la {
constexpr int H = 1536, NH = 12, NKV = 2, G = 6, D = 128, NQKV = (NH + 2 * NKV) * D;
constexpr int GRID = pk::G, NW = 8, NT = NW * 64, RMAX = 16;
constexpr int KC = H / 32, KPW = KC / NW;        // 48 k-blocks, 6 per wave
constexpr int TQ = NQKV / 16, TO = H / 16;       // 128 q|k|v tiles, 96 o_proj tiles
constexpr int O0 = TQ;                           // o_proj workgroups [O0, O0 + TO)
constexpr int XST = H + 8;                       // padded LDS row (elements)
constexpr int XS = 0, XS_B = RMAX * XST * 2;
constexpr int RED = XS + XS_B, RED_B = NW * 256 * 4;
constexpr int PT = RED + RED_B, PT_B = NW * 16 * 32 * 2;
constexpr int NWS = PT + PT_B, NWS_B = H * 2;              // input_layernorm weight
constexpr int SM = NWS + NWS_B, SM_B = 64 + 4 * (2 * RMAX + 1) + 12;
// 82 KB: one workgroup per CU (two would share a CU while another idles)
constexpr int TOTAL = (SM + SM_B) > 82 * 1024 ? (SM + SM_B) : 82 * 1024;
constexpr int PART = G * D + 2 * G;              // floats per unit partial: O[6][128], then (m, l) x 6
constexpr int GEN = 15;                          // this kernel's generation line in the sync buffer
static_assert(SM + SM_B <= 160 * 1024, "lm attn LDS");
}  // namespace la

DEV void la_stamp(const LmAttnArgs& a, int k) {
  if (a.stamps && threadIdx.x == 0) a.stamps[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memrealtime();
}

template <int CTRL>
DEV float la_dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
DEV float la_max16(float v) {   // max over the 16 lanes of a DPP row (attention.hip row16_max)
  v = fmaxf(v, la_dppf<0xB1>(v));
  v = fmaxf(v, la_dppf<0x4E>(v));
  v = fmaxf(v, la_dppf<0x141>(v));
  return fmaxf(v, la_dppf<0x140>(v));
}
DEV float la_sum16(float v) {
  v += la_dppf<0xB1>(v);
  v += la_dppf<0x4E>(v);
  v += la_dppf<0x141>(v);
  return v + la_dppf<0x140>(v);
}

DEV float wave_max(float v) {   // every lane ends with the wave's max (wave_sum's steps)
  v = fmaxf(v, la_dppf<0xB1>(v));
  v = fmaxf(v, la_dppf<0x4E>(v));
  v = fmaxf(v, la_dppf<0x141>(v));
  v = fmaxf(v, la_dppf<0x140>(v));
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__global__ void __launch_bounds__(la::NT) k_lm_attn(LmAttnArgs a) {
  using namespace la;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + XS);        // phase 1: [16][XST] A rows; phase 4: attention rows
  float* red = (float*)(smem + RED);    // [8 waves][256] MFMA partials
  bf16* pt = (bf16*)(smem + PT);        // [8 waves][16][32] P tiles
  bf16* nw_s = (bf16*)(smem + NWS);
  float* inv_s = (float*)(smem + SM);   // [16]
  int* pre = (int*)(smem + SM + 64);    // [2R + 1] unit prefix over (row, kv head) pairs
  unsigned* ok_s = (unsigned*)(smem + SM + 64 + 4 * (2 * RMAX + 1));

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, w = blockIdx.x, R = a.R;
  const int r16 = lane & 15, g4 = lane >> 4;
  const RopeEpi& RP = a.qkv.rope;
  const bool qt = w < TQ, ot = w >= O0 && w < O0 + TO;
  unsigned g0 = 0;
  if (threadIdx.x == 0)
    g0 = __hip_atomic_load((hl_gu32*)(a.sync + GEN * pk::LINE), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;
  // the attention units: pair p = row * NKV + kv head holds ceil(len / 32) of
  // them (positions read first: a wait for them then leaves the streams in flight)
  int nunit = 0;
  if (threadIdx.x < 2 * RMAX) {
    const int qi = threadIdx.x / NKV;
    nunit = qi < R ? (RP.pos[qi] + 1 + 31) / 32 : 0;
  }
  la_stamp(a, 0);
  bf16x4 rv_pre = (bf16x4){0, 0, 0, 0};   // o_proj's residual operand (variant 4: loaded at entry)
  if ((a.variant & 4) && ot && wave == 0 && r16 < R)
    rv_pre = *(const bf16x4*)(rm_bf(a.res, r16) + 16 * (w - O0) + 4 * g4);

  // ================= phase 1: q|k|v tile (workgroups < 128) / o_proj weights (128..223)
  bf16x8 wq[KPW], wo[KPW];
  const int ln = hl_vopaque(lane);
  // wave 0's RoPE epilogue operands (row m = lane & 15, columns 16 w + 4 g ..): position,
  // slot and bias first, the cos / sin row (dependent on the position) after the weights
  int rp = 0, rs = 0;
  bf16x4 rb4 = (bf16x4){0, 0, 0, 0}, cs4 = rb4, sn4 = rb4;
  if (qt && wave == 0) {
    const int mm = min(r16, R - 1);
    rp = RP.pos[mm];
    rs = RP.slots[mm];
    rb4 = *(const bf16x4*)(a.qkv.epi.bias + 16 * w + 4 * g4);
  }
  if (qt) {
    const int qn = (a.variant & 1) ? R * 3 : RMAX * 3;
    for (int q = wave; q < qn; q += NW) {   // row q / 3, 64-chunk piece q % 3 (rows >= R re-read R - 1)
      const int m = q / 3, i = q - m * 3;
      hl_dma16<false>(xs + m * XST + i * 512, rm_bf(a.qkv.a, min(m, R - 1)) + (i * 64 + ln) * 8);
    }
    if (wave < 3) hl_dma16<false>(nw_s + wave * 512, a.nw + (wave * 64 + ln) * 8);
    const bf16* wp = hl_opaque(a.qkv.w) + ((long long)w * KC + wave * KPW) * 512 + ln * 8;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) wq[kk] = hl_ldnt(wp + (long long)kk * 512);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // this wave's A-side DMA (KPW = 6 weight loads younger)
    if (wave == 0 && RP.cs_tab) {
      const int j = 8 * (w & 7) + 4 * (g4 & 1);
      cs4 = *(const bf16x4*)(RP.cs_tab + (long long)rp * D + j);
      sn4 = *(const bf16x4*)(RP.cs_tab + (long long)rp * D + 64 + j);
    }
  } else if (ot && !(a.variant & 2)) {
    const bf16* wp = hl_opaque(a.ow) + ((long long)(w - O0) * KC + wave * KPW) * 512 + ln * 8;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) wo[kk] = hl_ldnt(wp + (long long)kk * 512);
  }
  if (threadIdx.x < 2 * RMAX) pre[threadIdx.x + 1] = nunit;
  __syncthreads();
  if (threadIdx.x == 0) {
    pre[0] = 0;
    for (int p = 1; p <= 2 * RMAX; ++p) pre[p] += pre[p - 1];
  }
  la_stamp(a, 1);
  if (qt) {
    const int mr = (a.variant & 1) ? R : RMAX;   // (rows >= R of the MFMA are never stored)
    for (int m = wave; m < mr; m += NW) {   // inverse RMS in k_rmsnorm's order
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
    for (int e = hl_vopaque((int)threadIdx.x); e < mr * (H / 8); e += NT) {   // xform<XF_NORM>, in place
      const int m = e / (H / 8), c = e - m * (H / 8);
      const bf16x8 xv = *(const bf16x8*)(xs + m * XST + c * 8);
      const bf16x8 wv = *(const bf16x8*)(nw_s + c * 8);
      const float inv = inv_s[m];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = tobf(rb(rb(bf(xv[j]) * inv) * bf(wv[j])));
      *(bf16x8*)(xs + m * XST + c * 8) = o;
    }
    __syncthreads();
    // D[n][m]: A = the weight tile (row n = lane & 15), B = the A rows (column m)
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int kc = wave * KPW + kk;
      acc = mfma16(wq[kk], *(const bf16x8*)(xs + r16 * XST + kc * 32 + 8 * g4), acc);
    }
    *(f32x4*)(red + wave * 256 + lane * 4) = acc;
    __syncthreads();
    if (wave == 0) {   // the 8 K slices in order; lane: row m = lane & 15, columns 16 w + 4 g + i
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float s = 0.f;
#pragma unroll
        for (int wv = 0; wv < NW; ++wv) s += red[wv * 256 + lane * 4 + i];
        v[i] = s;
      }
      // epi_rope's arithmetic on the prefetched operands
      const int n0 = 16 * w, hh = n0 / D, tt = (n0 % D) >> 4, m = r16;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = rb(v[i] + bf(rb4[i]));   // q/k/v_proj output (bf16)
      if (hh < NH + NKV) {
        float u[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) u[i] = xor32(v[i]);
        if (g4 < 2 && m < R) {
          const int j = 8 * tt + 4 * g4;
          float cs[4], sn[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (RP.cs_tab) {
              cs[i] = bf(cs4[i]);
              sn[i] = bf(sn4[i]);
            } else {
              const float f = (float)rp * RP.inv_freq[j + i];
              cs[i] = rb(cosf(f));
              sn[i] = rb(sinf(f));
            }
          }
          bf16x4 o1, o2;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            o1[i] = tobf(rb(v[i] * cs[i]) + rb(-u[i] * sn[i]));
            o2[i] = tobf(rb(u[i] * cs[i]) + rb(v[i] * sn[i]));
          }
          bf16* dst = hh < NH ? RP.q_out + (long long)m * NH * D + hh * D
                              : RP.kv.k + (long long)RP.layer * RP.kv.s_layer + (long long)rs * RP.kv.s_slot +
                                    (long long)(hh - NH) * RP.kv.s_head + (long long)rp * D;
          MemWT::st8(dst + j, o1);
          MemWT::st8(dst + j + 64, o2);
        }
      } else if (m < R) {   // V cache in 32-position blocks of [dim][position] (common.h v_off)
        bf16* hb = RP.kv.v + (long long)RP.layer * RP.kv.s_layer + (long long)rs * RP.kv.s_slot +
                   (long long)(hh - NH - NKV) * RP.kv.s_head;
        const int dim0 = (n0 % D) + 4 * g4;
#pragma unroll
        for (int i = 0; i < 4; ++i) MemWT::st2(hb + v_off(dim0 + i, rp), tobf(v[i]));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  la_stamp(a, 2);
  __syncthreads();
  if (threadIdx.x == 0) ok_s[0] = hl_grid_wait_gen(a.sync, GEN, g0, 1, w, a.err) ? 1u : 0u;
  __syncthreads();
  la_stamp(a, 3);
  if (!ok_s[0]) return;
  if (ot && (a.variant & 2)) {
    const bf16* wp = hl_opaque(a.ow) + ((long long)(w - O0) * KC + wave * KPW) * 512 + ln * 8;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) wo[kk] = hl_ldnt(wp + (long long)kk * 512);
  }

  // ================= phase 2: attention units (row, kv head, 32 keys), one wave each
  const int U = pre[2 * R];
  for (int u = w + GRID * wave; u < U; u += GRID * NW) {
    int p = 0;
    while (pre[p + 1] <= u) ++p;
    const int qi = p / NKV, kh = p - qi * NKV, c0 = (u - pre[p]) * 32;
    const int len = RP.pos[qi] + 1, w1 = min(len, c0 + 32);
    const long long cbase = (long long)RP.layer * RP.kv.s_layer + (long long)RP.slots[qi] * RP.kv.s_slot +
                            (long long)kh * RP.kv.s_head;
    const bf16* K = RP.kv.k + cbase;
    const bf16* VB = RP.kv.v + cbase;
    bf16x8 qf[4], kf[2][4], vf[8];
    const bf16* qrow = RP.q_out + (long long)qi * NH * D + (kh * G + min(r16, G - 1)) * D + 8 * g4;
#pragma unroll
    for (int c = 0; c < 4; ++c) qf[c] = MemWT::ld16(qrow + 32 * c);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int key = min(c0 + 16 * tt + r16, w1 - 1);
#pragma unroll
      for (int c = 0; c < 4; ++c) kf[tt][c] = hl_ldnt(K + (long long)key * D + 32 * c + 8 * g4);
    }
    const int kb = min(c0 + 8 * g4, (w1 - 1) & ~7);
#pragma unroll
    for (int j = 0; j < 8; ++j) vf[j] = hl_ldnt(VB + v_off(16 * j + r16, kb));
    if (r16 >= G) {
#pragma unroll
      for (int c = 0; c < 4; ++c) qf[c] = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
    if (c0 + 32 > w1) {   // the row's tail unit: keys kb + e >= w1 contribute nothing
      const int kb2 = c0 + 8 * g4;
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) vf[j][e] = kb2 + e < w1 ? vf[j][e] : (bf16)0.f;
    }
    f32x4 sacc[2];   // lane: S[head 4 g + i][key c0 + 16 tt + r]
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      sacc[tt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 4; ++c) sacc[tt] = mfma16(qf[c], kf[tt][c], sacc[tt]);
    }
    float mv[4], lv[4], pp[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float s0 = c0 + r16 < w1 ? sacc[0][i] * a.scale : -INFINITY;
      const float s1 = c0 + 16 + r16 < w1 ? sacc[1][i] * a.scale : -INFINITY;
      const float mx = la_max16(fmaxf(s0, s1));
      pp[0][i] = __expf(s0 - mx);
      pp[1][i] = __expf(s1 - mx);
      lv[i] = la_sum16(pp[0][i] + pp[1][i]);
      mv[i] = mx;
    }
    bf16* ptw = pt + wave * 512;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 4; ++i) ptw[(4 * g4 + i) * 32 + 16 * tt + r16] = (bf16)pp[tt][i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bf16x8 pa = *(const bf16x8*)(ptw + r16 * 32 + 8 * g4);
    f32x4 o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = mfma16(pa, vf[j], (f32x4){0.f, 0.f, 0.f, 0.f});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // the unit's partial: O[head][dim], then (m, l) per head.  O goes through this
    // wave's 3 KB of LDS (xs is free in this phase) so that each lane stores whole
    // 16-byte pieces (as 8-byte write-through halves: narrower sc1 stores cost
    // several times more per byte)
    float* pu = a.part + (long long)u * PART;
    float* ow = (float*)xs + wave * (G * D);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 4 * g4 + i;
      if (h < G) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ow[h * D + 16 * j + r16] = o[j][i];
        if (r16 == 0) {
          const float2 mlv = make_float2(mv[i], lv[i]);
          __hip_atomic_store((gu64*)(pu + G * D + 2 * h), __builtin_bit_cast(unsigned long long, mlv),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < G * D / 256; ++q) {
      const f32x4 v4 = *(const f32x4*)(ow + (q * 64 + lane) * 4);
      const u64x2 uv = __builtin_bit_cast(u64x2, v4);
      __hip_atomic_store((gu64*)(pu + (q * 64 + lane) * 4), uv[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((gu64*)(pu + (q * 64 + lane) * 4 + 2), uv[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the LDS reads done before the next unit's writes
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  la_stamp(a, 4);
  __syncthreads();
  if (threadIdx.x == 0) ok_s[0] = hl_grid_wait_gen(a.sync, GEN, g0, 2, w, a.err) ? 1u : 0u;
  __syncthreads();
  la_stamp(a, 5);
  if (!ok_s[0]) return;

  // ================= phase 3: merge, one wave per (row, query head); lane: dims 2 l, 2 l + 1.
  // One round of loads for <= 32 units: lane u's (m, l) of units u and u + 64, and
  // every lane's O pairs of units 0..31, issued together; the weights
  // e_u = e^{m_u - M} then reach every lane by readlane, summed in unit order.
  for (int x = w + GRID * wave; x < R * NH; x += GRID * NW) {
    const int qi = x / NH, hq = x - qi * NH, kh = hq / G, h = hq - kh * G;
    const int u0 = pre[qi * NKV + kh], nu = pre[qi * NKV + kh + 1] - u0;   // 1 .. LA_MAX_KEYS / 32
    const float* pb = a.part + (long long)u0 * PART;
    const unsigned long long ml0 = MemWT::l64(pb + (long long)min(lane, nu - 1) * PART + G * D + 2 * h);
    const unsigned long long ml1 = MemWT::l64(pb + (long long)min(lane + 64, nu - 1) * PART + G * D + 2 * h);
    unsigned long long ov[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) ov[q] = MemWT::l64(pb + (long long)min(q, nu - 1) * PART + h * D + 2 * lane);
    const float m0 = lane < nu ? __uint_as_float((unsigned)ml0) : -INFINITY;
    const float m1 = lane + 64 < nu ? __uint_as_float((unsigned)ml1) : -INFINITY;
    const float M = wave_max(fmaxf(m0, m1));
    const float e0 = lane < nu ? __expf(m0 - M) : 0.f, e1 = lane + 64 < nu ? __expf(m1 - M) : 0.f;
    const float el0 = e0 * __uint_as_float((unsigned)(ml0 >> 32)), el1 = e1 * __uint_as_float((unsigned)(ml1 >> 32));
    float n0 = 0.f, n1 = 0.f, den = 0.f;
    for (int s0 = 0; s0 < nu; s0 += 32) {
      if (s0) {
#pragma unroll
        for (int q = 0; q < 32; ++q) ov[q] = MemWT::l64(pb + (long long)min(s0 + q, nu - 1) * PART + h * D + 2 * lane);
      }
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int u = s0 + q;
        if (u < nu) {
          const float e = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u < 64 ? e0 : e1), u & 63));
          const float el = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(u < 64 ? el0 : el1), u & 63));
          n0 += e * __uint_as_float((unsigned)ov[q]);
          n1 += e * __uint_as_float((unsigned)(ov[q] >> 32));
          den += el;
        }
      }
    }
    const bf16 b0 = tobf(n0 / den), b1 = tobf(n1 / den);
    const unsigned bits = (unsigned)__builtin_bit_cast(unsigned short, b0) |
                          ((unsigned)__builtin_bit_cast(unsigned short, b1) << 16);
    __hip_atomic_store((hl_gu32*)(a.att + (long long)qi * H + hq * D + 2 * lane), bits, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  la_stamp(a, 6);
  __syncthreads();
  if (threadIdx.x == 0) ok_s[0] = hl_grid_wait_gen(a.sync, GEN, g0, 3, w, a.err) ? 1u : 0u;
  __syncthreads();
  la_stamp(a, 7);
  if (!ok_s[0] || !ot) return;

  // ================= phase 4: o_proj tile w - O0 over the attention rows + residual
  for (int q = wave; q < ((a.variant & 1) ? R * 3 : RMAX * 3); q += NW) {
    const int m = q / 3, i = q - m * 3;
    hl_dma16<true>(xs + m * XST + i * 512, a.att + (long long)min(m, R - 1) * H + (i * 64 + ln) * 8);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  {
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      const int kc = wave * KPW + kk;
      acc = mfma16(wo[kk], *(const bf16x8*)(xs + r16 * XST + kc * 32 + 8 * g4), acc);
    }
    *(f32x4*)(red + wave * 256 + lane * 4) = acc;
  }
  __syncthreads();
  if (wave == 0 && r16 < R) {   // EPI_RES: out = bf16(res + bf16(acc)), row m = lane & 15
    const int m = r16, n = 16 * (w - O0) + 4 * g4;
    const bf16x4 rv = (a.variant & 4) ? rv_pre : *(const bf16x4*)(rm_bf(a.res, m) + n);
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) s += red[wv * 256 + lane * 4 + i];
      o[i] = tobf(bf(rv[i]) + rb(s));
    }
    *(bf16x4*)(rm_bfw(a.out, m) + n) = o;
  }
  la_stamp(a, 8);
}

bool lm_attn_fits(int H, int nh, int nkv, int d, int R, int keys) {
  if (H != la::H || nh != la::NH || nkv != la::NKV || d != la::D || R < 1 || R > la::RMAX || keys < 1 ||
      keys > LA_MAX_KEYS)
    return false;
  static const bool ok = persist_resident_kernel((const void*)k_lm_attn, la::NT, la::TOTAL, la::GRID);
  return ok;
}

size_t lm_attn_part_floats(int R, int keys) { return (size_t)R * la::NKV * ((keys + 31) / 32) * la::PART; }

int launch_lm_attn(const LmAttnArgs& a, int keys, hipStream_t st) {
  if (!lm_attn_fits(la::H, la::NH, la::NKV, la::D, a.R, keys) || a.qkv.M != a.R || a.qkv.N != la::NQKV ||
      a.qkv.K != la::H || !a.qkv.epi.bias || !a.part || !a.att || !a.sync || !a.err)
    return 3;
  hipLaunchKernelGGL(k_lm_attn, dim3(la::GRID), dim3(la::NT), la::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
