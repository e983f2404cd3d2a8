// Device helpers of the GEMV / GEMM family shared by the per-op kernels
// (gemm.hip) and the persistent chain kernel (chain.hip): weight-stream loads,
// the A-operand transforms (XF_*) and the epilogues (EPI_*).
//
// Memory policy MP: every load of bytes that another workgroup may have written
// in the SAME launch, and every store of such bytes, goes through MP.  MemPlain
// (the per-op kernels: a kernel boundary publishes) is a plain access; MemWT
// (chain.hip) is the in-launch hand-off form of MI355X_MICROARCH.md's table,
// first row: write-through (sc1) stores, L1-bypassing (sc1) loads.
#pragma once
#include "kernels.h"

struct MemPlain {
  static DEV bf16x8 ld16(const bf16* p) { return *(const bf16x8*)p; }
  static DEV bf16x4 ld8(const bf16* p) { return *(const bf16x4*)p; }
  static DEV float ldf(const float* p) { return *p; }
  static DEV void st8(bf16* p, bf16x4 v) { *(bf16x4*)p = v; }
  static DEV void st2(bf16* p, bf16 v) { *p = v; }
  static DEV void stf(float* p, float v) { *p = v; }
};

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
// global (address_space 1) views: the hand-off words must be global_ accesses, never flat_
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned short gu16;
typedef __attribute__((address_space(1))) float gf32;
struct MemWT {
  static DEV unsigned long long l64(const void* p) {
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static DEV bf16x8 ld16(const bf16* p) {
    const u64x2 v = {l64(p), l64(p + 4)};
    return __builtin_bit_cast(bf16x8, v);
  }
  static DEV bf16x4 ld8(const bf16* p) { return __builtin_bit_cast(bf16x4, l64(p)); }
  static DEV float ldf(const float* p) { return __hip_atomic_load((gf32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
  static DEV void st8(bf16* p, bf16x4 v) {
    __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  static DEV void st2(bf16* p, bf16 v) {
    __hip_atomic_store((gu16*)p, __builtin_bit_cast(unsigned short, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  static DEV void stf(float* p, float v) { __hip_atomic_store((gf32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
};

// Weight-stream load.  Decode weights are read once per step (GBs against a
// 256 MB Infinity Cache), so they go out non-temporal (MI355X_MICROARCH.md
// "nt-weights"; -2.2 % step time against the default policy).
// KEEP (GemmArgs::keep): weights re-read soon — the diffusion head's 170 MB per
// step is read S times per token and stays in the Infinity Cache with the
// default policy (tools/head_mall.py: -7 % per head step).
template <bool KEEP = false>
DEV bf16x8 ldw(const bf16* p) {
  if (!KEEP) return __builtin_nontemporal_load((const bf16x8*)p);
  return *(const bf16x8*)p;
}

DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------ A transform
// Inverse RMS of rows [m0, m0 + nrows) (local index i -> inv_s[i]); same
// summation order as k_rmsnorm (lane-strided 8-element chunks, wave sum).
template <class MP = MemPlain>
DEV void row_inv(const RowMap& am, int M, int K, float eps, int m0, int nrows, float* inv_s, int wave, int NW,
                 int lane) {
  const int nch = K >> 3;
  for (int i = wave; i < nrows; i += NW) {
    const int m = m0 + i;
    float ss = 0.f;
    if (m < M) {
      const bf16* x = rm_bf(am, m);
      for (int c = lane; c < nch; c += 64) {
        const bf16x8 v = MP::ld16(x + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) inv_s[i] = rsqrtf(ss / (float)K + eps);
  }
}
DEV void row_inv(const GemmArgs& a, int m0, int nrows, float* inv_s, int wave, int NW, int lane) {
  row_inv<MemPlain>(a.a, a.M, a.K, a.xf.eps, m0, nrows, inv_s, wave, NW, lane);
}

template <int XF, class MP = MemPlain>
DEV bf16x8 xform(const GemmArgs& a, bf16x8 x, int m, int k, float inv) {
  bf16x8 o;
  if (XF == XF_NORM) {
    bf16x8 wv, sh, sc;
    if (a.xf.w) wv = *(const bf16x8*)(a.xf.w + k);
    const bf16* md = a.xf.mod ? a.xf.mod + (long long)m * a.xf.mod_ld : nullptr;
    if (md) {
      sh = *(const bf16x8*)(md + a.xf.shift_off + k);
      sc = *(const bf16x8*)(md + a.xf.scale_off + k);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = rb(bf(x[j]) * inv);
      if (a.xf.w) t = rb(t * bf(wv[j]));
      if (md) t = rb(rb(t * rb(1.0f + bf(sc[j]))) + bf(sh[j]));
      o[j] = tobf(t);
    }
  } else if (XF == XF_SILU_ADD) {
    const bf16x8 v = *(const bf16x8*)(a.xf.vec + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = tobf(silu_f(rb(bf(x[j]) + bf(v[j]))));
  } else {
    o = x;
  }
  return o;
}

// ------------------------------------------------------------------ epilogues
// One 16(n) x 16(m) MFMA tile in the C/D layout: lane l holds m = m0 + (l & 15),
// n = n0 + 4*(l >> 4) + i, i = 0..3.  Every lane of the wave must call this
// (cross-lane exchanges), rows m >= M are dropped inside.

// RoPE epilogue (Qwen2 q/k/v projection + apply_rotary_pos_emb + cache append;
// transformers modeling_qwen2.py:99-134, 195-247).  Packed q/k rows: tile tt of
// head h holds dims [8tt, 8tt+8) in rows 0..7 and [64+8tt, 64+8tt+8) in rows
// 8..15 (weights.py: _rope_pack); v rows are in natural order.
template <class MP = MemPlain>
DEV void epi_rope(const GemmArgs& a, int m, int n0, int lane, float v[4]) {
  const RopeEpi& R = a.rope;
  constexpr int d = 128;
  const int g = lane >> 4;
  if (a.epi.bias) {
    const bf16x4 b = *(const bf16x4*)(a.epi.bias + n0 + 4 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += bf(b[i]);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = rb(v[i]);  // q/k/v_proj output (bf16)
  const int h = n0 / d, tt = (n0 % d) >> 4;
  if (h < R.nh + R.nkv) {
    float u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = xor32(v[i]);
    if (g >= 2 || m >= a.M) return;
    const int j = 8 * tt + 4 * g;
    const int p = R.pos[m];
    // cos / sin: the engine's table holds exactly bf16(cosf / sinf(p * inv_freq))
    // (k_rope_table), so the table and the inline form are bit-identical
    float cs4[4], sn4[4];
    if (R.cs_tab) {
      const bf16x4 c4 = *(const bf16x4*)(R.cs_tab + (long long)p * d + j);
      const bf16x4 s4 = *(const bf16x4*)(R.cs_tab + (long long)p * d + 64 + j);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cs4[i] = bf(c4[i]);
        sn4[i] = bf(s4[i]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float f = (float)p * R.inv_freq[j + i];
        cs4[i] = rb(cosf(f));
        sn4[i] = rb(sinf(f));
      }
    }
    bf16x4 o1, o2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float cs = cs4[i], sn = sn4[i];
      o1[i] = tobf(rb(v[i] * cs) + rb(-u[i] * sn));
      o2[i] = tobf(rb(u[i] * cs) + rb(v[i] * sn));
    }
    bf16* dst = h < R.nh ? R.q_out + (long long)m * R.nh * d + h * d
                         : R.kv.k + (long long)R.layer * R.kv.s_layer + (long long)R.slots[m] * R.kv.s_slot +
                               (long long)(h - R.nh) * R.kv.s_head + (long long)p * d;
    MP::st8(dst + j, o1);
    MP::st8(dst + j + 64, o2);
  } else {
    if (m >= a.M) return;
    // V cache in 32-position blocks of [dim][position] (common.h v_off)
    const int hv = h - R.nh - R.nkv;
    bf16* hb = R.kv.v + (long long)R.layer * R.kv.s_layer + (long long)R.slots[m] * R.kv.s_slot +
               (long long)hv * R.kv.s_head;
    const int dim0 = (n0 % d) + 4 * g, p = R.pos[m];
#pragma unroll
    for (int i = 0; i < 4; ++i) MP::st2(hb + v_off(dim0 + i, p), tobf(v[i]));
  }
}

// CFG combine + DPM-Solver++ update (sample_speech_tokens,
// modeling_vibevoice_inference.py:717-724; DPMSolverMultistepScheduler.step,
// dpm_solver.py:935-1022) on the final linear's rows: rows [0, n) are the
// conditional and [n, 2n) the unconditional v-predictions, 2n <= 16 so row r and
// its partner r + n sit in the same 16-lane group.
template <class MP = MemPlain>
DEV void epi_dpm(const GemmArgs& a, const DpmEpi& P, int n0, int lane, const float v[4]) {
  const int g = lane >> 4, r = lane & 15, n = P.n;
  float e[4], u[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = rb(v[i]);  // final_layer.linear output (bf16, no bias)
#pragma unroll
  for (int i = 0; i < 4; ++i) u[i] = __shfl(e[i], (lane + n) & 63);
  if (r >= n) return;
  const DpmCoef& k = P.k;
  const long long off = (long long)r * a.N + n0 + 4 * g;
  const bf16x4 xv = MP::ld8(P.x + off);
  const bf16x4 mv = MP::ld8(P.m1 + off);
  bf16x4 xo, mo;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float c = e[i], un = u[i];
    const float vv = rb(un + rb(k.cfg * rb(c - un)));
    const float xs = bf(xv[i]);
    const float x0 = rb(rb(k.alpha_s * xs) - rb(k.sigma_s * vv));
    float out = k.c_x * xs - rb(k.c_d0 * x0);
    if (k.order == 2) {
      const float d1 = rb(k.inv_r0 * rb(x0 - bf(mv[i])));
      out = out - rb(k.c_d1 * d1);
    }
    if (P.noise) out = out + k.c_n * P.noise[off + i];
    xo[i] = tobf(out);
    mo[i] = tobf(x0);
  }
  MP::st8(P.x + off, xo);
  MP::st8(P.m1 + off, mo);
}

// Row-contiguous epilogue forms for tiles staged through LDS (k_gemm_xl): 8
// consecutive output columns n .. n+7 of row m per lane, so the stores are 16
// bytes and a wave instruction covers whole 128-byte row segments (epi_tile's
// lane holds 4 columns x 1 row: 16 rows x 32 bytes per instruction, 16 x 16 for
// SiLU*up -- the 16K-token gate|up GEMM spent 30 % of its time in those stores).
// Same arithmetic as epi_tile, value for value.
DEV bool a16(const void* p) { return ((unsigned long long)p & 15) == 0; }
DEV bool rm8(const RowMap& r) { return a16(r.base) && r.sT % 8 == 0 && r.sB % 8 == 0; }
DEV bool epi_row8_ok(const GemmArgs& a) {
  const EpiArgs& e = a.epi;
  if (e.pack) return true;   // host-checked (launch_gemm): EPI_SILU_MUL, 16-byte aligned base
  if (e.kind != EPI_STORE && e.kind != EPI_GELU && e.kind != EPI_RES && e.kind != EPI_SILU_MUL) return false;
  if (!rm8(e.out) || (e.bias && !a16(e.bias))) return false;
  if (e.kind == EPI_RES && (!rm8(e.res) || (e.gamma && !a16(e.gamma)) || (e.gate.base && !rm8(e.gate)))) return false;
  return true;
}
DEV void epi_row8(const GemmArgs& a, int m, int n, const float v_in[8]) {
  const EpiArgs& e = a.epi;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = v_in[i];
  if (e.bias) {
    const bf16x8 b = *(const bf16x8*)(e.bias + n);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += bf(b[i]);
  }
  bf16x8 o;
  if (e.kind == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = tobf(v[i]);
  } else if (e.kind == EPI_GELU) {
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = tobf(gelu_f(rb(v[i])));
  } else {  // EPI_RES
    const bf16x8 r = *(const bf16x8*)(rm_bf(e.res, m) + n);
    float s[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
    bool scaled = false;
    if (e.gamma || e.gate.base) {
      const bf16x8 gm = e.gamma ? *(const bf16x8*)(e.gamma + n) : *(const bf16x8*)(rm_bf(e.gate, m) + n);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = bf(gm[i]);
      scaled = true;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float y = rb(v[i]);
      if (scaled) y = rb(s[i] * y);
      o[i] = tobf(bf(r[i]) + y);
    }
  }
  *(bf16x8*)(rm_bfw(e.out, m) + n) = o;
}
// SiLU(gate) * up for act columns col .. col+7 of row m (gate / up: the 16-column
// tile's rows 0..7 / 8..15, epi_tile's EPI_SILU_MUL pairing)
DEV void epi_silu8(const GemmArgs& a, int m, int col, const float gt[8], const float up[8]) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = tobf(rb(silu_f(rb(gt[i]))) * rb(up[i]));
  if (a.epi.pack) {   // act row length N / 2; columns col .. col+7 = one lane's 16 bytes of a block
    const int na = a.N >> 1;
    bf16* p = (bf16*)a.epi.out.base + ((long long)(m >> 4) * (na >> 5) + (col >> 5)) * 512 +
              ((m & 15) + 16 * ((col & 31) >> 3)) * 8;
    *(bf16x8*)p = o;
  } else {
    *(bf16x8*)(rm_bfw(a.epi.out, m) + col) = o;
  }
}

// Row-contiguous RoPE epilogue (k_gemm_xl, the prefill's q|k|v projection):
// epi_rope's arithmetic for one row m and one 16-column q/k tile at n0 (lo = its
// columns 0..7 = dims j..j+7, hi = columns 8..15 = dims 64+j..), 16-byte stores
DEV bool rope_row8_ok(const GemmArgs& a) {
  const RopeEpi& R = a.rope;
  return a.epi.kind == EPI_ROPE && a16(R.q_out) && a16(R.kv.k) && a16(R.kv.v) && (!a.epi.bias || a16(a.epi.bias)) &&
         (!R.cs_tab || a16(R.cs_tab)) && R.kv.s_layer % 8 == 0 && R.kv.s_slot % 8 == 0 && R.kv.s_head % 8 == 0;
}
DEV void rope_qk8(const GemmArgs& a, int m, int n0, const float lo[8], const float hi[8]) {
  const RopeEpi& R = a.rope;
  constexpr int d = 128;
  float v[8], u[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = lo[i];
    u[i] = hi[i];
  }
  if (a.epi.bias) {
    const bf16x8 b0 = *(const bf16x8*)(a.epi.bias + n0), b1 = *(const bf16x8*)(a.epi.bias + n0 + 8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[i] += bf(b0[i]);
      u[i] += bf(b1[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[i] = rb(v[i]);
    u[i] = rb(u[i]);
  }
  const int h = n0 / d, j = ((n0 % d) >> 4) * 8, p = R.pos[m];
  float cs[8], sn[8];
  if (R.cs_tab) {
    const bf16x8 c8 = *(const bf16x8*)(R.cs_tab + (long long)p * d + j);
    const bf16x8 s8 = *(const bf16x8*)(R.cs_tab + (long long)p * d + 64 + j);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      cs[i] = bf(c8[i]);
      sn[i] = bf(s8[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float f = (float)p * R.inv_freq[j + i];
      cs[i] = rb(cosf(f));
      sn[i] = rb(sinf(f));
    }
  }
  bf16x8 o1, o2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    o1[i] = tobf(rb(v[i] * cs[i]) + rb(-u[i] * sn[i]));
    o2[i] = tobf(rb(u[i] * cs[i]) + rb(v[i] * sn[i]));
  }
  bf16* dst = h < R.nh ? R.q_out + (long long)m * R.nh * d + h * d
                       : R.kv.k + (long long)R.layer * R.kv.s_layer + (long long)R.slots[m] * R.kv.s_slot +
                             (long long)(h - R.nh) * R.kv.s_head + (long long)p * d;
  *(bf16x8*)(dst + j) = o1;
  *(bf16x8*)(dst + j + 64) = o2;
}
// V column n (one dim) of rows m0 .. m0+7 into the blocked V cache: one 16-byte
// store when the 8 rows are consecutive positions p0 .. p0+7 (p0 % 8 == 0) of one
// slot -- a prompt's rows -- else 8 two-byte stores (epi_rope's form)
DEV void rope_v8(const GemmArgs& a, int m0, int n, const float vin[8]) {
  const RopeEpi& R = a.rope;
  const float b = a.epi.bias ? bf(a.epi.bias[n]) : 0.f;
  const int dim = n % 128, hv = n / 128 - R.nh - R.nkv;
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = tobf(rb(vin[k] + b));
  const long long hoff = (long long)R.layer * R.kv.s_layer + (long long)hv * R.kv.s_head;
  bool run = m0 + 7 < a.M;
  const int s0 = run ? R.slots[m0] : 0, p0 = run ? R.pos[m0] : 0;
  run = run && (p0 & 7) == 0;
  if (run) {
#pragma unroll
    for (int k = 1; k < 8; ++k) run = run && R.slots[m0 + k] == s0 && R.pos[m0 + k] == p0 + k;
  }
  if (run) {
    *(bf16x8*)(R.kv.v + hoff + (long long)s0 * R.kv.s_slot + v_off(dim, p0)) = o;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (m0 + k < a.M)
        R.kv.v[hoff + (long long)R.slots[m0 + k] * R.kv.s_slot + v_off(dim, R.pos[m0 + k])] = o[k];
  }
}

template <class MP = MemPlain>
DEV void epi_tile(const GemmArgs& a, int m, int n0, int lane, const float v_in[4]) {
  const EpiArgs& e = a.epi;
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = v_in[i];
  const int g = lane >> 4;
  if (e.kind == EPI_ROPE) {
    epi_rope<MP>(a, m, n0, lane, v);
    return;
  }
  if (e.kind == EPI_CFG_DPM) {
    epi_dpm<MP>(a, a.dpm, n0, lane, v);
    return;
  }
  if (e.kind == EPI_SILU_MUL) {
    // rows 0..7 of the tile are gate, 8..15 the matching up rows; lane g<2 holds
    // gate rows 4g+i, lane g+2 holds up rows 8+4g+i
    float u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = xor32(v[i]);
    if (g >= 2 || m >= a.M) return;
    const int col = (n0 >> 1) + 4 * g;
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = tobf(rb(silu_f(rb(v[i]))) * rb(u[i]));
    MP::st8(rm_bfw(e.out, m) + col, o);
    return;
  }
  if (m >= a.M) return;
  const int n = n0 + 4 * g;
  if (e.bias) {
    const bf16x4 b = *(const bf16x4*)(e.bias + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += bf(b[i]);
  }
  if (e.kind == EPI_F32) {
    float* o = (float*)e.out.base + rm_off(e.out, m) + n;
#pragma unroll
    for (int i = 0; i < 4; ++i) MP::stf(o + i, v[i]);
    return;
  }
  bf16x4 o;
  if (e.kind == EPI_STORE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = tobf(v[i]);
  } else if (e.kind == EPI_GELU) {
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = tobf(gelu_f(rb(v[i])));
  } else {  // EPI_RES
    const bf16x4 r = MP::ld8(rm_bf(e.res, m) + n);
    float s[4] = {1.f, 1.f, 1.f, 1.f};
    bool scaled = false;
    if (e.gamma) {
      const bf16x4 gm = *(const bf16x4*)(e.gamma + n);
#pragma unroll
      for (int i = 0; i < 4; ++i) s[i] = bf(gm[i]);
      scaled = true;
    } else if (e.gate.base) {
      const bf16x4 gm = MP::ld8(rm_bf(e.gate, m) + n);
#pragma unroll
      for (int i = 0; i < 4; ++i) s[i] = bf(gm[i]);
      scaled = true;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float y = rb(v[i]);
      if (scaled) y = rb(s[i] * y);
      o[i] = tobf(bf(r[i]) + y);
    }
  }
  MP::st8(rm_bfw(e.out, m) + n, o);
}

