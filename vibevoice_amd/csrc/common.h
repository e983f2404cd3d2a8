// Shared device helpers for the VibeVoice MI355X (gfx950) kernels.
//
// Storage type is bf16 (__bf16); arithmetic is fp32.  `rb()` rounds a float to
// bf16 and back: the reference runs a bf16 model on the GPU
// (demo/inference_from_file.py:265) where every torch op rounds its output to
// bf16, so kernels call rb() exactly where a torch op boundary sits in the
// reference and keep fp32 everywhere else.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DEV __device__ __forceinline__

DEV float bf(bf16 x) { return (float)x; }
DEV bf16 tobf(float x) { return (bf16)x; }
// Round to bf16 and back (a rounding point of the reference's bf16 torch ops).
// The conversion is inline asm so the optimizer cannot see through it: written
// as (float)(bf16)x, LLVM narrows e.g. y + rb(g * v) into bf16 arithmetic and
// then contracts it into one FMA, dropping the product's rounding.
DEV float rb(float x) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, 0" : "=v"(r) : "v"(x));
  return __uint_as_float(r << 16);
}

// MFMA 16x16x32 bf16 -> fp32: a = 16 rows x 32 k (lane l: row l & 15, k 8(l >> 4)..+7),
// b likewise for the 16 columns; d lane l: column l & 15, rows 4(l >> 4) + i
DEV f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// V cache of one (layer, slot, kv head): positions in blocks of 32, each block
// [128 dims][32 positions] (8 KB contiguous) -- attention's P.V operand loads
// (8 positions of one dim per lane) then read whole 1 KB pieces instead of
// 64 B slices of rows max_ctx apart (64K context: 37 -> see DESIGN.md).
// Element (dim i, position p):
DEV long long v_off(int i, int p) { return (long long)(p >> 5) * (128 * 32) + i * 32 + (p & 31); }

DEV float silu_f(float x) { return x / (1.0f + __expf(-x)); }
// GELU, exact erf form (transformers ACT2FN["gelu"]; modular_vibevoice_tokenizer.py:589)
DEV float gelu_f(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }

// GELU with erf by Abramowitz & Stegun 7.1.26 (|erf error| <= 1.5e-7, branch-free:
// one reciprocal, one exp, a degree-5 polynomial) -- for VALU-bound epilogues over
// many rows (codec_tile.hip); the result is rounded to bf16 by the caller.
DEV float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __frcp_rn(1.0f + 0.3275911f * z);
  const float p = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float e = 1.0f - p * __expf(-z * z);          // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + copysignf(e, x));
}

// Whole-wave sum: the four 16-lane rows by DPP butterflies (quad xor 1, 2,
// half-row and row mirror), then across rows by gfx950's v_permlane16_swap /
// v_permlane32_swap -- VALU moves instead of six dependent ds_bpermute LDS round
// trips (every normalising GEMV prologue and k_rmsnorm run one per row).  Each
// step adds a lane pair in both orders, so every lane ends with the same bits.
// Call with the whole wave active.
template <int CTRL>
DEV float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of N lanes (N = 2 .. 64), same step order for every N
template <int N>
DEV float group_sum(float v) {
  if (N >= 2) v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  if (N >= 4) v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  if (N >= 8) v += dpp_mov<0x141>(v);   // row_half_mirror
  if (N >= 16) v += dpp_mov<0x140>(v);  // row_mirror
  if (N >= 32) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  }
  if (N >= 64) {
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(b[0]) + __uint_as_float(b[1]);
  }
  return v;
}
DEV float wave_sum(float v) { return group_sum<64>(v); }
// runtime group width (a wave-uniform power of two <= 64; every lane of a group active)
DEV float group_sum_n(float v, int n) {
  switch (n) {
    case 64: return group_sum<64>(v);
    case 32: return group_sum<32>(v);
    case 16: return group_sum<16>(v);
    case 8: return group_sum<8>(v);
    case 4: return group_sum<4>(v);
    case 2: return group_sum<2>(v);
    default: return v;
  }
}
// the lane 32 apart (lane l < 32: l + 32, else l - 32), by v_permlane32_swap
DEV float xor32(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((__lane_id() & 32) ? a[0] : a[1]);
}
// Row addressing shared by every kernel that reads or writes "rows".
// Logical row m belongs to group g = m / T (a sample), row t = m % T inside it.
// The group's storage slot is idx[g] when idx != nullptr (streaming state is
// kept per sample slot), else g.  Offsets are in elements.
struct RowMap {
  void* base;
  long long sB;   // elements between slots
  long long sT;   // elements between rows of one slot
  int T;          // rows per group
  int pad_;
  const int* idx; // device int[groups] or nullptr
};

DEV long long rm_off(const RowMap& r, int m) {
  if (r.T == (1 << 30) && !r.idx) return (long long)m * r.sT;   // a plain row-major map (no division)
  int g = m / r.T;
  int t = m - g * r.T;
  long long s = r.idx ? (long long)r.idx[g] : (long long)g;
  return s * r.sB + (long long)t * r.sT;
}
DEV const bf16* rm_bf(const RowMap& r, int m) { return (const bf16*)r.base + rm_off(r, m); }
// a map known to have no slot table (r.idx == nullptr): no conditional load
DEV const bf16* rm_bf_plain(const RowMap& r, int m) {
  const int g = m / r.T;
  return (const bf16*)r.base + (long long)g * r.sB + (long long)(m - g * r.T) * r.sT;
}
DEV bf16* rm_bfw(const RowMap& r, int m) { return (bf16*)r.base + rm_off(r, m); }

// Epilogues (what a GEMM does with acc = sum_k A[m,k] W[n,k]):
enum {
  EPI_STORE = 0,     // y = bf16(acc + bias)
  EPI_GELU = 1,      // y = bf16(gelu(bf16(acc + bias)))
  EPI_SILU_MUL = 2,  // W rows packed [gate 8 | up 8] per 16: y = bf16(bf16(silu(bf16 g)) * bf16 u)
  EPI_RES = 3,       // y = bf16(res + bf16(s * bf16(acc + bias)))  s: none / gamma[n] / gate[m,n]
  EPI_F32 = 4,       // y(float) = acc + bias
  EPI_ROPE = 5,      // Qwen2 q|k|v rows (rope-paired packing): RoPE q -> q_out, RoPE k / v -> KV cache
  EPI_CFG_DPM = 6,   // diffusion-head final rows [cond n | uncond n]: CFG combine + DPM-Solver++ step
};

// Transforms applied to the A operand as it is loaded (fused producers):
enum {
  XF_NONE = 0,
  XF_NORM = 1,       // a = RMSNorm(row)[*w][modulate(shift, scale)]   (row = whole K)
  XF_SILU_ADD = 2,   // a = bf16(silu(bf16(row + vec)))
  XF_MIX = 3,        // a = ffn_norm(x + gamma * dwconv(norm(x)))  (codec Block1D, M <= 16)
  XF_ATTN_MERGE = 4, // a = the attention output merged from its key splits' partials (o_proj, M <= 16)
};

struct EpiArgs {
  int kind;
  int pack;             // EPI_SILU_MUL on the 256 x 256 tile: out.base receives the act rows
                        // MFMA-fragment-packed (the next GEMM's A, GemmArgs::apack)
  const bf16* bias;     // [N] or nullptr
  RowMap out;           // bf16 (float for EPI_F32)
  RowMap res;           // residual rows (EPI_RES), may alias out
  const bf16* gamma;    // [N] per-column scale (EPI_RES) or nullptr
  RowMap gate;          // per-(m,n) scale (EPI_RES) when gate.base != nullptr
};
