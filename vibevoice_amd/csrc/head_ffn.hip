// One diffusion-head FFN layer per launch at decode batch (2n <= 4 rows):
//   x += gate * down(SiLU(gate_proj(h)) * up_proj(h)),  h = modulate(norm(x), shift, scale)
// (modular_vibevoice_diffusion_head.py:96-161, HeadLayer.forward + FeedForwardNetwork).
//
// Why (DESIGN.md "Fused head FFN"): at B = 1 the head runs S x L = 40 of these
// layers per token as two GEMV launches each (gate|up, then down), and each
// launch pays a kernel boundary, a ramp with its weight stream not yet started,
// the A rows' dependent round trip and an epilogue tail.  Here the down
// projection is a split-K over each workgroup's own SwiGLU hidden slice:
//   * workgroup w owns hidden units [18w, 18w + 18) of F = 4,608 (G = 256
//     workgroups, one per CU); it streams their 36 gate / up rows (110 KB into
//     registers) and the matching 18 rows of down_proj^T (55 KB by LDS DMA),
//     all issued at entry, so the layer's 42.5 MB stream never waits on an input;
//   * it writes its [R][H] fp32 partial of down to its own slab (write-through),
//     arrives on an XCD-sharded counter, and waits for the grid (bounded);
//   * then every workgroup reduces 12 (R = 2) of the R x H outputs over the 256
//     slabs in a FIXED order (slab-major 16 x 16 tree), so results are
//     deterministic, and applies the gated residual.
// (A barrier-free form -- partials tagged with the launch generation, each
// reducer polling its slabs' tags -- measured 22 us per layer against 15 us:
// write-through stores took ~4 us to become visible and the polls flooded the
// memory system; tools/head_ffn_stamps.py, DESIGN.md "Fused head FFN".)
// Arithmetic: the A transform is k_gemv1's term for term (row_inv's summation
// order, xform's rounding points), SiLU*up and the gated residual round as
// epi_silu8 / epi_row8; the dot products run on v_dot2c_f32_bf16 (fp32
// accumulation of exact bf16 products), a different summation order than the
// MFMA path -- within the head's parity bounds, not bit-identical to it.
//
// Grid wait: every workgroup must be resident at once.  G = 256 <= the CU
// count, and a workgroup (9 waves, <= 96 VGPRs, <= 68 KB LDS) leaves room for a
// second one per CU, so two such launches from two engines also fit together.
// The wait gives up after ~200 ms (error word; vv_sync_error), never hangs.
// Counters are monotonic (no per-launch memset): shard s counts arrivals of the
// workgroups w % 8 == s (32 per launch), its 32nd arrival of a launch bumps the
// top counter, whose 8th bumps the generation word the waiters poll; all
// periods divide 2^32, so wrap-around keeps the counts aligned.
#include "gemv_dev.h"

// the LDS DMA below sets m0 in inline asm: listed as clobbered for the reader,
// though hipcc reserves m0 (no other instruction of these kernels uses it)
#pragma clang diagnostic ignored "-Winline-asm"

namespace hf {
constexpr int H = 1536, F = 4608, G = 256;
constexpr int HPW = F / G;          // hidden units per workgroup (18)
constexpr int ROWS = 2 * HPW;       // gate / up rows per workgroup (36)
constexpr int NT = 576;             // threads (9 waves)
constexpr int NCH = H / 8;          // 16-byte chunks per row (192)
constexpr int KS = NT / ROWS;       // lanes per gate / up row (16, one DPP row)
constexpr int CPT = NCH / KS;       // chunks per lane per row (12)
constexpr int PS = NT / NCH;        // down_proj subsets (3)
constexpr int UPS = HPW / PS;       // down rows per subset (6)
constexpr int LINE = 32;            // words per counter line
static_assert(ROWS * KS == NT && KS * CPT == NCH && PS * NCH == NT && PS * UPS == HPW, "head_ffn geometry");
static_assert(KS == 16, "the gate / up row reduction is one 16-lane DPP row");
}  // namespace hf

typedef __attribute__((address_space(1))) const bf16x8 hf_gbf16x8;
typedef __attribute__((address_space(1))) unsigned hf_gu32;
// global (not flat) loads: a flat load also counts in lgkmcnt, so the LDS waits
// of the prologue would wait for the weight stream
DEV bf16x8 hf_ld(const bf16* p) { return *(hf_gbf16x8*)p; }

DEV float dot8(bf16x8 w, bf16x8 x, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 0, 1), __builtin_shufflevector(x, x, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 2, 3), __builtin_shufflevector(x, x, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 4, 5), __builtin_shufflevector(x, x, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 6, 7), __builtin_shufflevector(x, x, 6, 7), acc, false);
  return acc;
}

// ST: the stamped diagnostic instantiation (its own copy, so the stores do not
// perturb the product kernel's wait counts)
template <int R, bool ST>
__global__ void __launch_bounds__(hf::NT) __attribute__((amdgpu_waves_per_eu(5))) k_head_ffn(HeadFfnArgs a) {
  using namespace hf;
  constexpr int E = R * H / G;                 // outputs reduced per workgroup (12 at R = 2)
  constexpr int APT = (R * NCH + NT - 1) / NT; // A chunks per thread
  static_assert(E % 2 == 0 && E * 16 <= NT, "head_ffn reduce geometry");
  __shared__ __attribute__((aligned(16))) bf16 xs[R * H];               // x rows, then the transformed rows
  // this workgroup's down_proj^T rows (LDS DMA, [UPS][NT][8]: lane t's 16 bytes
  // of row s at (s * NT + t) * 8); once read into registers, the same bytes hold
  // the down subsets 1, 2 (p2) and then the reduce scratch
  __shared__ __attribute__((aligned(16))) bf16 dn_s[UPS * NT * 8];
  __shared__ float inv_s[R], gu_s[ROWS * R], h_s[HPW * R];
  __shared__ unsigned ok_s;
  float* p2 = (float*)dn_s;
  static_assert(2 * NCH * R * 8 * 4 <= UPS * NT * 16 && (G * (E + 1) + E * 16) * 4 <= UPS * NT * 16,
                "p2 / reduce scratch fit in the down rows' LDS");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int w = blockIdx.x;
  auto stamp = [&](int k) {
    if constexpr (ST) {
      if (t == 0) a.stamps[w * 8 + k] = __builtin_amdgcn_s_memrealtime();
    }
  };
  stamp(0);
  if constexpr (ST) {   // placement: XCC_ID << 32 | HW_ID (cu / sh / se fields)
    if (t == 0)
      a.stamps[w * 8 + 6] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                            __builtin_amdgcn_s_getreg((31 << 11) | 4);
  }
  unsigned* gen = a.sync + 9 * LINE;
  // the generation at entry (before this workgroup arrives); read by every lane,
  // unconditionally, so no branch join waits for it ahead of the streams below
  const unsigned g0 = __hip_atomic_load((hf_gu32*)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

  // (1) A side first (vmcnt waits are in issue order): x, norm weight, shift,
  // scale of chunk q = (row q / NCH, chunk q % NCH); unconditional loads of a
  // clamped chunk, so the weight stream below keeps a static wait count
  bf16x8 xa[APT], nwa[APT], sha[APT], sca[APT];
#pragma unroll
  for (int k = 0; k < APT; ++k) {
    const int q = min(t + k * NT, R * NCH - 1), r = q / NCH, c = q - r * NCH;
    const bf16* md = a.mod + r * a.ldmod;
    xa[k] = hf_ld(a.x + r * a.ldx + 8 * c);
    nwa[k] = hf_ld(a.nw + 8 * c);
    sha[k] = hf_ld(md + a.shift_off + 8 * c);
    sca[k] = hf_ld(md + a.scale_off + 8 * c);
  }
  // the epilogue's gate and residual values of this workgroup's outputs, now (the
  // residual rows are this launch's x: nobody writes them before the grid wait)
  const int f0 = w * E;
  bf16 gate_pre, res_pre;
  {
    const int f = f0 + min(t, E - 1), r = f / H, col = f - r * H;
    gate_pre = *(const __attribute__((address_space(1))) bf16*)(a.mod + r * a.ldmod + a.gate_off + col);
    res_pre = *(const __attribute__((address_space(1))) bf16*)(a.res + r * a.ldres + col);
  }
  // (2) the whole weight stream at once: this lane's gate / up row chunks into
  // registers, then its down_proj^T rows by LDS DMA (no registers: <= 96 VGPRs
  // keeps two workgroups per CU; head weights stay in the Infinity Cache:
  // default policy)
  // The DMA goes first: hipcc cannot tell its LDS target from xs, so the first
  // LDS store below waits for it -- which, issued ahead of the gate / up loads,
  // is a wait for the A side's round trip only, not for the register stream.
  bf16x8 wg[CPT], wd[UPS];
  const int q2 = t / NCH, c2 = t - q2 * NCH;
  const bf16* dp = a.dn + (long long)(w * HPW + q2 * UPS) * H + 8 * c2;
  // (inline asm: the builtin makes hipcc drain every load, vmcnt(0), before the
  // first LDS access that follows, as it cannot tell dn_s from xs; its own wait
  // counts stay exact for the register loads issued after these)
#pragma unroll
  for (int s = 0; s < UPS; ++s) {
    const unsigned lds = __builtin_amdgcn_readfirstlane(
        (unsigned)(unsigned long long)(__attribute__((address_space(3))) bf16*)(dn_s + (s * NT + 64 * wave) * 8));
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(dp + (long long)s * H)
                 : "memory", "m0");
  }
  const bf16* gp = a.gu + ((long long)w * CPT * NT + t) * 8;
#pragma unroll
  for (int i = 0; i < CPT; ++i) wg[i] = hf_ld(gp + (long long)i * NT * 8);

  // (3) x rows to LDS; inverse RMS in row_inv's order (lane l: chunks l, l + 64, ...)
#pragma unroll
  for (int k = 0; k < APT; ++k)
    if (t + k * NT < R * NCH) *(bf16x8*)(xs + 8 * (t + k * NT)) = xa[k];
  __syncthreads();
  if (wave < R) {
    float ss = 0.f;
    for (int c = lane; c < NCH; c += 64) {
      const bf16x8 v = *(const bf16x8*)(xs + wave * H + 8 * c);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
    }
    ss = wave_sum(ss);
    if (lane == 0) inv_s[wave] = rsqrtf(ss / (float)H + a.eps);
  }
  __syncthreads();
  // modulate(norm(x)): xform<XF_NORM>'s rounding points
#pragma unroll
  for (int k = 0; k < APT; ++k) {
    const int q = t + k * NT;
    if (q < R * NCH) {
      const float inv = inv_s[q / NCH];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = rb(bf(xa[k][j]) * inv);
        v = rb(v * bf(nwa[k][j]));
        v = rb(rb(v * rb(1.0f + bf(sca[k][j]))) + bf(sha[k][j]));
        o[j] = tobf(v);
      }
      *(bf16x8*)(xs + 8 * q) = o;
    }
  }
  __syncthreads();
  stamp(1);

  // (4) gate / up: row rho = t / KS of this workgroup's 36 (2u = gate of unit u,
  // 2u + 1 = its up), chunks i * KS + kap; the 16 lanes of a row reduce by DPP
  {
    const int rho = t / KS, kap = t - rho * KS;
    float acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = i * KS + kap;
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = dot8(wg[i], *(const bf16x8*)(xs + r * H + 8 * c), acc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = group_sum<16>(acc[r]);
    if (kap == 0)
#pragma unroll
      for (int r = 0; r < R; ++r) gu_s[rho * R + r] = acc[r];
  }
  __syncthreads();
  stamp(2);
  if (t < HPW * R) {   // SiLU(gate) * up, rounded to the bf16 activation (epi_silu8)
    const int u = t / R, r = t - u * R;
    const float g = gu_s[2 * u * R + r], up = gu_s[(2 * u + 1) * R + r];
    h_s[u * R + r] = bf(tobf(rb(silu_f(rb(g))) * rb(up)));
  }
  __syncthreads();

  // (5) down: subset q2 of 6 hidden units x columns [8 c2, 8 c2 + 8); subsets
  // summed 0 + 1 + 2 in that order; the workgroup's partial to its slab
  // this lane's own DMA'd down rows (the DMA is older than every load still
  // counted), then the barrier before the region is reused as p2
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < UPS; ++s) wd[s] = *(const bf16x8*)(dn_s + (s * NT + t) * 8);
  __syncthreads();
  float y[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) y[r][e] = 0.f;
#pragma unroll
  for (int s = 0; s < UPS; ++s) {
    float wf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) wf[e] = bf(wd[s][e]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float hv = h_s[(q2 * UPS + s) * R + r];
#pragma unroll
      for (int e = 0; e < 8; ++e) y[r][e] = fmaf(hv, wf[e], y[r][e]);
    }
  }
  if (q2 > 0) {
    float* d = p2 + ((q2 - 1) * NCH + c2) * R * 8;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int e = 0; e < 8; e += 4) *(f32x4*)(d + r * 8 + e) = (f32x4){y[r][e], y[r][e + 1], y[r][e + 2], y[r][e + 3]};
  }
  __syncthreads();
  if (q2 == 0) {   // the workgroup's partial, written through (sc1), then the arrival
    const float* d1 = p2 + c2 * R * 8;
    const float* d2 = p2 + (NCH + c2) * R * 8;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float* sl = a.slab + ((long long)w * R + r) * H + 8 * c2;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const float v0 = (y[r][e] + d1[r * 8 + e]) + d2[r * 8 + e];
        const float v1 = (y[r][e + 1] + d1[r * 8 + e + 1]) + d2[r * 8 + e + 1];
        const unsigned long long b =
            (unsigned long long)__float_as_uint(v0) | ((unsigned long long)__float_as_uint(v1) << 32);
        __hip_atomic_store((gu64*)(sl + e), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the slab is written through before the arrival
  }
  __syncthreads();
  stamp(3);

  // (6) arrival and the bounded grid wait
  if (t == 0) {
    unsigned ok = 1;
    const unsigned v = __hip_atomic_fetch_add((hf_gu32*)(a.sync + (w & 7) * LINE), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if ((v + 1) % (G / 8) == 0) {
      const unsigned v2 = __hip_atomic_fetch_add((hf_gu32*)(a.sync + 8 * LINE), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      if ((v2 + 1) % 8 == 0) __hip_atomic_fetch_add((hf_gu32*)gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load((hf_gu32*)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // ~200 ms at 100 MHz
        __hip_atomic_store((hf_gu32*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    ok_s = ok;
  }
  __syncthreads();
  if (!ok_s) return;

  // (7) outputs [f0, f0 + E) of the flat [R][H] block: slab p's values to LDS
  // (thread p), then 16 x 16 fixed-order partial sums, then the gated residual
  float* red = p2;
  float* s4 = p2 + G * (E + 1);
  if (t < G) {   // all of this lane's slab loads in flight, then the LDS stores
    const float* sl = a.slab + (long long)t * R * H + f0;
    unsigned long long b[E / 2];
#pragma unroll
    for (int k = 0; k < E / 2; ++k) b[k] = MemWT::l64(sl + 2 * k);
#pragma unroll
    for (int k = 0; k < E / 2; ++k) {
      red[t * (E + 1) + 2 * k] = __uint_as_float((unsigned)b[k]);
      red[t * (E + 1) + 2 * k + 1] = __uint_as_float((unsigned)(b[k] >> 32));
    }
  }
  __syncthreads();
  stamp(4);
  if (t < E * 16) {
    const int e = t >> 4, qq = t & 15;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) s += red[(qq * 16 + p) * (E + 1) + e];
    s4[e * 16 + qq] = s;
  }
  __syncthreads();
  if (t < E) {
    float s = 0.f;
#pragma unroll
    for (int qq = 0; qq < 16; ++qq) s += s4[t * 16 + qq];
    const int f = f0 + t, r = f / H, col = f - r * H;
    float v = rb(s);
    v = rb(bf(gate_pre) * v);
    a.out[r * a.ldx + col] = tobf(bf(res_pre) + v);
  }
  stamp(5);
}

bool head_ffn_fits(int H, int F, int R) {
  return H == hf::H && F == hf::F && (R == 2 || R == 4) && head_ffn_grid() >= hf::G;
}

// the CU count (every workgroup of the grid wait must be resident at once)
int head_ffn_grid() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return cus;
}

int launch_head_ffn(const HeadFfnArgs& a, hipStream_t st) {
  if (!head_ffn_fits(hf::H, hf::F, a.R)) return 1;
  if (a.stamps) {
    if (a.R == 2) hipLaunchKernelGGL((k_head_ffn<2, true>), dim3(hf::G), dim3(hf::NT), 0, st, a);
    else hipLaunchKernelGGL((k_head_ffn<4, true>), dim3(hf::G), dim3(hf::NT), 0, st, a);
  } else if (a.R == 2) {
    hipLaunchKernelGGL((k_head_ffn<2, false>), dim3(hf::G), dim3(hf::NT), 0, st, a);
  } else {
    hipLaunchKernelGGL((k_head_ffn<4, false>), dim3(hf::G), dim3(hf::NT), 0, st, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
