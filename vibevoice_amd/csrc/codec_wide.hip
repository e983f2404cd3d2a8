// A whole wide codec stage (C = 256 at T = 200, C = 512 at T = 40: the acoustic
// decoder's third and fourth stages, the semantic encoder's fourth and fifth) in
// ONE launch: its three Block1Ds (modular_vibevoice_tokenizer.py:620-684),
// streaming form (:914-951), one frame of T rows per sample.
//
// Why not codec_tile.hip's form: a workgroup that owns a time tile would stream
// the stage's whole 3 (C = 256) or 12 MB (C = 512) of weights through one CU.
// Here a CLUSTER of S = C / 32 workgroups shares each 16-row time tile:
//   * every member recomputes the tile's causal halo and mixer (norm ->
//     depthwise conv -> gamma residual -> FFN norm) for all C channels
//     (codec_tile.hip's arithmetic: rows t < 0 from the conv histories);
//   * member s owns hidden units [128 s, 128 s + 128): fc1 over them (MFMA, its
//     8 weight tiles in registers, one per wave) -> GELU -> hidden slice in LDS
//     -> its K-slice of fc2 (MFMA) = an fp32 partial of the block output;
//   * reduce-scatter: member s sums output columns [32 s, 32 s + 32) over the S
//     partials (fixed order), + bias, ffn_gamma, + y -> bf16; all-gather: every
//     member reads the whole [rows][C] block output for the next block.
// So each CU streams only 128 KB of weights per block (one 16 x C fc1 tile and
// a 128-wide K slice of fc2 per wave), and the hand-offs stay inside a cluster:
// two cluster-wide waits per block (one for the last block, whose owners write
// the stage output rows directly).  Hand-off stores are write-through, loads sc1
// (persist_dev.h conventions); a wait gives up after ~200 ms and sets the
// engine's error word (vv_sync_error*), it never hangs.  The launch needs its
// n x tiles x S workgroups co-resident (<= 256 at one per CU): the engine runs
// it only under the grid-waiting kernels' rule (persist_on) and otherwise takes
// the launch-per-op path.
#include <atomic>

#include "persist_dev.h"

namespace cw {
constexpr int NTH = 512, NW = 8;
template <int C>
struct Geo {
  static constexpr int S = C / 32;               // cluster members (8 / 16)
  static constexpr int R = 16;                   // output rows per tile
  static constexpr int N8 = C / 8, RPP = NTH / N8;
  static constexpr int F = 4 * C, HSL = 128;     // hidden units per member
  static constexpr int NL = R + 18;              // local rows (halo of three k = 7 convs)
  static constexpr int XLD = C + 8, HLD = HSL + 8;
  static constexpr int NK1 = C / 32;             // fc1 K chunks (one 16-unit tile per wave)
  static constexpr int NTW2 = C / 16 / NW;       // fc2 output tiles per wave (2 / 4)
  static constexpr int NK2F = F / 32;            // fc2 K chunks of the whole hidden width
  static constexpr int PR = 40;                  // rows of a partial slab
  // LDS (bytes): x rows (y in place after the conv), conv input rows, fc1 input
  // rows, hidden slice (+16 rows: row tiles start at the block's first row)
  static constexpr int X = 0, X_B = NL * XLD * 2;
  static constexpr int NRM = X + X_B, NRM_B = (NL + 6) * XLD * 2;
  static constexpr int A = NRM + NRM_B, A_B = (NL + 16) * XLD * 2;
  static constexpr int H = A + A_B, H_B = (NL + 16) * HLD * 2;
  static constexpr int SM = H + H_B, SM_B = 16;
  static constexpr int TOTAL = SM + SM_B;
  static_assert(TOTAL <= 160 * 1024, "LDS");
  static_assert(C / S == 32 && F / S == HSL, "cluster geometry");
};
}  // namespace cw

DEV void cw_st16f(float* p, f32x4 v) {   // 16 B of fp32, write-through
  const u64x2 u = __builtin_bit_cast(u64x2, v);
  __hip_atomic_store((gu64*)p, u[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64*)(p + 2), u[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV f32x4 cw_ld16f(const float* p) {
  const u64x2 u = {MemWT::l64(p), MemWT::l64(p + 2)};
  return __builtin_bit_cast(f32x4, u);
}

template <int C>
__global__ void __launch_bounds__(cw::NTH, 1) k_codec_wide(CodecWideArgs a) {
  using G = cw::Geo<C>;
  using namespace cw;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + G::X);
  bf16* ns = (bf16*)(smem + G::NRM);
  bf16* as = (bf16*)(smem + G::A);
  bf16* hs = (bf16*)(smem + G::H);
  unsigned* ok_s = (unsigned*)(smem + G::SM);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int tile = blockIdx.x / G::S, s = blockIdx.x - tile * G::S, smp = blockIdx.y;
  const int ntiles = gridDim.x / G::S;
  const long long slot = a.slots[smp];
  const int T = a.T;
  const int t0 = tile * G::R, B = min(t0 + G::R, T);
  const int L0 = t0 - 18;
  const int S_lo = max(0, L0);
  const int c2 = tid % G::N8, rp = tid / G::N8;
  const bool last_tile = B == T;
  const int cluster = smp * ntiles + tile;
  unsigned* cnt = a.sync + (long long)cluster * pk::LINE;
  float* slab = a.slab + (long long)cluster * G::S * G::PR * C;
  bf16* xg = a.xbuf + (long long)cluster * G::PR * C;
  unsigned base = 0, nwait = 0;
  if (tid == 0)   // fewer than S arrivals can precede this read (this member's own is missing)
    base = __hip_atomic_load((hl_gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / G::S * G::S;
  auto stamp = [&](int k) {
    if (a.stamps && tid == 0)
      a.stamps[((long long)smp * gridDim.x + blockIdx.x) * 16 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // cluster-wide wait: every wave's write-through stores drained, one arrival,
  // lane 0 polls (bounded) -> false: gave up (error word set)
  auto cluster_wait = [&]() -> bool {
    ++nwait;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add((hl_gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
      unsigned ok = 1;
      while ((unsigned)(__hip_atomic_load((hl_gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - base) <
             (unsigned)G::S * nwait) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - tw > 20000000ull) {   // ~200 ms at 100 MHz
          __hip_atomic_store((hl_gu32*)a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      ok_s[0] = ok;
    }
    __syncthreads();
    return ok_s[0] != 0;
  };

  // ---------------------------------------------------------------- stage input rows [S_lo, B) -> X
  constexpr int QIN = (G::NL * G::N8 + NTH - 1) / NTH;
  bf16x8 vin[QIN];
#pragma unroll
  for (int q = 0; q < QIN; ++q) {
    const int e = min(tid + q * NTH, (B - S_lo) * G::N8 - 1);
    const int i = e / G::N8, c = e - i * G::N8;
    vin[q] = *(const bf16x8*)(a.x + ((long long)smp * T + S_lo + i) * C + c * 8);
  }
  // ---------------------------------------------------------------- operands of a block
  struct Aux {
    bf16x8 wn, bb, gv, wf, wk[7], hv;
    bf16x4 b1, b2, g2;
  };
  const int nu = s * G::HSL + wave * 16;        // this wave's fc1 tile: hidden units nu .. nu + 15
  const int rcol = s * 32 + 4 * (tid & 7);      // reduce-scatter: this thread's 4 output columns
  auto load_aux = [&](int j, Aux& x) {
    const CodecTileBlock& b = a.b[j];
    x.wn = *(const bf16x8*)(b.norm + c2 * 8);
    x.bb = *(const bf16x8*)(b.dw_b + c2 * 8);
    x.gv = *(const bf16x8*)(b.gamma + c2 * 8);
    x.wf = *(const bf16x8*)(b.ffn_norm + c2 * 8);
#pragma unroll
    for (int k = 0; k < 7; ++k) x.wk[k] = *(const bf16x8*)(b.dw_w + (size_t)c2 * 56 + k * 8);
    const int h = min(tid / G::N8, 5);
    x.hv = *(const bf16x8*)(b.mix + slot * b.mix_sB + (long long)h * C + c2 * 8);
    x.b1 = *(const bf16x4*)(b.fc1_b + nu + 4 * g4);
    x.b2 = *(const bf16x4*)(b.fc2_b + rcol);
    x.g2 = *(const bf16x4*)(b.ffn_gamma + rcol);
  };
  bf16x8 w1[G::NK1], w2[G::NTW2 * 4];
  auto load_w1 = [&](int j) {
    const bf16* f1 = a.b[j].fc1_w + (long long)(nu >> 4) * G::NK1 * 512 + lane * 8;
#pragma unroll
    for (int c = 0; c < G::NK1; ++c) w1[c] = *(const bf16x8*)(f1 + c * 512);
  };
  // (fc2's fragments go out after the block's mixer norm -- at C = 512 after its
  // fc1: issued with fc1's they made it spill)
  auto load_w2 = [&](int j) {
#pragma unroll
    for (int i = 0; i < G::NTW2; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        w2[i * 4 + c] = *(const bf16x8*)(a.b[j].fc2_w +
                                         ((long long)(wave * G::NTW2 + i) * G::NK2F + s * 4 + c) * 512 + lane * 8);
  };
  Aux ax;
  load_aux(0, ax);
  load_w1(0);
#pragma unroll
  for (int q = 0; q < QIN; ++q) {
    const int e = tid + q * NTH;
    if (e < (B - S_lo) * G::N8) {
      const int i = e / G::N8, c = e - i * G::N8;
      *(bf16x8*)(xs + (S_lo + i - L0) * G::XLD + c * 8) = vin[q];
    }
  }
  __syncthreads();
  stamp(1);

  bool ok = true;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const CodecTileBlock& bj = a.b[j];
    const int lo = max(0, L0 + 6 * (j + 1));
    const int cs = lo - 6;
    // ---- M1: conv input rows = norm(x) (history rows t < 0 from the buffer)
    if (tid < 6 * G::N8) {
      const int t = tid / G::N8 - 6;
      if (t >= cs) *(bf16x8*)(ns + (t - L0 + 6) * G::XLD + c2 * 8) = ax.hv;
    }
    for (int p = max(cs, 0); p < B; p += G::RPP) {
      const int t = p + rp, tc = min(t, B - 1);
      const bf16x8 v = *(const bf16x8*)(xs + (tc - L0) * G::XLD + c2 * 8);
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) ss += bf(v[q]) * bf(v[q]);
      ss = group_sum<G::N8>(ss);
      const float inv = rsqrtf(ss / (float)C + a.eps);
      bf16x8 o8;
#pragma unroll
      for (int q = 0; q < 8; ++q) o8[q] = tobf(rb(rb(bf(v[q]) * inv) * bf(ax.wn[q])));
      if (t < B) {
        *(bf16x8*)(ns + (t - L0 + 6) * G::XLD + c2 * 8) = o8;
        if (s == 0 && t >= T - 6) *(bf16x8*)(bj.mix + slot * bj.mix_sB + (long long)(6 + t) * C + c2 * 8) = o8;
      }
    }
    constexpr bool W2_LATE = G::NK1 > 8;   // C = 512: fc2's fragments only after fc1's are consumed (registers)
    if (!W2_LATE) load_w2(j);
    __syncthreads();
    // ---- M2: depthwise conv + gamma residual -> y (over x, in place); FFN norm -> fc1's input rows
    for (int p = lo; p < B; p += G::RPP) {
      const int t = p + rp, tc = min(t, B - 1);
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const bf16x8 v = *(const bf16x8*)(ns + (tc - L0 + k) * G::XLD + c2 * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int f = q * 7 + k;
          acc[q] += bf(ax.wk[f >> 3][f & 7]) * bf(v[q]);
        }
      }
      const bf16x8 xv = *(const bf16x8*)(xs + (tc - L0) * G::XLD + c2 * 8);
      bf16x8 y8;
      float ss = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        y8[q] = tobf(bf(xv[q]) + rb(rb(acc[q] + bf(ax.bb[q])) * bf(ax.gv[q])));
        ss += bf(y8[q]) * bf(y8[q]);
      }
      ss = group_sum<G::N8>(ss);
      const float inv = rsqrtf(ss / (float)C + a.eps);
      bf16x8 o8;
#pragma unroll
      for (int q = 0; q < 8; ++q) o8[q] = tobf(rb(rb(bf(y8[q]) * inv) * bf(ax.wf[q])));
      if (t < B) {   // (item (t, c2) is read and written by this thread alone: y over x in place)
        *(bf16x8*)(xs + (t - L0) * G::XLD + c2 * 8) = y8;
        *(bf16x8*)(as + (t - L0) * G::XLD + c2 * 8) = o8;
      }
    }
    __syncthreads();
    stamp(2 + 4 * j);
    const int rb0 = lo - L0, nmt = (B - lo + 15) >> 4;
    // ---- F1: this member's 128 hidden units (wave: one 16-unit tile) + GELU -> hidden slice
    {
      const bf16x4 b1 = ax.b1;
      for (int mt = 0; mt < nmt; ++mt) {
        const bf16* xrow = as + (rb0 + mt * 16 + r16) * G::XLD + 8 * g4;
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < G::NK1; ++c) acc = mfma16(w1[c], *(const bf16x8*)(xrow + c * 32), acc);
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = tobf(gelu_fast(rb(acc[q] + bf(b1[q]))));
        *(bf16x4*)(hs + (rb0 + mt * 16 + r16) * G::HLD + wave * 16 + 4 * g4) = o;
      }
    }
    if (W2_LATE) load_w2(j);
    __syncthreads();
    // ---- F2: the fc2 partial over this member's K slice -> its slab (write-through)
    for (int mt = 0; mt < nmt; ++mt) {
      const bf16* hrow = hs + (rb0 + mt * 16 + r16) * G::HLD + 8 * g4;
      bf16x8 hv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) hv[c] = *(const bf16x8*)(hrow + c * 32);
      const int t = lo + mt * 16 + r16;
#pragma unroll
      for (int i = 0; i < G::NTW2; ++i) {
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) acc = mfma16(w2[i * 4 + c], hv[c], acc);
        const int n = (wave * G::NTW2 + i) * 16 + 4 * g4;
        if (t < B) cw_st16f(slab + ((long long)s * G::PR + (t - L0)) * C + n, acc);
      }
    }
    stamp(3 + 4 * j);
    ok = cluster_wait() && ok;
    stamp(4 + 4 * j);
    // ---- reduce-scatter: output columns [32 s, 32 s + 32) of rows [lo, B), fixed member order
    {
      const int ri = tid >> 3;   // 64 rows per pass
      for (int p = lo; p < B; p += NTH / 8) {
        const int t = p + ri;
        if (t < B) {
          // the S partials in member order, 8 loads in flight at a time (registers)
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int m0 = 0; m0 < G::S; m0 += 8) {
            f32x4 v[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = cw_ld16f(slab + ((long long)(m0 + m) * G::PR + (t - L0)) * C + rcol);
#pragma unroll
            for (int m = 0; m < 8; ++m) acc = m0 + m == 0 ? v[m] : acc + v[m];
          }
          const bf16x4 yv = *(const bf16x4*)(xs + (t - L0) * G::XLD + rcol);
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = tobf(bf(yv[q]) + rb(bf(ax.g2[q]) * rb(acc[q] + bf(ax.b2[q]))));
          if (j < 2) MemWT::st8(xg + (long long)(t - L0) * C + rcol, o);
          else if (t >= t0) *(bf16x4*)(rm_bfw(a.out, smp * T + t) + rcol) = o;
        }
      }
    }
    if (j == 2) break;
    ok = cluster_wait() && ok;
    stamp(5 + 4 * j);
    // ---- all-gather: block j's output rows [lo, B) -> X; then block j+1's operands
    {
      constexpr int QG = (G::NL * G::N8 + NTH - 1) / NTH;
      bf16x8 gv[QG];
#pragma unroll
      for (int q = 0; q < QG; ++q) {
        const int e = min(tid + q * NTH, (B - lo) * G::N8 - 1);
        const int i = e / G::N8, c = e - i * G::N8;
        gv[q] = MemWT::ld16(xg + (long long)(lo + i - L0) * C + c * 8);
      }
      load_aux(j + 1, ax);
      load_w1(j + 1);
#pragma unroll
      for (int q = 0; q < QG; ++q) {
        const int e = tid + q * NTH;
        if (e < (B - lo) * G::N8) {
          const int i = e / G::N8, c = e - i * G::N8;
          *(bf16x8*)(xs + (lo + i - L0) * G::XLD + c * 8) = gv[q];
        }
      }
    }
    __syncthreads();
  }
  stamp(15);
}

// ================================================================ host
template <int C>
static int cw_launch(const CodecWideArgs& a, hipStream_t st) {
  using G = cw::Geo<C>;
  const int tiles = (a.T + G::R - 1) / G::R;
  hipLaunchKernelGGL(k_codec_wide<C>, dim3(tiles * G::S, a.n), dim3(cw::NTH), G::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Grids larger than one resident wave (B = 8: n x tiles x S = 384 / 832
// workgroups): only a CLUSTER waits on its own members, never on another
// cluster, and workgroups are dispatched in index order (x fastest, so a
// cluster's S members are consecutive).  The lowest-indexed cluster that is not
// wholly resident then only waits for slots held by lower-indexed workgroups, of
// complete clusters that finish without waiting on anything later -- so every
// cluster completes; the waits stay bounded (~200 ms, error word) regardless.
// Off by default: at B = 8 every one of the 832 / 384 workgroups re-reads its
// member's weights (320 MB of L2 / Infinity-Cache reads for the C = 256 stage),
// and the step measured 4.015 ms against 3.968 with the k_mix + GEMM path
// (same build, bench.py --batch 8); tests/test_gpu_codec.py runs it at n = 8.
static std::atomic<int> g_cw_over{0};
void codec_wide_oversubscribe(int on) { g_cw_over = on ? 1 : 0; }

template <int C>
static bool cw_resident(int n, int T) {
  using G = cw::Geo<C>;
  static const bool fits = persist_resident_kernel((const void*)k_codec_wide<C>, cw::NTH, G::TOTAL, 1);
  int dev = 0, cus = 0, nb = 0;
  if (!fits || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)k_codec_wide<C>, cw::NTH, G::TOTAL) != hipSuccess)
    return false;
  const int grid = n * ((T + G::R - 1) / G::R) * G::S;
  return persist_resident(nb, cus, 0, grid) || (g_cw_over && persist_resident(nb, cus, 0, G::S));
}

// shapes the cluster kernel takes, with every workgroup of the launch co-resident
bool codec_wide_fits(int C, int T, int n, int depth, int ctx) {
  if (depth != 3 || ctx != 6 || n < 1 || T < 1) return false;
  if (C == 256) return cw_resident<256>(n, T);
  if (C == 512) return cw_resident<512>(n, T);
  return false;
}

// workspace: sync lines per cluster, partial slabs, block outputs
size_t codec_wide_slab_floats(int C, int T, int n) {
  const int tiles = (T + 15) / 16;
  return (size_t)n * tiles * (C / 32) * 40 * C;
}
size_t codec_wide_xbuf_elems(int C, int T, int n) { return (size_t)n * ((T + 15) / 16) * 40 * C; }

int launch_codec_wide(const CodecWideArgs& a, int C, hipStream_t st) {
  if (a.n <= 0 || a.T <= 0) return 0;
  if (!codec_wide_fits(C, a.T, a.n, a.depth, 6)) return 3;
  if (C == 256) {
    static const bool attr = hipFuncSetAttribute((const void*)k_codec_wide<256>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, cw::Geo<256>::TOTAL) == hipSuccess;
    if (!attr) return 2;
    return cw_launch<256>(a, st);
  }
  static const bool attr = hipFuncSetAttribute((const void*)k_codec_wide<512>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, cw::Geo<512>::TOTAL) == hipSuccess;
  if (!attr) return 2;
  return cw_launch<512>(a, st);
}
