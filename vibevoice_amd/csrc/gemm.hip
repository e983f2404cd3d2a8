// bf16 MFMA GEMMs for gfx950:  Y[m, n] = epi( sum_k xf(A)[m, k] * W[n, k] )
//
// W is a PyTorch Linear weight [N, K], or a conv weight that the loader
// re-packed to the same [N, K] form (see vibevoice_amd/weights.py), stored in
// MFMA-fragment order ("mfma_pack"): the 16 x 32 block (tile t, chunk c) is 1 KB
// contiguous at (t * K/32 + c) * 512 elements, lane l's 8 elements at l * 8 =
// W[16t + (l & 15)][32c + 8(l >> 4) .. +7] — every wave load is one coalesced
// 1 KB read instead of 16 row fragments of 64 B.
//   * causal conv k, stride s, channels-last input buffer with (k - s) history
//     rows in front:  A row t = buffer + t*s*C_in, K = k*C_in  (lda = s*C_in),
//   * 2-tap ConvTranspose (k = 2r, stride r): A row t = rows [t-1, t] of the
//     input buffer (1 history row), N = r*C_out and one output row = r
//     consecutive channels-last output rows.
// so every linear / conv layer on the hot path is this one kernel family.
//
// Fusions (the producer / consumer of each GEMM folded into it):
//   * A transform (XF_*): RMSNorm (+ weight, + adaLN modulate) of the A rows, or
//     SiLU(row + vec), applied to each A fragment as it is loaded.  The inverse
//     RMS of the block's rows is computed in a prologue (every workgroup redoes
//     it: at M <= 64 that is a few KB of L2 reads against MBs of weights).
//   * epilogues (EPI_*): bias, GELU, SiLU(gate)*up, gated / layer-scaled
//     residual, RoPE + KV-cache append, CFG + DPM-Solver++ update.
//
// Two shapes:
//   k_gemv : M <= 64 (LM decode rows, diffusion-head rows, codec stage at T=1).
//            HBM-bound weight stream.  MFMA 16x16x32 with W as the A operand
//            (16 weight rows = the MFMA M dim) and the <=16*MREP activation rows
//            as the B operand.  One workgroup per 16 weight rows; up to 16 waves
//            split K and each wave issues U chunks (U x 1 KB per wave) of weight
//            loads before its first MFMA, so a 16-wave workgroup keeps >100 KB in
//            flight (the "GEMV / M <= 16" row of cdna_hip_programming.md: no LDS
//            staging).  Waves reduce through LDS.  Cross-workgroup split-K (agent
//            release / ticket / acquire, Guideline 16) only for few-tile shapes.
//   k_gemm : M > 64 (codec stages at T >= 8, LM prefill).  64 x BN workgroup
//            tile, 4 waves of 32 x BN/2, operands straight from L2.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "kernels.h"
#include "gemv_dev.h"

// Diagnostic timestamps (tools/gemv_stamps.py): 100 MHz real-time clock, one
// lane per workgroup, to a buffer nothing else reads (a.stamps == nullptr in
// every product call).
DEV void stamp(const GemmArgs& a, int which) {
  if (a.stamps && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    a.stamps[((long long)blockIdx.y * gridDim.x + blockIdx.x) * 4 + which] = t;
  }
}

// ------------------------------------------------------------------ GEMV
// Index math of the prologues.  blockDim.x is a 16-bit implicit kernel
// argument; gfx950 has no 16-bit scalar load, so a read of it that the
// compiler cannot prove unclobbered (any global store earlier in the kernel,
// e.g. a timing stamp) becomes a VECTOR load + s_waitcnt vmcnt(0): a whole
// memory round trip before the first A / weight load was issued.  Kernels read
// it once, first (a scalar load), and the K ranges use 32-bit arithmetic (the
// 64-bit divisions were ~300 VALU instructions ahead of the first load).
DEV int part_of(int len, int i, int n) { return (int)((unsigned)(len * i) / (unsigned)n); }
// Split-K hand-off of the 16 x (16*MREP) fp32 tile between the workgroups of one
// tile column: every split stores its slab, takes a ticket, the last arriver
// sums the slabs in split order (deterministic) and runs the epilogue.
//   handoff 0: plain stores + agent release / acquire fences (Guideline 16 R1)
//   handoff 1: sc1 (write-through) 4-B stores, vmcnt(0) in every storing wave,
//              one agent atomic per workgroup, sc1 loads by the last arriver
//              (MI355X_MICROARCH.md "Valid forms", first table row)
// Returns true in the workgroup that must run the epilogue (red[] = sums).
DEV bool splitk_handoff(const GemmArgs& a, float* red, int TILE, unsigned* last_flag, int NT) {
  float* slab = a.ws + ((long long)blockIdx.x * a.ksplit + blockIdx.y) * TILE;
  const int t = threadIdx.x;
  if (a.handoff == 1) {
    for (int e = t; e < TILE; e += NT) __hip_atomic_store(slab + e, red[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    for (int e = t; e < TILE; e += NT) slab[e] = red[e];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    if (a.handoff != 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned tk = __hip_atomic_fetch_add(&a.counters[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last_flag = tk == (unsigned)(a.ksplit - 1) ? 1u : 0u;
    if (*last_flag) {
      if (a.handoff != 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(&a.counters[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!*last_flag) return false;
  const float* slabs = a.ws + (long long)blockIdx.x * a.ksplit * TILE;
  for (int e = t; e < TILE; e += NT) {
    float s = 0.f;
    if (a.handoff == 1) {
      for (int k = 0; k < a.ksplit; ++k) s += __hip_atomic_load(slabs + k * TILE + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (int k = 0; k < a.ksplit; ++k) s += slabs[k * TILE + e];
    }
    red[e] = s;
  }
  __syncthreads();
  return true;
}

// M <= 16: the workgroup's A rows (its K range, transformed) are staged once in
// LDS; each wave streams its weight chunks with a two-deep register ping-pong
// (U chunks = U KB per wave in flight while the previous U are multiplied).
// RW instantiations: the fused RMSNorm prologue with whole rows per wave.  Wave
// w loads rows w*RPW .. w*RPW+RPW-1 (lane l: 8-column items l, l+64, ...), so a
// row's sum of squares is one in-register accumulation + wave_sum and the norm
// is applied before the A rows ever reach LDS: one barrier instead of three and
// no LDS round trip of partial sums.  Each row's summation order is the one the
// item-per-thread form used (per-item partials when that form was "fast", one
// running sum otherwise = k_rmsnorm's), so both forms are bit-identical.
// (Rejected variants -- weights issued twice as deep before the prologue, a
// one-round-trip M = 16 prologue, epilogue operands prefetched at kernel start --
// are recorded with their measurements in DESIGN.md and no longer built.)
// TPW = 5: the balanced many-tile form (gemv_resolve): one workgroup per CU, 4 or
// 5 tiles each, 2 waves per tile (10 waves)
constexpr int gemv1_max_waves(int tpw) { return tpw == 5 ? 10 : 8; }
template <int U, int XF, bool KEEP = false, int TPW = 1, int RW = 0>
__global__ void __launch_bounds__(64 * gemv1_max_waves(TPW)) k_gemv1(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float inv_s[16];
  __shared__ float red[gemv1_max_waves(TPW) * 256];
  __shared__ unsigned last_flag;
  const int NT = blockDim.x, NW = NT >> 6;   // first: a scalar load (see part_of)
  // XF_MIX: the (<= 4) samples' conv-buffer slot bases, read before any store
  // so they are scalar loads issued together (as guarded per-slot vector loads
  // each took a round trip of its own)
  long long sbase[4] = {0, 0, 0, 0};
  if constexpr (XF == XF_MIX) {
    const int nsl = a.M / a.xf.T;
#pragma unroll
    for (int q = 0; q < 4; ++q) sbase[q] = (long long)a.xf.slots[min(q, nsl - 1)] * a.xf.buf_sB;
  }
  stamp(a, 0);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  // The workgroup owns TPW consecutive 16-row weight tiles and stages the A
  // rows once for all of them (at M = 16 one tile per workgroup re-read the
  // whole A block per 16 weight rows: as many L2 bytes as weight bytes, and the
  // LDS it needed capped residency at 2 workgroups per CU).  Waves are
  // tile-major: wave = tile_in_group * KW + k-slice.
  const int KW = TPW == 1 ? NW : NW / TPW;
  const int tw = TPW == 1 ? 0 : wave / KW, kwv = TPW == 1 ? wave : wave - tw * KW;
  const int ntile = a.N >> 4;
  // tiles [T0, T0 + ntl) of this workgroup: an even share of the grid's (<= TPW
  // each; = TPW * blockIdx.x .. when the grid is ntile / TPW workgroups)
  const int T0 = TPW == 1 ? blockIdx.x : part_of(ntile, blockIdx.x, gridDim.x);
  const int ntl = TPW == 1 ? 1 : part_of(ntile, blockIdx.x + 1, gridDim.x) - T0;
  const int tile = T0 + tw;
  const bool tile_ok = TPW == 1 || tw < ntl;
  const int nchunk = a.K >> 5;
  // this workgroup's chunk range, then each wave's
  const int b0 = a.ksplit == 1 ? 0 : part_of(nchunk, blockIdx.y, a.ksplit);
  const int b1 = a.ksplit == 1 ? nchunk : part_of(nchunk, blockIdx.y + 1, a.ksplit);
  const int c0 = b0 + part_of(b1 - b0, kwv, KW);
  const int c1 = tile_ok ? b0 + part_of(b1 - b0, kwv + 1, KW) : c0;
  // MFMA-packed W (a wave past the last tile streams nothing; its clamped
  // prologue loads read tile 0)
  const bf16* wrow = a.w + (long long)(tile_ok ? tile : 0) * a.K * 16 + lane * 8;
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};

  // ---- A staging into LDS (rows [0, M) x chunks [b0, b1), row stride padded
  // 16 B), overlapped with the first weight chunks.  vmcnt waits are in issue
  // order, so every A-side load (row chunk + its transform operands) is issued
  // BEFORE the weight loads: the prologue then waits only for its own bytes and
  // the weight stream stays in flight through the norm math.
  const int kw = (b1 - b0) * 32;         // elements staged per row
  const int lds_ld = kw + 8;
  const int n8 = kw >> 3;
  bf16* xs = (bf16*)smem;
  float* part = (float*)(smem + (((size_t)a.M * lds_ld * 2 + 15) & ~(size_t)15));
  bf16x8 wa[U], wb[U];
  constexpr int Q = 4;   // A items per thread on the fast path
  const bool fast = a.M * n8 <= Q * NT;
  // row-per-wave norm prologue: items per lane per row (IPR) x rows per wave (RPW)
  // (RW instantiations only; the host picks them for eligible shapes, gemv1_rw)
  const int ipr = n8 >> 6, rpw = (a.M + NW - 1) / NW;
  const int rw = ipr == 3 && rpw == 1 ? 31 : ipr == 3 ? 32 : 71;
  // whole rows per wave: loads (A, norm weight, adaLN shift / scale; all
  // unconditional, clamped to valid rows, so no branch join waits on them),
  // then the weight stream, then sums, wave_sum and the norm in registers
  auto stage_rw = [&](auto ipr_c, auto rpw_c, auto mod_c) {
    constexpr int IPR = decltype(ipr_c)::value, RPW = decltype(rpw_c)::value, QR = IPR * RPW;
    constexpr bool MOD = decltype(mod_c)::value;   // adaLN operands possible (their registers reserved)
    bf16x8 xv[QR], wv[QR], sh[MOD ? QR : 1], sc[MOD ? QR : 1];
    const bool has_w = a.xf.w != nullptr, has_mod = MOD && a.xf.mod != nullptr;
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int m = min(wave * RPW + r, a.M - 1);
      const bf16* xr = rm_bf(a.a, m);
      const bf16* wp = has_w ? a.xf.w : xr;
      const bf16* md = has_mod ? a.xf.mod + (long long)m * a.xf.mod_ld : xr;
      const int so = has_mod ? a.xf.shift_off : 0, co = has_mod ? a.xf.scale_off : 0;
#pragma unroll
      for (int i = 0; i < IPR; ++i) {
        const int k = (lane + 64 * i) * 8;
        xv[r * IPR + i] = *(const bf16x8*)(xr + k);
        wv[r * IPR + i] = *(const bf16x8*)(wp + k);
        if (has_mod) {
          sh[MOD ? r * IPR + i : 0] = *(const bf16x8*)(md + so + k);
          sc[MOD ? r * IPR + i : 0] = *(const bf16x8*)(md + co + k);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) wa[u] = ldw<KEEP>(wrow + min(c0 + u, max(c1 - 1, 0)) * 512);
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < IPR; ++i) {
        if (fast) {   // the item-per-thread fast form: per-item partials, then items in order
          float p = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) p += bf(xv[r * IPR + i][j]) * bf(xv[r * IPR + i][j]);
          ss += p;
        } else {      // the staged form / k_rmsnorm: one running sum
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += bf(xv[r * IPR + i][j]) * bf(xv[r * IPR + i][j]);
        }
      }
      ss = wave_sum(ss);
      const float inv = rsqrtf(ss / (float)a.K + a.xf.eps);
      const int m = wave * RPW + r;
      // (the uniform has_w / has_mod tests stay per element: hoisting them into
      // specialised copies raised the kernel to 180 VGPRs, 3 -> 2 waves / SIMD)
      if (m < a.M) {
#pragma unroll
        for (int i = 0; i < IPR; ++i) {
          const int q = r * IPR + i;
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = rb(bf(xv[q][j]) * inv);
            if (has_w) t = rb(t * bf(wv[q][j]));
            if (has_mod) t = rb(rb(t * rb(1.0f + bf(sc[MOD ? q : 0][j]))) + bf(sh[MOD ? q : 0][j]));
            o[j] = tobf(t);
          }
          *(bf16x8*)(xs + m * lds_ld + (lane + 64 * i) * 8) = o;
        }
      }
    }
  };
  // K = 3,584 rows with adaLN operands (VibeVoice-Large head): the raw A row
  // goes straight to its LDS row by 16-byte LDS DMA (lane l's item i lands at
  // (l + 64 i) * 8, the row layout), so only the norm weight and shift / scale
  // take registers; the row is read back by its own lanes after a counted vmcnt
  // (the 21 operand loads and the U weight loads issued after it stay in flight)
  auto stage_rw_dma = [&]() {
    constexpr int IPR = 7;
    bf16x8 wv[IPR], sh[IPR], sc[IPR];
    const bool has_w = a.xf.w != nullptr;
    const int m = min(wave, a.M - 1);
    bf16* xrow_l = xs + m * lds_ld;
    if (wave < a.M) {
      const bf16* xr = rm_bf(a.a, m);
      const bf16* wp = has_w ? a.xf.w : xr;
      const bf16* md = a.xf.mod + (long long)m * a.xf.mod_ld;
#pragma unroll
      for (int i = 0; i < IPR; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(xr + (lane + 64 * i) * 8),
                                         (__attribute__((address_space(3))) void*)(xrow_l + 64 * i * 8), 16, 0, 0);
      // the counted wait below needs exactly these loads younger than the DMA,
      // in this order: sched_barrier fences keep the scheduler from moving any
      // of them across
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < IPR; ++i) {
        const int k = (lane + 64 * i) * 8;
        wv[i] = *(const bf16x8*)(wp + k);
        sh[i] = *(const bf16x8*)(md + a.xf.shift_off + k);
        sc[i] = *(const bf16x8*)(md + a.xf.scale_off + k);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; ++u) wa[u] = ldw<KEEP>(wrow + min(c0 + u, max(c1 - 1, 0)) * 512);
    __builtin_amdgcn_sched_barrier(0);
    if (wave < a.M) {
      // the DMA is older than 3 * IPR operand loads and the weight loads
      constexpr int after = 3 * IPR + U;
      __builtin_amdgcn_s_waitcnt((after & 15) | ((after >> 4) << 14) | (7 << 4) | (15 << 8));
      bf16x8 xv[IPR];
#pragma unroll
      for (int i = 0; i < IPR; ++i) xv[i] = *(const bf16x8*)(xrow_l + (lane + 64 * i) * 8);
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < IPR; ++i) {
        if (fast) {
          float p = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) p += bf(xv[i][j]) * bf(xv[i][j]);
          ss += p;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += bf(xv[i][j]) * bf(xv[i][j]);
        }
      }
      ss = wave_sum(ss);
      const float inv = rsqrtf(ss / (float)a.K + a.xf.eps);
#pragma unroll
      for (int i = 0; i < IPR; ++i) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = rb(bf(xv[i][j]) * inv);
          if (has_w) t = rb(t * bf(wv[i][j]));
          t = rb(rb(t * rb(1.0f + bf(sc[i][j]))) + bf(sh[i][j]));
          o[j] = tobf(t);
        }
        *(bf16x8*)(xrow_l + (lane + 64 * i) * 8) = o;
      }
    }
  };
  if constexpr (RW == 2) {   // its own instantiation: its registers would cost the others occupancy
    stage_rw_dma();
  } else if constexpr (RW == 1) {
    using I = std::true_type;
    if (rw == 31) stage_rw(std::integral_constant<int, 3>(), std::integral_constant<int, 1>(), I());
    else if (rw == 32) stage_rw(std::integral_constant<int, 3>(), std::integral_constant<int, 2>(), I());
    else stage_rw(std::integral_constant<int, 7>(), std::integral_constant<int, 1>(), std::false_type());
  } else if (XF == XF_ATTN_MERGE) {
    // o_proj's A rows = the decode attention output, merged from the key splits'
    // partials k_attn left (AttnArgs::defer): out = sum_s e^{m_s - M} o_s /
    // sum_s e^{m_s - M} l_s in split order -- the attention kernel's own merge
    // term for term (bit-identical), one round trip of partial loads here instead
    // of a ticket + merge at the attention's tail.  Item (m, 8 dims of head hq).
    const int nsp = a.xf.nsplit;
    // the weight stream first: the merge's two dependent round trips (query
    // length, then the partials) then overlap it instead of preceding it
#pragma unroll
    for (int u = 0; u < U; ++u) wa[u] = ldw<KEEP>(wrow + min(c0 + u, max(c1 - 1, 0)) * 512);
#pragma unroll 1
    for (int e = threadIdx.x; e < a.M * n8; e += NT) {
      const int m = e / n8, k = (e - m * n8) * 8;
      const int hq = k >> 7, j0 = k & 127;
      const int len = a.xf.qpos[m] + 1;
      const int cc = (len + nsp - 1) / nsp;
      const int rch = max(a.xf.chunk, (cc + 31) / 32 * 32);
      const int nact = (len + rch - 1) / rch;
      const long long p0 = ((long long)m * (a.K >> 7) + hq) * nsp;
      float mv[8], lv[8];
      float4 o0[8], o1[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s < nact) {
          const float2 ml = *(const float2*)(a.xf.part_ml + (p0 + s) * 2);
          mv[s] = ml.x;
          lv[s] = ml.y;
          o0[s] = *(const float4*)(a.xf.part_o + (p0 + s) * 128 + j0);
          o1[s] = *(const float4*)(a.xf.part_o + (p0 + s) * 128 + j0 + 4);
        }
      }
      float M = -INFINITY;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        if (s < nact) M = fmaxf(M, mv[s]);
      float num[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, den = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        if (s < nact) {
          const float w = __expf(mv[s] - M);
          num[0] += w * o0[s].x;
          num[1] += w * o0[s].y;
          num[2] += w * o0[s].z;
          num[3] += w * o0[s].w;
          num[4] += w * o1[s].x;
          num[5] += w * o1[s].y;
          num[6] += w * o1[s].z;
          num[7] += w * o1[s].w;
          den += w * lv[s];
        }
      }
      bf16x8 o8;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) o8[jj] = tobf(num[jj] / den);
      *(bf16x8*)(xs + m * lds_ld + k) = o8;
    }
  } else if (XF == XF_MIX) {
    // Codec Block1D front half for the M = ns * T rows (k_mix's math and
    // summation order, elementwise.hip): every workgroup recomputes it (a few
    // tens of KB of L2 reads next to its weight slice); workgroup 0 also stores
    // the conv-buffer rows and y.  One dependent global round trip: operands,
    // x rows and history rows are issued together ahead of the weight stream
    // (the slot ids come through the scalar cache), the raw x rows stay in LDS
    // (xs) and are overwritten by y, then by fc1's normalised input.
    const int C = a.K, T = a.xf.T, ctx = a.xf.ctx, ns = a.M / T;
    bf16* nrm = (bf16*)part;                                 // [ns][ctx + T][C] conv input rows
    float* ssp = (float*)(nrm + (size_t)ns * (ctx + T) * C); // [M][n8] partial sums of squares
    const bool writer = blockIdx.x == 0;
    const int c2 = threadIdx.x % n8;                         // fixed: NT % n8 == 0
    bf16x8 wk[7], bb, gv, wf, wn;
#pragma unroll
    for (int k = 0; k < 7; ++k) wk[k] = *(const bf16x8*)(a.xf.dw_w + (size_t)c2 * 56 + k * 8);
    bb = *(const bf16x8*)(a.xf.dw_b + c2 * 8);
    gv = *(const bf16x8*)(a.xf.gamma + c2 * 8);
    wf = *(const bf16x8*)(a.xf.ffn_w + c2 * 8);
    wn = *(const bf16x8*)(a.xf.w + c2 * 8);
    // items [0, M*n8): x row m; [M*n8, (M + ns*ctx)*n8): history row h of sample s.
    // Every load is unconditional from an address chosen by selects (items past
    // the end re-read the last one): guarded loads, and rm_off's optional slot
    // lookup, compiled to a branch + s_waitcnt vmcnt(0) per item -- eight
    // serialized round trips per pass.  (x rows: host-checked plain map, no idx.)
    // Rows, not items: the n8 consecutive threads of a row share it, so thread t
    // takes rows t / n8 + j * (NT / n8) -- no per-item division (the item form
    // spent ~100 VALU per item on index math ahead of the weight stream).
    constexpr int CTX = 6;                                    // host-checked (k = 7)
    const int nrow = a.M + ns * CTX, rpt = NT / n8, rt = threadIdx.x / n8, nx = a.M * n8;
    const bf16* xbase = (const bf16*)a.a.base;
    for (int r0 = 0, first = 1; r0 < nrow; r0 += 8 * rpt, first = 0) {
      bf16x8 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int R = min(r0 + rt + q * rpt, nrow - 1);
        const int mx = min(R, a.M - 1), gx = mx / a.a.T;
        const bf16* px = xbase + gx * a.a.sB + (long long)(mx - gx * a.a.T) * a.a.sT;
        const int hr = max(R - a.M, 0), s_ = hr / CTX;
        long long sb = sbase[0];
#pragma unroll
        for (int q2 = 1; q2 < 4; ++q2) sb = s_ == q2 ? sbase[q2] : sb;
        const bf16* ph = a.xf.buf + sb + (long long)(hr - s_ * CTX) * C;
        v[q] = *(const bf16x8*)((R < a.M ? px : ph) + c2 * 8);
      }
      if (first) {
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = ldw<KEEP>(wrow + min(c0 + u, max(c1 - 1, 0)) * 512);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int R = r0 + rt + q * rpt;
        if (R < a.M) {
          *(bf16x8*)(xs + R * lds_ld + c2 * 8) = v[q];
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += bf(v[q][j]) * bf(v[q][j]);
          ssp[R * n8 + c2] = ss;
        } else if (R < nrow) {
          const int hr = R - a.M, s_ = hr / CTX;
          *(bf16x8*)(nrm + ((size_t)s_ * (CTX + T) + (hr - s_ * CTX)) * C + c2 * 8) = v[q];
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int m = wave; m < a.M; m += NW) {                   // k_mix's row-sum order (64 lanes)
      float ss = 0.f;
      for (int c = lane; c < n8; c += 64) ss += ssp[m * n8 + c];
      ss = wave_sum(ss);
      if (lane == 0) inv_s[m] = rsqrtf(ss / (float)C + a.xf.eps);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // mixer norm of the new rows -> conv input rows; workgroup 0 appends them to the buffer
    for (int e = threadIdx.x; e < nx; e += NT) {
      const int m = e / n8, s_ = m / T, t = m - s_ * T;
      const bf16x8 v = *(const bf16x8*)(xs + m * lds_ld + c2 * 8);
      const float rr = inv_s[m];
      bf16x8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8[j] = tobf(rb(rb(bf(v[j]) * rr) * bf(wn[j])));
      *(bf16x8*)(nrm + ((size_t)s_ * (ctx + T) + ctx + t) * C + c2 * 8) = o8;
      if (writer) {
        long long sb = sbase[0];
#pragma unroll
        for (int q2 = 1; q2 < 4; ++q2) sb = s_ == q2 ? sbase[q2] : sb;
        *(bf16x8*)(a.xf.buf + sb + (long long)(ctx + t) * C + c2 * 8) = o8;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // depthwise conv + gamma residual: y over the raw x in xs (workgroup 0 stores y)
    for (int e = threadIdx.x; e < nx; e += NT) {
      const int m = e / n8, s_ = m / T, t = m - s_ * T;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const bf16x8 v = *(const bf16x8*)(nrm + ((size_t)s_ * (ctx + T) + t + k) * C + c2 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int f = j * 7 + k;
          acc[j] += bf(wk[f >> 3][f & 7]) * bf(v[j]);
        }
      }
      bf16x8* px = (bf16x8*)(xs + m * lds_ld + c2 * 8);
      const bf16x8 xv = *px;
      bf16x8 y8;
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        y8[j] = tobf(bf(xv[j]) + rb(rb(acc[j] + bf(bb[j])) * bf(gv[j])));
        ss += bf(y8[j]) * bf(y8[j]);
      }
      if (writer) *(bf16x8*)(a.xf.y + (long long)m * C + c2 * 8) = y8;
      *px = y8;
      ssp[e] = ss;
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int m = wave; m < a.M; m += NW) {
      float ss = 0.f;
      for (int c = lane; c < n8; c += 64) ss += ssp[m * n8 + c];
      ss = wave_sum(ss);
      if (lane == 0) inv_s[m] = rsqrtf(ss / (float)C + a.xf.eps);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    for (int e = threadIdx.x; e < nx; e += NT) {             // FFN pre-norm, in place
      const int m = e / n8;
      bf16x8* px = (bf16x8*)(xs + m * lds_ld + c2 * 8);
      const bf16x8 y8 = *px;
      const float rr = inv_s[m];
      bf16x8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8[j] = tobf(rb(rb(bf(y8[j]) * rr) * bf(wf[j])));
      *px = o8;
    }
  } else if (fast) {
    bf16x8 xv[Q], wv[Q], sh[Q], sc[Q];
    // every A-side load unconditional (items past the end re-read the last;
    // absent operands re-read the row) and, for a plain row map, no slot
    // lookup: a guarded load compiled to a branch + s_waitcnt vmcnt(0) at its
    // join, so each item waited for the one before it and the weight stream
    // behind them was issued several round trips late
    const int ne = a.M * n8;
    const bool has_w = XF == XF_NORM ? a.xf.w != nullptr : XF == XF_SILU_ADD;
    const bool has_mod = XF == XF_NORM && a.xf.mod != nullptr;
    auto fast_loads = [&](auto plain_c) {
      constexpr bool PLAIN = decltype(plain_c)::value;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int e = min(threadIdx.x + q * NT, ne - 1);
        const int m = e / n8, k = b0 * 32 + (e - m * n8) * 8;
        const bf16* xr = PLAIN ? rm_bf_plain(a.a, m) : rm_bf(a.a, m);
        xv[q] = *(const bf16x8*)(xr + k);
        if (XF == XF_NORM || XF == XF_SILU_ADD) {
          const bf16* wp = has_w ? (XF == XF_NORM ? a.xf.w : a.xf.vec) : xr;
          wv[q] = *(const bf16x8*)(wp + k);
        }
        if (XF == XF_NORM) {
          const bf16* md = has_mod ? a.xf.mod + (long long)m * a.xf.mod_ld : xr;
          sh[q] = *(const bf16x8*)(md + (has_mod ? a.xf.shift_off : 0) + k);
          sc[q] = *(const bf16x8*)(md + (has_mod ? a.xf.scale_off : 0) + k);
        }
      }
    };
    if (a.a.idx) fast_loads(std::false_type());
    else fast_loads(std::true_type());
#pragma unroll
    for (int u = 0; u < U; ++u) wa[u] = ldw<KEEP>(wrow + min(c0 + u, max(c1 - 1, 0)) * 512);
    if (XF == XF_NORM) {
      // per-item sums of squares -> LDS, rows reduced in a fixed order
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int e = threadIdx.x + q * NT;
        if (e < a.M * n8) {
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += bf(xv[q][j]) * bf(xv[q][j]);
          part[e] = ss;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (a.ksplit == 1) {
        for (int m = wave; m < a.M; m += NW) {
          float ss = 0.f;
          for (int c = lane; c < n8; c += 64) ss += part[m * n8 + c];
          ss = wave_sum(ss);
          if (lane == 0) inv_s[m] = rsqrtf(ss / (float)a.K + a.xf.eps);
        }
      } else {
        row_inv(a, 0, a.M, inv_s, wave, NW, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = threadIdx.x + q * NT;
      if (e < a.M * n8) {
        const int m = e / n8, k8 = (e - m * n8) * 8;
        bf16x8 o = xv[q];
        if (XF == XF_NORM) {
          const float inv = inv_s[m];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float t = rb(bf(xv[q][j]) * inv);
            if (a.xf.w) t = rb(t * bf(wv[q][j]));
            if (a.xf.mod) t = rb(rb(t * rb(1.0f + bf(sc[q][j]))) + bf(sh[q][j]));
            o[j] = tobf(t);
          }
        } else if (XF == XF_SILU_ADD) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = tobf(silu_f(rb(bf(xv[q][j]) + bf(wv[q][j]))));
        }
        *(bf16x8*)(xs + m * lds_ld + k8) = o;
      }
    }
  } else {
    // many rows (B >= 8 batches): weights first, then the A rows in batches
#pragma unroll
    for (int u = 0; u < U; ++u) wa[u] = ldw<KEEP>(wrow + min(c0 + u, max(c1 - 1, 0)) * 512);
    const int ne = a.M * n8;
    const bool plain = !a.a.idx;
    for (int e0 = threadIdx.x; e0 < ne; e0 += 4 * NT) {
      bf16x8 xv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {   // unconditional loads (see the fast path)
        const int e = min(e0 + q * NT, ne - 1);
        const int m = e / n8, k8 = (e - m * n8) * 8;
        xv[q] = *(const bf16x8*)((plain ? rm_bf_plain(a.a, m) : rm_bf(a.a, m)) + b0 * 32 + k8);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = e0 + q * NT;
        if (e < a.M * n8) {
          const int m = e / n8, k8 = (e - m * n8) * 8;
          *(bf16x8*)(xs + m * lds_ld + k8) = xv[q];
        }
      }
    }
    if (XF != XF_NONE) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (XF == XF_NORM) {
        if (a.ksplit == 1) {
          for (int m = wave; m < a.M; m += NW) {
            float ss = 0.f;
            for (int c = lane; c < n8; c += 64) {
              const bf16x8 v = *(const bf16x8*)(xs + m * lds_ld + c * 8);
#pragma unroll
              for (int j = 0; j < 8; ++j) ss += bf(v[j]) * bf(v[j]);
            }
            ss = wave_sum(ss);
            if (lane == 0) inv_s[m] = rsqrtf(ss / (float)a.K + a.xf.eps);
          }
        } else {
          row_inv(a, 0, a.M, inv_s, wave, NW, lane);
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
      for (int e = threadIdx.x; e < a.M * n8; e += NT) {
        const int m = e / n8, k8 = (e - m * n8) * 8;
        bf16x8* px = (bf16x8*)(xs + m * lds_ld + k8);
        *px = xform<XF>(a, *px, m, b0 * 32 + k8, XF == XF_NORM ? inv_s[m] : 0.f);
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  stamp(a, 1);

  f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
  // A fragment reads are unconditional (a guarded LDS read compiled to an
  // exec-masked ds_read + lgkmcnt(0) per chunk): lanes of rows >= M read row
  // M - 1 -- they only feed output columns the epilogue drops -- and chunks past
  // the wave's range re-read its last chunk against a zeroed weight fragment
  const bf16* xrow = xs + min(r, a.M - 1) * lds_ld + 8 * g - b0 * 32;
  auto compute = [&](bf16x8 (&wf)[U], int c) {
    bf16x8 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = *(const bf16x8*)(xrow + min(c + u, c1 - 1) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bf16x8 w = c + u < c1 ? wf[u] : zero8;
      acc = mfma(w, x[u], acc);
    }
  };
  auto load = [&](bf16x8 (&wf)[U], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) wf[u] = ldw<KEEP>(wrow + min(c + u, max(c1 - 1, 0)) * 512);
  };
  for (int c = c0; c < c1; c += 2 * U) {
    load(wb, c + U);
    compute(wa, c);
    load(wa, c + 2 * U);
    compute(wb, c + U);
  }
  stamp(a, 2);

  // ---- reduce each tile's K-slice waves (tile t's sum lands in slab t * KW)
#pragma unroll
  for (int i = 0; i < 4; ++i) red[(wave * 4 + i) * 64 + lane] = acc[i];
  __syncthreads();
  if (KW > 1) {
    for (int e = threadIdx.x; e < TPW * 256; e += NT) {
      const int base = (e >> 8) * KW * 256 + (e & 255);
      float s = 0.f;
      for (int w = 1; w < KW; ++w) s += red[base + w * 256];
      red[base] += s;
    }
    __syncthreads();
  }
  if (a.ksplit > 1 && !splitk_handoff(a, red, 256, &last_flag, NT)) return;   // host: ksplit > 1 => TPW == 1
  if (wave < TPW && (TPW == 1 || wave < ntl)) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = red[wave * KW * 256 + i * 64 + lane];
    epi_tile(a, r, (T0 + wave) * 16, lane, v);
    if (a.stamps) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(a, 3);
    }
  }
}

// 16 < M <= 64: A fragments loaded straight from global / L2, transform per
// chunk; weights ping-ponged as in k_gemv1.
template <int MREP, int U, int XF>
__global__ void __launch_bounds__(512) k_gemv(GemmArgs a) {
  __shared__ float red[8 * MREP * 256];
  __shared__ float inv_s[64];
  __shared__ unsigned last_flag;
  const int NT = blockDim.x, NW = NT >> 6;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int nchunk = a.K >> 5;
  const int b0 = a.ksplit == 1 ? 0 : part_of(nchunk, blockIdx.y, a.ksplit);
  const int b1 = a.ksplit == 1 ? nchunk : part_of(nchunk, blockIdx.y + 1, a.ksplit);
  const int c0 = b0 + part_of(b1 - b0, wave, NW);
  const int c1 = b0 + part_of(b1 - b0, wave + 1, NW);
  const bf16* wrow = a.w + (long long)(n0 >> 4) * a.K * 16 + lane * 8;  // MFMA-packed W
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  if (XF == XF_NORM) {
    row_inv(a, 0, 16 * MREP, inv_s, wave, NW, lane);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  const bf16* xrow[MREP];
  bool xok[MREP];
  float inv[MREP];
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr) {
    const int m = r + 16 * mr;
    xok[mr] = m < a.M;
    xrow[mr] = rm_bf(a.a, min(m, a.M - 1)) + 8 * g;   // rows >= M: a valid row, results dropped
    inv[mr] = XF == XF_NORM ? inv_s[m] : 0.f;
  }
  f32x4 acc[MREP];
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr) acc[mr] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // each chunk's A fragments travel with its weight chunk (vmcnt waits are in
  // issue order: loading A inside compute would wait for the next batch too)
  bf16x8 wa[U], wb[U], xa[U][MREP], xb[U][MREP];
  auto load = [&](bf16x8 (&wf)[U], bf16x8 (&xf)[U][MREP], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cc = min(c + u, max(c1 - 1, 0));
#pragma unroll
      for (int mr = 0; mr < MREP; ++mr) xf[u][mr] = *(const bf16x8*)(xrow[mr] + cc * 32);
      wf[u] = ldw(wrow + cc * 512);
    }
  };
  auto compute = [&](bf16x8 (&wf)[U], bf16x8 (&xf)[U][MREP], int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = c + u < c1;
      const int cc = min(c + u, max(c1 - 1, 0));
      const bf16x8 w = ok ? wf[u] : zero8;
#pragma unroll
      for (int mr = 0; mr < MREP; ++mr) {
        bf16x8 x = (xok[mr] && ok) ? xf[u][mr] : zero8;
        if (XF != XF_NONE && xok[mr] && ok) x = xform<XF>(a, x, r + 16 * mr, cc * 32 + 8 * g, inv[mr]);
        acc[mr] = mfma(w, x, acc[mr]);
      }
    }
  };
  load(wa, xa, c0);
  for (int c = c0; c < c1; c += 2 * U) {
    load(wb, xb, c + U);
    compute(wa, xa, c);
    load(wa, xa, c + 2 * U);
    compute(wb, xb, c + U);
  }
  const int TILE = MREP * 256;
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * MREP * 4 + mr * 4 + i) * 64 + lane] = acc[mr][i];
  __syncthreads();
  if (NW > 1) {
    for (int e = threadIdx.x; e < TILE; e += NT) {
      float s = 0.f;
      for (int w = 1; w < NW; ++w) s += red[w * TILE + e];
      red[e] += s;
    }
    __syncthreads();
  }
  if (a.ksplit > 1 && !splitk_handoff(a, red, TILE, &last_flag, NT)) return;
  for (int mr = wave; mr < MREP; mr += NW) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = red[(mr * 4 + i) * 64 + lane];
    epi_tile(a, r + 16 * mr, n0, lane, v);
  }
}

// 16 < M <= 64 with many weight tiles (B >= 9 decode rows, the batched head
// adaLN, 64-row codec stages).  k_gemv re-reads the A fragments from L2 for
// every 16 weight rows -- at M = 64 four times the weight bytes (B = 32: LM
// gate|up 51 us for 55 MB).  Here each of the 8 waves holds the A fragments of
// its K slice (GW_NCH chunks per K block) in registers and applies them to the
// workgroup's TPW weight tiles, streaming those tiles' chunks of the slice with
// a ping-pong over tiles; the 8 slices reduce in LDS per tile, in wave order,
// before the epilogue.  A crosses L2 once per workgroup.
constexpr int GW_NCH = 6;   // 32-column chunks per wave per K block (8 waves: 1,536 columns)

template <int MREP, int TPW, bool KEEP>
__global__ void __launch_bounds__(512) k_gemvw(GemmArgs a) {
  __shared__ float red[8][MREP * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int ntile = a.N >> 4, nchunk = a.K >> 5;
  const int t0 = blockIdx.x * TPW;
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  f32x4 acc[TPW][MREP];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int mr = 0; mr < MREP; ++mr) acc[i][mr] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // rows >= M read row M - 1 (their output columns are dropped): no guarded loads
  const bf16* arow[MREP];
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr) arow[mr] = rm_bf(a.a, min(16 * mr + r, a.M - 1)) + 8 * g;
  for (int kb = 0; kb < nchunk; kb += 8 * GW_NCH) {
    const int cw = kb + wave * GW_NCH;        // this wave's first chunk of the block (wave-uniform)
    if (cw >= nchunk) continue;
    bf16x8 xf[GW_NCH][MREP];
#pragma unroll
    for (int c = 0; c < GW_NCH; ++c)
#pragma unroll
      for (int mr = 0; mr < MREP; ++mr) xf[c][mr] = *(const bf16x8*)(arow[mr] + min(cw + c, nchunk - 1) * 32);
    bf16x8 wa[GW_NCH], wb[GW_NCH];
    auto wload = [&](bf16x8 (&w)[GW_NCH], int i) {
      const int t = min(t0 + i, ntile - 1);
      const bf16* wr = a.w + (long long)t * a.K * 16 + lane * 8;
#pragma unroll
      for (int c = 0; c < GW_NCH; ++c) w[c] = ldw<KEEP>(wr + min(cw + c, nchunk - 1) * 512);
    };
    auto mac = [&](bf16x8 (&w)[GW_NCH], int i) {
#pragma unroll
      for (int c = 0; c < GW_NCH; ++c) {
        const bf16x8 wc = cw + c < nchunk ? w[c] : zero8;   // chunks past K: zero weights
#pragma unroll
        for (int mr = 0; mr < MREP; ++mr) acc[i][mr] = mfma(wc, xf[c][mr], acc[i][mr]);
      }
    };
    wload(wa, 0);
#pragma unroll
    for (int i = 0; i < TPW; i += 2) {
      if (i + 1 < TPW) wload(wb, i + 1);
      mac(wa, i);
      if (i + 2 < TPW) wload(wa, i + 2);
      if (i + 1 < TPW) mac(wb, i + 1);
    }
  }
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
#pragma unroll
    for (int mr = 0; mr < MREP; ++mr)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave][mr * 256 + j * 64 + lane] = acc[i][mr][j];
    __syncthreads();
    for (int e = threadIdx.x; e < MREP * 256; e += 512) {
      float sum = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sum += red[w][e];
      red[0][e] = sum;
    }
    __syncthreads();
    const int t = t0 + i;
    if (t < ntile) {
      for (int mr = wave; mr < MREP; mr += 8) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = red[0][mr * 256 + j * 64 + lane];
        epi_tile(a, 16 * mr + r, t * 16, lane, v);
      }
    }
    __syncthreads();
  }
}

template <int MREP, int TPW>
static void launch_gemvw_t(const GemmArgs& a, hipStream_t st) {
  const dim3 grid((a.N / 16 + TPW - 1) / TPW);
  if (a.keep) hipLaunchKernelGGL((k_gemvw<MREP, TPW, true>), grid, dim3(512), 0, st, a);
  else hipLaunchKernelGGL((k_gemvw<MREP, TPW, false>), grid, dim3(512), 0, st, a);
}

static std::atomic<int> g_gemvw{1};   // diagnostic: 0 = k_gemv for every 16 < M <= 64 (vv_gemv_tune_wide)
extern "C" int vv_gemv_tune_wide(int on) {
  g_gemvw = on;
  return 0;
}

// 16 < M <= 64, >= 256 tiles, plain A (no transform), one K split
static bool launch_gemvw(const GemmArgs& a, hipStream_t st) {
  const int tiles = a.N / 16;
  if (!g_gemvw || a.M <= 16 || a.M > 64 || tiles < 256 || a.xf.kind != XF_NONE || a.epi.kind == EPI_CFG_DPM)
    return false;
  const int mrep = (a.M + 15) / 16;
  const int tpw = tiles >= 1024 ? 4 : tiles >= 512 ? 2 : 1;   // ~256-340 workgroups
  if (mrep == 2) {
    if (tpw == 4) launch_gemvw_t<2, 4>(a, st);
    else if (tpw == 2) launch_gemvw_t<2, 2>(a, st);
    else launch_gemvw_t<2, 1>(a, st);
  } else if (mrep == 3) {
    if (tpw == 4) launch_gemvw_t<3, 4>(a, st);
    else if (tpw == 2) launch_gemvw_t<3, 2>(a, st);
    else launch_gemvw_t<3, 1>(a, st);
  } else {
    if (tpw == 4) launch_gemvw_t<4, 4>(a, st);
    else if (tpw == 2) launch_gemvw_t<4, 2>(a, st);
    else launch_gemvw_t<4, 1>(a, st);
  }
  return true;
}

// ------------------------------------------------------------------ tiled GEMM (M > 64)
template <int BN, int XF>
__global__ void __launch_bounds__(256) k_gemm(GemmArgs a) {
  constexpr int NT = BN / 32;  // 16-wide n tiles per wave (wave covers BN/2 columns)
  __shared__ float inv_s[64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const int m_blk = blockIdx.x * 64;
  const int m_base = m_blk + wm * 32;
  const int n_base = blockIdx.y * BN + wn * (BN / 2);
  if (XF == XF_NORM) {
    row_inv(a, m_blk, 64, inv_s, wave, 4, lane);
    __syncthreads();
  }
  const bf16* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wrow[nt] = a.w + (long long)((n_base >> 4) + nt) * a.K * 16 + lane * 8;
  // rows past M read row M - 1 (unconditional loads: a guarded load compiles to a
  // branch + a vmcnt(0) wait); their products land in rows the epilogue drops
  const bf16* xrow[2];
  bool xok[2];
  float inv[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = m_base + mt * 16 + r;
    xok[mt] = m < a.M;
    xrow[mt] = rm_bf(a.a, min(m, a.M - 1)) + 8 * g;
    inv[mt] = XF == XF_NORM ? inv_s[min(m, a.M - 1) - m_blk] : 0.f;
  }
  f32x4 acc[2][NT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  const int nk = a.K >> 5;
  // two register sets of 2 chunks each: the loads of chunks c + 4 .. go out while
  // chunks c .. compute (one set in flight per round trip left the loop
  // latency-bound: the 320-row codec fc2 at C = 512, K 2,048, took 24 us)
  bf16x8 wfA[2][NT], xfA[2][2], wfB[2][NT], xfB[2][2];
  auto load = [&](int c, bf16x8 (&wf)[2][NT], bf16x8 (&xf)[2][2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int cc = min(c + u, nk - 1);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wf[u][nt] = *(const bf16x8*)(wrow[nt] + cc * 512);   // re-read across row tiles: default policy
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) xf[u][mt] = *(const bf16x8*)(xrow[mt] + cc * 32);
    }
  };
  auto comp = [&](int c, bf16x8 (&wf)[2][NT], bf16x8 (&xf)[2][2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (c + u >= nk) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) wf[u][nt] = zero8;
      }
      if (XF != XF_NONE) {
        const int k = min(c + u, nk - 1) * 32 + 8 * g;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
          if (xok[mt]) xf[u][mt] = xform<XF>(a, xf[u][mt], m_base + mt * 16 + r, k, inv[mt]);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma(wf[u][nt], xf[u][mt], acc[mt][nt]);
    }
  };
  load(0, wfA, xfA);
  if (2 < nk) load(2, wfB, xfB);
  for (int c = 0; c < nk; c += 4) {
    comp(c, wfA, xfA);
    if (c + 4 < nk) load(c + 4, wfA, xfA);
    if (c + 2 < nk) {
      comp(c + 2, wfB, xfB);
      if (c + 6 < nk) load(c + 6, wfB, xfB);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
      epi_tile(a, m_base + mt * 16 + r, n_base + nt * 16, lane, v);
    }
}

// ------------------------------------------------------------------ LDS-staged GEMM (prefill-sized M)
// M >= GEMM_BIG_M rows (a prompt's prefill: thousands of tokens through every
// projection).  k_gemm's operands come straight from L2
// per wave (4 fragments per 4 MFMAs); here a 128 x 128 tile of 4 waves (each
// 64 x 64: 4 weight tiles x 4 row tiles, 16 accumulators) stages each 64-deep
// K step in LDS with 16-byte global_load_lds: the packed weight blocks are
// already 1 KB MFMA fragments (one wave instruction each), and the A rows are
// gathered per lane into the same fragment order (lane l <- row l & 15,
// k 8(l >> 4)), so every LDS read is a conflict-free lane-linear ds_read_b128.
// One __shared__ array (a second LDS object makes hipcc wait vmcnt(0) early,
// cdna_hip_programming.md §5 trap 4a), two barriers per K step, ~3 workgroups
// per CU overlap each other's staging.  Workgroups are remapped XCD-major so
// each XCD's L2 holds a compact block of (row tile, weight tile) pairs.
constexpr int GB_M = 128, GB_N = 128, GB_K = 64;
constexpr int GEMM_BIG_M = 256;
constexpr int GEMM_BIG_TILES = 256;

template <int NS>
__global__ void __launch_bounds__(256) k_gemm_big(GemmArgs a) {
  constexpr int STAGE = 2 * 16 * 512;   // [W blocks 16][A blocks 16] x 1 KB
  __shared__ __attribute__((aligned(16))) bf16 sm[NS * STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntm = (a.M + GB_M - 1) / GB_M, ntn = a.N / GB_N, total = ntm * ntn;
  // XCD-major remap: consecutive ids go round-robin over the 8 XCDs; give XCD x
  // the contiguous range [x * per, (x + 1) * per) of tiles
  const int per = (total + 7) >> 3;
  const int t = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  if (t >= total) return;
  // grouped order inside the range: 4 row tiles sweep the weight tiles together
  constexpr int GM = 4;
  const int grp = t / (GM * ntn), gm = min(GM, ntm - grp * GM), tin = t - grp * GM * ntn;
  const int tm = grp * GM + tin % gm, tn = tin / gm;
  const int nchunk = a.K >> 5, nks = a.K >> 6;
  // staging: wave w fills W blocks 4w..4w+3 and A blocks 4w..4w+3 (block j = (tile j >> 1, chunk j & 1))
  const bf16* wsrc[4];
  const bf16* asrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = 4 * wave + i;
    wsrc[i] = a.w + ((long long)(tn * 8 + (j >> 1)) * nchunk + (j & 1)) * 512 + lane * 8;
    const int m = min(tm * GB_M + (j >> 1) * 16 + r, a.M - 1);
    asrc[i] = rm_bf(a.a, m) + (j & 1) * 32 + 8 * g;
  }
  auto issue = [&](int ks) {
    bf16* st = sm + (ks % NS) * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = 4 * wave + i;
      __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + (long long)ks * 1024),
                                       (__attribute__((address_space(3))) void*)(st + j * 512), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + ks * GB_K),
                                       (__attribute__((address_space(3))) void*)(st + 16 * 512 + j * 512), 16, 0, 0);
    }
  };
  f32x4 acc[4][4];   // [weight tile nt][row tile mt]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[nt][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (NS > 1) issue(0);
  for (int ks = 0; ks < nks; ++ks) {
    if (NS == 1) {
      issue(ks);
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else if (ks + 1 < nks) {
      // step ks + 1 streams into the other stage (released by the previous
      // step's closing barrier) while this one computes; raw barriers so the
      // prefetch stays in flight (cdna_hip_programming.md "Pipelining across barriers")
      issue(ks + 1);
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    const bf16* wl = sm + (ks % NS) * STAGE;
    const bf16* al = wl + 16 * 512;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      bf16x8 wf[4], xf[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) wf[nt] = *(const bf16x8*)(wl + ((wn * 4 + nt) * 2 + c) * 512 + lane * 8);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) xf[mt] = *(const bf16x8*)(al + ((wm * 4 + mt) * 2 + c) * 512 + lane * 8);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[nt][mt] = mfma(wf[nt], xf[mt], acc[nt][mt]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  // epilogue: one epi_tile body in a rolled loop, the accumulators rotated
  // through acc[0][0] (16 unrolled copies of epi_tile's RoPE / DPM forms
  // spilled the accumulators to scratch)
#pragma unroll 1
  for (int i = 0; i < 16; ++i) {
    float v[4] = {acc[0][0][0], acc[0][0][1], acc[0][0][2], acc[0][0][3]};
    epi_tile(a, tm * GB_M + (wm * 4 + (i & 3)) * 16 + r, tn * GB_N + (wn * 4 + (i >> 2)) * 16, lane, v);
#pragma unroll
    for (int k = 0; k < 15; ++k) acc[k >> 2][k & 3] = acc[(k + 1) >> 2][(k + 1) & 3];
  }
}

// ------------------------------------------------------------------ host launch
static std::atomic<int> g_tune_nw{0}, g_tune_ks{0}, g_tune_handoff{-1}, g_tune_waves{0}, g_tune_u{0}, g_tune_tpw{0};
static std::atomic<int> g_gemv_bal{1};   // diagnostic (vv_gemv_tune_bal): 0 = ntile / 8 workgroups at M >= 8
extern "C" int vv_gemv_tune_bal(int on) {
  g_gemv_bal = on ? 1 : 0;
  return 0;
}
static std::atomic<int> g_gemv_max_m{64};   // more rows than this: the tiled k_gemm (vv_gemv_tune_maxm)
extern "C" int vv_gemv_tune_maxm(int m) {
  g_gemv_max_m = m > 0 ? m : 64;
  return 0;
}
static std::atomic<unsigned long long*> g_stamps{nullptr};
static const bool g_shape_log = getenv("VV_GEMM_LOG") != nullptr;

// diagnostic: GEMV launches record per-workgroup timestamps into buf (nullptr: off)
extern "C" int vv_gemv_stamps(void* buf) {
  g_stamps = (unsigned long long*)buf;
  return 0;
}

extern "C" int vv_gemv_tune(int nw, int ks, int handoff, int target_waves, int u) {
  g_tune_nw = nw;
  g_tune_ks = ks;
  g_tune_handoff = handoff;
  g_tune_waves = target_waves;
  g_tune_u = u;
  return 0;
}

// diagnostic: force k_gemv1's tiles per workgroup (0: plan)
extern "C" int vv_gemv_tune_tpw(int tpw) {
  g_tune_tpw = tpw;
  return 0;
}

struct GemmPlan { int nw, ksplit, u, tpw, grid = 0; };   // grid: workgroups when not ntile / tpw

// Measured on MI355X (tools/gemv_sweep.py two-pass min, profiles/r01_gemv_sweep*.txt).
// Cross-workgroup split-K only for few-tile, long-row shapes (the M >= 8 down
// projections and codec fc2, and the M < 8 LM down projection, listed below):
// a hand-off costs >= 2 us in the sc1 form and up to 30 us with fences, which
// only those shapes win back in extra CUs.  Waves per workgroup (nw) and weight
// chunks in flight per wave (u):
//   * >= 1024 tiles (LM gate|up, head adaLN): 2 waves — every workgroup resident
//     in the first round (4-wave groups left a second-round tail: 16.7 -> 14.0 us)
//   * few tiles, long rows (LM / head down): 8 waves x 4; 128 tiles x K >= 8192
//     (codec fc2): 4 x 8; at M >= 8 two workgroups split K (the shapes
//     where the hand-off pays, profiles/r01_gemv_sweep_ks.txt: B = 8 LM down
//     18.7 -> 15.5 us, head down 13.0 -> 12.3, B = 8 codec fc2 13.1 -> 12.0),
//     and at M < 8 for < 128 tiles x K >= 8192 (LM down: 96 tiles reach only 96
//     CUs; same-box interleaved A/B, 5 pairs: B = 1 step 3.749 -> 3.725 ms,
//     B = 2 4.41 -> 4.30 ms)
//   * 16 < M <= 64 (k_gemv): 4 waves, 1 for >= 1024 tiles (the batched head
//     adaLN, M = 2 x 10 steps: 35 -> 20.5 us)
//   * few tiles, short rows (qkv, o_proj): 4 x 8, all chunks in flight at once
//   * 8 <= M <= 16 otherwise: 8 x 2; with many tiles the workgroup owns tpw
//     tiles that share one staging of the A rows (tools/gemv_sweep.py --tpw,
//     profiles/r01_gemv_sweep_tpw.txt: B = 8 LM gate|up 30.5 -> 20.0 us, head
//     gate|up 4 tiles per group 15.6 us)
// diagnostic (vv_gemv_tune_shape): plan overrides for one (N, K) at M <= m_max,
// for same-box A/Bs of a single shape inside the loop (tools/ab_bench.py)
struct ShapeTune { int N, K, mmax, nw, ks, u, tpw; };
static ShapeTune g_shape_tune[8];
static std::atomic<int> g_nshape_tune{0};
extern "C" int vv_gemv_tune_shape(int N, int K, int mmax, int nw, int ks, int u, int tpw) {
  if (N <= 0) {
    g_nshape_tune = 0;
    return 0;
  }
  const int n = g_nshape_tune;
  if (n >= 8) return 1;
  g_shape_tune[n] = {N, K, mmax, nw, ks, u, tpw};
  g_nshape_tune = n + 1;   // published after the entry (seq_cst store)
  return 0;
}

static GemmPlan gemv_plan(int N, int K, int M) {
  const int ntune = g_nshape_tune;
  for (int i = 0; i < ntune; ++i) {
    const ShapeTune& s = g_shape_tune[i];
    if (s.N == N && s.K == K && M <= s.mmax) return {s.nw, s.ks, s.u, s.tpw};
  }
  const int chunks = K / 32, tiles = N / 16;
  int nw = 4, ks = 1, u = 4, tpw = 1;
  if (tiles <= 128 && chunks >= 128) {
    if (M >= 8) {   // batched rows: 2-way split-K (sc1 hand-off) reaches 2x the CUs
      ks = 2;
      if (chunks == 256 && tiles == 128) nw = 8;   // codec fc2, C = 2,048: 8 x 4 (B = 8 in-loop A/B: -53 us per step)
      else if (chunks >= 256 && M <= 16) {
        // long rows: split K until the workgroup's A slice fits k_gemv1's 64 KB of
        // LDS (staged once) instead of k_gemv's per-wave A fragment reads from L2
        // (LM down at B = 8, M 16 x K 8,960: 5 ways; B = 8 step 5.15 -> 5.05 ms in
        // interleaved in-loop runs, profiles/r03_gemv_rw_ab.txt; the same rule for
        // the codec fc2 above cost +20 us); 8 waves x 4 chunks
        while (ks < 8 && (size_t)M * ((chunks + ks - 1) / ks * 32 + 8) * 2 > 65536) ++ks;
        nw = 8;
      } else if (chunks >= 256) u = 8;
      else {
        nw = 8;
        // 4 splits at M > 16 (the codec fc2 at C = 1,024, B = 8: 64 rows x N 1,024 x
        // K 4,096 on 64 tiles; interleaved in-loop pairs, B = 8 step 3.921 / 3.923 ->
        // 3.893 / 3.896 ms; 8 splits x 2 chunks 3.935)
        if (M > 16) ks = 4;
      }
    } else if (tiles < 128 && chunks >= 256) {   // M < 8 LM down: 2-way split-K, 8 waves x 4
      ks = 2;
      nw = 8;
    } else if (tiles == 128 && chunks >= 256) {
      if (chunks == 256) nw = 8;   // codec fc2 at C = 2,048 (K 8,192): 8 x 4 (in-loop A/Bs below)
      else u = 8;
    } else {
      nw = 8;
    }
  } else if (M > 16) {
    nw = tiles >= 1024 ? 1 : 4;   // k_gemv (A from L2 per chunk): batched head adaLN 35 -> 20.5 us
  } else if (M >= 8 && tiles <= 8 && chunks >= 32) {
    // the head's final layer (N 64, K 1,536: 4 tiles) at B = 8: 8-way split-K so 32
    // workgroups share the 16-row RMSNorm prologue and the stream (interleaved
    // in-loop pairs: B = 8 step -20..-40 us; at M = 2 the hand-off costs more
    // than it saves, +20..+50 us)
    nw = 8;
    u = 2;
    ks = 8;
  } else if (M >= 8) {
    nw = 8;
    u = 2;
    if (tiles >= 1024) {  // many tiles: 8 tiles per workgroup (one wave each) share one A staging
      tpw = 8;
      u = M > 8 ? 4 : 8;
    } else if (tiles >= 512) {
      // 2 tiles per workgroup (256 workgroups: the codec fc1 at C = 2,048, N 8,192 x
      // K 2,048, B = 8) -- 4 reached only 128 CUs; interleaved in-loop pairs, B = 8
      // step 3.953 / 3.948 -> 3.927 / 3.920 ms (tools/ab_bench.py gemv_tune_shape)
      tpw = 2;
      u = 4;
    }
  } else if (tiles >= 1024) {
    // (VibeVoice-Large's K 3,584 rows too: 4 waves x 2 chunks won the bare-GEMV
    // sweep, 46.1 -> 43.8 us, but lost in the loop, 7.07 -> 7.15 ms per step)
    nw = 2;
  } else if (tiles <= 128) {
    // LM q|k|v (128 tiles x K 1,536) with codec fc2 above: 8 waves x 4 chunks
    // instead of 4 x 8, interleaved in-loop pairs -5 .. -26 us per B = 1 step
    if (tiles == 128 && chunks <= 64) nw = 8;
    else u = 8;
  } else if (tiles >= 512 && chunks <= 64) {
    u = 2;   // head gate|up (576 tiles x K 1,536): 6 interleaved in-loop pairs, B = 1 step -13 us vs u = 4
  }
  if (g_tune_waves > 0) {
    int wpt = (g_tune_waves + tiles - 1) / tiles;
    const int maxw = (chunks + 3) / 4;
    if (wpt > maxw) wpt = maxw;
    if (wpt < 1) wpt = 1;
    nw = wpt < 4 ? wpt : 4;
    ks = (wpt + nw - 1) / nw;
  }
  if (g_tune_nw > 0) nw = g_tune_nw;
  if (g_tune_ks > 0) ks = g_tune_ks;
  if (g_tune_u > 0) u = g_tune_u;
  if (g_tune_tpw > 0) tpw = g_tune_tpw;
  if (ks > chunks) ks = chunks;
  return {nw, ks, u, tpw};
}

static int max_waves(int) { return 8; }

// k_gemv1's dynamic LDS: the staged A slice (+ per-item sums of squares for
// the fused RMSNorm).  Built-in limit 64 KB.  Up to GEMV1_LDS_MAX is possible
// with the per-kernel opt-in (one workgroup may hold 160 KiB; k_gemv1's static
// arrays take ~8.3 KB) so the B = 8 down projections (M = 16 rows of 4,480 /
// 2,304 columns per K split) stage A once per workgroup instead of k_gemv's
// per-wave fragment loads -- measured slower (B = 8 step 5.51 -> 5.83 ms: one
// workgroup per CU leaves too few weight loads in flight), so it stays a hook.
constexpr size_t GEMV1_LDS_MAX = 151552, GEMV1_LDS_DEFAULT = 65536;
static std::atomic<size_t> g_gemv1_lds_max{GEMV1_LDS_DEFAULT};   // diagnostic (vv_gemv_tune_lds)
extern "C" int vv_gemv_tune_lds(int bytes) {
  g_gemv1_lds_max = bytes > 0 && (size_t)bytes <= GEMV1_LDS_MAX ? (size_t)bytes : GEMV1_LDS_DEFAULT;
  return 0;
}
static size_t gemv1_lds(const GemmArgs& a) {
  const int nchunk = a.K >> 5;
  const size_t kw = ((nchunk + a.ksplit - 1) / a.ksplit) * 32;
  const size_t xs = ((size_t)a.M * (kw + 8) * sizeof(bf16) + 15) & ~(size_t)15;
  return xs + (a.xf.kind == XF_NORM ? (size_t)a.M * (kw / 8) * sizeof(float) : 0);
}
static bool gemv1_fits(const GemmArgs& a) { return gemv1_lds(a) <= g_gemv1_lds_max; }

template <int U, int XF, bool KEEP, int TPW, int RW>
static void go_gemv1(const GemmArgs& a, dim3 grid, dim3 block, size_t lds, hipStream_t st) {
  if (lds > 65536) {   // > 64 KB of dynamic LDS needs the opt-in, once per instantiation
    static const bool attr = hipFuncSetAttribute((const void*)k_gemv1<U, XF, KEEP, TPW, RW>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)GEMV1_LDS_MAX) == hipSuccess;
    (void)attr;   // a refused opt-in surfaces as the launch error
  }
  hipLaunchKernelGGL((k_gemv1<U, XF, KEEP, TPW, RW>), grid, block, lds, st, a);
}

// Row-per-wave norm prologue (k_gemv1's RW form) for this launch?  Whole rows
// of K = 1,536 (3 items per lane) at up to 2 rows per wave, or K = 3,584 (7
// items) at one row per wave without adaLN operands (their registers would cost
// occupancy).  A separate instantiation: compiled into the item-per-thread
// kernels it cost them registers / SGPR spills (B = 1 step 3.57 -> 3.66 ms).
// Interleaved same-box runs (profiles/r03_gemv_rw_ab.txt): B = 8 step 5.45-5.47
// -> 5.14-5.16 ms (M = 16 LM gate|up 19.98 -> 17.11 us, q|k|v 11.20 -> 8.63,
// head gate|up 15.62 -> 12.45 in tools/gemv_variants.py), VibeVoice-Large B = 1
// 7.14 -> 6.85 ms (K = 3,584 rows), 1.5B B = 1 3.597 -> 3.588 ms.
// Diagnostic: vv_gemv_tune_rw(min rows; 99 = off).
// The K = 3,584 adaLN rows (VibeVoice-Large head) take the LDS-DMA form (RW 2).
// Diagnostic: vv_gemv_tune_rw(min rows; 99 = off; -1 = built-in without RW 2).
static std::atomic<int> g_rw_min_m{1};
static std::atomic<bool> g_rw_dma{true};
extern "C" int vv_gemv_tune_rw(int min_m) {
  g_rw_min_m = min_m > 0 ? min_m : 1;
  g_rw_dma = min_m >= 0;
  return 0;
}
static int gemv1_rw(const GemmArgs& a, int nw) {
  if (a.xf.kind != XF_NORM || a.ksplit != 1 || a.M < g_rw_min_m || a.K % 512) return 0;
  const int ipr = a.K / 512, rpw = (a.M + nw - 1) / nw;
  if (ipr == 3 && rpw <= 2) return 1;
  if (ipr == 7 && rpw == 1) return !a.xf.mod ? 1 : g_rw_dma ? 2 : 0;
  return 0;
}

// TPW is a template argument so the one-tile form (every M < 8 launch) keeps
// its straight-line index math (a runtime tiles-per-group cost 1 us per launch)
template <int XF, int TPW, int RW>
static void launch_gemv1_rw(const GemmArgs& a, int u, dim3 grid, dim3 block, size_t lds, hipStream_t st) {
  if (a.keep) {
    if (u == 4) go_gemv1<4, XF, true, TPW, RW>(a, grid, block, lds, st);
    else if (u == 2) go_gemv1<2, XF, true, TPW, RW>(a, grid, block, lds, st);
    else go_gemv1<8, XF, true, TPW, RW>(a, grid, block, lds, st);
  } else {
    if (u == 4) go_gemv1<4, XF, false, TPW, RW>(a, grid, block, lds, st);
    else if (u == 2) go_gemv1<2, XF, false, TPW, RW>(a, grid, block, lds, st);
    else go_gemv1<8, XF, false, TPW, RW>(a, grid, block, lds, st);
  }
}
template <int XF, int TPW>
static void launch_gemv1(const GemmArgs& a, int u, dim3 grid, dim3 block, size_t lds, hipStream_t st) {
  const int rw = XF == XF_NORM ? gemv1_rw(a, block.x / 64) : 0;
  if (rw == 1) launch_gemv1_rw<XF_NORM, TPW, 1>(a, u, grid, block, lds, st);
  else if (rw == 2 && TPW == 1) launch_gemv1_rw<XF_NORM, 1, 2>(a, u, grid, block, lds, st);
  else launch_gemv1_rw<XF, TPW, 0>(a, u, grid, block, lds, st);
}

template <int XF>
static void launch_gemv_xf(const GemmArgs& a, int mrep, int u, dim3 grid, dim3 block, hipStream_t st) {
  if (mrep == 1 && !gemv1_fits(a)) {
    hipLaunchKernelGGL((k_gemv<1, 8, XF>), grid, block, 0, st, a);
    return;
  }
  if (mrep == 1) {
    const size_t lds = gemv1_lds(a);
    if (a.tpw == 1) launch_gemv1<XF, 1>(a, u, grid, block, lds, st);
    else if (a.tpw == 2) launch_gemv1<XF, 2>(a, u, grid, block, lds, st);
    else if (a.tpw == 4) launch_gemv1<XF, 4>(a, u, grid, block, lds, st);
    else if (a.tpw == 5) launch_gemv1<XF, 5>(a, u, grid, block, lds, st);
    else launch_gemv1<XF, 8>(a, u, grid, block, lds, st);
    return;
  }
  switch (mrep) {
    case 2: hipLaunchKernelGGL((k_gemv<2, 4, XF>), grid, block, 0, st, a); break;
    case 3: hipLaunchKernelGGL((k_gemv<3, 2, XF>), grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL((k_gemv<4, 2, XF>), grid, block, 0, st, a); break;
  }
}

// ------------------------------------------------------------------ 256 x 256 tile (prefill, large batches)
// cdna_hip_programming.md §5: the 128² two-barrier structure (k_gemm_big) tops
// out near 900 TF; a 256 x 256 tile at one 8-wave workgroup per CU halves the
// operand bytes per FLOP and keeps a 3-stage-deep LDS-DMA ring in flight across
// raw barriers.  Here:
//   * 8 waves as 2 (rows m) x 4 (weight rows n): wave (wr, wc) owns 128 m x 64 n
//     = 8 x 4 accumulator tiles (128 VGPRs);
//   * K in 32-wide stages, a ring of 4 stages in LDS (4 x 32 KB: 16 A + 16 W one-KB
//     fragment blocks).  Step s computes stage s from registers while the wave
//     reads stage s + 1's fragments into its second register set; stage s + 4 is
//     issued into stage s's buffer right after the barrier that ends every wave's
//     reads of it, so three stages are in flight; each step waits with a counted
//     vmcnt (never 0 in the loop) and ONE raw s_barrier (a __syncthreads() would
//     drain the ring);
//   * the packed weight blocks are MFMA fragments already (one 1 KB glds per wave
//     instruction, lane-linear) and A rows are gathered per lane into the same
//     order, so every ds_read_b128 is lane-linear and conflict-free (no swizzle);
//   * one __shared__ array (a second LDS object makes hipcc drain vmcnt(0) before
//     every k-step, §5 item 4a); loads hand-interleaved between the MFMAs.
// K order of accumulation per output is k_gemm's (chunk by chunk): bit-identical.
// s_waitcnt immediates (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] |
// vmcnt[5:4] << 14; a field at its maximum does not wait).  The builtin, unlike an
// asm wait, is seen by hipcc's waitcnt pass, which then does not re-wait (with
// lgkmcnt(0)) for fragments this wait already retired
constexpr unsigned WC_VM12 = 0x0F7C, WC_VM8_LGKM0 = 0x0078, WC_LGKM0 = 0xC07F, WC_VM0 = 0x0F70;
// (Measured and rejected, DESIGN.md "Prefill": the wave tile on
// v_mfma_f32_32x32x16_bf16 -- 0.305 vs 0.443 of peak on gate|up -- and the
// ablation builds that located the ceiling; neither is built any more.)
constexpr int GX_M = 256, GX_N = 256, GX_NS = 4;
// fewest 256 x 256 tiles that take k_gemm_xl: 3/4 of the 256 CUs.  One round of
// 192 tiles (the diffusion head's down projection at M = 8,192: 32 x 6) runs
// at the per-tile rate of k_gemm_xl's multi-round launches (~1,000 TF/s at
// 384 tiles, DESIGN.md "MFMA utilisation") where k_gemm_big's 768 128² tiles
// reached 665 TF/s
constexpr int GX_MIN_TILES = 192;
constexpr int GX_STAGE = 32 * 512;                       // elements per stage
constexpr size_t GX_LDS = (size_t)GX_NS * GX_STAGE * 2;   // 128 KB

__global__ void __launch_bounds__(512) k_gemm_xl(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16 smx[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // scalar: the glds LDS bases (M0) too
  const int r = lane & 15, g = lane >> 4;
  const int wr = wave >> 2, wc = wave & 3;
  const int ntm = (a.M + GX_M - 1) / GX_M, ntn = a.N / GX_N, total = ntm * ntn;
  // XCD-major remap (bijective for any total), then groups of 4 row tiles sweep the weight tiles
  const int nb = gridDim.x, xcd = (int)(blockIdx.x & 7), q8 = nb >> 3, r8 = nb & 7;
  const int t = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (int)(blockIdx.x >> 3);
  if (t >= total) return;
  constexpr int GM = 4;
  const int grp = t / (GM * ntn), gm = min(GM, ntm - grp * GM), tin = t - grp * GM * ntn;
  const int tm = grp * GM + tin % gm, tn = tin / gm;
  const int nch = a.K >> 5;
  // staging: wave w fills A blocks 2w, 2w + 1 (row tiles) and W blocks 2w, 2w + 1 (weight tiles)
  const bf16* asrc[2];
  const bf16* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = 2 * wave + i;
    if (a.apack) {   // packed rows: one contiguous 1 KB block per (row tile, chunk), like W
      asrc[i] = (const bf16*)a.a.base + (long long)min(tm * 16 + j, (a.M - 1) >> 4) * nch * 512 + lane * 8;
    } else {
      const int m = min(tm * GX_M + j * 16 + r, a.M - 1);
      asrc[i] = rm_bf(a.a, m) + 8 * g;
    }
    wsrc[i] = a.w + (long long)(tn * 16 + j) * nch * 512 + lane * 8;
  }
  auto issue = [&](int s) {
    bf16* st = smx + (s & (GX_NS - 1)) * GX_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 2 * wave + i;
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (a.apack ? (long long)s * 512 : (long long)s * 32)),
                                       (__attribute__((address_space(3))) void*)(st + j * 512), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + (long long)s * 512),
                                       (__attribute__((address_space(3))) void*)(st + (16 + j) * 512), 16, 0, 0);
    }
  };
  // one of a stage's 4 glds pieces per wave (q: block i = q >> 1, A (even) or W (odd))
  auto issue_piece = [&](int s, int q) {
    bf16* st = smx + (s & (GX_NS - 1)) * GX_STAGE;
    const int i = q >> 1, j = 2 * wave + i;
    if (q & 1)
      __builtin_amdgcn_global_load_lds((const void*)(wsrc[i] + (long long)s * 512),
                                       (__attribute__((address_space(3))) void*)(st + (16 + j) * 512), 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + (a.apack ? (long long)s * 512 : (long long)s * 32)),
                                       (__attribute__((address_space(3))) void*)(st + j * 512), 16, 0, 0);
  };
  f32x4 acc[4][8];   // [weight tile nt][row tile mt]
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // fragments of stage s are read into registers during step s - 1 (two register
  // sets), so each wave's LDS reads of the next stage overlap its MFMAs
  auto frags = [&](int s, bf16x8 (&wf)[4], bf16x8 (&xf)[8]) {
    const bf16* st = smx + (s & (GX_NS - 1)) * GX_STAGE;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) wf[nt] = *(const bf16x8*)(st + (16 + wc * 4 + nt) * 512 + lane * 8);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) xf[mt] = *(const bf16x8*)(st + (wr * 8 + mt) * 512 + lane * 8);
  };
  auto macs = [&](const bf16x8 (&wf)[4], const bf16x8 (&xf)[8]) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) acc[nt][mt] = mfma(wf[nt], xf[mt], acc[nt][mt]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read (glds)
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // DS read
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);   // MFMA
    }
    // keep the MFMAs above the next step's asm waits ("memory" does not order
    // register-only instructions, cdna_hip_programming.md §5.7 rule 18)
    __builtin_amdgcn_sched_barrier(0);
  };
  // ring: stages s + 1 .. s + 3 in flight while stage s computes; exactly 4 glds
  // per wave per step (stages past the end re-load the last one into a buffer
  // nothing reads again), so vmcnt(8) retires stage s + 1 at every step and each
  // half-step below is one basic block the scheduler can interleave
  const int last = nch - 1;
  issue(0);
  issue(min(1, last));
  issue(min(2, last));
  issue(min(3, last));
  __builtin_amdgcn_s_waitcnt(WC_VM12);
  __builtin_amdgcn_s_barrier();
  bf16x8 wa[4], xa[8], wb[4], xb[8];
  frags(0, wa, xa);
  int s = 0;
  // A step in 4 pinned groups (sched_barrier fences): 1 glds piece of stage
  // s + 4, 3 fragment reads of stage s + 1, then the 8 MFMAs of weight tile nt = q
  // on stage s -- the loads' issue cost (M0 set-up, ~60+ cycles per LDS-DMA
  // piece) sits between MFMAs instead of in front of all 32 with the matrix pipe
  // idle.  Hand-placed: sched_group_barrier did not move the glds, and
  // s_setprio is a scheduling boundary (with it around the MFMAs every load
  // issued ahead of all 32).
  auto step = [&](int sis, int srd, const bf16x8 (&wf)[4], const bf16x8 (&xf)[8], bf16x8 (&wn)[4],
                  bf16x8 (&xn)[8]) {
    const bf16* st = smx + (srd & (GX_NS - 1)) * GX_STAGE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      issue_piece(sis, q);
#pragma unroll
      for (int f = 3 * q; f < 3 * q + 3; ++f) {
        if (f < 4) wn[f] = *(const bf16x8*)(st + (16 + wc * 4 + f) * 512 + lane * 8);
        else xn[f - 4] = *(const bf16x8*)(st + (wr * 8 + f - 4) * 512 + lane * 8);
      }
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) acc[q][mt] = mfma(wf[q], xf[mt], acc[q][mt]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (; s + 1 < nch; s += 2) {
    __builtin_amdgcn_s_waitcnt(WC_VM8_LGKM0);
    __builtin_amdgcn_s_barrier();
    step(min(s + 4, last), s + 1, wa, xa, wb, xb);
    __builtin_amdgcn_s_waitcnt(WC_VM8_LGKM0);
    __builtin_amdgcn_s_barrier();
    step(min(s + 5, last), min(s + 2, last), wb, xb, wa, xa);
  }
  if (s < nch) {   // odd stage count: the last stage is in set a
    __builtin_amdgcn_s_waitcnt(WC_LGKM0);
    macs(wa, xa);
  }
  __builtin_amdgcn_s_waitcnt(WC_VM0);   // the past-the-end re-loads land before the workgroup ends
  // epilogue: the accumulators go through the (now idle) LDS ring, 16 tiles per
  // wave at a time, so ONE epi_tile body runs in a rolled loop that indexes
  // memory (unrolled copies of the RoPE / DPM forms spill; rotating 32
  // accumulators through one register tile cost ~4,000 moves per wave -- 30 % of
  // a K = 1536 tile)
  __syncthreads();   // every wave is past its reads of the last stage
  // pass p (row tiles 64 p .. 64 p + 63 of the wave's 128) -> this wave's LDS
  // region as [64 rows][64 cols] f32, odd rows' float4 slots XOR-shifted by one
  auto stage_ep = [&](float* ep, int p) {
    auto sw = [](int row, int col) { return row * 64 + (col ^ ((row & 1) << 2)); };
#pragma unroll
    for (int mq = 0; mq < 4; ++mq)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) *(f32x4*)(ep + sw(mq * 16 + r, nt * 16 + 4 * g)) = acc[nt][4 * p + mq];
  };
  if (rope_row8_ok(a)) {
    // q|k|v + RoPE + KV append in the same row-contiguous staging: a q / k lane
    // takes one row's 16-column tile (its two RoPE halves), a V lane one column
    // over 8 consecutive rows (one 16-byte store into the [dim][32 pos] block)
    float* ep = (float*)smx + wave * (64 * 64);
    auto sw = [](int row, int col) { return row * 64 + (col ^ ((row & 1) << 2)); };
    const int mb = tm * GX_M + wr * 128, nb = tn * GX_N + wc * 64;
    const bool vhead = (nb >> 7) >= a.rope.nh + a.rope.nkv;   // a wave's 64 columns lie in one head
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      stage_ep(ep, p);
      if (!vhead) {
#pragma unroll 1
        for (int it = 0; it < 4; ++it) {
          const int row = it * 16 + (lane >> 2), tq = lane & 3, m = mb + 64 * p + row;
          float lo[8], hi[8];
          *(f32x4*)lo = *(const f32x4*)(ep + sw(row, 16 * tq));
          *(f32x4*)(lo + 4) = *(const f32x4*)(ep + sw(row, 16 * tq + 4));
          *(f32x4*)hi = *(const f32x4*)(ep + sw(row, 16 * tq + 8));
          *(f32x4*)(hi + 4) = *(const f32x4*)(ep + sw(row, 16 * tq + 12));
          if (m < a.M) rope_qk8(a, m, nb + 16 * tq, lo, hi);
        }
      } else {
#pragma unroll 1
        for (int it = 0; it < 8; ++it) {
          const int r0 = it * 8, m0 = mb + 64 * p + r0;
          float vv[8];
#pragma unroll
          for (int k2 = 0; k2 < 8; ++k2) vv[k2] = ep[sw(r0 + k2, lane)];
          if (m0 < a.M) rope_v8(a, m0, nb + lane, vv);
        }
      }
    }
    return;
  }
  if (epi_row8_ok(a)) {
    // row-contiguous form: per wave and pass, 4 m-tiles x its 4 n-tiles -> LDS
    // [64 rows][64 cols] f32 (16 KB per wave, the whole ring for 8 waves; odd rows'
    // float4 slots XOR-shifted by one so the b128 reads below are conflict-free),
    // then every lane takes 8 consecutive columns of a row: 16-byte stores, 8 rows
    // x 128 bytes per instruction (SiLU*up: 16 rows x 64 bytes).  A wave reads
    // only its own region and its LDS ops run in order: no barrier between passes.
    float* ep = (float*)smx + wave * (64 * 64);
    auto sw = [](int row, int col) { return row * 64 + (col ^ ((row & 1) << 2)); };
    const int mb = tm * GX_M + wr * 128, nb = tn * GX_N + wc * 64;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      stage_ep(ep, p);
      if (a.epi.kind == EPI_SILU_MUL) {
#pragma unroll 1
        for (int it = 0; it < 4; ++it) {
          const int row = it * 16 + (lane >> 2), a4 = lane & 3, m = mb + 64 * p + row;
          float gt[8], up[8];
          *(f32x4*)gt = *(const f32x4*)(ep + sw(row, 16 * a4));
          *(f32x4*)(gt + 4) = *(const f32x4*)(ep + sw(row, 16 * a4 + 4));
          *(f32x4*)up = *(const f32x4*)(ep + sw(row, 16 * a4 + 8));
          *(f32x4*)(up + 4) = *(const f32x4*)(ep + sw(row, 16 * a4 + 12));
          if (m < a.M) epi_silu8(a, m, (nb >> 1) + 8 * a4, gt, up);
        }
      } else {
#pragma unroll 1
        for (int it = 0; it < 8; ++it) {
          const int row = it * 8 + (lane >> 3), c8 = lane & 7, m = mb + 64 * p + row;
          float v[8];
          *(f32x4*)v = *(const f32x4*)(ep + sw(row, 8 * c8));
          *(f32x4*)(v + 4) = *(const f32x4*)(ep + sw(row, 8 * c8 + 4));
          if (m < a.M) epi_row8(a, m, nb + 8 * c8, v);
        }
      }
    }
    return;
  }
  float* ep = (float*)smx + wave * (16 * 256);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) ep[t * 256 + j * 64 + lane] = acc[2 * h + (t >> 3)][t & 7][j];
#pragma unroll 1
    for (int t = 0; t < 16; ++t) {
      const int i = 16 * h + t;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = ep[t * 256 + j * 64 + lane];
      epi_tile(a, tm * GX_M + (wr * 8 + (i & 7)) * 16 + r, tn * GX_N + (wc * 4 + (i >> 3)) * 16, lane, v);
    }
  }
}

// diagnostic (vv_gemm_tune_big): 0 keeps every M > 64 GEMM on k_gemm; 1 / 2 LDS
// stages of the 128² tile (k_gemm_big); 3 (built-in) = the 256² tile (k_gemm_xl)
// where it applies, else k_gemm_big<2>; + 4 ignores the tile-count thresholds
static std::atomic<int> g_gemm_big{3}, g_gemm_big_any{0};
extern "C" int vv_gemm_tune_big(int mode) {
  g_gemm_big_any = mode >= 0 && (mode & 4) ? 1 : 0;
  g_gemm_big = mode < 0 ? 3 : mode & 3;
  return 0;
}

bool gemm_uses_xl(const GemmArgs& a) {
  const int total_xl = ((a.M + GX_M - 1) / GX_M) * (a.N / GX_N);
  return !(a.M <= 64 && (a.M <= 16 || a.M <= g_gemv_max_m || a.epi.kind == EPI_CFG_DPM)) && a.epi.kind != EPI_CFG_DPM &&
         g_gemm_big == 3 && a.M >= GEMM_BIG_M && a.N % GX_N == 0 && a.K % 32 == 0 &&
         (total_xl >= GX_MIN_TILES || g_gemm_big_any);
}

constexpr int GEMM_BN32 = 128;   // fewer 64-wide-tile workgroups than this: 32-wide tiles
template <int XF>
static int launch_gemm_xf(const GemmArgs& a, hipStream_t st) {
  // k_gemm_big only with >= one 128 x 128 tile per CU or >= 2^30 MACs: the
  // decode loop's codec GEMMs (B = 8: 320 - 1,600 rows x 256 - 1,024 columns
  // x K <= 1,024: 24 - 104 such tiles) are faster as k_gemm's 4x more 64 x 64
  // workgroups (B = 8 step 5.53 ms vs 5.83), a 1K-token prompt's o / down /
  // q|k|v projections (108 - 144 tiles, K >= 1,536) on k_gemm_big (14.5 -> 13.4 ms)
  // k_gemm_xl with >= GX_MIN_TILES 256 x 256 tiles (16K-token prefill: 384 - 4,480 tiles)
  const int total_xl = ((a.M + GX_M - 1) / GX_M) * (a.N / GX_N);
  if (XF == XF_NONE && g_gemm_big == 3 && a.M >= GEMM_BIG_M && a.N % GX_N == 0 && a.K % 32 == 0 &&
      (total_xl >= GX_MIN_TILES || g_gemm_big_any)) {
    static const bool attr = hipFuncSetAttribute((const void*)k_gemm_xl, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)GX_LDS) == hipSuccess;   // once (thread-safe static init)
    if (!attr) return 2;
    hipLaunchKernelGGL(k_gemm_xl, dim3(total_xl), dim3(512), GX_LDS, st, a);
    return 0;
  }
  const int total = ((a.M + GB_M - 1) / GB_M) * (a.N / GB_N);
  if (XF == XF_NONE && g_gemm_big && a.M >= GEMM_BIG_M && a.N % GB_N == 0 && a.K % GB_K == 0 &&
      (total >= GEMM_BIG_TILES || (long long)a.M * a.N * a.K >= (1LL << 30) || g_gemm_big_any)) {
    if (g_gemm_big == 1) hipLaunchKernelGGL(k_gemm_big<1>, dim3(((total + 7) >> 3) * 8), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_gemm_big<2>, dim3(((total + 7) >> 3) * 8), dim3(256), 0, st, a);
    return 0;
  }
  // 64-wide tiles unless that leaves fewer than GEMM_BN32 workgroups (the
  // codec's 200-row stage: fc2 N = 256 is 16 workgroups of K = 1,024)
  const int wg64 = ((a.M + 63) / 64) * (a.N / 64);
  if (a.N % 64 == 0 && wg64 >= GEMM_BN32) {
    dim3 grid((a.M + 63) / 64, a.N / 64);
    hipLaunchKernelGGL((k_gemm<64, XF>), grid, dim3(256), 0, st, a);
  } else if (a.N % 32 == 0) {
    dim3 grid((a.M + 63) / 64, a.N / 32);
    hipLaunchKernelGGL((k_gemm<32, XF>), grid, dim3(256), 0, st, a);
  } else {
    return 1;
  }
  return 0;
}

// LDS of the XF_MIX GEMV (A rows + history/new rows + partial sums), 0 when
// the fused form does not apply (rows > 16, rows not whole samples, C outside
// [512, 2048] — k_mix's summation order needs >= 64 chunks — or > 64 KB)
size_t gemv_mix_lds(int M, int T, int C) {
  if (M <= 0 || M > 16 || T <= 0 || M % T || M / T > 4 || C < 512 || C > 2048 || C % 256) return 0;
  const int rows = (M / T) * (6 + T), n8 = C / 8;
  const size_t xs = ((size_t)M * (C + 8) * 2 + 15) & ~(size_t)15;
  const size_t lds = xs + (size_t)rows * C * 2 + (size_t)M * n8 * 4;
  return lds <= 98304 ? lds : 0;
}

// The decode-GEMV launch plan for a (M <= 64): waves, K split, tiles per
// workgroup; sets a.ksplit / a.handoff / a.tpw (launch_gemm, vv_gemv_plan).
// CUs of the current device (cached per device)
static int device_cus() {
  static std::atomic<int> cache[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  int v = cache[dev].load();
  if (!v) {
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cache[dev] = v;
  }
  return v;
}

static GemmPlan gemv_resolve(GemmArgs& a) {
  const int mrep = (a.M + 15) / 16;
  GemmPlan p = gemv_plan(a.N, a.K, a.M);
  if (p.nw > max_waves(mrep)) p.nw = max_waves(mrep);
  a.ksplit = p.ksplit;
  if (a.ksplit > 1 && (!a.ws || !a.counters || a.N / 16 > 65536)) a.ksplit = 1;
  // Rows too long for one workgroup to stage in k_gemv1's LDS at one K split
  // (VibeVoice-Large's LM down projection, M = 2 x K 18,944 = 76 KB): split K
  // until the slice fits, 8 waves x 4 chunks (tools/gemv_sweep.py --large: 48.4 ->
  // 27.1 us), instead of k_gemv re-loading A fragments from L2 per chunk.
  if (mrep == 1 && a.M < 8 && a.xf.kind == XF_NONE && !g_tune_ks && a.ws && a.counters && a.N / 16 <= 65536 &&
      !gemv1_fits(a)) {
    GemmArgs t = a;
    while (!gemv1_fits(t) && t.ksplit < 4) t.ksplit *= 2;
    if (gemv1_fits(t)) {
      a.ksplit = t.ksplit;
      if (!g_tune_nw) p.nw = 8;
      if (!g_tune_u) p.u = 4;
    }
  }
  const int ho = g_tune_handoff;
  a.handoff = ho >= 0 ? ho : 1;
  a.tpw = 1;
  if (mrep == 1 && a.ksplit == 1 && a.xf.kind != XF_MIX && (p.tpw == 2 || p.tpw == 4 || p.tpw == 8) && p.nw % p.tpw == 0 && gemv1_fits(a))
    a.tpw = p.tpw;
  // Many tiles at M >= 8 (B = 8 LM gate|up: 1,120 tiles): ntile / 8 = 140
  // workgroups streamed from 140 of the 256 CUs (tools/gemv_stamps.py: 8.2 us of
  // stream per workgroup).  Balanced form: one workgroup per CU, an even share of
  // 4 or 5 tiles each, 2 waves per tile (k_gemv1<.., 5, ..>).
  if (g_gemv_bal && a.tpw == 8 && a.M >= 8 && a.xf.kind != XF_ATTN_MERGE) {
    const int ncu = device_cus(), tiles = a.N / 16;
    if (ncu > 0 && (tiles + ncu - 1) / ncu == 5) {
      a.tpw = 5;
      p.nw = 10;
      p.grid = ncu;
    }
  }
  return p;
}

// Host-only plan query (no device work; tests and tools): the kernel form and
// launch plan launch_gemm would use for an M <= 16 GEMV.  out[7] = {kernel
// (0 k_gemv1, 1 k_gemv: A fragments from L2), waves, K splits, chunks in flight,
// tiles per workgroup, norm prologue form (0 item per thread, 1 row per wave,
// 2 row per wave with LDS-DMA rows), dynamic LDS bytes}.
extern "C" int vv_gemv_plan(int M, int N, int K, int xf, int has_w, int has_mod, int* out) {
  if (M <= 0 || M > 16 || K % 32 || N % 16 || !out || (xf != XF_NONE && xf != XF_NORM && xf != XF_SILU_ADD)) return 1;
  static const bf16 dummy[8] = {};
  static unsigned dummy_ctr[1];
  GemmArgs a{};
  a.M = M;
  a.N = N;
  a.K = K;
  a.xf.kind = xf;
  a.xf.w = has_w ? dummy : nullptr;
  a.xf.mod = has_mod ? dummy : nullptr;
  static float dummy_ws[1];
  a.ws = dummy_ws;   // planning only tests these for null
  a.counters = dummy_ctr;
  const GemmPlan p = gemv_resolve(a);
  const bool g1 = gemv1_fits(a);
  out[0] = g1 ? 0 : 1;
  out[1] = p.nw;
  out[2] = a.ksplit;
  out[3] = p.u;
  out[4] = a.tpw;
  out[5] = g1 && xf == XF_NORM ? gemv1_rw(a, p.nw) : 0;
  out[6] = g1 ? (int)gemv1_lds(a) : 0;
  return 0;
}

// returns 0 ok, else an error code (see engine.cpp)
int launch_gemm(GemmArgs a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (a.K % 32 != 0 || a.N % 16 != 0) return 1;
  if (a.apack && (a.xf.kind != XF_NONE || !gemm_uses_xl(a))) return 1;   // only k_gemm_xl reads packed A rows
  if (a.epi.pack && (a.epi.kind != EPI_SILU_MUL || a.xf.kind != XF_NONE || !gemm_uses_xl(a) || (a.N >> 1) % 32 ||
                     ((unsigned long long)a.epi.out.base & 15)))
    return 1;   // ... and only its row-contiguous SiLU*up epilogue writes them
  if (a.xf.kind == XF_NORM && a.K % 8 != 0) return 1;
  if (a.epi.kind == EPI_ROPE && (a.rope.kv.d != 128 || !a.rope.pos || !a.rope.slots)) return 1;
  if (a.epi.kind == EPI_CFG_DPM && (a.M > 16 || 2 * a.dpm.n != a.M)) return 1;
  a.stamps = g_stamps;
  if (g_shape_log) {   // VV_GEMM_LOG=1: one line per launch (shape census for profiles/)
    fprintf(stderr, "vv_gemm M=%d N=%d K=%d xf=%d epi=%d\n", a.M, a.N, a.K, a.xf.kind, a.epi.kind);
  }
  if (a.M <= 64 && (a.M <= 16 || a.M <= g_gemv_max_m || a.epi.kind == EPI_CFG_DPM)) {
    if (launch_gemvw(a, st)) return hipGetLastError() == hipSuccess ? 0 : 2;
    const int mrep = (a.M + 15) / 16;
    const GemmPlan p = gemv_resolve(a);
    dim3 grid(p.grid ? p.grid : (a.N / 16 + a.tpw - 1) / a.tpw, a.ksplit), block(64 * p.nw);
    if (a.xf.kind == XF_MIX) {
      const size_t lds = gemv_mix_lds(a.M, a.xf.T, a.K);
      if (mrep != 1 || a.ksplit != 1 || !lds || (64 * p.nw) % (a.K / 8) || a.xf.ctx != 6 || a.a.idx) return 1;
      // tiles per workgroup (diagnostic plans only so far): the Block1D front half is
      // recomputed once per workgroup, so fewer, wider workgroups recompute it less
      const int mt = (p.tpw == 2 || p.tpw == 4) && p.nw % p.tpw == 0 ? p.tpw : 1;
      a.tpw = mt;
      grid.x = (a.N / 16 + mt - 1) / mt;
      // > 64 KB of dynamic LDS needs the opt-in (one workgroup may hold 160 KiB); once, thread-safe
      static const bool attr =
          hipFuncSetAttribute((const void*)k_gemv1<4, XF_MIX>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304) ==
              hipSuccess &&
          hipFuncSetAttribute((const void*)k_gemv1<4, XF_MIX, false, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              98304) == hipSuccess &&
          hipFuncSetAttribute((const void*)k_gemv1<4, XF_MIX, false, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              98304) == hipSuccess;
      if (!attr) return 2;
      if (mt == 4) hipLaunchKernelGGL((k_gemv1<4, XF_MIX, false, 4>), grid, block, lds, st, a);
      else if (mt == 2) hipLaunchKernelGGL((k_gemv1<4, XF_MIX, false, 2>), grid, block, lds, st, a);
      else hipLaunchKernelGGL((k_gemv1<4, XF_MIX>), grid, block, lds, st, a);
      return hipGetLastError() == hipSuccess ? 0 : 2;
    }
    if (a.xf.kind == XF_ATTN_MERGE) {   // o_proj on the attention's split partials: one plan form
      if (mrep != 1 || a.xf.nsplit < 1 || a.xf.nsplit > 8 || a.K % 128 || !a.xf.part_o || !a.xf.part_ml || !a.xf.qpos)
        return 1;
      a.ksplit = 1;
      a.tpw = 1;
      const size_t lds = gemv1_lds(a);
      hipLaunchKernelGGL((k_gemv1<8, XF_ATTN_MERGE, false, 1>), dim3(a.N / 16, 1), block, lds, st, a);
      return hipGetLastError() == hipSuccess ? 0 : 2;
    }
    switch (a.xf.kind) {
      case XF_NORM: launch_gemv_xf<XF_NORM>(a, mrep, p.u, grid, block, st); break;
      case XF_SILU_ADD: launch_gemv_xf<XF_SILU_ADD>(a, mrep, p.u, grid, block, st); break;
      default: launch_gemv_xf<XF_NONE>(a, mrep, p.u, grid, block, st); break;
    }
  } else {
    if (a.epi.kind == EPI_CFG_DPM) return 1;
    int rc;
    switch (a.xf.kind) {
      case XF_NORM: rc = launch_gemm_xf<XF_NORM>(a, st); break;
      case XF_SILU_ADD: rc = launch_gemm_xf<XF_SILU_ADD>(a, st); break;
      default: rc = launch_gemm_xf<XF_NONE>(a, st); break;
    }
    if (rc) return rc;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
