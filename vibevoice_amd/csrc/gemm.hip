// bf16 MFMA GEMMs for gfx950:  Y[m, n] = epi( sum_k A[m, k] * W[n, k] )
//
// W is a PyTorch Linear weight [N, K] (K contiguous), or a conv weight that the
// loader re-packed to the same [N, K] form (see vibevoice_amd/weights.py):
//   * causal conv k, stride s, channels-last input buffer with (k - s) history
//     rows in front:  A row t = buffer + t*s*C_in, K = k*C_in  (lda = s*C_in),
//   * 2-tap ConvTranspose (k = 2r, stride r): A row t = rows [t-1, t] of the
//     input buffer (1 history row), N = r*C_out and one output row = r
//     consecutive channels-last output rows.
// so every linear / conv layer on the hot path is this one kernel family.
//
// Two shapes:
//   k_gemv : M <= 64 (LM decode rows, diffusion-head rows, codec stage at T=1).
//            HBM-bound weight stream.  MFMA 16x16x32 with W as the A operand
//            (16 weight rows = the MFMA M dim) and the <=16*MREP activation rows
//            as the B operand; each wave streams a contiguous K range straight
//            to VGPRs (no LDS: the "GEMV / M <= 16" row of the guide), waves of a
//            workgroup split K and reduce through LDS, and workgroups may split
//            K further with an agent-scope release/acquire ticket (last arriver
//            reduces the fp32 slabs and runs the epilogue).
//   k_gemm : M > 64 (codec stages at T >= 8, LM prefill).  64 x BN workgroup
//            tile, 4 waves of 32 x BN/2, operands straight from L2.
#include "kernels.h"


// ---- epilogue on one 16(n) x 16(m) MFMA tile held in the C/D layout:
// lane l holds m = m0 + (l & 15), n = n0 + 4*(l >> 4) + i, i = 0..3.
DEV void epi_tile(const EpiArgs& e, int M, int N, int m, int n0, int lane, const float v_in[4]) {
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = v_in[i];
  const int g = lane >> 4;
  if (e.kind == EPI_SILU_MUL) {
    // rows 0..7 of the tile are gate, 8..15 the matching up rows; lane g<2 holds
    // gate rows 4g+i, lane g+2 holds up rows 8+4g+i
    float u[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) u[i] = __shfl_xor(v[i], 32);
    if (g >= 2 || m >= M) return;
    const int col = (n0 >> 1) + 4 * g;
    bf16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = tobf(rb(silu_f(rb(v[i]))) * rb(u[i]));
    *(bf16x4*)(rm_bfw(e.out, m) + col) = o;
    return;
  }
  if (m >= M) return;
  const int n = n0 + 4 * g;
  if (e.bias) {
    bf16x4 b = *(const bf16x4*)(e.bias + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] += bf(b[i]);
  }
  if (e.kind == EPI_F32) {
    float* o = (float*)e.out.base + rm_off(e.out, m) + n;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = v[i];
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
    bf16x4 r = *(const bf16x4*)(rm_bf(e.res, m) + n);
    float s[4] = {1.f, 1.f, 1.f, 1.f};
    bool scaled = false;
    if (e.gamma) {
      bf16x4 gm = *(const bf16x4*)(e.gamma + n);
#pragma unroll
      for (int i = 0; i < 4; ++i) s[i] = bf(gm[i]);
      scaled = true;
    } else if (e.gate.base) {
      bf16x4 gm = *(const bf16x4*)(rm_bf(e.gate, m) + n);
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
  *(bf16x4*)(rm_bfw(e.out, m) + n) = o;
}

DEV f32x4 mfma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------ GEMV
template <int MREP, int U>
__global__ void __launch_bounds__(1024) k_gemv(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, NW = blockDim.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int nchunk = a.K >> 5;
  const int gw = blockIdx.y * NW + wave, GW = gridDim.y * NW;
  const int c0 = (int)((long long)nchunk * gw / GW);
  const int c1 = (int)((long long)nchunk * (gw + 1) / GW);

  const bf16* wrow = a.w + (long long)(n0 + r) * a.ldw + 8 * g;
  const bf16* xrow[MREP];
  bool xok[MREP];
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr) {
    const int m = r + 16 * mr;
    xok[mr] = m < a.M;
    xrow[mr] = xok[mr] ? rm_bf(a.a, m) + 8 * g : nullptr;
  }
  f32x4 acc[MREP];
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr) acc[mr] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};

  int c = c0;
  for (; c + U <= c1; c += U) {
    bf16x8 wf[U], xf[U][MREP];
#pragma unroll
    for (int u = 0; u < U; ++u) wf[u] = *(const bf16x8*)(wrow + (c + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mr = 0; mr < MREP; ++mr)
        xf[u][mr] = xok[mr] ? *(const bf16x8*)(xrow[mr] + (c + u) * 32) : zero8;
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mr = 0; mr < MREP; ++mr) acc[mr] = mfma(wf[u], xf[u][mr], acc[mr]);
  }
  for (; c < c1; ++c) {
    bf16x8 wf = *(const bf16x8*)(wrow + c * 32);
#pragma unroll
    for (int mr = 0; mr < MREP; ++mr) {
      bf16x8 xf = xok[mr] ? *(const bf16x8*)(xrow[mr] + c * 32) : zero8;
      acc[mr] = mfma(wf, xf, acc[mr]);
    }
  }

  // ---- reduce the NW waves of this workgroup:  red[wave][mr*4 + i][lane]
  const int TILE = MREP * 256;
#pragma unroll
  for (int mr = 0; mr < MREP; ++mr)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * MREP * 4 + mr * 4 + i) * 64 + lane] = acc[mr][i];
  __syncthreads();
  for (int e = threadIdx.x; e < TILE; e += blockDim.x) {
    float s = 0.f;
    for (int w = 1; w < NW; ++w) s += red[w * TILE + e];
    red[e] += s;
  }
  __syncthreads();

  if (a.ksplit > 1) {
    // ---- cross-workgroup split-K: plain slab stores, agent release, ticket;
    // the last arriver acquires and reduces (cdna_hip_programming.md §5,
    // "In-launch split-K reduction"; Guideline 16).
    __shared__ unsigned last_flag;
    float* slab = a.ws + ((long long)blockIdx.x * a.ksplit + blockIdx.y) * TILE;
    for (int e = threadIdx.x; e < TILE; e += blockDim.x) slab[e] = red[e];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      unsigned t = __hip_atomic_fetch_add(&a.counters[blockIdx.x], 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
      last_flag = (t == (unsigned)(a.ksplit - 1)) ? 1u : 0u;
      if (last_flag) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (!last_flag) return;
    const float* slabs = a.ws + (long long)blockIdx.x * a.ksplit * TILE;
    for (int e = threadIdx.x; e < TILE; e += blockDim.x) {
      float s = 0.f;
      for (int k = 0; k < a.ksplit; ++k) s += slabs[k * TILE + e];
      red[e] = s;
    }
    if (threadIdx.x == 0)
      __hip_atomic_store(&a.counters[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  }
  // ---- epilogue: wave mr handles MFMA tile mr (lane layout preserved)
  for (int mr = wave; mr < MREP; mr += NW) {
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = red[(mr * 4 + i) * 64 + lane];
    epi_tile(a.epi, a.M, a.N, r + 16 * mr, n0, lane, v);
  }
}

// ------------------------------------------------------------------ tiled GEMM (M > 64)
template <int BN>
__global__ void __launch_bounds__(256) k_gemm(GemmArgs a) {
  constexpr int NT = BN / 32;  // 16-wide n tiles per wave (wave covers BN/2 columns)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;
  const int m_base = blockIdx.x * 64 + wm * 32;
  const int n_base = blockIdx.y * BN + wn * (BN / 2);
  const bf16* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wrow[nt] = a.w + (long long)(n_base + nt * 16 + r) * a.ldw + 8 * g;
  const bf16* xrow[2];
  bool xok[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = m_base + mt * 16 + r;
    xok[mt] = m < a.M;
    xrow[mt] = xok[mt] ? rm_bf(a.a, m) + 8 * g : nullptr;
  }
  f32x4 acc[2][NT];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  const int nk = a.K >> 5;
  int c = 0;
  for (; c + 2 <= nk; c += 2) {
    bf16x8 wf[2][NT], xf[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wf[u][nt] = *(const bf16x8*)(wrow[nt] + (c + u) * 32);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) xf[u][mt] = xok[mt] ? *(const bf16x8*)(xrow[mt] + (c + u) * 32) : zero8;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma(wf[u][nt], xf[u][mt], acc[mt][nt]);
  }
  for (; c < nk; ++c) {
    bf16x8 wf[NT], xf[2];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) wf[nt] = *(const bf16x8*)(wrow[nt] + c * 32);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) xf[mt] = xok[mt] ? *(const bf16x8*)(xrow[mt] + c * 32) : zero8;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma(wf[nt], xf[mt], acc[mt][nt]);
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      float v[4] = {acc[mt][nt][0], acc[mt][nt][1], acc[mt][nt][2], acc[mt][nt][3]};
      epi_tile(a.epi, a.M, a.N, m_base + mt * 16 + r, n_base + nt * 16, lane, v);
    }
}

// ------------------------------------------------------------------ host launch
struct GemmPlan { int nw, ksplit; };

static GemmPlan gemv_plan(int N, int K) {
  const int tiles = N / 16, chunks = K / 32;
  int wpt = (2048 + tiles - 1) / tiles;
  int maxw = chunks / 4 > 0 ? chunks / 4 : 1;
  if (wpt > maxw) wpt = maxw;
  if (wpt < 1) wpt = 1;
  int ks = (256 + tiles - 1) / tiles;
  if (ks > wpt) ks = wpt;
  if (ks < 1) ks = 1;
  int nw = (wpt + ks - 1) / ks;
  if (nw > 16) nw = 16;
  return {nw, ks};
}

// returns 0 ok, else an error code (see engine.cpp)
int launch_gemm(GemmArgs a, hipStream_t st) {
  if (a.M <= 0) return 0;
  if (a.K % 32 != 0 || a.N % 16 != 0) return 1;
  if (a.epi.kind == EPI_SILU_MUL && a.N % 16 != 0) return 1;
  if (a.M <= 64) {
    GemmPlan p = gemv_plan(a.N, a.K);
    const int mrep = (a.M + 15) / 16;
    a.ksplit = p.ksplit;
    if (a.ksplit > 1 && (!a.ws || !a.counters)) a.ksplit = 1;
    dim3 grid(a.N / 16, a.ksplit), block(64 * p.nw);
    size_t lds = (size_t)p.nw * mrep * 256 * sizeof(float);
    if (lds < (size_t)mrep * 256 * sizeof(float)) lds = (size_t)mrep * 256 * sizeof(float);
    switch (mrep) {
      case 1: hipLaunchKernelGGL((k_gemv<1, 8>), grid, block, lds, st, a); break;
      case 2: hipLaunchKernelGGL((k_gemv<2, 4>), grid, block, lds, st, a); break;
      case 3: hipLaunchKernelGGL((k_gemv<3, 4>), grid, block, lds, st, a); break;
      default: hipLaunchKernelGGL((k_gemv<4, 2>), grid, block, lds, st, a); break;
    }
  } else {
    if (a.N % 64 == 0) {
      dim3 grid((a.M + 63) / 64, a.N / 64);
      hipLaunchKernelGGL((k_gemm<64>), grid, dim3(256), 0, st, a);
    } else if (a.N % 32 == 0) {
      dim3 grid((a.M + 63) / 64, a.N / 32);
      hipLaunchKernelGGL((k_gemm<32>), grid, dim3(256), 0, st, a);
    } else {
      return 1;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
