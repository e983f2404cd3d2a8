// A whole codec stage of Block1Ds at T = 1, C = 2,048, one sample, in ONE
// persistent launch: the acoustic decoder's first stage and the semantic
// encoder's last (8 blocks each; modular_vibevoice_tokenizer.py:620-684
// Block1D: x + gamma * dwconv(norm(x)), then + ffn_gamma * fc2(gelu(fc1(ffn_norm(.))))).
//
// Why (DESIGN.md "Codec stage"): as separate launches each block is a fused
// XF_MIX fc1 GEMV (13.6 us for 33.5 MB) and an fc2 GEMV (11.2 us for 33.5 MB):
// each stream starts only when its launch does, behind the A row's round trip.
// Here the grid of 256 workgroups (one per CU) stays resident for the stage and
// streams block j+1's 256 KB slice per CU while block j's hand-offs run.
//
// Decomposition per workgroup w (C = 2,048, F = 8,192, G = 256):
//   * front half: the control wave recomputes norm / conv / residual / FFN norm
//     for the whole row (k_mix's and XF_MIX's arithmetic and summation order),
//     the conv's six history taps ahead of time (during the previous block's
//     first wait);
//     workgroup 0 appends the new conv-input row to the block's buffer;
//   * fc1: w owns hidden units [32w, 32w + 32) (MFMA tiles 2w, 2w + 1: one
//     contiguous 128 KB slice, LDS DMA) -> GELU -> 64 B of the hidden row,
//     written through; grid wait;
//   * fc2: w owns output columns [8w, 8w + 8) (half of MFMA tile w / 2, 128 KB,
//     in registers: 16 chunks per compute thread) over the whole hidden row (LDS
//     DMA) -> gamma residual -> 16 B of the next block's input; grid wait.
// Weight stream order per compute wave: block j+1's fc1 DMA, then its fc2
// register loads, both issued right after block j's fc2 products (each wave DMAs
// and reads only its own LDS chunks); the fc1 dots wait with an explicit
// vmcnt(16) (the fc2 loads may still fly), the fc2 dots with hipcc's own
// vmcnt(0).  Measured per block (tools/codec_stage_stamps.py, DESIGN.md "Codec
// stage"): ~18.5 us, the second wait running behind the 256 KB stream; issuing
// the fc1 slice a wait earlier put 128 KB behind each wait instead and measured
// the same (17.8 us per block, the codec step 14 us slower).  The compute waves'
// queues carry nothing but weights; the control wave does every other global
// access.  Hand-offs: write-through stores + the grid wait of persist_dev.h.
//
// Arithmetic: the front half is XF_MIX's term for term (bit-identical); fc1 /
// fc2 are fp32 sums of exact bf16 products (v_dot2c) in a fixed order --
// a different order than the MFMA GEMVs', so not bit-identical to the
// launch-per-GEMV path (tests: within bf16 of it and of the oracle, bitwise
// run to run).  Epilogues are epi_row8's EPI_GELU / EPI_RES.
#include <type_traits>

#include "persist_dev.h"

namespace cs {
constexpr int C = 2048, F = 4 * C, G = pk::G, CTX = 6;
constexpr int NTC = 512, NT = NTC + 64;     // 8 compute waves + the control wave
constexpr int NCH = C / 8;                  // 16-byte chunks of a row (= G: chunk w holds workgroup w's columns)
constexpr int CPT = 16;                     // weight chunks per compute thread per GEMV
constexpr int ROWS1 = F / G;                // fc1 rows per workgroup (32: two MFMA tiles)
constexpr int ROWS2 = C / G;                // fc2 rows per workgroup (8: half a tile)
static_assert(ROWS1 * C / 8 == CPT * NTC && ROWS2 * F / 8 == CPT * NTC && NCH == G && NCH == 4 * 64,
              "codec stage geometry");
// LDS carve-up (bytes)
constexpr int W1 = 0, W1_B = ROWS1 * C * 2;            // fc1 slice (DMA), 128 KB
constexpr int HS = W1 + W1_B, HS_B = F * 2;            // hidden row (fc2 phase) / fc1 input row (fc1 phase)
constexpr int PA = HS + HS_B, PA_B = C * 4;            // the conv's history taps summed (fp32)
constexpr int W6 = PA + PA_B, W6_B = C * 2;            // the conv's tap on the new row
constexpr int RED = W6 + W6_B, RED_B = 8 * ROWS1 * 4;  // compute-wave partials
constexpr int SM = RED + RED_B, SM_B = 64;             // ok flag, this workgroup's 8 columns of y
constexpr int TOTAL = SM + SM_B;
static_assert(TOTAL <= 160 * 1024, "one workgroup per CU");
}  // namespace cs

// the four 16-lane rows of a wave summed per lane position (lanes l, l ^ 16, l ^ 32, l ^ 48)
DEV float cs_rows_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__global__ void __launch_bounds__(cs::NT) k_codec_stage(CodecStageArgs a) {
  using namespace cs;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* w1_s = (bf16*)(smem + W1);
  bf16* h_s = (bf16*)(smem + HS);     // fc2 phase: the hidden row
  bf16* a_s = (bf16*)(smem + HS);     // fc1 phase: fc1's input row (same bytes)
  float* pa_s = (float*)(smem + PA);  // [NCH][8]
  bf16* w6_s = (bf16*)(smem + W6);    // [NCH][8]
  float* red = (float*)(smem + RED);
  unsigned* ok_s = (unsigned*)(smem + SM);
  bf16* y_s = (bf16*)(smem + SM + 16);

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool ctl = wave == NTC / 64;
  const int w = blockIdx.x;
  const long long slot = a.slots[0];
  unsigned g0 = 0, nwait = 0;
  if (ctl) __builtin_amdgcn_s_setprio(3);
  if (ctl) g0 = __hip_atomic_load((hl_gu32*)hl_gen(a.sync), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;
  // diagnostics (tools/codec_stage_stamps.py): per block j, slot 8j + k, k =
  // 0 front half begins, 1 fc1 input in LDS, 2 (compute wave 0) fc1 slice landed,
  // 3 fc1 partials in LDS, 4 hidden-row wait released, 5 hidden row in LDS,
  // 6 fc2 partials in LDS, 7 next-input wait released
  auto stamp = [&](int k, bool by_ctl) {
    if (a.stamps && threadIdx.x == (by_ctl ? NTC : 0)) a.stamps[w * 64 + k] = __builtin_amdgcn_s_memrealtime();
  };

  // ---- the weight stream of block j (compute waves): fc1 slice by LDS DMA
  // (chunk g = i * NTC + t of the contiguous slice -> LDS 16 g), then the fc2
  // slice into registers (chunk g: k-block g >> 5, k-sub (g >> 3) & 3, row g & 7
  // of the workgroup's half tile; a wave's load = eight full 128-byte runs)
  bf16x8 w2[CPT];
  auto issue_fc1 = [&](int j, int t) {
    const bf16* g1 = hl_opaque(a.b[j].fc1_w) + (long long)w * ROWS1 * C;
#pragma unroll
    for (int i = 0; i < CPT; ++i)
      hl_dma16<false, true>(w1_s + (i * NTC + 64 * wave) * 8, g1 + ((long long)i * NTC + t) * 8);
  };
  auto issue_fc2 = [&](int j, int t) {
    const bf16* g2 = hl_opaque(a.b[j].fc2_w) + (long long)(w >> 1) * F * 16 + (w & 1) * 64;
    const int r = t & 7, s = (t >> 3) & 3;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int kc = (i * NTC + t) >> 5;
      w2[i] = hl_ldnt(g2 + (long long)kc * 512 + (16 * s + r) * 8);
    }
  };
  // Paced halves (pubfirst == 3): chunks [8 h, 8 h + 8) of a slice, at most 6 of
  // this wave's loads in flight (48 KB per CU).  A hand-off read waits behind
  // every load queued chip-wide ahead of it (a whole 256 KB per CU block stream:
  // ~9 us); ~2 us of stream in flight still keeps each CU at its ~25 GB/s.
  auto pace = [&]() {   // pubfirst 3 / 4 / 5: at most 6 / 10 / 14 in flight
    if (a.pubfirst == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (a.pubfirst == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  };
  auto issue_fc1_half = [&](int j, int t, auto hc) {
    constexpr int h = decltype(hc)::value;
    const bf16* g1 = hl_opaque(a.b[j].fc1_w) + (long long)w * ROWS1 * C;
#pragma unroll
    for (int i = 8 * h; i < 8 * h + 8; ++i) {
      hl_dma16<false, true>(w1_s + (i * NTC + 64 * wave) * 8, g1 + ((long long)i * NTC + t) * 8);
      if (i & 1) pace();
    }
  };
  auto issue_fc2_half = [&](int j, int t, auto hc) {
    constexpr int h = decltype(hc)::value;
    const bf16* g2 = hl_opaque(a.b[j].fc2_w) + (long long)(w >> 1) * F * 16 + (w & 1) * 64;
    const int r = t & 7, s = (t >> 3) & 3;
#pragma unroll
    for (int i = 8 * h; i < 8 * h + 8; ++i) {
      const int kc = (i * NTC + t) >> 5;
      w2[i] = hl_ldnt(g2 + (long long)kc * 512 + (16 * s + r) * 8);
      if (i & 1) pace();
    }
  };

  // ---- the conv's history taps of block jb for chunks c = lane + 64 q, q in
  // {q0, q0 + 1} (control wave): XF_MIX's tap order, taps 0..5 summed; the
  // sum and tap 6 parked in LDS for the front half
  auto hist = [&](int jb, int q0) {
    const int lane = hl_vopaque((int)threadIdx.x & 63);
    const bf16* mb = hl_opaque(a.b[jb].mix) + slot * a.b[jb].mix_sB;
    const bf16* dw = hl_opaque(a.b[jb].dw_w);
    bf16x8 hv[2][CTX], wk[2][7];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int c = lane + 64 * (q0 + qq);
#pragma unroll
      for (int r = 0; r < CTX; ++r) hv[qq][r] = hl_ld(mb + (long long)r * C + c * 8);
#pragma unroll
      for (int k = 0; k < 7; ++k) wk[qq][k] = hl_ld(dw + (long long)c * 56 + k * 8);
    }
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int c = lane + 64 * (q0 + qq);
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < CTX; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int f = j * 7 + k;
          acc[j] += bf(wk[qq][f >> 3][f & 7]) * bf(hv[qq][k][j]);
        }
      bf16x8 t6;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = j * 7 + 6;
        t6[j] = wk[qq][f >> 3][f & 7];
      }
      *(f32x4*)(pa_s + c * 8) = (f32x4){acc[0], acc[1], acc[2], acc[3]};
      *(f32x4*)(pa_s + c * 8 + 4) = (f32x4){acc[4], acc[5], acc[6], acc[7]};
      *(bf16x8*)(w6_s + c * 8) = t6;
    }
  };

  // ---- the front half of block j (control wave; chunks c = lane + 64 q):
  // y = x + gamma * dwconv(norm(x)) (workgroup 0 appends norm(x) to the conv
  // buffer), a = ffn_norm(y) -> LDS; this workgroup's 8 columns of y -> LDS
  // (split in two: with pubfirst == 2 the loads go out before the compute waves
  // issue the block's weight stream, so they are not queued behind it)
  bf16x8 xv[4], nw[4], db[4], gm[4], fw[4];
  auto front_load = [&](int j) {
    const int lane = hl_vopaque((int)threadIdx.x & 63);
    const CodecStageBlock& B = a.b[j];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = lane + 64 * q;
      xv[q] = j == 0 ? hl_ld(a.x + c * 8) : MemWT::ld16(hl_opaque(a.xe) + c * 8);   // this launch's rows: sc1
      nw[q] = hl_ld(B.norm + c * 8);
      db[q] = hl_ld(B.dw_b + c * 8);
      gm[q] = hl_ld(B.gamma + c * 8);
      fw[q] = hl_ld(B.ffn_norm + c * 8);
    }
  };
  auto front = [&](int j) {
    const int lane = hl_vopaque((int)threadIdx.x & 63);
    const CodecStageBlock& B = a.b[j];
    float ss = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // per-chunk sums, then chunks in ascending order (XF_MIX's)
      float s8 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s8 += bf(xv[q][e]) * bf(xv[q][e]);
      ss += s8;
    }
    const float inv = rsqrtf(wave_sum(ss) / (float)C + a.eps);
    bf16x8 yv[4];
    float ss2 = 0.f;
    bf16* nb = B.mix + slot * B.mix_sB + (long long)a.ctx * C;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = lane + 64 * q;
      bf16x8 nr;
#pragma unroll
      for (int e = 0; e < 8; ++e) nr[e] = tobf(rb(rb(bf(xv[q][e]) * inv) * bf(nw[q][e])));
      if (w == 0) *(bf16x8*)(nb + c * 8) = nr;   // read by the next frame's launch
      const f32x4 p0 = *(const f32x4*)(pa_s + c * 8), p1 = *(const f32x4*)(pa_s + c * 8 + 4);
      const bf16x8 t6 = *(const bf16x8*)(w6_s + c * 8);
      float acc[8] = {p0[0], p0[1], p0[2], p0[3], p1[0], p1[1], p1[2], p1[3]};
      float s8 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[e] += bf(t6[e]) * bf(nr[e]);
        yv[q][e] = tobf(bf(xv[q][e]) + rb(rb(acc[e] + bf(db[q][e])) * bf(gm[q][e])));
        s8 += bf(yv[q][e]) * bf(yv[q][e]);
      }
      ss2 += s8;
      if (c == w) *(bf16x8*)y_s = yv[q];
    }
    const float inv2 = rsqrtf(wave_sum(ss2) / (float)C + a.eps);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = lane + 64 * q;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = tobf(rb(rb(bf(yv[q][e]) * inv2) * bf(fw[q][e])));
      *(bf16x8*)(a_s + c * 8) = o;
    }
  };

  // The two roles run separate loops (so the compute waves' 64 weight registers
  // are not live in the control wave's code) with the same barriers B1 .. B6.
  if (ctl) {
    const int lane = threadIdx.x & 63;
    // arrival (behind this wave's own stores), `between` while the grid gathers,
    // then the poll; false: a wait gave up
    auto grid_wait = [&](auto between) -> bool {
      ++nwait;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) hl_arrive(a.sync, w);
      between();
      if (lane == 0) ok_s[0] = hl_poll(a.sync, g0, nwait, a.err) ? 1u : 0u;
      __syncthreads();
      return ok_s[0] != 0;
    };
    hist(0, 0);
    hist(0, 2);
    for (int j = 0; j < a.depth; ++j) {
      const bool last = j + 1 == a.depth;
      stamp(8 * j + 0, true);
      front_load(j);
      if (j > 0 && a.pubfirst == 2) __syncthreads();   // B0: these loads ahead of the block's stream
      front(j);
      __syncthreads();   // B1: fc1's input row in LDS
      stamp(8 * j + 1, true);
      __syncthreads();   // B2: the compute waves' fc1 partials in LDS
      stamp(8 * j + 3, true);
      if (lane < ROWS1 / 4) {   // 4 hidden units per lane, epi_row8's EPI_GELU
        const bf16x4 b1 = *(const bf16x4*)(a.b[j].fc1_b + ROWS1 * w + 4 * lane);
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int u = 4 * lane + e;
          float sacc = 0.f;
#pragma unroll
          for (int v = 0; v < NTC / 64; ++v) sacc += red[v * ROWS1 + u];
          o[e] = tobf(gelu_f(rb(sacc + bf(b1[e]))));
        }
        MemWT::st8(hl_opaque(a.h) + ROWS1 * w + 4 * lane, o);
      }
      if (!grid_wait([&] {
            if (!last) {   // (here, not in the next wait: that one runs behind the next block's stream)
              hist(j + 1, 0);
              hist(j + 1, 2);
            }
          }))
        return;   // B3
      stamp(8 * j + 4, true);
      {
        const bf16* hp = hl_opaque(a.h) + hl_vopaque(lane) * 8;   // (per-lane addresses not hoisted)
#pragma unroll
        for (int i = 0; i < F / 8 / 64; ++i) hl_dma16<true>(h_s + i * 512, hp + i * 512);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();   // B4: the hidden row in LDS
      stamp(8 * j + 5, true);
      __syncthreads();   // B5: the compute waves' fc2 partials in LDS
      stamp(8 * j + 6, true);
      if (lane < ROWS2) {   // epi_row8's EPI_RES with ffn_gamma
        const int col = ROWS2 * w + lane;
        float sacc = 0.f;
#pragma unroll
        for (int v = 0; v < NTC / 64; ++v) sacc += red[v * ROWS2 + lane];
        const float yv = rb(bf(a.b[j].ffn_gamma[col]) * rb(sacc + bf(a.b[j].fc2_b[col])));
        const bf16 o = tobf(bf(y_s[lane]) + yv);
        if (last) rm_bfw(a.out, 0)[col] = o;   // the launch's end publishes it
        else MemWT::st2(a.xe + col, o);
      }
      if (!last && a.pubfirst) {
        // the output and the arrival go out ahead of the next block's stream
        // (behind it they waited up to its whole length), then B5b releases the
        // compute waves to issue it; the poll follows
        ++nwait;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) hl_arrive(a.sync, w);
        __syncthreads();   // B5b
        if (lane == 0) ok_s[0] = hl_poll(a.sync, g0, nwait, a.err) ? 1u : 0u;
        __syncthreads();   // B6
        if (!ok_s[0]) return;
      } else if (!last && !grid_wait([] {})) return;   // B6
      stamp(8 * j + 7, true);
    }
  } else if (a.pubfirst >= 3) {
    // paced: block j's fc1 slice in two halves (during the previous block's
    // second wait and this block's front half), its fc2 slice in two halves
    // (during the first wait and the hidden-row DMA); barriers as below
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    issue_fc1(0, threadIdx.x);
    for (int j = 0; j < a.depth; ++j) {
      const bool last = j + 1 == a.depth;
      if (j > 0) issue_fc1_half(j, hl_vopaque((int)threadIdx.x), H1());
      __syncthreads();   // B1
      {   // fc1: row (t & 15) of tiles 2w / 2w + 1 over this thread's 16 chunks
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's fc1 DMA
        stamp(8 * j + 2, false);
        const int t = hl_vopaque((int)threadIdx.x), s = (t & 63) >> 4;
        float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          const int kc = (8 * i + wave) & 63;
          const bf16x8 wv = *(const bf16x8*)(w1_s + (i * NTC + t) * 8);
          const bf16x8 av = *(const bf16x8*)(a_s + kc * 32 + 8 * s);
          if (i < CPT / 2) acc0 = hl_dot8(wv, av, acc0);
          else acc1 = hl_dot8(wv, av, acc1);
        }
        acc0 = cs_rows_sum(acc0);
        acc1 = cs_rows_sum(acc1);
        if ((t & 63) < 16) {
          red[wave * ROWS1 + (t & 15)] = acc0;
          red[wave * ROWS1 + 16 + (t & 15)] = acc1;
        }
      }
      __syncthreads();   // B2
      issue_fc2_half(j, hl_vopaque((int)threadIdx.x), H0());
      __syncthreads();   // B3
      if (!ok_s[0]) return;
      issue_fc2_half(j, hl_vopaque((int)threadIdx.x), H1());
      __syncthreads();   // B4
      {   // fc2: row (t & 7) of the half tile over this thread's 16 chunks
        const int t = hl_vopaque((int)threadIdx.x), s = (t >> 3) & 3;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          const int kc = (i * NTC + t) >> 5;
          acc = hl_dot8(w2[i], *(const bf16x8*)(h_s + kc * 32 + 8 * s), acc);
        }
        acc += __shfl_xor(acc, 8);
        acc += __shfl_xor(acc, 16);
        acc += __shfl_xor(acc, 32);
        if ((t & 63) < ROWS2) red[wave * ROWS2 + (t & 63)] = acc;
      }
      __syncthreads();   // B5
      if (!last) {
        __syncthreads();   // B5b: the control wave's output and arrival issued
        issue_fc1_half(j + 1, hl_vopaque((int)threadIdx.x), H0());
        __syncthreads();   // B6
        if (!ok_s[0]) return;
      }
    }
  } else {
    issue_fc1(0, threadIdx.x);
    issue_fc2(0, threadIdx.x);
    for (int j = 0; j < a.depth; ++j) {
      const bool last = j + 1 == a.depth;
      if (j > 0 && a.pubfirst == 2) {   // B0: the control wave's front-half loads issued; then this block's stream
        __syncthreads();
        issue_fc1(j, hl_vopaque((int)threadIdx.x));
        issue_fc2(j, hl_vopaque((int)threadIdx.x));
      }
      __syncthreads();   // B1
      {   // fc1: row (t & 15) of tiles 2w / 2w + 1 over this thread's 16 chunks
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // this wave's fc1 DMA (the fc2 loads may fly)
        stamp(8 * j + 2, false);
        const int t = hl_vopaque((int)threadIdx.x), s = (t & 63) >> 4;
        float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          const int kc = (8 * i + wave) & 63;
          const bf16x8 wv = *(const bf16x8*)(w1_s + (i * NTC + t) * 8);
          const bf16x8 av = *(const bf16x8*)(a_s + kc * 32 + 8 * s);
          if (i < CPT / 2) acc0 = hl_dot8(wv, av, acc0);
          else acc1 = hl_dot8(wv, av, acc1);
        }
        acc0 = cs_rows_sum(acc0);
        acc1 = cs_rows_sum(acc1);
        if ((t & 63) < 16) {
          red[wave * ROWS1 + (t & 15)] = acc0;
          red[wave * ROWS1 + 16 + (t & 15)] = acc1;
        }
      }
      __syncthreads();   // B2
      __syncthreads();   // B3
      if (!ok_s[0]) return;
      __syncthreads();   // B4
      {   // fc2: row (t & 7) of the half tile over this thread's 16 chunks
        const int t = hl_vopaque((int)threadIdx.x), s = (t >> 3) & 3;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          const int kc = (i * NTC + t) >> 5;
          acc = hl_dot8(w2[i], *(const bf16x8*)(h_s + kc * 32 + 8 * s), acc);
        }
        acc += __shfl_xor(acc, 8);
        acc += __shfl_xor(acc, 16);
        acc += __shfl_xor(acc, 32);
        if ((t & 63) < ROWS2) red[wave * ROWS2 + (t & 63)] = acc;
      }
      __syncthreads();   // B5
      if (!last) {
        if (a.pubfirst) __syncthreads();   // B5b: the control wave's output and arrival issued
        if (a.pubfirst != 2) {
          // the next block's slices: fc1 into this wave's own LDS chunks (read by
          // no other wave), then fc2 into the registers
          issue_fc1(j + 1, hl_vopaque((int)threadIdx.x));
          issue_fc2(j + 1, hl_vopaque((int)threadIdx.x));
        }
        __syncthreads();   // B6
        if (!ok_s[0]) return;
      }
    }
  }
}

// ============================================================================
// C = 1,024 stages (the acoustic decoder's second, T = 8; the semantic
// encoder's sixth, T = 2), M = T rows of one sample.  Per workgroup and block:
// fc1 one MFMA tile (hidden units [16w, 16w + 16), 32 KB, LDS DMA), fc2 a
// quarter tile (output columns [4w, 4w + 4), 32 KB, registers: 4 chunks per
// compute thread); 64 KB per CU per block.  The front half (XF_MIX's, over T
// rows: the conv runs across the new rows and the 6 history rows) is staged in
// LDS and computed by all nine waves (the compute waves touch no global memory
// but their weights, so their vmcnt queue stays clean); the control wave DMAs
// the rows in, prefetches the next block's history rows and vectors during the
// first wait, and does every store.
namespace cs2 {
constexpr int C = 1024, F = 4 * C, G = pk::G, CTX = 6, K7 = 7;
constexpr int NTC = 512, NT = NTC + 64;
constexpr int NCH = C / 8;                   // 128 chunks per row
constexpr int CPT = 4;                       // weight chunks per compute thread per GEMV
constexpr int ROWS1 = F / G, ROWS2 = C / G;  // 16 / 4
static_assert(ROWS1 * C / 8 == CPT * NTC && ROWS2 * F / 8 == CPT * NTC, "codec stage (C = 1,024) geometry");
template <int M>
struct Lds {
  static constexpr int W1 = 0, W1_B = ROWS1 * C * 2;                          // fc1 slice, 32 KB
  static constexpr int XS_B = M * C * 2, AS_B = M * C * 2, H_B = M * F * 2;
  static constexpr int HR = W1 + W1_B, HR_B = H_B > XS_B + AS_B ? H_B : XS_B + AS_B;   // hidden rows | x / y + a rows
  static constexpr int NRM = HR + HR_B, NRM_B = (CTX + M) * C * 2;            // conv input rows
  static constexpr int VEC = NRM + NRM_B, VEC_B = 4 * C * 2 + C * K7 * 2;     // norm, dw_b, gamma, ffn_norm; dw_w
  static constexpr int SSP = VEC + VEC_B, SSP_B = M * NCH * 4;                // per-chunk sums of squares
  static constexpr int RED = SSP + SSP_B, RED_B = 8 * M * ROWS1 * 4;          // compute-wave partials
  static constexpr int SM = RED + RED_B, SM_B = (4 + 2 * M + M * ROWS2) * 4;  // ok, inv / inv2, y of the own columns
  static constexpr int TOTAL = SM + SM_B;
  static_assert(TOTAL <= 160 * 1024, "one workgroup per CU");
};
}  // namespace cs2

template <int M>
__global__ void __launch_bounds__(cs2::NT) k_codec_stage_s(CodecStageArgs a) {
  using namespace cs2;
  using LL = Lds<M>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* w1_s = (bf16*)(smem + LL::W1);
  bf16* h_s = (bf16*)(smem + LL::HR);          // fc2 phase: [M][F]
  bf16* x_s = (bf16*)(smem + LL::HR);          // front half: [M][C] x, then y
  bf16* a_s = x_s + M * C;                     // [M][C] fc1 input
  bf16* nrm_s = (bf16*)(smem + LL::NRM);       // [CTX + M][C]
  bf16* vec_s = (bf16*)(smem + LL::VEC);       // norm | dw_b | gamma | ffn_norm, each [C]; dw_w [C][7]
  float* ssp = (float*)(smem + LL::SSP);       // [M][NCH]
  float* red = (float*)(smem + LL::RED);
  float* sm = (float*)(smem + LL::SM);
  unsigned* ok_s = (unsigned*)sm;
  float* inv_s = sm + 4;                       // [M]
  float* inv2_s = inv_s + M;                   // [M]
  bf16* y4_s = (bf16*)(inv2_s + M);            // [M][4] y of this workgroup's columns

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool ctl = wave == NTC / 64;
  const int w = blockIdx.x, lane = threadIdx.x & 63;
  const long long slot = a.slots[0];
  unsigned g0 = 0, nwait = 0;
  if (ctl) __builtin_amdgcn_s_setprio(3);
  if (ctl) g0 = __hip_atomic_load((hl_gu32*)hl_gen(a.sync), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & ~7u;
  auto stamp = [&](int k, bool by_ctl) {   // k_codec_stage's slots (tools/codec_stage_stamps.py)
    if (a.stamps && threadIdx.x == (by_ctl ? NTC : 0)) a.stamps[w * 64 + k] = __builtin_amdgcn_s_memrealtime();
  };

  // ---- weights (compute waves): fc1 tile w by DMA (chunk g = i * NTC + t ->
  // LDS 16 g), fc2 quarter tile into registers (lane l of wave v, load i: row
  // l >> 4 of the quarter, k-sub (l >> 2) & 3, k-block 32 i + 4 v + (l & 3): a
  // wave's load covers 16 full 64-byte runs, and a row's lanes are one 16-lane
  // group, summed by DPP)
  bf16x8 w2[CPT];
  auto issue = [&](int j, int t) {
    const bf16* g1 = hl_opaque(a.b[j].fc1_w) + (long long)w * ROWS1 * C;
#pragma unroll
    for (int i = 0; i < CPT; ++i)
      hl_dma16<false, true>(w1_s + (i * NTC + 64 * wave) * 8, g1 + ((long long)i * NTC + t) * 8);
    const bf16* g2 = hl_opaque(a.b[j].fc2_w) + (long long)(w >> 2) * F * 16 + (w & 3) * 32;
    const int l = t & 63, r = l >> 4, s = (l >> 2) & 3, kk = l & 3;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int kc = 32 * i + 4 * wave + kk;
      w2[i] = hl_ldnt(g2 + (long long)kc * 512 + (16 * s + r) * 8);
    }
  };
  // ---- control wave: block jb's history rows -> nrm_s[0 .. CTX), its vectors -> vec_s (LDS DMA)
  auto prefetch = [&](int jb) {
    const int ln = hl_vopaque(lane);
    const bf16* mb = hl_opaque(a.b[jb].mix) + slot * a.b[jb].mix_sB;
#pragma unroll
    for (int i = 0; i < CTX * NCH / 64; ++i) hl_dma16<false>(nrm_s + i * 512, mb + (i * 64 + ln) * 8);
    const bf16* v4[4] = {hl_opaque(a.b[jb].norm), hl_opaque(a.b[jb].dw_b), hl_opaque(a.b[jb].gamma),
                         hl_opaque(a.b[jb].ffn_norm)};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < NCH / 64; ++i) hl_dma16<false>(vec_s + q * C + i * 512, v4[q] + (i * 64 + ln) * 8);
    // the depthwise taps transposed to [7][C] (so a chunk's taps are 7 conflict-free
    // 16-byte LDS reads): column chunks ln, ln + 64 of [C][7], 7 x 16 B each
    const bf16* dw = hl_opaque(a.b[jb].dw_w);
#pragma unroll
    for (int cc = 0; cc < NCH / 64; ++cc) {
      const int c = ln + 64 * cc;
      bf16x8 wk[K7];
#pragma unroll
      for (int k = 0; k < K7; ++k) wk[k] = hl_ld(dw + (long long)c * 56 + k * 8);
#pragma unroll
      for (int k = 0; k < K7; ++k) {
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int f = q * 7 + k;
          o[q] = wk[f >> 3][f & 7];
        }
        *(bf16x8*)(vec_s + 4 * C + k * C + c * 8) = o;
      }
    }
  };
  // every thread: per-chunk sums of squares of rows src (XF_MIX's per-chunk order) -> ssp
  auto chunk_ss = [&](const bf16* src) {
    for (int e = hl_vopaque((int)threadIdx.x); e < M * NCH; e += NT) {
      const bf16x8 v = *(const bf16x8*)(src + e * 8);
      float s8 = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s8 += bf(v[k]) * bf(v[k]);
      ssp[e] = s8;
    }
  };
  // one wave per row: chunks lane, lane + 64 in order, wave_sum (XF_MIX's row order)
  auto row_inv = [&](float* dst) {
    const int ln = hl_vopaque(lane);
    for (int m = wave; m < M; m += NT / 64) {
      float ss = 0.f;
      for (int c = ln; c < NCH; c += 64) ss += ssp[m * NCH + c];
      ss = wave_sum(ss);
      if (lane == 0) dst[m] = rsqrtf(ss / (float)C + a.eps);
    }
  };
  auto grid_wait = [&](auto between) -> bool {
    ++nwait;
    if (ctl) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) hl_arrive(a.sync, w);
      between();
      if (lane == 0) ok_s[0] = hl_poll(a.sync, g0, nwait, a.err) ? 1u : 0u;
    }
    __syncthreads();
    return ok_s[0] != 0;
  };

  if (!ctl) issue(0, threadIdx.x);
  if (ctl) prefetch(0);
  // pubfirst >= 3: block j + 1's weights (64 KB per CU) issued after the second
  // wait, under the front half, instead of ahead of the output and the wait
  const bool late = a.pubfirst >= 3;
  for (int j = 0; j < a.depth; ++j) {
    const bool last = j + 1 == a.depth;
    stamp(8 * j + 0, true);
    if (late && j > 0 && !ctl) issue(j, hl_vopaque((int)threadIdx.x));
    // ================= front half over the M rows (all waves, from LDS)
    if (ctl) {   // the block's input rows (this launch's: sc1)
      const int ln = hl_vopaque(lane);
      const bf16* src = j == 0 ? hl_opaque(a.x) : hl_opaque(a.xe);
#pragma unroll
      for (int i = 0; i < M * NCH / 64; ++i) {
        if (j == 0) hl_dma16<false>(x_s + i * 512, src + (i * 64 + ln) * 8);
        else hl_dma16<true>(x_s + i * 512, src + (i * 64 + ln) * 8);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(40 + 4 * j, true);
    }
    __syncthreads();
    chunk_ss(x_s);
    __syncthreads();
    row_inv(inv_s);
    __syncthreads();
    stamp(41 + 4 * j, true);
    for (int e = hl_vopaque((int)threadIdx.x); e < M * NCH; e += NT) {   // mixer norm -> the conv input rows
      const int m = e / NCH, c = e - m * NCH;
      const bf16x8 v = *(const bf16x8*)(x_s + e * 8), nw = *(const bf16x8*)(vec_s + c * 8);
      const float rr = inv_s[m];
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = tobf(rb(rb(bf(v[k]) * rr) * bf(nw[k])));
      *(bf16x8*)(nrm_s + (CTX + m) * C + c * 8) = o;
    }
    __syncthreads();
    if (ctl && w == 0) {   // workgroup 0 appends the new conv-input rows to the block's buffer
      bf16* nb = hl_opaque(a.b[j].mix) + slot * a.b[j].mix_sB + (long long)a.ctx * C;
      for (int e = hl_vopaque(lane); e < M * NCH; e += 64) *(bf16x8*)(nb + e * 8) = *(const bf16x8*)(nrm_s + CTX * C + e * 8);
    }
    // depthwise conv + gamma residual: y over x.  Thread (chunk c, row group):
    // the 8 channels [8c, 8c + 8) of RPT consecutive rows, so the 7 taps and the
    // window's input rows are converted once for RPT rows (one element per
    // thread converted every tap for every element: 3.3 us per block, VALU-bound
    // in all 256 workgroups).  Each output still sums its taps k = 0 .. 6 in order.
    constexpr int RPT = M >= 4 ? 4 : M;
    for (int e = hl_vopaque((int)threadIdx.x); e < NCH * (M / RPT); e += NT) {
      const int c = e % NCH, m0 = RPT * (e / NCH);
      float wt[K7][8];
#pragma unroll
      for (int k = 0; k < K7; ++k) {
        const bf16x8 wk = *(const bf16x8*)(vec_s + 4 * C + k * C + c * 8);   // tap k of the chunk's 8 columns
#pragma unroll
        for (int q = 0; q < 8; ++q) wt[k][q] = bf(wk[q]);
      }
      float acc[RPT][8];
#pragma unroll
      for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[i][q] = 0.f;
#pragma unroll
      for (int r = 0; r < RPT + K7 - 1; ++r) {   // window row m0 + r: tap r - i of output row m0 + i
        const bf16x8 v = *(const bf16x8*)(nrm_s + (m0 + r) * C + c * 8);
        float vf[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) vf[q] = bf(v[q]);
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
          const int k = r - i;
          if (k >= 0 && k < K7) {
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[i][q] += wt[k][q] * vf[q];
          }
        }
      }
      const bf16x8 bb = *(const bf16x8*)(vec_s + C + c * 8), gv = *(const bf16x8*)(vec_s + 2 * C + c * 8);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int ei = (m0 + i) * NCH + c;
        const bf16x8 xv = *(const bf16x8*)(x_s + ei * 8);
        bf16x8 y8;
        float s8 = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          y8[q] = tobf(bf(xv[q]) + rb(rb(acc[i][q] + bf(bb[q])) * bf(gv[q])));
          s8 += bf(y8[q]) * bf(y8[q]);
        }
        *(bf16x8*)(x_s + ei * 8) = y8;
        ssp[ei] = s8;
      }
    }
    __syncthreads();
    stamp(42 + 4 * j, true);
    row_inv(inv2_s);
    __syncthreads();
    stamp(43 + 4 * j, true);
    for (int e = hl_vopaque((int)threadIdx.x); e < M * NCH; e += NT) {   // FFN pre-norm -> fc1's input rows
      const int m = e / NCH, c = e - m * NCH;
      const bf16x8 y8 = *(const bf16x8*)(x_s + e * 8), fw = *(const bf16x8*)(vec_s + 3 * C + c * 8);
      const float rr = inv2_s[m];
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = tobf(rb(rb(bf(y8[k]) * rr) * bf(fw[k])));
      *(bf16x8*)(a_s + e * 8) = o;
    }
    if (threadIdx.x < M * ROWS2) {   // y of this workgroup's 4 columns, for the fc2 epilogue
      const int tt = hl_vopaque((int)threadIdx.x), m = tt / ROWS2, r = tt - m * ROWS2;
      y4_s[tt] = x_s[m * C + ROWS2 * w + r];
    }
    __syncthreads();   // B1
    stamp(8 * j + 1, true);
    // ================= fc1: M rows x 16 hidden units
    if (!ctl) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // this wave's fc1 DMA (the fc2 loads may fly)
      stamp(8 * j + 2, false);
      const int t = hl_vopaque((int)threadIdx.x), s = (t & 63) >> 4;
      float acc[M];
#pragma unroll
      for (int m = 0; m < M; ++m) acc[m] = 0.f;
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int kc = 8 * i + wave;
        const bf16x8 wv = *(const bf16x8*)(w1_s + (i * NTC + t) * 8);
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m] = hl_dot8(wv, *(const bf16x8*)(a_s + m * C + kc * 32 + 8 * s), acc[m]);
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        acc[m] = cs_rows_sum(acc[m]);
        if ((t & 63) < 16) red[(wave * M + m) * ROWS1 + (t & 15)] = acc[m];
      }
    }
    __syncthreads();   // B2
    stamp(8 * j + 3, true);
    if (ctl && lane < M * ROWS1 / 4) {   // 4 hidden units per lane, epi_row8's EPI_GELU
      const int ln = hl_vopaque(lane), m = ln / (ROWS1 / 4), u0 = 4 * (ln - m * (ROWS1 / 4));
      const bf16x4 b1 = *(const bf16x4*)(a.b[j].fc1_b + ROWS1 * w + u0);
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float sacc = 0.f;
#pragma unroll
        for (int v = 0; v < NTC / 64; ++v) sacc += red[(v * M + m) * ROWS1 + u0 + e];
        o[e] = tobf(gelu_f(rb(sacc + bf(b1[e]))));
      }
      MemWT::st8(hl_opaque(a.h) + (long long)m * F + ROWS1 * w + u0, o);
    }
    if (!grid_wait([&] { if (ctl && !last) prefetch(j + 1); })) return;   // B3
    stamp(8 * j + 4, true);
    // ================= fc2: M rows x 4 columns over the whole hidden rows
    if (ctl) {
      const bf16* hp = hl_opaque(a.h) + hl_vopaque(lane) * 8;
#pragma unroll
      for (int i = 0; i < M * F / 8 / 64; ++i) hl_dma16<true>(h_s + i * 512, hp + i * 512);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();   // B4
    stamp(8 * j + 5, true);
    if (!ctl) {
      const int l = hl_vopaque((int)threadIdx.x & 63), s = (l >> 2) & 3, kk = l & 3;
      float acc[M];
#pragma unroll
      for (int m = 0; m < M; ++m) acc[m] = 0.f;
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const int kc = 32 * i + 4 * wave + kk;
#pragma unroll
        for (int m = 0; m < M; ++m) acc[m] = hl_dot8(w2[i], *(const bf16x8*)(h_s + m * F + kc * 32 + 8 * s), acc[m]);
      }
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float v = group_sum<16>(acc[m]);
        if ((l & 15) == 0) red[(wave * M + m) * ROWS2 + (l >> 4)] = v;
      }
    }
    __syncthreads();   // B5
    stamp(8 * j + 6, true);
    if (!late && !ctl && !last) issue(j + 1, hl_vopaque((int)threadIdx.x));
    if (ctl && lane < M * ROWS2) {   // epi_row8's EPI_RES with ffn_gamma
      const int ln = hl_vopaque(lane), m = ln / ROWS2, r = ln - m * ROWS2, col = ROWS2 * w + r;
      float sacc = 0.f;
#pragma unroll
      for (int v = 0; v < NTC / 64; ++v) sacc += red[(v * M + m) * ROWS2 + r];
      const float yv = rb(bf(a.b[j].ffn_gamma[col]) * rb(sacc + bf(a.b[j].fc2_b[col])));
      const bf16 o = tobf(bf(y4_s[ln]) + yv);
      if (last) rm_bfw(a.out, m)[col] = o;
      else MemWT::st2(hl_opaque(a.xe) + (long long)m * C + col, o);
    }
    if (!last && !grid_wait([] {})) return;   // B6
    stamp(8 * j + 7, true);
  }
}

// One workgroup per CU, all resident from the start: the plain launch checks
// nothing, so each build is checked here (kernels.h persist_resident).
bool persist_resident_kernel(const void* k, int nt, int lds, int grid) {
  hipFuncAttributes fa{};
  int nb = 0, dev = 0, cus = 0;
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess ||
      hipFuncGetAttributes(&fa, k) != hipSuccess || hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, nt, lds) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  return persist_resident(nb, cus, (long long)fa.localSizeBytes, grid);
}
static bool stage_resident(int C, int M) {
  static const bool ok2048 = persist_resident_kernel((const void*)k_codec_stage, cs::NT, cs::TOTAL, cs::G);
  static const bool ok1024_2 = persist_resident_kernel((const void*)k_codec_stage_s<2>, cs2::NT, cs2::Lds<2>::TOTAL, cs2::G);
  static const bool ok1024_8 = persist_resident_kernel((const void*)k_codec_stage_s<8>, cs2::NT, cs2::Lds<8>::TOTAL, cs2::G);
  if (C == cs::C && M == 1) return ok2048;
  if (C == cs2::C && M == 2) return ok1024_2;
  if (C == cs2::C && M == 8) return ok1024_8;
  return false;
}

bool codec_stage_fits(int C, int T, int n, int depth) {
  return n == 1 && depth >= 1 && depth <= 8 && stage_resident(C, T);
}

int launch_codec_stage(const CodecStageArgs& a, hipStream_t st) {
  if (!stage_resident(a.C, a.M)) return 3;
  if (a.C == cs::C) hipLaunchKernelGGL(k_codec_stage, dim3(cs::G), dim3(cs::NT), cs::TOTAL, st, a);
  else if (a.M == 2) hipLaunchKernelGGL((k_codec_stage_s<2>), dim3(cs2::G), dim3(cs2::NT), cs2::Lds<2>::TOTAL, st, a);
  else hipLaunchKernelGGL((k_codec_stage_s<8>), dim3(cs2::G), dim3(cs2::NT), cs2::Lds<8>::TOTAL, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
