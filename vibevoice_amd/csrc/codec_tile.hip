// A whole narrow codec stage (C = 128 / 64 / 32: the acoustic decoder's last
// three stages, the semantic / acoustic encoders' first three) in ONE launch per
// stage: the transition conv that feeds it (decoder ConvTranspose r = 2,
// encoder strided conv r = 2, or the encoder's 1 -> 32 stem), its three Block1Ds
// (modular_vibevoice_tokenizer.py:620-684) and, for the decoder's last stage,
// the C -> 1 head conv (:908-920) -- streaming form (:914-951), one frame of
// T rows per sample.
//
// Decomposition: workgroup (x, sample) owns output rows [t0, t0 + R) of the
// stage and RECOMPUTES its causal halo instead of exchanging it: a k = 7
// depthwise conv needs 6 rows before its output, so block j's output is computed
// over rows [t0 - E - 6 (2 - j), B) and the stage input over [t0 - E - 18, B)
// (E = 6 when the head conv follows).  Rows t < 0 come from the per-slot conv
// histories (ConvBuf rows 0..ctx-1); nothing another workgroup writes is read, so
// the launch has no inter-workgroup dependency at all (any residency, any n).
// Everything between the stage's input rows and its output rows stays in LDS.
//
// Per block: mixer RMSNorm -> depthwise conv + bias -> gamma residual -> FFN
// RMSNorm (one 16-byte chunk per thread, a row's chunks in one lane group so the
// row sums are DPP reductions in registers) -> fc1 (MFMA 16x16x32, weights in
// registers, hidden rows + GELU into LDS) -> fc2 (MFMA) -> ffn_gamma residual.
// The arithmetic is k_block's / k_mix's term for term (codec_block.hip) except
// the GELU: erf by a 5-term rational approximation (gelu_fast, |error| <= 1.5e-7
// before the bf16 rounding of the output) instead of ocml's erff, whose two
// branch paths made fc1 + GELU ~8 us of a C = 128 block (tools/codec_tile_stamps.py).
// The transition GEMM sums its 32-wide K chunks in order in one fp32 accumulator
// (EPI_STORE's rounding); the head conv is k_conv_cout1's order.
//
// Weight stream (8 waves, weights shared by every workgroup through L2): each
// wave holds its fragments of one GEMM in registers; block j+1's fc1 fragments
// (and its per-channel vectors / history rows) are issued right after block j's
// fc1 products, its fc2 fragments after block j's fc2 products, so every weight
// fragment has a whole phase to arrive.  All loads are branch-free (clamped
// addresses) so hipcc's vmcnt accounting stays exact in the unrolled code.
#include "kernels.h"

namespace ct {
constexpr int NTH = 512, NW = 8;   // 8 waves
template <int C, int R_>
struct Geo {
  static constexpr int R = R_;                   // output rows per workgroup (16, or 2048 / C for many samples)
  static constexpr int N8 = C / 8;               // 16-byte chunks per row
  static constexpr int RPP = NTH / N8;           // rows per elementwise pass
  static constexpr int F = 4 * C;
  static constexpr int XLD = C + 8, HLD = F + 8; // LDS row strides (+16 B against bank conflicts)
  static constexpr int NLP = (R + 24 + 15) / 16 * 16;   // local rows (halo 18 + head 6), padded to tiles
  static constexpr int NT1 = F / 16, NK1 = C / 32, NT2 = C / 16, NK2 = F / 32;
  // LDS carve-up (bytes)
  static constexpr int X = 0, X_B = NLP * XLD * 2;                    // block input / output rows
  static constexpr int Y = X + X_B, Y_B = NLP * XLD * 2;              // mixer residual y
  static constexpr int NRM = Y + Y_B, NRM_B = (NLP + 6) * XLD * 2;    // conv input rows (6 before row L0)
  // (+16 rows: a block's row tiles start at its first output row, so the last one may run 15 rows past NLP)
  static constexpr int A = NRM + NRM_B, A_B = (NLP + 16) * XLD * 2;   // fc1 input rows
  static constexpr int H = A + A_B, H_B = (NLP + 16) * HLD * 2;       // hidden rows (transition input first)
  static constexpr int TOTAL = H + H_B;
  static_assert(TOTAL <= 160 * 1024, "one workgroup per CU at most");
  static_assert(NTH % N8 == 0 && 64 % N8 == 0, "a row's chunks in one lane group");
};
// a GEMM of NT 16-row weight tiles over 8 waves: NTW tiles per wave, row tiles strided by RS
template <int NT>
struct Split {
  static constexpr int NTW = NT >= NW ? NT / NW : 1;
  static constexpr int RS = NT >= NW ? 1 : NW / NT;
};
}  // namespace ct

template <int K>
DEV void ct_load_frags(bf16x8 (&f)[K], const bf16* w, int nk, int t0, int lane) {
  // K fragments: tile t0 + i / nk, chunk i % nk (MFMA-packed 1 KB blocks)
#pragma unroll
  for (int i = 0; i < K; ++i) f[i] = *(const bf16x8*)(w + ((long long)(t0 + i / nk) * nk + i % nk) * 512 + lane * 8);
}

template <int C, int PRE, int POST, int R>
__global__ void __launch_bounds__(ct::NTH, 1) k_codec_tile(CodecTileArgs a) {
  using G = ct::Geo<C, R>;
  using namespace ct;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* xs = (bf16*)(smem + G::X);
  bf16* ys = (bf16*)(smem + G::Y);
  bf16* ns = (bf16*)(smem + G::NRM);
  bf16* as = (bf16*)(smem + G::A);
  bf16* hs = (bf16*)(smem + G::H);
  bf16* ps = hs;   // transition input rows (dead before the first fc1)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int smp = blockIdx.y;
  const long long slot = a.slots[smp];
  const int T = a.T;
  const int t0 = blockIdx.x * G::R;
  const int B = min(t0 + G::R, T);
  constexpr int E = POST == CT_POST_HEAD ? 6 : 0;
  const int L0 = t0 - E - 18;                   // local row 0 (may be negative)
  const int S_lo = max(0, L0);                  // first stage-input row computed
  const int c2 = tid % G::N8, rp = tid / G::N8; // this thread's chunk, row-in-pass
  const bool last_tile = B == T;
  // diagnostics (tools/codec_tile_stamps.py): 0 start, 1 input rows in LDS, 2 transition done,
  // per block j 3 + 4j mixer norm, 4 + 4j conv / FFN norm, 5 + 4j fc1, 6 + 4j fc2; 15 end
  auto stamp = [&](int k) {
    if (a.stamps && tid == 0)
      a.stamps[((long long)blockIdx.y * gridDim.x + blockIdx.x) * 16 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---------------------------------------------------------------- input rows
  // PRE none: the stage input rows; convT: transition buffer rows [S_lo / 2,
  // B / 2 + 1) (1 history row first); sconv: buffer rows [2 S_lo, 2 B + 2) (2
  // history rows); stem: audio samples [S_lo, B + 6) (6 history samples).
  constexpr int CI = PRE == CT_PRE_CONVT ? 2 * C : PRE == CT_PRE_SCONV ? C / 2 : C;
  constexpr int CI8 = CI / 8, PLD = CI + 8;
  constexpr int PROWS = PRE == CT_PRE_CONVT ? G::NLP / 2 + 1 : PRE == CT_PRE_SCONV ? 2 * G::NLP + 2 : G::NLP;
  constexpr int QIN = PRE == CT_PRE_STEM ? 1 : (PROWS * CI8 + NTH - 1) / NTH;
  const int p_lo = PRE == CT_PRE_CONVT ? S_lo / 2 : PRE == CT_PRE_SCONV ? 2 * S_lo : S_lo;
  const int p_hi = PRE == CT_PRE_CONVT ? B / 2 + 1 : PRE == CT_PRE_SCONV ? 2 * B + 2 : B;   // exclusive
  bf16x8 vin[QIN];
  bf16 sin1 = (bf16)0.f;
  if (PRE == CT_PRE_STEM) {
    const int i = min(tid, B + 6 - S_lo - 1);
    sin1 = a.pre_buf[slot * a.pre_sB + S_lo + i];   // buffer element S_lo + i = sample S_lo + i - 6
  } else {
#pragma unroll
    for (int q = 0; q < QIN; ++q) {
      const int e = min(tid + q * NTH, (p_hi - p_lo) * CI8 - 1);
      const int i = e / CI8, c = e - i * CI8;
      const bf16* src = PRE == CT_PRE_NONE ? a.x + ((long long)smp * T + p_lo + i) * C + c * 8
                                           : a.pre_buf + slot * a.pre_sB + (long long)(p_lo + i) * CI + c * 8;
      vin[q] = *(const bf16x8*)src;
    }
  }

  // ---------------------------------------------------------------- per-block operands
  struct Aux {   // one set in registers: block j+1's overwrites block j's once its mixer and fc1 are done
    bf16x8 wn, bb, gv, wf, wk[7], hv;
    bf16x4 b1[ct::Split<G::NT1>::NTW];
  };
  using S1 = ct::Split<G::NT1>;
  using S2 = ct::Split<G::NT2>;
  const int nt1 = wave * S1::NTW;                               // fc1: tiles nt1 .. + NTW, every row tile
  const int nt2 = G::NT2 >= NW ? wave : wave % G::NT2;          // fc2: one tile, row tiles strided by RS
  const int rs2 = G::NT2 >= NW ? 0 : wave / G::NT2;
  auto load_aux = [&](int j, Aux& x) {
    const CodecTileBlock& b = a.b[j];
    x.wn = *(const bf16x8*)(b.norm + c2 * 8);
    x.bb = *(const bf16x8*)(b.dw_b + c2 * 8);
    x.gv = *(const bf16x8*)(b.gamma + c2 * 8);
    x.wf = *(const bf16x8*)(b.ffn_norm + c2 * 8);
#pragma unroll
    for (int k = 0; k < 7; ++k) x.wk[k] = *(const bf16x8*)(b.dw_w + (size_t)c2 * 56 + k * 8);
    const int h = min(tid / G::N8, 5);   // history row h (threads >= 6 * N8 load a copy of row 5)
    x.hv = *(const bf16x8*)(b.mix + slot * b.mix_sB + (long long)h * C + c2 * 8);
#pragma unroll
    for (int i = 0; i < S1::NTW; ++i) x.b1[i] = *(const bf16x4*)(b.fc1_b + (nt1 + i) * 16 + 4 * g4);
  };
  Aux ax;
  load_aux(0, ax);

  // transition weights: convT N = 2C, K = 4C; sconv N = C, K = 2C
  constexpr int NTP = PRE == CT_PRE_CONVT ? C / 8 : C / 16;
  constexpr int NKP = PRE == CT_PRE_CONVT ? C / 8 : C / 16;
  using SP = ct::Split<NTP>;
  constexpr bool GEMM_PRE = PRE == CT_PRE_CONVT || PRE == CT_PRE_SCONV;
  constexpr int KP = GEMM_PRE ? SP::NTW * NKP : 1;
  const int ntp = NTP >= NW ? wave * SP::NTW : wave % NTP;
  const int rsp = NTP >= NW ? 0 : wave / NTP;
  bf16x8 wp[KP];
  bf16x4 bp[GEMM_PRE ? SP::NTW : 1];
  if (GEMM_PRE) {
    ct_load_frags<KP>(wp, a.pre_w, NKP, ntp, lane);
#pragma unroll
    for (int i = 0; i < SP::NTW; ++i) bp[i] = *(const bf16x4*)(a.pre_b + (ntp + i) * 16 + 4 * g4);
  }
  constexpr int K1 = S1::NTW * G::NK1, K2 = G::NK2;
  bf16x8 w1[K1], w2[K2];
  bf16x4 b2c, g2c;
  auto load_w2 = [&](int j) {   // fc2's fragments + its bias / ffn_gamma for this wave's tile
    ct_load_frags<K2>(w2, a.b[j].fc2_w, G::NK2, nt2, lane);
    b2c = *(const bf16x4*)(a.b[j].fc2_b + nt2 * 16 + 4 * g4);
    g2c = *(const bf16x4*)(a.b[j].ffn_gamma + nt2 * 16 + 4 * g4);
  };
  // C = 128: fc2's 16 fragments go out at the start of each block's fc1 instead
  // (live through the mixer beside fc1's 16 and the block operands they spilled)
  constexpr bool W2_LATE = K2 > 8;
  if (!GEMM_PRE) {   // (with a transition GEMM: after it, so its fragments and these are never live together)
    ct_load_frags<K1>(w1, a.b[0].fc1_w, G::NK1, nt1, lane);
    if (!W2_LATE) load_w2(0);
  }

  // ---------------------------------------------------------------- stage input rows -> X (local row t - L0)
  if (PRE == CT_PRE_STEM) {
    float* sf = (float*)hs;   // samples [S_lo - 6, B) as floats
    if (tid < B + 6 - S_lo) sf[tid] = bf(sin1);
    __syncthreads();
    // k_conv_cin1: acc over k, then + b, 8 channels per item
    for (int e = tid; e < (B - S_lo) * G::N8; e += NTH) {
      const int i = e / G::N8, c = e - i * G::N8;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += bf(a.pre_w[(c * 8 + j) * 7 + k]) * sf[i + k];
        o[j] = tobf(acc + bf(a.pre_b[c * 8 + j]));
      }
      *(bf16x8*)(xs + (S_lo + i - L0) * G::XLD + c * 8) = o;
    }
  } else {
    bf16* dst = PRE == CT_PRE_NONE ? xs : ps;
    const int ld = PRE == CT_PRE_NONE ? G::XLD : PLD;
    const int off = PRE == CT_PRE_NONE ? S_lo - L0 : 0;
#pragma unroll
    for (int q = 0; q < QIN; ++q) {
      const int e = tid + q * NTH;
      if (e < (p_hi - p_lo) * CI8) {
        const int i = e / CI8, c = e - i * CI8;
        *(bf16x8*)(dst + (off + i) * ld + c * 8) = vin[q];
      }
    }
  }
  __syncthreads();
  stamp(1);
  if (GEMM_PRE) {
    // transition GEMM over its rows: convT row u = S_lo / 2 + m reads buffer rows
    // m, m + 1 (local) and yields stage rows 2u, 2u + 1; sconv row S_lo + m reads
    // buffer rows 2m .. 2m + 3
    const int nrow = PRE == CT_PRE_CONVT ? (B - S_lo) / 2 : B - S_lo;
    const int nmt = (nrow + 15) >> 4;
    for (int mt = rsp; mt < nmt; mt += SP::RS) {
#pragma unroll
      for (int i = 0; i < SP::NTW; ++i) {
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
        const int m = mt * 16 + r16;
#pragma unroll
        for (int c = 0; c < NKP; ++c) {
          const int k0 = c * 32;
          const int prow = PRE == CT_PRE_CONVT ? m + k0 / CI : 2 * m + k0 / CI;
          const bf16x8 xv = *(const bf16x8*)(ps + min(prow, PROWS - 1) * PLD + k0 % CI + 8 * g4);
          acc = mfma16(wp[i * NKP + c], xv, acc);
        }
        const int n = (ntp + i) * 16 + 4 * g4;
        if (m < nrow) {
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = tobf(acc[q] + bf(bp[i][q]));
          const int t = PRE == CT_PRE_CONVT ? 2 * (S_lo / 2 + m) + n / C : S_lo + m;
          *(bf16x4*)(xs + (t - L0) * G::XLD + n % C) = o;
        }
      }
    }
    ct_load_frags<K1>(w1, a.b[0].fc1_w, G::NK1, nt1, lane);
    if (!W2_LATE) load_w2(0);
    __syncthreads();
  }
  stamp(2);

  // ---------------------------------------------------------------- the blocks
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const CodecTileBlock& bj = a.b[j];
    const int lo = max(0, L0 + 6 * (j + 1));   // first output row of block j
    const int cs = lo - 6;                       // first conv input row
    // ---- M1: conv input rows = norm(x) (history rows t < 0 from the buffer)
    if (tid < 6 * G::N8) {
      const int t = tid / G::N8 - 6;
      if (t >= cs) *(bf16x8*)(ns + (t - L0 + 6) * G::XLD + c2 * 8) = ax.hv;
    }
    const int r0 = max(cs, 0);
    for (int p = r0; p < B; p += G::RPP) {
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
        if (t >= T - 6) *(bf16x8*)(bj.mix + slot * bj.mix_sB + (long long)(6 + t) * C + c2 * 8) = o8;
      }
    }
    __syncthreads();
    stamp(3 + 4 * j);
    // ---- M2: depthwise conv + gamma residual -> y; FFN norm -> fc1's input rows
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
      if (t < B) {
        *(bf16x8*)(ys + (t - L0) * G::XLD + c2 * 8) = y8;
        *(bf16x8*)(as + (t - L0) * G::XLD + c2 * 8) = o8;
      }
    }
    __syncthreads();
    stamp(4 + 4 * j);
    // row tiles start at the block's first output row (local row lo - L0), not on a
    // 16-row boundary: a block of 28 / 22 / 16 rows takes 2 / 2 / 1 tiles
    const int rb0 = lo - L0, nmt = (B - lo + 15) >> 4;
    // ---- F1: fc1 + bias + GELU -> hidden rows
    {
      if (W2_LATE) load_w2(j);
      for (int mt = 0; mt < nmt; ++mt) {
        const bf16* xrow = as + (rb0 + mt * 16 + r16) * G::XLD + 8 * g4;
#pragma unroll
        for (int i = 0; i < S1::NTW; ++i) {
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int c = 0; c < G::NK1; ++c) acc = mfma16(w1[i * G::NK1 + c], *(const bf16x8*)(xrow + c * 32), acc);
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = tobf(gelu_fast(rb(acc[q] + bf(ax.b1[i][q]))));
          *(bf16x4*)(hs + (rb0 + mt * 16 + r16) * G::HLD + (nt1 + i) * 16 + 4 * g4) = o;
        }
      }
      if (j < 2) {   // block j+1's operands, then its fc1 fragments
        load_aux(j + 1, ax);
        ct_load_frags<K1>(w1, a.b[j + 1].fc1_w, G::NK1, nt1, lane);
      }
      __syncthreads();
      stamp(5 + 4 * j);
      // ---- F2: fc2 + bias, ffn_gamma, + y -> the block output rows (X)
      for (int mt = rs2; mt < nmt; mt += S2::RS) {
        const bf16* hrow = hs + (rb0 + mt * 16 + r16) * G::HLD + 8 * g4;
        f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < G::NK2; ++c) acc = mfma16(w2[c], *(const bf16x8*)(hrow + c * 32), acc);
        const int t = lo + mt * 16 + r16;
        const int n = nt2 * 16 + 4 * g4;
        if (t >= lo && t < B) {
          const bf16x4 yv = *(const bf16x4*)(ys + (t - L0) * G::XLD + n);
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = tobf(bf(yv[q]) + rb(bf(g2c[q]) * rb(acc[q] + bf(b2c[q]))));
          *(bf16x4*)(xs + (t - L0) * G::XLD + n) = o;
          if (j == 2 && POST == CT_POST_NONE && t >= t0) *(bf16x4*)(rm_bfw(a.out, smp * T + t) + n) = o;
        }
      }
      if (j < 2 && !W2_LATE) load_w2(j + 1);
      __syncthreads();
      stamp(6 + 4 * j);
    }
  }

  // ---------------------------------------------------------------- head conv (decoder's last stage)
  if (POST == CT_POST_HEAD) {
    // the head buffer's history rows t in [-6, 0) stand in for block outputs t < 0
    if (tid < 6 * G::N8) {
      const int t = tid / G::N8 - 6;
      if (t >= t0 - 6) {
        const bf16x8 v = *(const bf16x8*)(a.head_buf + slot * a.head_sB + (long long)(t + 6) * C + c2 * 8);
        *(bf16x8*)(xs + (t - L0) * G::XLD + c2 * 8) = v;
      }
    }
    // this frame's last 6 rows -> the head buffer (the next frame's history, k_roll)
    if (last_tile) {
      for (int e = tid; e < 6 * G::N8; e += NTH) {
        const int t = T - 6 + e / G::N8, c = e % G::N8;
        *(bf16x8*)(a.head_buf + slot * a.head_sB + (long long)(6 + t) * C + c * 8) =
            *(const bf16x8*)(xs + (t - L0) * G::XLD + c * 8);
      }
    }
    __syncthreads();
    // k_conv_cout1's order: acc over k, then 8-channel chunks
    for (int t = t0 + tid; t < B; t += NTH) {
      float acc = 0.f;
      for (int k = 0; k < 7; ++k) {
        const bf16* r = xs + (t - 6 + k - L0) * G::XLD;
        const bf16* wk = a.head_w + k * C;
#pragma unroll
        for (int c = 0; c < C; c += 8) {
          const bf16x8 v = *(const bf16x8*)(r + c);
          const bf16x8 wv = *(const bf16x8*)(wk + c);
#pragma unroll
          for (int q = 0; q < 8; ++q) acc += bf(wv[q]) * bf(v[q]);
        }
      }
      const bf16 y = tobf(acc + bf(a.head_b[0]));
      *rm_bfw(a.audio, smp * T + t) = y;
      if (a.audio2.base) *rm_bfw(a.audio2, smp * T + t) = y;
    }
  }
  stamp(15);
}

// ================================================================ host
template <int C, int PRE, int POST, int R>
static int ct_launch(const CodecTileArgs& a, hipStream_t st) {
  using G = ct::Geo<C, R>;
  static const bool attr =
      hipFuncSetAttribute((const void*)k_codec_tile<C, PRE, POST, R>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          G::TOTAL) == hipSuccess;
  if (!attr) return 2;
  hipLaunchKernelGGL((k_codec_tile<C, PRE, POST, R>), dim3((a.T + G::R - 1) / G::R, a.n), dim3(ct::NTH), G::TOTAL,
                     st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
// Rows per workgroup: 16 while the launch fits one wave of workgroups (one per CU:
// the shortest chain, the most CUs); with more samples 2048 / C, so the halo a
// workgroup recomputes is a smaller share of its rows (B = 8 at C = 32: 400
// workgroups of 64 rows instead of 1,600 of 16).
template <int C, int PRE, int POST>
static int ct_pick(const CodecTileArgs& a, hipStream_t st) {
  if ((long long)a.n * ((a.T + 15) / 16) <= 256 || C >= 128) return ct_launch<C, PRE, POST, 16>(a, st);
  return ct_launch<C, PRE, POST, (C >= 128 ? 16 : 2048 / C)>(a, st);
}

bool codec_tile_fits(int C, int pre, int post, int depth, int ctx) {
  if (depth != 3 || ctx != 6) return false;
  switch (C) {
    case 128: return (pre == CT_PRE_NONE || pre == CT_PRE_SCONV) && post == CT_POST_NONE;
    case 64: return (pre == CT_PRE_CONVT || pre == CT_PRE_SCONV) && post == CT_POST_NONE;
    case 32: return (pre == CT_PRE_CONVT && post == CT_POST_HEAD) || (pre == CT_PRE_STEM && post == CT_POST_NONE);
    default: return false;
  }
}

int launch_codec_tile(const CodecTileArgs& a, int C, int pre, int post, hipStream_t st) {
  if (a.n <= 0 || a.T <= 0) return 0;
  if (!codec_tile_fits(C, pre, post, a.depth, 6)) return 1;
  if (pre == CT_PRE_CONVT && a.T % 2) return 1;
  if (C == 128 && pre == CT_PRE_NONE) return ct_pick<128, CT_PRE_NONE, CT_POST_NONE>(a, st);
  if (C == 128) return ct_pick<128, CT_PRE_SCONV, CT_POST_NONE>(a, st);
  if (C == 64 && pre == CT_PRE_CONVT) return ct_pick<64, CT_PRE_CONVT, CT_POST_NONE>(a, st);
  if (C == 64) return ct_pick<64, CT_PRE_SCONV, CT_POST_NONE>(a, st);
  if (C == 32 && pre == CT_PRE_CONVT) return ct_pick<32, CT_PRE_CONVT, CT_POST_HEAD>(a, st);
  return ct_pick<32, CT_PRE_STEM, CT_POST_NONE>(a, st);
}
