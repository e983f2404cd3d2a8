// Persistent GEMV chains: a sequence of dependent decode GEMVs (M <= 16 rows)
// in ONE launch of one workgroup per CU.
//
// Why (DESIGN.md "Persistent chains"): at B = 1 the diffusion head is 10 steps x
// 10 dependent GEMVs per token and the LM 28 x 5 launches.  Each launch pays a
// kernel boundary, a ramp in which its weight stream has not started, the
// A rows' dependent round trip and an epilogue tail with no loads in flight
// (time ~ 5.2 us + bytes / 6.4 TB/s per GEMV).  Here every workgroup walks the
// op list, and the weights of its NEXT unit -- of the same op or of the next one
// -- are already in flight while it reduces, stores, signals and waits for the
// next op's inputs (MI355X_MICROARCH.md "prefetch-credit").
//
// Work split: op j's 16-row weight tiles are cut into units; unit u runs on
// workgroup u % G.  Tiles [0, t1) are whole-tile units of tpw tiles (kw waves
// per tile split K, tpw * kw <= 8); tiles [t1, N/16) are split ks2 ways along
// K (kw2 waves each) with a write-through fp32 slab per split and a ticket: the
// last arriver sums the slabs in split order and runs the epilogue.
//
// Hand-offs (MI355X_MICROARCH.md "Valid forms", hand-off table row 1): every
// byte another workgroup reads in this launch is stored write-through (sc1) and
// loaded with sc1 loads (gemv_dev.h MemWT); each storing wave drains vmcnt(0),
// the workgroup barrier follows, then ONE lane adds the tiles it finished to
// done[j].  The first unit of op j on a workgroup waits (one lane polls done[j-1]
// relaxed, s_sleep between polls, bounded) until op j-1 has all its tiles.
// Completion is transitive (op j-1's units waited for op j-2), so one counter
// orders every earlier producer.  done[] and the tickets are zeroed by a memset
// node before every launch (cdna_hip_programming.md Guideline 16: re-initialise
// every call).
//
// Arithmetic is k_gemv1's (gemm.hip) term for term: same A staging and
// transform order, same per-wave K ranges for a given (kw, ksplit), same wave
// and split summation order, same epilogues.  With the per-op launch plan
// mirrored (vv_chain_tune(2)) the chain is bit-identical to the per-op kernels;
// the default plan re-splits K to balance the 256 CUs.
#include <atomic>
#include <cstdio>
#include <vector>

#include "gemv_dev.h"

// waves per workgroup and workgroups per CU: one 8-wave workgroup per CU (two
// 4-wave workgroups per CU measured slower, DESIGN.md "Persistent chains")
constexpr int CH_NW = 8, CH_WGPC = 1;

// global (address_space 1) loads: a flat load also counts in lgkmcnt, so every
// LDS wait would wait for the weight stream in flight
typedef __attribute__((address_space(1))) const bf16x8 gbf16x8;
DEV bf16x8 gld16(const bf16* p) { return *(gbf16x8*)p; }
DEV bf16x8 ldw_rt(const bf16* p, int keep) {
  return keep ? *(gbf16x8*)p : __builtin_nontemporal_load((gbf16x8*)p);
}

// A unit of op `op`: tiles [tile0, tile0 + ntl), split ks of nks, kw waves per tile
struct UnitGeo {
  int tile0, ntl, ks, nks, kw;
};
DEV UnitGeo unit_geo(const ChainOp& op, int u) {
  UnitGeo q;
  if (u < op.nu1) {
    q.tile0 = u * op.tpw;
    q.ntl = min(op.tpw, op.t1 - q.tile0);
    q.ks = 0;
    q.nks = 1;
    q.kw = op.kw;
  } else {
    const int v = u - op.nu1;
    q.tile0 = op.t1 + v / op.ks2;
    q.ntl = 1;
    q.ks = v - (v / op.ks2) * op.ks2;
    q.nks = op.ks2;
    q.kw = op.kw2;
  }
  return q;
}

// this wave's weight stream for a unit: packed rows of its tile, chunks [c0, c1)
struct WaveGeo {
  const bf16* wrow;
  int c0, c1, keep;
};
DEV WaveGeo wave_geo(const ChainOp& op, int u, int wave, int lane) {
  const GemmArgs& a = op.g;
  const UnitGeo q = unit_geo(op, u);
  const int tw = wave / q.kw, kwv = wave - tw * q.kw;
  const int tile = q.tile0 + tw;
  const bool ok = tw < q.ntl;
  const int nchunk = a.K >> 5;
  const int b0 = (int)((long long)nchunk * q.ks / q.nks), b1 = (int)((long long)nchunk * (q.ks + 1) / q.nks);
  WaveGeo w;
  w.c0 = b0 + (int)((long long)(b1 - b0) * kwv / q.kw);
  w.c1 = ok ? b0 + (int)((long long)(b1 - b0) * (kwv + 1) / q.kw) : w.c0;
  w.wrow = a.w + (long long)(ok ? tile : 0) * a.K * 16 + lane * 8;
  w.keep = a.keep;
  return w;
}

// U loads, unconditional (chunks past the range re-read the last one: a
// guarded load leaves hipcc no static vmcnt count, and it then drains every
// batch with vmcnt(0))
template <int U>
DEV void issue(bf16x8 (&wf)[U], const WaveGeo& w, int c) {
  const int last = max(w.c1 - 1, 0);
  if (w.keep) {
#pragma unroll
    for (int i = 0; i < U; ++i) wf[i] = *(gbf16x8*)(w.wrow + (long long)min(c + i, last) * 512);
  } else {
#pragma unroll
    for (int i = 0; i < U; ++i) wf[i] = __builtin_nontemporal_load((gbf16x8*)(w.wrow + (long long)min(c + i, last) * 512));
  }
}

DEV void advance(const ChainArgs& A, int& j, int& u) {
  while (j < A.nops && u >= A.ops[j].nunit) {
    ++j;
    u = blockIdx.x;
  }
}

// A rows [0, M) x chunks [b0, b1) of the unit's split, transformed, into LDS
// (k_gemv1's staging paths and arithmetic; every load is an sc1 load).
template <int XF>
DEV void stage_a(const GemmArgs& a, const RowMap& am, int b0, int b1, int nks, int fast_nt, bf16* xs, float* part,
                 float* inv_s) {
  using MP = MemWT;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, NW = CH_NW;
  const int kw = (b1 - b0) * 32, lds_ld = kw + 8, n8 = kw >> 3;
  constexpr int Q = 4;
  if (a.M * n8 <= Q * fast_nt) {   // k_gemv1's fast path (fast_nt <= blockDim.x: every item covered)
    bf16x8 xv[Q], wv[Q], sh[Q], sc[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = threadIdx.x + q * blockDim.x;
      if (e < a.M * n8) {
        const int m = e / n8, k = b0 * 32 + (e - m * n8) * 8;
        xv[q] = MP::ld16(rm_bf(am, m) + k);
        if (XF == XF_NORM) {
          if (a.xf.w) wv[q] = gld16(a.xf.w + k);
          if (a.xf.mod) {
            const bf16* md = a.xf.mod + (long long)m * a.xf.mod_ld;
            sh[q] = gld16(md + a.xf.shift_off + k);
            sc[q] = gld16(md + a.xf.scale_off + k);
          }
        } else if (XF == XF_SILU_ADD) {
          wv[q] = gld16(a.xf.vec + k);
        }
      }
    }
    if (XF == XF_NORM) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int e = threadIdx.x + q * blockDim.x;
        if (e < a.M * n8) {
          float ss = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) ss += bf(xv[q][j]) * bf(xv[q][j]);
          part[e] = ss;
        }
      }
      __syncthreads();
      if (nks == 1) {
        for (int m = wave; m < a.M; m += NW) {
          float ss = 0.f;
          for (int c = lane; c < n8; c += 64) ss += part[m * n8 + c];
          ss = wave_sum(ss);
          if (lane == 0) inv_s[m] = rsqrtf(ss / (float)a.K + a.xf.eps);
        }
      } else {
        row_inv<MP>(am, a.M, a.K, a.xf.eps, 0, a.M, inv_s, wave, NW, lane);
      }
      __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int e = threadIdx.x + q * blockDim.x;
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
    for (int e0 = threadIdx.x; e0 < a.M * n8; e0 += 4 * blockDim.x) {
      bf16x8 xv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = e0 + q * blockDim.x;
        if (e < a.M * n8) {
          const int m = e / n8, k8 = (e - m * n8) * 8;
          xv[q] = MP::ld16(rm_bf(am, m) + b0 * 32 + k8);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = e0 + q * blockDim.x;
        if (e < a.M * n8) {
          const int m = e / n8, k8 = (e - m * n8) * 8;
          *(bf16x8*)(xs + m * lds_ld + k8) = xv[q];
        }
      }
    }
    if (XF != XF_NONE) {
      __syncthreads();
      if (XF == XF_NORM) {
        if (nks == 1) {
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
          row_inv<MP>(am, a.M, a.K, a.xf.eps, 0, a.M, inv_s, wave, NW, lane);
        }
        __syncthreads();
      }
      for (int e = threadIdx.x; e < a.M * n8; e += blockDim.x) {
        const int m = e / n8, k8 = (e - m * n8) * 8;
        bf16x8* px = (bf16x8*)(xs + m * lds_ld + k8);
        *px = xform<XF, MP>(a, *px, m, b0 * 32 + k8, XF == XF_NORM ? inv_s[m] : 0.f);
      }
    }
  }
  __syncthreads();
}

// done[] layout: per op j, 8 shard counters (workgroups w with w % 8 == s, i.e.
// one XCD's under round-robin placement) and one top counter, each on its own
// 128-byte line.  A workgroup adds 1 to its shard after its last unit of op j;
// the shard's last arriver (told by the returned value) adds 1 to the top.
// (MI355X_MICROARCH.md "fanin": one counter serialises ~12 ns per arrival.)
constexpr int CH_LINE = 32;          // words per counter line
DEV unsigned* shard_ctr(const ChainArgs& A, int j, int s) { return A.done + ((long long)j * 9 + s) * CH_LINE; }
DEV int op_wgs(const ChainArgs& A, int j) { return min(A.ops[j].nunit, (int)gridDim.x); }

DEV void signal_done(const ChainArgs& A, int j) {
  const int nwg = op_wgs(A, j), s = blockIdx.x & 7;
  const unsigned cnt = (unsigned)(nwg / 8 + (s < nwg % 8 ? 1 : 0));
  typedef __attribute__((address_space(1))) unsigned gu32;
  const unsigned v = __hip_atomic_fetch_add((gu32*)shard_ctr(A, j, s), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (v == cnt - 1) __hip_atomic_fetch_add((gu32*)shard_ctr(A, j, 8), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bounded wait for op j's top counter: one lane polls (relaxed sc1 loads,
// s_sleep between), the workgroup barrier releases the others.  Returns false
// after ~200 ms (the error word is set; the launch then drains).
DEV bool wait_done(const ChainArgs& A, int j, unsigned* abort_s) {
  if (threadIdx.x == 0) {
    const unsigned tgt = (unsigned)min(8, op_wgs(A, j));
    typedef __attribute__((address_space(1))) unsigned gu32;
    gu32* top = (gu32*)shard_ctr(A, j, 8);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned ab = 0;
    while (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tgt) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
        __hip_atomic_store((gu32*)A.err, 1u + (unsigned)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ab = 1;
        break;
      }
    }
    *abort_s = ab;
  }
  __syncthreads();
  return *abort_s == 0;
}

DEV void chain_stamp(const ChainArgs& A, int j, int which) {
  if (A.stamps && threadIdx.x == 0)
    A.stamps[((long long)blockIdx.x * A.nops + j) * 4 + which] = __builtin_amdgcn_s_memrealtime();
}

template <int U>
__global__ void __launch_bounds__(64 * CH_NW) k_chain(ChainArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float inv_s[16];
  __shared__ float red[CH_NW * 256];
  __shared__ unsigned last_flag, abort_s;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int G = gridDim.x;
  const bf16x8 zero8 = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};

  int j = 0, u = blockIdx.x;
  advance(A, j, u);
  if (j >= A.nops) return;
  WaveGeo cur = wave_geo(A.ops[j], u, wave, lane);
  bf16x8 wa[U], wb[U];
  issue<U>(wa, cur, cur.c0);
  int staged = -1;
  int prev_j = -1;
  while (j < A.nops) {
    const ChainOp& op = A.ops[j];
    const GemmArgs& a = op.g;
    const UnitGeo q = unit_geo(op, u);
    int jn = j, un = u + G;
    advance(A, jn, un);
    WaveGeo nx;
    if (jn < A.nops) nx = wave_geo(A.ops[jn], un, wave, lane);
    // inputs of op j: op j - 1 complete (its units waited for theirs)
    if (j != prev_j) {
      chain_stamp(A, j, 0);
      if (j > 0 && !wait_done(A, j - 1, &abort_s)) return;
      chain_stamp(A, j, 1);
    }
    prev_j = j;

    RowMap am = a.a;
    if (op.bind & CH_BIND_AX) am.base = A.x;
    const int nchunk = a.K >> 5;
    const int b0 = (int)((long long)nchunk * q.ks / q.nks), b1 = (int)((long long)nchunk * (q.ks + 1) / q.nks);
    const int lds_ld = (b1 - b0) * 32 + 8;
    bf16* xs = (bf16*)smem;
    float* part = (float*)(smem + (((size_t)a.M * lds_ld * 2 + 15) & ~(size_t)15));
    const int key = (j * 64 + q.nks) * 64 + q.ks;   // the staged slice: op, split count, split
    if (key != staged) {
      switch (op.xf) {
        case XF_NORM: stage_a<XF_NORM>(a, am, b0, b1, q.nks, op.fast, xs, part, inv_s); break;
        case XF_SILU_ADD: stage_a<XF_SILU_ADD>(a, am, b0, b1, q.nks, op.fast, xs, part, inv_s); break;
        default: stage_a<XF_NONE>(a, am, b0, b1, q.nks, op.fast, xs, part, inv_s); break;
      }
      staged = key;
    }

    // weight stream (wa already in flight); the last batch's slot takes the next unit's chunks
    f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
    const bf16* xrow = xs + min(r, a.M - 1) * lds_ld + 8 * g - b0 * 32;
    const int c1 = cur.c1;
    auto compute = [&](bf16x8 (&wf)[U], int c) {
      bf16x8 x[U];
#pragma unroll
      for (int i = 0; i < U; ++i) x[i] = *(const bf16x8*)(xrow + min(c + i, c1 - 1) * 32);
#pragma unroll
      for (int i = 0; i < U; ++i) {
        const bf16x8 w = c + i < c1 ? wf[i] : zero8;
        acc = mfma(w, x[i], acc);
      }
    };
    bool pre = false;
    for (int c = cur.c0; c < c1; c += 2 * U) {
      issue<U>(wb, cur, c + U);
      compute(wa, c);
      if (c + 2 * U < c1) {
        issue<U>(wa, cur, c + 2 * U);
      } else if (jn < A.nops) {
        issue<U>(wa, nx, nx.c0);
        pre = true;
      }
      if (c + U < c1) compute(wb, c + U);
    }
    if (!pre && jn < A.nops) issue<U>(wa, nx, nx.c0);

    // reduce the tile's K-slice waves (tile tw's sum lands in slab tw * kw)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(wave * 4 + i) * 64 + lane] = acc[i];
    __syncthreads();
    const int KW = q.kw;
    if (KW > 1) {
      for (int e = threadIdx.x; e < q.ntl * 256; e += blockDim.x) {
        const int base = (e >> 8) * KW * 256 + (e & 255);
        float s = 0.f;
        for (int w2 = 1; w2 < KW; ++w2) s += red[base + w2 * 256];
        red[base] += s;
      }
      __syncthreads();
    }
    bool epi = true;
    if (q.nks > 1) {   // split: write-through slab, ticket, the last arriver sums in split order
      float* slab = A.slabs + op.slab_off + ((long long)(q.tile0 - op.t1) * q.nks + q.ks) * 256;
      for (int e = threadIdx.x; e < 256; e += blockDim.x) MemWT::stf(slab + e, red[e]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned* tk = A.tickets + op.ticket_off + (q.tile0 - op.t1);
        const unsigned v = __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)tk, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
        last_flag = v == (unsigned)(q.nks - 1) ? 1u : 0u;
      }
      __syncthreads();
      epi = last_flag != 0;
      if (epi) {
        const float* slabs = A.slabs + op.slab_off + (long long)(q.tile0 - op.t1) * q.nks * 256;
        for (int e = threadIdx.x; e < 256; e += blockDim.x) {
          float s = 0.f;
          for (int k = 0; k < q.nks; ++k) s += MemWT::ldf(slabs + k * 256 + e);
          red[e] = s;
        }
        __syncthreads();
      }
    }
    if (epi && wave < q.ntl) {
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = red[wave * KW * 256 + i * 64 + lane];
      const int n0 = (q.tile0 + wave) * 16;
      if (op.bind & CH_BIND_DPM) {   // per-call latent / noise / CFG scale, per-step coefficients
        DpmEpi P = a.dpm;
        P.x = A.x;
        P.noise = A.noise ? A.noise + (long long)op.rep * A.noise_rep : nullptr;
        P.k = A.coef[op.rep];
        P.k.cfg = A.cfg;
        epi_dpm<MemWT>(a, P, n0, lane, v);
      } else {
        epi_tile<MemWT>(a, r, n0, lane, v);
      }
    }
    if (jn != j) {   // last unit of op j here: every storing wave drains, the barrier, one arrival
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) signal_done(A, j);
      chain_stamp(A, j, 2);
    } else {
      __syncthreads();   // red[] is rewritten by the next unit
    }
    j = jn;
    u = un;
    cur = nx;
  }
}

// ------------------------------------------------------------------ host
// Plan one op (fills the split fields of *op from op->g).  mode 1: the per-op
// launch plan (gemv_plan_query), bit-identical to gemm.hip's kernels; mode 0:
// the balanced plan.  Returns the op's dynamic LDS bytes, or 0 if the op cannot
// run in a chain.
size_t chain_plan_op(ChainOp* op, int G, int mode) {
  const GemmArgs& a = op->g;
  if (a.M < 1 || a.M > 16 || a.K % 32 || a.N % 16 || a.xf.kind == XF_MIX) return 0;
  if (a.epi.kind == EPI_CFG_DPM && 2 * a.dpm.n != a.M) return 0;
  const int T = a.N / 16, C = a.K / 32;
  int t1, tpw, kw, ks2, kw2, fast;
  if (mode == 1) {
    int nw, ks, tp;
    if (gemv_plan_query(a, &nw, &ks, &tp, &fast)) return 0;
    if (nw > CH_NW) return 0;   // the per-op plan's workgroup is wider than the chain's
    if (ks > 1) {
      t1 = 0;
      tpw = 1;
      kw = nw;
      ks2 = ks;
      kw2 = nw;
    } else {
      t1 = T;
      tpw = CH_NW / nw;   // the launch's workgroups side by side: same per-tile wave split
      if (tp > 1) tpw = tp;   // tiles-per-workgroup plans already use all 8 waves
      kw = nw / (tp > 1 ? tp : 1);
      if (tpw * kw > CH_NW) return 0;
      ks2 = 1;
      kw2 = nw;
    }
  } else {
    // one unit per workgroup (units run one after another inside a workgroup,
    // so a second round doubles an op's span): T >= G -> units of tpw =
    // ceil(T / G) whole tiles, kw = 8 / tpw waves each; T < G -> whole tiles,
    // or each tile split ks2 ways along K when the chunks saved per workgroup
    // outweigh a hand-off (~40 chunks of stream, tools/chain_bench.py timelines)
    if (T >= G) {
      tpw = (T + G - 1) / G;
      if (tpw > CH_NW) return 0;
      kw = CH_NW / tpw;
      kw2 = kw;
      t1 = T;
      ks2 = 1;
    } else {
      tpw = 1;
      kw = CH_NW;
      kw2 = CH_NW;
      ks2 = 1;
      long best = C;
      for (int s = 2; s <= 16 && s <= C && T * s <= G; s *= 2) {
        const long cost = (C + s - 1) / s + 40;
        if (cost < best) {
          best = cost;
          ks2 = s;
        }
      }
      t1 = ks2 > 1 ? 0 : T;
    }
    fast = 64 * CH_NW;
    if (ks2 > 1 && T - t1 > CH_TMAX) return 0;
  }
  op->xf = a.xf.kind;
  op->t1 = t1;
  op->tpw = tpw;
  op->kw = kw;
  op->ks2 = ks2;
  op->kw2 = kw2;
  op->fast = fast;
  op->nu1 = (t1 + tpw - 1) / tpw;
  op->nunit = op->nu1 + (T - t1) * ks2;
  op->target = T;
  // LDS: the widest staged A slice (+ per-item sums of squares for XF_NORM)
  size_t lds = 0;
  for (int s : {1, ks2}) {
    const size_t kwe = (size_t)((C + s - 1) / s + 1) * 32;
    size_t l = (((size_t)a.M * (kwe + 8) * 2 + 15) & ~(size_t)15);
    if (a.xf.kind == XF_NORM) l += (size_t)a.M * (kwe / 8) * 4;
    if (l > lds) lds = l;
  }
  return lds;
}

int chain_grid() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  return cus * CH_WGPC;
}

static std::atomic<int> g_chain_u{8};   // weight chunks per wave per batch (diagnostic hook vv_chain_tune_u)
extern "C" int vv_chain_tune_u(int u) {
  g_chain_u = u == 4 ? 4 : 8;
  return 0;
}

int launch_chain(const ChainArgs& A, size_t lds, hipStream_t st) {
  constexpr size_t LDS_MAX = 151552;
  if (lds > LDS_MAX) return 1;
  static const bool attr =   // once (thread-safe static init)
      hipFuncSetAttribute((const void*)k_chain<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX) ==
          hipSuccess &&
      hipFuncSetAttribute((const void*)k_chain<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX) ==
          hipSuccess;
  if (!attr) return 2;
  const int G = chain_grid();
  if (G <= 0) return 2;
  if (g_chain_u == 4) hipLaunchKernelGGL(k_chain<4>, dim3(G), dim3(64 * CH_NW), lds, st, A);
  else hipLaunchKernelGGL(k_chain<8>, dim3(G), dim3(64 * CH_NW), lds, st, A);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
