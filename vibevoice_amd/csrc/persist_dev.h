// Device helpers of the persistent kernels (head_loop.hip, codec_stage.hip): one
// workgroup per CU (G = 256), a control wave doing the hand-offs, grid-wide waits
// on XCD-sharded counters.
#pragma once
#include "gemv_dev.h"

#pragma clang diagnostic ignored "-Winline-asm"

namespace pk {
constexpr int G = 256;              // workgroups of a persistent launch (one per CU)
constexpr int LINE = 32;            // words per counter line
}  // namespace pk

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const bf16x8 hl_gbf16x8;
typedef __attribute__((address_space(1))) unsigned hl_gu32;
DEV bf16x8 hl_ld(const bf16* p) { return *(hl_gbf16x8*)p; }
// a weight-stream load: global (a flat load would also count in lgkmcnt, so every
// LDS wait would drain the stream) and non-temporal (gemv_dev.h ldw)
DEV bf16x8 hl_ldnt(const bf16* p) { return __builtin_nontemporal_load((hl_gbf16x8*)p); }

DEV float hl_dot8(bf16x8 w, bf16x8 x, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 0, 1), __builtin_shufflevector(x, x, 0, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 2, 3), __builtin_shufflevector(x, x, 2, 3), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 4, 5), __builtin_shufflevector(x, x, 4, 5), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(w, w, 6, 7), __builtin_shufflevector(x, x, 6, 7), acc, false);
  return acc;
}

// 16-byte LDS DMA (global_load_lds_dwordx4): lane l's 16 bytes from gptr land at
// lds_base + 16 l (lds_base wave-uniform).  Inline asm, so hipcc neither drains
// the queue before the first LDS access nor counts it: the issuing wave waits
// with an explicit s_waitcnt vmcnt.  SC1: the bytes were written in this launch
// (write-through stores, MI355X_MICROARCH.md's hand-off table: sc1 loads).
// NT: a weight stream read once per token (no reuse before eviction: the
// non-temporal policy keeps it from evicting what does stay in the caches).
template <bool SC1, bool NT = false>
DEV void hl_dma16(const void* lds_base, const void* gptr) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(
      (unsigned)(unsigned long long)(__attribute__((address_space(3))) const unsigned char*)lds_base);
  if (NT)
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off nt" ::"s"(lds), "v"(gptr) : "memory", "m0");
  else if (SC1)
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off sc1" ::"s"(lds), "v"(gptr) : "memory", "m0");
  else
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds), "v"(gptr) : "memory", "m0");
}

// A kernel-argument pointer re-read inside a loop: hipcc would otherwise hoist
// every per-lane address derived from it out of the step / layer loops and keep
// dozens of them live (VGPR spills); through this opaque copy they are recomputed
// where used (a few VALU each).
template <class T>
DEV T* hl_opaque(T* p) {
  asm volatile("" : "+s"(p));
  return p;
}
DEV int hl_vopaque(int v) {   // the same for a per-lane value
  asm volatile("" : "+v"(v));
  return v;
}

// element (row j, column k) of an MFMA-packed [N][K] weight (weights.py mfma_pack):
// the 16-byte chunk holding columns k .. k+7 (k % 8 == 0)
DEV const bf16* hl_packed(const bf16* w, int K, int j, int k) {
  return w + ((long long)((j >> 4) * (K >> 5) + (k >> 5)) * 64 + (j & 15) + 16 * ((k & 31) >> 3)) * 8;
}

// One grid-wide wait: arrival of this workgroup + poll until k waits of this
// launch have completed.  Control wave, lane 0, behind the control wave's own
// s_waitcnt vmcnt(0) (it made every store this workgroup publishes).  The
// arrival adds to this workgroup's XCD shard counter (w % 8: 32 workgroups
// each); a shard's 32nd arrival of a wait bumps this kernel's generation word,
// so one wait completes when the generation has advanced by 8.  Two chained
// device-scope atomics before the release (round 4's k_head_ffn chained three:
// shard -> top -> generation).  Measured against (DESIGN.md "Persistent head"):
// polling all 256 per-workgroup flags (2x slower: 256 pollers sweeping the same
// lines) and polling the 8 shard counters without the generation word (one
// atomic per wait, but 8 lines per poll: 755 -> 774 us per head sample).
// Counters are monotonic across launches and compared wrap-safe.
//
// The launch's base generation: only this kernel bumps its word (line 11; the
// shard counters are shared with k_head_ffn, 256 workgroups and 32 arrivals per
// shard per wait in both), 8 per wait, so it is a multiple of 8 between
// launches.  A workgroup reading it at entry may see up to 7 bumps of the first
// wait (other shards complete it; its own cannot): base = word rounded down to 8.
DEV unsigned* hl_gen(unsigned* sync) { return sync + 11 * pk::LINE; }

// arrival of workgroup w (lane 0 of the control wave)
DEV void hl_arrive(unsigned* sync, int w) {
  using namespace pk;
  const unsigned v = __hip_atomic_fetch_add((hl_gu32*)(sync + (w & 7) * LINE), 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
  if ((v + 1) % (G / 8) == 0) __hip_atomic_fetch_add((hl_gu32*)hl_gen(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// poll the generation word until it has advanced by 8 k from g0; false: gave up
// after ~200 ms (error word set).  (A/B builds, tools/ab_lib.sh: two polls in
// flight half a round trip apart, or s_sleep 4 between polls: B = 1 within
// +-0.01 ms of this one-at-a-time loop.)
DEV bool hl_poll_word(unsigned* gen, unsigned g0, unsigned k, unsigned* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((unsigned)(__hip_atomic_load((hl_gu32*)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - g0) < 8 * k) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // ~200 ms at 100 MHz
      __hip_atomic_store((hl_gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}
// poll until k waits of this launch (base generation g0) have completed; false:
// gave up after ~200 ms (error word set)
DEV bool hl_poll(unsigned* sync, unsigned g0, unsigned k, unsigned* err) {
  return hl_poll_word(hl_gen(sync), g0, k, err);
}
DEV bool hl_grid_wait(unsigned* sync, unsigned g0, unsigned k, int w, unsigned* err) {
  hl_arrive(sync, w);
  return hl_poll(sync, g0, k, err);
}

// the arrival half of hl_grid_wait_gen (lane 0 of a wave, behind that wave's vmcnt(0))
DEV void hl_arrive_gen(unsigned* sync, int gen_line, int w) {
  using namespace pk;
  const unsigned v = __hip_atomic_fetch_add((hl_gu32*)(sync + (w & 7) * LINE), 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
  if ((v + 1) % (G / 8) == 0)
    __hip_atomic_fetch_add((hl_gu32*)(sync + gen_line * LINE), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the poll half: until k waits of this launch (base g0) completed; false: gave up
// after ~200 ms (error word set).  (Polling by scalar loads that miss the scalar
// cache was tried: the hand-offs took 11-20 us instead of 1.4-3.)
DEV bool hl_poll_gen(unsigned* sync, int gen_line, unsigned g0, unsigned k, unsigned* err) {
  return hl_poll_word(sync + gen_line * pk::LINE, g0, k, err);
}

// the same wait on the generation word at line `gen_line` of `sync` (a kernel of
// its own: only it bumps that word, 8 per wait; the shard lines are shared)
DEV bool hl_grid_wait_gen(unsigned* sync, int gen_line, unsigned g0, unsigned k, int w, unsigned* err) {
  using namespace pk;
  unsigned* gen = sync + gen_line * LINE;
  const unsigned v = __hip_atomic_fetch_add((hl_gu32*)(sync + (w & 7) * LINE), 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
  if ((v + 1) % (G / 8) == 0) __hip_atomic_fetch_add((hl_gu32*)gen, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return hl_poll_word(gen, g0, k, err);
}
