// libvibevoice_hip.so — native engine for VibeVoice's generate loop on MI355X.
//
// Owns: borrowed weight pointers, the compacted LM KV cache, per-slot streaming
// conv state of the acoustic decoder and semantic encoder, workspaces, and the
// diffusion schedule.  Every entry point only enqueues kernels on the caller's
// stream (no host sync, no allocation after vv_finalize except the grow-only
// prefill / voice-prompt workspaces).  C ABI: include/vibevoice_hip.h.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/vibevoice_hip_diag.h"
#include "kernels.h"

static thread_local std::string g_err;

#define FAIL(msg)        \
  do {                   \
    g_err = (msg);       \
    return -1;           \
  } while (0)
#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      g_err = std::string(#x) + ": " + hipGetErrorString(e_);                     \
      return -1;                                                                  \
    }                                                                             \
  } while (0)
#define KCHK(x)                                                                   \
  do {                                                                            \
    int r_ = (x);                                                                 \
    if (r_) {                                                                     \
      g_err = std::string("kernel launch rejected (") + std::to_string(r_) + "): " + #x; \
      return -1;                                                                  \
    }                                                                             \
  } while (0)
#define CHK(x)          \
  do {                  \
    if ((x) != 0) return -1; \
  } while (0)

namespace {

struct Weight {
  const void* p = nullptr;
  std::vector<int64_t> shape;
};

// Per-slot conv input buffer: [ctx history rows | rows of this step (+ zero pad)] x C
struct ConvBuf {
  bf16* base = nullptr;
  long long sB = 0;  // elements per slot
  int ctx = 0, T = 0, C = 0, rows = 0;
};

// Bumped whenever a workspace moves: a hipGraph captured earlier bakes the old
// pointers in, so the host drops its graphs when this changes (vv_ws_epoch).
static std::atomic<int> g_ws_epoch{0};
// Contexts per device that may run the one-launch kernels with grid-wide waits
// (k_lm_ffn, k_head_m16, k_codec_stage*: one workgroup per CU).  Two such
// launches from two contexts cannot be resident together, so they run only while
// ONE finalized context of the device is registered; a change of that count bumps
// the epoch, so hosts re-capture graphs that baked in the other path.  Contexts
// of OTHER processes are invisible here: a shared-GPU deployment turns the
// kernels off (VIBEVOICE_PERSISTENT=0 or vv_set_persistent).
static std::mutex g_hl_mu;
static std::map<int, int> g_hl_ctxs;
static void hl_register(int device, int delta) {
  std::lock_guard<std::mutex> lk(g_hl_mu);
  const int before = g_hl_ctxs[device];
  const int after = before + delta;
  g_hl_ctxs[device] = after;
  if ((before == 1) != (after == 1) || (before <= 2) != (after <= 2)) g_ws_epoch.fetch_add(1);
}
static int hl_count(int device) {
  std::lock_guard<std::mutex> lk(g_hl_mu);
  auto it = g_hl_ctxs.find(device);
  return it == g_hl_ctxs.end() ? 0 : it->second;
}

// wait counters + error word of a grid-waiting kernel family (persist_dev.h: 13 lines of 32 words)
static constexpr size_t SYNC_BYTES = 2048;
static constexpr int CW_LINES = 256;   // wide codec stage clusters per C (n x tiles <= 256 by residency)

// Process default for new contexts: VIBEVOICE_PERSISTENT=0 in the environment
// turns the grid-waiting kernels off (e.g. several processes sharing one GPU).
static bool persist_env_default() {
  static const bool on = [] {
    const char* e = getenv("VIBEVOICE_PERSISTENT");
    return !(e && e[0] == '0');
  }();
  return on;
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int ensure(size_t b) {
    if (b <= bytes) return 0;
    if (p) g_ws_epoch.fetch_add(1);
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    if (hipMalloc(&p, b) != hipSuccess) {
      g_err = "hipMalloc failed (" + std::to_string(b) + " bytes)";
      return -1;
    }
    bytes = b;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

// One causal conv stack of the σ-VAE codec (acoustic decoder, or an encoder),
// laid out for `slots` sample slots and `T0` input rows per call.
struct ConvNet {
  bool decoder = true;
  std::string wp;             // weight-name prefix: "dec", "sem", "aenc"
  int nst = 0;
  int depth[VV_MAX_STAGES] = {}, chans[VV_MAX_STAGES] = {}, rat[VV_MAX_STAGES] = {}, T[VV_MAX_STAGES] = {};
  int in_ch = 0, out_ch = 0, T0 = 0, slots = 0, nmax = 0;
  int Tin[VV_MAX_STAGES] = {};  // rows entering the strided conv before stage i (encoder)
  ConvBuf stem, head;
  std::vector<std::vector<ConvBuf>> mix;
  ConvBuf tr[VV_MAX_STAGES];
  DevBuf state;               // all ConvBufs
  DevBuf work;                // X stages + A + F
  bf16* X[VV_MAX_STAGES] = {};
  bf16* Y[VV_MAX_STAGES] = {};   // residual ping-pong partner of X (k_mix output)
  bf16* A = nullptr;
  bf16* F = nullptr;
  std::vector<RollDesc> rolls;
  DevBuf d_rolls;
};

}  // namespace

// diagnostic: attention launches record per-workgroup timestamps (nullptr: off)
static std::atomic<unsigned long long*> g_attn_stamps{nullptr};
extern "C" int vv_attn_stamps(void* buf) {
  g_attn_stamps = (unsigned long long*)buf;
  return 0;
}

struct vv_ctx {
  vv_config cfg;
  int device = 0;
  std::unordered_map<std::string, Weight> w;
  bool finalized = false;
  // LM
  int qkv_n = 0, lm_slots = 0;
  DevBuf kv_k, kv_v;
  KVLayout kv;
  DevBuf lm_ws;  // h, a, qkv, q, att, act
  size_t lm_ws_tokens = 0;
  DevBuf attn_part, attn_cnt;
  DevBuf norm_ws;   // pre-normalised A rows of XF_NORM GEMMs with > 16 rows
  DevBuf valid_ids;
  int n_valid = 0;
  // split-K
  DevBuf splitk_ws, splitk_cnt;
  // diffusion
  int steps = 0;
  std::vector<DpmCoef> coef;
  DevBuf temb, tfreq_tmp;
  DevBuf head_ws;
  // codec
  ConvNet dec, sem, aenc;
  ConvNet senc;     // the semantic encoder laid out for one non-streaming call (vv_semantic_encode)
  DevBuf codec_ws;  // connectors
  DevBuf slot_scratch;
  DevBuf unit_sb;   // bf16 {1, 0}: identity scaling / bias for vv_codec_decode
  // tensor parallelism of the LM (Megatron split, configuration_vibevoice.py:175-183):
  // this engine holds rank tp_rank's shard; the residual stream is all-reduced
  // after o_proj and down_proj
  int tp_rank = 0, tp_size = 1;
  int head_tp = 0;      // 1: the diffusion head's FFN is sharded too (vv_tp_shard_head; head_ffn is local)
  ncclComm_t comm = nullptr;
  DevBuf zero_rows;     // [2 * max_batch][H] zeros: the residual of a sharded head's rank > 0
  // grid-wide waits of the one-launch kernels (persist_dev.h): head_m16.hip's
  // counters (lines 0-7 shards, line 12 its generation) + the error word (line 10)
  DevBuf hf_sync;
  DevBuf lf_sync;   // lm_ffn.hip's wait counters (+ k_lm_ffn16's column-group tickets)
  DevBuf lf_slab;   // k_lm_ffn16's down partials [48][4][16][32] fp32
  DevBuf la_part;   // k_lm_attn's per-unit attention partials (lm_attn_part_floats)
  DevBuf m16_buf;   // head_m16.hip's distributed A side: row partial sums of squares [16][192] f32 + rows [16][H]
  DevBuf cs_sync;          // persistent codec stage (codec_stage.hip): its wait counters
  DevBuf cw_sync;          // wide codec stages (codec_wide.hip): one counter line per cluster, per C
  DevBuf cw_slab, cw_xbuf; // ... their partial slabs and block outputs
  bool persist_ok = true;       // this context may run one-launch (grid-waiting) kernels (vv_set_persistent)
  bool persist_capable = false; // some grid-waiting kernel fits this engine's shapes (vv_finalize)
  bool persist_follow = false;  // unregistered, runs them while exactly one context is registered (vv_set_persistent 2)
  bool hl_registered = false;   // counted in g_hl_ctxs (its device's grid-waiting contexts)
  bool head_gemv = true;        // the head FFN's GEMV layout is bound (head.<l>.gu_w / down_w)
  DevBuf rope_tab;   // [max_ctx][cos 64 | sin 64] bf16 (k_rope_table)
};

// ------------------------------------------------------------------ helpers
static const bf16* W(vv_ctx* c, const std::string& n) {
  auto it = c->w.find(n);
  if (it == c->w.end()) return nullptr;
  return (const bf16*)it->second.p;
}

static int need(vv_ctx* c, const std::string& n, const std::vector<int64_t>& shape) {
  auto it = c->w.find(n);
  if (it == c->w.end()) FAIL("missing weight: " + n);
  if (!shape.empty() && it->second.shape != shape) {
    std::string s = "shape mismatch for " + n + ": got [";
    for (auto v : it->second.shape) s += std::to_string(v) + ",";
    s += "] want [";
    for (auto v : shape) s += std::to_string(v) + ",";
    FAIL(s + "]");
  }
  return 0;
}

static GemmArgs gemm_args(vv_ctx* c, int M, int N, int K, RowMap a, const bf16* w, int epi, RowMap out,
                          const bf16* bias = nullptr) {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.M = M;
  g.N = N;
  g.K = K;
  g.ksplit = 1;
  g.a = a;
  g.w = w;
  g.ldw = K;
  g.epi.kind = epi;
  g.epi.bias = bias;
  g.epi.out = out;
  g.ws = (float*)c->splitk_ws.p;
  g.counters = (unsigned*)c->splitk_cnt.p;
  return g;
}

static ATransform xf_norm(const bf16* w, float eps, const bf16* mod = nullptr, long long mod_ld = 0, int shift_off = 0,
                          int scale_off = 0) {
  ATransform x;
  memset(&x, 0, sizeof(x));
  x.kind = XF_NORM;
  x.eps = eps;
  x.w = w;
  x.mod = mod;
  x.mod_ld = mod_ld;
  x.shift_off = shift_off;
  x.scale_off = scale_off;
  return x;
}

static int rmsnorm(int M, int C, RowMap in, RowMap out, const bf16* w, float eps, hipStream_t st,
                   const bf16* mod = nullptr, long long mod_ld = 0, int shift_off = 0, int scale_off = 0,
                   int pack = 0);

// test switch (vv_norm_pack): 1 = the normalised rows feeding a 256 x 256-tile
// GEMM are written MFMA-fragment-packed (16K-token gate|up 1055 -> 948 us, q|k|v
// 98 -> 92: one contiguous 1 KB load per A block instead of 16 row pieces)
static std::atomic<int> g_norm_pack{1};
extern "C" int vv_norm_pack(int on) {
  g_norm_pack = on;
  return 0;
}

static int gemm(vv_ctx* c, GemmArgs g, hipStream_t st) {
  if (!g.w) FAIL("gemm: null weight");
  if (g.xf.kind == XF_NORM && g.M > 16) {
    // more rows than one MFMA tile: the GEMV / GEMM kernels would re-normalise
    // the A block in every workgroup (B = 32: LM gate|up 334 us); normalise it
    // once (k_rmsnorm: the same arithmetic and summation order, bit-identical)
    GemmArgs probe = g;
    probe.xf.kind = XF_NONE;
    const int pack = g_norm_pack && g.K % 32 == 0 && gemm_uses_xl(probe) ? 1 : 0;
    CHK(c->norm_ws.ensure((size_t)(g.M + 15) / 16 * 16 * g.K * sizeof(bf16)));
    CHK(rmsnorm(g.M, g.K, g.a, rowmap(c->norm_ws.p, g.K), g.xf.w, g.xf.eps, st, g.xf.mod, g.xf.mod_ld,
                g.xf.shift_off, g.xf.scale_off, pack));
    g.a = rowmap(c->norm_ws.p, g.K);
    g.apack = pack;
    g.xf.kind = XF_NONE;
  }
  KCHK(launch_gemm(g, st));
  return 0;
}

static int rmsnorm(int M, int C, RowMap in, RowMap out, const bf16* w, float eps, hipStream_t st,
                   const bf16* mod, long long mod_ld, int shift_off, int scale_off, int pack) {
  NormArgs a;
  memset(&a, 0, sizeof(a));
  a.pack = pack;
  a.M = M;
  a.C = C;
  a.eps = eps;
  a.in = in;
  a.out = out;
  a.w = w;
  a.has_mod = mod != nullptr;
  a.mod = mod;
  a.mod_ld = mod_ld;
  a.shift_off = shift_off;
  a.scale_off = scale_off;
  KCHK(launch_rmsnorm(a, st));
  return 0;
}

// ------------------------------------------------------------------ grid-waiting kernels
// The context half of the decision every one-launch (grid-waiting) kernel takes
// before its launch; the kernel half is its *_fits (shape + persist_resident on
// the occupancy query).  Both halves are vv_persist_decision for the tests.
static bool persist_ctx_ok(int enabled, int contexts_on_device) { return enabled && contexts_on_device == 1; }
static bool persist_on(vv_ctx* c) {
  return persist_ctx_ok(c->persist_ok && (c->hl_registered || c->persist_follow) ? 1 : 0, hl_count(c->device));
}
extern "C" int vv_persist_decision(int blocks_per_cu, int cus, int scratch_bytes, int grid, int contexts_on_device,
                                   int enabled) {
  return persist_resident(blocks_per_cu, cus, scratch_bytes, grid) && persist_ctx_ok(enabled, contexts_on_device) ? 1
                                                                                                                   : 0;
}

// ------------------------------------------------------------------ codec layout
static void convnet_shape(vv_ctx* c, ConvNet& n, bool decoder, const std::string& wp, int nf, int in_ch, int out_ch,
                          int T0, int slots) {
  const vv_config& k = c->cfg;
  n.decoder = decoder;
  n.wp = wp;
  n.nst = k.n_stages;
  n.in_ch = in_ch;
  n.out_ch = out_ch;
  n.T0 = T0;
  n.slots = slots;
  n.nmax = slots;
  for (int i = 0; i < n.nst; ++i) {
    if (decoder) {
      n.depth[i] = k.dec_depths[i];
      n.chans[i] = nf << (n.nst - 1 - i);
      n.rat[i] = i == 0 ? 1 : k.ratios[i - 1];
      n.T[i] = i == 0 ? T0 : n.T[i - 1] * n.rat[i];
      n.Tin[i] = i == 0 ? T0 : n.T[i - 1];
    } else {
      n.depth[i] = k.enc_depths[i];
      n.chans[i] = nf << i;
      n.rat[i] = i == 0 ? 1 : k.ratios[n.nst - 1 - i];  // encoder ratios are reversed
      n.Tin[i] = i == 0 ? T0 : n.T[i - 1];
      n.T[i] = i == 0 ? T0 : (n.T[i - 1] + n.rat[i] - 1) / n.rat[i];
    }
  }
}

static int convnet_alloc(ConvNet& n, int kernel) {
  // layout the per-slot buffers
  std::vector<ConvBuf*> all;
  size_t total = 0;
  auto add = [&](ConvBuf& b, int ctx, int T, int rows_pad, int C) {
    b.ctx = ctx;
    b.T = T;
    b.C = C;
    b.rows = ctx + rows_pad;
    b.sB = (long long)b.rows * C;
    all.push_back(&b);
    total += (size_t)b.sB * n.slots;
  };
  add(n.stem, kernel - 1, n.T0, n.T0, n.in_ch);
  n.mix.assign(n.nst, {});
  for (int i = 0; i < n.nst; ++i) {
    if (i > 0) {
      if (n.decoder) {
        add(n.tr[i], 1, n.Tin[i], n.Tin[i], n.chans[i - 1]);
      } else {
        const int s = n.rat[i];
        add(n.tr[i], s, n.Tin[i], n.T[i] * s, n.chans[i - 1]);
      }
    }
    n.mix[i].resize(n.depth[i]);
    for (int j = 0; j < n.depth[i]; ++j) add(n.mix[i][j], kernel - 1, n.T[i], n.T[i], n.chans[i]);
  }
  add(n.head, kernel - 1, n.T[n.nst - 1], n.T[n.nst - 1], n.chans[n.nst - 1]);
  CHK(n.state.ensure(total * sizeof(bf16)));
  HIPCHK(hipMemset(n.state.p, 0, total * sizeof(bf16)));
  bf16* p = (bf16*)n.state.p;
  n.rolls.clear();
  for (ConvBuf* b : all) {
    b->base = p;
    p += (size_t)b->sB * n.slots;
    RollDesc r;
    r.base = b->base;
    r.sB = b->sB;
    r.ctx = b->ctx;
    r.T = b->T;
    r.C = b->C;
    r.pad_ = 0;
    n.rolls.push_back(r);
  }
  CHK(n.d_rolls.ensure(n.rolls.size() * sizeof(RollDesc)));
  HIPCHK(hipMemcpy(n.d_rolls.p, n.rolls.data(), n.rolls.size() * sizeof(RollDesc), hipMemcpyHostToDevice));
  // transient work: X per stage + A (normed rows) + F (ffn hidden)
  size_t xw = 0, aw = 0, fw = 0;
  for (int i = 0; i < n.nst; ++i) {
    xw += (size_t)n.T[i] * n.chans[i];
    aw = std::max(aw, (size_t)n.T[i] * n.chans[i]);
    fw = std::max(fw, (size_t)n.T[i] * n.chans[i] * 4);
  }
  const size_t per = 2 * xw + aw + fw;
  CHK(n.work.ensure(per * n.nmax * sizeof(bf16)));
  bf16* q = (bf16*)n.work.p;
  for (int i = 0; i < n.nst; ++i) {
    n.X[i] = q;
    q += (size_t)n.T[i] * n.chans[i] * n.nmax;
    n.Y[i] = q;
    q += (size_t)n.T[i] * n.chans[i] * n.nmax;
  }
  n.A = q;
  q += aw * n.nmax;
  n.F = q;
  return 0;
}

static int convnet_check(vv_ctx* c, ConvNet& n) {
  const std::string& p = n.wp;
  const int k = 7;
  if (n.decoder) {
    CHK(need(c, p + ".stem_w", {n.chans[0], (int64_t)k * n.in_ch}));
  } else {
    CHK(need(c, p + ".stem_w", {n.chans[0], (int64_t)k}));
  }
  CHK(need(c, p + ".stem_b", {n.chans[0]}));
  for (int i = 0; i < n.nst; ++i) {
    const int C = n.chans[i];
    if (i > 0) {
      const std::string t = p + ".tr" + std::to_string(i);
      const int Ci = n.chans[i - 1], r = n.rat[i];
      if (n.decoder) {
        CHK(need(c, t + "_w", {(int64_t)r * C, 2LL * Ci}));
        CHK(need(c, t + "_b", {(int64_t)r * C}));
      } else {
        CHK(need(c, t + "_w", {C, 2LL * r * Ci}));
        CHK(need(c, t + "_b", {C}));
      }
    }
    for (int j = 0; j < n.depth[i]; ++j) {
      const std::string b = p + ".s" + std::to_string(i) + ".b" + std::to_string(j);
      CHK(need(c, b + ".dw_w", {C, k}));
      CHK(need(c, b + ".dw_b", {C}));
      CHK(need(c, b + ".gamma", {C}));
      CHK(need(c, b + ".fc1_w", {4LL * C, C}));
      CHK(need(c, b + ".fc1_b", {4LL * C}));
      CHK(need(c, b + ".fc2_w", {C, 4LL * C}));
      CHK(need(c, b + ".fc2_b", {C}));
      CHK(need(c, b + ".ffn_gamma", {C}));
    }
  }
  const int Cl = n.chans[n.nst - 1];
  if (n.decoder) {
    CHK(need(c, p + ".head_w", {k, Cl}));
    CHK(need(c, p + ".head_b", {1}));
  } else {
    CHK(need(c, p + ".head_w", {n.out_ch, (int64_t)k * Cl}));
    CHK(need(c, p + ".head_b", {n.out_ch}));
  }
  return 0;
}

// Rows of ConvBuf b, starting after its history, for the active samples (slot map).
static RowMap buf_in_rows(const ConvBuf& b, int T, const int* slots) {
  return rowmap(b.base + (long long)b.ctx * b.C, b.C, T, b.sB, slots);
}

// Codec Block1D front half folded into fc1's prologue where it fits (XF_MIX);
// off only for the bit-exactness test against the k_mix path.
static std::atomic<int> g_mix_fusion{3};   // bit 0: XF_MIX, bit 1: k_block
extern "C" int vv_codec_mix_fusion(int mask) {
  g_mix_fusion = mask & 3;
  return 0;
}

// A codec stage of Block1Ds of one sample (C = 2,048 at T = 1, C = 1,024 at
// T = 2 / 8) runs as ONE persistent launch (codec_stage.hip) while the context is the device's only one registered for
// persistent kernels (persist_on); 0 = the launch-per-GEMV path (A/B and tests).
static std::atomic<int> g_codec_stage{1};
// Bits 1..3 pick how the C = 2,048 form issues its weight stream (A/B only):
// 0 = the default, the split, paced stream (CodecStageArgs::pubfirst 5); v > 0 =
// pubfirst v - 1 (1: round 5's whole-block stream at each block's end).
extern "C" int vv_codec_stage(int on) {
  g_codec_stage = on & 15;
  return 0;
}
static bool codec_stage_any(const ConvNet& net) {
  for (int i = 0; i < net.nst; ++i)
    if (codec_stage_fits(net.chans[i], net.T[i], 1, net.depth[i])) return true;
  return false;
}
static bool codec_stage_on(vv_ctx* c, const ConvNet& net, int i, int n) {
  return g_codec_stage && c->cs_sync.p && codec_stage_fits(net.chans[i], net.T[i], n, net.depth[i]) &&
         persist_on(c);
}
static std::atomic<unsigned long long*> g_codec_stage_stamps{nullptr};
static std::atomic<int> g_codec_stage_stamp_at{0};
// diagnostic: the acoustic decoder's stage `stage` records [256][64] per-workgroup phase stamps
extern "C" int vv_codec_stage_stamps(void* buf, int stage) {
  g_codec_stage_stamps = (unsigned long long*)buf;
  g_codec_stage_stamp_at = stage;
  return 0;
}
extern "C" int vv_codec_stage_active(vv_ctx* c) {
  return c && c->finalized && codec_stage_on(c, c->dec, 0, 1) ? 1 : 0;
}

// The narrow stages (C <= 128) as ONE launch each (codec_tile.hip: transition
// conv + three Block1Ds [+ the decoder's head conv], halo recomputed per
// workgroup); 0 = k_block per Block1D + the transition GEMMs (A/B and tests).
static std::atomic<int> g_codec_tile{1};
extern "C" int vv_codec_tile(int on) {
  g_codec_tile = on ? 1 : 0;
  return 0;
}
// diagnostic: tile launches record [n][tiles][16] phase stamps at buf + 4096 x (3 x net + stage index among
// the tiled stages) (net 0 decoder, 1 encoders); nullptr: off
static std::atomic<unsigned long long*> g_codec_tile_stamps{nullptr};
extern "C" int vv_codec_tile_stamps(void* buf) {
  g_codec_tile_stamps = (unsigned long long*)buf;
  return 0;
}
// the transition fused into stage i's tile launch (CT_PRE_*), or -1: none applies
static int tile_pre(const ConvNet& net, int i) {
  const int C = net.chans[i];
  int pre = CT_PRE_NONE;
  if (net.decoder && i > 0 && net.rat[i] == 2 && net.chans[i - 1] == 2 * C) pre = CT_PRE_CONVT;
  if (!net.decoder && i > 0 && net.rat[i] == 2 && 2 * net.chans[i - 1] == C) pre = CT_PRE_SCONV;
  if (!net.decoder && i == 0 && net.in_ch == 1) pre = CT_PRE_STEM;
  if (net.decoder && i == 0) return -1;   // (the decoder's stem stage is the widest)
  const int post = net.decoder && i == net.nst - 1 ? CT_POST_HEAD : CT_POST_NONE;
  if (!g_codec_tile || !codec_tile_fits(C, pre, post, net.depth[i], net.mix[i].empty() ? 0 : net.mix[i][0].ctx))
    return -1;
  return pre;
}

// The wide stages (C = 256 / 512) as ONE launch each (codec_wide.hip: clusters of
// C / 32 workgroups per 16-row tile) under the grid-waiting kernels' rule
// (persist_on: the launch's workgroups must be co-resident); 0 = k_mix + fc1 /
// fc2 GEMMs per Block1D (A/B and tests).
static std::atomic<int> g_codec_wide{1};
extern "C" int vv_codec_wide(int on) {
  g_codec_wide = on ? 1 : 0;
  return 0;
}
extern "C" int vv_codec_wide_over(int on) {   // diagnostic: 1 = grids past one resident wave too (B = 8)
  codec_wide_oversubscribe(on);
  return 0;
}
static std::atomic<unsigned long long*> g_codec_wide_stamps{nullptr};
extern "C" int vv_codec_wide_stamps(void* buf) {   // diagnostic: [n][tiles x S][16] at buf + 8192 x (2 x net + (C == 512))
  g_codec_wide_stamps = (unsigned long long*)buf;
  return 0;
}
// some stage of the net has a wide-stage shape the cluster kernel takes (one sample)
static bool codec_wide_any(const ConvNet& net) {
  for (int i = 0; i < net.nst; ++i)
    if (!net.mix[i].empty() && codec_wide_fits(net.chans[i], net.T[i], 1, net.depth[i], net.mix[i][0].ctx)) return true;
  return false;
}
static bool wide_on(vv_ctx* c, const ConvNet& net, int i, int n) {
  const int C = net.chans[i];
  return g_codec_wide && (C == 256 || C == 512) && persist_on(c) && c->cw_sync.p && !net.mix[i].empty() &&
         codec_wide_fits(C, net.T[i], n, net.depth[i], net.mix[i][0].ctx) && n * ((net.T[i] + 15) / 16) <= CW_LINES;
}
extern "C" int vv_codec_wide_active(vv_ctx* c, int n) {   // 1: some acoustic-decoder stage runs it now
  if (!c || !c->finalized) return 0;
  for (int i = 0; i < c->dec.nst; ++i)
    if (wide_on(c, c->dec, i, n)) return 1;
  return 0;
}

// diffusion steps whose adaLN modulations are computed in one GEMM
static constexpr int HEAD_SC = 16;

// One block stack + transitions.  n active samples (slots[n]); input rows already
// in `stem` (rows [ctx, ctx+T0)).  Decoder: writes audio to out (+ out2).
// Encoder: writes [n, out_ch] features to out.
static int convnet_run(vv_ctx* c, ConvNet& net, int n, const int* slots, RowMap out, RowMap out2, hipStream_t st) {
  const std::string& p = net.wp;
  const float eps = c->cfg.codec_eps;
  const int k = 7;
  // ---- stem (the encoders' is fused into stage 0's tile launch where it applies)
  if (net.decoder || tile_pre(net, 0) != CT_PRE_STEM) {
    const int T = net.T[0], C = net.chans[0];
    RowMap xo = rowmap(net.X[0], C, T, (long long)T * C);
    if (net.decoder) {
      RowMap a = rowmap(net.stem.base, net.stem.C, T, net.stem.sB, slots);
      GemmArgs g = gemm_args(c, n * T, C, k * net.in_ch, a, W(c, p + ".stem_w"), EPI_STORE, xo, W(c, p + ".stem_b"));
      CHK(gemm(c, g, st));
    } else {
      ConvIn1Args a;
      a.M = n * T;
      a.C = C;
      a.K = k;
      a.buf = rowmap(net.stem.base, 1, T, net.stem.sB, slots);
      a.w = W(c, p + ".stem_w");
      a.b = W(c, p + ".stem_b");
      a.out = xo;
      KCHK(launch_conv_cin1(a, st));
    }
  }
  bool head_done = false;
  for (int i = 0; i < net.nst; ++i) {
    const int T = net.T[i], C = net.chans[i];
    RowMap X = rowmap(net.X[i], C, T, (long long)T * C);
    const int tpre = tile_pre(net, i);
    if (i > 0 && tpre != CT_PRE_CONVT && tpre != CT_PRE_SCONV) {
      const ConvBuf& tb = net.tr[i];
      const int Ci = net.chans[i - 1], r = net.rat[i];
      const std::string t = p + ".tr" + std::to_string(i);
      if (net.decoder) {
        // 2-tap ConvTranspose: input row t = buffer rows [t, t+1] (1 history row)
        RowMap a = rowmap(tb.base, Ci, net.Tin[i], tb.sB, slots);
        RowMap o = rowmap(net.X[i], (long long)r * C, net.Tin[i], (long long)T * C);
        GemmArgs g = gemm_args(c, n * net.Tin[i], r * C, 2 * Ci, a, W(c, t + "_w"), EPI_STORE, o, W(c, t + "_b"));
        CHK(gemm(c, g, st));
      } else {
        // strided causal conv, k = 2r, ctx = r: output row t = buffer rows [t*r, t*r + 2r)
        RowMap a = rowmap(tb.base, (long long)r * Ci, T, tb.sB, slots);
        GemmArgs g = gemm_args(c, n * T, C, 2 * r * Ci, a, W(c, t + "_w"), EPI_STORE, X, W(c, t + "_b"));
        CHK(gemm(c, g, st));
      }
    }
    if (tpre >= 0) {
      // the whole narrow stage in one launch (codec_tile.hip)
      CodecTileArgs A;
      memset(&A, 0, sizeof(A));
      A.n = n;
      A.T = T;
      A.depth = net.depth[i];
      A.eps = eps;
      A.slots = slots;
      A.x = net.X[i];
      if (tpre == CT_PRE_STEM) {
        A.pre_buf = net.stem.base;
        A.pre_sB = net.stem.sB;
        A.pre_w = W(c, p + ".stem_w");
        A.pre_b = W(c, p + ".stem_b");
      } else if (tpre != CT_PRE_NONE) {
        const std::string t = p + ".tr" + std::to_string(i);
        A.pre_buf = net.tr[i].base;
        A.pre_sB = net.tr[i].sB;
        A.pre_w = W(c, t + "_w");
        A.pre_b = W(c, t + "_b");
      }
      for (int j = 0; j < net.depth[i]; ++j) {
        const std::string b = p + ".s" + std::to_string(i) + ".b" + std::to_string(j);
        CodecTileBlock& Bk = A.b[j];
        Bk.norm = W(c, b + ".norm");
        Bk.dw_w = W(c, b + ".dw_w");
        Bk.dw_b = W(c, b + ".dw_b");
        Bk.gamma = W(c, b + ".gamma");
        Bk.ffn_norm = W(c, b + ".ffn_norm");
        Bk.fc1_w = W(c, b + ".fc1_w");
        Bk.fc1_b = W(c, b + ".fc1_b");
        Bk.fc2_w = W(c, b + ".fc2_w");
        Bk.fc2_b = W(c, b + ".fc2_b");
        Bk.ffn_gamma = W(c, b + ".ffn_gamma");
        Bk.mix = net.mix[i][j].base;
        Bk.mix_sB = net.mix[i][j].sB;
      }
      int post = CT_POST_NONE;
      if (net.decoder && i == net.nst - 1) {
        post = CT_POST_HEAD;
        A.head_w = W(c, p + ".head_w");
        A.head_b = W(c, p + ".head_b");
        A.head_buf = net.head.base;
        A.head_sB = net.head.sB;
        A.audio = out;
        A.audio2 = out2;
        head_done = true;
      } else {
        const ConvBuf& nb = (i + 1 < net.nst) ? net.tr[i + 1] : net.head;
        A.out = buf_in_rows(nb, T, slots);
      }
      if (unsigned long long* sp = g_codec_tile_stamps.load())
        A.stamps = sp + 4096 * (3 * (net.decoder ? 0 : 1) + (C == 128 ? (net.decoder ? 0 : 2) : C == 64 ? 1 : (net.decoder ? 2 : 0)));
      KCHK(launch_codec_tile(A, C, tpre, post, st));
      continue;
    }
    if (wide_on(c, net, i, n)) {
      // the whole wide stage in one launch of clusters (codec_wide.hip)
      CodecWideArgs A;
      memset(&A, 0, sizeof(A));
      A.n = n;
      A.T = T;
      A.depth = net.depth[i];
      A.eps = eps;
      A.slots = slots;
      A.x = net.X[i];
      for (int j = 0; j < net.depth[i]; ++j) {
        const std::string b = p + ".s" + std::to_string(i) + ".b" + std::to_string(j);
        CodecTileBlock& Bk = A.b[j];
        Bk.norm = W(c, b + ".norm");
        Bk.dw_w = W(c, b + ".dw_w");
        Bk.dw_b = W(c, b + ".dw_b");
        Bk.gamma = W(c, b + ".gamma");
        Bk.ffn_norm = W(c, b + ".ffn_norm");
        Bk.fc1_w = W(c, b + ".fc1_w");
        Bk.fc1_b = W(c, b + ".fc1_b");
        Bk.fc2_w = W(c, b + ".fc2_w");
        Bk.fc2_b = W(c, b + ".fc2_b");
        Bk.ffn_gamma = W(c, b + ".ffn_gamma");
        Bk.mix = net.mix[i][j].base;
        Bk.mix_sB = net.mix[i][j].sB;
      }
      const ConvBuf& nb = (i + 1 < net.nst) ? net.tr[i + 1] : net.head;
      A.out = buf_in_rows(nb, T, slots);
      CHK(c->cw_slab.ensure(codec_wide_slab_floats(C, T, n) * sizeof(float)));
      CHK(c->cw_xbuf.ensure(codec_wide_xbuf_elems(C, T, n) * sizeof(bf16)));
      A.sync = (unsigned*)c->cw_sync.p + (C == 512 ? CW_LINES * 32 : 0);
      A.err = (unsigned*)c->hf_sync.p + 10 * 32;
      A.slab = (float*)c->cw_slab.p;
      A.xbuf = (bf16*)c->cw_xbuf.p;
      if (unsigned long long* sp = g_codec_wide_stamps.load()) A.stamps = sp + 8192 * (2 * (net.decoder ? 0 : 1) + (C == 512));
      const int rc = launch_codec_wide(A, C, st);
      if (rc) FAIL("wide codec stage: launch failed (" + std::to_string(rc) + ")");
      continue;
    }
    if (codec_stage_on(c, net, i, n)) {
      // the whole stage (one sample) in one persistent launch (codec_stage.hip)
      CodecStageArgs A;
      memset(&A, 0, sizeof(A));
      A.depth = net.depth[i];
      A.ctx = net.mix[i][0].ctx;
      A.C = C;
      A.M = T;
      A.eps = eps;
      A.slots = slots;
      A.x = net.X[i];
      A.xe = net.Y[i];
      A.h = net.F;
      const ConvBuf& nb = (i + 1 < net.nst) ? net.tr[i + 1] : net.head;
      A.out = buf_in_rows(nb, T, slots);
      for (int j = 0; j < net.depth[i]; ++j) {
        const std::string b = p + ".s" + std::to_string(i) + ".b" + std::to_string(j);
        CodecStageBlock& B = A.b[j];
        B.norm = W(c, b + ".norm");
        B.dw_w = W(c, b + ".dw_w");
        B.dw_b = W(c, b + ".dw_b");
        B.gamma = W(c, b + ".gamma");
        B.ffn_norm = W(c, b + ".ffn_norm");
        B.fc1_w = W(c, b + ".fc1_w");
        B.fc1_b = W(c, b + ".fc1_b");
        B.fc2_w = W(c, b + ".fc2_w");
        B.fc2_b = W(c, b + ".fc2_b");
        B.ffn_gamma = W(c, b + ".ffn_gamma");
        B.mix = net.mix[i][j].base;
        B.mix_sB = net.mix[i][j].sB;
        if (net.mix[i][j].ctx != A.ctx) FAIL("codec stage: conv buffers of one stage differ in history length");
      }
      A.sync = (unsigned*)c->cs_sync.p;
      A.err = (unsigned*)c->hf_sync.p + 10 * 32;
      A.stamps = net.decoder && i == g_codec_stage_stamp_at ? g_codec_stage_stamps.load() : nullptr;
      {
        const int v = (g_codec_stage.load() >> 1) & 7;
        A.pubfirst = v ? v - 1 : 5;
      }
      const int rc = launch_codec_stage(A, st);
      if (rc) FAIL("persistent codec stage: launch failed (" + std::to_string(rc) + ": " +
                   hipGetErrorString(hipGetLastError()) + ")");
      continue;
    }
    const int Rb = std::max(1, std::min(T, 2048 / C));
    if ((g_mix_fusion & 2) && block_lds(Rb, C)) {
      // narrow stage: each Block1D is one k_block launch; the residual
      // ping-pongs X -> Y -> X (a workgroup reads halo rows other workgroups own)
      for (int j = 0; j < net.depth[i]; ++j) {
        const std::string b = p + ".s" + std::to_string(i) + ".b" + std::to_string(j);
        const ConvBuf& mb = net.mix[i][j];
        BlockArgs ba;
        memset(&ba, 0, sizeof(ba));
        MixArgs& mx = ba.mix;
        mx.n = n;
        mx.T = T;
        mx.C = C;
        mx.R = Rb;
        mx.eps = eps;
        mx.ctx = mb.ctx;
        mx.x = (j & 1) ? net.Y[i] : net.X[i];
        mx.buf = mb.base;
        mx.buf_sB = mb.sB;
        mx.slots = slots;
        mx.norm_w = W(c, b + ".norm");
        mx.dw_w = W(c, b + ".dw_w");
        mx.dw_b = W(c, b + ".dw_b");
        mx.gamma = W(c, b + ".gamma");
        mx.ffn_norm_w = W(c, b + ".ffn_norm");
        ba.w1 = W(c, b + ".fc1_w");
        ba.b1 = W(c, b + ".fc1_b");
        ba.w2 = W(c, b + ".fc2_w");
        ba.b2 = W(c, b + ".fc2_b");
        ba.g2 = W(c, b + ".ffn_gamma");
        if (j == net.depth[i] - 1) {
          const ConvBuf& nb = (i + 1 < net.nst) ? net.tr[i + 1] : net.head;
          ba.out = buf_in_rows(nb, T, slots);
        } else {
          ba.out = rowmap((j & 1) ? net.X[i] : net.Y[i], C, T, (long long)T * C);
        }
        KCHK(launch_block(ba, st));
      }
      continue;
    }
    for (int j = 0; j < net.depth[i]; ++j) {
      const std::string b = p + ".s" + std::to_string(i) + ".b" + std::to_string(j);
      const ConvBuf& mb = net.mix[i][j];
      RowMap Y = rowmap(net.Y[i], C, T, (long long)T * C);
      RowMap Fm = rowmap(net.F, 4LL * C);
      if ((g_mix_fusion & 1) && gemv_mix_lds(n * T, T, C)) {
        // few rows (T = 1, 8 stages at small batch): the mix runs in fc1's prologue
        GemmArgs g = gemm_args(c, n * T, 4 * C, C, X, W(c, b + ".fc1_w"), EPI_GELU, Fm, W(c, b + ".fc1_b"));
        g.xf.kind = XF_MIX;
        g.xf.eps = eps;
        g.xf.w = W(c, b + ".norm");
        g.xf.T = T;
        g.xf.ctx = mb.ctx;
        g.xf.buf = mb.base;
        g.xf.buf_sB = mb.sB;
        g.xf.slots = slots;
        g.xf.dw_w = W(c, b + ".dw_w");
        g.xf.dw_b = W(c, b + ".dw_b");
        g.xf.gamma = W(c, b + ".gamma");
        g.xf.ffn_w = W(c, b + ".ffn_norm");
        g.xf.y = net.Y[i];
        CHK(gemm(c, g, st));
      } else {
      // mixer norm + depthwise conv + gamma residual (X -> Y) + ffn_norm (-> A), one launch
      MixArgs mx;
      memset(&mx, 0, sizeof(mx));
      mx.n = n;
      mx.T = T;
      mx.C = C;
      mx.R = std::max(1, std::min(T, 2048 / C));   // R * C / 8 = 256 conv items: one per thread
      mx.eps = eps;
      mx.ctx = mb.ctx;
      mx.x = net.X[i];
      mx.y = net.Y[i];
      mx.a = net.A;
      mx.buf = mb.base;
      mx.buf_sB = mb.sB;
      mx.slots = slots;
      mx.norm_w = W(c, b + ".norm");
      mx.dw_w = W(c, b + ".dw_w");
      mx.dw_b = W(c, b + ".dw_b");
      mx.gamma = W(c, b + ".gamma");
      mx.ffn_norm_w = W(c, b + ".ffn_norm");
      KCHK(launch_mix(mx, st));
      CHK(gemm(c, gemm_args(c, n * T, 4 * C, C, rowmap(net.A, C), W(c, b + ".fc1_w"), EPI_GELU, Fm,
                            W(c, b + ".fc1_b")), st));
      }
      RowMap o = X;
      const bool last = j == net.depth[i] - 1;
      if (last) {
        const ConvBuf& nb = (i + 1 < net.nst) ? net.tr[i + 1] : net.head;
        o = buf_in_rows(nb, T, slots);
      }
      GemmArgs g = gemm_args(c, n * T, C, 4 * C, Fm, W(c, b + ".fc2_w"), EPI_RES, o, W(c, b + ".fc2_b"));
      g.epi.res = Y;
      g.epi.gamma = W(c, b + ".ffn_gamma");
      CHK(gemm(c, g, st));
    }
  }
  // ---- head (disable_last_norm: no final norm, modular_vibevoice_tokenizer.py:908-911)
  const int Tl = net.T[net.nst - 1], Cl = net.chans[net.nst - 1];
  if (head_done) {
  } else if (net.decoder) {
    Conv1Args a;
    a.M = n * Tl;
    a.C = Cl;
    a.K = k;
    a.buf = rowmap(net.head.base, Cl, Tl, net.head.sB, slots);
    a.w = W(c, p + ".head_w");
    a.b = W(c, p + ".head_b");
    a.out = out;
    a.out2 = out2;
    KCHK(launch_conv_cout1(a, st));
  } else {
    RowMap a = rowmap(net.head.base, Cl, Tl, net.head.sB, slots);
    GemmArgs g = gemm_args(c, n * Tl, net.out_ch, k * Cl, a, W(c, p + ".head_w"), EPI_STORE, out, W(c, p + ".head_b"));
    CHK(gemm(c, g, st));
  }
  return 0;
}

static int convnet_roll(ConvNet& net, int n, const int* slots, int mode, hipStream_t st) {
  KCHK(launch_roll((const RollDesc*)net.d_rolls.p, (int)net.rolls.size(), slots, n, mode, st));
  return 0;
}

// ------------------------------------------------------------------ C ABI
extern "C" {

const char* vv_last_error(void) { return g_err.c_str(); }
int vv_ws_epoch(void) { return g_ws_epoch.load(); }

int vv_create(const vv_config* cfg, int device, vv_ctx** out) {
  if (!cfg || !out) FAIL("vv_create: null argument");
  if (cfg->head_dim != 128) FAIL("head_dim must be 128");
  if (cfg->n_stages < 1 || cfg->n_stages > VV_MAX_STAGES) FAIL("n_stages out of range");
  if (cfg->n_heads % cfg->n_kv_heads || cfg->n_heads / cfg->n_kv_heads > 8) FAIL("unsupported GQA ratio");
  if (cfg->max_batch < 1 || cfg->max_batch > 32) FAIL("max_batch must be in [1, 32]");
  HIPCHK(hipSetDevice(device));
  vv_ctx* c = new vv_ctx();
  c->cfg = *cfg;
  c->device = device;
  c->persist_ok = persist_env_default();
  *out = c;
  return 0;
}

void vv_destroy(vv_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  if (c->hl_registered) hl_register(c->device, -1);
  DevBuf* bufs[] = {&c->norm_ws, &c->kv_k, &c->kv_v, &c->lm_ws, &c->attn_part, &c->attn_cnt, &c->valid_ids, &c->splitk_ws, &c->splitk_cnt,
                    &c->temb, &c->tfreq_tmp, &c->head_ws, &c->codec_ws, &c->slot_scratch, &c->unit_sb,
                    &c->rope_tab, &c->zero_rows, &c->hf_sync, &c->cs_sync, &c->m16_buf, &c->lf_sync,
                    &c->cw_sync, &c->cw_slab, &c->cw_xbuf, &c->lf_slab, &c->la_part};
  for (DevBuf* b : bufs) b->release();
  ConvNet* nets[] = {&c->dec, &c->sem, &c->aenc, &c->senc};
  for (ConvNet* n : nets) {
    n->state.release();
    n->work.release();
    n->d_rolls.release();
  }
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int vv_bind_weight(vv_ctx* c, const char* name, const void* p, const int64_t* shape, int ndim) {
  if (!c || !name || !p) FAIL("vv_bind_weight: null argument");
  Weight w;
  w.p = p;
  w.shape.assign(shape, shape + ndim);
  c->w[name] = w;
  return 0;
}

int vv_set_valid_ids(vv_ctx* c, int n, const int* ids) {
  if (n < 1 || n > 4) FAIL("vv_set_valid_ids: 1..4 ids");
  CHK(c->valid_ids.ensure(4 * sizeof(int)));
  HIPCHK(hipMemcpy(c->valid_ids.p, ids, n * sizeof(int), hipMemcpyHostToDevice));
  c->n_valid = n;
  return 0;
}

int vv_finalize(vv_ctx* c) {
  const vv_config& k = c->cfg;
  HIPCHK(hipSetDevice(c->device));
  const int H = k.hidden, d = k.head_dim;
  c->qkv_n = (k.n_heads + 2 * k.n_kv_heads) * d;
  // ---- LM weights
  CHK(need(c, "lm.embed", {}));
  CHK(need(c, "lm.lm_head", {}));
  CHK(need(c, "lm.inv_freq", {d / 2}));
  CHK(need(c, "lm.norm", {H}));
  for (int l = 0; l < k.n_layers; ++l) {
    const std::string p = "lm." + std::to_string(l);
    CHK(need(c, p + ".in_norm", {H}));
    CHK(need(c, p + ".qkv_w", {c->qkv_n, H}));
    CHK(need(c, p + ".qkv_b", {c->qkv_n}));
    CHK(need(c, p + ".o_w", {H, (int64_t)k.n_heads * d}));
    CHK(need(c, p + ".post_norm", {H}));
    CHK(need(c, p + ".gu_w", {2LL * k.intermediate, H}));
    CHK(need(c, p + ".down_w", {H, k.intermediate}));
  }
  // ---- diffusion head
  const int L = k.head_layers, F = k.head_ffn, D = k.latent_dim;
  CHK(need(c, "head.noisy_w", {H, D}));
  CHK(need(c, "head.cond_w", {H, H}));
  CHK(need(c, "head.t0_w", {H, 256}));
  CHK(need(c, "head.t2_w", {H, H}));
  CHK(need(c, "head.ada_w", {(3LL * L + 2) * H, H}));
  // the FFN in the GEMV layout (weights.py: 16-row gate|up tiles of 8 gate + 8 up rows)
  c->head_gemv = true;
  for (int l = 0; l < L; ++l) {
    const std::string p = "head." + std::to_string(l);
    CHK(need(c, p + ".norm", {H}));
    CHK(need(c, p + ".gu_w", {2LL * F, H}));
    CHK(need(c, p + ".down_w", {H, F}));
  }
  CHK(need(c, "head.final_w", {D, H}));
  // grid-wait words + the error word (always present: vv_sync_error_async reads it)
  CHK(c->hf_sync.ensure(SYNC_BYTES));
  HIPCHK(hipMemset(c->hf_sync.p, 0, SYNC_BYTES));
  // ---- connectors + latent scaling
  CHK(need(c, "conn.ac.fc1_w", {H, D}));
  CHK(need(c, "conn.se.fc1_w", {H, k.semantic_dim}));
  for (const char* q : {"conn.ac", "conn.se"}) {
    const std::string s(q);
    CHK(need(c, s + ".fc1_b", {H}));
    CHK(need(c, s + ".norm", {H}));
    CHK(need(c, s + ".fc2_w", {H, H}));
    CHK(need(c, s + ".fc2_b", {H}));
  }
  CHK(need(c, "speech_scaling_factor", {}));
  CHK(need(c, "speech_bias_factor", {}));
  // ---- codec nets
  const int hop = [&] {
    int h = 1;
    for (int i = 0; i + 1 < k.n_stages; ++i) h *= k.ratios[i];
    return h;
  }();
  convnet_shape(c, c->dec, true, "dec", k.dec_n_filters, D, 1, 1, k.max_batch);
  convnet_shape(c, c->sem, false, "sem", k.sem_n_filters, 1, k.semantic_dim, hop, k.max_batch);
  CHK(convnet_check(c, c->dec));
  CHK(convnet_check(c, c->sem));
  const bool has_aenc = c->w.count("aenc.stem_w") > 0;
  if (has_aenc) {
    convnet_shape(c, c->aenc, false, "aenc", k.ac_enc_n_filters, 1, D, hop, 1);
    CHK(convnet_check(c, c->aenc));
  }
  CHK(convnet_alloc(c->dec, 7));
  CHK(convnet_alloc(c->sem, 7));
  // the persistent codec stage's wait counters; a context that can run it (or
  // the persistent head, or the one-launch head layer at 16 rows) counts in the
  // device's registry (hl_register)
  CHK(c->cs_sync.ensure(SYNC_BYTES));
  HIPCHK(hipMemset(c->cs_sync.p, 0, SYNC_BYTES));
  CHK(c->lf_sync.ensure(SYNC_BYTES));
  HIPCHK(hipMemset(c->lf_sync.p, 0, SYNC_BYTES));
  if (k.max_batch >= 2 && lm_ffn16_fits(k.hidden, k.intermediate, 16)) CHK(c->lf_slab.ensure(48 * 4 * 16 * 32 * sizeof(float)));
  const int la_rows = std::min(2 * k.max_batch, 16), la_keys = std::min(k.max_ctx, LA_MAX_KEYS);
  const bool la_fits = lm_attn_fits(k.hidden, k.n_heads, k.n_kv_heads, k.head_dim, la_rows, la_keys) &&
                       c->qkv_n == (k.n_heads + 2 * k.n_kv_heads) * k.head_dim;
  if (la_fits) CHK(c->la_part.ensure(lm_attn_part_floats(la_rows, la_keys) * sizeof(float)));
  CHK(c->cw_sync.ensure(2 * CW_LINES * 128));
  HIPCHK(hipMemset(c->cw_sync.p, 0, 2 * CW_LINES * 128));
  if (c->head_gemv && head_m16_fits(k.hidden, k.head_ffn, 16))
  {
    CHK(c->m16_buf.ensure(16 * 192 * sizeof(float) + 16 * (size_t)k.hidden * sizeof(bf16)));
    HIPCHK(hipMemset(c->m16_buf.p, 0, 16 * 192 * sizeof(float)));
  }
  c->persist_capable = codec_stage_any(c->dec) || codec_stage_any(c->sem) || codec_wide_any(c->dec) ||
                       codec_wide_any(c->sem) ||
                       (c->head_gemv && head_m16_fits(k.hidden, k.head_ffn, 16)) ||
                       lm_ffn_fits(k.hidden, k.intermediate, 2) || lm_ffn16_fits(k.hidden, k.intermediate, 16) || la_fits;
  if (c->persist_ok && !c->persist_follow && c->persist_capable && !c->hl_registered) {
    c->hl_registered = true;
    hl_register(c->device, +1);
  }
  // ---- LM KV cache: [layer][slot][kv_head][ctx][d]
  c->lm_slots = 2 * k.max_batch;
  c->kv.d = d;
  // position stride of the cache rounded up to 64 (128 B): V^T rows [dim][ctx]
  // are read 16 B at a time by the attention kernel, and an odd stride left
  // every other row misaligned
  c->kv.max_ctx = (k.max_ctx + 63) / 64 * 64;
  c->kv.s_head = (long long)c->kv.max_ctx * d;
  c->kv.s_slot = c->kv.s_head * k.n_kv_heads;
  c->kv.s_layer = c->kv.s_slot * c->lm_slots;
  const size_t kvb = (size_t)c->kv.s_layer * k.n_layers * sizeof(bf16);
  CHK(c->kv_k.ensure(kvb));
  CHK(c->kv_v.ensure(kvb + 256));
  // RoPE cos / sin per position (the q|k|v epilogue reads it instead of cosf / sinf)
  if (d == 128) {
    CHK(c->rope_tab.ensure((size_t)c->kv.max_ctx * 128 * sizeof(bf16)));
    KCHK(launch_rope_table(c->kv.max_ctx, (const float*)W(c, "lm.inv_freq"), (bf16*)c->rope_tab.p, nullptr));
    HIPCHK(hipDeviceSynchronize());
  }
  c->kv.k = (bf16*)c->kv_k.p;
  c->kv.v = (bf16*)c->kv_v.p;
  // ---- attention split partials for decode (2 * max_batch rows, <= 64 splits) + tickets
  CHK(c->attn_part.ensure((size_t)2 * k.max_batch * k.n_heads * 256 * (d + 2) * sizeof(float)));
  CHK(c->attn_cnt.ensure(65536 * sizeof(unsigned)));
  HIPCHK(hipMemset(c->attn_cnt.p, 0, 65536 * sizeof(unsigned)));
  // ---- split-K slabs + tickets
  CHK(c->splitk_ws.ensure(64ull << 20));
  CHK(c->splitk_cnt.ensure(65536 * sizeof(unsigned)));
  HIPCHK(hipMemset(c->splitk_cnt.p, 0, 65536 * sizeof(unsigned)));
  // ---- diffusion workspace (rows = 2 * max_batch)
  {
    const size_t R = 2 * (size_t)k.max_batch;
    const size_t mod = (3 * (size_t)L + 2) * H;
    const size_t elems = R * H * 6 + HEAD_SC * R * (mod + H) + R * F + R * D * 3 + (size_t)k.max_batch * D * 2;
    CHK(c->head_ws.ensure(elems * sizeof(bf16)));
  }
  CHK(c->codec_ws.ensure((size_t)k.max_batch * (4 * H + 2 * 256) * sizeof(bf16) + 4096));
  CHK(c->zero_rows.ensure((size_t)2 * k.max_batch * H * sizeof(bf16)));
  HIPCHK(hipMemset(c->zero_rows.p, 0, (size_t)2 * k.max_batch * H * sizeof(bf16)));
  CHK(c->slot_scratch.ensure(4096));
  {
    const uint16_t one_zero[2] = {0x3F80, 0x0000};
    CHK(c->unit_sb.ensure(sizeof(one_zero)));
    HIPCHK(hipMemcpy(c->unit_sb.p, one_zero, sizeof(one_zero), hipMemcpyHostToDevice));
  }
  HIPCHK(hipDeviceSynchronize());
  c->finalized = true;
  return 0;
}

int vv_set_schedule(vv_ctx* c, int steps, const float* coef, const void* tfreq, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!c->finalized) FAIL("vv_set_schedule before vv_finalize");
  if (steps < 1 || steps > 1000) FAIL("steps out of range");
  const int H = c->cfg.hidden;
  c->coef.resize(steps);
  for (int s = 0; s < steps; ++s) {
    const float* q = coef + 8 * s;
    DpmCoef& e = c->coef[s];
    e.alpha_s = q[0];
    e.sigma_s = q[1];
    e.c_x = q[2];
    e.c_d0 = q[3];
    e.c_d1 = q[4];
    e.inv_r0 = q[5];
    e.order = (int)q[6];
    e.c_n = q[7];
    e.cfg = 0.f;
  }
  // sized for the largest schedule once, so captured graphs keep valid pointers
  CHK(c->temb.ensure((size_t)1000 * H * sizeof(bf16)));
  CHK(c->tfreq_tmp.ensure((size_t)1000 * H * sizeof(bf16)));
  // t_emb = Linear2(SiLU(Linear0(t_freq)))  (TimestepEmbedder.forward, diffusion_head.py:90-93)
  bf16* t1 = (bf16*)c->tfreq_tmp.p;
  CHK(gemm(c, gemm_args(c, steps, H, 256, rowmap(tfreq, 256), W(c, "head.t0_w"), EPI_STORE, rowmap(t1, H)), st));
  KCHK(launch_silu(steps * H, t1, t1, st));
  CHK(gemm(c, gemm_args(c, steps, H, H, rowmap(t1, H), W(c, "head.t2_w"), EPI_STORE, rowmap(c->temb.p, H)), st));
  c->steps = steps;
  HIPCHK(hipStreamSynchronize(st));
  return 0;
}

int vv_kv_copy(vv_ctx* c, int n, const int* slots, const int* src, const int* dst, vv_stream vst) {
  if (!c->finalized) FAIL("vv_kv_copy before vv_finalize");
  KCHK(launch_kv_copy(c->kv, c->cfg.n_layers, c->cfg.n_kv_heads, n, slots, src, dst, (hipStream_t)vst));
  return 0;
}

int vv_kv_synthetic(vv_ctx* c, int n, const int* slots, int p0, int p1, unsigned seed, vv_stream vst) {
  if (!c->finalized) FAIL("vv_kv_synthetic before vv_finalize");
  if (p0 < 0 || p1 > c->cfg.max_ctx || p0 > p1) FAIL("vv_kv_synthetic: positions outside [0, max_ctx)");
  KCHK(launch_kv_fill(c->kv, c->cfg.n_layers, c->cfg.n_kv_heads, n, slots, p0, p1, seed, (hipStream_t)vst));
  return 0;
}

int vv_embed(vv_ctx* c, int n, const int* ids, void* out, vv_stream vst) {
  const int H = c->cfg.hidden;
  KCHK(launch_gather_rows(n, H, W(c, "lm.embed"), H, ids, rowmap(out, H), (hipStream_t)vst));
  return 0;
}

// ------------------------------------------------------------------ LM pass
// test switch (vv_rope_table): 0 = the q|k|v epilogue computes cos / sin inline
static std::atomic<int> g_rope_tab{1};
extern "C" int vv_rope_table(int on) {
  g_rope_tab = on;
  return 0;
}
// One forward of ntok token rows, split so that a tensor-parallel group can
// interleave its ranks layer by layer (vv_lm_forward_group) or all-reduce over
// RCCL between the halves (vv_lm_forward).
// Decode attention with a deferred split merge (vv_attn_defer): contexts of 2..8
// chunks of g_defer_chunk keys run that many splits per (row, kv head), each
// leaves its (m, l, o) partial and o_proj merges them while staging its A rows
// (XF_ATTN_MERGE) -- the split parallelism without a ticket or a merge pass.
// Rows: B = 1 (2 rows) gains 1.5 % at K = 750; at B = 8 (16 rows) o_proj's
// staging of 16 rows' partials cost more than the splits saved (5.79 vs 5.67 ms),
// so by default only <= 4 rows defer.
static std::atomic<int> g_attn_defer{4}, g_defer_chunk{128};
// longest split of the deferred-merge plan (keys); longer contexts take the
// grouped plan's many splits (diagnostic vv_attn_defer_max)
static std::atomic<int> g_defer_max{1024};
extern "C" int vv_attn_defer_max(int keys) {
  g_defer_max = keys <= 0 ? 1024 : keys;
  return 0;
}
extern "C" int vv_attn_defer(int on, int chunk) {
  if (chunk % 32 || chunk < 32 || on < 0) return 1;
  g_attn_defer = on == 1 ? 4 : on;   // 1: the default row limit; n >= 2: up to n rows (<= 16)
  g_defer_chunk = chunk;
  return 0;
}
// Long contexts (> 8 splits of 1,024 keys, i.e. > 8,192 keys) with <= 16 rows:
// up to 120 splits of >= 256 keys (65K: 120 x 544, so the one long row's 2 kv
// heads fill 240 CUs where 1,024-key splits busied 128), merged in <= 8
// groups of <= 16 consecutive splits by each group's last-arriving workgroup;
// o_proj merges the group partials (XF_ATTN_MERGE) -- no k_attn_merge launch.
// 120, not 128: k_attn takes one CU per workgroup (234 VGPRs), and the
// dispatcher does not deal workgroups to the 8 XCDs strictly round-robin
// (tools/attn_long_stamps.py: 256 workgroups landed 30 / 34 on two XCDs), so
// with 256 keyed workgroups two CUs ran two in turn and the launch took twice
// as long as its median workgroup.
static std::atomic<int> g_attn_group{120};   // diagnostic (vv_attn_group): 0 = the 1,024-key plan + k_attn_merge
extern "C" int vv_attn_group(int on) {      // 1 = default; n >= 2: at most n splits (<= 128)
  g_attn_group = on == 1 ? 120 : on <= 0 ? 0 : std::min(on, 128);
  return 0;
}
struct LmPass {
  int ntok = 0, nsplit = 1, chunk = 64, prefill = 0, defer = 0, group = 0, ngroups = 0;
  int maxp = 0;   // keys of the longest row (max position + 1)
  bf16 *h = nullptr, *q = nullptr, *att = nullptr, *act = nullptr;
  RowMap in_m, hm;
  const int *slot = nullptr, *pos = nullptr;
  const float* inv_freq = nullptr;
};

// The decode attention's plan for a pass of ntok rows over max_pos_p1 keys
// (lm_begin; vv_attn_pass_plan reports it to the CPU tests): prefill kernel or
// not, key splits, deferred merge (o_proj merges), grouped merge.
struct AttnPassPlan {
  int prefill = 0, nsplit = 1, chunk = 64, defer = 0, group = 0, ngroups = 0;
};
static AttnPassPlan attn_pass_plan(int ntok, int lm_slots, int head_dim, int n_kv, int max_pos_p1) {
  AttnPassPlan P;
  P.prefill = attn_use_prefill(ntok, lm_slots) ? 1 : 0;
  P.nsplit = P.prefill ? 1 : attn_plan(ntok, n_kv, max_pos_p1, &P.chunk);
  if (!P.prefill && g_attn_defer && ntok <= g_attn_defer && ntok <= 16 && head_dim == 128) {
    // 2..8 splits of >= g_defer_chunk keys, up to 8 x 1,024 keys (longer contexts
    // keep attn_plan's many 1,024-key splits: the merge input grows with them)
    int ch = g_defer_chunk, ns = (max_pos_p1 + ch - 1) / ch;
    if (ns > 8) {
      ch = ((max_pos_p1 + 7) / 8 + 31) / 32 * 32;
      ns = (max_pos_p1 + ch - 1) / ch;
    }
    if (ns >= 2 && ns <= 8 && ch <= g_defer_max) {
      P.defer = 1;
      P.nsplit = ns;
      P.chunk = ch;
    }
  }
  if (!P.prefill && !P.defer && g_attn_group && P.nsplit > 8 && ntok <= 16 && head_dim == 128) {
    int ns = std::min((int)g_attn_group, (max_pos_p1 + 255) / 256);
    const int ch = ((max_pos_p1 + ns - 1) / ns + 31) / 32 * 32;
    ns = (max_pos_p1 + ch - 1) / ch;
    const int gs = (ns + 7) / 8, ng = (ns + gs - 1) / gs;
    // the two limits the kernels have: k_attn's group merge holds <= 16 split
    // partials (GMAX), o_proj's XF_ATTN_MERGE staging <= 8 group partials (with
    // gs = ceil(ns / 8) and ns <= 128 both hold by construction; checked, not
    // assumed -- tests/test_capi_cpu.py sweeps the plan against them)
    if (gs <= 16 && ng <= 8) {
      P.nsplit = ns;
      P.chunk = ch;
      P.group = gs;
      P.ngroups = ng;
    }
  }
  return P;
}
// diagnostic: out = {prefill, nsplit, chunk, defer, group, ngroups}
extern "C" int vv_attn_pass_plan(int ntok, int lm_slots, int head_dim, int n_kv, int max_pos_p1, int* out) {
  if (!out || ntok <= 0 || max_pos_p1 <= 0) return 1;
  const AttnPassPlan P = attn_pass_plan(ntok, lm_slots, head_dim, n_kv, max_pos_p1);
  const int v[6] = {P.prefill, P.nsplit, P.chunk, P.defer, P.group, P.ngroups};
  for (int i = 0; i < 6; ++i) out[i] = v[i];
  return 0;
}

static int lm_begin(vv_ctx* c, LmPass& P, int ntok, const void* embeds, int embed_rows, const int* slot,
                    const int* pos, int max_pos_p1) {
  if (!c->finalized) FAIL("vv_lm_forward before vv_finalize");
  if (max_pos_p1 > c->cfg.max_ctx) FAIL("position beyond max_ctx");
  const vv_config& k = c->cfg;
  const int H = k.hidden, d = k.head_dim, I = k.intermediate, nhd = k.n_heads * d;
  const size_t per = (size_t)H * 3 + c->qkv_n + nhd * 2 + I;
  if ((size_t)ntok > c->lm_ws_tokens) {
    // + 16 act rows: a packed act block (vv_norm_pack) rounds the rows up to 16
    CHK(c->lm_ws.ensure((per * ntok + (size_t)16 * I) * sizeof(bf16) + 256));
    c->lm_ws_tokens = ntok;
  }
  P.ntok = ntok;
  P.maxp = max_pos_p1;
  P.h = (bf16*)c->lm_ws.p;
  bf16* a = P.h + (size_t)ntok * H;
  bf16* qkv = a + (size_t)ntok * H;
  P.q = qkv + (size_t)ntok * c->qkv_n;
  P.att = P.q + (size_t)ntok * nhd;
  P.act = P.att + (size_t)ntok * nhd;
  const AttnPassPlan ap = attn_pass_plan(ntok, c->lm_slots, k.head_dim, k.n_kv_heads, max_pos_p1);
  P.prefill = ap.prefill;
  P.nsplit = ap.nsplit;
  P.chunk = ap.chunk;
  P.defer = ap.defer;
  P.group = ap.group;
  P.ngroups = ap.ngroups;
  if (P.nsplit > 1) {
    if ((size_t)ntok * k.n_kv_heads * std::max(1, P.ngroups) > 65536) FAIL("attention split tickets exhausted");
    CHK(c->attn_part.ensure((size_t)ntok * k.n_heads * (P.nsplit + P.ngroups) * (d + 2) * sizeof(float)));
  }
  // token row m reads embeds row m % embed_rows (the negative CFG rows consume the
  // positive rows' embeddings, :594-596); layer 0's attention residual writes h
  if (embed_rows <= 0 || embed_rows > ntok) embed_rows = ntok;
  P.in_m = rowmap(embeds, H, embed_rows, 0);
  P.hm = rowmap(P.h, H);
  P.slot = slot;
  P.pos = pos;
  P.inv_freq = (const float*)W(c, "lm.inv_freq");
  return 0;
}

// residual epilogue of a row-parallel projection: rank 0 adds the residual,
// the other ranks contribute their partial only (the all-reduce sums them)
static void tp_residual(vv_ctx* c, GemmArgs& g, const RowMap& res) {
  if (c->tp_rank == 0) {
    g.epi.kind = EPI_RES;
    g.epi.res = res;
  } else {
    g.epi.kind = EPI_STORE;
  }
}

// the LM attention half at decode in one launch (lm_attn.hip): <= 16 rows of the
// 1.5B shapes, contexts <= LA_MAX_KEYS, unsharded, while the context is the
// device's only registered one; 0 = the three launches (q|k|v, k_attn, o_proj)
static std::atomic<int> g_lm_attn{1};
static std::atomic<unsigned long long*> g_lm_attn_stamps{nullptr};
extern "C" int vv_lm_attn(int on) {
  g_lm_attn = on & 15;   // bits 1..3 (A/B): clear those LmAttnArgs::variant bits
  return 0;
}
extern "C" int vv_lm_attn_stamps(void* buf) {   // diagnostic: k_lm_attn launches record [256][16] phase stamps
  g_lm_attn_stamps = (unsigned long long*)buf;
  return 0;
}
static bool lm_attn_on(vv_ctx* c, const LmPass& P) {
  const vv_config& k = c->cfg;
  return g_lm_attn && c->la_part.p && c->lf_sync.p && !P.prefill && c->tp_size == 1 && !c->comm &&
         c->qkv_n == (k.n_heads + 2 * k.n_kv_heads) * k.head_dim && !P.hm.idx && P.hm.sT == k.hidden &&
         P.hm.T >= P.ntok && P.maxp <= std::min(k.max_ctx, LA_MAX_KEYS) &&
         lm_attn_fits(k.hidden, k.n_heads, k.n_kv_heads, k.head_dim, P.ntok, P.maxp) &&
         lm_attn_part_floats(P.ntok, P.maxp) * sizeof(float) <= c->la_part.bytes && persist_on(c);
}
extern "C" int vv_lm_attn_active(vv_ctx* c, int ntok, int max_pos_p1) {
  if (!c || !c->finalized) return 0;
  LmPass P;
  P.ntok = ntok;
  P.maxp = max_pos_p1;
  P.prefill = attn_use_prefill(ntok, c->lm_slots) ? 1 : 0;
  P.hm = rowmap(nullptr, c->cfg.hidden);
  return lm_attn_on(c, P) ? 1 : 0;
}

// input_layernorm .. o_proj (+ residual on rank 0)
static int lm_attn_half(vv_ctx* c, LmPass& P, int l, hipStream_t st) {
  const vv_config& k = c->cfg;
  const int H = k.hidden, d = k.head_dim, nhd = k.n_heads * d;
  const std::string p = "lm." + std::to_string(l);
  {
    // input_layernorm -> q|k|v projection (+bias) -> RoPE -> q / KV cache, one launch
    GemmArgs g = gemm_args(c, P.ntok, c->qkv_n, H, l == 0 ? P.in_m : P.hm, W(c, p + ".qkv_w"), EPI_ROPE, RowMap{},
                           W(c, p + ".qkv_b"));
    g.xf = xf_norm(W(c, p + ".in_norm"), k.rms_eps);
    g.rope.nh = k.n_heads;
    g.rope.nkv = k.n_kv_heads;
    g.rope.layer = l;
    g.rope.q_out = P.q;
    g.rope.slots = P.slot;
    g.rope.pos = P.pos;
    g.rope.inv_freq = P.inv_freq;
    g.rope.cs_tab = g_rope_tab ? (const bf16*)c->rope_tab.p : nullptr;
    g.rope.kv = c->kv;
    if (lm_attn_on(c, P)) {
      LmAttnArgs a;
      memset(&a, 0, sizeof(a));
      a.qkv = g;
      a.nw = W(c, p + ".in_norm");
      a.eps = k.rms_eps;
      a.scale = 1.0f / sqrtf((float)d);
      a.R = P.ntok;
      a.ow = W(c, p + ".o_w");
      a.res = l == 0 ? P.in_m : P.hm;
      a.out = P.hm;
      a.att = P.att;
      a.part = (float*)c->la_part.p;
      a.sync = (unsigned*)c->lf_sync.p;
      a.err = (unsigned*)c->hf_sync.p + 10 * 32;
      a.stamps = g_lm_attn_stamps.load();
      a.variant = 7 ^ (g_lm_attn.load() >> 1);
      KCHK(launch_lm_attn(a, P.maxp, st));
      return 0;
    }
    CHK(gemm(c, g, st));
  }
  AttnArgs at;
  memset(&at, 0, sizeof(at));
  at.stamps = g_attn_stamps;
  at.nq = P.ntok;
  at.nh = k.n_heads;
  at.nkv = k.n_kv_heads;
  at.layer = l;
  at.nsplit = P.nsplit;
  at.chunk = P.chunk;
  at.prefill = P.prefill;
  at.defer = P.defer;
  at.counters = (unsigned*)c->attn_cnt.p;
  at.scale = 1.0f / sqrtf((float)d);
  at.q = P.q;
  at.out = P.att;
  at.slots = P.slot;
  at.pos = P.pos;
  at.kv = c->kv;
  at.part_o = (float*)c->attn_part.p;
  at.part_ml = at.part_o ? at.part_o + (size_t)P.ntok * k.n_heads * P.nsplit * d : nullptr;
  at.group = P.group;
  at.ngroups = P.ngroups;
  if (P.group) {
    at.part_o2 = at.part_ml + (size_t)P.ntok * k.n_heads * P.nsplit * 2;
    at.part_ml2 = at.part_o2 + (size_t)P.ntok * k.n_heads * P.ngroups * d;
  }
  KCHK(launch_attn(at, st));
  GemmArgs g = gemm_args(c, P.ntok, H, nhd, rowmap(P.att, nhd), W(c, p + ".o_w"), EPI_RES, P.hm);
  if (P.defer) {
    g.xf.kind = XF_ATTN_MERGE;
    g.xf.part_o = at.part_o;
    g.xf.part_ml = at.part_ml;
    g.xf.qpos = P.pos;
    g.xf.nsplit = P.nsplit;
    g.xf.chunk = P.chunk;
  } else if (P.group) {   // the groups' partials: group g spans keys [g, g + 1) x group x chunk
    g.xf.kind = XF_ATTN_MERGE;
    g.xf.part_o = at.part_o2;
    g.xf.part_ml = at.part_ml2;
    g.xf.qpos = P.pos;
    g.xf.nsplit = P.ngroups;
    g.xf.chunk = P.group * P.chunk;
  }
  tp_residual(c, g, l == 0 ? P.in_m : P.hm);
  CHK(gemm(c, g, st));
  return 0;
}

// the LM MLP block in one launch (lm_ffn.hip) at decode with <= 2 rows, unsharded,
// while the context is the device's only registered one; 0 = two GEMV launches
static std::atomic<int> g_lm_ffn{1};
static std::atomic<unsigned long long*> g_lm_ffn_stamps{nullptr};
extern "C" int vv_lm_ffn_stamps(void* buf) {   // diagnostic: k_lm_ffn16 launches record [256][16] phase stamps
  g_lm_ffn_stamps = (unsigned long long*)buf;
  return 0;
}
extern "C" int vv_lm_ffn(int on) {   // bit 0: on; bit 1: not at 3..16 rows (k_lm_ffn16)
  g_lm_ffn = on & 3;
  return 0;
}
static bool lm_ffn_on(vv_ctx* c, const LmPass& P) {
  const vv_config& k = c->cfg;
  const bool shape = P.ntok <= 2 ? lm_ffn_fits(k.hidden, k.intermediate, P.ntok)
                                 : (g_lm_ffn & 2) == 0 && c->lf_slab.p && lm_ffn16_fits(k.hidden, k.intermediate, P.ntok);
  return g_lm_ffn && c->lf_sync.p && !P.prefill && c->tp_size == 1 && !c->comm && !P.hm.idx && P.hm.sT == k.hidden &&
         P.hm.T >= P.ntok && shape && persist_on(c);
}
extern "C" int vv_lm_ffn_active(vv_ctx* c, int ntok) {
  LmPass P;
  P.ntok = ntok;
  P.hm = rowmap(nullptr, c->cfg.hidden);
  return c && c->finalized && lm_ffn_on(c, P) ? 1 : 0;
}

// post_attention_layernorm .. down_proj (+ residual on rank 0)
static int lm_mlp_half(vv_ctx* c, LmPass& P, int l, hipStream_t st) {
  const vv_config& k = c->cfg;
  const int H = k.hidden, I = k.intermediate;
  const std::string p = "lm." + std::to_string(l);
  if (lm_ffn_on(c, P)) {
    LmFfnArgs a;
    memset(&a, 0, sizeof(a));
    a.x = (const bf16*)P.hm.base;
    a.out = (bf16*)P.hm.base;
    a.ldx = H;
    a.R = P.ntok;
    a.eps = k.rms_eps;
    a.nw = W(c, p + ".post_norm");
    a.gu = W(c, p + ".gu_w");
    a.dn = W(c, p + ".down_w");
    a.act = P.act;
    a.sync = (unsigned*)c->lf_sync.p;
    a.err = (unsigned*)c->hf_sync.p + 10 * 32;
    a.slab = (float*)c->lf_slab.p;
    a.stamps = g_lm_ffn_stamps.load();
    if (P.ntok <= 2) KCHK(launch_lm_ffn(a, st));
    else KCHK(launch_lm_ffn16(a, st));
    return 0;
  }
  // post_attention_layernorm fused into gate|up's A load
  GemmArgs g = gemm_args(c, P.ntok, 2 * I, H, P.hm, W(c, p + ".gu_w"), EPI_SILU_MUL, rowmap(P.act, I));
  g.xf = xf_norm(W(c, p + ".post_norm"), k.rms_eps);
  GemmArgs d = gemm_args(c, P.ntok, H, I, rowmap(P.act, I), W(c, p + ".down_w"), EPI_RES, P.hm);
  tp_residual(c, d, P.hm);
  // prefill: SiLU*up written MFMA-fragment-packed for the down projection when
  // both take the 256 x 256 tile (16K rows: down 449 -> 388 us)
  GemmArgs gp = g;
  gp.xf.kind = XF_NONE;
  if (g_norm_pack && I % 32 == 0 && gemm_uses_xl(gp) && gemm_uses_xl(d)) {
    g.epi.pack = 1;
    d.apack = 1;
  }
  CHK(gemm(c, g, st));
  CHK(gemm(c, d, st));
  return 0;
}

// Diagnostic (bench.py's roofline of the LM MLP block): `reps` passes over the
// LM layers' MLP blocks alone on `ntok` decode rows (hidden [ntok][H], act
// [ntok][I] scratch), as lm_mlp_half runs them (k_lm_ffn or the GEMV pair).
extern "C" int vv_lm_mlp_replay(vv_ctx* c, int ntok, void* hidden, void* act, int reps, vv_stream vst) {
  if (!c || !c->finalized || ntok < 1 || ntok > 2 * c->cfg.max_batch || !hidden || !act)
    FAIL("vv_lm_mlp_replay: bad arguments");
  LmPass P;
  P.ntok = ntok;
  P.h = (bf16*)hidden;
  P.hm = rowmap(hidden, c->cfg.hidden);
  P.act = (bf16*)act;
  for (int r = 0; r < reps; ++r)
    for (int l = 0; l < c->cfg.n_layers; ++l) CHK(lm_mlp_half(c, P, l, (hipStream_t)vst));
  return 0;
}

// Benchmarks only (bench.py --tp: the collective's share of an LM pass):
// skip the all-reduces of a communicator engine — the outputs are then wrong.
static std::atomic<int> g_tp_null{0};
extern "C" int vv_tp_null_collective(int on) {
  g_tp_null = on ? 1 : 0;
  return 0;
}

static int tp_allreduce(vv_ctx* c, LmPass& P, hipStream_t st) {
  if (!c->comm) {
    if (c->tp_size > 1) FAIL("tensor-parallel engine without a communicator (vv_tp_init)");
    return 0;
  }
  if (g_tp_null) return 0;
  const ncclResult_t r = ncclAllReduce(P.h, P.h, (size_t)P.ntok * c->cfg.hidden, ncclBfloat16, ncclSum, c->comm, st);
  if (r != ncclSuccess) FAIL(std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  return 0;
}

static int lm_end(vv_ctx* c, LmPass& P, int nout, const int* out_idx, void* hidden_out, float* logits_out,
                  hipStream_t st) {
  if (nout <= 0) return 0;
  const vv_config& k = c->cfg;
  // gather the output rows + final norm + the valid-id lm_head rows, one launch
  KCHK(launch_final_head(nout, k.hidden, P.h, out_idx, W(c, "lm.norm"), k.rms_eps, (bf16*)hidden_out,
                         W(c, "lm.lm_head"), (const int*)c->valid_ids.p, logits_out ? c->n_valid : 0, logits_out,
                         st));
  return 0;
}

int vv_lm_forward(vv_ctx* c, int ntok, const void* embeds, int embed_rows, const int* slot, const int* pos,
                  int max_pos_p1, int nout, const int* out_idx, void* hidden_out, float* logits_out, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (ntok <= 0) return 0;
  LmPass P;
  CHK(lm_begin(c, P, ntok, embeds, embed_rows, slot, pos, max_pos_p1));
  for (int l = 0; l < c->cfg.n_layers; ++l) {
    CHK(lm_attn_half(c, P, l, st));
    CHK(tp_allreduce(c, P, st));
    CHK(lm_mlp_half(c, P, l, st));
    CHK(tp_allreduce(c, P, st));
  }
  return lm_end(c, P, nout, out_idx, hidden_out, logits_out, st);
}

// Diagnostic (bench.py's candidate roofline of the LM attention half): `reps`
// passes over the LM layers' attention halves alone on `ntok` decode rows
// (embeds [ntok][H] as layer 0's input; later layers read / write the pass's own
// hidden rows), as lm_attn_half runs them (k_lm_attn or the three launches).
extern "C" int vv_lm_attn_replay(vv_ctx* c, int ntok, const void* embeds, const int* slot, const int* pos,
                                 int max_pos_p1, int reps, vv_stream vst) {
  if (!c || !c->finalized || ntok < 1 || ntok > 2 * c->cfg.max_batch || !embeds || !slot || !pos)
    FAIL("vv_lm_attn_replay: bad arguments");
  LmPass P;
  CHK(lm_begin(c, P, ntok, embeds, ntok, slot, pos, max_pos_p1));
  for (int r = 0; r < reps; ++r)
    for (int l = 0; l < c->cfg.n_layers; ++l) CHK(lm_attn_half(c, P, l, (hipStream_t)vst));
  return 0;
}

int vv_lm_forward_group(int n, vv_ctx* const* ctxs, int ntok, const void* embeds, int embed_rows, const int* slot,
                        const int* pos, int max_pos_p1, int nout, const int* out_idx, void* hidden_out,
                        float* logits_out, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (n < 1 || n > 8) FAIL("vv_lm_forward_group: 1..8 ranks");
  if (ntok <= 0) return 0;
  std::vector<LmPass> P(n);
  SumRows sr;
  sr.n = n;
  for (int r = 0; r < n; ++r) {
    if (ctxs[r]->tp_rank != r || ctxs[r]->tp_size != n) FAIL("vv_lm_forward_group: engine r must be TP rank r of n");
    CHK(lm_begin(ctxs[r], P[r], ntok, embeds, embed_rows, slot, pos, max_pos_p1));
    sr.p[r] = P[r].h;
  }
  const long long count = (long long)ntok * ctxs[0]->cfg.hidden;
  for (int l = 0; l < ctxs[0]->cfg.n_layers; ++l) {
    for (int r = 0; r < n; ++r) CHK(lm_attn_half(ctxs[r], P[r], l, st));
    KCHK(launch_sum_rows(sr, count, st));
    for (int r = 0; r < n; ++r) CHK(lm_mlp_half(ctxs[r], P[r], l, st));
    KCHK(launch_sum_rows(sr, count, st));
  }
  return lm_end(ctxs[0], P[0], nout, out_idx, hidden_out, logits_out, st);
}

int vv_tp_unique_id(void* out, int nbytes) {
  if (nbytes < (int)sizeof(ncclUniqueId)) FAIL("vv_tp_unique_id: buffer smaller than ncclUniqueId");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) FAIL(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
}

int vv_tp_init(vv_ctx* c, int rank, int size, const void* unique_id) {
  if (size < 1 || rank < 0 || rank >= size) FAIL("vv_tp_init: bad rank / size");
  c->tp_rank = rank;
  c->tp_size = size;
  if (!unique_id) return 0;  // group emulation in one process: no communicator
  HIPCHK(hipSetDevice(c->device));
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  const ncclResult_t r = ncclCommInitRank(&c->comm, size, id, rank);
  if (r != ncclSuccess) FAIL(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  return 0;
}

// Every grid-wait counter of the context back to 0 and the error word cleared,
// with nothing in flight (the device is synchronised): after a wait gave up, the
// counters of that launch stay part-advanced, and a later launch's base
// generation (persist_dev.h) would let a wait release early.
int vv_sync_reset(vv_ctx* c) {
  if (!c->finalized) FAIL("vv_sync_reset before vv_finalize");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipDeviceSynchronize());
  for (DevBuf* b : {&c->hf_sync, &c->cs_sync, &c->lf_sync})
    if (b->p) HIPCHK(hipMemset(b->p, 0, SYNC_BYTES));
  if (c->cw_sync.p) HIPCHK(hipMemset(c->cw_sync.p, 0, c->cw_sync.bytes));
  HIPCHK(hipDeviceSynchronize());
  return 0;
}
// A grid wait of a one-launch kernel gave up (workgroups not co-resident):
// every output since the last call is invalid.  Reset on read (with the wait
// counters: vv_sync_reset).
// (hipMemcpy on the null stream does not wait for non-blocking streams, where
// the host's generate() runs: synchronise the device first)
int vv_sync_error(vv_ctx* c) {
  unsigned v = 0;
  if (c->hf_sync.p) {
    HIPCHK(hipDeviceSynchronize());
    if (hipMemcpy(&v, (unsigned*)c->hf_sync.p + 10 * 32, 4, hipMemcpyDeviceToHost) != hipSuccess)
      FAIL("vv_sync_error: reading the error word failed (hipMemcpy)");
    if (v) CHK(vv_sync_reset(c));
  }
  return v ? 1 : 0;
}
// Stream-ordered form: enqueue on st a copy of the error word to dst (4 bytes of
// pinned host or device memory) and its reset, behind everything queued before.
// The host reads dst once an event recorded after this call has completed
// (GenerateSession: with each step's logits read-back, and before audio leaves
// for a streamer); when it reads 1 it calls vv_sync_reset before anything else.
int vv_sync_error_async(vv_ctx* c, void* dst, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!dst) FAIL("vv_sync_error_async: dst is NULL");
  if (!c->finalized) FAIL("vv_sync_error_async before vv_finalize");
  unsigned* word = (unsigned*)c->hf_sync.p + 10 * 32;
  HIPCHK(hipMemcpyAsync(dst, word, 4, hipMemcpyDefault, st));
  HIPCHK(hipMemsetAsync(word, 0, 4, st));
  return 0;
}
// Per-context switch of the grid-waiting kernels (default: on unless
// VIBEVOICE_PERSISTENT=0).  Off: the context neither launches them nor counts in
// the device's registry, so it never demotes another context (the standalone
// tokenizer API's codec context) nor contends with it.  Bumps the workspace
// epoch: graphs captured with the other path are re-captured.
int vv_set_persistent(vv_ctx* c, int on) {
  if (!c) FAIL("vv_set_persistent: null context");
  if (on < 0 || on > 2) FAIL("vv_set_persistent: 0 (off), 1 (on) or 2 (follow)");
  c->persist_ok = on != 0;
  c->persist_follow = on == 2;
  if (on == 2) c->persist_ok = true;
  if (c->finalized) {
    if ((!c->persist_ok || c->persist_follow) && c->hl_registered) {
      c->hl_registered = false;
      hl_register(c->device, -1);
    } else if (c->persist_ok && !c->persist_follow && c->persist_capable && !c->hl_registered) {
      c->hl_registered = true;
      hl_register(c->device, +1);
    }
  }
  g_ws_epoch.fetch_add(1);
  return 0;
}
int vv_persistent_active(vv_ctx* c) { return c && c->finalized && persist_on(c) ? 1 : 0; }
// Diagnostic (tests): raise the error word as a grid wait that gave up would.
extern "C" int vv_diag_raise_sync_error(vv_ctx* c) {
  if (!c->finalized) FAIL("vv_diag_raise_sync_error before vv_finalize");
  HIPCHK(hipDeviceSynchronize());
  const unsigned one = 1;
  HIPCHK(hipMemcpy((unsigned*)c->hf_sync.p + 10 * 32, &one, 4, hipMemcpyHostToDevice));
  // ... and leave the counters part-advanced as a launch that gave up does: 5
  // arrivals on shard 0, 3 generation bumps (lines 11 and 12) of every family
  for (DevBuf* b : {&c->hf_sync, &c->cs_sync, &c->lf_sync}) {
    if (!b->p) continue;
    for (int line : {0, 11, 12}) {
      unsigned v = 0;
      unsigned* p = (unsigned*)b->p + line * 32;
      HIPCHK(hipMemcpy(&v, p, 4, hipMemcpyDeviceToHost));
      v += line == 0 ? 5u : 3u;
      HIPCHK(hipMemcpy(p, &v, 4, hipMemcpyHostToDevice));
    }
  }
  return 0;
}
// Diagnostic (tests): word 0 of the 13 counter lines of each wait family
// (head, codec stage, LM MLP) -> out[39].  Between launches a consistent set has
// every shard line (0-7) a multiple of 32 and every generation line a multiple of 8.
extern "C" int vv_diag_sync_words(vv_ctx* c, unsigned* out) {
  if (!c->finalized) FAIL("vv_diag_sync_words before vv_finalize");
  HIPCHK(hipDeviceSynchronize());
  int i = 0;
  for (DevBuf* b : {&c->hf_sync, &c->cs_sync, &c->lf_sync})
    for (int line = 0; line < 13; ++line, ++i) {
      out[i] = 0;
      if (b->p) HIPCHK(hipMemcpy(out + i, (unsigned*)b->p + line * 32, 4, hipMemcpyDeviceToHost));
    }
  return 0;
}

// ------------------------------------------------------------------ diffusion head
// One rank's buffers and operands of a vv_diffusion_sample call.
struct HeadRun {
  int n = 0, R = 0;
  long long MODW = 0;
  bf16 *cat = nullptr, *condp = nullptr, *xh = nullptr, *mods = nullptr, *sa = nullptr, *act = nullptr, *v = nullptr,
       *m1 = nullptr;
  bf16 *xh2 = nullptr, *lat2 = nullptr, *m12 = nullptr;   // k_head_fin's double buffers (state rows, latents, history)
  const bf16* cond = nullptr;
  RowMap xh_m;
  bool keep = false;
};

// layout, condition rows and cond_proj (step-invariant: once per token)
static int head_begin(vv_ctx* c, int n, const void* pos_h, const void* neg_h, HeadRun& h, hipStream_t st) {
  const vv_config& k = c->cfg;
  const int H = k.hidden, F = k.head_ffn, D = k.latent_dim, L = k.head_layers;
  h.n = n;
  h.R = 2 * n;
  h.MODW = (3LL * L + 2) * H;
  const int R = h.R;
  h.cat = (bf16*)c->head_ws.p;
  h.condp = h.cat + (size_t)R * H;
  bf16* sc = h.condp + (size_t)R * H;
  h.xh = sc + (size_t)R * H;
  bf16* a = h.xh + (size_t)R * H;
  h.mods = a + (size_t)R * H;                             // [HEAD_SC steps][R][MODW]
  h.sa = h.mods + (size_t)HEAD_SC * R * h.MODW;           // [HEAD_SC steps][R][H] adaLN inputs
  h.act = h.sa + (size_t)HEAD_SC * R * H;
  h.v = h.act + (size_t)R * F;
  h.m1 = h.v + (size_t)R * D;
  h.lat2 = h.m1 + (size_t)R * D;        // (head_ws: R * D * 3 + max_batch * D * 2 after act)
  h.m12 = h.lat2 + (size_t)R * D;
  h.xh2 = a;                            // (head_ws: the spare [R][H] after xh)
  h.xh_m = rowmap(h.xh, H);
  // condition rows cat[pos_h, neg_h]: used in place when the caller's rows are adjacent
  h.cond = (const bf16*)pos_h;
  if ((const bf16*)neg_h != (const bf16*)pos_h + (size_t)n * H) {
    HIPCHK(hipMemcpyAsync(h.cat, pos_h, (size_t)n * H * sizeof(bf16), hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(h.cat + (size_t)n * H, neg_h, (size_t)n * H * sizeof(bf16), hipMemcpyDeviceToDevice, st));
    h.cond = h.cat;
  }
  // the per-step head weights (noisy, gate|up, down, final: 170 MB at 1.5B) are
  // re-read by every diffusion step: default cache policy keeps them in the
  // Infinity Cache (256 MB) across the S steps.  VibeVoice-Large's (925 MB per
  // step; 231 MB per rank at TP = 4) stream non-temporal like the LM's
  h.keep = (size_t)L * 3 * F * H * sizeof(bf16) <= (192ull << 20) && !(c->head_tp && c->tp_size > 1);
  CHK(gemm(c, gemm_args(c, R, H, H, rowmap(h.cond, H), W(c, "head.cond_w"), EPI_STORE, rowmap(h.condp, H)), st));
  return 0;
}

static int head_gemm(vv_ctx* c, const HeadRun& h, GemmArgs g, hipStream_t st) {
  g.keep = h.keep ? 1 : 0;
  return gemm(c, g, st);
}

// all adaLN modulations ([shift|scale|gate] x L, [shift|scale] final) of up to
// HEAD_SC steps in ONE GEMM: the condition is step-invariant and the timesteps
// are the schedule's, so silu(cond_proj(c) + t_emb[s]) is known for every step
// up front -- the 3LH+2H x H adaLN matrix is read once per chunk, not per step
static int head_mods(vv_ctx* c, const HeadRun& h, int s, hipStream_t st) {
  if (s % HEAD_SC) return 0;
  const int H = c->cfg.hidden, sc = std::min(HEAD_SC, c->steps - s);
  KCHK(launch_head_cond(sc, h.R, H, h.condp, (const bf16*)c->temb.p + (size_t)s * H, h.sa, st));
  CHK(gemm(c, gemm_args(c, sc * h.R, (int)h.MODW, H, rowmap(h.sa, H), W(c, "head.ada_w"), EPI_STORE,
                        rowmap(h.mods, h.MODW)), st));
  return 0;
}

// 2n <= 16 rows in the GEMV layout: the layer as one launch (head_m16.hip) while the context is
// the device's only registered one; 0 = two GEMV launches (A/B and tests)
static std::atomic<int> g_head_m16{1};
// layers l >= 1 build the A side distributed (HeadM16Args::pre) from the previous
// layer's row partials; 0 = every workgroup transforms the whole A side
static std::atomic<int> g_head_m16_pre{1};
extern "C" int vv_head_m16_pre(int on) {
  g_head_m16_pre = on;
  return 0;
}
static std::atomic<unsigned long long*> g_head_m16_stamps{nullptr};
extern "C" int vv_head_m16_stamps(void* buf) {   // diagnostic: [256][16] per-workgroup phase stamps
  g_head_m16_stamps = (unsigned long long*)buf;
  return 0;
}
extern "C" int vv_head_m16(int on) {
  g_head_m16 = on;   // A/B variants: bit 1 / bit 3 HeadM16Args::a_first on / off (default: > 8 rows),
                     // bit 2 the down weights' earlier issue point
  return 0;
}
// the one-launch layer applies (R <= 16 rows, GEMV layout, unsharded, sole context)
static bool m16_on(vv_ctx* c, int R) {
  return g_head_m16 && !c->head_tp && c->head_gemv && c->m16_buf.p && head_m16_fits(c->cfg.hidden, c->cfg.head_ffn, R) &&
         persist_on(c);
}

// ... with the A side built distributed (HeadM16Args::pre) above 4 rows: at 2 -
// 4 rows the whole A side is 18 - 36 KB per CU and the extra grid wait costs more
// than it saves (n = 1 head sample 659 us whole vs 688 us distributed,
// tools/head_m16_stamps.py)
static bool m16_pre(vv_ctx* c, int R) { return g_head_m16_pre && R > 4 && m16_on(c, R); }

// x = noisy_images_proj(cat[x, x])  -- both halves read the same n latent rows
static int head_noisy(vv_ctx* c, const HeadRun& h, const void* x_io, hipStream_t st) {
  const int H = c->cfg.hidden, D = c->cfg.latent_dim;
  if (m16_pre(c, h.R)) {   // + the row partials layer 0's distributed A side reads
    HeadNoisyArgs a;
    a.lat = (const bf16*)x_io;
    a.w = (const bf16*)W(c, "head.noisy_w");
    a.x = (bf16*)h.xh;
    a.ssp = (float*)c->m16_buf.p;
    a.n = h.n;
    a.R = h.R;
    a.D = D;
    a.ldx = H;
    KCHK(launch_head_noisy16(a, st));
    return 0;
  }
  return head_gemm(c, h, gemm_args(c, h.R, H, D, rowmap(x_io, D, h.n, 0), W(c, "head.noisy_w"), EPI_STORE, h.xh_m),
                   st);
}

extern "C" int vv_head_m16_active(vv_ctx* c, int n) {
  const vv_config& k = c->cfg;
  return c && c->finalized && g_head_m16 && !c->head_tp && c->head_gemv && head_m16_fits(k.hidden, k.head_ffn, 2 * n) &&
                 persist_on(c)
             ? 1
             : 0;
}
// layer l of step s: modulate(norm(x)) -> gate|up -> SiLU*up -> down -> x += gate * (.)
// With the FFN sharded (vv_tp_shard_head) this rank holds head_ffn / tp_size of
// the hidden columns: gate|up column-parallel, down row-parallel; rank 0 adds
// the residual, the others contribute gate * partial only (onto zero rows), and
// the caller sums x over the ranks (all-reduce).
static int head_layer(vv_ctx* c, const HeadRun& h, int s, int l, hipStream_t st) {
  const vv_config& k = c->cfg;
  const int H = k.hidden, F = k.head_ffn;
  const std::string p = "head." + std::to_string(l);
  const bf16* mod = h.mods + (size_t)(s % HEAD_SC) * h.R * h.MODW;
  const int o = 3 * H * l;
  // modulate(norm(x), shift, scale) fused into gate|up's A load
  GemmArgs g = gemm_args(c, h.R, 2 * F, H, h.xh_m, W(c, p + ".gu_w"), EPI_SILU_MUL, rowmap(h.act, F));
  g.xf = xf_norm(W(c, p + ".norm"), k.head_eps, mod, h.MODW, o, o + H);
  const bool partial = c->head_tp && c->tp_size > 1 && c->tp_rank > 0;
  if (m16_on(c, h.R)) {
    // 2n <= 16 rows, GEMV layout: one launch with two grid-wide waits (head_m16.hip)
    HeadM16Args a;
    memset(&a, 0, sizeof(a));
    a.x = h.xh;
    a.out = h.xh;
    a.ldx = H;
    a.mod = mod;
    a.ldmod = h.MODW;
    a.shift_off = o;
    a.scale_off = o + H;
    a.gate_off = o + 2 * H;
    a.R = h.R;
    a.eps = k.head_eps;
    a.nw = W(c, p + ".norm");
    a.gu = W(c, p + ".gu_w");
    a.dn = W(c, p + ".down_w");
    a.act = h.act;
    a.sync = (unsigned*)c->hf_sync.p;
    a.err = (unsigned*)c->hf_sync.p + 10 * 32;
    a.stamps = g_head_m16_stamps;
    // the A side ahead of every weight load: at 16 rows (B = 8) a whole head
    // sample 890 -> 860 us, at 2 rows (B = 1) 595 -> 603 us (tools/head_m16_stamps.py)
    a.a_first = (g_head_m16.load() & 2) ? 1 : (g_head_m16.load() & 8) ? 0 : (h.R > 8 ? 1 : 0);
    a.late_down = (g_head_m16.load() & 4) ? 0 : 1;
    a.ssp = (float*)c->m16_buf.p;
    a.xt = (bf16*)((char*)c->m16_buf.p + 16 * 192 * sizeof(float));
    a.pre = m16_pre(c, h.R) ? 1 : 0;   // (layer 0: the partials of k_head_noisy16)
    KCHK(launch_head_m16(a, st));
    return 0;
  }
  if (!c->head_gemv)
    FAIL("diffusion head: " + std::to_string(h.R) + " rows need the GEMV layout (head.<l>.gu_w / down_w), which this "
         "engine did not bind (packed for max_batch <= 2: weights.head_layout_for)");
  CHK(head_gemm(c, h, g, st));
  g = gemm_args(c, h.R, H, F, rowmap(h.act, F), W(c, p + ".down_w"), EPI_RES, h.xh_m);
  g.epi.res = partial ? rowmap(c->zero_rows.p, H) : h.xh_m;
  g.epi.gate = rowmap(mod + o + 2 * H, h.MODW);
  return head_gemm(c, h, g, st);
}

// final layer: modulate(norm_final(x)) -> linear -> CFG + DPM-Solver++ step on x
static int head_final(vv_ctx* c, const HeadRun& h, int s, void* x_io, float cfg_scale, const float* sde_noise,
                      hipStream_t st) {
  const vv_config& k = c->cfg;
  const int H = k.hidden, D = k.latent_dim, L = k.head_layers;
  const bf16* mod = h.mods + (size_t)(s % HEAD_SC) * h.R * h.MODW;
  DpmCoef e = c->coef[s];
  e.cfg = cfg_scale;
  // sde-dpmsolver++: this step's [2n, D] fp32 draw; rows [0, n) update the live latents
  const float* zs = sde_noise ? sde_noise + (size_t)s * h.R * D : nullptr;
  GemmArgs g = gemm_args(c, h.R, D, H, h.xh_m, W(c, "head.final_w"), EPI_STORE, rowmap(h.v, D));
  g.xf = xf_norm(nullptr, k.head_eps, mod, h.MODW, 3 * H * L, 3 * H * L + H);
  if (h.R <= 16) {
    g.epi.kind = EPI_CFG_DPM;
    g.dpm.n = h.n;
    g.dpm.k = e;
    g.dpm.x = (bf16*)x_io;
    g.dpm.m1 = h.m1;
    g.dpm.noise = zs;
    CHK(head_gemm(c, h, g, st));
  } else {
    CHK(head_gemm(c, h, g, st));
    KCHK(launch_cfg_dpm(h.n, D, e, h.v, (bf16*)x_io, h.m1, zs, st));
  }
  return 0;
}

// Diagnostic (bench.py's roofline of the head FFN layer): the condition rows
// and step 0's modulations as vv_diffusion_sample sets them up, then `reps`
// passes over the head_layers FFN layers alone (the kernels the loop launches
// for them at this n: the fused layer, or gate|up + down), on stream st.
extern "C" int vv_head_layers_replay(vv_ctx* c, int n, const void* pos_h, const void* neg_h, int reps,
                                     vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!c->finalized || c->steps == 0) FAIL("vv_head_layers_replay: engine not finalized or no schedule");
  if (n <= 0 || n > c->cfg.max_batch) FAIL("vv_head_layers_replay: bad n");
  if (c->head_tp && (c->tp_size > 1 || c->comm)) FAIL("vv_head_layers_replay: sharded head");
  HeadRun h;
  CHK(head_begin(c, n, pos_h, neg_h, h, st));
  CHK(head_mods(c, h, 0, st));
  for (int r = 0; r < reps; ++r)
    for (int l = 0; l < c->cfg.head_layers; ++l) CHK(head_layer(c, h, 0, l, st));
  return 0;
}

int vv_tp_shard_head(vv_ctx* c, int on) {
  if (on && c->tp_size > 1 && c->cfg.head_ffn % 32) FAIL("vv_tp_shard_head: the local head FFN width must be a multiple of 32");
  c->head_tp = on ? 1 : 0;
  return 0;
}

// step s's final layer + DPM and step s + 1's noisy projection as ONE launch
// (head_fin.hip) at 2n <= 16 rows with the head's weights cache-resident; 0 = the
// two launches (A/B and tests)
static std::atomic<int> g_head_fin{1};
extern "C" int vv_head_fin(int on) {
  g_head_fin = on ? 1 : 0;
  return 0;
}
static bool head_fin_on(vv_ctx* c, const HeadRun& h) {
  const vv_config& k = c->cfg;
  return g_head_fin && !c->head_tp && h.keep && head_fin_fits(k.hidden, k.latent_dim, h.R) && c->steps >= 3;
}
extern "C" int vv_head_fin_active(vv_ctx* c, int n) {
  if (!c || !c->finalized) return 0;
  HeadRun h;
  h.n = n;
  h.R = 2 * n;
  const vv_config& k = c->cfg;
  h.keep = (size_t)k.head_layers * 3 * k.head_ffn * k.hidden * sizeof(bf16) <= (192ull << 20) && !(c->head_tp && c->tp_size > 1);
  return head_fin_on(c, h) ? 1 : 0;
}
// lat / m1 read, lat_out / m1_out written; the state rows h.xh read, xo written
static int head_fin(vv_ctx* c, const HeadRun& h, int s, const bf16* lat, bf16* lat_out, const bf16* m1, bf16* m1_out,
                    bf16* xo, float cfg_scale, const float* sde_noise, hipStream_t st) {
  const vv_config& k = c->cfg;
  const int H = k.hidden, D = k.latent_dim, L = k.head_layers;
  HeadFinArgs a;
  memset(&a, 0, sizeof(a));
  a.n = h.n;
  a.R = h.R;
  a.eps = k.head_eps;
  a.shift_off = 3 * H * L;
  a.scale_off = 3 * H * L + H;
  a.ldmod = h.MODW;
  a.x = h.xh;
  a.mod = h.mods + (size_t)(s % HEAD_SC) * h.R * h.MODW;
  a.fw = W(c, "head.final_w");
  a.k = c->coef[s];
  a.k.cfg = cfg_scale;
  a.lat = lat;
  a.lat_out = lat_out;
  a.m1 = m1;
  a.m1_out = m1_out;
  a.noise = sde_noise ? sde_noise + (size_t)s * h.R * D : nullptr;
  a.nw = W(c, "head.noisy_w");
  a.xo = xo;
  a.ssp = m16_pre(c, h.R) ? (float*)c->m16_buf.p : nullptr;   // (layer 0's distributed A side at > 4 rows)
  KCHK(launch_head_fin(a, st));
  return 0;
}

int vv_diffusion_sample(vv_ctx* c, int n, const void* pos_h, const void* neg_h, void* x_io, float cfg_scale,
                        const float* sde_noise, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!c->finalized || c->steps == 0) FAIL("vv_diffusion_sample: engine not finalized or no schedule");
  if (n <= 0) return 0;
  const vv_config& k = c->cfg;
  if (n > k.max_batch) FAIL("vv_diffusion_sample: n > max_batch");
  const bool sharded = c->head_tp && (c->tp_size > 1 || c->comm);   // (a 1-rank communicator: tests)
  if (sharded && !c->comm) FAIL("sharded diffusion head without a communicator (vv_tp_init; one process: "
                                "vv_diffusion_sample_group)");
  const int H = k.hidden, D = k.latent_dim, L = k.head_layers;
  HeadRun h;
  CHK(head_begin(c, n, pos_h, neg_h, h, st));
  const int R = h.R;
  const long long MODW = h.MODW;
  // k_head_fin fuses step s's final layer with step s + 1's noisy projection for
  // an EVEN number of steps [s0, S - 1), so that the latents, the DPM history and
  // the state rows ping-pong back to x_io / m1 / xh for the last step's final
  // layer (the GEMV path, in place)
  const bool fin = !sharded && head_fin_on(c, h);
  const int nfused = !fin ? 0 : (c->steps - 1) % 2 == 0 ? c->steps - 1 : c->steps - 2;
  const int s0 = c->steps - 1 - nfused;
  bf16* lat[2] = {(bf16*)x_io, h.lat2};
  bf16* hist[2] = {h.m1, h.m12};
  bf16* xs[2] = {h.xh, h.xh2};
  int cur = 0;
  for (int s = 0; s < c->steps; ++s) {
    h.xh = xs[cur];
    h.xh_m = rowmap(h.xh, H);
    h.m1 = hist[cur];
    CHK(head_mods(c, h, s, st));
    if (!(nfused && s > s0)) CHK(head_noisy(c, h, lat[cur], st));   // (else: the previous k_head_fin)
    for (int l = 0; l < L; ++l) {
      CHK(head_layer(c, h, s, l, st));
      if (sharded && !g_tp_null) {   // x = sum over the ranks (rank 0 carried the residual)
        const ncclResult_t r = ncclAllReduce(h.xh, h.xh, (size_t)R * H, ncclBfloat16, ncclSum, c->comm, st);
        if (r != ncclSuccess) FAIL(std::string("ncclAllReduce (head): ") + ncclGetErrorString(r));
      }
    }
    if (nfused && s >= s0 && s + 1 < c->steps) {
      CHK(head_fin(c, h, s, lat[cur], lat[cur ^ 1], hist[cur], hist[cur ^ 1], xs[cur ^ 1], cfg_scale, sde_noise, st));
      cur ^= 1;
    } else {
      CHK(head_final(c, h, s, lat[cur], cfg_scale, sde_noise, st));
    }
  }
  if (cur != 0) FAIL("vv_diffusion_sample: internal (latent buffers did not return)");
  return 0;
}

int vv_diffusion_sample_group(int nr, vv_ctx* const* ctxs, int n, const void* pos_h, const void* neg_h, void* x_io,
                              float cfg_scale, const float* sde_noise, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (nr < 1 || nr > 8) FAIL("vv_diffusion_sample_group: 1..8 ranks");
  if (n <= 0) return 0;
  HeadRun h[8];
  SumRows sr;
  sr.n = nr;
  for (int r = 0; r < nr; ++r) {
    vv_ctx* c = ctxs[r];
    if (c->tp_rank != r || c->tp_size != nr || !c->head_tp)
      FAIL("vv_diffusion_sample_group: engine r must be TP rank r of n with a sharded head (vv_tp_shard_head)");
    if (!c->finalized || c->steps != ctxs[0]->steps) FAIL("vv_diffusion_sample_group: engines not finalized alike");
    if (n > c->cfg.max_batch) FAIL("vv_diffusion_sample_group: n > max_batch");
    CHK(head_begin(c, n, pos_h, neg_h, h[r], st));
    sr.p[r] = h[r].xh;
  }
  const vv_config& k = ctxs[0]->cfg;
  const long long count = (long long)h[0].R * k.hidden;
  for (int s = 0; s < ctxs[0]->steps; ++s) {
    for (int r = 0; r < nr; ++r) {
      CHK(head_mods(ctxs[r], h[r], s, st));
      CHK(head_noisy(ctxs[r], h[r], x_io, st));
    }
    for (int l = 0; l < k.head_layers; ++l) {
      for (int r = 0; r < nr; ++r) CHK(head_layer(ctxs[r], h[r], s, l, st));
      KCHK(launch_sum_rows(sr, count, st));
    }
    // the latent update once (every rank would compute the same; rank 0's x is the sum)
    CHK(head_final(ctxs[0], h[0], s, x_io, cfg_scale, sde_noise, st));
  }
  return 0;
}

static int connector(vv_ctx* c, const char* which, int n, int din, RowMap x, RowMap out, const RowMap* res,
                     hipStream_t st) {
  const int H = c->cfg.hidden;
  const std::string p(which);
  bf16* t1 = (bf16*)c->codec_ws.p;
  bf16* t2 = t1 + (size_t)c->cfg.max_batch * H;
  RowMap t1m = rowmap(t1, H), t2m = rowmap(t2, H);
  CHK(gemm(c, gemm_args(c, n, H, din, x, W(c, p + ".fc1_w"), EPI_STORE, t1m, W(c, p + ".fc1_b")), st));
  // LlamaRMSNorm(eps=1e-6) (modeling_vibevoice.py:62) fused into fc2's A load
  GemmArgs g = gemm_args(c, n, H, H, t1m, W(c, p + ".fc2_w"), res ? EPI_RES : EPI_STORE, out, W(c, p + ".fc2_b"));
  g.xf = xf_norm(W(c, p + ".norm"), 1e-6f);
  if (res) g.epi.res = *res;
  CHK(gemm(c, g, st));
  return 0;
}

int vv_connector(vv_ctx* c, int which, int n, const void* x, void* out, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  const int H = c->cfg.hidden;
  const int din = which == 0 ? c->cfg.latent_dim : c->cfg.semantic_dim;
  // chunk rows through the max_batch-sized connector workspace
  for (int r0 = 0; r0 < n; r0 += c->cfg.max_batch) {
    const int m = std::min(c->cfg.max_batch, n - r0);
    CHK(connector(c, which == 0 ? "conn.ac" : "conn.se", m, din, rowmap((const bf16*)x + (size_t)r0 * din, din),
                  rowmap((bf16*)out + (size_t)r0 * H, H), nullptr, st));
  }
  return 0;
}

int vv_codec_step(vv_ctx* c, int n, const int* slots, const void* latent, void* audio_out, void* sem_out,
                  void* embeds_out, const int* embed_rows, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!c->finalized) FAIL("vv_codec_step before vv_finalize");
  if (n <= 0) return 0;
  if (n > c->cfg.max_batch) FAIL("vv_codec_step: n > max_batch");
  const int H = c->cfg.hidden, D = c->cfg.latent_dim, S = c->cfg.semantic_dim;
  ConvNet& dn = c->dec;
  ConvNet& sn = c->sem;
  const int hop = dn.T[dn.nst - 1];
  // decoder input: latent / scaling - bias  (modeling_vibevoice_inference.py:651)
  KCHK(launch_latent_to_dec(n, D, (const bf16*)latent, W(c, "speech_scaling_factor"), W(c, "speech_bias_factor"),
                            buf_in_rows(dn.stem, 1, slots), st));
  // decoder -> audio chunk (also written as the semantic encoder's input rows)
  CHK(convnet_run(c, dn, n, slots, rowmap(audio_out, 1, hop, hop), buf_in_rows(sn.stem, hop, slots), st));
  CHK(convnet_roll(dn, n, slots, 0, st));
  // semantic encoder -> [n, S]
  bf16* sem = sem_out ? (bf16*)sem_out : (bf16*)c->codec_ws.p + (size_t)c->cfg.max_batch * 2 * H;
  CHK(convnet_run(c, sn, n, slots, rowmap(sem, S, 1, S), RowMap{}, st));
  CHK(convnet_roll(sn, n, slots, 0, st));
  // next input embedding = acoustic_connector(latent) + semantic_connector(sem)  (:682-687)
  if (embeds_out) {
    bf16* ac = (bf16*)c->codec_ws.p + (size_t)c->cfg.max_batch * 3 * H;
    RowMap acm = rowmap(ac, H);
    CHK(connector(c, "conn.ac", n, D, rowmap(latent, D), acm, nullptr, st));
    RowMap outm = rowmap(embeds_out, H, 1, H, embed_rows);
    CHK(connector(c, "conn.se", n, S, rowmap(sem, S), outm, &acm, st));
  }
  return 0;
}

int vv_codec_reset(vv_ctx* c, int n, const int* slots, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (n <= 0) return 0;
  CHK(convnet_roll(c->dec, n, slots, 1, st));
  CHK(convnet_roll(c->sem, n, slots, 1, st));
  return 0;
}

// The two halves of vv_codec_step as separate calls: the reference's standalone
// tokenizer API (acoustic_tokenizer.decode / semantic_tokenizer.encode with a
// VibeVoiceTokenizerStreamingCache, modular_vibevoice_tokenizer.py:1081-1108,
// 193-256), one frame per call.  Slot state is the same per-slot ConvBuf
// history vv_codec_step keeps.
int vv_codec_decode(vv_ctx* c, int n, const int* slots, const void* z, void* audio_out, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!c->finalized) FAIL("vv_codec_decode before vv_finalize");
  if (n <= 0) return 0;
  if (n > c->cfg.max_batch) FAIL("vv_codec_decode: n > max_batch");
  ConvNet& dn = c->dec;
  const int hop = dn.T[dn.nst - 1];
  // z is already the decoder input (latent / scaling - bias, done by the caller):
  // identity scale / bias keep the copy bit-exact
  const bf16* one = (const bf16*)c->unit_sb.p;
  KCHK(launch_latent_to_dec(n, c->cfg.latent_dim, (const bf16*)z, one, one + 1, buf_in_rows(dn.stem, 1, slots), st));
  CHK(convnet_run(c, dn, n, slots, rowmap(audio_out, 1, hop, hop), RowMap{}, st));
  CHK(convnet_roll(dn, n, slots, 0, st));
  return 0;
}

int vv_codec_encode(vv_ctx* c, int n, const int* slots, const void* audio, void* sem_out, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (!c->finalized) FAIL("vv_codec_encode before vv_finalize");
  if (n <= 0) return 0;
  if (n > c->cfg.max_batch) FAIL("vv_codec_encode: n > max_batch");
  ConvNet& sn = c->sem;
  const int hop = c->dec.T[c->dec.nst - 1];
  // audio rows [n, hop] -> the encoder stem's input rows of each slot (one row of
  // hop channels-last samples per slot)
  RowMap in = rowmap(sn.stem.base + (long long)sn.stem.ctx * sn.stem.C, hop, 1, sn.stem.sB, slots);
  KCHK(launch_copy_rows1(n, hop, (const bf16*)audio, hop, in, st));
  const int S = c->cfg.semantic_dim;
  CHK(convnet_run(c, sn, n, slots, rowmap(sem_out, S, 1, S), RowMap{}, st));
  CHK(convnet_roll(sn, n, slots, 0, st));
  return 0;
}

int vv_codec_reset_net(vv_ctx* c, int net, int n, const int* slots, vv_stream vst) {
  hipStream_t st = (hipStream_t)vst;
  if (n <= 0) return 0;
  if (net != 0 && net != 1) FAIL("vv_codec_reset_net: net must be 0 (acoustic decoder) or 1 (semantic encoder)");
  CHK(convnet_roll(net == 0 ? c->dec : c->sem, n, slots, 1, st));
  return 0;
}

// Non-streaming encode of nv clips of L samples (zero-padded to a common L) by
// one of the σ-VAE encoders, laid out for this call: nv slots, T0 = L.  The
// per-layer right zero padding of the strided-conv inputs (ConvBuf rows past
// the input, zeroed per call) is the reference's non-streaming extra padding
// (modular_vibevoice_tokenizer.py:127-133, :393-408), so a clip that ends in a
// partial frame gives ceil(L / hop) frames as the reference does.
static int encode_nonstreaming(vv_ctx* c, ConvNet& net, const char* wp, int nf, int out_ch, int nv, int L,
                               const void* audio, void* out, hipStream_t st) {
  if (net.slots != nv || net.T0 != L || net.wp != wp) {
    convnet_shape(c, net, false, wp, nf, 1, out_ch, L, nv);
    CHK(convnet_alloc(net, 7));
  } else {
    HIPCHK(hipMemsetAsync(net.state.p, 0, net.state.bytes, st));
  }
  CHK(c->slot_scratch.ensure(sizeof(int) * (size_t)std::max(nv, 1024)));
  std::vector<int> ids(nv);
  for (int i = 0; i < nv; ++i) ids[i] = i;
  int* d_ids = (int*)c->slot_scratch.p;
  HIPCHK(hipMemcpyAsync(d_ids, ids.data(), nv * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpy2DAsync(net.stem.base + net.stem.ctx, net.stem.sB * sizeof(bf16), audio, (size_t)L * sizeof(bf16),
                          (size_t)L * sizeof(bf16), nv, hipMemcpyDeviceToDevice, st));
  const int Tl = net.T[net.nst - 1];
  CHK(convnet_run(c, net, nv, d_ids, rowmap(out, out_ch, Tl, (long long)Tl * out_ch), RowMap{}, st));
  HIPCHK(hipStreamSynchronize(st));  // d_ids scratch is reused by the next call
  return 0;
}

int vv_acoustic_encode(vv_ctx* c, int nv, int L, const void* audio, void* mean_out, vv_stream vst) {
  if (!c->w.count("aenc.stem_w")) FAIL("acoustic encoder weights not bound");
  if (nv <= 0 || L <= 0) return 0;
  return encode_nonstreaming(c, c->aenc, "aenc", c->cfg.ac_enc_n_filters, c->cfg.latent_dim, nv, L, audio, mean_out,
                             (hipStream_t)vst);
}

int vv_semantic_encode(vv_ctx* c, int nv, int L, const void* audio, void* mean_out, vv_stream vst) {
  if (!c->finalized) FAIL("vv_semantic_encode before vv_finalize");
  if (nv <= 0 || L <= 0) return 0;
  return encode_nonstreaming(c, c->senc, "sem", c->cfg.sem_n_filters, c->cfg.semantic_dim, nv, L, audio, mean_out,
                             (hipStream_t)vst);
}

int vv_vae_features(vv_ctx* c, int nv, int frames, const void* mean, const void* stdv, const void* noise, void* feat,
                    vv_stream vst) {
  KCHK(launch_vae_features(nv * frames, c->cfg.latent_dim, frames, (const bf16*)mean, (const bf16*)stdv,
                           (const bf16*)noise, W(c, "speech_scaling_factor"), W(c, "speech_bias_factor"),
                           (bf16*)feat, (hipStream_t)vst));
  return 0;
}

int vv_scatter_rows(vv_ctx* c, int n, int C, const void* src, int64_t lds, const int* idx, void* dst, int64_t ldd,
                    vv_stream vst) {
  (void)c;
  // dst[idx[i]] = src[i]: a gather with the roles of the maps swapped
  RowMap dm = rowmap(dst, ldd, 1, ldd, idx);
  KCHK(launch_gather_rows(n, C, (const bf16*)src, lds, nullptr, dm, (hipStream_t)vst));
  return 0;
}

// diagnostic (vv_gemm_tune_apack): vv_gemm_bf16's A is MFMA-fragment packed (k_gemm_xl only)
static std::atomic<int> g_gemm_apack{0};
extern "C" int vv_gemm_tune_apack(int on) {
  g_gemm_apack = on;
  return 0;
}

int vv_gemm_bf16(int M, int N, int K, const void* A, int64_t lda, const void* Wt, const void* bias, int epi, void* Y,
                 int64_t ldy, const void* res, const void* gamma, vv_ctx* c, vv_stream vst) {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.M = M;
  g.N = N;
  g.K = K;
  g.ksplit = 1;
  g.a = rowmap(A, lda);
  g.w = (const bf16*)Wt;
  g.ldw = K;
  g.epi.kind = epi;
  g.epi.bias = (const bf16*)bias;
  g.epi.out = rowmap(Y, ldy);
  g.epi.res = rowmap(res, ldy);
  g.epi.gamma = (const bf16*)gamma;
  g.apack = g_gemm_apack;
  if (c) {
    g.ws = (float*)c->splitk_ws.p;
    g.counters = (unsigned*)c->splitk_cnt.p;
  } else {
    // standalone calls (tests): a process-wide split-K workspace
    static DevBuf ws, cnt;
    if (!cnt.p) {
      CHK(ws.ensure(64ull << 20));
      CHK(cnt.ensure(65536 * sizeof(unsigned)));
      HIPCHK(hipMemset(cnt.p, 0, 65536 * sizeof(unsigned)));
    }
    g.ws = (float*)ws.p;
    g.counters = (unsigned*)cnt.p;
  }
  KCHK(launch_gemm(g, (hipStream_t)vst));
  return 0;
}

int vv_gemm_bf16_norm(int M, int N, int K, const void* A, int64_t lda, const void* norm_w, float eps, const void* Wt,
                      int epi, void* Y, int64_t ldy, vv_ctx* c, vv_stream vst) {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.M = M;
  g.N = N;
  g.K = K;
  g.ksplit = 1;
  g.a = rowmap(A, lda);
  g.w = (const bf16*)Wt;
  g.ldw = K;
  g.epi.kind = epi;
  g.epi.out = rowmap(Y, ldy);
  g.xf = xf_norm((const bf16*)norm_w, eps);
  if (c) {   // the engine's own dispatch (M > 16: k_rmsnorm once, then the GEMV on normalised rows)
    g.ws = (float*)c->splitk_ws.p;
    g.counters = (unsigned*)c->splitk_cnt.p;
    CHK(gemm(c, g, (hipStream_t)vst));
    return 0;
  }
  KCHK(launch_gemm(g, (hipStream_t)vst));
  return 0;
}

int vv_attention_bf16(int nq, int nh, int nkv, const void* q, const void* k_cache, const void* v_cache,
                      int64_t s_slot, int64_t s_head, const int* slots, const int* pos, int max_pos_p1, void* out,
                      vv_ctx* c, vv_stream vst) {
  if (!c) FAIL("vv_attention_bf16: needs an engine for split workspaces");
  KVLayout kv;
  kv.k = (bf16*)k_cache;
  kv.v = (bf16*)v_cache;
  kv.s_layer = 0;
  kv.s_slot = s_slot;
  kv.s_head = s_head;
  kv.d = 128;
  kv.max_ctx = (int)(s_head / 128);
  if (s_head % (128 * 32)) FAIL("vv_attention_bf16: the V cache is blocked by 32 positions (s_head % 4096 != 0)");
  AttnArgs at;
  memset(&at, 0, sizeof(at));
  int chunk = 0;
  // the slot count is unknown here: auto keeps k_attn (vv_attn_prefill(1) forces k_attn_pf)
  at.prefill = attn_use_prefill(nq, nq) ? 1 : 0;
  at.nsplit = at.prefill ? 1 : attn_plan(nq, nkv, max_pos_p1, &chunk);
  if (at.nsplit > 1) {
    if ((size_t)nq * nkv > 65536) FAIL("attention split tickets exhausted");
    CHK(c->attn_part.ensure((size_t)nq * nh * at.nsplit * (128 + 2) * sizeof(float)));
  }
  at.nq = nq;
  at.nh = nh;
  at.nkv = nkv;
  at.layer = 0;
  at.chunk = chunk;
  at.scale = 1.0f / sqrtf(128.f);
  at.q = (const bf16*)q;
  at.out = (bf16*)out;
  at.slots = slots;
  at.pos = pos;
  at.kv = kv;
  at.counters = (unsigned*)c->attn_cnt.p;
  at.part_o = (float*)c->attn_part.p;
  at.part_ml = at.part_o + (size_t)nq * nh * at.nsplit * 128;
  at.stamps = g_attn_stamps;
  KCHK(launch_attn(at, (hipStream_t)vst));
  return 0;
}

int vv_rmsnorm_bf16(int M, int C, const void* x, int64_t ldx, const void* w, float eps, void* y, int64_t ldy,
                    vv_stream vst) {
  return rmsnorm(M, C, rowmap(x, ldx), rowmap(y, ldy), (const bf16*)w, eps, (hipStream_t)vst);
}

}  // extern "C"
