// Bit-exactness probe of the fused codec Block1D (k_block) against k_mix +
// k_gemm(fc1, GELU) + k_gemm(fc2, gamma residual) on random data: one sample,
// C channels, T rows.  Reports mismatches of y, fc1's input, the hidden rows and
// the block output.  Build: make -C tools block_check  (links the library objects)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../vibevoice_amd/csrc/kernels.h"

static void ck(hipError_t e, const char* w) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", w, hipGetErrorString(e));
    exit(1);
  }
}

static std::vector<bf16> rnd(size_t n, float scale, unsigned& s) {
  std::vector<bf16> v(n);
  for (auto& x : v) {
    s = s * 1664525u + 1013904223u;
    x = (bf16)(scale * (((s >> 9) & 0xffff) / 32768.0f - 1.0f));
  }
  return v;
}

static bf16* up(const std::vector<bf16>& h) {
  bf16* d;
  ck(hipMalloc(&d, h.size() * sizeof(bf16)), "malloc");
  ck(hipMemcpy(d, h.data(), h.size() * sizeof(bf16), hipMemcpyHostToDevice), "h2d");
  return d;
}

static std::vector<bf16> down(const bf16* d, size_t n) {
  std::vector<bf16> h(n);
  ck(hipMemcpy(h.data(), d, n * sizeof(bf16), hipMemcpyDeviceToHost), "d2h");
  return h;
}

static int cmp(const char* what, const std::vector<bf16>& a, const std::vector<bf16>& b) {
  int bad = 0;
  float mx = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    uint16_t x, y;
    memcpy(&x, &a[i], 2);
    memcpy(&y, &b[i], 2);
    if (x != y) {
      ++bad;
      float d = (float)a[i] - (float)b[i];
      if (d < 0) d = -d;
      if (d > mx) mx = d;
    }
  }
  printf("  %-8s %8d / %8zu differ (max |d| %.5f)\n", what, bad, a.size(), mx);
  return bad;
}

int main(int argc, char** argv) {
  const int C = argc > 1 ? atoi(argv[1]) : 128, T = argc > 2 ? atoi(argv[2]) : 800;
  const int R = 2048 / C, ctx = 6;
  unsigned s = 12345;
  auto hx = rnd((size_t)T * C, 1.0f, s), hbuf = rnd((size_t)(ctx + T) * C, 1.0f, s);
  auto hnw = rnd(C, 1.0f, s), hdw = rnd((size_t)C * 7, 0.3f, s), hdb = rnd(C, 0.1f, s), hg = rnd(C, 0.5f, s);
  auto hfw = rnd(C, 1.0f, s), hw1 = rnd((size_t)4 * C * C, 0.1f, s), hb1 = rnd(4 * C, 0.1f, s);
  auto hw2 = rnd((size_t)4 * C * C, 0.05f, s), hb2 = rnd(C, 0.1f, s), hg2 = rnd(C, 0.5f, s);
  int zero = 0, *slots;
  ck(hipMalloc(&slots, 4), "malloc");
  ck(hipMemcpy(slots, &zero, 4, hipMemcpyHostToDevice), "h2d");
  bf16 *x = up(hx), *buf1 = up(hbuf), *buf2 = up(hbuf), *nw = up(hnw), *dw = up(hdw), *db = up(hdb), *g = up(hg),
       *fw = up(hfw), *w1 = up(hw1), *b1 = up(hb1), *w2 = up(hw2), *b2 = up(hb2), *gm2 = up(hg2);
  std::vector<bf16> z((size_t)T * 4 * C);
  bf16 *y = up(z), *a = up(z), *f = up(z), *o1 = up(z), *o2 = up(z), *a2 = up(z), *f2 = up(z);

  MixArgs m;
  memset(&m, 0, sizeof(m));
  m.n = 1, m.T = T, m.C = C, m.R = R, m.eps = 1e-5f, m.ctx = ctx, m.x = x, m.y = y, m.a = a, m.buf = buf1;
  m.buf_sB = (long long)(ctx + T) * C, m.slots = slots, m.norm_w = nw, m.dw_w = dw, m.dw_b = db, m.gamma = g;
  m.ffn_norm_w = fw;
  if (launch_mix(m, 0)) return fprintf(stderr, "launch_mix refused\n"), 1;
  GemmArgs g1;
  memset(&g1, 0, sizeof(g1));
  g1.M = T, g1.N = 4 * C, g1.K = C, g1.ksplit = 1, g1.a = rowmap(a, C), g1.w = w1, g1.ldw = C;
  g1.epi.kind = EPI_GELU, g1.epi.bias = b1, g1.epi.out = rowmap(f, 4 * C);
  if (launch_gemm(g1, 0)) return fprintf(stderr, "fc1 refused\n"), 1;
  GemmArgs g2 = g1;
  g2.N = C, g2.K = 4 * C, g2.a = rowmap(f, 4 * C), g2.w = w2, g2.ldw = 4 * C;
  g2.epi.kind = EPI_RES, g2.epi.bias = b2, g2.epi.out = rowmap(o1, C), g2.epi.res = rowmap(y, C), g2.epi.gamma = gm2;
  if (launch_gemm(g2, 0)) return fprintf(stderr, "fc2 refused\n"), 1;

  BlockArgs b;
  memset(&b, 0, sizeof(b));
  b.mix = m;
  b.mix.buf = buf2;
  b.mix.y = nullptr, b.mix.a = nullptr;
  b.w1 = w1, b.b1 = b1, b.w2 = w2, b.b2 = b2, b.g2 = gm2, b.out = rowmap(o2, C);
  b.dbg_a = a2, b.dbg_h = f2;
  if (launch_block(b, 0)) return fprintf(stderr, "k_block refused\n"), 1;
  ck(hipDeviceSynchronize(), "sync");

  printf("C=%d T=%d R=%d\n", C, T, R);
  int bad = cmp("buffer", down(buf1, (size_t)(ctx + T) * C), down(buf2, (size_t)(ctx + T) * C));
  bad += cmp("fc1 in", down(a, (size_t)T * C), down(a2, (size_t)T * C));
  bad += cmp("hidden", down(f, (size_t)T * 4 * C), down(f2, (size_t)T * 4 * C));
  bad += cmp("out", down(o1, (size_t)T * C), down(o2, (size_t)T * C));
  {  // first mismatches against a double-precision fc2 (packed weights: block (t, c) at (t*K/32 + c)*512)
    auto O1 = down(o1, (size_t)T * C), O2 = down(o2, (size_t)T * C), F = down(f, (size_t)T * 4 * C);
    auto Y = down(y, (size_t)T * C);
    const int K = 4 * C;
    int shown = 0;
    for (int m = 0; m < T && shown < 8; ++m)
      for (int n = 0; n < C && shown < 8; ++n) {
        uint16_t p1, p2;
        memcpy(&p1, &O1[(size_t)m * C + n], 2);
        memcpy(&p2, &O2[(size_t)m * C + n], 2);
        if (p1 == p2) continue;
        double acc = 0;
        for (int k = 0; k < K; ++k) {
          const int t = n / 16, rr = n % 16, cc = k / 32, kk = k % 32;
          const size_t idx = ((size_t)t * (K / 32) + cc) * 512 + (size_t)(rr + 16 * (kk / 8)) * 8 + kk % 8;
          acc += (double)(float)hw2[idx] * (double)(float)F[(size_t)m * K + k];
        }
        const double v = acc + (float)hb2[n];
        const float rv = (float)(bf16)(float)v, sv = (float)(bf16)((float)hg2[n] * rv);
        const float ex = (float)(bf16)((float)Y[(size_t)m * C + n] + sv);
        printf("    expected from fp64 acc: %+.6f   (g2 %+.5f)\n", ex, (float)hg2[n]);
        printf("  m %4d n %3d  gemm %+.6f block %+.6f | fp64 pre-epilogue %+.8f (bf16-rounding boundary?)"
               " y %+.5f\n", m, n, (float)O1[(size_t)m * C + n], (float)O2[(size_t)m * C + n], v,
               (float)Y[(size_t)m * C + n]);
        ++shown;
      }
  }
  return bad ? 2 : 0;
}
