// Launch-floor microbenchmark (tools only): what does one kernel boundary cost
// on this box?  empty kernel / large kernarg struct / one dependent HBM load.
#include <hip/hip_runtime.h>
struct Big { char pad[448]; float* p; };
__global__ void k_empty() {}
__global__ void k_big(Big b) { if (threadIdx.x == 0 && blockIdx.x == 100000) b.p[0] = 1.f; }
__global__ void k_load(const float* __restrict__ x, float* y, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] * 2.f;
}
extern "C" int fl_launch(int kind, int blocks, int threads, void* x, void* y, int n, void* st) {
  hipStream_t s = (hipStream_t)st;
  if (kind == 0) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(threads), 0, s);
  else if (kind == 1) { Big b; b.p = (float*)y; hipLaunchKernelGGL(k_big, dim3(blocks), dim3(threads), 0, s, b); }
  else hipLaunchKernelGGL(k_load, dim3(blocks), dim3(threads), 0, s, (const float*)x, (float*)y, n);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
