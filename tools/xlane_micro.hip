// Throughput of cross-lane primitives on gfx950 (lab tool, not part of the library).
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 4096
template <int KIND>
__global__ __launch_bounds__(1024) void k(double* out, int iters) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 * 2, a5 = a0 * 3, a6 = a0 * 5, a7 = a0 * 7;
  for (int it = 0; it < iters; ++it) {
#define STEP(a, b)                                                                                       \
  if constexpr (KIND == 0) { a = fma(a, 1.0000001, b); }                                                 \
  else if constexpr (KIND == 1) {                                                                        \
    long long x = __double_as_longlong(a), y = __double_as_longlong(b);                                 \
    auto l = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)y, false, false);                   \
    auto h = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);   \
    a = __longlong_as_double(((long long)h[0] << 32) | l[0]);                                            \
    b = __longlong_as_double(((long long)h[1] << 32) | l[1]);                                            \
  } else if constexpr (KIND == 2) {                                                                      \
    a = __builtin_amdgcn_update_dpp(0.0, a, 0x124, 0xF, 0xF, false);                                     \
  } else if constexpr (KIND == 3) {                                                                      \
    a = __shfl_xor(a, 16);                                                                               \
  } else if constexpr (KIND == 4) {                                                                      \
    long long x = __double_as_longlong(a);                                                               \
    unsigned lo = __builtin_amdgcn_readlane((unsigned)x, 17), hi = __builtin_amdgcn_readlane((unsigned)(x >> 32), 17); \
    a = fma(__longlong_as_double(((long long)hi << 32) | lo), 1.0000001, b);                             \
  }
    STEP(a0, a1) STEP(a2, a3) STEP(a4, a5) STEP(a6, a7) STEP(a1, a0) STEP(a3, a2) STEP(a5, a4) STEP(a7, a6)
  }
  out[blockIdx.x * 1024 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
template <int KIND>
void run(const char* nm, double* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0), hipEventCreate(&e1);
  const int iters = 4096;
  hipLaunchKernelGGL(k<KIND>, dim3(256), dim3(1024), 0, 0, d, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<KIND>, dim3(256), dim3(1024), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // per SIMD: 4 waves x iters x 8 ops
  const double ops = 4.0 * iters * 8;
  printf("%-28s %.3f ms  -> %.2f cycles/op/wave at 2.4 GHz (per SIMD, 4 waves)\n", nm, ms, ms * 1e-3 * 2.4e9 / ops);
}
int main() {
  double* d;
  hipMalloc(&d, 256 * 1024 * 8);
  run<0>("f64 fma", d);
  run<1>("permlane32_swap x2 (dbl pair)", d);
  run<2>("dpp row_ror (f64 = 2 movs)", d);
  run<3>("shfl_xor 16 (bpermute)", d);
  run<4>("readlane x2 + fma", d);
  return 0;
}
