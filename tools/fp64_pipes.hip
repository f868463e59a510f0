// Micro-benchmark: do the FP64 VALU and the FP64 MFMA pipes of a gfx950 SIMD run concurrently?
// Modes (512-thread workgroups = 2 waves per SIMD, one workgroup per CU x 4):
//   0: every wave issues v_fma_f64 (8 independent chains)
//   1: every wave issues v_mfma_f64_16x16x4_f64 (4 independent accumulators)
//   2: waves 0-3 VALU, waves 4-7 MFMA (split across the two waves of each SIMD)
//   3: every wave interleaves both streams (4 MFMA + 32 FMA per iteration)
// Prints TFLOP/s per pipe.  Build: hipcc -O3 --offload-arch=gfx950 tools/fp64_pipes.hip -o tools/fp64_pipes
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double __attribute__((ext_vector_type(4))) d4_t;

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

__device__ __forceinline__ void valu_block(double (&v)[8], double a, double b) {
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = fma(v[q], a, b);
}

__device__ __forceinline__ void mfma_block(d4_t (&c)[4], double a, double b) {
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[q], 0, 0, 0);
}

__global__ __launch_bounds__(512) void k_pipes(int mode, int iters, double* out) {
  const int wave = threadIdx.x >> 6;
  double a = 0.999999 + 1e-9 * threadIdx.x, b = 1e-7 * (threadIdx.x & 7);
  double v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = q;
  d4_t c[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = d4_t{0, 0, 0, 0};
  const bool do_valu = mode == 0 || mode == 3 || (mode == 2 && wave < 4);
  const bool do_mfma = mode == 1 || mode == 3 || (mode == 2 && wave >= 4);
  if (do_valu && do_mfma) {
    for (int it = 0; it < iters; ++it) {
      mfma_block(c, a, b);
      valu_block(v, a, b);
    }
  } else if (do_valu) {
    for (int it = 0; it < iters; ++it) valu_block(v, a, b);
  } else if (do_mfma) {
    for (int it = 0; it < iters; ++it) mfma_block(c, a, b);
  }
  double s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += v[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
  if (s == 12345.678) out[threadIdx.x] = s;
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  double* out;
  CHECK(hipMalloc(&out, 4096 * sizeof(double)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int grid = cus * 4;  // 4 x 512 threads per CU = 32 waves: full occupancy
  for (int mode = 0; mode < 4; ++mode) {
    k_pipes<<<grid, 512>>>(mode, 100, out);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    k_pipes<<<grid, 512>>>(mode, iters, out);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    // per wave per iteration: VALU 32 FMA x 64 lanes x 2 flop; MFMA 4 x 16*16*4*2 flop
    const double waves = (double)grid * 8;
    double valu_waves = 0, mfma_waves = 0;
    if (mode == 0) valu_waves = waves;
    if (mode == 1) mfma_waves = waves;
    if (mode == 2) valu_waves = mfma_waves = waves / 2;
    if (mode == 3) valu_waves = mfma_waves = waves;
    const double vf = valu_waves * iters * 32 * 64 * 2, mf = mfma_waves * iters * 4 * 2048.0;
    printf("mode %d: %.3f ms  VALU %.1f TFLOP/s  MFMA %.1f TFLOP/s  total %.1f TFLOP/s\n", mode, ms,
           vf / ms * 1e-9, mf / ms * 1e-9, (vf + mf) / ms * 1e-9);
  }
  printf("CUs %d, clock %d kHz\n", cus, prop.clockRate);
  return 0;
}
