// Workgroup-level complex GEMM for the small (chi x chi) contractions of the environment chains.
//
// C[i][j] = sum_k a(i, k) * b(k, j) over an m x n output, computed by one 256-thread workgroup
// in 64 x 64 output blocks; k is staged through LDS in tiles of 16 (As[k][i], Bs[k][j], row
// padding 65 so the column-wise fills and the broadcast reads stay conflict-light); each thread
// owns a 4 x 4 register block (rows 4*ty.., cols 4*tx..).  Accessors a / b return zero outside
// the valid range; store(i, j, v) is called for i < m, j < n.  Callers provide the LDS tiles.
#pragma once

#include "aqc_internal.h"

namespace aqc {

constexpr int kGemmThreads = 256;

struct GemmLds {
  cplx As[16][65];
  cplx Bs[16][65];
};

// A_KFAST / B_KFAST choose the tile-load order: consecutive threads walk k (use when the source
// is contiguous along k) instead of the output dimension.
template <bool A_KFAST = false, bool B_KFAST = false, typename FA, typename FB, typename FS>
__device__ __forceinline__ void block_cgemm_valu(int m, int n, int k, FA a, FB b, FS store, GemmLds& lds) {
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  for (int bi = 0; bi < m; bi += 64) {
    for (int bj = 0; bj < n; bj += 64) {
      cplx acc[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = cmk(0, 0);
      for (int k0 = 0; k0 < k; k0 += 16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = tid + q * kGemmThreads;
          const int ka = A_KFAST ? (e & 15) : (e >> 6), ia = A_KFAST ? (e >> 4) : (e & 63);
          const int kb = B_KFAST ? (e & 15) : (e >> 6), ib = B_KFAST ? (e >> 4) : (e & 63);
          lds.As[ka][ia] = (bi + ia < m && k0 + ka < k) ? a(bi + ia, k0 + ka) : cmk(0, 0);
          lds.Bs[kb][ib] = (bj + ib < n && k0 + kb < k) ? b(k0 + kb, bj + ib) : cmk(0, 0);
        }
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < 16; ++kk) {
          cplx av[4], bv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) av[r] = lds.As[kk][4 * ty + r];
#pragma unroll
          for (int c = 0; c < 4; ++c) bv[c] = lds.Bs[kk][4 * tx + c];
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = cfma(av[r], bv[c], acc[r][c]);
        }
        __syncthreads();
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int i = bi + 4 * ty + r, j = bj + 4 * tx + c;
          if (i < m && j < n) store(i, j, acc[r][c]);
        }
    }
  }
}

// The same contract on the FP64 matrix cores: each of the 4 waves owns a 32 x 32 quarter of the
// 64 x 64 output block as 2 x 2 tiles of v_mfma_f64_16x16x4_f64 (A operand: lane l holds
// A[l & 15][k = l >> 4], B: B[k = l >> 4][l & 15]; C/D: col = lane & 15, row = (lane >> 4) +
// 4 * reg).  A complex product is four real MFMAs into two accumulators (Re += Ar Br + (-Ai) Bi,
// Im += Ar Bi + Ai Br).  Per 16-deep k tile a wave reads 4 KB of operands from LDS for 64
// MFMAs, against 32 KB for the register-blocked VALU form: the LDS port stops being the limit.
typedef double __attribute__((ext_vector_type(4))) d4_t;

// PREFETCH: fetch the next k tile into registers while the MFMAs run on the current one (pays
// where the tile loads are the latency, e.g. the split's indirect column reads: 8.9 -> 7.6
// ms/step; it costs the register-heavy ISL chain 20%).
// tid_in >= 0: the caller's 256-thread sub-group rank (several sub-groups of a larger workgroup
// each running their own block; every sub-group must then make the same calls with the same m, n,
// k so the barriers pair up); active = false runs only those barriers (an idle sub-group).
template <bool A_KFAST = false, bool B_KFAST = false, bool PREFETCH = false, typename FA, typename FB, typename FS>
__device__ __forceinline__ void block_cgemm(int m, int n, int k, FA a, FB b, FS store, GemmLds& lds, int tid_in = -1,
                                            bool active = true) {
  const int tid = tid_in >= 0 ? tid_in : (int)threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  for (int bi = 0; bi < m; bi += 64) {
    for (int bj = 0; bj < n; bj += 64) {
      d4_t cr[2][2], ci[2][2];
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) cr[r][c] = d4_t{0, 0, 0, 0}, ci[r][c] = d4_t{0, 0, 0, 0};
      cplx pa[PREFETCH ? 4 : 1], pb[PREFETCH ? 4 : 1];
      auto fetch = [&](int k0) {
#pragma unroll
        for (int q = 0; q < (PREFETCH ? 4 : 0); ++q) {
          const int e = tid + q * kGemmThreads;
          const int ka = A_KFAST ? (e & 15) : (e >> 6), ia = A_KFAST ? (e >> 4) : (e & 63);
          const int kb = B_KFAST ? (e & 15) : (e >> 6), ib = B_KFAST ? (e >> 4) : (e & 63);
          pa[q] = (bi + ia < m && k0 + ka < k) ? a(bi + ia, k0 + ka) : cmk(0, 0);
          pb[q] = (bj + ib < n && k0 + kb < k) ? b(k0 + kb, bj + ib) : cmk(0, 0);
        }
      };
      if constexpr (PREFETCH) {
        if (active) fetch(0);
      }
      for (int k0 = 0; k0 < k; k0 += 16) {
        if (active) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int e = tid + q * kGemmThreads;
          const int ka = A_KFAST ? (e & 15) : (e >> 6), ia = A_KFAST ? (e >> 4) : (e & 63);
          const int kb = B_KFAST ? (e & 15) : (e >> 6), ib = B_KFAST ? (e >> 4) : (e & 63);
          if constexpr (PREFETCH) {
            lds.As[ka][ia] = pa[q];
            lds.Bs[kb][ib] = pb[q];
          } else {
            lds.As[ka][ia] = (bi + ia < m && k0 + ka < k) ? a(bi + ia, k0 + ka) : cmk(0, 0);
            lds.Bs[kb][ib] = (bj + ib < n && k0 + kb < k) ? b(k0 + kb, bj + ib) : cmk(0, 0);
          }
        }
        }
        __syncthreads();
        if constexpr (PREFETCH) {
          if (active && k0 + 16 < k) fetch(k0 + 16);
        }
        if (active) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int kk = 4 * ks + lk;
          cplx av[2], bv[2];
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            av[t] = lds.As[kk][wr + 16 * t + li];
            bv[t] = lds.Bs[kk][wc + 16 * t + li];
          }
#pragma unroll
          for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              cr[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r].x, bv[c].x, cr[r][c], 0, 0, 0);
              cr[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[r].y, bv[c].y, cr[r][c], 0, 0, 0);
              ci[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r].x, bv[c].y, ci[r][c], 0, 0, 0);
              ci[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r].y, bv[c].x, ci[r][c], 0, 0, 0);
            }
        }
        }
        __syncthreads();
      }
#pragma unroll
      for (int r = 0; r < 2; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = bi + wr + 16 * r + lk + 4 * q, jj = bj + wc + 16 * c + li;
            if (active && i < m && jj < n) store(i, jj, cmk(cr[r][c][q], ci[r][c][q]));
          }
    }
  }
}

// One 64 x 64 output block (rows bi.., cols bj..) of block_cgemm's product left in the wave's
// accumulators: cr / ci[r][c][q] hold C[bi + wr + 16 r + lk + 4 q][bj + wc + 16 c + li] (the
// Gram SVD moves them through the LDS itself).  block_cgemm keeps its own copy of the loop: built
// on this function, the chain's split spilled 160 VGPRs.
template <bool A_KFAST = false, bool B_KFAST = false, bool PREFETCH = false, typename FA, typename FB>
__device__ __forceinline__ void block_cgemm_tile(int m, int n, int k, int bi, int bj, FA a, FB b, GemmLds& lds,
                                                 int tid, bool active, d4_t (&cr)[2][2], d4_t (&ci)[2][2]) {
  const int wave = tid >> 6, lane = tid & 63;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) cr[r][c] = d4_t{0, 0, 0, 0}, ci[r][c] = d4_t{0, 0, 0, 0};
  cplx pa[PREFETCH ? 4 : 1], pb[PREFETCH ? 4 : 1];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int q = 0; q < (PREFETCH ? 4 : 0); ++q) {
      const int e = tid + q * kGemmThreads;
      const int ka = A_KFAST ? (e & 15) : (e >> 6), ia = A_KFAST ? (e >> 4) : (e & 63);
      const int kb = B_KFAST ? (e & 15) : (e >> 6), ib = B_KFAST ? (e >> 4) : (e & 63);
      pa[q] = (bi + ia < m && k0 + ka < k) ? a(bi + ia, k0 + ka) : cmk(0, 0);
      pb[q] = (bj + ib < n && k0 + kb < k) ? b(k0 + kb, bj + ib) : cmk(0, 0);
    }
  };
  if constexpr (PREFETCH) {
    if (active) fetch(0);
  }
  for (int k0 = 0; k0 < k; k0 += 16) {
    if (active) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = tid + q * kGemmThreads;
        const int ka = A_KFAST ? (e & 15) : (e >> 6), ia = A_KFAST ? (e >> 4) : (e & 63);
        const int kb = B_KFAST ? (e & 15) : (e >> 6), ib = B_KFAST ? (e >> 4) : (e & 63);
        if constexpr (PREFETCH) {
          lds.As[ka][ia] = pa[q];
          lds.Bs[kb][ib] = pb[q];
        } else {
          lds.As[ka][ia] = (bi + ia < m && k0 + ka < k) ? a(bi + ia, k0 + ka) : cmk(0, 0);
          lds.Bs[kb][ib] = (bj + ib < n && k0 + kb < k) ? b(k0 + kb, bj + ib) : cmk(0, 0);
        }
      }
    }
    __syncthreads();
    if constexpr (PREFETCH) {
      if (active && k0 + 16 < k) fetch(k0 + 16);
    }
    if (active) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int kk = 4 * ks + lk;
        cplx av[2], bv[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          av[t] = lds.As[kk][wr + 16 * t + li];
          bv[t] = lds.Bs[kk][wc + 16 * t + li];
        }
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            cr[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r].x, bv[c].x, cr[r][c], 0, 0, 0);
            cr[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[r].y, bv[c].y, cr[r][c], 0, 0, 0);
            ci[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r].x, bv[c].y, ci[r][c], 0, 0, 0);
            ci[r][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[r].y, bv[c].x, ci[r][c], 0, 0, 0);
          }
      }
    }
    __syncthreads();
  }
}

}  // namespace aqc
