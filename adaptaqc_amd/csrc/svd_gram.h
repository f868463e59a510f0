// Two-site SVD through the Gram matrix, its tridiagonal form and inverse iteration -- the fast
// path of the 2 chi = 128 two-site update when the truncation keeps K <= 64 singular triplets.
//
// X = theta' (L x C, or its conjugate transpose so that L >= C):
//   S1  G = X^H X: the 16 x 16 tiles on and above the diagonal on the FP64 matrix cores, three
//       real products per complex tile (3M), X streamed once through double-buffered LDS chunks
//   S2  G's upper triangle through the LDS (packed) into registers: thread t holds row t/8,
//       columns t%8 + 8i (i < 16)
//   S3  Householder tridiagonalisation G = Q T Q^H (LAPACK zhetd2, lower): two barriers per column
//       (the column pass in every wave with reflector k's zlarfg scalars in wave 0 beside it; then
//       the rows' p, v, z and p^H v partials, one row per thread of waves 0-1), the column, the
//       reflector and p = tau G v in double-buffered LDS vectors (zeros at and above the diagonal:
//       a mask-free rank-2 update), the reflectors packed into the work buffer
//   S4  the top K eigenvalues of the real symmetric tridiagonal T: one 256-point Sturm pass and
//       a binary search bracket each, then 5-section (4 lanes per eigenvalue each evaluate one
//       Sturm count -- the minors' three-term recurrence, one dependent FMA per row -- one ballot
//       picks the subinterval; 12 rounds)
//   S5  inverse iteration (unpivoted LDL^T of T - lambda I, three solves) per eigenvector, Gram-
//       Schmidt inside clusters (gaps below 1e-7 ||T||), sigma^2 = z^T T z
//   S6  back-transformation V = Q Z: blocks of 16 reflectors in compact WY form on the matrix
//       cores, V in the accumulators throughout; output W = V Sigma
// The output follows the QR-preconditioned register Jacobi's contract (TwoSiteJob::qr = 1): work
// column c (length C, rows in X's column order) = right singular vector c of X times sigma_c, sig[c]
// = sigma_c (0 for c >= K), so rank / split are unchanged.
//
// Accuracy: forming G squares the condition number, so eigenpairs are accurate to eps ||G|| in
// absolute terms: singular values to eps sigma_1^2 / sigma_i and the kept subspace to eps sigma_1^2
// / (sigma_K^2 - sigma_{K+1}^2) -- 1e-14 on the bench's thetas (tools/gram_svd_proto.py), as
// accurate as the Jacobi.  Small singular values are not resolved: the path declines (returns
// false, the caller runs the Jacobi) unless lambda_K > 1e-9 lambda_1, i.e. unless every kept
// value is far above the noise floor and above the reduce_zeros CHOP (1e-16), so the truncation
// decisions (kept count, tail sum, renormalisation) are the Jacobi's.  It also declines K > 64.
//
// Included into mps.hip's anonymous namespace.
#pragma once

constexpr int kGramMaxK = 128;    // kept triplets (the whole 2 chi = 128 side)
constexpr int kGramNarrowK = 64;  // up to here S5 runs on wave 0 from the LDS and S6 in one pass
// Settled choices (each measured against its alternative):
// S3: wave 0 raises its issue priority while it forms a reflector's scalars; the reflectors' base
//     pointer in SGPRs; the rows' partial products summed in the wave (DPP) before phase B; the
//     column pass prefetches column i + 1's LDS operands while column i computes; one row per lane
//     (two rows per lane measured slower: 0.68 M against 0.64 M ticks)
// S4: 4 lanes per eigenvalue (5-section), 12 rounds after the first 256-shift pass (8 x 9 x 9 and
//     16 x 17 x 7 measured 108 K / 145 K against 98 K ticks: the pass is FP64-issue-bound)
// S5: three inverse-iteration steps per eigenvector; the LDL^T pivots from the leading minors'
//     recurrence (one FMA + the guard on the chain)
// S6: the compact-WY factors of every reflector block precomputed during S5 by the idle waves
//     1-3, 5-7, 9-11 (not 4 and 8, which share SIMD 0 with wave 0's inverse iteration: S5 133 K ->
//     120 K ticks, k_chain -0.8% against waves 4..11, profiles/r5_s6_skip0_ab.json); W2 = T (Y^H V) on the matrix cores inside the mg == 0 waves; the next block's
//     reflectors fetched after B4
constexpr double kGramRelFloor = 1e-9;
// shader-clock ticks of the phases (thread 0), summed over calls: S1, S2+S3, S4, S5, S6, output,
// S3's column steps, S5's inverse iteration, S3's phase A (column pass + zlarfg + first barrier)
__device__ unsigned long long g_gram_ticks[12];
static_assert(kGramNarrowK == 64, "S5: the narrow inverse iteration (tid < K) stays on wave 0");
// path counters (thread 0 of each call): [0] calls, [1] taken, [2] declined by shape (K > 64, ...),
// [3] declined at the eigenvalue floor (lambda_K <= 1e-9 lambda_1 -> the Jacobi runs)
__device__ unsigned long long g_gram_stats[6];  // calls, taken, declined (shape), declined (decision / floor), certificates, certified

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

// Sum over the 64 lanes, result uniform: DPP row sums, then the four rows through readlane (no
// LDS crossbar; every lane must be active).
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v = aqc::row_sum16(v);
  double s = 0.0;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), 16 * rr);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), 16 * rr);
    s += __hiloint2double(hi, lo);
  }
  return s;
}

// g[i] for a wave-uniform i (a scalar switch, no per-lane selects)
__device__ __forceinline__ cplx pick16(const cplx (&g)[16], int i) {
  switch (i) {
#define AQC_PICK(n) \
  case n:           \
    return g[n];
    AQC_PICK(0) AQC_PICK(1) AQC_PICK(2) AQC_PICK(3) AQC_PICK(4) AQC_PICK(5) AQC_PICK(6) AQC_PICK(7)
    AQC_PICK(8) AQC_PICK(9) AQC_PICK(10) AQC_PICK(11) AQC_PICK(12) AQC_PICK(13) AQC_PICK(14)
#undef AQC_PICK
    default:
      return g[15];
  }
}

// a wave-uniform double moved to SGPRs (readfirstlane of both halves)
__device__ __forceinline__ double uniform_d(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// lane l's double broadcast to the wave (readlane of both halves; l uniform)
__device__ __forceinline__ double bcast_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// this lane's index in the wave from the lane counter (mbcnt), recomputed where it is called
// (the empty asm keeps it from being hoisted, and so from being spilled and reloaded)
__device__ __forceinline__ int fresh_lane() {
  int l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(l));
  return l;
}
// a wave-uniform pointer moved to SGPRs
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return (T*)(((unsigned long long)hi << 32) | lo);
}
// 1 for a negative q (sign bit; q is never -0 here)
__device__ __forceinline__ int sign_bit(double q) { return (int)((unsigned)__double2hiint(q) >> 31); }

// Sturm count (eigenvalues of T below x) by the three-term recurrence of the leading principal
// minors, p_{i+1} = (d_i - x) p_i - e_{i-1}^2 p_{i-1} (Wilkinson's bisection), counting sign
// changes.  Its dependent chain is one FMA per row -- the product e^2 p_{i-1} and d_i - x are off
// it -- where the ratio form q = (d - x) - e^2 / q carried a reciprocal and its Newton step
// (6 dependent FP64 operations per row).  de[i] = (d_i, e_{i-1}^2) pre-scaled by 1 / ||T|| (and
// x with them), so |p| grows at most 3.1x per row; every 4 rows both minors are rescaled by the
// larger one's binary exponent (a common positive factor leaves the signs alone), which also
// keeps runs of tiny pivots from underflowing.  The sign of each minor is its high word shifted
// arithmetically (0 or -1); the xor of consecutive ones is -1 on a change.
__device__ __forceinline__ int sturm_count_poly(const double2* de, int C, double xn) {
  double p0 = 1.0, p1 = de[0].x - xn;
  int s1 = __double2hiint(p1) >> 31;
  int neg = s1;  // -(sign changes): p_0 = 1 is positive
  int i = 1;
  auto step = [&](double2 e) {
    const double p2 = fma(e.x - xn, p1, -(e.y * p0));
    const int s2 = __double2hiint(p2) >> 31;
    neg += s1 ^ s2;
    s1 = s2;
    p0 = p1;
    p1 = p2;
  };
  auto rescale = [&]() {
    const int ex = max(__builtin_amdgcn_frexp_exp(p0), __builtin_amdgcn_frexp_exp(p1));
    p0 = __builtin_amdgcn_ldexp(p0, -ex);
    p1 = __builtin_amdgcn_ldexp(p1, -ex);
  };
  // the next four rows' (d, e^2) are read while the current four run (read and used four at a
  // time, every group of rows waited out an LDS round trip: about half of the pass).  Two named
  // register sets alternate (a rotating copy would wait for its reads at the loop's end); the
  // index is clamped at the end instead of a branch (the extra reads are unused).
  auto rd4 = [&](int i0, double2& r0, double2& r1, double2& r2, double2& r3) {
    r0 = de[min(i0, C - 1)], r1 = de[min(i0 + 1, C - 1)], r2 = de[min(i0 + 2, C - 1)], r3 = de[min(i0 + 3, C - 1)];
  };
  double2 a0, a1, a2, a3, b0, b1, b2, b3;
  rd4(1, a0, a1, a2, a3);
  for (; i + 8 <= C; i += 8) {
    rd4(i + 4, b0, b1, b2, b3);
    __builtin_amdgcn_sched_barrier(0);
    step(a0);
    step(a1);
    step(a2);
    step(a3);
    rescale();
    rd4(i + 8, a0, a1, a2, a3);
    __builtin_amdgcn_sched_barrier(0);
    step(b0);
    step(b1);
    step(b2);
    step(b3);
    rescale();
  }
  if (i + 4 <= C) {
    step(a0);
    step(a1);
    step(a2);
    step(a3);
    rescale();
    i += 4;
  }
  for (; i < C; ++i) step(de[i]);
  return -neg;
}

__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = r * fma(-x, r, 2.0);
  r = r * fma(-x, r, 2.0);
  return r;
}

// S6's precomputed compact-WY factors in the work buffer: after the reflectors (at most 8128 complex
// at C = 128) and clear of the output W written after S6's loop, 512 complex per block (S, then T)
constexpr size_t kTfacOff = 16384;
// K > 64: the inverse iteration's pivots (128 x 128 doubles, row-major, vector i in column i), then
// (after S5) the first 64 vectors, stashed for S6's second pass; complex offset in the work buffer
// (aqc::kGramWorkElems covers it)
constexpr size_t kWideOff = 20480;
static_assert(kWideOff + 8192 <= aqc::kGramWorkElems, "Gram-path scratch exceeds the work buffer");
static_assert(kChainLdsBytes >= 128 * 128 * 8, "S5 (K > 64): 128 x 128 vectors in the dynamic LDS");
typedef __attribute__((address_space(1))) double gdbl_t;

// S6's compact-WY factors of reflector block b, computed during S5 by an idle wave (gram_svd_body)
__device__ __forceinline__ void s6_factors(int b, int C, cplx* hh, const cplx* s_tau, int lane) {
  // block b of S6's loop (reflectors k0 .. k1 - 1, counted from the last): S = Y^H Y, then T by
  // zlarft, into the work scratch after the reflectors (S at [0, 256), T at [256, 512) of the
  // block's 512).  Read back through agent-scope loads: the same addresses were read by the
  // previous update's S6 on this CU, so the L1 may hold them.
  const int k1 = C - 1 - 16 * b, k0 = k1 > 16 ? k1 - 16 : 0, nb = k1 - k0;
  const int li = lane & 15, lk = lane >> 4;
  aqc::d4_t sr = {0, 0, 0, 0}, si = {0, 0, 0, 0};
  for (int r0 = 0; r0 < C; r0 += 4) {  // A[m = i][k = row] = conj(Y[row][i]), B = Y
    const int row = r0 + lk, k = k0 + li;
    const cplx y = (li < nb && row > k && row < C) ? aqc::ldg(hh + (size_t)k * (2 * C - k - 1) / 2 + (row - k - 1))
                                                   : aqc::cmk(0, 0);
    sr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, y.x, sr, 0, 0, 0);
    sr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, y.y, sr, 0, 0, 0);
    si = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, y.y, si, 0, 0, 0);
    si = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, y.x, si, 0, 0, 0);
  }
  cplx* Sg = hh + kTfacOff + (size_t)b * 512;
#pragma unroll
  for (int q = 0; q < 4; ++q) aqc::stg(Sg + (lk + 4 * q) * 16 + li, aqc::cmk(sr[q], si[q]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // zlarft (forward, columnwise): lane (a, g) holds T[a][g + 4 m]; T[a][i] = -tau_i sum_{a <= bb < i}
  // T[a][bb] S[bb][i], T[i][i] = tau_i -- the recurrence of the in-loop form
  const int a = lane >> 2, g = lane & 3;
  cplx tq[4] = {aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0)};
  for (int i = 0; i < 16; ++i) {
    const cplx tau = i < nb ? s_tau[k0 + i] : aqc::cmk(0, 0);
    cplx acc = aqc::cmk(0, 0);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int bb = g + 4 * m;
      if (4 * m < i && bb < i) {
        const gdbl_t* sp = (const gdbl_t*)(const double*)(Sg + bb * 16 + i);
        const cplx sv = aqc::cmk(__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                 __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        acc = aqc::cfma(tq[m], sv, acc);
      }
    }
    acc.x = aqc::row_sum4(acc.x);
    acc.y = aqc::row_sum4(acc.y);
    const cplx ti = aqc::cmul(tau, acc);
    const cplx val = a < i ? aqc::cmk(-ti.x, -ti.y) : (a == i ? tau : aqc::cmk(0, 0));
    if (g == (i & 3)) tq[i >> 2] = val;
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) aqc::stg(Sg + 256 + a * 16 + g + 4 * m, tq[m]);
}

// Gram-Schmidt inside clusters of the S5 vectors (zb[row * ZS + i]), one wave
template <int ZS>
__device__ __forceinline__ void gs_clusters(int K, int C, double* zb, const double* s_lam, double s_tn, int lane) {
  // clusters: gaps below 1e-7 ||T|| (dstein's 1e-3 is far more conservative than three
  // inverse-iteration steps need: at gaps above ~1e-10 the vectors come out orthogonal to
  // 1e-14 on their own, tools/gram_svd_proto.py)
  const double ortol = 1e-7 * s_tn;
  int start = 0;
  for (int i = 1; i < K; ++i) {
    if (s_lam[i - 1] - s_lam[i] >= ortol) {
      start = i;
      continue;
    }
    for (int jj = start; jj < i; ++jj) {
      double dp = 0.0;
      for (int row = lane; row < C; row += 64) dp = fma(zb[row * ZS + i], zb[row * ZS + jj], dp);
      dp = wave_sum_d(dp);
      for (int row = lane; row < C; row += 64) zb[row * ZS + i] = fma(-dp, zb[row * ZS + jj], zb[row * ZS + i]);
    }
    double n2 = 0.0;
    for (int row = lane; row < C; row += 64) n2 = fma(zb[row * ZS + i], zb[row * ZS + i], n2);
    n2 = wave_sum_d(n2);
    const double sc = 1.0 / sqrt(n2);
    for (int row = lane; row < C; row += 64) zb[row * ZS + i] *= sc;
  }
}

// sigma^2 of S5 vector i: the Rayleigh quotient z^T T z (zb[row * ZS + i])
template <int ZS>
__device__ __forceinline__ double rayleigh(int i, int C, const double* zb, const double* s_d, const double* s_e) {
  // z^T T z with eight rows' loads in flight and two partial sums (the rows one at a time waited
  // out an LDS round trip each); the last row's e term is masked by zeroing its factor
  double s2a = 0.0, s2b = 0.0;
  int r0 = 0;
  constexpr int U = 8;
  for (; r0 + U <= C; r0 += U) {
    double zz[U + 1], dd[U], ee[U];
#pragma unroll
    for (int u = 0; u <= U; ++u) zz[u] = zb[min(r0 + u, C - 1) * ZS + i];
#pragma unroll
    for (int u = 0; u < U; ++u) dd[u] = s_d[r0 + u], ee[u] = r0 + u < C - 1 ? s_e[r0 + u] : 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s2a = fma(dd[u] * zz[u], zz[u], s2a);
      s2b = fma(2.0 * ee[u] * zz[u], zz[u + 1], s2b);
    }
  }
  for (; r0 < C; ++r0) {
    const double z = zb[r0 * ZS + i];
    s2a = fma(s_d[r0] * z, z, s2a);
    if (r0 < C - 1) s2b = fma(2.0 * s_e[r0] * z, zb[(r0 + 1) * ZS + i], s2b);
  }
  const double s2 = s2a + s2b;
  return s2 > 0.0 ? s2 : 0.0;
}

// S6's block loop: V (C x 64 from column c0 of Z, in the MFMA accumulator layout -- see
// gram_svd_body) -= Y (T (Y^H V)) over the reflector blocks from the last, then W columns c0 + col
// = V sigma into the work buffer.  Every thread of the workgroup.
__device__ __forceinline__ void s6_back(const TwoSiteJob& j, cplx* hh, int C, int K, int c0, aqc::d4_t (&vre)[2],
                                        aqc::d4_t (&vim)[2], const double* s_sig2, int tid, int lane, int wave,
                                        int wave_s) {
  extern __shared__ double2 xbuf[];
  const int nt = wave & 3, mg = wave >> 2, li = lane & 15, lk = lane >> 4;
  // LDS (complex units): Y [128][16] (column index swizzled by row & 15: conflict-free reads along
  // rows and along columns), Y^H V partials of waves 4..15, T (from S5's precompute), W2 = T Y^H V
  cplx* Yl = xbuf;
  cplx* Pw = Yl + 2048;
  cplx* Tl = Pw + 12 * 256;      // [16][17]
  cplx* W2l = Tl + 3 * 256 + 16 * 64;
  auto fetch_y = [&](int k0, int nb, cplx (&y)[2]) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + 1024 * u, row = e >> 4, i = e & 15, k = k0 + i;
      y[u] = (i < nb && row > k && row < C) ? aqc::ldg(hh + (size_t)k * (2 * C - k - 1) / 2 + (row - k - 1))
                                            : aqc::cmk(0, 0);
    }
  };
  cplx ynx[2];
  {
    const int k1 = C - 1, k0 = k1 > 16 ? k1 - 16 : 0;
    fetch_y(k0, k1 - k0, ynx);
  }
  __syncthreads();  // V's initial values are read from zb: the LDS can be overwritten now
  for (int k1 = C - 1; k1 > 0; k1 -= 16) {
    const int k0 = k1 > 16 ? k1 - 16 : 0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + 1024 * u, row = e >> 4, i = e & 15;
      Yl[row * 16 + (i ^ (row & 15))] = ynx[u];
    }
    if (tid < 256) {  // this block's T from S5 (agent-scope loads: see the precompute)
      const gdbl_t* tp = (const gdbl_t*)(const double*)(hh + kTfacOff + (size_t)((C - 1 - k1) >> 4) * 512 + 256 + tid);
      Tl[(tid >> 4) * 17 + (tid & 15)] = aqc::cmk(__hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                                  __hip_atomic_load(tp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    __syncthreads();  // B1: Y
    // Y^H V over this wave's 32 rows: A[m = i][k = row] = conj(Y[row][i])
    // (3M: conj(y) v = P1 - P2 + i (P3 - P1 - P2), P1 = yr vr, P2 = -yi vi, P3 = (yr - yi)(vr + vi):
    // three MFMAs per k step instead of four -- S6 is matrix-core-bound)
    aqc::d4_t wr, wi;
    {
      aqc::d4_t p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0}, p3 = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (32 * mg + 16 * t + 15 > k0) {  // rows <= k0 of Y are zero (uniform per wave)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const int row = 32 * mg + 16 * t + 4 * s + lk;
            const cplx y = Yl[row * 16 + (li ^ (row & 15))];
            p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, vre[t][s], p1, 0, 0, 0);
            p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, vim[t][s], p2, 0, 0, 0);
            p3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x - y.y, vre[t][s] + vim[t][s], p3, 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) wr[q] = p1[q] - p2[q], wi[q] = p3[q] - p1[q] - p2[q];
    }
    // D layout: row b = lk + 4 q (reflector), column li
    if (mg > 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) Pw[((mg - 1) * 4 + nt) * 256 + (lk + 4 * q) * 16 + li] = aqc::cmk(wr[q], wi[q]);
    }
    __syncthreads();  // B2: partials
    if (mg == 0) {
      // Y^H V of column tile nt summed in registers, then W2 = T (Y^H V) for that tile on the matrix
      // cores right here: the sum's D layout (row lk + 4 q, column li) is the B operand of k-step q
      // and T (in the LDS since B1) the A operand -- no W1 round trip through the LDS, no B3
      aqc::d4_t br, bi, p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0}, p3 = {0, 0, 0, 0};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int b = lk + 4 * q;
        cplx w = aqc::cmk(wr[q], wi[q]);
#pragma unroll
        for (int m = 0; m < 3; ++m) w = aqc::cadd(w, Pw[(m * 4 + nt) * 256 + b * 16 + li]);
        br[q] = w.x;
        bi[q] = w.y;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const cplx t = Tl[li * 17 + 4 * q + lk];  // A[m = li][k = lk] = T[li][4 q + lk]
        p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(t.x, br[q], p1, 0, 0, 0);
        p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(t.y, bi[q], p2, 0, 0, 0);
        p3 = __builtin_amdgcn_mfma_f64_16x16x4f64(t.x + t.y, br[q] + bi[q], p3, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) W2l[(lk + 4 * q) * 64 + 16 * nt + li] = aqc::cmk(p1[q] - p2[q], p3[q] - p1[q] - p2[q]);
    }
    __syncthreads();  // B4: W2
    // the next block's reflectors, in flight during the V update: issued before B1 they were
    // drained by the spill reloads' vmcnt(0) waits between B1 and B4
    if (k0 > 0) {
      const int n1 = k0, n0 = n1 > 16 ? n1 - 16 : 0;
      fetch_y(n0, n1 - n0, ynx);
    }
    // V -= Y W2: A[m = row][k = b] = Y[row][b], B[k = b][n] = W2[b][n].  The lane's indices come
    // from the lane counter and the wave index in an SGPR: derived from the thread id (whose VGPR
    // is spilled) their reload's vmcnt(0) drained the next block's reflector loads issued above
    const int vl_ = fresh_lane();
    const int vmg = wave_s >> 2, vnt = wave_s & 3, vli = vl_ & 15, vlk = vl_ >> 4;
    // (3M: y w = P1 - P2 + i (P3 - P1 - P2), P1 = yr wr, P2 = yi wi, P3 = (yr + yi)(wr + wi); -P3
    // straight into vim, P1 and P2 into two temporaries)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (32 * vmg + 16 * t + 15 > k0) {
        const int row = 32 * vmg + 16 * t + vli;
        aqc::d4_t p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int b = 4 * s + vlk;
          const cplx y = Yl[row * 16 + (b ^ (row & 15))];
          const cplx w = W2l[b * 64 + 16 * vnt + vli];
          p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, w.x, p1, 0, 0, 0);
          p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, w.y, p2, 0, 0, 0);
          vim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-(y.x + y.y), w.x + w.y, vim[t], 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) vre[t][q] += p2[q] - p1[q], vim[t][q] += p1[q] + p2[q];
      }
    }
    __syncthreads();  // B5: Y, W2 and the partials are overwritten next block
  }
  {  // the reflectors are dead (last read before B1 of the last block): W overwrites them (a
     // first pass of K > 64 writes columns 64.. past them)
    const int col = c0 + 16 * nt + li;
    if (col < K) {
      const double sg = sqrt(s_sig2[col]);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = 32 * mg + 16 * t + lk + 4 * q;
          if (row < C) aqc::stg(j.work + (size_t)col * C + row, aqc::cmk(vre[t][q] * sg, vim[t][q] * sg));
        }
      }
    }
  }
}

// S5 for K > 64 kept vectors (gram_svd_body): the inverse iteration of the narrow path for vector i
// by thread i (waves 0-1), the vectors in the LDS at stride 128 (zb[row * 128 + i]), the pivots in
// the work scratch (Db[row * 128 + i], lanes along a row: one 512-byte access per wave).  The pivots
// are read back through agent-scope loads, eight rows ahead of the chain: a previous update's reads
// of the same addresses on this CU may sit in the L1.
__device__ __noinline__ void s5_wide(int i, int C, const double* s_d, const double* s_e, const double* s_e2,
                                     double lam, double tn, double* zb, double* Db) {
  for (int row = 0; row < C; ++row) {  // deterministic start vector, in [-1, 1) (as the narrow path)
    unsigned int h = (unsigned int)(row * 2654435761u) ^ (unsigned int)((i + 1) * 40503u);
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    zb[row * 128 + i] = (double)(h & 0xFFFFFu) * (2.0 / 1048576.0) - 1.0;
  }
  auto ldd = [&](int row) {
    return __hip_atomic_load((const gdbl_t*)(Db + row * 128 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  constexpr int U = 8;
  const double itn = 1.0 / fmax(tn, 1e-300), lamn = lam * itn;
  {  // L D L^T = T - lam I, the pivots from the leading minors (see the narrow path)
    double p0 = 0.0, p1 = 1.0;
    for (int row = 0; row < C; ++row) {
      const double d = s_d[row], e2 = s_e2[max(row - 1, 0)];
      const double dmx = fma(d, itn, -lamn), t = (e2 * itn * itn) * p0;
      const double lim = 2.220446049250313e-16 * fabs(p1);
      double p = fma(dmx, p1, -t);
      p = fabs(p) < lim ? copysign(lim, p) : p;
      aqc::stg(Db + row * 128 + i, p1 * rcp_nr(p) * itn);
      p0 = p1;
      p1 = p;
      if ((row & 7) == 7) {
        const int ex = max(__builtin_amdgcn_frexp_exp(p0), __builtin_amdgcn_frexp_exp(p1));
        p0 = __builtin_amdgcn_ldexp(p0, -ex);
        p1 = __builtin_amdgcn_ldexp(p1, -ex);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  double sc = 1.0;
  for (int it = 0; it < 3; ++it) {
    double yp = 0.0;
    int r0 = 0;
    for (; r0 + U <= C; r0 += U) {
      double zz[U], ee[U], dp[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rm = max(r0 + u - 1, 0);
        zz[u] = zb[(r0 + u) * 128 + i], ee[u] = s_e[rm], dp[u] = ldd(rm);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double y = fma(-ee[u] * dp[u], yp, zz[u] * sc);
        zb[(r0 + u) * 128 + i] = y;
        yp = y;
      }
    }
    for (; r0 < C; ++r0) {
      const int rm = max(r0 - 1, 0);
      const double y = fma(-s_e[rm] * ldd(rm), yp, zb[r0 * 128 + i] * sc);
      zb[r0 * 128 + i] = y;
      yp = y;
    }
    double zn = 0.0, n2 = 0.0;
    int r1 = C - 1;
    for (; r1 - U + 1 >= 0; r1 -= U) {
      double yy[U], ee[U], dd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int row = r1 - u;
        yy[u] = zb[row * 128 + i], ee[u] = s_e[min(row, C - 2)], dd[u] = ldd(row);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        zn = fma(-ee[u] * dd[u], zn, yy[u] * dd[u]);
        zb[(r1 - u) * 128 + i] = zn;
        n2 = fma(zn, zn, n2);
      }
    }
    for (; r1 >= 0; --r1) {
      const double d = ldd(r1);
      zn = fma(-s_e[min(r1, C - 2)] * d, zn, zb[r1 * 128 + i] * d);
      zb[r1 * 128 + i] = zn;
      n2 = fma(zn, zn, n2);
    }
    const double rs = __builtin_amdgcn_rsq(n2);
    sc = rs * fma(-0.5 * n2 * rs, rs, 1.5);
  }
  for (int row = 0; row < C; ++row) zb[row * 128 + i] *= sc;
}

// S5 and S6 of gram_svd_body for K > 64 kept triplets (kept out of the body's register allocation:
// the K <= 64 path is the one the batched chains run).  S5: vector i by thread i of waves 0-1
// (s5_wide), the factors' precompute on the waves off SIMDs 0 and 1 (2-3, 6-7, 10-11, 14-15);
// Gram-Schmidt and the Rayleigh quotients at stride 128; S6 in two passes of 64 columns, the last
// vectors first (their W lands in [64 C, 128 C), past the reflectors), the first 64 stashed in the
// work scratch (the pivots there are dead by then) and read back with agent-scope loads.
__device__ __noinline__ void gram_wide(const TwoSiteJob& j, cplx* hh, int C, int K, const double* s_d,
                                       const double* s_e, const double* s_e2, const double* s_lam, double s_tn,
                                       const cplx* s_tau, double* s_sig2) {
  extern __shared__ double2 xbuf[];
  const int tid = fresh_tid(), lane = tid & 63, wave = tid >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);
  double* zb = reinterpret_cast<double*>(xbuf);  // zb[row * 128 + i]
  double* scratch = reinterpret_cast<double*>(j.work + kWideOff);
  const int nblk = (C - 1 + 15) >> 4;
  if (tid < K) {
    s5_wide(tid, C, s_d, s_e, s_e2, s_lam[tid], s_tn, zb, scratch);
  } else if ((wave & 3) >= 2) {
    const int b = 2 * (wave >> 2) + (wave & 3) - 2;  // (uniform per wave)
    if (b < nblk) s6_factors(b, C, hh, s_tau, lane);
  }
  __syncthreads();
  if (wave == 0) gs_clusters<128>(K, C, zb, s_lam, s_tn, lane);
  __syncthreads();
  if (tid < K) s_sig2[tid] = rayleigh<128>(tid, C, zb, s_d, s_e);
  __syncthreads();
  const int nt = wave & 3, mg = wave >> 2, li = lane & 15, lk = lane >> 4;
  for (int pass = 0; pass < 2; ++pass) {
    const int c0 = pass == 0 ? kGramNarrowK : 0;
    aqc::d4_t vre[2], vim[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 32 * mg + 16 * t + lk + 4 * q, col = 16 * nt + li;
        double v = 0.0;
        if (row < C && c0 + col < K)
          v = pass == 0 ? zb[row * 128 + c0 + col]
                        : __hip_atomic_load((const gdbl_t*)(scratch + row * 64 + col), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        vre[t][q] = v;
        vim[t][q] = 0.0;
      }
    }
    if (pass == 0)  // the first 64 vectors to the scratch (read before s6_back's first barrier)
      for (int e = tid; e < C * 64; e += 1024) aqc::stg(scratch + e, zb[(e >> 6) * 128 + (e & 63)]);
    s6_back(j, hh, C, K, c0, vre, vim, s_sig2, tid, lane, wave, wave_s);
  }
}

// The kept count assumed the values in CHOP's error band chopped (gram_keep's second attempt):
// ||X - X V V^H||_F^2, the exact weight of X outside the kept right singular space, must then be
// below CHOP / 2 (gram_big.hip's k_gb_cert at 2 chi > 128).  V = W / sigma from S6's output (work,
// column c at c * C).  Y = X V (L x K) into the work scratch past W, then the residual in 64 x 64
// blocks on the matrix cores, one block per 256-thread sub-group.  Returns the sum (every thread).
// (A call: its accumulators stay out of the body's register allocation.)
__device__ __noinline__ double gram_cert128(const TwoSiteJob& j, int C, int K, const double* sig2) {
  extern __shared__ double2 xbuf[];
  __shared__ double red[16];
  const int tid = fresh_tid(), sg = tid >> 8, lt = tid & 255, wave = lt >> 6, lane = tid & 63;
  const int M = 2 * j.dims[0], N = 2 * j.dims[2];
  const bool tr = M < N;
  const int L = tr ? N : M;
  const cplx* th = j.theta;
  const cplx* W = j.work;
  cplx* Y = j.work + 16384;  // L x K, row stride 128
  static_assert(16384 + 128 * 128 <= aqc::kGramWorkElems, "certificate scratch");
  auto xel = [&](int R, int c) { return tr ? aqc::cconj(aqc::ldg(th + (size_t)R * M + c)) : aqc::ldg(th + (size_t)c * M + R); };
  // W and Y through agent-scope loads: this CU's previous update (its certificate, its split) read
  // the same addresses, and the L1 may still hold those lines (as for S6's factors)
  auto lda = [](const cplx* p) {
    const gdbl_t* q = (const gdbl_t*)(const double*)p;
    return aqc::cmk(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                    __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  };
  aqc::GemmLds& lds = reinterpret_cast<aqc::GemmLds*>(xbuf)[sg];
  const int bi = 64 * (sg >> 1), bj = 64 * (sg & 1);
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32, li = lane & 15, lk = lane >> 4;
  aqc::d4_t cr[2][2], ci[2][2];
  aqc::block_cgemm_tile<false, false, false>(
      L, K, C, bi, bj, [&](int R, int c) { return xel(R, c); },
      [&](int c, int k) { return aqc::cscale(lda(W + (size_t)k * C + c), 1.0 / sqrt(sig2[k])); }, lds, lt,
      bi < L && bj < K, cr, ci);
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = bi + wr + 16 * r + lk + 4 * q, col = bj + wc + 16 * c + li;
        if (row < L && col < K) aqc::stg(Y + (size_t)row * 128 + col, aqc::cmk(cr[r][c][q], ci[r][c][q]));
      }
  __syncthreads();
  aqc::block_cgemm_tile<false, false, false>(
      L, C, K, bi, bj, [&](int R, int k) { return lda(Y + (size_t)R * 128 + k); },
      [&](int k, int c) { return aqc::cscale(aqc::cconj(lda(W + (size_t)k * C + c)), 1.0 / sqrt(sig2[k])); }, lds,
      lt, bi < L && bj < C, cr, ci);
  double acc = 0.0;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = bi + wr + 16 * r + lk + 4 * q, col = bj + wc + 16 * c + li;
        if (row < L && col < C) {
          const cplx x = xel(row, col);
          const double dx = x.x - cr[r][c][q], dy = x.y - ci[r][c][q];
          acc = fma(dx, dx, fma(dy, dy, acc));
        }
      }
  acc = wave_sum_dpp(acc);
  if (lane == 0) red[tid >> 6] = acc;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < 16; ++w) t += red[w];
  __syncthreads();
  return t;
}

// Gram-path SVD of one 2 chi x 2 chi theta'; 1024 threads; `xbuf` = the workgroup's dynamic LDS
// (>= 4 GemmLds).  Returns false (work untouched beyond scratch, caller runs the Jacobi) when the
// fast path does not apply.  Uniform in the workgroup.
// Returns 0: declined (the caller runs the register Jacobi), 1: done, 2: done if gram_certified.
// Off by default (measured slower, profiles/r6_s3_tail_ab.json: k_chain 35.6 -> 37.75 ms -- one
// wave issuing the whole 32 x 32 block's 12 FMAs per element, four wave reductions and three LDS
// round trips per column costs more than the main loop's late columns with their two barriers);
// -DAQC_S3_TAIL=1 builds it (parity green: test_gpu_svd / headline / mps / threshold).
#ifndef AQC_S3_TAIL
#define AQC_S3_TAIL 0
#endif
constexpr int kS3Tail = 32;
#if defined(__HIP_DEVICE_COMPILE__)
using s3_lcplx = __attribute__((address_space(3))) cplx;
using s3_ldbl = __attribute__((address_space(3))) double;
#else
using s3_lcplx = cplx;
using s3_ldbl = double;
#endif
// S3's last kS3Tail = 32 columns (columns T0 = C - 32 .. C - 2) in wave 0 alone.  On entry every
// thread holds G^(T0 - 1) in the main layout (row r, columns q + 8 i) and the LDS reflector T0 - 1
// (p, v at buffer (T0 - 1) & 1, a2): the trailing block gets that reflector's rank-2 update and goes
// through the LDS to wave 0, lane l holding row l >> 1, columns (l & 1) + 2 i (i < 16) of it.  Then
// per column k' = 0 .. 30 (global K = T0 + k') the lower zhetd2 step with the main loop's zlarfg
// formulas -- column k' below the diagonal from its lane pairs, p = tau A v from the lanes' 16
// columns (v, p through a wave-private LDS vector), a2 = -tau (p^H v) / 2, A -= v p^H + (p + 2
// Re(a2) v) v^H -- with only wave-level reductions: no workgroup barrier per column (the main
// loop's two barriers and phase B hand-off cost ~3 K ticks a column at its end).  Writes d, e, tau
// and the reflectors exactly where the main loop does.
__device__ __forceinline__ void s3_tail(cplx (&g)[16], int C, int r0, int q0, int tid, int lane, int wave,
                                        s3_lcplx* lb, cplx* hh) {
  const int T0 = C - kS3Tail;
  s3_lcplx* pvb = lb;
  s3_lcplx* vbb = lb + 256;
  s3_lcplx* tauS = lb + 1921;
  s3_ldbl* eS = (s3_ldbl*)(lb + 2050);
  s3_ldbl* dS = (s3_ldbl*)(lb + 2114);
  s3_lcplx* a2b = lb + 2178;
  s3_lcplx* tile = lb + 2304;  // [32][33]
  s3_lcplx* vt = lb + 2304 + 32 * 33;
  s3_lcplx* pt = vt + 32;
  {  // reflector T0 - 1's update of the trailing block, which goes to the LDS
    const int bp = (T0 - 1) & 1;
    const int r = r0, q = q0;
    if (r >= T0 && r < C) {
      const cplx vr = vbb[bp * 128 + r], pr = pvb[bp * 128 + r];
      const double a2r2 = 2.0 * a2b[bp].x;
      const cplx wr = aqc::cmk(fma(a2r2, vr.x, pr.x), fma(a2r2, vr.y, pr.y));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = q + 8 * i;
        if (c >= T0 && c < C) {
          const cplx vc = vbb[bp * 128 + c], pc = pvb[bp * 128 + c];
          cplx x = g[i];
          x.x = fma(-vr.x, pc.x, fma(-vr.y, pc.y, fma(-wr.x, vc.x, fma(-wr.y, vc.y, x.x))));
          x.y = fma(-vr.y, pc.x, fma(vr.x, pc.y, fma(-wr.y, vc.x, fma(wr.x, vc.y, x.y))));
          tile[(r - T0) * 33 + (c - T0)] = x;
        }
      }
    }
  }
  __syncthreads();
  if (wave == 0) {
    const int rr = lane >> 1, h = lane & 1;
#pragma unroll
    for (int i = 0; i < 16; ++i) g[i] = tile[rr * 33 + 2 * i + h];
    for (int kk = 0; kk < kS3Tail - 1; ++kk) {
      const int K = T0 + kk;
      // column kk below the diagonal, on both lanes of each row
      cplx x = h == (kk & 1) ? pick16(g, kk >> 1) : aqc::cmk(0, 0);
      x.x += __shfl_xor(x.x, 1);
      x.y += __shfl_xor(x.y, 1);
      const double xn2 = wave_sum_dpp(h == 0 && rr > kk + 1 ? aqc::cnorm2(x) : 0.0);
      const double dkk = bcast_d(x.x, 2 * kk);  // (the diagonal: row kk, column kk)
      const cplx alpha = aqc::cmk(bcast_d(x.x, 2 * (kk + 1)), bcast_d(x.y, 2 * (kk + 1)));
      // zlarfg, as the main loop's wave 0
      const double x2 = fma(alpha.x, alpha.x, fma(alpha.y, alpha.y, xn2));
      double rs = __builtin_amdgcn_rsq(x2);
      rs = rs * fma(-0.5 * x2 * rs, rs, 1.5);
      rs = rs * fma(-0.5 * x2 * rs, rs, 1.5);
      const double nn = x2 * rs;
      const bool triv = xn2 == 0.0 && alpha.y == 0.0;
      const double beta = triv ? alpha.x : (alpha.x >= 0.0 ? -nn : nn);
      const double ib = alpha.x >= 0.0 ? -rs : rs;
      const double dr = alpha.x - beta, di = alpha.y, id2 = rcp_nr(fma(dr, dr, di * di));
      const cplx tau = triv ? aqc::cmk(0, 0) : aqc::cmk((beta - alpha.x) * ib, -alpha.y * ib);
      const cplx scl = triv ? aqc::cmk(0, 0) : aqc::cmk(dr * id2, -di * id2);
      // v: 1 at kk + 1, scl x below, 0 above
      cplx v = rr > kk + 1 ? aqc::cmul(x, scl) : aqc::cmk(rr == kk + 1 ? 1.0 : 0.0, 0.0);
      if (lane == 0) {
        tauS[K] = tau;
        eS[K] = beta;
        dS[K] = dkk;
      }
      if (h == 0) {
        vt[rr] = v;
        if (rr > kk) aqc::stg(hh + (size_t)K * (2 * C - K - 1) / 2 + (T0 + rr - K - 1), v);  // GLOBAL, not FLAT
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      // p = tau A v (v_c = 0 at and above kk: no masks; v_c read where used, so that no 16 of
      // them stay live beside the block)
      cplx acc = aqc::cmk(0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (2 * i + 1 > kk) acc = aqc::cfma(g[i], vt[2 * i + h], acc);  // (uniform skip)
      acc.x += __shfl_xor(acc.x, 1);
      acc.y += __shfl_xor(acc.y, 1);
      const cplx p = rr > kk ? aqc::cmul(tau, acc) : aqc::cmk(0, 0);
      const double ktx = wave_sum_dpp(h == 0 ? fma(p.x, v.x, p.y * v.y) : 0.0);
      const double kty = wave_sum_dpp(h == 0 ? fma(p.x, v.y, -p.y * v.x) : 0.0);
      const cplx a2 = aqc::cscale(aqc::cmul(tau, aqc::cmk(ktx, kty)), -0.5);
      if (h == 0) pt[rr] = p;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      const double a2r2 = 2.0 * a2.x;
      const cplx w = aqc::cmk(fma(a2r2, v.x, p.x), fma(a2r2, v.y, p.y));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (2 * i + 1 > kk) {  // (uniform)
          const cplx pc = pt[2 * i + h], vci = vt[2 * i + h];
          g[i].x = fma(-v.x, pc.x, fma(-v.y, pc.y, fma(-w.x, vci.x, fma(-w.y, vci.y, g[i].x))));
          g[i].y = fma(-v.y, pc.x, fma(v.x, pc.y, fma(-w.y, vci.x, fma(w.x, vci.y, g[i].y))));
        }
      }
    }
    // d_{C-1}: the last diagonal entry after reflector C - 2's update
    const cplx glast = pick16(g, (kS3Tail - 1) >> 1);
    const double dl = bcast_d(glast.x, 2 * (kS3Tail - 1) + ((kS3Tail - 1) & 1));
    if (lane == 0) dS[C - 1] = dl;
  }
}

// AQC_GRAM_INLINE=1: the body inlined into its callers (no call frame: the callee-saved VGPR saves
// of a real call go to scratch on every update)
#ifndef AQC_GRAM_INLINE
#define AQC_GRAM_INLINE 0
#endif
#if AQC_GRAM_INLINE
__device__ __forceinline__
#else
__device__ __noinline__
#endif
int gram_svd_body(const TwoSiteJob& j) {
  extern __shared__ double2 xbuf[];
  __shared__ double s_d[128], s_e[128], s_e2[128], s_lam[128], s_err[128], s_sig2[kGramMaxK], s_tail;
  __shared__ int s_K, s_cert;
  __shared__ cplx s_tau[128];
  __shared__ double s_lo, s_hi, s_tn;
  __shared__ double2 s_de[128];
  const int chl = j.dims[0], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = M < N;
  const int L = tr ? N : M, C = tr ? M : N;
  // eigenvalues computed: the top KE (max_chi, if it binds, caps the kept count first); the kept
  // count K itself follows reduce_zeros on them after S4 (gram_keep)
  const int KE = (j.max_chi > 0 && j.max_chi < C) ? j.max_chi : C;
  // (j.work holds the packed reflectors, <= 8128 complex: capacity 64)
  const int tid = fresh_tid(), lane = tid & 63, wave = tid >> 6;
  const int wave_s = __builtin_amdgcn_readfirstlane(wave);  // (uniform: an SGPR)
  if (tid == 0) atomicAdd(&g_gram_stats[0], 1ull);
  if (C < 4 || C > 128 || L > 128 || j.cap < 64) {
    if (tid == 0) atomicAdd(&g_gram_stats[2], 1ull);
    return 0;
  }
  const cplx* th = j.theta;
  unsigned long long t_last = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
  auto tick = [&](int ph) {
    if (tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      atomicAdd(&g_gram_ticks[ph], t - t_last);
      t_last = t;
    }
  };
  // the tridiagonalisation's two per-step phases (t_b: A, t_a: B) add up in registers (one atomic
  // each at the end)
  unsigned long long t_a = 0, t_b = 0;
  auto tick_step = [&](unsigned long long& acc) {
    if (tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc += t - t_last;
      t_last = t;
    }
  };
  // ---- S1: G = X^H X on the matrix cores.  Only the 16 x 16 tiles on and above the diagonal
  // (36 at C = 128), dealt to the 16 waves round-robin (at most 3 each, 9 per SIMD; the 64 x 64
  // sub-group blocks of round 2 computed 48 tiles on 12 waves, 12 per SIMD).  Each complex tile
  // is three real products (the 3M form of conj(a + ib)(c + id) = (ac + bd) + i(ad - bc)):
  // P1 = Xr^T Xr, P2 = Xi^T Xi, P3 = (Xr + Xi)^T (Xr - Xi); Re G = P1 + P2, Im G = P1 - P2 - P3
  // (absolute error a few eps ||X||^2, the Gram path's eps ||G|| budget).  X streams once through
  // double-buffered LDS chunks of 8 rows (Xr, Xi, Xr + Xi, Xr - Xi), the next chunk's global
  // load in flight during the current chunk's MFMAs: 256 KB read per SVD (768 KB before). ----
  const int r0 = tid >> 3, q0 = tid & 7;
  const int r = r0, q = q0;
  cplx g[16];
  {
    constexpr int KC = 8, PITCH = 144;  // rows per chunk; row pitch (doubles): rows k, k + 1 on
                                        // opposite bank halves for the 16-lane operand reads
    constexpr int ARR = KC * PITCH, BUF = 4 * ARR;
    double* sb = reinterpret_cast<double*>(xbuf);
    const int nt = (C + 15) >> 4, ntile = nt * (nt + 1) / 2;
    int tI[3], tJ[3];
    bool tact[3];
    // C = 128 (nt = 8): each wave's tiles share their row block, so the wave reads the A operands
    // once per step for all its tiles (12 instead of 18 LDS operand reads; the pass is LDS-bound);
    // 15 waves of 1-3 tiles, 9 tiles per SIMD (wave w on SIMD w % 4).  Entry: row block,
    // first column block, tile count.
    const bool rs = nt == 8;  // uniform
    if (rs) {
      constexpr unsigned kTab[16] = {0x300, 0x322, 0x333, 0x355, 0x330, 0x352, 0x241, 0x244,
                                     0x311, 0x260, 0x261, 0x264, 0x000, 0x177, 0x263, 0x266};
      const unsigned e = kTab[wave];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        tact[u] = u < (int)(e >> 8);
        tI[u] = e & 15;
        tJ[u] = ((e >> 4) & 15) + u;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 3; ++u) {  // tile t -> (ti <= tj), row-major over the upper triangle
        int t = wave + 16 * u, ti = 0;
        tact[u] = t < ntile;
        while (tact[u] && t >= nt - ti) t -= nt - ti++;
        tI[u] = ti;
        tJ[u] = ti + t;
      }
    }
    const int nch = (L + KC - 1) / KC;
    auto fetch = [&](int ch) {  // this thread's element of chunk ch (zero outside X)
      const int kk = ch * KC + (tr ? tid >> 7 : tid & 7), c = tr ? tid & 127 : tid >> 3;
      if (kk >= L || c >= C) return aqc::cmk(0, 0);
      // (raw: the conjugate of the transposed case is taken in stash, so that the load stays in
      // flight during the chunk's MFMAs instead of being waited for here)
      return tr ? aqc::ldg(th + (size_t)kk * M + c) : aqc::ldg(th + (size_t)c * M + kk);
    };
    auto stash = [&](int buf, cplx x) {
      if (tr) x.y = -x.y;
      const int o = buf * BUF + (tr ? tid >> 7 : tid & 7) * PITCH + (tr ? tid & 127 : tid >> 3);
      sb[o] = x.x;
      sb[o + ARR] = x.y;
      sb[o + 2 * ARR] = x.x + x.y;
      sb[o + 3 * ARR] = x.x - x.y;
    };
    aqc::d4_t p1[3], p2[3], p3[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) p1[u] = p2[u] = p3[u] = aqc::d4_t{0, 0, 0, 0};
    stash(0, fetch(0));
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      const bool more = ch + 1 < nch;
      cplx xn = aqc::cmk(0, 0);
      if (more) xn = fetch(ch + 1);
      const double* cb = sb + (ch & 1) * BUF;
      // the lane index from the lane counter, per chunk: derived from the (spilled) thread id, its
      // reload's vmcnt wait drained the next chunk's load issued just above
      const int fl = fresh_lane();
#pragma unroll
      for (int ks = 0; ks < KC / 4; ++ks) {
        const int row = (4 * ks + (fl >> 4)) * PITCH + (fl & 15);
        if (rs) {  // uniform: the row block's operands once, then each tile's column block
          const int oi = row + 16 * tI[0];
          const double ar = cb[oi], ai = cb[ARR + oi], as = cb[2 * ARR + oi];
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            if (tact[u]) {  // uniform per wave
              const int oj = row + 16 * tJ[u];
              p1[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, cb[oj], p1[u], 0, 0, 0);
              p2[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, cb[ARR + oj], p2[u], 0, 0, 0);
              p3[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(as, cb[3 * ARR + oj], p3[u], 0, 0, 0);
            }
          }
        } else {
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            if (tact[u]) {  // uniform per wave
              const int oi = row + 16 * tI[u], oj = row + 16 * tJ[u];
              p1[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(cb[oi], cb[oj], p1[u], 0, 0, 0);
              p2[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(cb[ARR + oi], cb[ARR + oj], p2[u], 0, 0, 0);
              p3[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(cb[2 * ARR + oi], cb[3 * ARR + oj], p3[u], 0, 0, 0);
            }
          }
        }
      }
      if (more) stash((ch + 1) & 1, xn);
      __syncthreads();
    }
    // ---- S2: the upper triangle through the LDS (free after the last chunk's barrier) into the
    // tridiagonalisation's register layout: thread (r, q) holds row r, columns q + 8 i.  LDS:
    // block (0, 1) square (row stride 65) then the packed upper triangles of the diagonal 64 x 64
    // blocks (column-major, entry (a, b), a <= b, at b (b + 1) / 2 + a): 8320 complex ----
    cplx* gsq = xbuf;
    auto up_index = [](int a, int b) {  // G[a][b], a <= b
      if (b < 64) return 64 * 65 + b * (b + 1) / 2 + a;
      if (a >= 64) return 64 * 65 + 2080 + (b - 64) * (b - 63) / 2 + (a - 64);
      return a * 65 + (b - 64);
    };
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      if (tact[u]) {  // MFMA C/D layout: row (lane >> 4) + 4 q, column lane & 15
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int a = 16 * tI[u] + (lane >> 4) + 4 * qq, b = 16 * tJ[u] + (lane & 15);
          if (a <= b && b < C)
            gsq[up_index(a, b)] = aqc::cmk(p1[u][qq] + p2[u][qq], p1[u][qq] - p2[u][qq] - p3[u][qq]);
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = q + 8 * i, rw = r;
      cplx v = aqc::cmk(0, 0);
      if (rw < C && c < C) {
        v = gsq[c >= rw ? up_index(rw, c) : up_index(c, rw)];
        if (c < rw) v.y = -v.y;
      }
      g[i] = v;
    }
    __syncthreads();  // the reflectors' scratch reuses the LDS
  }
  tick(0);
  // reflector k at hh[k (2C - k - 1) / 2 + (row - k - 1)].  The base is uniform: moved to SGPRs
  // (as a VGPR pair it was spilled, and phase B's scratch reload waited out vmcnt(0) every column)
  cplx* hh = uniform_ptr(j.work);
  // ---- S3: tridiagonalisation (zhetd2, lower), one barrier per column ----
  // Reflector k (v_{k+1} = 1, p = tau G^(k) v, a2 = -tau (p^H v) / 2, w = p + a2 v,
  // G^(k+1) = G^(k) - v w^H - w v^H on the trailing block) reaches the registers one phase late,
  // fused with the next reflector's product: column k + 1 of G^(k+1) below the diagonal is
  // z_r - s v_r with z_r = G^(k)[r][k+1] - p_r (known before the barrier) and the scalar
  // s = conj(p_{k+1}) + 2 Re(a2) (after it).  A phase reads (p, v, z) of reflector k - 1 from the
  // LDS, reduces p^H v and |z - s v|^2 in every wave (two rows per lane: no cross-wave partial
  // sums, the column is formed explicitly, no cancellation), forms reflector k, updates g by
  // reflector k - 1 and multiplies it by reflector k's column in one pass over the columns, and
  // writes (p, v, z) of reflector k.  LDS vectors are double-buffered by phase parity and zero
  // where the reflector vanishes, so neither the update nor the product needs masks.
  // LDS addressing for the column loop from one base laundered once: from a non-inlined function
  // the dynamic LDS base and the function's own __shared__ arrays are found through a table in
  // memory, and the compiler re-read it with an s_load per column group -- whose lgkmcnt(0) wait
  // drained every outstanding LDS read.  The loop's scalars live in the dynamic LDS too; d, e and
  // tau go to the static arrays after the loop.
#if defined(__HIP_DEVICE_COMPILE__)
  using lcplx = __attribute__((address_space(3))) cplx;
  using ldbl = __attribute__((address_space(3))) double;
#else  // (the host pass only parses device code)
  using lcplx = cplx;
  using ldbl = double;
#endif
  lcplx* lb = (lcplx*)xbuf;
  asm volatile("" : "+s"(lb));
  lcplx* pvb = lb;           // [2][128] p   (0 at and above row k)
  lcplx* vbb = lb + 256;     // [2][128] v   (0 at and above row k, 1 at k + 1)
  lcplx* xvb = lb + 512;     // [2][128] x = z - s v, column k + 1 of G^(k+1) below row k + 1 (else 0)
  lcplx* accp = lb + 768;    // [8][128] the column pass's partial products g x, per lane of a row
  lcplx* gk1b = lb + 1792;   // [128] G^(k)[r][k+1]
  lcplx* tauS = lb + 1921;   // reflector k's tau at tauS[k]; tauS[-1] = 0 ("reflector -1")
  ldbl* eS = (ldbl*)(lb + 2050);  // [128] beta_k = e_k
  ldbl* dS = (ldbl*)(lb + 2114);  // [128] d_k
  lcplx* a2b = lb + 2178;    // [2] reflector k's a2 = -tau (p^H v) / 2, by phase parity
  lcplx* scal = lb + 2180;   // reflector k's 1 / (alpha - beta), tau / (alpha - beta)
  lcplx* ktp = lb + 2183;    // [2] p^H v partials of phase B's two waves (rows 0-63, 64-127)
  volatile __attribute__((address_space(3))) int* hsf =
      (volatile __attribute__((address_space(3))) int*)(lb + 2185);  // [2] phase B's hand-off flags: k + 1
  // "reflector -1": none, and column 0 of G as x (s = 0)
  if (tid == 0) {
    tauS[-1] = aqc::cmk(0, 0);
    a2b[1] = aqc::cmk(0, 0);
    hsf[0] = hsf[1] = 0;
  }
  if (q == 0) {
    pvb[128 + r] = aqc::cmk(0, 0);
    vbb[128 + r] = aqc::cmk(0, 0);
    xvb[128 + r] = (r > 0 && r < C) ? g[0] : aqc::cmk(0, 0);
  }
  __syncthreads();
  // the last kS3Tail columns in wave 0 alone (AQC_S3_TAIL): no workgroup barrier per column
  const bool s3tail = AQC_S3_TAIL && C >= 64;
  const int kEnd = s3tail ? C - kS3Tail : C - 1;
  for (int k = 0; k < kEnd; ++k) {
    const int b = k & 1, bp = b ^ 1;
    // q and r laundered through an empty asm each step: otherwise the compiler hoists the 16
    // columns' loop-invariant index / address values out of the k loop and spills them
    int q = q0, r = r0;
    asm volatile("" : "+v"(q), "+v"(r));
    // rows >= k change this phase (row k: reflector k - 1's update gives d_k): waves whose rows
    // are all below k only clear their LDS entries (uniform branch)
    const bool wact = wave * 8 + 7 >= k;
    // Phase A: reflector k - 1's scalars (every active wave: the column pass needs a2 and s), the
    // column pass, and -- in wave 0 alone, whose rows are finished from k = 8 on -- reflector k's
    // zlarfg scalars, handed to the other waves through the LDS behind a second barrier.  (With
    // every wave forming them redundantly, four waves per SIMD issued the whole scalar chain: it
    // was 60% of this loop's time.)
    double a2x = 0.0;  // Re(a2) of reflector k - 1 (an LDS broadcast, held in an SGPR)
    if (wact) a2x = uniform_d(a2b[bp].x);
    if (wave == 0) {
      __builtin_amdgcn_s_setprio(3);
      // column k of G^(k) below the diagonal: x_r (r > k, formed by phase B); alpha = x_{k+1}
      double xn2;
      {
        const cplx x0 = xvb[bp * 128 + lane], x1 = xvb[bp * 128 + 64 + lane];
        const double n0 = lane > k + 1 ? aqc::cnorm2(x0) : 0.0, n1 = lane + 64 > k + 1 ? aqc::cnorm2(x1) : 0.0;
        xn2 = wave_sum_dpp(n0 + n1);
      }
      const cplx alpha = xvb[bp * 128 + k + 1];
      // reflector k's scalars (zlarfg); rsq / rcp seeds with Newton steps (full precision)
      // instead of the IEEE sqrt / divide sequences
      const double x2 = fma(alpha.x, alpha.x, fma(alpha.y, alpha.y, xn2));
      double rs = __builtin_amdgcn_rsq(x2);
      rs = rs * fma(-0.5 * x2 * rs, rs, 1.5);
      rs = rs * fma(-0.5 * x2 * rs, rs, 1.5);
      const double nn = x2 * rs;
      const bool triv = xn2 == 0.0 && alpha.y == 0.0;  // H = I
      const double beta = triv ? alpha.x : (alpha.x >= 0.0 ? -nn : nn);
      const double ib = alpha.x >= 0.0 ? -rs : rs;  // 1 / beta
      const double dr = alpha.x - beta, di = alpha.y, id2 = rcp_nr(fma(dr, dr, di * di));
      const cplx tau = triv ? aqc::cmk(0, 0) : aqc::cmk((beta - alpha.x) * ib, -alpha.y * ib);
      const cplx scl = triv ? aqc::cmk(0, 0) : aqc::cmk(dr * id2, -di * id2);  // 1 / (alpha - beta)
      if (lane == 0) {
        tauS[k] = tau;
        eS[k] = beta;
        scal[0] = scl;
        scal[1] = aqc::cmul(tau, scl);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (wact) {
      // the own row's reflector k - 1 entries and w_r (the Hermitian rank-2 update needs only
      // Re(a2): v w^H + w v^H = v p^H + (p + 2 Re(a2) v) v^H, so no per-column w_c)
      cplx acc = aqc::cmk(0, 0);
      const cplx vr = vbb[bp * 128 + r];
      const cplx pr = pvb[bp * 128 + r];
      const double a2r2 = 2.0 * a2x;
      const cplx wr = aqc::cmk(fma(a2r2, vr.x, pr.x), fma(a2r2, vr.y, pr.y));
      const double nvx = -vr.x, nvy = -vr.y, nwx = -wr.x, nwy = -wr.y;
      // one pass: g -= v_r conj(p_c) + w_r conj(v_c) (reflector k - 1), acc += g x_c (reflector k):
      // 12 FMAs per element (x_c comes formed from phase B, not re-formed from z_c - s v_c by each
      // of the eight row lanes holding column c: 16 until round 5)
      auto col = [&](int i, const cplx& vc, const cplx& pc, const cplx& xc) {
        g[i].x = fma(nvx, pc.x, fma(nvy, pc.y, fma(nwx, vc.x, fma(nwy, vc.y, g[i].x))));
        g[i].y = fma(nvy, pc.x, fma(vr.x, pc.y, fma(nwy, vc.x, fma(wr.x, vc.y, g[i].y))));
        acc = aqc::cfma(g[i], xc, acc);
      };
      // Rolling prefetch: column i + 1's v, p, z are requested before column i is computed, so
      // each LDS round trip hides behind one column's 16 FMAs (loaded and consumed one column at a
      // time, every column waited out a full LDS latency: ~4 K of a step's ~4.6 K ticks).  The
      // active columns start at group k / (8 GR) of GR column registers (uniform: every column q + 8 i
      // of a lower group is below k, so v_c = p_c = z_c = 0 there and the pass would change nothing);
      // its first column is loaded up front.  (Groups of four registers -- 32 columns -- until round 5.)
#ifndef AQC_S3_GROUP
#define AQC_S3_GROUP 2
#endif
      constexpr int GR = AQC_S3_GROUP;  // column registers per skip group
      const int gi0 = k / (8 * GR);
      cplx cv, cp, cz;
      {
        const int c = q + 8 * GR * gi0;
        cv = vbb[bp * 128 + c], cp = pvb[bp * 128 + c], cz = xvb[bp * 128 + c];
      }
#pragma unroll
      for (int gi = 0; gi < 16 / GR; ++gi) {
        if (gi >= gi0) {  // uniform; v_c = p_c = z_c = 0 for c < k
#pragma unroll
          for (int ii = 0; ii < GR; ++ii) {
            const int i = GR * gi + ii;
            cplx nv = cv, np = cp, nz = cz;
            if (i + 1 < 16) {
              const int c = q + 8 * (i + 1);
              nv = vbb[bp * 128 + c], np = pvb[bp * 128 + c], nz = xvb[bp * 128 + c];
            }
            __builtin_amdgcn_sched_barrier(0);
            col(i, cv, cp, cz);
            cv = nv, cp = np, cz = nz;
          }
        }
      }
      // (the product used x_{k+1} = alpha where reflector k has alpha - beta: corrected in phase B)
      // (k + 1) >> 3 == k >> 3 except every eighth column: the same register, so one pick
      cplx gk = pick16(g, k >> 3);
      // (materialised here: picked only under the d_k store below, it moved into that branch and
      // the allocator spilled g's imaginary parts for the whole pass)
      asm volatile("" : "+v"(gk.x), "+v"(gk.y));
      const cplx gk1 = ((k + 1) & 7) ? gk : pick16(g, (k + 1) >> 3);
      if (q == (k & 7) && r == k) dS[k] = gk.x;  // G^(k)[k][k]
      // the row's eight partial products are in eight adjacent lanes of this wave: summed here
      // (DPP, VALU slack -- the pass is LDS-bound), so phase B reads one value per row
      acc.x = aqc::row_sum8(acc.x);
      acc.y = aqc::row_sum8(acc.y);
      if (q == 0) accp[r] = acc;
      if (q == ((k + 1) & 7)) gk1b[r] = gk1;
    }
    __syncthreads();
    tick_step(t_b);
    // Phase B, one row per thread of waves 0 and 1: reflector k's p and v (the row's eight partial
    // products summed from the LDS; every row, so finished rows get their zeros); the two waves hand
    // each other their halves of p^H v through the LDS (a flag per wave, no workgroup barrier), then
    // each forms a2, s = conj(p_{k+1}) + 2 Re(a2) and its rows' x = z - s v with z_r = G^(k)[r][k+1]
    // - p_r -- the next column pass's operand, formed once here instead of by each of the eight row
    // lanes holding a column.  (All 128 rows in wave 0 alone, two per lane: phase B 131 K -> 226 K
    // ticks, which ate the pass's gain.)
    if (wave < 2) {
      int rr = tid;
      asm volatile("" : "+v"(rr));  // (laundered like q and r)
      const double beta = eS[k];
      const cplx ts = scal[1], scl = scal[0];
      const cplx g1 = gk1b[rr];
      cplx sum = accp[rr];
      sum.x = fma(-beta, g1.x, sum.x);  // x_{k+1} = alpha where reflector k has alpha - beta
      sum.y = fma(-beta, g1.y, sum.y);
      const bool rowact = rr > k && rr < C, below = rr > k + 1 && rr < C;
      cplx p = aqc::cmul(ts, sum);
      if (!rowact) p = aqc::cmk(0, 0);
      // reflector k's v: 1 at k + 1, scl x_r below, 0 above
      cplx v = aqc::cmul(xvb[bp * 128 + rr], scl);
      if (!below) v = aqc::cmk(rr == k + 1 ? 1.0 : 0.0, 0.0);
      pvb[b * 128 + rr] = p;
      vbb[b * 128 + rr] = v;
      if (rowact) aqc::stg(hh + (size_t)k * (2 * C - k - 1) / 2 + (rr - k - 1), v);  // GLOBAL, not FLAT
      // z_r parked in x's slot until s is known (nothing of the row stays live across the wait)
      xvb[b * 128 + rr] = below ? aqc::csub(g1, p) : aqc::cmk(0, 0);
      const double ktx = wave_sum_dpp(fma(p.x, v.x, p.y * v.y)), kty = wave_sum_dpp(fma(p.x, v.y, -p.y * v.x));
      if (lane == 0) ktp[wave] = aqc::cmk(ktx, kty);
      // (the LDS serves one wave's requests in order: partial, then flag; the fence keeps the
      // compiler from reordering the two stores and waits for both)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) hsf[wave] = k + 1;
      while (hsf[wave ^ 1] != k + 1) __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const cplx a2 = aqc::cscale(aqc::cmul(tauS[k], aqc::cadd(ktp[0], ktp[1])), -0.5);  // (same order in both)
      const cplx pk = pvb[b * 128 + k + 1];
      const double sx = -(pk.x + 2.0 * a2.x), sy = pk.y;  // -s
      int r2 = tid;
      asm volatile("" : "+v"(r2));
      if (r2 > k + 1 && r2 < C) xvb[b * 128 + r2] = aqc::cfma(aqc::cmk(sx, sy), vbb[b * 128 + r2], xvb[b * 128 + r2]);
      if (tid == 0) a2b[b] = a2;
    }
    __syncthreads();
    tick_step(t_a);
  }
  if (s3tail) {
    s3_tail(g, C, r0, q0, tid, lane, wave, lb, hh);
  } else
  // d_{C-1}: reflector C - 2's update of the last diagonal entry
  if (wave == (C - 1) >> 3) {
    const int bp = (C - 2) & 1;
    const cplx a2 = a2b[bp];
    const bool own = r0 == C - 1 && q0 == ((C - 1) & 7);
    const int gi = (C - 1) >> 3;
    if (own) {
      const cplx v = vbb[bp * 128 + C - 1], p = pvb[bp * 128 + C - 1];
      const cplx w = aqc::cfma(a2, v, p);
      const cplx gl = pick16(g, gi);
      dS[C - 1] = gl.x - 2.0 * (v.x * w.x + v.y * w.y);  // Re(g - v conj(w) - w conj(v))
    }
  }
  __syncthreads();
  for (int i = tid; i < C; i += 1024) {
    s_d[i] = dS[i];
    if (i < C - 1) {
      s_e[i] = eS[i];
      s_tau[i] = tauS[i];
    }
  }
  __syncthreads();
  if (tid == 0) {
    atomicAdd(&g_gram_ticks[6], t_a + t_b);
    atomicAdd(&g_gram_ticks[8], t_b);
  }
  tick(1);
  // ---- S4: top-K eigenvalues of T by multisection ----
  if (wave == 0) {  // Gershgorin interval, ||T||, e^2 and the (d, e^2) pairs: two rows per lane
    double lo = 1e300, hi = -1e300, tn = 0.0;
    for (int i = lane; i < C; i += 64) {
      const double el = i > 0 ? fabs(s_e[i - 1]) : 0.0, er = i < C - 1 ? fabs(s_e[i]) : 0.0;
      const double di = s_d[i];
      lo = fmin(lo, di - el - er);
      hi = fmax(hi, di + el + er);
      tn = fmax(tn, fabs(di) + el + er);
      if (i < C - 1) s_e2[i] = s_e[i] * s_e[i];
      s_de[i] = make_double2(di, i > 0 ? s_e[i - 1] * s_e[i - 1] : 0.0);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      lo = fmin(lo, __shfl_xor(lo, off));
      hi = fmax(hi, __shfl_xor(hi, off));
      tn = fmax(tn, __shfl_xor(tn, off));
    }
    if (lane == 0) {
      const double span = fmax(hi - lo, 1e-300);
      s_lo = lo - 1e-12 * span;
      s_hi = hi + 1e-12 * span;
      s_tn = tn;
    }
    // the Sturm recurrence's rows scaled by 1 / ||T|| (sturm_count_poly)
    const double itn = 1.0 / fmax(tn, 1e-300);
    for (int i = lane; i < C; i += 64) {
      const double2 de = s_de[i];
      s_de[i] = make_double2(de.x * itn, de.y * itn * itn);
    }
  }
  __syncthreads();
  {
    // Multisection with the polynomial Sturm count (one dependent FMA per row): a pass is now
    // issue-bound at ~7 VALU instructions per row and wave, so one wave per SIMD runs it.  One
    // pass of kFirst = 256 shifts (waves 0-3) brackets every eigenvalue to span / 257, then
    // kRounds rounds of (kG + 1)-section with kG = 4 lanes per eigenvalue (64 x 4 = 256 lanes)
    // narrow it by 5^12 (span x 1.6e-11 at the end; the 1024-point pass + 17^6 of round 2 gave
    // 4e-11).  Waves 4-15 sit S4 out.  (Ratio form, 16 lanes x 17-section, 7 passes: 0.20 M
    // ticks; ratio form, 8 lanes x 9-section, 9 passes: 0.15 M.)
    constexpr int kG = 4, kFirst = 256, kRounds = 12;
    static_assert(kG == 4 || kG == 8 || kG == 16, "lanes per eigenvalue");
    const int eid = tid / kG, sub = tid % kG;
    const int a = C - 1 - eid;  // ascending index of the eid-th largest eigenvalue
    int* cntb = reinterpret_cast<int*>(xbuf);
    const double lo0 = s_lo, span0 = s_hi - s_lo;
    const double itn = 1.0 / fmax(s_tn, 1e-300);
    constexpr double kInvF = 1.0 / (kFirst + 1), kInvG = 1.0 / (kG + 1);
    if (tid < kFirst) cntb[tid] = sturm_count_poly(s_de, C, (lo0 + span0 * (double)(tid + 1) * kInvF) * itn);
    __syncthreads();
    // with a tail threshold above the Gram form's noise the reduce_zeros decisions compare sums of
    // small eigenvalues with it: three more rounds bring the brackets (span x 1.6e-11) down to that
    // noise (gram_keep)
    const int rounds = kRounds + (j.thr > 1e-12 * s_tn ? 3 : 0);
    if (tid < KE * kG) {  // (whole kG-lane groups)
      double lo, hi;
      {
        int l = 0, h = kFirst;  // first t with cnt[t] >= a + 1 (kFirst: none)
        while (l < h) {
          const int m = (l + h) >> 1;
          if (cntb[m] >= a + 1) h = m;
          else l = m + 1;
        }
        lo = l > 0 ? lo0 + span0 * (double)l * kInvF : s_lo;
        hi = l < kFirst ? lo0 + span0 * (double)(l + 1) * kInvF : s_hi;
      }
      for (int round = 0; round < rounds; ++round) {
        const double x = lo + (hi - lo) * (double)(sub + 1) * kInvG;
        const int cnt = sturm_count_poly(s_de, C, x * itn);
        const unsigned long long bal = __ballot(cnt >= a + 1);
        const unsigned int gm = (unsigned int)(bal >> (lane & ~(kG - 1))) & ((1u << kG) - 1u);
        const int f = gm ? __builtin_ctz(gm) : kG;
        const double nhi = f < kG ? lo + (hi - lo) * (double)(f + 1) * kInvG : hi;
        const double nlo = f > 0 ? lo + (hi - lo) * (double)f * kInvG : lo;
        lo = nlo;
        hi = nhi;
      }
      if (sub == 0) {
        s_lam[eid] = 0.5 * (lo + hi);
        s_err[eid] = 0.5 * (hi - lo);
      }
    }
  }
  __syncthreads();
  if (tid == 0) s_K = aqc::gram_keep(s_lam, s_err, KE, C, j.max_chi, j.thr, s_tn, kGramRelFloor, s_tail, &s_cert);
  __syncthreads();
  tick(2);
  const int K = s_K;  // (uniform)
  if (K < 0) {  // open decisions / below the floor
    if (tid == 0) atomicAdd(&g_gram_stats[3], 1ull);
    return 0;
  }
  if (K > kGramNarrowK) {  // (uniform)
    gram_wide(j, hh, C, K, s_d, s_e, s_e2, s_lam, s_tn, s_tau, s_sig2);
    tick(4);
  } else {
  // ---- S5: inverse iteration, Gram-Schmidt in clusters, Rayleigh quotients ----
  double* zb = reinterpret_cast<double*>(xbuf);  // zb[row * 64 + i]
  double* Db = zb + 128 * 64;                    // 1 / D_row of vector i at Db[row * 64 + i]
  if (tid < K) {
    const int i = tid;
    const double lam = s_lam[i];
    const double piv = 2.220446049250313e-16 * s_tn;
    for (int row = 0; row < C; ++row) {  // deterministic start vector, in [-1, 1)
      unsigned int h = (unsigned int)(row * 2654435761u) ^ (unsigned int)((i + 1) * 40503u);
      h ^= h >> 13;
      h *= 0x5bd1e995u;
      h ^= h >> 15;
      zb[row * 64 + i] = (double)(h & 0xFFFFFu) * (2.0 / 1048576.0) - 1.0;
    }
    // L D L^T = T - lam I once (no pivoting; tiny pivots -> +-eps ||T||): 1 / D_row to Db.  The
    // recurrences below are serial per lane: T's entries and the vectors' rows are loaded eight
    // rows ahead of the dependent chain (read one at a time, every step waited out an LDS round
    // trip: 161 K ticks for S5)
    constexpr int U = 8;
    // (full chunks unguarded -- C is uniform but not known to the compiler, whose per-row guards
    // became exec-mask branches -- then a scalar tail; clamped indices with zero carries make the
    // first / last rows regular)
    // The pivots as ratios of the leading minors of T - lam I (the recurrence of S4's Sturm count,
    // in units of ||T||): D_row = p_row / p_{row-1}, p_row = (d - lam) p_{row-1} - e^2 p_{row-2},
    // so the dependent chain is one FMA and the pivot guard (|D| < eps -> +-eps) per row; each
    // 1 / D = p_{row-1} / p_row is formed off the chain.  Rescaled by the binary exponent every
    // chunk of 8 rows (the guard bounds the shrink per row by eps, the growth by 3).
    (void)piv;
    const double itn = 1.0 / fmax(s_tn, 1e-300), lamn = lam * itn;
    double p0 = 0.0, p1 = 1.0;  // p_{row-2}, p_{row-1}; row 0 has no e term
    auto fac_row = [&](int row, double d, double e2, double& unused) {
      (void)unused;
      const double dmx = fma(d, itn, -lamn), t = (e2 * itn * itn) * p0;
      const double lim = 2.220446049250313e-16 * fabs(p1);
      double p = fma(dmx, p1, -t);
      p = fabs(p) < lim ? copysign(lim, p) : p;
      Db[row * 64 + i] = p1 * rcp_nr(p) * itn;
      p0 = p1;
      p1 = p;
    };
    {
      double rdp = 0.0;
      int r0 = 0;
      for (; r0 + U <= C; r0 += U) {
        double dd[U], ee[U];
#pragma unroll
        for (int u = 0; u < U; ++u) dd[u] = s_d[r0 + u], ee[u] = s_e2[max(r0 + u - 1, 0)];
#pragma unroll
        for (int u = 0; u < U; ++u) fac_row(r0 + u, dd[u], ee[u], rdp);
        const int ex = max(__builtin_amdgcn_frexp_exp(p0), __builtin_amdgcn_frexp_exp(p1));
        p0 = __builtin_amdgcn_ldexp(p0, -ex);
        p1 = __builtin_amdgcn_ldexp(p1, -ex);
      }
      for (; r0 < C; ++r0) fac_row(r0, s_d[r0], s_e2[max(r0 - 1, 0)], rdp);
    }
    double sc = 1.0;  // the previous iteration's normalisation, applied as the forward solve reads
    for (int it = 0; it < 3; ++it) {
      // forward solve L y = sc z in place (L_{row, row-1} = e_{row-1} / D_{row-1}), then L^T-solve
      // z = D^-1 y - L^T z from the bottom
      // (one dependent FMA per row in both solves: the row's coefficients -e_{r-1} / D_{r-1} and
      // z sc, or e_r / D_r and y / D_r, are formed off the chain)
      double yp = 0.0;
      auto fwd_row = [&](int row, double z, double e, double dp) {
        const double y = fma(-e * dp, yp, z * sc);
        zb[row * 64 + i] = y;
        yp = y;
      };
      int r0 = 0;
      for (; r0 + U <= C; r0 += U) {
        double zz[U], ee[U], dp[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rm = max(r0 + u - 1, 0);
          zz[u] = zb[(r0 + u) * 64 + i], ee[u] = s_e[rm], dp[u] = Db[rm * 64 + i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) fwd_row(r0 + u, zz[u], ee[u], dp[u]);
      }
      for (; r0 < C; ++r0) {
        const int rm = max(r0 - 1, 0);
        fwd_row(r0, zb[r0 * 64 + i], s_e[rm], Db[rm * 64 + i]);
      }
      double zn = 0.0, n2 = 0.0;
      auto bwd_row = [&](int row, double y, double e, double d) {
        zn = fma(-e * d, zn, y * d);
        zb[row * 64 + i] = zn;
        n2 = fma(zn, zn, n2);
      };
      int r1 = C - 1;  // rows r1, r1 - 1, ..., r1 - U + 1
      for (; r1 - U + 1 >= 0; r1 -= U) {
        double yy[U], ee[U], dd[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = r1 - u;
          yy[u] = zb[row * 64 + i], ee[u] = s_e[min(row, C - 2)], dd[u] = Db[row * 64 + i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) bwd_row(r1 - u, yy[u], ee[u], dd[u]);
      }
      for (; r1 >= 0; --r1) bwd_row(r1, zb[r1 * 64 + i], s_e[min(r1, C - 2)], Db[r1 * 64 + i]);
      const double rs = __builtin_amdgcn_rsq(n2);
      sc = rs * fma(-0.5 * n2 * rs, rs, 1.5);
    }
    {  // the last iteration's normalisation
      int r0 = 0;
      for (; r0 + U <= C; r0 += U) {
        double zz[U];
#pragma unroll
        for (int u = 0; u < U; ++u) zz[u] = zb[(r0 + u) * 64 + i];
#pragma unroll
        for (int u = 0; u < U; ++u) zb[(r0 + u) * 64 + i] = zz[u] * sc;
      }
      for (; r0 < C; ++r0) zb[r0 * 64 + i] *= sc;
    }
    if (tid == 0) atomicAdd(&g_gram_ticks[7], __builtin_amdgcn_s_memtime() - t_last);  // S5 A: inverse iteration
  }
  else if ((wave & 3) != 0 && wave - 1 - (wave >> 2) < ((C - 1 + 15) >> 4)) {  // (uniform per wave)
    s6_factors(wave - 1 - (wave >> 2), C, hh, s_tau, lane);
  }
  __syncthreads();
  if (wave == 0) gs_clusters<64>(K, C, zb, s_lam, s_tn, lane);  // (uniform loop over wave 0)
  __syncthreads();
  if (tid < K) s_sig2[tid] = rayleigh<64>(tid, C, zb, s_d, s_e);
  __syncthreads();
  tick(3);
  // ---- S6: V = Q Z on the matrix cores, 16 reflectors at a time in compact WY form (LAPACK
  // zlarft / zlarfb, forward, columnwise): H_k0 ... H_k0+15 = I - Y T Y^H, V <- V - Y (T (Y^H V)),
  // blocks from the last reflectors down.  V (C x 64) is 8 x 4 tiles of 16 x 16 in the MFMA
  // accumulator layout: wave w holds column tile w & 3 and row tiles 2 (w >> 2), 2 (w >> 2) + 1
  // (lane l: column l & 15, rows (l >> 4) + 4 q) -- which is also the B-operand layout of Y^H V, so
  // V never leaves the registers.  Per block: Y^H V as four partial products per column tile
  // (three of them through the LDS), T from S5's precompute, W2 = T (Y^H V) on the matrix cores in
  // the summing waves, V -= Y W2; four barriers. ----
  const int nt = wave & 3, mg = wave >> 2, li = lane & 15, lk = lane >> 4;
  aqc::d4_t vre[2], vim[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 32 * mg + 16 * t + lk + 4 * q, col = 16 * nt + li;
      vre[t][q] = (row < C && col < K) ? zb[row * 64 + col] : 0.0;
      vim[t][q] = 0.0;
    }
  }
  s6_back(j, hh, C, K, 0, vre, vim, s_sig2, tid, lane, wave, wave_s);
  tick(4);
  }  // (K <= 64)
  for (int c = tid; c < C; c += 1024) aqc::stg(j.sig + c, c < K ? sqrt(s_sig2[c]) : 0.0);
  if (tid == 0) aqc::stg(j.sig + kSigTail, s_tail);  // the tail gram_keep dropped (rank_body)
  tick(5);
  if (s_cert) return 2;  // (uniform) the caller runs gram_certified
  if (tid == 0) {
    atomicMax(&j.flags[2], 1);
    atomicAdd(&g_gram_stats[1], 1ull);
  }
  return 1;
}

// After gram_svd_body returned 2 (its kept count assumed the values in CHOP's error band chopped):
// the certificate on its output (W, sig); true if it holds (the update stands), false if not (the
// caller runs the register Jacobi, which rewrites W and sig).  A separate call so that neither its
// accumulators nor the call itself enter the body's register allocation.
__device__ __noinline__ bool gram_certified(const TwoSiteJob& j) {
  const int tid = fresh_tid();
  __shared__ double s_s2[128];
  __shared__ int s_k;
  const int M = 2 * j.dims[0], N = 2 * j.dims[2], C = M < N ? M : N;
  if (tid == 0) s_k = 0;
  __syncthreads();
  if (tid < C) {
    const double sg = aqc::ldg(j.sig + tid);
    s_s2[tid] = sg * sg;
    if (sg > 0.0) atomicMax(&s_k, tid + 1);
  }
  __syncthreads();
  if (tid == 0) atomicAdd(&g_gram_stats[4], 1ull);
  const double cs = gram_cert128(j, C, s_k, s_s2);
  const bool ok = cs < 0.5 * aqc::kReduceChop;
  if (tid == 0) {
    atomicAdd(&g_gram_stats[ok ? 5 : 3], 1ull);
    if (ok) {
      atomicMax(&j.flags[2], 1);
      atomicAdd(&g_gram_stats[1], 1ull);
    } else {
      aqc::stg(j.sig + kSigTail, 0.0);  // (the body's tail belongs to its kept count, not the Jacobi's)
    }
  }
  __syncthreads();
  return ok;
}

__global__ __launch_bounds__(1024) void k_svd_gram(const TwoSiteJob* __restrict__ jobs) {
  const TwoSiteJob& j = jobs[blockIdx.x];
  const int g = j.gram ? gram_svd_body(j) : 0;
  if (g == 1) return;
  __syncthreads();
  if (g == 2 && gram_certified(j)) return;
  jacobi_reg_body<128, 8, 16>(j);
}
