// Multi-workgroup Gram-path SVD for the large two-site updates (2 chi = C in 256 / 512 / 1024:
// chi = 128, the 100-qubit chi = 256 MPS preparation of BASELINE config 5, and chi up to 512).
//
// The block one-sided Jacobi (bjacobi.hip) spends ~2.5 C^3 complex MACs per sweep and needs 15-18
// sweeps at C = 512: five times the LAPACK-nominal flops.  The Gram path needs one G = X^H X, one
// Householder tridiagonalisation (4/3 C^3 MACs), the top-K eigenpairs of the tridiagonal and one
// back-transformation -- but a C x C Hermitian matrix above C = 128 no longer fits one CU (the
// 2 chi = 128 kernel holds G in the VGPRs of one 1024-thread workgroup, svd_gram.h).  Here:
//
//   k_gb_gram     G = X^H X (X = theta' or theta'^H so that L >= C) on the FP64 matrix cores, one
//                 64 x 64 block per 256-thread workgroup, into a per-job C x C scratch.
//   k_gb_tridiag  LAPACK zhetd2 (lower) over P = C^2 / 16384 workgroups per job: workgroup g holds
//                 the rows r = g (mod P) of G in its VGPRs (16 complex per thread), cyclic so the
//                 shrinking trailing block stays balanced.  Per column k every workgroup forms the
//                 reflector v_k itself from row k (zlarfg; conj(row k) = column k), computes
//                 p_r = tau (G v)_r for its rows, and publishes p_r -- and, on the owner of row
//                 k + 1, that row as it is BEFORE this step's update -- in one exchange: sc1 stores,
//                 s_waitcnt vmcnt(0), a workgroup barrier, one agent-scope counter add; the
//                 consumers poll the counter with sc1 loads and read the payload with sc1 loads (the
//                 hand-off form of the MI355X guide's "Valid forms" table, row 1).  From p every
//                 workgroup forms w = p - tau/2 (p^H v) v and, from the old row k + 1, the new row
//                 k + 1 = old - conj(w) - w_{k+1} conj(v): the next column needs no second hand-off.
//                 One exchange per column; spins bounded (100 ms, then the job declines).
//   k_gb_eig      one workgroup per job: the top K eigenvalues of T by multisection with the
//                 polynomial Sturm count, inverse iteration (LDL^T of T - lambda I, three solves,
//                 vectors in a per-job scratch), Gram-Schmidt inside clusters, sigma^2 = z^T T z.
//                 Declines (status 1) unless lambda_K > 1e-9 lambda_1, as the 2 chi = 128 path does.
//   k_gb_back     V = Q Z, one wave per eigenvector: the reflectors, last first, staged through the
//                 LDS eight at a time; output W = V Sigma, sig, qr = 1 -- the contract of the
//                 2 chi = 128 Gram path (work column c = right singular vector c of X times
//                 sigma_c), so k_rank / k_split_* run unchanged.
// Jobs that decline (floor, timeout, gram disabled) run the block Jacobi afterwards (the host reads
// the statuses once, after k_gb_eig).
#include <cstdlib>
#include <cstring>

#include "aqc_gemm.h"
#include "mps_internal.h"

namespace aqc {

// calls, taken, declined (gram off / shape), declined at the eigenvalue floor, exchange timeouts
__device__ unsigned long long g_gbig_stats[5];
// shader-clock ticks of job 0's first workgroup (thread 0), summed over calls: tridiagonalisation
// phases [0] pass + row sums, [1] publish (stores, vmcnt, barrier), [2] counter wait, [3] reads + p^H v,
// [4] w, new row, next reflector; [5] k_gb_eig, [6] k_gb_back (job 0, block 0)
__device__ unsigned long long g_gbig_ticks[8];

namespace {

constexpr double kGbRelFloor = 1e-9;
constexpr unsigned long long kSpinTicks = 10000000ull;  // s_memrealtime (100 MHz): 100 ms

typedef __attribute__((address_space(1))) double gdbl;
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) int gi32;

// sc1 stores / loads (bypass the CU's L1; the hand-off form that needs no agent fences)
__device__ __forceinline__ void st_sc1(cplx* p, cplx v) {
  gdbl* q = (gdbl*)(double*)p;
  __hip_atomic_store(q, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ cplx ld_sc1(const cplx* p) {
  gdbl* q = (gdbl*)(double*)p;
  return cmk(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

struct GBArgs {
  cplx* G;         // per job CT x CT: G, then the reflectors (row k = v_k at columns > k)
  double* d;       // per job CT
  double* e;       // per job CT
  cplx* tau;       // per job CT
  double* z;       // per job CT x CT: eigenvector i at z[row * CT + i]
  double* dinv;    // per job CT x CT: inverse-iteration pivots
  double* sig2;    // per job CT
  double* lam;     // per job CT: the top K eigenvalues of T, descending
  double* tn;      // per job: ||T|| (Gershgorin)
  cplx* xch;       // per job 4 x CT: p (two buffers), old row k + 1 (two buffers)
  unsigned* cnt;   // per job 32 words (128 B)
  int* status;     // per job: 0 ok, 1 declined (gram off / shape), 2 floor, 3 exchange timeout
};

__device__ __forceinline__ double wave_sum_b(double v) {
  v = row_sum16(v);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

template <int TPR>
__device__ __forceinline__ double group_reduce(double v) {
  v = row_sum16(v);
  if constexpr (TPR >= 32) v += __shfl_xor(v, 16);
  if constexpr (TPR >= 64) v += __shfl_xor(v, 32);
  return v;
}

__device__ __forceinline__ void job_dims(const TwoSiteJob& j, int& M, int& L, int& C, bool& tr, int& K) {
  M = 2 * j.dims[0];
  const int N = 2 * j.dims[2];
  tr = M < N;
  L = tr ? N : M;
  C = tr ? M : N;
  K = C;
  if (j.max_chi > 0 && j.max_chi < K) K = j.max_chi;
}

// ---- G = X^H X ------------------------------------------------------------------------------
// grid ((CT / 64)^2, nj), 256 threads.  Entries outside C x C are zero.
template <int CT>
__global__ __launch_bounds__(256) void k_gb_gram(const TwoSiteJob* __restrict__ jobs, GBArgs a) {
  const int jb = blockIdx.y;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    atomicAdd(&g_gbig_stats[0], 1ull);
    const int st = (!j.gram || C < 4) ? 1 : 0;
    *(gi32*)(a.status + jb) = st;
    if (st) atomicAdd(&g_gbig_stats[2], 1ull);
  }
  if (!j.gram || C < 4) return;
  constexpr int nbt = CT / 64;
  const int bi = (blockIdx.x / nbt) * 64, bj = (blockIdx.x % nbt) * 64;
  cplx* G = a.G + (size_t)jb * CT * CT;
  const cplx* th = j.theta;
  __shared__ GemmLds lds;
  const int m = bi < C ? min(64, C - bi) : 0, n = bj < C ? min(64, C - bj) : 0;
  auto store = [&](int i, int jj, cplx v) { stg(G + (size_t)(bi + i) * CT + bj + jj, v); };
  if (m > 0 && n > 0) {
    if (!tr) {  // X[R][c] = theta[c * M + R]: contiguous along the contraction
      block_cgemm<true, true>(
          m, n, L, [&](int i, int k) { return cconj(ldg(th + (size_t)(bi + i) * M + k)); },
          [&](int k, int jj) { return ldg(th + (size_t)(bj + jj) * M + k); }, store, lds);
    } else {  // X = theta^H: X[R][c] = conj(theta[R * M + c])
      block_cgemm<false, false>(
          m, n, L, [&](int i, int k) { return ldg(th + (size_t)k * M + bi + i); },
          [&](int k, int jj) { return cconj(ldg(th + (size_t)k * M + bj + jj)); }, store, lds);
    }
  }
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int i = e >> 6, jj = e & 63;
    if (i >= m || jj >= n) stg(G + (size_t)(bi + i) * CT + bj + jj, cmk(0, 0));
  }
}

// zlarfg on (alpha, x) with ||x||^2 = xn2: beta (real), tau, scale = 1 / (alpha - beta)
__device__ __forceinline__ void zlarfg_s(cplx alpha, double xn2, cplx& tau, double& beta, cplx& scale) {
  if (xn2 == 0.0 && alpha.y == 0.0) {
    tau = cmk(0, 0);
    beta = alpha.x;
    scale = cmk(0, 0);
    return;
  }
  const double nrm = sqrt(alpha.x * alpha.x + alpha.y * alpha.y + xn2);
  beta = alpha.x >= 0.0 ? -nrm : nrm;
  tau = cmk((beta - alpha.x) / beta, -alpha.y / beta);
  const cplx den = cmk(alpha.x - beta, alpha.y);
  const double id = 1.0 / cnorm2(den);
  scale = cmk(den.x * id, -den.y * id);
}

// ---- tridiagonalisation over P workgroups per job -----------------------------------------------
// grid (P * njobs_in_round), 1024 threads.  Thread t: local row t / TPR (global r = lr P + g),
// columns q + TPR i (q = t % TPR, i < 16).  Per column k: one pass over the registers applies the
// deferred rank-2 update of reflector k - 1 and forms (G v_k)_r; the exchange; p^H v; w_k and the new
// row k + 1; reflector k + 1's zlarfg.  Five workgroup barriers per column.
template <int CT>
__global__ __launch_bounds__(1024) void k_gb_tridiag(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  constexpr int R = 16384 / CT, TPR = CT / 16, P = CT / R;
  const int jb = job0 + (int)blockIdx.x / P, g = (int)blockIdx.x % P;
  if (*(const gi32*)(a.status + jb) != 0) return;  // uniform over the job's workgroups
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = tid / TPR, q = tid % TPR, r = lr * P + g;
  const bool tick = jb == 0 && g == 0 && tid == 0;
  cplx* G = a.G + (size_t)jb * CT * CT;
  cplx* xch = a.xch + (size_t)jb * 4 * CT;
  unsigned* cnt = a.cnt + (size_t)jb * 32;
  double* dd = a.d + (size_t)jb * CT;
  double* ee = a.e + (size_t)jb * CT;
  cplx* tt = a.tau + (size_t)jb * CT;
  __shared__ cplx vL[2][CT], wL[CT], rhoL[CT];
  __shared__ double redd[16];
  __shared__ cplx redc[16];
  __shared__ int s_abort;
  unsigned long long tk[5] = {0, 0, 0, 0, 0}, tl = tick ? __builtin_amdgcn_s_memtime() : 0;
  auto tmark = [&](int ph) {
    if (tick) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      tk[ph] += t - tl;
      tl = t;
    }
  };
  cplx A[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) A[i] = ldg(G + (size_t)r * CT + q + TPR * i);
  cplx vt = cmk(0, 0), tau = cmk(0, 0);
  if (tid < CT) {
    rhoL[tid] = ldg(G + tid);  // row 0
    wL[tid] = cmk(0, 0);       // no deferred update before column 0
    vL[1][tid] = cmk(0, 0);
  }
  if (tid == 0) s_abort = 0;
  __syncthreads();
  // reflector 0 from row 0
  auto reflector = [&](int k, cplx xt) {  // after rhoL holds row k and redd the partial norms
    double xn2 = 0.0;
#pragma unroll
    for (int w = 0; w < 16; ++w) xn2 += redd[w];
    cplx sc;
    double beta;
    zlarfg_s(cconj(rhoL[k + 1]), xn2, tau, beta, sc);
    vt = tid == k + 1 ? cmk(1, 0) : (tid > k + 1 && tid < CT ? cmul(xt, sc) : cmk(0, 0));
    if (tid < CT) vL[k & 1][tid] = vt;
    if (g == 0 && tid == 0) {
      stg(dd + k, rhoL[k].x);
      stg(ee + k, beta);
      stg(tt + k, tau);
    }
  };
  {
    const cplx xt = tid < CT ? cconj(rhoL[tid]) : cmk(0, 0);
    const double part = wave_sum_b((tid >= 2 && tid < CT) ? cnorm2(xt) : 0.0);
    if (lane == 0) redd[wave] = part;
    __syncthreads();
    reflector(0, xt);
    __syncthreads();
  }
  for (int k = 0; k < CT - 1; ++k) {
    const int cur = k & 1, prv = cur ^ 1;
    // ---- the deferred update G -= v w^H + w v^H of reflector k - 1, then s = (G v_k)_r
    cplx s = cmk(0, 0);
    {
      const cplx vr = vL[prv][r], wr = wL[r];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = q + TPR * i;
        A[i] = csub(A[i], cadd(cmulc(vr, wL[c]), cmulc(wr, vL[prv][c])));
        s = cfma(A[i], vL[cur][c], s);
      }
    }
    s.x = group_reduce<TPR>(s.x);
    s.y = group_reduce<TPR>(s.y);
    const cplx pr = r > k ? cmul(tau, s) : cmk(0, 0);
    tmark(0);
    cplx* xp = xch + cur * CT;
    cplx* xr = xch + (2 + cur) * CT;
    if (q == 0) st_sc1(xp + r, pr);
    if (r == k + 1) {  // the row's owner: row k + 1 before this step's update
#pragma unroll
      for (int i = 0; i < 16; ++i) st_sc1(xr + q + TPR * i, A[i]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    tmark(1);
    if (tid == 0) {
      __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)P * (unsigned)(k + 1);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
          s_abort = 1;
          break;
        }
      }
    }
    __syncthreads();
    if (s_abort) {
      if (tid == 0 && g == 0) {
        *(gi32*)(a.status + jb) = 3;
        atomicAdd(&g_gbig_stats[4], 1ull);
      }
      return;
    }
    tmark(2);
    // ---- w = p - tau / 2 (p^H v) v, the new row k + 1, reflector k to row k of the scratch
    const cplx pt = tid < CT ? ld_sc1(xp + tid) : cmk(0, 0);
    const cplx ro = tid < CT ? ld_sc1(xr + tid) : cmk(0, 0);
    const cplx pk1 = ld_sc1(xp + k + 1);
    const cplx pvp = cconjmul(pt, vt);
    const double px = wave_sum_b(pvp.x), py = wave_sum_b(pvp.y);
    if (lane == 0) redc[wave] = cmk(px, py);
    __syncthreads();
    tmark(3);
    cplx pv = cmk(0, 0);
#pragma unroll
    for (int w = 0; w < 16; ++w) pv = cadd(pv, redc[w]);
    const cplx a2 = cscale(cmul(tau, pv), -0.5);
    const cplx wt = cfma(a2, vt, pt);
    const cplx wk1 = cadd(pk1, a2);
    const cplx rho = csub(csub(ro, cconj(wt)), cmulc(wk1, vt));
    if (tid < CT) {
      wL[tid] = wt;  // (w_{k-1} was last read in this step's pass, before the exchange's barrier)
      rhoL[tid] = rho;
      if (g == 0 && tid > k) stg(G + (size_t)k * CT + tid, vt);
    }
    if (k == CT - 2) {
      if (g == 0 && tid == CT - 1) stg(dd + CT - 1, rho.x);
      break;
    }
    // ---- reflector k + 1 from the new row k + 1 (v_{k-1}'s buffer is free: read in the pass)
    const cplx xt = tid < CT ? cconj(rho) : cmk(0, 0);
    const double part = wave_sum_b((tid >= k + 3 && tid < CT) ? cnorm2(xt) : 0.0);
    if (lane == 0) redd[wave] = part;
    __syncthreads();
    reflector(k + 1, xt);
    __syncthreads();
    tmark(4);
  }
  if (tick) {
#pragma unroll
    for (int i = 0; i < 5; ++i) atomicAdd(&g_gbig_ticks[i], tk[i]);
  }
}

// Sturm count of T (rows de[i] = (d_i, e_{i-1}^2) scaled by 1 / ||T||) below xn: the leading
// minors' three-term recurrence, rescaled every four rows (as svd_gram.h's sturm_count_poly).
__device__ __forceinline__ int sturm_poly(const double2* de, int C, double xn) {
  double p0 = 1.0, p1 = de[0].x - xn;
  int s1 = __double2hiint(p1) >> 31;
  int neg = s1;
  int i = 1;
  for (; i + 4 <= C; i += 4) {
    double2 r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) r[u] = de[i + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double p2 = fma(r[u].x - xn, p1, -(r[u].y * p0));
      const int s2 = __double2hiint(p2) >> 31;
      neg += s1 ^ s2;
      s1 = s2;
      p0 = p1;
      p1 = p2;
    }
    const int ex = max(__builtin_amdgcn_frexp_exp(p0), __builtin_amdgcn_frexp_exp(p1));
    p0 = __builtin_amdgcn_ldexp(p0, -ex);
    p1 = __builtin_amdgcn_ldexp(p1, -ex);
  }
  for (; i < C; ++i) {
    const double p2 = fma(de[i].x - xn, p1, -(de[i].y * p0));
    const int s2 = __double2hiint(p2) >> 31;
    neg += s1 ^ s2;
    s1 = s2;
    p0 = p1;
    p1 = p2;
  }
  return -neg;
}

__device__ __forceinline__ double rcp_nr2(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = r * fma(-x, r, 2.0);
  r = r * fma(-x, r, 2.0);
  return r;
}

// ---- eigenpairs of T: grid (nj), 1024 threads ----
template <int CT>
__global__ __launch_bounds__(1024) void k_gb_eig(const TwoSiteJob* __restrict__ jobs, GBArgs a) {
  const int jb = blockIdx.x;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  __shared__ double s_d[CT], s_e[CT], s_e2[CT], s_lam[CT];
  __shared__ double2 s_de[CT];
  __shared__ int cntb[256];
  __shared__ double s_lo, s_hi, s_tn;
  __shared__ double rlo[16], rhi[16], rtn[16];
  const double* dd = a.d + (size_t)jb * CT;
  const double* ee = a.e + (size_t)jb * CT;
  for (int i = tid; i < CT; i += 1024) {
    s_d[i] = ldg(dd + i);
    s_e[i] = i < CT - 1 ? ldg(ee + i) : 0.0;
  }
  __syncthreads();
  {
    double lo = 1e300, hi = -1e300, tn = 0.0;
    for (int i = tid; i < CT; i += 1024) {
      const double el = i > 0 ? fabs(s_e[i - 1]) : 0.0, er = fabs(s_e[i]);
      const double di = s_d[i];
      lo = fmin(lo, di - el - er);
      hi = fmax(hi, di + el + er);
      tn = fmax(tn, fabs(di) + el + er);
      s_e2[i] = s_e[i] * s_e[i];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      lo = fmin(lo, __shfl_xor(lo, off));
      hi = fmax(hi, __shfl_xor(hi, off));
      tn = fmax(tn, __shfl_xor(tn, off));
    }
    if (lane == 0) rlo[wave] = lo, rhi[wave] = hi, rtn[wave] = tn;
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < 16; ++w) lo = fmin(lo, rlo[w]), hi = fmax(hi, rhi[w]), tn = fmax(tn, rtn[w]);
      lo = fmin(lo, rlo[0]), hi = fmax(hi, rhi[0]), tn = fmax(tn, rtn[0]);
      const double span = fmax(hi - lo, 1e-300);
      s_lo = lo - 1e-12 * span;
      s_hi = hi + 1e-12 * span;
      s_tn = tn;
    }
    __syncthreads();
    const double itn = 1.0 / fmax(s_tn, 1e-300);
    for (int i = tid; i < CT; i += 1024)
      s_de[i] = make_double2(s_d[i] * itn, i > 0 ? s_e2[i - 1] * itn * itn : 0.0);
  }
  __syncthreads();
  // multisection: one 256-shift pass, then 12 rounds of 5-section with 4 lanes per eigenvalue
  {
    constexpr int kG = 4, kFirst = 256, kRounds = 12;
    const double lo0 = s_lo, span0 = s_hi - s_lo;
    const double itn = 1.0 / fmax(s_tn, 1e-300);
    constexpr double kInvF = 1.0 / (kFirst + 1), kInvG = 1.0 / (kG + 1);
    if (tid < kFirst) cntb[tid] = sturm_poly(s_de, CT, (lo0 + span0 * (double)(tid + 1) * kInvF) * itn);
    __syncthreads();
    const int sub = tid % kG;
    for (int b0 = 0; b0 < K; b0 += 1024 / kG) {
      const int eid = b0 + tid / kG;
      const int a_ = CT - 1 - min(eid, CT - 1);  // ascending index of the eid-th largest
      double lo, hi;
      {
        int l = 0, h = kFirst;
        while (l < h) {
          const int m = (l + h) >> 1;
          if (cntb[m] >= a_ + 1) h = m;
          else l = m + 1;
        }
        lo = l > 0 ? lo0 + span0 * (double)l * kInvF : s_lo;
        hi = l < kFirst ? lo0 + span0 * (double)(l + 1) * kInvF : s_hi;
      }
      for (int round = 0; round < kRounds; ++round) {
        const double x = lo + (hi - lo) * (double)(sub + 1) * kInvG;
        const int cnt = sturm_poly(s_de, CT, x * itn);
        const unsigned long long bal = __ballot(cnt >= a_ + 1);
        const unsigned int gm = (unsigned int)(bal >> (lane & ~(kG - 1))) & ((1u << kG) - 1u);
        const int f = gm ? __builtin_ctz(gm) : kG;
        const double nhi = f < kG ? lo + (hi - lo) * (double)(f + 1) * kInvG : hi;
        const double nlo = f > 0 ? lo + (hi - lo) * (double)f * kInvG : lo;
        lo = nlo;
        hi = nhi;
      }
      if (eid < K && sub == 0) s_lam[eid] = 0.5 * (lo + hi);
    }
  }
  __syncthreads();
  if (!(s_lam[0] > 0.0) || !(s_lam[K - 1] > kGbRelFloor * s_lam[0])) {  // uniform
    if (tid == 0) {
      *(gi32*)(a.status + jb) = 2;
      atomicAdd(&g_gbig_stats[3], 1ull);
    }
    return;
  }
  for (int i = tid; i < K; i += 1024) stg(a.lam + (size_t)jb * CT + i, s_lam[i]);
  if (tid == 0) stg(a.tn + jb, s_tn);
  if (jb == 0 && tid == 0) atomicAdd(&g_gbig_ticks[5], __builtin_amdgcn_s_memtime() - t_start);
}

typedef unsigned __attribute__((ext_vector_type(2))) u2_t;
__device__ __forceinline__ double bld(__amdgpu_buffer_rsrc_t r, unsigned lo, unsigned uo) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, lo, uo, 0));
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned lo, unsigned uo, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2_t, v), r, lo, uo, 0);
}

// ---- inverse iteration: grid (ceil(K / 64), nj), one wave, one lane per eigenvector ----
// L D L^T = T - lambda I without pivoting (pivots from the leading minors' recurrence, units of
// ||T||, guarded at eps), three solves from a deterministic start vector, sigma^2 = z^T T z.  The
// vectors and pivots live in the per-job scratch (row-major, lanes along a row: one 512-byte
// access per wave and row), addressed through a buffer resource (one lane offset, the row as the
// uniform offset); the solves' recurrences are serial per lane, so each row's operands are read
// U rows ahead of the chain.
template <int CT>
__global__ __launch_bounds__(64) void k_gb_inv(const TwoSiteJob* __restrict__ jobs, GBArgs a) {
  const int jb = blockIdx.y;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  if ((int)blockIdx.x * 64 >= K) return;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  __shared__ double s_d[CT], s_e[CT];
  for (int r = threadIdx.x; r < CT; r += 64) {
    s_d[r] = ldg(a.d + (size_t)jb * CT + r);
    s_e[r] = r < CT - 1 ? ldg(a.e + (size_t)jb * CT + r) : 0.0;
  }
  __syncthreads();
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= K) return;  // (no barrier below)
  const double tn = ldg(a.tn + jb), itn = 1.0 / fmax(tn, 1e-300);
  const double lamn = ldg(a.lam + (size_t)jb * CT + i) * itn;
  const __amdgpu_buffer_rsrc_t rz = make_rsrc(a.z + (size_t)jb * CT * CT, (unsigned)(CT * CT * 8));
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dinv + (size_t)jb * CT * CT, (unsigned)(CT * CT * 8));
  const unsigned lo = (unsigned)i * 8u;
  constexpr unsigned RS = CT * 8;  // row stride in bytes
  constexpr int U = 16;
  for (int row = 0; row < CT; ++row) {  // deterministic start vector in [-1, 1)
    unsigned int h = (unsigned int)(row * 2654435761u) ^ (unsigned int)((i + 1) * 40503u);
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    bst(rz, lo, row * RS, (double)(h & 0xFFFFFu) * (2.0 / 1048576.0) - 1.0);
  }
  {  // the pivots 1 / D_row
    double p0 = 0.0, p1 = 1.0;
    for (int row = 0; row < CT; ++row) {
      const double e2 = row > 0 ? s_e[row - 1] * s_e[row - 1] : 0.0;
      const double dmx = fma(s_d[row], itn, -lamn), t = (e2 * itn * itn) * p0;
      const double lim = 2.220446049250313e-16 * fabs(p1);
      double p = fma(dmx, p1, -t);
      p = fabs(p) < lim ? copysign(lim, p) : p;
      bst(rd, lo, row * RS, p1 * rcp_nr2(p) * itn);
      p0 = p1;
      p1 = p;
      if ((row & 7) == 7) {
        const int ex = max(__builtin_amdgcn_frexp_exp(p0), __builtin_amdgcn_frexp_exp(p1));
        p0 = __builtin_amdgcn_ldexp(p0, -ex);
        p1 = __builtin_amdgcn_ldexp(p1, -ex);
      }
    }
  }
  double sc = 1.0;
  for (int it = 0; it < 3; ++it) {
    double yp = 0.0;
    {  // L y = sc z (rows ascending); row r needs z_r and 1 / D_{r-1}
      double zz[U], dp[U], nz[U], nd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) zz[u] = bld(rz, lo, u * RS), dp[u] = bld(rd, lo, max(u - 1, 0) * RS);
      for (int r0 = 0; r0 < CT; r0 += U) {
        const int n0 = min(r0 + U, CT - U);  // (the last block re-reads itself: no branch)
#pragma unroll
        for (int u = 0; u < U; ++u) nz[u] = bld(rz, lo, (n0 + u) * RS), nd[u] = bld(rd, lo, (n0 + u - 1) * RS);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = r0 + u;
          const double e = row > 0 ? s_e[row - 1] : 0.0;
          const double y = fma(-e * dp[u], yp, zz[u] * sc);
          bst(rz, lo, row * RS, y);
          yp = y;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) zz[u] = nz[u], dp[u] = nd[u];
      }
    }
    double zn = 0.0, n2 = 0.0;
    {  // z = D^-1 y - L^T z (rows descending); row r needs y_r and 1 / D_r
      double yy[U], dv[U], ny[U], nd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) yy[u] = bld(rz, lo, (CT - 1 - u) * RS), dv[u] = bld(rd, lo, (CT - 1 - u) * RS);
      for (int r1 = CT - 1; r1 >= 0; r1 -= U) {
        const int n1 = max(r1 - U, U - 1);
#pragma unroll
        for (int u = 0; u < U; ++u) ny[u] = bld(rz, lo, (n1 - u) * RS), nd[u] = bld(rd, lo, (n1 - u) * RS);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = r1 - u;
          const double e = s_e[row];  // (0 past the last row)
          zn = fma(-e * dv[u], zn, yy[u] * dv[u]);
          bst(rz, lo, row * RS, zn);
          n2 = fma(zn, zn, n2);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) yy[u] = ny[u], dv[u] = nd[u];
      }
    }
    const double rs = __builtin_amdgcn_rsq(n2);
    sc = rs * fma(-0.5 * n2 * rs, rs, 1.5);
  }
  // normalise, and sigma^2 = z^T T z on the normalised rows
  double s2a = 0.0, s2b = 0.0, zprev = 0.0;
  for (int r0 = 0; r0 < CT; r0 += U) {
    double zz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) zz[u] = bld(rz, lo, (r0 + u) * RS) * sc;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = r0 + u;
      bst(rz, lo, row * RS, zz[u]);
      s2a = fma(s_d[row] * zz[u], zz[u], s2a);
      if (row > 0) s2b = fma(2.0 * s_e[row - 1] * zprev, zz[u], s2b);
      zprev = zz[u];
    }
  }
  const double s2 = s2a + s2b;
  stg(a.sig2 + (size_t)jb * CT + i, s2 > 0.0 ? s2 : 0.0);
  if (jb == 0 && i == 0) atomicAdd(&g_gbig_ticks[7], __builtin_amdgcn_s_memtime() - t_start);
}

// ---- Gram-Schmidt inside clusters (eigenvalue gaps below 1e-7 ||T||; the vectors of separated
// eigenvalues come out orthogonal to ~1e-14 from three inverse-iteration steps), then the cluster
// members' sigma^2 again: grid (nj), one wave ----
template <int CT>
__global__ __launch_bounds__(64) void k_gb_gs(const TwoSiteJob* __restrict__ jobs, GBArgs a) {
  const int jb = blockIdx.x;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  const int lane = threadIdx.x;
  const double* lam = a.lam + (size_t)jb * CT;
  const double ortol = 1e-7 * ldg(a.tn + jb);
  double* zb = a.z + (size_t)jb * CT * CT;
  const double* dd = a.d + (size_t)jb * CT;
  const double* ee = a.e + (size_t)jb * CT;
  int start = 0;
  for (int i = 1; i < K; ++i) {
    if (ldg(lam + i - 1) - ldg(lam + i) >= ortol) {
      start = i;
      continue;
    }
    for (int jj = start; jj < i; ++jj) {
      double dp = 0.0;
      for (int row = lane; row < CT; row += 64) dp = fma(zb[(size_t)row * CT + i], zb[(size_t)row * CT + jj], dp);
      dp = wave_sum_b(dp);
      for (int row = lane; row < CT; row += 64)
        zb[(size_t)row * CT + i] = fma(-dp, zb[(size_t)row * CT + jj], zb[(size_t)row * CT + i]);
    }
    double n2 = 0.0;
    for (int row = lane; row < CT; row += 64) n2 = fma(zb[(size_t)row * CT + i], zb[(size_t)row * CT + i], n2);
    n2 = wave_sum_b(n2);
    const double sc = 1.0 / sqrt(n2);
    double s2 = 0.0;
    for (int row = lane; row < CT; row += 64) {
      const double z = zb[(size_t)row * CT + i] * sc;
      zb[(size_t)row * CT + i] = z;
      s2 = fma(ldg(dd + row) * z, z, s2);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    for (int row = lane; row < CT - 1; row += 64)
      s2 = fma(2.0 * ldg(ee + row) * zb[(size_t)row * CT + i], zb[(size_t)(row + 1) * CT + i], s2);
    s2 = wave_sum_b(s2);
    if (lane == 0) stg(a.sig2 + (size_t)jb * CT + i, s2 > 0.0 ? s2 : 0.0);
  }
}

// ---- V = Q Z, output: grid (CT / 16, nj), 1024 threads (one wave per eigenvector); dynamic LDS
// kRB x CT complex (the staged reflectors) ----
constexpr int kRB = 8;

template <int CT>
__global__ __launch_bounds__(1024) void k_gb_back(const TwoSiteJob* __restrict__ jobs, GBArgs a) {
  constexpr int MR = CT / 64;  // rows per lane
  const int jb = blockIdx.y;
  if (*(const gi32*)(a.status + jb) != 0) return;
  TwoSiteJob& j = const_cast<TwoSiteJob&>(jobs[jb]);
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  extern __shared__ cplx Yl[];  // [kRB][CT]
  __shared__ cplx s_tau[kRB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int col = blockIdx.x * 16 + wave;
  const bool act = col < K;
  const double* zb = a.z + (size_t)jb * CT * CT;
  const cplx* Y = a.G + (size_t)jb * CT * CT;
  const cplx* tau = a.tau + (size_t)jb * CT;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  cplx V[MR];
#pragma unroll
  for (int m = 0; m < MR; ++m) V[m] = cmk(act ? ldg(zb + (size_t)(lane + 64 * m) * CT + col) : 0.0, 0.0);
  // the next group's reflectors are loaded into registers while the current group is applied
  constexpr int PE = kRB * CT / 1024;
  cplx ny[PE], ntau = cmk(0, 0);
  auto fetch = [&](int k1) {
    const int k0 = max(k1 - kRB + 1, 0), nb = k1 - k0 + 1;
#pragma unroll
    for (int u = 0; u < PE; ++u) {
      const int e = tid + 1024 * u, b = e / CT, row = e % CT, k = k0 + b;
      ny[u] = (b < nb && row > k) ? ldg(Y + (size_t)k * CT + row) : cmk(0, 0);
    }
    if (tid < kRB) ntau = tid < nb ? ldg(tau + k0 + tid) : cmk(0, 0);
  };
  fetch(CT - 2);
  for (int k1 = CT - 2; k1 >= 0; k1 -= kRB) {  // reflectors k1, k1 - 1, ..., k0 (last first)
    const int k0 = max(k1 - kRB + 1, 0), nb = k1 - k0 + 1;
    __syncthreads();  // the previous group's reflectors are consumed
#pragma unroll
    for (int u = 0; u < PE; ++u) Yl[tid + 1024 * u] = ny[u];
    if (tid < kRB) s_tau[tid] = ntau;
    __syncthreads();
    if (k1 - kRB >= 0) fetch(k1 - kRB);
    if (act) {
      for (int b = nb - 1; b >= 0; --b) {
        const int k = k0 + b;
        const cplx* yv = Yl + b * CT;
        cplx dot = cmk(0, 0);
#pragma unroll
        for (int m = 0; m < MR; ++m)
          if (64 * m + 63 > k) dot = cfmac(yv[lane + 64 * m], V[m], dot);  // y^H V
        dot.x = wave_sum_b(dot.x);
        dot.y = wave_sum_b(dot.y);
        const cplx f = cmul(s_tau[b], dot);
#pragma unroll
        for (int m = 0; m < MR; ++m)
          if (64 * m + 63 > k) V[m] = csub(V[m], cmul(yv[lane + 64 * m], f));
      }
    }
  }
  if (act) {
    const double sg = sqrt(ldg(a.sig2 + (size_t)jb * CT + col));
#pragma unroll
    for (int m = 0; m < MR; ++m) {
      const int row = lane + 64 * m;
      if (row < C) stg(j.work + (size_t)col * C + row, cscale(V[m], sg));
    }
    if (lane == 0) stg(j.sig + col, sg);
  }
  for (int c = blockIdx.x * 16 + tid; c < min(C, blockIdx.x * 16 + 16); c += 1024)
    if (c >= K) stg(j.sig + c, 0.0);
  if (jb == 0 && blockIdx.x == 0 && tid == 0) atomicAdd(&g_gbig_ticks[6], __builtin_amdgcn_s_memtime() - t_start);
  if (blockIdx.x == 0 && tid == 0) {
    j.qr = 1;
    atomicMax(&j.flags[2], 1);
    atomicAdd(&g_gbig_stats[1], 1ull);
  }
}

struct GBBuffers {
  int ct = 0, nj = 0;
  cplx* G = nullptr;
  double *d = nullptr, *e = nullptr, *z = nullptr, *dinv = nullptr, *sig2 = nullptr, *lam = nullptr, *tn = nullptr;
  cplx* tau = nullptr;
  cplx* xch = nullptr;
  unsigned* cnt = nullptr;
  int* status = nullptr;
  int* host_status = nullptr;
  TwoSiteJob* djobs = nullptr;  // declined jobs for the block Jacobi
  TwoSiteJob* hjobs = nullptr;  // pinned
};

GBBuffers& gb_buffers() {
  static GBBuffers b;
  return b;
}

void gb_free(GBBuffers& b) {
  hipFree(b.G), hipFree(b.d), hipFree(b.e), hipFree(b.z), hipFree(b.dinv), hipFree(b.sig2), hipFree(b.tau);
  hipFree(b.lam), hipFree(b.tn);
  hipFree(b.xch), hipFree(b.cnt), hipFree(b.status), hipFree(b.djobs);
  hipHostFree(b.host_status), hipHostFree(b.hjobs);
  b = GBBuffers();
}

int gb_ensure(GBBuffers& b, int ct, int nj, hipStream_t st) {
  if (b.ct >= ct && b.nj >= nj) return AQC_OK;
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  const int c = std::max(ct, b.ct), n = std::max(nj, b.nj);
  gb_free(b);
  const size_t cc = (size_t)c * c * n;
  AQC_HIP_CHECK(hipMalloc(&b.G, cc * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.z, cc * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.dinv, cc * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.d, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.e, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.sig2, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.lam, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.tn, (size_t)n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.tau, (size_t)c * n * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.xch, (size_t)4 * c * n * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.cnt, (size_t)32 * n * sizeof(unsigned)));
  AQC_HIP_CHECK(hipMalloc(&b.status, (size_t)n * sizeof(int)));
  AQC_HIP_CHECK(hipMalloc(&b.djobs, (size_t)n * sizeof(TwoSiteJob)));
  AQC_HIP_CHECK(hipHostMalloc(&b.host_status, (size_t)n * sizeof(int)));
  AQC_HIP_CHECK(hipHostMalloc(&b.hjobs, (size_t)n * sizeof(TwoSiteJob)));
  b.ct = c, b.nj = n;
  return AQC_OK;
}

template <int CT>
int run_gram_big(const TwoSiteJob* hjobs, const TwoSiteJob* jobs, int nj, int cap_max, hipStream_t st) {
  GBBuffers& b = gb_buffers();
  int rc = gb_ensure(b, CT, nj, st);
  if (rc != AQC_OK) return rc;
  static bool attr = false;
  if (!attr) {
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_gb_back<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kRB * 256 * (int)sizeof(cplx)));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_gb_back<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kRB * 512 * (int)sizeof(cplx)));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_gb_back<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      kRB * 1024 * (int)sizeof(cplx)));
    attr = true;
  }
  GBArgs a;
  a.G = b.G, a.d = b.d, a.e = b.e, a.tau = b.tau, a.z = b.z, a.dinv = b.dinv, a.sig2 = b.sig2;
  a.lam = b.lam, a.tn = b.tn;
  a.xch = b.xch, a.cnt = b.cnt, a.status = b.status;
  AQC_HIP_CHECK(hipMemsetAsync(b.cnt, 0, (size_t)32 * nj * sizeof(unsigned), st));
  hipLaunchKernelGGL((k_gb_gram<CT>), dim3((CT / 64) * (CT / 64), nj), dim3(256), 0, st, jobs, a);
  AQC_CHECK_LAUNCH();
  // the tridiagonalisation's workgroups of a job must all be resident together (they exchange a
  // vector per column): rounds of at most min(240, resident capacity) workgroups, whole jobs each
  constexpr int P = CT * CT / 16384;
  static int resident = -1;
  if (resident < 0) {
    int dev = 0, ncu = 0, per_cu = 0;
    AQC_HIP_CHECK(hipGetDevice(&dev));
    AQC_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    AQC_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_gb_tridiag<CT>, 1024, 0));
    resident = ncu * std::min(per_cu, 1);
  }
  const int per_round = std::min(240, resident) / P;
  if (per_round < 1) {  // cannot hold one job's workgroups at once: every job declines
    AQC_HIP_CHECK(hipMemsetAsync(b.status, 0x7f, (size_t)nj * sizeof(int), st));
  } else {
    for (int j0 = 0; j0 < nj; j0 += per_round) {
      const int nr = std::min(per_round, nj - j0);
      hipLaunchKernelGGL((k_gb_tridiag<CT>), dim3(P * nr), dim3(1024), 0, st, jobs, a, j0);
      AQC_CHECK_LAUNCH();
    }
  }
  hipLaunchKernelGGL((k_gb_eig<CT>), dim3(nj), dim3(1024), 0, st, jobs, a);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_gb_inv<CT>), dim3(CT / 64, nj), dim3(64), 0, st, jobs, a);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_gb_gs<CT>), dim3(nj), dim3(64), 0, st, jobs, a);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_gb_back<CT>), dim3(CT / 16, nj), dim3(1024), kRB * CT * sizeof(cplx), st, jobs, a);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipMemcpyAsync(b.host_status, b.status, (size_t)nj * sizeof(int), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  int nd = 0;
  for (int i = 0; i < nj; ++i)
    if (b.host_status[i] != 0) b.hjobs[nd++] = hjobs[i];  // host copies keep qr = 0 (Jacobi contract)
  if (nd == 0) return AQC_OK;
  AQC_HIP_CHECK(hipMemcpyAsync(b.djobs, b.hjobs, (size_t)nd * sizeof(TwoSiteJob), hipMemcpyHostToDevice, st));
  return block_jacobi(b.djobs, nd, cap_max, st);
}

int g_gram_big = -1;  // -1: from AQC_BIG_GRAM (default on)

}  // namespace

int big_svd(const TwoSiteJob* hjobs, const TwoSiteJob* jobs, int nj, int side, int cap_max, hipStream_t st) {
  if (g_gram_big < 0) {
    const char* s = std::getenv("AQC_BIG_GRAM");
    g_gram_big = (s && std::strcmp(s, "0") == 0) ? 0 : 1;
  }
  if (!g_gram_big || side > 1024) return block_jacobi(jobs, nj, cap_max, st);
  if (side <= 256) return run_gram_big<256>(hjobs, jobs, nj, cap_max, st);
  if (side <= 512) return run_gram_big<512>(hjobs, jobs, nj, cap_max, st);
  return run_gram_big<1024>(hjobs, jobs, nj, cap_max, st);
}

}  // namespace aqc

extern "C" int aqc_svd_gram_big_ticks(double* out) {
  AQC_REQUIRE(out, "aqc_svd_gram_big_ticks: null argument");
  unsigned long long t[8];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(aqc::g_gbig_ticks), sizeof(t)));
  for (int i = 0; i < 8; ++i) out[i] = (double)t[i];
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(aqc::g_gbig_ticks), z, sizeof(z)));
  return AQC_OK;
}

extern "C" int aqc_svd_gram_big_stats(double* out) {
  AQC_REQUIRE(out, "aqc_svd_gram_big_stats: null argument");
  unsigned long long t[5];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(aqc::g_gbig_stats), sizeof(t)));
  for (int i = 0; i < 5; ++i) out[i] = (double)t[i];
  unsigned long long z[5] = {0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(aqc::g_gbig_stats), z, sizeof(z)));
  return AQC_OK;
}
