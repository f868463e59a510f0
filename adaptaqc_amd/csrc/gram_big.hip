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
//                 One exchange per column; spins bounded (100 ms, then the job declines).  At C = 512
//                 in two stages (aqc_gb_set_stages, the default): columns 0 .. 255 over 16
//                 workgroups, 256 .. 383 over 4 from the first stage's hand-off, a round's second
//                 stage beside the next round's first.  Stops at column C - 128 (aqc_gb_set_tail,
//                 the default) and leaves the trailing block to:
//   k_gb_tail     the last 128 columns of a job in one workgroup (exchange through the LDS, wave 0
//                 forms the reflectors); on the side stream, beside the next round's k_gb_tridiag.
//   k_gb_eig      the top K eigenvalues of T by multisection with the polynomial Sturm count, 64
//                 per workgroup;
//   k_gb_inv      inverse iteration (LDL^T of T - lambda I, three solves, one lane per vector,
//                 vectors in a per-job scratch), sigma^2 = z^T T z; declines (status 2) unless
//                 lambda_K > 1e-9 lambda_1, as the 2 chi = 128 path does;
//   k_gb_gs       Gram-Schmidt inside clusters of close eigenvalues.
//   k_gb_tfac     compact WY factors T of the reflectors in blocks of 16 (LAPACK zlarft), on a
//                 third stream beside k_gb_eig / k_gb_inv / k_gb_gs.
//   k_gb_back     V = Q Z on the matrix cores, 16 columns per workgroup, blocks of 16 reflectors
//                 from the last (V -= Y T Y^H V); output W = V Sigma, sig, qr = 1 -- the contract of the
//                 2 chi = 128 Gram path (work column c = right singular vector c of X times
//                 sigma_c), so k_rank / k_split_* run unchanged.
// Jobs that decline (floor, timeout, gram disabled) run the block Jacobi afterwards (the host reads
// the statuses once, after k_gb_eig).
// The per-job GEMM kernels (k_gb_gram, k_gb_back) run on 1-D grids that put a job's workgroups on
// one XCD (aqc_internal.h xcd_job_block: they share the job's operand panels in that XCD's L2).
#include <cstdlib>
#include <cstring>

#include "aqc_gemm.h"
#include "mps_internal.h"

namespace aqc {

// calls, taken, declined (gram off / shape), declined at the eigenvalue floor, exchange timeouts
__device__ unsigned long long g_gbig_stats[8];
// shader-clock ticks of job 0's first workgroup (thread 0), summed over calls: tridiagonalisation
// phases [0] pass + row sums, [1] publish (stores, vmcnt, barrier), [2] counter wait, [3] reads + p^H v,
// [4] w, new row, partial norms; [5] k_gb_eig (job 0, block 0), [6] k_gb_back (job 0, block 0), [7] k_gb_inv (job 0,
// lane 0), [8] the next reflector's zlarfg
__device__ unsigned long long g_gbig_ticks[9];

namespace {

constexpr double kGbRelFloor = 1e-9;
constexpr unsigned long long kSpinTicks = 10000000ull;  // s_memrealtime (100 MHz): 100 ms
// the counter-wait limit in force (aqc_gb_set_spin_limit: tests force the timeout decline with 0)
unsigned long long g_gb_spin = kSpinTicks;
// the trailing 128 columns in one workgroup (aqc_gb_set_tail; -1: from AQC_GB_TAIL, default on)
int g_gb_tail = -1;
// two exchange stages at 2 chi = 512 (-1: from AQC_GB_STAGES, default 2)
int g_gb_stages = -1;

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

// rows of X (L = max(2 chi_l, 2 chi_r)) per Gram side C: at CT = 1024 a job may have L = 2048 (bond
// capacity 1024); the certificate's Y = X V (L x K) then needs twice the C x C G scratch
template <int CT>
constexpr int kGLong = CT >= 1024 ? 2 : 1;

struct GBArgs {
  cplx* G;         // per job CT x CT: G, then the reflectors (row k = v_k at columns > k); the
                   // certificate's Y (kGLong CT x CT) after them
  size_t gstride;  // elements of G per job: kGLong<CT> CT^2
  cplx* tfac;      // per job (CT / 16) x 16 x 16: compact WY factors T of the reflector blocks
  cplx* yc;        // per job CT x CT: the reflectors column-major (v_k[row] at row * CT + k)
  double* d;       // per job CT
  double* e;       // per job CT
  cplx* tau;       // per job CT
  double* z;       // per job CT x CT: eigenvector i at z[row * CT + i]
  double* dinv;    // per job CT x CT: inverse-iteration pivots
  double* sig2;    // per job CT
  double* lam;     // per job CT: the top K eigenvalues of T, descending
  double* err;     // per job CT: their multisection brackets' half widths
  int* kept;       // per job: the kept count (reduce_zeros on lam, k_gb_keep)
  double* tail;    // per job: the tail sum that decision dropped (to sig[kSigTail])
  int* cert;       // per job: the decision assumed the open-CHOP values chopped (k_gb_cert checks)
  double* certsum; // per job: ||X - X V V^H||_F^2 (k_gb_cert)
  double* tn;      // per job: ||T|| (Gershgorin)
  cplx* xch;       // per job 8 x CT: p (two buffers), old row k + 1 (two buffers); from 4 CT the
                   // hand-off to the next stage (v, v', w, the scalars: apart from the exchange
                   // buffers, which a slower workgroup may still be reading when workgroup 0 ends)
  unsigned* cnt;   // per job 32 words (128 B)
  int* status;     // per job: 0 ok, 1 declined (gram off / shape), 2 floor, 3 exchange timeout
  unsigned long long spin;  // counter-wait limit (s_memrealtime ticks, 100 MHz) before a timeout
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
// grid (nbt (nbt + 1) / 2, nj) with nbt = CT / 64, 256 threads.  Entries outside C x C are zero.
template <int CT>
__global__ __launch_bounds__(256) void k_gb_gram(const TwoSiteJob* __restrict__ jobs, GBArgs a, int nj) {
  int jb, bx;
  if (!xcd_job_block(nj, jb, bx)) return;  // (a job's blocks on one XCD: they share X's panels)
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  // (C > CT: both sides above the class -- 2 chi_l, 2 chi_r > 1024 -- declines to the block Jacobi)
  const bool decline = !j.gram || C < 4 || C > CT;
  if (bx == 0 && threadIdx.x == 0) {
    atomicAdd(&g_gbig_stats[0], 1ull);
    *(gi32*)(a.status + jb) = decline ? 1 : 0;
    if (decline) atomicAdd(&g_gbig_stats[2], 1ull);
  }
  if (decline) return;
  // blocks on and above the diagonal (bi <= bj), the one below mirrored: G is Hermitian
  constexpr int nbt = CT / 64;
  int bi = 0, rem = bx;
  while (rem >= nbt - bi) rem -= nbt - bi, ++bi;
  const int bj = (bi + rem) * 64;
  bi *= 64;
  cplx* G = a.G + (size_t)jb * a.gstride;
  const cplx* th = j.theta;
  __shared__ GemmLds lds;
  const int m = bi < C ? min(64, C - bi) : 0, n = bj < C ? min(64, C - bj) : 0;
  auto store = [&](int i, int jj, cplx v) {
    stg(G + (size_t)(bi + i) * CT + bj + jj, v);
    if (bi != bj) stg(G + (size_t)(bj + jj) * CT + bi + i, cconj(v));
  };
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
    if (i >= m || jj >= n) {
      stg(G + (size_t)(bi + i) * CT + bj + jj, cmk(0, 0));
      stg(G + (size_t)(bj + jj) * CT + bi + i, cmk(0, 0));
    }
  }
}

__device__ __forceinline__ double rcp_nr2(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = r * fma(-x, r, 2.0);
  r = r * fma(-x, r, 2.0);
  return r;
}

// ---- tridiagonalisation over P workgroups per job -----------------------------------------------
// Column exchange: sc1 stores, s_waitcnt vmcnt(0), a barrier and one counter add per workgroup; the
// consumers poll the counter with one lane (the MI355X guide's "Valid forms" row 1).  (The guide's
// 8-byte {data, tag} granules -- every consumer thread polling its values' tags, no store
// acknowledgement or counter -- measured slower at C = 512: 14.6 K ticks per column waiting against
// 5.4 K, the 16 K polling threads per job crowd the fabric.)

// sum over aligned groups of N (16, 32, 64) lanes, result in every lane of the group; VALU only
// (DPP row sums, then v_permlane16_swap / v_permlane32_swap: the partner row's value without the
// LDS crossbar)
template <int N>
__device__ __forceinline__ double lane_sum(double v) {
  v = row_sum16(v);
  if constexpr (N >= 32) {
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  if constexpr (N >= 64) {
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    v = __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
  }
  return v;
}

// sum of f(0) .. f(N - 1) as a balanced tree (log2 N dependent adds instead of N - 1)
template <int N, class F>
__device__ __forceinline__ double tree_sum(F f) {
  if constexpr (N == 1) {
    return f(0);
  } else {
    return tree_sum<N / 2>(f) + tree_sum<N - N / 2>([&](int w) { return f(w + N / 2); });
  }
}

// zlarfg with the divisions as reciprocals (rcp + two Newton steps: full precision)
__device__ __forceinline__ void zlarfg_f(cplx alpha, double xn2, cplx& tau, double& beta, cplx& scale) {
  if (xn2 == 0.0 && alpha.y == 0.0) {
    tau = cmk(0, 0);
    beta = alpha.x;
    scale = cmk(0, 0);
    return;
  }
  const double nrm = sqrt(fma(alpha.x, alpha.x, fma(alpha.y, alpha.y, xn2)));
  beta = alpha.x >= 0.0 ? -nrm : nrm;
  const double rb = rcp_nr2(beta);
  tau = cmk((beta - alpha.x) * rb, -alpha.y * rb);
  const cplx den = cmk(alpha.x - beta, alpha.y);
  const double id = rcp_nr2(cnorm2(den));
  scale = cmk(den.x * id, -den.y * id);
}

// grid (P * njobs_in_round), 1024 threads.  Thread t: row group t / TPG of RPL rows (local rows
// RPL * group + u, global r = local P + g), columns q + TPG i (q = t % TPG, i < CPL).  RPL = 1 is
// the one instantiated: two rows per lane read each column's v, w operands from the LDS once for
// both, but the register tile then spilled (40 VGPRs at 2 chi = 512: 0.49 against 0.36 ms per
// config-5 gate).  Per column k:
//   pass      the deferred rank-2 update G -= v w^H + w v^H of reflector k - 1 and s = (G v_k)_r in
//             one sweep over the registers; column blocks and row groups at or above k are dead and
//             skipped
//   exchange  p_r = tau_k s_r and conj(G[r][k + 1]) (row k + 1 as it was before this update, by
//             symmetry: every workgroup its rows' entries) out, all p and that row in; d_k, e_k, tau_k and this workgroup's slice of v_k go to the scratch
//             here, where their store latency hides behind the wait
//   tail      p^H v (one workgroup reduction), w_k = p + a2 v, the new row k + 1 = old - conj(w) -
//             w_{k+1} conj(v), its norm below the subdiagonal (a second reduction); wave 0 alone
//             forms reflector k + 1 (zlarfg's scalars and v into the LDS; in every wave the
//             redundant scalar chain cost 4x its issue)
//
// Stages (CF: the job's size; CT: the trailing block this launch starts from, K0 = CF - CT; TS: the
// trailing block it hands off, with TAIL): CF = CT = 512 runs columns 0 .. 255 over 16 workgroups
// and hands the trailing 256 over to CT = 256 (4 workgroups, columns 256 .. 383, from the hand-off
// of reflector 255: its deferred update, v_256 and its scalars), which hands the last 128 to
// k_gb_tail.  A job's workgroups then fall from 16 to 4 for the second stage, so one round's
// second stages run beside the next round's first (the columns in the exchange per wave of rounds:
// 256 + 256 + 128 instead of 384 + 384).
template <int CT, int RPL, bool TAIL, int CF = CT, int TS = 128>
__global__ __launch_bounds__(1024) void k_gb_tridiag(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  constexpr int K0 = CF - CT;
  static_assert(K0 >= 0 && TS >= 128 && TS < CT, "stage sizes");
  constexpr int CPL = 16 / RPL, TPG = CT / CPL;
  constexpr int R = RPL * (1024 / TPG), P = CT / R;
  static_assert(TPG <= 64 && TPG >= 16, "row group inside one wave");
  // waves holding entries of the CT-long vectors (the others' partial sums are zero)
  constexpr int kRW = CT / 64 < 16 ? CT / 64 : 16;
  const int jb = job0 + (int)blockIdx.x / P, g = (int)blockIdx.x % P;
  if (*(const gi32*)(a.status + jb) != 0) return;  // uniform over the job's workgroups
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = tid / TPG, q = tid % TPG;
  int rr[RPL];
#pragma unroll
  for (int u = 0; u < RPL; ++u) rr[u] = (grp * RPL + u) * P + g;
  // (phase ticks on the last wave: its rows stay active to the end)
  const bool tick = jb == 0 && g == 0 && tid == 960;
  // (local indices: the stage's trailing block starts at row / column K0 of the job's G)
  cplx* G = a.G + (size_t)jb * a.gstride + (size_t)K0 * CF + K0;
  double* dd = a.d + (size_t)jb * CF + K0;
  double* ee = a.e + (size_t)jb * CF + K0;
  cplx* tt = a.tau + (size_t)jb * CF + K0;
  cplx* xch = a.xch + (size_t)jb * 8 * CF;
  cplx* hoff = xch + 4 * CF;  // the stage hand-off
  unsigned* cnt = a.cnt + (size_t)jb * 32 + (K0 ? 16 : 0);  // (a second stage: its own 64-byte line)
  __shared__ cplx vL[2][CT], wL[CT], rhoL[CT];
  __shared__ double redd[16];
  __shared__ cplx redc[16];
  __shared__ cplx s_tau, s_pk1;
  __shared__ double s_beta, s_dk;
  __shared__ int s_abort;
  // phase ticks of job 0's first workgroup, thread 0 (kept in the LDS: per-lane counters would take
  // 14 VGPRs from the register tile)
  __shared__ unsigned long long s_tk[7];
  if (tick) {
    for (int i = 0; i < 6; ++i) s_tk[i] = 0;
    s_tk[6] = __builtin_amdgcn_s_memtime();
  }
  auto tmark = [&](int ph) {
    if (tick) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      s_tk[ph] += t - s_tk[6];
      s_tk[6] = t;
    }
  };
  cplx A[RPL][CPL];
#pragma unroll
  for (int u = 0; u < RPL; ++u)
#pragma unroll
    for (int i = 0; i < CPL; ++i) A[u][i] = ldg(G + (size_t)rr[u] * CF + q + TPG * i);
  if constexpr (K0 == 0) {
    if (tid < CT) {
      rhoL[tid] = ldg(G + tid);  // row 0
      wL[tid] = cmk(0, 0);       // no deferred update before column 0
      vL[1][tid] = cmk(0, 0);
    }
  } else {  // the previous stage's hand-off (K0 even: v_K0 in vL[0])
    if (tid < CT) {
      vL[0][tid] = ldg(hoff + K0 + tid);
      vL[1][tid] = ldg(hoff + CF + K0 + tid);
      wL[tid] = ldg(hoff + 2 * CF + K0 + tid);
    }
    if (tid == 0) {
      s_tau = ldg(hoff + 3 * CF);
      const cplx bd = ldg(hoff + 3 * CF + 1);
      s_beta = bd.x;
      s_dk = bd.y;
    }
  }
  if (tid == 0) s_abort = 0;
  // reflector k from rhoL = row k and the partial norms in redd, by wave 0 alone: zlarfg's scalars
  // and v_k (1 at k + 1, conj(rho_k[c]) scale below, 0 above) into vL[k & 1]
  auto reflector = [&](int k) {
    double xn2 = tree_sum<kRW>([&](int w) { return redd[w]; });
    cplx tau_, sc;
    double beta;
    zlarfg_f(cconj(rhoL[k + 1]), xn2, tau_, beta, sc);
    // (one base address per lane, offsets 1 KB apart: with c = lane + 64 i kept per i, the eight
    // addresses were hoisted out of the column loop and spilled -- a scratch reload and a full
    // vmcnt wait per entry on the zlarfg chain)
    const cplx* rp = rhoL + lane;
    cplx* vp = vL[k & 1] + lane;
    const int d0 = lane - (k + 1);
#pragma unroll
    for (int i = 0; i < CT / 64; ++i) {
      const int d = d0 + 64 * i;
      vp[64 * i] = d == 0 ? cmk(1, 0) : (d > 0 ? cmul(cconj(rp[64 * i]), sc) : cmk(0, 0));
    }
    if (lane == 0) {
      s_tau = tau_;
      s_beta = beta;
      s_dk = rhoL[k].x;
    }
  };
  __syncthreads();
  if constexpr (K0 == 0) {
    const cplx xt = tid < CT ? cconj(rhoL[tid]) : cmk(0, 0);
    const double part = lane_sum<64>((tid >= 2 && tid < CT) ? cnorm2(xt) : 0.0);
    if (lane == 0) redd[wave] = part;
    __syncthreads();
    if (wave == 0) reflector(0);
    __syncthreads();
  }
  // with TAIL the loop stops at kt = CT - TS: the trailing TS columns run in the next stage
  int kt = TAIL ? CT - TS : CT - 1;
  asm volatile("" : "+s"(kt));  // (opaque: a constant trip count spilled the register tile)
  for (int k = 0; k < kt; ++k) {
    const int cur = k & 1, prv = cur ^ 1;
    // ---- the deferred update of reflector k - 1, then s = (G v_k)_r
    cplx s[RPL], xcol[RPL];  // xcol: this lane's G[r][k + 1] after the update (its publish)
#pragma unroll
    for (int u = 0; u < RPL; ++u) s[u] = cmk(0, 0), xcol[u] = cmk(0, 0);
    const int ic = (k + 1) / TPG;  // the register holding column k + 1 (uniform)
    if (rr[RPL - 1] > k) {
      cplx vr[RPL], wr[RPL];
#pragma unroll
      for (int u = 0; u < RPL; ++u) vr[u] = vL[prv][rr[u]], wr[u] = wL[rr[u]];
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        if (TPG * i + TPG - 1 > k) {
          const int c = q + TPG * i;
          const cplx vp = vL[prv][c], wc = wL[c], vc = vL[cur][c];
#pragma unroll
          for (int u = 0; u < RPL; ++u) {
            A[u][i] = csub(A[u][i], cadd(cmulc(vr[u], wc), cmulc(wr[u], vp)));
            s[u] = cfma(A[u][i], vc, s[u]);
            if (i == ic) xcol[u] = A[u][i];
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < RPL; ++u) s[u] = cmk(lane_sum<TPG>(s[u].x), lane_sum<TPG>(s[u].y));
    tmark(0);
    // (read after the pass: kept out of its register budget)
    const cplx tau = s_tau;
    const cplx vt = tid < CT ? vL[cur][tid] : cmk(0, 0);
    cplx* xp = xch + cur * CT;
    cplx* xr = xch + (2 + cur) * CT;
    if (q == 0) {
#pragma unroll
      for (int u = 0; u < RPL; ++u) st_sc1(xp + rr[u], rr[u] > k ? cmul(tau, s[u]) : cmk(0, 0));
    }
    // row k + 1 before this step's update, by Hermitian symmetry from column k + 1: every row's
    // lane holding that column publishes conj(A[r][k + 1]) (the owner alone writing the whole row
    // made its workgroup the last to publish every column)
    if (q == (k + 1) % TPG) {
#pragma unroll
      for (int u = 0; u < RPL; ++u) st_sc1(xr + rr[u], cconj(xcol[u]));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    tmark(1);
    if (tid == 0) {
      __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (g == 0) {  // the tridiagonal's entries and tau_k
        stg(dd + k, s_dk);
        stg(ee + k, s_beta);
        stg(tt + k, tau);
      }
      const unsigned target = (unsigned)P * (unsigned)(k + 1);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin) {
          s_abort = 1;
          break;
        }
      }
    }
    // reflector k to row k of the scratch, each workgroup its own CT / P contiguous entries (a
    // strided store here held the next publish wait: the stores must finish before it).  Row 0 is
    // read at entry by every workgroup of the job (rhoL, and workgroup 0's register rows), so at
    // k = 0 the store waits for the barrier behind thread 0's counter wait: only then has every
    // workgroup published column 0, i.e. passed its entry loads.  From k = 1 on this workgroup has
    // already seen step k - 1's full count, so every workgroup is past its entry.
    const bool own_row = tid > k && tid / (CT / P) == g;
    if (k > 0 && own_row) stg(G + (size_t)k * CF + tid, vt);
    __syncthreads();
    if (k == 0 && own_row && !s_abort) stg(G + tid, vt);
    if (s_abort) {
      if (tid == 0 && g == 0) {
        *(gi32*)(a.status + jb) = 3;
        atomicAdd(&g_gbig_stats[4], 1ull);
      }
      return;
    }
    tmark(2);
    const cplx pt = tid < CT ? ld_sc1(xp + tid) : cmk(0, 0);
    const cplx ro = tid < CT ? ld_sc1(xr + tid) : cmk(0, 0);
    // p_{k+1} to every thread through the LDS (one sc1 load of the same 16 bytes by every wave of
    // every workgroup queued at one memory channel)
    if (tid == k + 1) s_pk1 = pt;
    const cplx pvp = cconjmul(pt, vt);
    const double px = lane_sum<64>(pvp.x), py = lane_sum<64>(pvp.y);
    if (lane == 0) redc[wave] = cmk(px, py);
    __syncthreads();
    const cplx pk1 = s_pk1;
    tmark(3);
    // ---- w = p - tau / 2 (p^H v) v, the new row k + 1 and its norm below the subdiagonal
    cplx pv = cmk(0, 0);
#pragma unroll
    for (int w = 0; w < kRW; ++w) pv = cadd(pv, redc[w]);
    const cplx a2 = cscale(cmul(tau, pv), -0.5);
    const cplx wt = cfma(a2, vt, pt);
    const cplx wk1 = cadd(pk1, a2);
    const cplx rho = csub(csub(ro, cconj(wt)), cmulc(wk1, vt));
    if (tid < CT) {
      wL[tid] = wt;  // (w_{k-1} was last read in this step's pass, before the exchange's barrier)
      rhoL[tid] = rho;  // (row k: last read in the pass, for v_k)
    }
    if (k == CT - 2) {
      if (g == 0 && tid == CT - 1) stg(dd + CT - 1, rho.x);
      break;
    }
    const double part = lane_sum<64>((tid >= k + 3 && tid < CT) ? cnorm2(rho) : 0.0);
    if (lane == 0) redd[wave] = part;
    __syncthreads();
    tmark(4);
    if (wave == 0) reflector(k + 1);
    __syncthreads();
    tmark(5);
  }
  if constexpr (TAIL) {
    // ---- hand-off to k_gb_tail: the trailing block (rows and columns >= kt, reflector kt - 1's
    // update still deferred) to rows kt.. of the scratch (free until their reflectors: rows < kt
    // hold v_0 .. v_kt-1); workgroup 0 adds v_kt-1, v_kt, w_kt-1 and reflector kt's scalars
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      if (rr[u] >= kt) {
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
          const int c = q + TPG * i;
          if (TPG * i + TPG - 1 >= kt && c >= kt) stg(G + (size_t)rr[u] * CF + c, A[u][i]);
        }
      }
    }
    if (g == 0) {
      if (tid < CT) {
        stg(hoff + K0 + tid, vL[0][tid]);
        stg(hoff + CF + K0 + tid, vL[1][tid]);
        stg(hoff + 2 * CF + K0 + tid, wL[tid]);
      }
      if (tid == 0) {
        stg(hoff + 3 * CF, s_tau);
        stg(hoff + 3 * CF + 1, cmk(s_beta, s_dk));
      }
    }
  }
  if (tick) {
    for (int i = 0; i < 5; ++i) atomicAdd(&g_gbig_ticks[i], s_tk[i]);
    atomicAdd(&g_gbig_ticks[8], s_tk[5]);
  }
}

// ---- the last 128 columns in one workgroup: grid (njobs_in_round), 1024 threads ----
// k_gb_tridiag stops at column kt = CT - 128 and leaves the trailing block (reflector kt - 1's
// update still deferred) in rows kt.. of the scratch, v_kt-1, v_kt, w_kt-1 and reflector kt's
// scalars in the exchange buffer.  Thread t holds local row t / 8, columns t % 8 + 8 i (i < 16);
// per column the pass (as k_gb_tridiag's), p and the old row k + 1 into the LDS, one barrier; then
// wave 0 alone (two columns per lane) forms p^H v, w, the new row k + 1, its norm and the next
// reflector -- all reductions inside the wave -- and a second barrier.  No cross-workgroup
// exchange: this is the part of the tridiagonalisation where the trailing block is too small to
// pay for one.  Launched on the side stream, so a round's tails run beside the next round's
// k_gb_tridiag.
__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

template <int CT>
__global__ __launch_bounds__(1024) void k_gb_tail(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  constexpr int NT = 128, kt = CT - NT;
  const int jb = job0 + (int)blockIdx.x;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tr = tid >> 3, tq = tid & 7;
  const bool tick = jb == 0 && tid == 0;
  cplx* G = a.G + (size_t)jb * a.gstride;
  double* dd = a.d + (size_t)jb * CT;
  double* ee = a.e + (size_t)jb * CT;
  cplx* tt = a.tau + (size_t)jb * CT;
  const cplx* xch = a.xch + (size_t)jb * 8 * CT + 4 * CT;  // the previous stage's hand-off
  __shared__ cplx vL[2][NT], wL[NT], pL[NT], roL[NT];
  __shared__ cplx s_tau;
  __shared__ double s_beta, s_dk;
  __shared__ unsigned long long tk[6];  // phase ticks of job 0, thread 0 ([5]: the last mark)
  if (tick) {
    for (int i = 0; i < 5; ++i) tk[i] = 0;
    tk[5] = __builtin_amdgcn_s_memtime();
  }
  auto tmark = [&](int ph) {
    if (tick) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      tk[ph] += t - tk[5];
      tk[5] = t;
    }
  };
  cplx T[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) T[i] = ldg(G + (size_t)(kt + tr) * CT + kt + tq + 8 * i);
  if (tid < NT) {
    vL[0][tid] = ldg(xch + kt + tid);
    vL[1][tid] = ldg(xch + CT + kt + tid);
    wL[tid] = ldg(xch + 2 * CT + kt + tid);
  }
  if (tid == 0) {
    s_tau = ldg(xch + 3 * CT);
    const cplx bd = ldg(xch + 3 * CT + 1);
    s_beta = bd.x;
    s_dk = bd.y;
  }
  __syncthreads();
  for (int k = kt; k < CT - 1; ++k) {
    const int cur = k & 1, prv = cur ^ 1;
    const int kl = k - kt, kk = kl + 1, ic = kk >> 3;
    cplx s = cmk(0, 0), xcol = cmk(0, 0);
    if (tr > kl) {
      const cplx vr = vL[prv][tr], wr = wL[tr];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (8 * i + 7 > kl) {
          const int c = tq + 8 * i;
          const cplx vp = vL[prv][c], wc = wL[c], vc = vL[cur][c];
          T[i] = csub(T[i], cadd(cmulc(vr, wc), cmulc(wr, vp)));
          s = cfma(T[i], vc, s);
          if (i == ic) xcol = T[i];
        }
      }
    }
    s = cmk(group_sum<8>(s.x), group_sum<8>(s.y));
    tmark(0);
    const cplx tau = s_tau;
    if (tq == 0) pL[tr] = tr > kl ? cmul(tau, s) : cmk(0, 0);
    if (tq == (kk & 7)) roL[tr] = cconj(xcol);
    __syncthreads();
    tmark(1);
    if (wave == 0) {
      if (lane == 0) {
        stg(dd + k, s_dk);
        stg(ee + k, s_beta);
        stg(tt + k, tau);
      }
      cplx vt[2], pt[2], ro[2];
      cplx pvp = cmk(0, 0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        vt[h] = vL[cur][c];
        pt[h] = pL[c];
        ro[h] = roL[c];
        pvp = cadd(pvp, cconjmul(pt[h], vt[h]));
        if (c > kl) stg(G + (size_t)k * CT + kt + c, vt[h]);  // reflector k to row k of the scratch
      }
      const cplx pv = cmk(lane_sum<64>(pvp.x), lane_sum<64>(pvp.y));
      const cplx a2 = cscale(cmul(tau, pv), -0.5);
      const cplx wk1 = cadd(pL[kk], a2);
      cplx rho[2];
      double part = 0.0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = lane + 64 * h;
        const cplx wt = cfma(a2, vt[h], pt[h]);
        wL[c] = wt;  // (w_k-1 was last read in this step's pass, before the barrier)
        rho[h] = csub(csub(ro[h], cconj(wt)), cmulc(wk1, vt[h]));
        if (c > kl + 2) part += cnorm2(rho[h]);
      }
      tmark(3);
      if (k == CT - 2) {
        if (lane == 63) stg(dd + CT - 1, rho[1].x);
      } else {
        // reflector k + 1 from the new row k + 1 (local column kl + 2 is alpha)
        const double xn2 = lane_sum<64>(part);
        const int ca = kl + 2, cd = kl + 1;
        const cplx ra = (ca >> 6) ? rho[1] : rho[0];
        const double dk1 = readlane_d(((cd >> 6) ? rho[1] : rho[0]).x, cd & 63);
        const cplx alpha = cmk(readlane_d(ra.x, ca & 63), -readlane_d(ra.y, ca & 63));
        cplx tau_, sc;
        double beta;
        zlarfg_f(alpha, xn2, tau_, beta, sc);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = lane + 64 * h;
          vL[prv][c] = c == ca ? cmk(1, 0) : (c > ca ? cmul(cconj(rho[h]), sc) : cmk(0, 0));
        }
        if (lane == 0) {
          s_tau = tau_;
          s_beta = beta;
          s_dk = dk1;
        }
        tmark(4);
      }
    }
    if (k == CT - 2) break;
    __syncthreads();
    tmark(2);
  }
  if (tick) {
    for (int i = 0; i < 4; ++i) atomicAdd(&g_gbig_ticks[i], tk[i]);
    atomicAdd(&g_gbig_ticks[8], tk[4]);
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

// ---- the top K eigenvalues of T: grid (ceil(K / 64), nj), 256 threads -----------------------
// Multisection with the polynomial Sturm count (one dependent FMA per row; the pass is FP64-issue
// bound): every workgroup brackets all eigenvalues with one pass of 256 shifts, then narrows its
// 64 by 12 rounds of 5-section, 4 lanes per eigenvalue (span x 1.6e-11 at the end; the inverse
// iteration and the Rayleigh quotient take sigma^2 from there).  Eigenvalues to the scratch,
// descending; ||T|| (Gershgorin) with them.
template <int CT>
__global__ __launch_bounds__(256) void k_gb_eig(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.y;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  if ((int)blockIdx.x * 64 >= K) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  __shared__ double s_e[CT];
  __shared__ double2 s_de[CT];
  __shared__ int cntb[256];
  __shared__ double rlo[4], rhi[4], rtn[4];
  const double* dd = a.d + (size_t)jb * CT;
  const double* ee = a.e + (size_t)jb * CT;
  double lo = 1e300, hi = -1e300, tn = 0.0;
  for (int i = tid; i < CT; i += 256) s_e[i] = i < CT - 1 ? ldg(ee + i) : 0.0;
  __syncthreads();
  for (int i = tid; i < CT; i += 256) {
    const double el = i > 0 ? fabs(s_e[i - 1]) : 0.0, er = fabs(s_e[i]);
    const double di = ldg(dd + i);
    lo = fmin(lo, di - el - er);
    hi = fmax(hi, di + el + er);
    tn = fmax(tn, fabs(di) + el + er);
    s_de[i] = make_double2(di, i > 0 ? s_e[i - 1] * s_e[i - 1] : 0.0);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off));
    hi = fmax(hi, __shfl_xor(hi, off));
    tn = fmax(tn, __shfl_xor(tn, off));
  }
  if (lane == 0) rlo[wave] = lo, rhi[wave] = hi, rtn[wave] = tn;
  __syncthreads();
  lo = fmin(fmin(rlo[0], rlo[1]), fmin(rlo[2], rlo[3]));
  hi = fmax(fmax(rhi[0], rhi[1]), fmax(rhi[2], rhi[3]));
  tn = fmax(fmax(rtn[0], rtn[1]), fmax(rtn[2], rtn[3]));
  const double span = fmax(hi - lo, 1e-300);
  const double lo0 = lo - 1e-12 * span, hi0 = hi + 1e-12 * span, span0 = hi0 - lo0;
  const double itn = 1.0 / fmax(tn, 1e-300);
  for (int i = tid; i < CT; i += 256) {  // the Sturm rows scaled by 1 / ||T||
    const double2 de = s_de[i];
    s_de[i] = make_double2(de.x * itn, de.y * itn * itn);
  }
  __syncthreads();
  constexpr int kG = 4, kFirst = 256, kRounds = 12;
  constexpr double kInvF = 1.0 / (kFirst + 1), kInvG = 1.0 / (kG + 1);
  // three more rounds when the tail threshold sits above the Gram form's noise (aqc::gram_keep)
  const int rounds = kRounds + (j.thr > 1e-12 * tn ? 3 : 0);
  cntb[tid] = sturm_poly(s_de, CT, (lo0 + span0 * (double)(tid + 1) * kInvF) * itn);
  __syncthreads();
  const int sub = tid % kG, eid = blockIdx.x * 64 + tid / kG;
  const int a_ = CT - 1 - min(eid, CT - 1);  // ascending index of the eid-th largest
  double l2, h2;
  {
    int l = 0, h = kFirst;
    while (l < h) {
      const int m = (l + h) >> 1;
      if (cntb[m] >= a_ + 1) h = m;
      else l = m + 1;
    }
    l2 = l > 0 ? lo0 + span0 * (double)l * kInvF : lo0;
    h2 = l < kFirst ? lo0 + span0 * (double)(l + 1) * kInvF : hi0;
  }
  for (int round = 0; round < rounds; ++round) {
    const double x = l2 + (h2 - l2) * (double)(sub + 1) * kInvG;
    const int cnt = sturm_poly(s_de, CT, x * itn);
    const unsigned long long bal = __ballot(cnt >= a_ + 1);
    const unsigned int gm = (unsigned int)(bal >> (lane & ~(kG - 1))) & ((1u << kG) - 1u);
    const int f = gm ? __builtin_ctz(gm) : kG;
    const double nhi = f < kG ? l2 + (h2 - l2) * (double)(f + 1) * kInvG : h2;
    const double nlo = f > 0 ? l2 + (h2 - l2) * (double)f * kInvG : l2;
    l2 = nlo;
    h2 = nhi;
  }
  if (eid < K && sub == 0) {
    stg(a.lam + (size_t)jb * CT + eid, 0.5 * (l2 + h2));
    stg(a.err + (size_t)jb * CT + eid, 0.5 * (h2 - l2));
  }
  if (blockIdx.x == 0 && tid == 0) stg(a.tn + jb, tn);
  if (jb == 0 && blockIdx.x == 0 && tid == 0) atomicAdd(&g_gbig_ticks[5], __builtin_amdgcn_s_memtime() - t_start);
}

// ---- the kept count: reduce_zeros on the eigenvalues (aqc::gram_keep, as the 2 chi = 128 path):
// grid (nj), one thread.  An open decision or a kept value below the floor declines the job
// (status 2: the block Jacobi decides).  The kernels after it use the kept count. ----
template <int CT>
__global__ __launch_bounds__(64) void k_gb_keep(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.x;
  if (threadIdx.x != 0 || *(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  double tail = 0.0;
  int cert = 0;
  const int k = gram_keep(a.lam + (size_t)jb * CT, a.err + (size_t)jb * CT, K, C, j.max_chi, j.thr, ldg(a.tn + jb),
                          kGbRelFloor, tail, &cert);
  if (k < 0) {
    *(gi32*)(a.status + jb) = 2;
    atomicAdd(&g_gbig_stats[3], 1ull);
    return;
  }
  *(gi32*)(a.kept + jb) = k;
  *(gi32*)(a.cert + jb) = cert;
  stg(a.certsum + jb, 0.0);
  stg(a.tail + jb, tail);
  if (cert) atomicAdd(&g_gbig_stats[5], 1ull);
}

__device__ __forceinline__ int kept_count(const GBArgs& a, int jb) { return *(const gi32*)(a.kept + jb); }

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
__global__ __launch_bounds__(64) void k_gb_inv(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.y;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  K = kept_count(a, jb);
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
// members' sigma^2 again: grid (nj), 256 threads ----
// Member i of a cluster starting at `start` against members start .. i - 1 (already orthonormal) in
// block form, twice (classical Gram-Schmidt with re-orthogonalisation): all m = i - start dot
// products at once -- lanes along the members (coalesced 512-byte row pieces of the row-major
// scratch), the four waves splitting the rows, partials through the LDS -- then each row's update
// by its own thread.  (Round 5: one wave, sequential Gram-Schmidt with every dot product a column
// read strided by CT: 403 us a call at CT = 256 when the kept spectrum's tiny values form one wide
// cluster -- the absolute gap test puts every sigma^2 below 1e-7 ||T|| in it -- 23% of a C = 256
// update in the unbounded compile's Rotosolve layer.)
template <int CT>
__global__ __launch_bounds__(256) void k_gb_gs(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.x;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  K = kept_count(a, jb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const double* lam = a.lam + (size_t)jb * CT;
  const double ortol = 1e-7 * ldg(a.tn + jb);
  double* zb = a.z + (size_t)jb * CT * CT;
  const double* dd = a.d + (size_t)jb * CT;
  const double* ee = a.e + (size_t)jb * CT;
  __shared__ double part[4][64];
  __shared__ double dp[CT];
  __shared__ double red[2][4];
  auto block_sum2 = [&](double x, double y, double& sx, double& sy) {
    x = wave_sum_b(x);
    y = wave_sum_b(y);
    if (lane == 0) red[0][wave] = x, red[1][wave] = y;
    __syncthreads();
    sx = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    sy = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    __syncthreads();
  };
  int start = 0;
  for (int i = 1; i < K; ++i) {
    if (ldg(lam + i - 1) - ldg(lam + i) >= ortol) {  // (uniform)
      start = i;
      continue;
    }
    const int m = i - start;
    // ||z_i||^2 before the projection (the "twice is enough" test below)
    double nb = 0.0, unused = 0.0;
    for (int r = tid; r < CT; r += 256) {
      const double z = zb[(size_t)r * CT + i];
      nb = fma(z, z, nb);
    }
    block_sum2(nb, 0.0, nb, unused);
    double n2 = 0.0;
    for (int pass = 0; pass < 2; ++pass) {
      for (int c0 = 0; c0 < m; c0 += 64) {
        const int c = c0 + lane;
        double acc = 0.0;
        if (c < m) {
          const double* col = zb + start + c;
#pragma unroll 8
          for (int r = wave; r < CT; r += 4) acc = fma(zb[(size_t)r * CT + i], col[(size_t)r * CT], acc);
        }
        part[wave][lane] = acc;
        __syncthreads();
        if (wave == 0 && c < m) dp[c] = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
        __syncthreads();
      }
      n2 = 0.0;
      for (int r = tid; r < CT; r += 256) {
        const double* row = zb + (size_t)r * CT + start;
        double z = zb[(size_t)r * CT + i];
        for (int t = 0; t < m; ++t) z = fma(-dp[t], row[t], z);
        zb[(size_t)r * CT + i] = z;
        n2 = fma(z, z, n2);
      }
      // (its barriers also order the rows' updates before any later read.)  Kahan / Parlett: when
      // the projection kept more than half of ||z||^2 the vector was not nearly in the span, one
      // pass is orthogonal to rounding and the second is skipped
      block_sum2(n2, 0.0, n2, unused);
      if (n2 > 0.5 * nb) break;  // (uniform)
      nb = n2;
    }
    const double sc = 1.0 / sqrt(n2);
    for (int r = tid; r < CT; r += 256) zb[(size_t)r * CT + i] *= sc;
    __syncthreads();
    double s2a = 0.0, s2b = 0.0;
    for (int r = tid; r < CT; r += 256) {
      const double z = zb[(size_t)r * CT + i];
      s2a = fma(ldg(dd + r) * z, z, s2a);
      if (r < CT - 1) s2b = fma(2.0 * ldg(ee + r) * z, zb[(size_t)(r + 1) * CT + i], s2b);
    }
    block_sum2(s2a, s2b, s2a, s2b);
    const double s2 = s2a + s2b;
    if (tid == 0) stg(a.sig2 + (size_t)jb * CT + i, s2 > 0.0 ? s2 : 0.0);
  }
}

// ---- compact WY factors of the reflector blocks: grid (ceil((CT - 1) / 16), nj), 256 threads ----
// Block b holds reflectors k0 = 16 b ... k0 + 15 (row k of the scratch: v_k[row] at k * CT + row,
// rows > k); copied column-major (zeros at rows <= k) for k_gb_back.  S = Y^H Y (16 x 16,
// thread (a, i) one entry), then LAPACK zlarft (forward, columnwise) with one thread per row of T:
// T[a][i] = -tau_i sum_{a <= b < i} T[a][b] S[b][i], T[i][i] = tau_i.  H_k0 ... H_k0+15 = I - Y T Y^H.
template <int CT>
__global__ __launch_bounds__(256) void k_gb_tfac(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.y;
  if (*(const gi32*)(a.status + jb) != 0) return;
  const int k0 = blockIdx.x * 16, nb = min(16, CT - 1 - k0);
  const cplx* Y = a.G + (size_t)jb * a.gstride;  // row k = v_k (entries > k)
  cplx* Yc = a.yc + (size_t)jb * CT * CT;      // column-major copy, zeros at rows <= k
  const cplx* tau = a.tau + (size_t)jb * CT;
  __shared__ cplx S[16][17];
  const int ia = threadIdx.x >> 4, ib = threadIdx.x & 15;
  cplx acc = cmk(0, 0);
  if (ia < nb && ib < nb) {
    const int r0 = k0 + 1 + max(ia, ib);  // both vectors vanish at and above their own index
    for (int row = r0; row < CT; ++row)
      acc = cfmac(ldg(Y + (size_t)(k0 + ia) * CT + row), ldg(Y + (size_t)(k0 + ib) * CT + row), acc);
  }
  S[ia][ib] = acc;
  for (int row = threadIdx.x; row < CT; row += 256) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = k0 + i;
      stg(Yc + (size_t)row * CT + k, (i < nb && row > k) ? ldg(Y + (size_t)k * CT + row) : cmk(0, 0));
    }
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int ar = threadIdx.x;
    cplx T[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const cplx ti = i < nb ? ldg(tau + k0 + i) : cmk(0, 0);
      cplx v = cmk(0, 0);
      if (i == ar) v = ti;
      else if (i > ar) {
        cplx sm = cmk(0, 0);
#pragma unroll
        for (int b = 0; b < 16; ++b)
          if (b >= ar && b < i) sm = cfma(T[b], S[b][i], sm);
        v = cscale(cmul(ti, sm), -1.0);
      }
      T[i] = v;
    }
    cplx* To = a.tfac + ((size_t)jb * (CT / 16) + blockIdx.x) * 256 + ar * 16;
#pragma unroll
    for (int i = 0; i < 16; ++i) stg(To + i, T[i]);
  }
}

// ---- V = Q Z on the matrix cores, output: grid (ceil(K / 16), nj), 256 threads ----
// A workgroup owns 16 columns of V (C x 16, in the MFMA accumulator layout: wave w holds the row
// tiles w, w + 4, ... -- cyclic, so the zero rows above each block are skipped evenly); per block
// of 16 reflectors from the last: W1 = Y^H V (per wave over its rows, the four partials summed in
// the LDS), W2 = T W1, V -= Y W2.  Y's operands straight from the (L2-resident) scratch: a block's
// rows are contiguous in the column-major reflector store.  Output W = V Sigma, sig, qr = 1.
template <int CT, int NW = (CT / 64 > 4 ? CT / 64 : 4)>
__global__ __launch_bounds__(64 * NW) void k_gb_back(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0, int nr) {
  constexpr int NT = CT / (16 * NW);  // row tiles per wave
  int jr, bx;
  if (!xcd_job_block(nr, jr, bx)) return;  // (a job's column groups on one XCD: they share Y)
  const int jb = job0 + jr;
  if (*(const gi32*)(a.status + jb) != 0) return;
  TwoSiteJob& j = const_cast<TwoSiteJob&>(jobs[jb]);
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  K = kept_count(a, jb);
  const int col0 = bx * 16;
  if (bx == 0 && threadIdx.x == 0) stg(j.sig + kSigTail, ldg(a.tail + jb));  // (rank_body)
  if (col0 >= K) return;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lk = lane >> 4;
  const double* zb = a.z + (size_t)jb * CT * CT;
  // reflector v_kk at row (kk < CT - 1, rows > kk; column-major store), through a buffer resource
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.yc + (size_t)jb * CT * CT, (unsigned)(CT * CT * 16));
  auto yld = [&](int row, int kk) -> cplx {
    const cplx v = buf_ld(ry, (unsigned)(row * CT + kk) * 16u, 0u);
    return (row > kk && kk < CT - 1) ? v : cmk(0, 0);
  };
  const cplx* Tf = a.tfac + (size_t)jb * (CT / 16) * 256;
  __shared__ cplx Pw[NW][16][16];
  __shared__ cplx W1[16][17], W2[16][17], Tl[16][17];
  d4_t vre[NT], vim[NT];
  const int col = col0 + li;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int rt = w + NW * t;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * rt + lk + 4 * q;
      vre[t][q] = col < K ? ldg(zb + (size_t)row * CT + col) : 0.0;
      vim[t][q] = 0.0;
    }
  }
  for (int blk = (CT - 2) / 16; blk >= 0; --blk) {
    const int k0 = 16 * blk;
    if (tid < 256) Tl[tid >> 4][tid & 15] = ldg(Tf + (size_t)blk * 256 + tid);  // (>= 256 threads)
    // W1 partial = Y^H V over this wave's rows: A[m = i][k = row] = conj(Y[row][k0 + i])
    d4_t wr = {0, 0, 0, 0}, wi = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int rt = w + NW * t;
      if (16 * rt + 15 > k0) {  // rows <= k0 of the block vanish (uniform per wave)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int row = 16 * rt + 4 * s4 + lk, kk = k0 + li;
          const cplx y = yld(row, kk);
          wr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, vre[t][s4], wr, 0, 0, 0);
          wr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, vim[t][s4], wr, 0, 0, 0);
          wi = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, vim[t][s4], wi, 0, 0, 0);
          wi = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, vre[t][s4], wi, 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) Pw[w][lk + 4 * q][li] = cmk(wr[q], wi[q]);
    __syncthreads();
    if (tid < 256) {
      const int b = tid >> 4, c = tid & 15;
      cplx acc = Pw[0][b][c];
#pragma unroll
      for (int ww = 1; ww < NW; ++ww) acc = cadd(acc, Pw[ww][b][c]);
      W1[b][c] = acc;
    }
    __syncthreads();
    if (tid < 256) {
      const int i = tid >> 4, c = tid & 15;
      cplx acc = cmk(0, 0);
#pragma unroll
      for (int b = 0; b < 16; ++b)
        if (b >= i) acc = cfma(Tl[i][b], W1[b][c], acc);
      W2[i][c] = acc;
    }
    __syncthreads();
    // V -= Y W2: A[m = row][k = i] = Y[row][k0 + i], B[k = i][n = c] = W2[i][c]
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int rt = w + NW * t;
      if (16 * rt + 15 > k0) {
        const int row = 16 * rt + li;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const int kk = k0 + 4 * s4 + lk;
          const cplx y = yld(row, kk);
          const cplx ww = W2[4 * s4 + lk][li];
          vre[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.x, ww.x, vre[t], 0, 0, 0);
          vre[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, ww.y, vre[t], 0, 0, 0);
          vim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.x, ww.y, vim[t], 0, 0, 0);
          vim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, ww.x, vim[t], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // Tl, Pw, W1, W2 are overwritten next block
  }
  if (col < K) {
    const double sg = sqrt(ldg(a.sig2 + (size_t)jb * CT + col));
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int rt = w + NW * t;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * rt + lk + 4 * q;
        if (row < C) stg(j.work + (size_t)col * C + row, cmk(vre[t][q] * sg, vim[t][q] * sg));
      }
    }
    if (w == 0 && lk == 0) stg(j.sig + col, sg);
  }
  for (int c = col0 + tid; c < min(C, col0 + 16); c += 64 * NW)
    if (c >= K) stg(j.sig + c, 0.0);
  if (bx == 0)
    for (int c = ((K + 15) / 16) * 16 + tid; c < C; c += 64 * NW) stg(j.sig + c, 0.0);
  if (bx == 0 && tid == 0) {
    if (jb == 0) atomicAdd(&g_gbig_ticks[6], __builtin_amdgcn_s_memtime() - t_start);
    j.qr = 1;
    atomicMax(&j.flags[2], 1);
    atomicAdd(&g_gbig_stats[1], 1ull);
  }
}

// ---- the certificate of a rank-deficient decision (aqc::gram_keep's cert): every dropped sigma^2 is
// at most ||X - X V V^H||_F^2 (V the K kept right vectors, W / sigma from k_gb_back), computed from X
// itself -- so to eps ||X|| in sigma, where G's eigenvalues carry eps ||G||.  Below CHOP / 2 the
// open-CHOP values were all chopped, as LAPACK's sigma^2 ~ (eps sigma_1)^2 are in Aer; otherwise the
// job declines (status 4: the block Jacobi decides).  Y = X V into the (dead) G scratch (kGLong CT x CT
// per job: X has L <= kGLong CT rows), then R = X - Y V^H tile by tile with the squares summed per job;
// grid (kGLong CT / 64, CT / 64, nj).
template <int CT>
__device__ __forceinline__ cplx xval(const TwoSiteJob& j, bool tr, int M, int R, int c) {
  return tr ? cconj(ldg(j.theta + (size_t)R * M + c)) : ldg(j.theta + (size_t)c * M + R);
}

template <int CT>
__global__ __launch_bounds__(256) void k_gb_cert_y(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.z;
  if (*(const gi32*)(a.status + jb) != 0 || !*(const gi32*)(a.cert + jb)) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  K = kept_count(a, jb);
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  if (r0 >= L || c0 >= K) return;
  __shared__ GemmLds lds;
  cplx* Y = a.G + (size_t)jb * a.gstride;  // Y[R][kk] at R * CT + kk
  const double* sg = j.sig;
  block_cgemm(
      min(64, L - r0), min(64, K - c0), C, [&](int i, int c) { return xval<CT>(j, tr, M, r0 + i, c); },
      [&](int c, int kk) { return cscale(ldg(j.work + (size_t)(c0 + kk) * C + c), 1.0 / ldg(sg + c0 + kk)); },
      [&](int i, int kk, cplx v) { stg(Y + (size_t)(r0 + i) * CT + c0 + kk, v); }, lds);
}

template <int CT>
__global__ __launch_bounds__(256) void k_gb_cert_r(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.z;
  if (*(const gi32*)(a.status + jb) != 0 || !*(const gi32*)(a.cert + jb)) return;
  const TwoSiteJob& j = jobs[jb];
  int M, L, C, K;
  bool tr;
  job_dims(j, M, L, C, tr, K);
  K = kept_count(a, jb);
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  if (r0 >= L || c0 >= C) return;
  __shared__ GemmLds lds;
  __shared__ double red[256];
  const cplx* Y = a.G + (size_t)jb * a.gstride;
  const double* sg = j.sig;
  double acc = 0.0;
  block_cgemm(
      min(64, L - r0), min(64, C - c0), K, [&](int i, int kk) { return ldg(Y + (size_t)(r0 + i) * CT + kk); },
      [&](int kk, int c) { return cconj(cscale(ldg(j.work + (size_t)kk * C + c0 + c), 1.0 / ldg(sg + kk))); },
      [&](int i, int c, cplx v) { acc += cnorm2(csub(xval<CT>(j, tr, M, r0 + i, c0 + c), v)); }, lds);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(a.certsum + jb, red[0]);
}

// grid (nj): decline the jobs whose certificate fails (their W / sig were written by k_gb_back: the
// Jacobi contract is restored -- qr = 0, no handed-over tail -- before the host re-runs them)
template <int CT>
__global__ __launch_bounds__(64) void k_gb_cert_end(const TwoSiteJob* __restrict__ jobs, GBArgs a, int job0) {
  const int jb = job0 + (int)blockIdx.x;
  if (threadIdx.x != 0 || *(const gi32*)(a.status + jb) != 0 || !*(const gi32*)(a.cert + jb)) return;
  TwoSiteJob& j = const_cast<TwoSiteJob&>(jobs[jb]);
  const double r2 = __hip_atomic_load((const gdbl*)(a.certsum + jb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (r2 < 0.5 * kReduceChop) {
    atomicAdd(&g_gbig_stats[6], 1ull);
    return;
  }
  *(gi32*)(a.status + jb) = 4;
  j.qr = 0;
  stg(j.sig + kSigTail, 0.0);
  atomicAdd(&g_gbig_stats[7], 1ull);
  atomicAdd(&g_gbig_stats[1], ~0ull);  // (k_gb_back counted it as taken)
}

struct GBBuffers {
  int ct = 0, nj = 0;
  cplx* G = nullptr;
  double *d = nullptr, *e = nullptr, *z = nullptr, *dinv = nullptr, *sig2 = nullptr, *lam = nullptr, *tn = nullptr;
  double *err = nullptr, *tail = nullptr, *certsum = nullptr;
  int *kept = nullptr, *cert = nullptr;
  cplx* tau = nullptr;
  cplx* tfac = nullptr;
  cplx* yc = nullptr;
  cplx* xch = nullptr;
  unsigned* cnt = nullptr;
  int* status = nullptr;
  int* host_status = nullptr;
  TwoSiteJob* djobs = nullptr;  // declined jobs for the block Jacobi
  TwoSiteJob* hjobs = nullptr;  // pinned
};

void gb_free(GBBuffers& b) {
  hipFree(b.G), hipFree(b.d), hipFree(b.e), hipFree(b.z), hipFree(b.dinv), hipFree(b.sig2), hipFree(b.tau);
  hipFree(b.lam), hipFree(b.tn), hipFree(b.tfac), hipFree(b.yc);
  hipFree(b.err), hipFree(b.tail), hipFree(b.kept), hipFree(b.cert), hipFree(b.certsum);
  hipFree(b.xch), hipFree(b.cnt), hipFree(b.status), hipFree(b.djobs);
  hipHostFree(b.host_status), hipHostFree(b.hjobs);
  b = GBBuffers();
}

GBBuffers g_gb_buffers;
void release_gb_buffers() { gb_free(g_gb_buffers); }
GBBuffers& gb_buffers() {
  aqc::on_finalize(release_gb_buffers);
  return g_gb_buffers;
}

int gb_ensure(GBBuffers& b, int ct, int nj, hipStream_t st) {
  if (b.ct >= ct && b.nj >= nj) return AQC_OK;
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  const int c = std::max(ct, b.ct), n = std::max(nj, b.nj);
  gb_free(b);
  const size_t cc = (size_t)c * c * n;
  AQC_HIP_CHECK(hipMalloc(&b.G, (c >= 1024 ? 2 : 1) * cc * sizeof(cplx)));  // (kGLong)
  AQC_HIP_CHECK(hipMalloc(&b.z, cc * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.dinv, cc * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.d, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.e, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.sig2, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.lam, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.tn, (size_t)n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.err, (size_t)c * n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.tail, (size_t)n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.kept, (size_t)n * sizeof(int)));
  AQC_HIP_CHECK(hipMalloc(&b.cert, (size_t)n * sizeof(int)));
  AQC_HIP_CHECK(hipMalloc(&b.certsum, (size_t)n * sizeof(double)));
  AQC_HIP_CHECK(hipMalloc(&b.tfac, (size_t)(c / 16) * 256 * n * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.yc, cc * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.tau, (size_t)c * n * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.xch, (size_t)8 * c * n * sizeof(cplx)));
  AQC_HIP_CHECK(hipMalloc(&b.cnt, (size_t)32 * n * sizeof(unsigned)));
  AQC_HIP_CHECK(hipMalloc(&b.status, (size_t)n * sizeof(int)));
  AQC_HIP_CHECK(hipMalloc(&b.djobs, (size_t)n * sizeof(TwoSiteJob)));
  AQC_HIP_CHECK(hipHostMalloc(&b.host_status, (size_t)n * sizeof(int)));
  AQC_HIP_CHECK(hipHostMalloc(&b.hjobs, (size_t)n * sizeof(TwoSiteJob)));
  b.ct = c, b.nj = n;
  return AQC_OK;
}

// The side stream and the round events: created on first use, released (after aqc_finalize's
// device synchronisation) by release_gb_sync -- at exit the side stream's post kernels are ordered
// only by these events, so they must be drained before the runtime tears down.
hipStream_t g_gb_side[64] = {nullptr};
hipStream_t g_gb_side2[64] = {nullptr};  // the compact-WY factors beside the eigenpairs
std::vector<hipEvent_t> g_gb_events;
void release_gb_sync() {
  for (auto& s : g_gb_side)
    if (s) (void)hipStreamDestroy(s), s = nullptr;
  for (auto& s : g_gb_side2)
    if (s) (void)hipStreamDestroy(s), s = nullptr;
  for (hipEvent_t e : g_gb_events) (void)hipEventDestroy(e);
  g_gb_events.clear();
}

hipStream_t gb_side_stream(int which = 0) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipStream_t* tab = which ? g_gb_side2 : g_gb_side;
  if (!tab[dev]) {
    (void)hipStreamCreateWithFlags(&tab[dev], hipStreamNonBlocking);
    aqc::on_finalize(release_gb_sync);
  }
  return tab[dev];
}

hipEvent_t gb_event(int i) {  // (per process; the library stream orders their reuse)
  aqc::on_finalize(release_gb_sync);
  while ((int)g_gb_events.size() <= i) {
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    g_gb_events.push_back(e);
  }
  return g_gb_events[i];
}


template <int CT>
int run_gram_big(const TwoSiteJob* hjobs, const TwoSiteJob* jobs, int nj, int cap_max, hipStream_t st) {
  GBBuffers& b = gb_buffers();
  int rc = gb_ensure(b, CT, nj, st);
  if (rc != AQC_OK) return rc;
  GBArgs a;
  a.G = b.G, a.d = b.d, a.e = b.e, a.tau = b.tau, a.z = b.z, a.dinv = b.dinv, a.sig2 = b.sig2;
  a.gstride = (size_t)kGLong<CT> * CT * CT;
  a.lam = b.lam, a.tn = b.tn, a.tfac = b.tfac, a.yc = b.yc;
  a.err = b.err, a.kept = b.kept, a.tail = b.tail, a.cert = b.cert, a.certsum = b.certsum;
  a.xch = b.xch, a.cnt = b.cnt, a.status = b.status;
  a.spin = g_gb_spin;
  if (g_gb_tail < 0) {
    const char* e = std::getenv("AQC_GB_TAIL");
    g_gb_tail = (e && std::strcmp(e, "0") == 0) ? 0 : 1;
  }
  AQC_HIP_CHECK(hipMemsetAsync(b.cnt, 0, (size_t)32 * nj * sizeof(unsigned), st));
  hipLaunchKernelGGL((k_gb_gram<CT>), dim3(xcd_grid((CT / 64) * (CT / 64 + 1) / 2, nj)), dim3(256), 0, st, jobs, a, nj);
  AQC_CHECK_LAUNCH();
  // the tridiagonalisation's workgroups of a job must all be resident together (they exchange a
  // vector per column): rounds of at most min(240, resident capacity) workgroups, whole jobs each.
  // (One workgroup per CU: the 1024-thread workgroup holds 16 complex of G per thread in 128 VGPRs,
  // the whole register file at four waves per SIMD; a job's G is 4 MB at C = 512 against 512 KB of
  // registers per CU, so 24 config-5 jobs cannot be resident at once whatever the split.)
  constexpr int P = CT * CT / 16384;
  static int resident = -1;
  if (resident < 0) {
    int dev = 0, ncu = 0, per_cu = 0;
    AQC_HIP_CHECK(hipGetDevice(&dev));
    AQC_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    AQC_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)k_gb_tridiag<CT, 1, true>, 1024, 0));
    resident = ncu * std::min(per_cu, 1);
  }
  if (g_gb_stages < 0) {
    const char* e = std::getenv("AQC_GB_STAGES");
    g_gb_stages = (e && std::strcmp(e, "1") == 0) ? 1 : 2;
  }
  constexpr bool kCan2 = CT == 512;
  const bool two = kCan2 && g_gb_tail && g_gb_stages == 2;
  // (two stages: a round's first stage runs beside the previous round's second, P + P / 4
  // workgroups per job resident together)
  const int per_round = std::min(240, resident) / (two ? P + P / 4 : P);
  // the eigenpairs and back-transformation of a round's jobs run on a second stream, beside the next
  // round's tridiagonalisation (which leaves CUs free: 9 of 24 config-5 jobs hold 144 of 256)
  hipStream_t s2 = gb_side_stream();
  // the compact-WY factors need only the reflectors: on a third stream beside the eigenvalues,
  // inverse iteration and Gram-Schmidt (which need only T), joined before the back-transformation
  hipStream_t s3 = gb_side_stream(1);
  int evi = 0;  // events of this call, in order (gb_event: per process, reused call to call)
  auto post = [&](hipStream_t ps, int j0, int nr) -> int {
    if (s3 != ps) {
      hipEvent_t e0 = gb_event(evi++);
      AQC_HIP_CHECK(hipEventRecord(e0, ps));
      AQC_HIP_CHECK(hipStreamWaitEvent(s3, e0, 0));
    }
    hipLaunchKernelGGL((k_gb_tfac<CT>), dim3((CT - 1 + 15) / 16, nr), dim3(256), 0, s3, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_eig<CT>), dim3(CT / 64, nr), dim3(256), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_keep<CT>), dim3(nr), dim3(64), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_inv<CT>), dim3(CT / 64, nr), dim3(64), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_gs<CT>), dim3(nr), dim3(256), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    if (s3 != ps) {
      hipEvent_t e1 = gb_event(evi++);
      AQC_HIP_CHECK(hipEventRecord(e1, s3));
      AQC_HIP_CHECK(hipStreamWaitEvent(ps, e1, 0));
    }
    hipLaunchKernelGGL((k_gb_back<CT>), dim3(xcd_grid(CT / 16, nr)), dim3(CT / 64 > 4 ? CT : 256), 0, ps, jobs, a, j0, nr);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_cert_y<CT>), dim3(kGLong<CT> * CT / 64, CT / 64, nr), dim3(256), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_cert_r<CT>), dim3(kGLong<CT> * CT / 64, CT / 64, nr), dim3(256), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_gb_cert_end<CT>), dim3(nr), dim3(64), 0, ps, jobs, a, j0);
    AQC_CHECK_LAUNCH();
    return AQC_OK;
  };
  if (per_round < 1) {  // cannot hold one job's workgroups at once: every job declines
    AQC_HIP_CHECK(hipMemsetAsync(b.status, 0x7f, (size_t)nj * sizeof(int), st));
    rc = post(st, 0, nj);
    if (rc != AQC_OK) return rc;
  } else {
    // 2 chi = 512 with the tail: two exchange stages (k_gb_tridiag's comment); a round's second
    // stage and tail on s2, its compact-WY factors, eigenpairs and back-transformation on s3, so
    // that the next round's second stage does not queue behind them.  (Three streams, not four: a
    // process has four hardware queues by default, and with a fourth stream here the schedule's
    // streams shared queues with the caller's -- config 5 after config 2's four evaluation streams
    // ran 0.367 ms per gate against 0.293 alone; on three streams 0.290 both ways,
    // profiles/r5_cfg5_streams.json.)
    hipStream_t s4 = two ? s3 : s2;
    for (int j0 = 0; j0 < nj; j0 += per_round) {
      const int nr = std::min(per_round, nj - j0);
      if (two)
        hipLaunchKernelGGL((k_gb_tridiag<CT, 1, true, CT, (kCan2 ? CT / 2 : 128)>), dim3(P * nr), dim3(1024), 0, st, jobs, a, j0);
      else if (g_gb_tail)
        hipLaunchKernelGGL((k_gb_tridiag<CT, 1, true>), dim3(P * nr), dim3(1024), 0, st, jobs, a, j0);
      else
        hipLaunchKernelGGL((k_gb_tridiag<CT, 1, false>), dim3(P * nr), dim3(1024), 0, st, jobs, a, j0);
      AQC_CHECK_LAUNCH();
      hipEvent_t ev = gb_event(evi++);
      AQC_HIP_CHECK(hipEventRecord(ev, st));
      AQC_HIP_CHECK(hipStreamWaitEvent(s2, ev, 0));
      if (two) {
        constexpr int CH = kCan2 ? CT / 2 : CT;
        hipLaunchKernelGGL((k_gb_tridiag<CH, 1, true, CT, 128>), dim3(CH * CH / 16384 * nr), dim3(1024), 0, s2, jobs, a, j0);
        AQC_CHECK_LAUNCH();
      }
      if (g_gb_tail) {
        hipLaunchKernelGGL((k_gb_tail<CT>), dim3(nr), dim3(1024), 0, s2, jobs, a, j0);
        AQC_CHECK_LAUNCH();
      }
      if (two) {
        hipEvent_t e2 = gb_event(evi++);
        AQC_HIP_CHECK(hipEventRecord(e2, s2));
        AQC_HIP_CHECK(hipStreamWaitEvent(s4, e2, 0));
      }
      rc = post(s4, j0, nr);
      if (rc != AQC_OK) return rc;
    }
    hipEvent_t done = gb_event(evi++);
    AQC_HIP_CHECK(hipEventRecord(done, s4));
    AQC_HIP_CHECK(hipStreamWaitEvent(st, done, 0));
  }
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
  if (!g_gram_big || side > 2048) return block_jacobi(jobs, nj, cap_max, st);
  // chunks of at most 1.5 GB of per-job scratch (G, the two inverse-iteration arrays and the
  // column-major reflectors: 64 C^2 bytes per job), so that a large batch does not hold it all
  const int ct = side <= 256 ? 256 : side <= 512 ? 512 : 1024;
  const int chunk = std::max(1, (int)(((size_t)1536 << 20) / ((size_t)80 * ct * ct)));
  for (int j0 = 0; j0 < nj; j0 += chunk) {
    const int n = std::min(chunk, nj - j0);
    int rc;
    if (ct == 256) rc = run_gram_big<256>(hjobs + j0, jobs + j0, n, cap_max, st);
    else if (ct == 512) rc = run_gram_big<512>(hjobs + j0, jobs + j0, n, cap_max, st);
    else rc = run_gram_big<1024>(hjobs + j0, jobs + j0, n, cap_max, st);
    if (rc != AQC_OK) return rc;
  }
  return AQC_OK;
}

}  // namespace aqc

extern "C" int aqc_svd_gram_big_ticks(double* out) {
  AQC_REQUIRE(out, "aqc_svd_gram_big_ticks: null argument");
  unsigned long long t[9];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(aqc::g_gbig_ticks), sizeof(t)));
  for (int i = 0; i < 9; ++i) out[i] = (double)t[i];
  unsigned long long z[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(aqc::g_gbig_ticks), z, sizeof(z)));
  return AQC_OK;
}

extern "C" int aqc_svd_gram_big_stats(double* out) {
  AQC_REQUIRE(out, "aqc_svd_gram_big_stats: null argument");
  unsigned long long t[8];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(aqc::g_gbig_stats), sizeof(t)));
  for (int i = 0; i < 8; ++i) out[i] = (double)t[i];
  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(aqc::g_gbig_stats), z, sizeof(z)));
  return AQC_OK;
}

/* Counter-wait limit of the multi-workgroup tridiagonalisation, in microseconds (< 0: the default,
   100 ms).  A workgroup that waits longer for the rest of its job declines the job (status 3), which
   then runs the block Jacobi.  0 makes any wait that is not already satisfied a timeout: the tests
   use it to exercise the decline path. */
extern "C" int aqc_gb_set_spin_limit(double us) {
  aqc::g_gb_spin = us < 0 ? aqc::kSpinTicks : (unsigned long long)(us * 100.0);
  return AQC_OK;
}

/* The multi-workgroup tridiagonalisation's last 128 columns in one workgroup (1, the default) or
   over all of the job's workgroups to the end (0). */
extern "C" int aqc_gb_set_tail(int on) {
  AQC_REQUIRE(on == 0 || on == 1, "aqc_gb_set_tail: on must be 0 or 1");
  aqc::g_gb_tail = on;
  return AQC_OK;
}

/* 2 chi = 512 with the tail: the exchange in two stages (2, the default) or one (1). */
extern "C" int aqc_gb_set_stages(int n) {
  AQC_REQUIRE(n == 1 || n == 2, "aqc_gb_set_stages: n must be 1 or 2");
  aqc::g_gb_stages = n;
  return AQC_OK;
}
