// MPS engine: replaces qiskit-aer's matrix_product_state simulator as driven by
// adaptaqc/backends/aer_mps_backend.py:27-93 and the aqc_research.mps_operations measurements.
//
// Gate application follows Aer's algorithm (see oracle/mps.py for the restatement):
//   * 1-qubit gates act on the Gamma of the qubit's current site (here deferred and folded into
//     the next two-site update on that qubit, which is exact: truncation commutes with a local
//     unitary on either side of the cut);
//   * 2-qubit gates use "swap-left" routing with a lazily kept qubit permutation (host side);
//   * every two-site update = contract theta (k_theta), one-sided Jacobi SVD (k_jacobi),
//     reduce_zeros truncation + renormalisation (k_rank), and the lambda-divided split into the
//     two new Gammas (k_split_copy, k_split_gemm).
// Independent states advance in lock-step: one launch of each kernel serves one two-site
// update of every state in the batch (blockIdx.y / blockIdx.x = job).
#include <algorithm>
#include <cmath>
#include <chrono>
#include <cstring>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <unordered_set>

#include "aqc_gemm.h"
#include "mps_internal.h"

using aqc::cplx;

namespace aqc {

namespace {
std::mutex g_mps_stream_mu;
hipStream_t g_mps_streams[64] = {nullptr};
void release_mps_streams() {
  std::lock_guard<std::mutex> lk(g_mps_stream_mu);
  for (auto& s : g_mps_streams)
    if (s) (void)hipStreamDestroy(s), s = nullptr;
}
}  // namespace

hipStream_t mps_stream() {
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_mps_stream_mu);
  if (!g_mps_streams[dev]) {
    hipStreamCreateWithFlags(&g_mps_streams[dev], hipStreamNonBlocking);
    note_device(dev);
    on_finalize(release_mps_streams);
  }
  return g_mps_streams[dev];
}

// device dev's MPS stream if it exists (nullptr after aqc_finalize released it, or before first use)
hipStream_t mps_stream_if_any(int dev) {
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_mps_stream_mu);
  return g_mps_streams[dev];
}

}  // namespace aqc

namespace {

// threadIdx.x read through an empty asm: values a phase derives from it cannot be hoisted out of
// the chain loop in k_chain (where they would stay live across every other phase)
__device__ __forceinline__ int fresh_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

constexpr int kT = 256;
constexpr double kChop = 1e-16;
constexpr int kMaxSweeps = 60;
// rotation threshold: |a^H b| > tol_factor * L * eps * |a| |b|  (L = column length)
double g_jacobi_tol_factor = 1.0;
// Sweep stop of the register Jacobi: after a sweep whose counted rotations all had |t| <= this,
// the remaining off-diagonal is O(t^2) (quadratic convergence) and no further sweep is run.
constexpr double kDefaultTinyT = 1e-6;
double g_jacobi_tiny_t = kDefaultTinyT;
// dot-product noise floor of the Jacobi rotations, in units of eps ||W|| (|a| + |b|): off (a
// floor costs graded matrices their small singular vectors)
constexpr double kJacobiNoise = 0.0;
// Fused per-state chain (k_chain) for batches of >= g_chain_min_states states at 2 chi = 128
// (aqc_mps_set_fused_chain: 0 off, 1 from 32 states, 2 from one state).
bool g_fused_chain = true;
int g_chain_min_states = 32;
// dynamic LDS of the 1024-thread two-site kernels: four 64 x 64 GEMM tiles (>= the register
// Jacobi's 64 x 129 complex exchange buffer)
constexpr int kChainLdsBytes = 4 * (int)sizeof(aqc::GemmLds);

struct OneSiteJob {
  cplx* g;
  const int* dims;  // &dims[p]
  int cap;
  int pad;
  cplx u[4];
};

using aqc::TwoSiteJob;
using aqc::kMaxCap;
using aqc::kSigMax;
using aqc::kSigTail;
using aqc::kSigLen;

// ------------------------------------------------------------------------------------------
__global__ void k_mps_zero(cplx* gam, double* lam, int* dims, int n, int cap) {
  const size_t ss = (size_t)2 * cap * cap;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    gam[(size_t)i * ss] = aqc::cmk(1.0, 0.0);
  }
  for (int b = blockIdx.x * blockDim.x + threadIdx.x; b <= n; b += gridDim.x * blockDim.x) {
    lam[(size_t)b * cap] = 1.0;
    dims[b] = 1;
  }
}

__global__ __launch_bounds__(kT) void k_1q(const OneSiteJob* __restrict__ jobs) {
  const OneSiteJob& j = jobs[blockIdx.y];
  const int cl = j.dims[0], cr = j.dims[1];
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  for (int e = blockIdx.x * kT + threadIdx.x; e < cl * cr; e += gridDim.x * kT) {
    const int l = e / cr, r = e % cr;
    const size_t o = (size_t)l * cap + r;
    const cplx a0 = aqc::ldg(j.g + o), a1 = aqc::ldg(j.g + half + o);  // GLOBAL, not FLAT
    aqc::stg(j.g + o, aqc::cfma(j.u[1], a1, aqc::cmul(j.u[0], a0)));
    aqc::stg(j.g + half + o, aqc::cfma(j.u[3], a1, aqc::cmul(j.u[2], a0)));
  }
}

// theta[(s2*chr + r)*M + s1*chl + l] = sum_in G[out][in] * P_in[l][r],
// P_{s1' s2'}[l][r] = sum_m ll[l] Gp[s1'][l][m] lm[m] Gq[s2'][m][r] lr[r].
__global__ __launch_bounds__(kT) void k_theta(const TwoSiteJob* __restrict__ jobs, int nj) {
  int jb, tile;
  if (!aqc::xcd_job_block(nj, jb, tile)) return;  // (a job's tiles on one XCD: they share panels)
  const TwoSiteJob& j = jobs[jb];
  const int chl = j.dims[0], chm = j.dims[1], chr = j.dims[2];
  const int cap = j.cap;
  // (16 x 16 tiles, one position per thread: the small batches -- a single state's update at
  // capacity 64 is 16 workgroups here, 4 in k_theta32)
  const int tiles_r = (cap + 15) / 16;
  const int l0 = (tile / tiles_r) * 16, r0 = (tile % tiles_r) * 16;
  if (l0 >= chl || r0 >= chr) return;
  __shared__ cplx As[2][16][17];
  __shared__ cplx Bs[2][16][17];
  const int ty = threadIdx.x / 16, tx = threadIdx.x % 16;
  const int l = l0 + ty, r = r0 + tx;
  const size_t half = (size_t)cap * cap;
  cplx acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = aqc::cmk(0, 0);
  const double lll = l < chl ? j.ll[l] : 0.0;
  const double lrr = r < chr ? j.lr[r] : 0.0;
  for (int m0 = 0; m0 < chm; m0 += 16) {
    const int ma = m0 + tx, mb = m0 + ty;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      cplx a = aqc::cmk(0, 0), b = aqc::cmk(0, 0);
      if (l < chl && ma < chm) a = aqc::cscale(j.gp[s * half + (size_t)l * cap + ma], lll * j.lm[ma]);
      if (mb < chm && r < chr) b = aqc::cscale(j.gq[s * half + (size_t)mb * cap + r], lrr);
      As[s][ty][tx] = a;
      Bs[s][ty][tx] = b;
    }
    __syncthreads();
#pragma unroll 4
    for (int mm = 0; mm < 16; ++mm) {
      const cplx a0 = As[0][ty][mm], a1 = As[1][ty][mm];
      const cplx b0 = Bs[0][mm][tx], b1 = Bs[1][mm][tx];
      acc[0] = aqc::cfma(a0, b0, acc[0]);
      acc[1] = aqc::cfma(a0, b1, acc[1]);
      acc[2] = aqc::cfma(a1, b0, acc[2]);
      acc[3] = aqc::cfma(a1, b1, acc[3]);
    }
    __syncthreads();
  }
  if (l < chl && r < chr) {
    const int M = 2 * chl;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      cplx v = aqc::cmul(j.G[o * 4 + 0], acc[0]);
      v = aqc::cfma(j.G[o * 4 + 1], acc[1], v);
      v = aqc::cfma(j.G[o * 4 + 2], acc[2], v);
      v = aqc::cfma(j.G[o * 4 + 3], acc[3], v);
      const int s1 = o >> 1, s2 = o & 1;
      j.theta[(size_t)(s2 * chr + r) * M + s1 * chl + l] = v;
    }
  }
}

// The same with 32 x 32 tiles (the batches that fill the GPU with them: config 5's waves):
__global__ __launch_bounds__(kT) void k_theta32(const TwoSiteJob* __restrict__ jobs, int nj) {
  int jb, tile;
  if (!aqc::xcd_job_block(nj, jb, tile)) return;  // (a job's tiles on one XCD: they share panels)
  const TwoSiteJob& j = jobs[jb];
  const int chl = j.dims[0], chm = j.dims[1], chr = j.dims[2];
  const int cap = j.cap;
  // 32 x 32 output tiles, each thread 2 x 2 (l, r) positions x the four (s1, s2) products: per
  // 16-deep m step 8 LDS operand reads for 16 complex FMAs (16 x 16 tiles with one position per
  // thread read 4 for 4: the LDS port, not the FP64 rate, bounded them)
  const int tiles_r = (cap + 31) / 32;
  const int l0 = (tile / tiles_r) * 32, r0 = (tile % tiles_r) * 32;
  if (l0 >= chl || r0 >= chr) return;
  __shared__ cplx As[2][32][17];
  __shared__ cplx Bs[2][16][33];
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
  const size_t half = (size_t)cap * cap;
  cplx acc[2][2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int o = 0; o < 4; ++o) acc[i][jj][o] = aqc::cmk(0, 0);
  for (int m0 = 0; m0 < chm; m0 += 16) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + kT * q;
      {  // As[s][li][mm] = ll[l] Gp[s][l][m] lm[m]: consecutive threads along m
        const int s = e >> 9, li = (e >> 4) & 31, mm = e & 15, l = l0 + li, m = m0 + mm;
        As[s][li][mm] = (l < chl && m < chm) ? aqc::cscale(j.gp[s * half + (size_t)l * cap + m], j.ll[l] * j.lm[m])
                                             : aqc::cmk(0, 0);
      }
      {  // Bs[s][mm][ri] = Gq[s][m][r] lr[r]: consecutive threads along r
        const int s = e >> 9, mm = (e >> 5) & 15, ri = e & 31, m = m0 + mm, r = r0 + ri;
        Bs[s][mm][ri] = (m < chm && r < chr) ? aqc::cscale(j.gq[s * half + (size_t)m * cap + r], j.lr[r]) : aqc::cmk(0, 0);
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int mm = 0; mm < 16; ++mm) {
      cplx a[2][2], b[2][2];  // [s][i] / [s][jj]
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 2; ++i) a[s2][i] = As[s2][ty + 16 * i][mm], b[s2][i] = Bs[s2][mm][tx + 16 * i];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int o = 0; o < 4; ++o) acc[i][jj][o] = aqc::cfma(a[o >> 1][i], b[o & 1][jj], acc[i][jj][o]);
    }
    __syncthreads();
  }
  const int M = 2 * chl;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int l = l0 + ty + 16 * i, r = r0 + tx + 16 * jj;
      if (l < chl && r < chr) {
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          cplx v = aqc::cmul(j.G[o * 4 + 0], acc[i][jj][0]);
          v = aqc::cfma(j.G[o * 4 + 1], acc[i][jj][1], v);
          v = aqc::cfma(j.G[o * 4 + 2], acc[i][jj][2], v);
          v = aqc::cfma(j.G[o * 4 + 3], acc[i][jj][3], v);
          const int s1 = o >> 1, s2 = o & 1;
          j.theta[(size_t)(s2 * chr + r) * M + s1 * chl + l] = v;
        }
      }
    }
}

// ---- register-resident one-sided Jacobi (2*chi <= 128) ----------------------------------
// Every column of W stays in VGPRs for the whole decomposition.  CP/2 groups of 16 lanes; group
// g holds two columns ("S" and "M"), lane l holds rows l, l+16, ... (MAXR rows).  One sweep uses
// recursive halving: level 0 pairs every S with every M (CP/2 rounds; after each round the M
// columns shift by one group inside the sub-block), then each sub-block splits into its S half
// and its M half (one swap exchange) and the same is done inside both halves, down to single
// groups -- CP-1 rounds per sweep, every round a perfect matching, and only the M half of the
// columns crosses LDS per round.  Columns travel between groups, so each carries its id; it is
// written back to its own slot (slots >= C hold zero padding columns that are never written).
//
// Preconditioning (j.qr, Drmac-Veselic): W P = Q R by Householder QR with column pivoting, done
// in the same register layout, then the Jacobi runs on X = R^H.  The bench's two-site thetas
// (swap-routed, graded lambdas) need 14-25 sweeps plain and 7-9 after QRP, and a batched launch
// waits for its slowest decomposition.  X's orthogonalised columns are the singular vectors of
// the *other* side times sigma (rows mapped back through the pivot order P), which k_split
// handles by flipping its side test (tools/qrp_jacobi_proto.py is the numpy restatement).

using aqc::jacobi_params;
using aqc::jacobi_te;

// sortable pivot key: non-negative double bits with the low byte replaced by (255 - id), so
// that the 64-bit maximum is the largest trailing norm, ties to the lowest column id
__device__ __forceinline__ unsigned long long pivot_key(double v, int id) {
  return ((unsigned long long)__double_as_longlong(v) & ~255ull) | (unsigned long long)(255 - id);
}

// Householder step k on the pivot column x (this group's S or M): v (zlarfg convention, v_k = 1)
// and tau go to LDS, x becomes R's column (beta on the diagonal, zeros below).
template <int MAXR, int LPG>
__device__ __forceinline__ void qr_reflector(double (&xr)[MAXR], double (&xi)[MAXR], int k, int lane, double2* vb,
                                             double2* tb) {
  const int kr = k / LPG;
  double ar = 0, ai = 0, s2p[2] = {0, 0};  // two partial sums: this chain is on the critical path
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + LPG * i;
    if (i == kr) ar = xr[i], ai = xi[i];
    const double w = row > k ? 1.0 : 0.0;
    s2p[i & 1] = fma(w, fma(xr[i], xr[i], xi[i] * xi[i]), s2p[i & 1]);
  }
  ar = __shfl(ar, k % LPG, LPG);
  ai = __shfl(ai, k % LPG, LPG);
  const double s2 = aqc::group_sum<LPG>(s2p[0] + s2p[1]);
  double beta, tr_, ti_, cr = 0, ci = 0;  // tau = (tr_, ti_), scale = 1 / (alpha - beta)
  if (s2 == 0.0 && ai == 0.0) {
    beta = ar, tr_ = 0.0, ti_ = 0.0;
  } else {
    // rsq / rcp seeds + two Newton steps (full precision) instead of the IEEE sqrt / divide
    // sequences: this chain runs on one group while the workgroup waits at the next barrier
    const double x = fma(ar, ar, fma(ai, ai, s2));
    double r = __builtin_amdgcn_rsq(x);
    r = r * fma(-0.5 * x * r, r, 1.5);
    r = r * fma(-0.5 * x * r, r, 1.5);
    const double nrm = x * r;
    beta = ar >= 0.0 ? -nrm : nrm;
    const double ib = ar >= 0.0 ? -r : r;  // 1 / beta
    tr_ = (beta - ar) * ib;
    ti_ = -ai * ib;
    const double dr = ar - beta, di = ai, d2 = fma(dr, dr, di * di);
    double id2 = __builtin_amdgcn_rcp(d2);
    id2 = id2 * fma(-d2, id2, 2.0);
    id2 = id2 * fma(-d2, id2, 2.0);
    cr = dr * id2, ci = -di * id2;
  }
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + LPG * i;
    double2 v = make_double2(0, 0);
    if (row > k) v = make_double2(xr[i] * cr - xi[i] * ci, xr[i] * ci + xi[i] * cr);
    if (row == k) v = make_double2(1.0, 0.0);
    vb[row] = v;
    const double nr = row == k ? beta : (row > k ? 0.0 : xr[i]);
    const double ni = row >= k ? 0.0 : xi[i];
    xr[i] = nr, xi[i] = ni;
  }
  if (lane == 0) *tb = make_double2(tr_, ti_);
}

// LPG = lanes per column group (16: 1024 threads at CP = 128; 8: 512 threads with 16 rows per
// lane, the per-pair rotation parameters and reductions amortised over twice the rows).
// (The body is a device function so that the fused per-state chain, k_chain, runs it too.)
template <int CP, int MAXR, int LPG = 16, int XPAD = 0, int XNP = 0>
__device__ __forceinline__ void jacobi_reg_body(const TwoSiteJob& j) {
  static_assert(LPG * MAXR == CP, "LPG lanes x MAXR rows must cover the CP rows of a column");
  constexpr int kG = CP / 2;       // groups
  constexpr int kThreads = kG * LPG;
  // exchange-buffer stride (compile time: no guards); narrow groups pad a slot by LPG complex so
  // that consecutive slots alternate LDS bank halves (a ds_read_b128 lane group spans groups)
  constexpr int ld = LPG * MAXR + (LPG < 16 ? LPG : 0) + XPAD;
  constexpr int ldt = CP + 1;      // transpose-buffer stride (odd: conflict-free column writes)
  extern __shared__ double2 xbuf[];  // max(kG * ld, kG * ldt) complex
  __shared__ double fred[kThreads / 64];
  __shared__ int xid[kG];
  __shared__ int rot, big;
  __shared__ unsigned long long pkey[2];
  __shared__ double2 vb[2][CP];
  __shared__ double2 tb[2];
  __shared__ int perm_s[CP];
  const int chl = j.dims[0], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = M < N;
  const int L = tr ? N : M;
  const int C = tr ? M : N;
  const bool use_qr = j.qr != 0;
  const int tid = fresh_tid();
  const int g = tid / LPG, lane = tid % LPG;
  // plain doubles (real / imaginary planes) so the arrays stay in VGPRs
  double sr[MAXR], si[MAXR], mr[MAXR], mi[MAXR];
  int sid = g, mid = g + kG;  // column ids of S and M
  double f = 0.0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = lane + LPG * i;
    const int cs = g, cm = g + kG;
    double2 a = make_double2(0, 0), b = make_double2(0, 0);
    if (r < L && cs < C) a = tr ? aqc::cconj(j.theta[(size_t)r * M + cs]) : j.theta[(size_t)cs * M + r];
    if (r < L && cm < C) b = tr ? aqc::cconj(j.theta[(size_t)r * M + cm]) : j.theta[(size_t)cm * M + r];
    sr[i] = a.x;
    si[i] = a.y;
    mr[i] = b.x;
    mi[i] = b.y;
    f += a.x * a.x + a.y * a.y + b.x * b.x + b.y * b.y;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) f += __shfl_xor(f, off);
  if ((tid & 63) == 0) fred[tid >> 6] = f;
  if (tid == 0) pkey[0] = pkey[1] = 0ull;
  __syncthreads();
  // ||W||_F^2 is needed only after the QR: sum it now into fred[0] (one thread, ordered by the
  // QR's first barrier) rather than keep 16 partials live -- they were spilled to scratch
  if (tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += fred[w];
    fred[0] = s;
  }
  int Lj = L;  // row count of the matrix the Jacobi sees
  // dbg == 2 (aqc_svd_debug mode 2): thread 0 accumulates shader-clock ticks of the QR step's
  // phases -- [0] downdate + pivot key, [1] pivot barrier, [2] reflector + its barrier, [3] update
  // (kept in LDS, not registers: the QR loop has no VGPRs to spare)
  __shared__ unsigned long long qt[5];  // 4 phase totals, last tick
  const bool qtime = j.dbg == 2 && tid == 0;
  if (qtime) qt[0] = qt[1] = qt[2] = qt[3] = qt[4] = 0;
  auto qtick = [&](int ph) {
    if (qtime) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (ph >= 0) qt[ph] += t - qt[4];
      qt[4] = t;
    }
  };
  if (use_qr) {
    int ks = -1, km = -1;  // pivot step of S / M (-1: not pivoted yet)
    // Trailing squared norms (rows >= k) of S and M, downdated by the row leaving the trailing
    // block at every step (n -= |x_{k-1}|^2, LAPACK xLAQP2's scheme) and recomputed exactly when
    // they fall below sqrt(eps) of their last exact value (cancellation).
    double ns = 0, nm = 0, nsr = 0, nmr = 0;
    for (int k = 0; k < C; ++k) {
      const int b = k & 1;
      bool exact = k == 0;
      qtick(k == 0 ? -1 : 3);
      if (k > 0) {
        const int kr = (k - 1) / LPG, kl = (k - 1) % LPG;
        double xsr = 0, xsi = 0, xmr = 0, xmi = 0;  // row k-1 (select first, square once)
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          if (i == kr) xsr = sr[i], xsi = si[i], xmr = mr[i], xmi = mi[i];
        }
        ns -= __shfl(fma(xsr, xsr, xsi * xsi), kl, LPG);
        nm -= __shfl(fma(xmr, xmr, xmi * xmi), kl, LPG);
        exact = ns <= 1.5e-8 * nsr || nm <= 1.5e-8 * nmr;
      }
      if (exact) {
        ns = 0, nm = 0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const double w = (lane + LPG * i) >= k ? 1.0 : 0.0;
          ns = fma(w, fma(sr[i], sr[i], si[i] * si[i]), ns);
          nm = fma(w, fma(mr[i], mr[i], mi[i] * mi[i]), nm);
        }
        ns = aqc::group_sum<LPG>(ns);
        nm = aqc::group_sum<LPG>(nm);
        nsr = ns, nmr = nm;
      }
      const unsigned long long ka = (ks < 0 && sid < C) ? pivot_key(ns, sid) : 0ull;
      const unsigned long long kb = (km < 0 && mid < C) ? pivot_key(nm, mid) : 0ull;
      if (lane == 0) atomicMax(&pkey[b], ka > kb ? ka : kb);
      qtick(0);
      __syncthreads();
      const int p = 255 - (int)(pkey[b] & 255ull);
      qtick(1);
      if (tid == 0) pkey[b ^ 1] = 0ull;
      if (sid == p) {  // this group owns the pivot column: build the reflector
        qr_reflector<MAXR, LPG>(sr, si, k, lane, vb[b], &tb[b]);
        ks = k;
      } else if (mid == p) {
        qr_reflector<MAXR, LPG>(mr, mi, k, lane, vb[b], &tb[b]);
        km = k;
      }
      if (tid == 0) perm_s[k] = p;
      __syncthreads();
      qtick(2);
      // c <- H^H c = c - conj(tau) v (v^H c) for every unpivoted column
      const double2 tau = tb[b];
      double wsr = 0, wsi = 0, wmr = 0, wmi = 0;
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {  // v^H c (v re-read from LDS below: saves 4*MAXR VGPRs)
        const double2 v = vb[b][lane + LPG * i];
        wsr = fma(v.x, sr[i], fma(v.y, si[i], wsr));
        wsi = fma(v.x, si[i], fma(-v.y, sr[i], wsi));
        wmr = fma(v.x, mr[i], fma(v.y, mi[i], wmr));
        wmi = fma(v.x, mi[i], fma(-v.y, mr[i], wmi));
      }
      wsr = aqc::group_sum<LPG>(wsr);
      wsi = aqc::group_sum<LPG>(wsi);
      wmr = aqc::group_sum<LPG>(wmr);
      wmi = aqc::group_sum<LPG>(wmi);
      // f = conj(tau) * w ; c -= v * f
      const double as = ks < 0 ? 1.0 : 0.0, am = km < 0 ? 1.0 : 0.0;
      const double fsr = as * (tau.x * wsr + tau.y * wsi), fsi = as * (tau.x * wsi - tau.y * wsr);
      const double fmr = am * (tau.x * wmr + tau.y * wmi), fmi = am * (tau.x * wmi - tau.y * wmr);
      asm volatile("" ::: "memory");  // re-read v below instead of keeping 2*MAXR doubles live
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        const double2 v = vb[b][lane + LPG * i];
        sr[i] = fma(-v.x, fsr, fma(v.y, fsi, sr[i]));  // 2 FMAs per component, not mul+fma+add
        si[i] = fma(-v.x, fsi, fma(-v.y, fsr, si[i]));
        mr[i] = fma(-v.x, fmr, fma(v.y, fmi, mr[i]));
        mi[i] = fma(-v.x, fmi, fma(-v.y, fmr, mi[i]));
      }
    }
    // X = R^H: X[i][jx] = conj(R[jx][column pivoted at step i]); new S / M = X columns g, g + kG.
    // LDS holds half of the matrix, and the register halves whose R rows already went to LDS are
    // reused: half 0 sends R rows [0, kG) and lands X column g in (S-low, M-low); half 1 sends R
    // rows [kG, 2kG) and lands X column g + kG in (S-high, M-high); one register swap finishes.
    constexpr int H = MAXR / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = h * H; i < (h + 1) * H; ++i) {
        const int jx = lane + LPG * (i - h * H);
        if (ks >= 0) xbuf[jx * ldt + ks] = make_double2(sr[i], -si[i]);
        if (km >= 0) xbuf[jx * ldt + km] = make_double2(mr[i], -mi[i]);
      }
      __syncthreads();
      const bool real_col = g + h * kG < C;
#pragma unroll
      for (int i = h * H; i < (h + 1) * H; ++i) {
        const int ra = lane + LPG * (i - h * H), rb = ra + kG;  // X rows (pivot steps)
        double2 va = make_double2(0, 0), vb2 = make_double2(0, 0);
        if (real_col && ra < C) va = xbuf[g * ldt + ra];
        if (real_col && rb < C) vb2 = xbuf[g * ldt + rb];
        sr[i] = va.x, si[i] = va.y;
        mr[i] = vb2.x, mi[i] = vb2.y;
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {  // M-low <-> S-high
      const double tr0 = mr[i], ti0 = mi[i];
      mr[i] = sr[i + H], mi[i] = si[i + H];
      sr[i + H] = tr0, si[i + H] = ti0;
    }
    Lj = C;
  }
  __syncthreads();
  const double floor2 = fred[0] * 1e-24;
  const double tol = j.jtol * (double)Lj * 2.220446049250313e-16;
  const double tol2 = tol * tol;
  // Dot-product noise floor: columns made of rounding noise carry ~eps ||W|| absolute error (the
  // QR's, theta's own), so their products a^H b are only resolved above ~eps ||W|| (|a| + |b|):
  // below it a pair of small (near-)degenerate columns rotates by 45 degrees at noise level every
  // sweep and the loop never stops (61 sweeps on a spectrum 8 x 1 + 120 x 1e-6, with 2.6e-5
  // errors in the large values).  Rotations need |g|^2 > max(tol^2 |a|^2 |b|^2,
  // 2 (jnoise eps)^2 ||W||^2 (|a|^2 + |b|^2)).
  const double nfl2 = jacobi_noise2(j, fred[0]);
  qtick(3);
  const int max_sweeps = j.dbg >= 1 ? 0 : kMaxSweeps;
  const bool map_rows = use_qr && j.dbg == 0;
  // The M half of the columns moves into LDS slots (slot g <- this group's M) and stays there:
  // S stays in VGPRs.  Round r of a level with sub-blocks of m groups pairs S_g with slot
  // base + (li + r) mod m -- the parallel ordering's shift is addressing only -- and a slot is
  // written back only when its column was rotated, which late sweeps rarely do.  Level split:
  // the upper half swaps its S with slot g - h (the lower half's next partners).  One barrier
  // per round.  (A register-resident M with a per-round LDS shift moved every M column through
  // the ~79 B/clk LDS store path twice per round: 1.5x slower, tools/jacobi_lab.hip.)
  //
  // Scaled columns with tracked norms (the round is VALU-bound): a column is d * v (v stored,
  // d > 0, 1/d kept too) with its squared norm n tracked through the rotation identity
  // n_a' = n_a - t|g|, n_b' = n_b + t|g| (exact at every sweep start, recomputed when a norm
  // falls by more than 1e6: cancellation).  The rotation of the true columns
  //   a' = c a - s conj(e) b,  b' = s e a + c b   (t = s / c, e = g / |g|)
  // acts on the stored vectors as v_a' = v_a - mu v_b, v_b' = v_b + nu v_a with
  //   mu = t conj(e) d_b / d_a,  nu = t e d_a / d_b,  d' = c d:
  // 8 FMAs per row instead of 12, and only g = a^H b is reduced per round (2 sums, not 4).
  __shared__ double xnrm[kG], xscl[kG], xisc[kG];
  __syncthreads();  // the QR transpose's last reads of xbuf are done
#pragma unroll
  for (int i = 0; i < MAXR; ++i) xbuf[g * ld + lane + LPG * i] = make_double2(mr[i], mi[i]);
  if (lane == 0) {
    xid[g] = mid;
    xscl[g] = 1.0;
  }
  // Stop rule: a sweep whose counted rotations all moved at most jtiny^2 (default 1e-12) of their
  // pair's squared norms (t|g| <= jtiny^2 (|a|^2 + |b|^2)) is the last: the next sweep would move
  // them by less again (quadratic convergence), so the confirming sweep with no rotation at all is
  // skipped.
  const double tiny2 = j.jtiny * j.jtiny;
  double sd = 1.0, sn = 0.0;  // S: scale and tracked squared norm (uniform in the group)
  int sweeps = 0;
  for (sweeps = 0; sweeps < max_sweeps; ++sweeps) {
    {  // sweep start: fold the scales into the vectors, exact norms
      double2* own = xbuf + g * ld;
      const double od = xscl[g];
      double a = 0, b = 0;
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        sr[i] *= sd;
        si[i] *= sd;
        double2 v = own[lane + LPG * i];
        v.x *= od;
        v.y *= od;
        own[lane + LPG * i] = v;
        a = fma(sr[i], sr[i], fma(si[i], si[i], a));
        b = fma(v.x, v.x, fma(v.y, v.y, b));
      }
      a = aqc::group_sum<LPG>(a);
      b = aqc::group_sum<LPG>(b);
      sd = 1.0;
      sn = a;
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        xscl[g] = 1.0;
        xisc[g] = 1.0;
        xnrm[g] = b;
      }
      if (tid == 0) rot = big = 0;
    }
    __syncthreads();
    double isd = 1.0;
    int my_rot = 0, my_big = 0;
    for (int m = kG; m >= 1; m >>= 1) {  // level: sub-blocks of m groups
      const int li = g & (m - 1), base = g - li;
      for (int r = 0; r < m; ++r) {
        const int slot = base + ((li + r) & (m - 1));
        double2* col = xbuf + slot * ld;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const double2 v = col[lane + LPG * i];
          mr[i] = v.x;
          mi[i] = v.y;
        }
        const double mn = xnrm[slot], md = xscl[slot], imd = xisc[slot];
        // NP partial sums: with 16+ rows per lane and 1-2 waves per SIMD a single chain would
        // expose its FMA latency
        constexpr int NP = XNP ? XNP : (MAXR >= 16 ? 2 : 1);
        double gxp[NP], gyp[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) gxp[q] = gyp[q] = 0.0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          gxp[i % NP] = fma(sr[i], mr[i], fma(si[i], mi[i], gxp[i % NP]));   // conj(s) * m
          gyp[i % NP] = fma(sr[i], mi[i], fma(-si[i], mr[i], gyp[i % NP]));
        }
        double gx = gxp[0], gy = gyp[0];
#pragma unroll
        for (int q = 1; q < NP; ++q) gx += gxp[q], gy += gyp[q];
        gx = aqc::group_sum<LPG>(gx);
        gy = aqc::group_sum<LPG>(gy);
        const double dd = sd * md;
        gx *= dd;
        gy *= dd;
        const double g2 = gx * gx + gy * gy;
        const double thr = fmax(tol2 * sn * mn, nfl2 * (sn + mn));
        if (g2 > thr && sn > floor2 && mn > floor2) {
          // only rotations above dot-product noise keep the sweep loop going: a pair of
          // (near-)degenerate columns can otherwise flip-flop at |g| ~ tol forever
          double te, c, p;  // te = t / |g|, p = 1 + t^2
          jacobi_te(sn, mn, g2, te, c, p);
          if (g2 > 16.0 * thr) {
            my_rot = 1;
            // the rotation moves t|g| between the squared norms: above jtiny^2 of them it counts
            // (t|g| ~ t^2 (|a|^2 - |b|^2) for separated pairs -- |t| > jtiny -- and ~ |g| for a
            // (near-)degenerate pair, whose t stays O(1) at any |g|: a test on |t| alone stopped
            // with |g| ~ 1e-6 |a|^2 - |b|^2| left, 3e-8 errors in a degenerate pair's sigma)
            if (fabs(te) * g2 > tiny2 * (sn + mn)) my_big = 1;
          }
          const double ra = md * isd, ira = sd * imd;  // d_b / d_a and its inverse
          const double mux = te * gx * ra, muy = -te * gy * ra;   // mu = t conj(e) d_b / d_a
          const double nux = te * gx * ira, nuy = te * gy * ira;  // nu = t e d_a / d_b
#pragma unroll
          for (int i = 0; i < MAXR; ++i) {
            const double ar = sr[i], ai = si[i], br = mr[i], bi = mi[i];
            sr[i] = fma(-mux, br, fma(muy, bi, ar));
            si[i] = fma(-mux, bi, fma(-muy, br, ai));
            col[lane + LPG * i] = make_double2(fma(nux, ar, fma(-nuy, ai, br)), fma(nux, ai, fma(nuy, ar, bi)));
          }
          const double ic = p * c;  // 1 / c
          sd *= c;
          isd *= ic;
          const double md2 = md * c, imd2 = imd * ic;
          const double tg = te * g2;  // t |g|
          double sn2 = sn - tg, mn2 = mn + tg;
          if (sn2 < 1e-6 * sn || mn2 < 1e-6 * mn) {  // cancellation: recompute exactly
            double a = 0, b = 0;
            asm volatile("" ::: "memory");  // re-read M from LDS: keeps it out of VGPRs above
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {  // (this lane's own LDS writes: in order)
              const double2 v = col[lane + LPG * i];
              a = fma(sr[i], sr[i], fma(si[i], si[i], a));
              b = fma(v.x, v.x, fma(v.y, v.y, b));
            }
            sn2 = aqc::group_sum<LPG>(a) * sd * sd;
            mn2 = aqc::group_sum<LPG>(b) * md2 * md2;
          }
          sn = sn2;
          __builtin_amdgcn_wave_barrier();
          if (lane == 0) {
            xnrm[slot] = mn2;
            xscl[slot] = md2;
            xisc[slot] = imd2;
          }
        }
        __syncthreads();
      }
      if (m == 1) break;
      const int h = m >> 1;
      if (li >= h) {  // upper half: S <-> slot g - h (vectors, id, norm, scales)
        double2* col = xbuf + (g - h) * ld;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const double2 v = col[lane + LPG * i];
          col[lane + LPG * i] = make_double2(sr[i], si[i]);
          sr[i] = v.x;
          si[i] = v.y;
        }
        const int pid = xid[g - h];
        const double pn = xnrm[g - h], pd = xscl[g - h], pi = xisc[g - h];
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
          xid[g - h] = sid;
          xnrm[g - h] = sn;
          xscl[g - h] = sd;
          xisc[g - h] = isd;
        }
        sid = pid;
        sn = pn;
        sd = pd;
        isd = pi;
      }
      __syncthreads();
    }
    if (my_rot && lane == 0) atomicAdd(&rot, 1);
    if (my_big && lane == 0) atomicAdd(&big, 1);
    __syncthreads();
    if (rot == 0 || big == 0) break;
    __syncthreads();
  }
  // write columns to their own slots (with QR: rows mapped back through the pivot order) and
  // their norms: S from VGPRs, slot g's column from LDS, both with their scales applied
  double2* W = j.work;
  const int mid_out = xid[g];
  const double od = xscl[g];
  double ns = 0, nm = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + LPG * i;
    double2 mv = xbuf[g * ld + row];
    mv.x *= od;
    mv.y *= od;
    const double ar = sr[i] * sd, ai = si[i] * sd;
    if (row < Lj) {
      const int orow = map_rows ? perm_s[row] : row;
      if (sid < C) W[(size_t)sid * Lj + orow] = make_double2(ar, ai);
      if (mid_out < C) W[(size_t)mid_out * Lj + orow] = mv;
    }
    ns = fma(ar, ar, fma(ai, ai, ns));
    nm = fma(mv.x, mv.x, fma(mv.y, mv.y, nm));
  }
  ns = aqc::group_sum<LPG>(ns);
  nm = aqc::group_sum<LPG>(nm);
  if (lane == 0) {
    if (sid < C) j.sig[sid] = sqrt(ns);
    if (mid_out < C) j.sig[mid_out] = sqrt(nm);
  }
  if (tid == 0) {
    if (sweeps >= kMaxSweeps) atomicOr(&j.flags[1], 1);
    atomicMax(&j.flags[2], sweeps + 1);
  }
  if (qtime) {
    for (int ph = 0; ph < 4; ++ph) j.sig[ph] = (double)qt[ph];
  }
  if (j.dbg >= 1 && use_qr) {  // diagnostics: pivot order after the W columns
    for (int k = tid; k < C; k += kThreads) j.perm[k] = perm_s[k];
  }
}

template <int CP, int MAXR, int LPG = 16, int XPAD = 0, int XNP = 0>
__global__ __launch_bounds__(CP / 2 * LPG) void k_jacobi_reg(const TwoSiteJob* __restrict__ jobs) {
  jacobi_reg_body<CP, MAXR, LPG, XPAD, XNP>(jobs[blockIdx.x]);
}

#include "svd_gram.h"
// two-site SVDs at 2 chi = 128 try the Gram / tridiagonal path first (aqc_mps_set_svd_path; the
// initial value from AQC_SVD_PATH = 0 or 1, default 1)
int g_svd_gram = [] {
  const char* e = std::getenv("AQC_SVD_PATH");
  const int v = e ? std::atoi(e) : 1;
  return v >= 0 && v <= 1 ? v : 1;
}();
int g_debug_max_chi = 64;  // aqc_svd_debug's max_chi (the Gram path keeps K = min(C, max_chi))

// 2 chi = 128: the Gram path with the register Jacobi (16-lane groups, 1024 threads) as its
// in-kernel fallback, or the register Jacobi alone (aqc_mps_set_svd_path(0, ...)).  Dynamic LDS =
// kG x max(ld, CP + 1) complex.  Rejected shapes (measured on the bench's thetas, tools/jacobi_ab.py,
// tools/svd_phase_timing.py; removed from the library in round 3, see tools/lab/README.md):
// 8-lane groups (same sweep speed at two waves per SIMD, QR phase 20% slower), 4-lane groups
// (AGPR spills, 1.9x slower), four columns per group (11% slower).
void launch_jacobi_reg128(int nj, hipStream_t st, const TwoSiteJob* jp) {
  if (g_svd_gram) {
    hipLaunchKernelGGL(k_svd_gram, dim3(nj), dim3(1024), kChainLdsBytes, st, jp);
    return;
  }
  hipLaunchKernelGGL((k_jacobi_reg<128, 8>), dim3(nj), dim3(1024), 64 * 129 * 16, st, jp);
}

// Sort singular values, apply reduce_zeros, write lambda_m / dims[1] / perm / sorted sig.
template <int NT, int MAXC = kSigMax>
__device__ __forceinline__ void rank_body(const TwoSiteJob& j) {
  __shared__ double sv[MAXC];
  __shared__ int si[MAXC];
  __shared__ int kk_s;
  __shared__ double norm_s;
  const int chl = j.dims[0], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const int C = M < N ? M : N;
  int P = 1;
  while (P < C) P <<= 1;
  const int tid = fresh_tid();
  for (int i = tid; i < P; i += NT) {
    sv[i] = i < C ? aqc::ldg(j.sig + i) : -1.0;
    si[i] = i;
  }
  __syncthreads();
  // bitonic sort, descending by value, ascending index on ties
  for (int k = 2; k <= P; k <<= 1) {
    for (int s = k >> 1; s > 0; s >>= 1) {
      for (int i = tid; i < P; i += NT) {
        const int ixj = i ^ s;
        if (ixj > i) {
          const bool desc = (i & k) == 0;
          const double a = sv[i], b = sv[ixj];
          const bool a_first = (a > b) || (a == b && si[i] < si[ixj]);
          if (a_first != desc) {
            sv[i] = b;
            sv[ixj] = a;
            const int t = si[i];
            si[i] = si[ixj];
            si[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    int k = 0;
    for (int i = 0; i < C; ++i)
      if (sv[i] * sv[i] > kChop) ++k;
    if (k < 1) k = 1;
    if (j.max_chi > 0 && k > j.max_chi) k = j.max_chi;
    // (a Gram path that decided the kept count hands over the tail it removed: sig[kSigTail])
    double tail = aqc::ldg(j.sig + kSigTail);
    while (k > 1 && tail + sv[k - 1] * sv[k - 1] < j.thr) {
      tail += sv[k - 1] * sv[k - 1];
      --k;
    }
    aqc::stg(j.sig + kSigTail, 0.0);
    // the bond capacity is this library's limit, not Aer's: only a kept count above it (after the
    // whole reduce_zeros rule) overflows
    if (k > j.cap) {
      k = j.cap;
      atomicOr(&j.flags[0], 1);
    }
    double nn = 0.0;
    for (int i = 0; i < k; ++i) nn += sv[i] * sv[i];
    kk_s = k;
    norm_s = sqrt(nn);
    *(__attribute__((address_space(1))) int*)(j.dims + 1) = k;
  }
  __syncthreads();
  const int k = kk_s;
  for (int i = tid; i < k; i += NT) {
    aqc::stg(j.lm + i, sv[i] / norm_s);  // (GLOBAL stores: FLAT ones would also count on LGKM_CNT)
    *(__attribute__((address_space(1))) int*)(j.perm + i) = si[i];
    aqc::stg(j.sig + i + kSigMax, sv[i]);  // sorted copy lives past the raw norms
  }
}

__global__ __launch_bounds__(kT) void k_rank(const TwoSiteJob* __restrict__ jobs) { rank_body<kT>(jobs[blockIdx.x]); }

// Orthogonalised side: copy (scaled) columns of W into the Gamma they define.
// Element e = start, start + stride, ... of the copy.
__device__ __forceinline__ void split_copy_body(const TwoSiteJob& j, int start, int stride) {
  const int chl = j.dims[0], k = j.dims[1], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  // tr: W's columns are V-side (length N); the QR-preconditioned Jacobi flips the side
  const bool tr = (M < N) != (j.qr != 0);
  const int L = tr ? N : M;
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  const double* ss = j.sig + kSigMax;
  if (!tr) {
    // Gp'[s1][l][kk] = W[perm kk][s1*chl + l] / sig_kk / ll[l]
    for (int e = start; e < 2 * chl * k; e += stride) {
      const int kk = e % k, rr = e / k;
      const int s1 = rr / chl, l = rr % chl;
      const double d = aqc::ldg(ss + kk) * aqc::ldg(j.ll + l);
      const cplx w = aqc::ldg(j.work + (size_t)j.perm[kk] * L + rr);
      aqc::stg(j.gp + s1 * half + (size_t)l * cap + kk, d != 0.0 ? aqc::cscale(w, 1.0 / d) : aqc::cmk(0, 0));
    }
  } else {
    // Gq'[s2][kk][r] = conj(W[perm kk][s2*chr + r]) / sig_kk / lr[r]
    for (int e = start; e < 2 * chr * k; e += stride) {
      const int cc = e % N, kk = e / N;
      const int s2 = cc / chr, r = cc % chr;
      const double d = aqc::ldg(ss + kk) * aqc::ldg(j.lr + r);
      const cplx w = aqc::cconj(aqc::ldg(j.work + (size_t)j.perm[kk] * L + cc));
      aqc::stg(j.gq + s2 * half + (size_t)kk * cap + r, d != 0.0 ? aqc::cscale(w, 1.0 / d) : aqc::cmk(0, 0));
    }
  }
}

__global__ __launch_bounds__(kT) void k_split_copy(const TwoSiteJob* __restrict__ jobs) {
  split_copy_body(jobs[blockIdx.y], blockIdx.x * kT + threadIdx.x, gridDim.x * kT);
}

// Other side by one GEMM against the original theta (64 x 64 output blocks per workgroup,
// register-blocked, aqc_gemm.h):
//   !tr: Vh[kk][c] = sum_R conj(W_j[R]) theta[R][c] / sig^2 -> Gq'[s2][kk][r] = Vh / lr[r]
//    tr: U[R][kk]  = sum_c theta[R][c] W_j[c] / sig^2      -> Gp'[s1][l][kk] = U / ll[l]
// (tr: W's columns are V-side; the QR-preconditioned Jacobi flips the side, see k_split_copy.)
// Output block blk (64 x 64) of the split GEMM.  ltid >= 0: the caller's rank in a 256-thread
// sub-group of the fused chain, where an empty block still runs block_cgemm's barriers (inactive)
// so that the sub-groups' barriers pair up; the standalone kernel skips empty blocks instead.
__device__ __forceinline__ bool split_block_active(const TwoSiteJob& j, int blk) {
  const int chl = j.dims[0], k = j.dims[1], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = (M < N) != (j.qr != 0);
  const int rows = tr ? M : k, cols = tr ? k : N;
  const int bcols = (2 * j.cap + 63) / 64;
  return (blk / bcols) * 64 < rows && (blk % bcols) * 64 < cols;
}

// PF: register prefetch of the next k tile (the standalone kernel; the 1024-thread chain, at 128
// VGPRs per lane, runs without it)
template <bool PF = true>
__device__ __forceinline__ void split_gemm_body(const TwoSiteJob& j, int blk, aqc::GemmLds& lds, int ltid) {
  const int chl = j.dims[0], k = j.dims[1], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = (M < N) != (j.qr != 0);
  const int L = tr ? N : M;
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  const double* ss = j.sig + kSigMax;
  const int rows = tr ? M : k, cols = tr ? k : N;
  const int bcols = (2 * cap + 63) / 64;
  const int r0 = (blk / bcols) * 64, c0 = (blk % bcols) * 64;
  const bool active = r0 < rows && c0 < cols;
  const int mb = active ? min(64, rows - r0) : 64, nb = active ? min(64, cols - c0) : 64;
  const cplx* W = j.work;
  const int* perm = j.perm;
  const cplx* th = j.theta;
  if (!tr) {
    aqc::block_cgemm<true, true, PF>(
        mb, nb, L, [&](int kk, int R) { return aqc::cconj(W[(size_t)perm[r0 + kk] * L + R]); },
        [&](int R, int c) { return th[(size_t)(c0 + c) * M + R]; },
        [&](int kk, int c, cplx v) {
          const int kq = r0 + kk, cc = c0 + c, s2 = cc / chr, r = cc % chr;
          const double d = ss[kq] * ss[kq] * j.lr[r];
          j.gq[s2 * half + (size_t)kq * cap + r] = d != 0.0 ? aqc::cscale(v, 1.0 / d) : aqc::cmk(0, 0);
        },
        lds, ltid, active);
  } else {
    aqc::block_cgemm<false, true, PF>(
        mb, nb, L, [&](int R, int c) { return th[(size_t)c * M + r0 + R]; },
        [&](int c, int kk) { return W[(size_t)perm[c0 + kk] * L + c]; },
        [&](int R, int kk, cplx v) {
          const int Rr = r0 + R, kq = c0 + kk, s1 = Rr / chl, l = Rr % chl;
          const double d = ss[kq] * ss[kq] * j.ll[l];
          j.gp[s1 * half + (size_t)l * cap + kq] = d != 0.0 ? aqc::cscale(v, 1.0 / d) : aqc::cmk(0, 0);
        },
        lds, ltid, active);
  }
}

__global__ __launch_bounds__(aqc::kGemmThreads) void k_split_gemm(const TwoSiteJob* __restrict__ jobs, int nj) {
  int jb, blk;
  if (!aqc::xcd_job_block(nj, jb, blk)) return;  // (a job's blocks on one XCD: they share panels)
  const TwoSiteJob& j = jobs[jb];
  __shared__ aqc::GemmLds lds;
  if (!split_block_active(j, blk)) return;
  split_gemm_body(j, blk, lds, -1);
}

// ---- fused per-state chain (2 chi = 128) ----------------------------------------------------
// One 1024-thread workgroup runs one state's whole list of device ops -- for a two-site update
// theta (four 256-thread sub-groups, one P_{s1' s2'} each on the matrix cores, then the gate mix
// in place), the register Jacobi, the rank / truncation and the split -- with no grid-wide step
// between updates.  The lock-step batch (run_waves) pays, per update, the slowest decomposition
// of the whole launch and five launches; here a state's time is the sum of its own updates.
__device__ __forceinline__ void one_site_body(const OneSiteJob& j, int start, int stride) {
  const int cl = j.dims[0], cr = j.dims[1];
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  for (int e = start; e < cl * cr; e += stride) {
    const int l = e / cr, r = e % cr;
    const size_t o = (size_t)l * cap + r;
    const cplx a0 = aqc::ldg(j.g + o), a1 = aqc::ldg(j.g + half + o);  // GLOBAL, not FLAT
    aqc::stg(j.g + o, aqc::cfma(j.u[1], a1, aqc::cmul(j.u[0], a0)));
    aqc::stg(j.g + half + o, aqc::cfma(j.u[3], a1, aqc::cmul(j.u[2], a0)));
  }
}

struct ChainJob {
  const int* ops;  // >= 0: two-site job index; < 0: one-site job -(code + 1)
  int nops;
  int pad;
};

constexpr int kChainLds = kChainLdsBytes;  // >= the Jacobi's 64 x 129 complex
// phase ticks summed over workgroups: theta, Jacobi, rank, split, one-site
__device__ unsigned long long g_chain_ticks[5];

// The phases are separate (non-inlined) functions: inlined into one loop body the compiler kept
// values live across them and spilled hundreds of bytes per lane inside the Jacobi rounds.
// theta in the chain on the VALU: sub-group sg of 256 threads computes the 32 x 32 output quadrant
// (l0, r0) = 32 (sg >> 1, sg & 1) of all four P_{s1 s2} = (ll lm Gamma_p[s1]) (Gamma_q[s2] lr),
// thread (ty, tx) = (lt / 16, lt % 16) rows l0 + tx + 16 i, columns r0 + ty + 16 jj (i, jj < 2):
// 16 complex accumulators, 8 LDS reads per 64 FMAs (one output per thread read 4 per 16 and was
// LDS-bound), then the gate mix in registers and coalesced theta writes (lanes along l).  Every
// sub-group runs the same m steps, so the barriers pair up.  Kept as the A/B form of the MFMA
// theta below (-DAQC_THETA_MFMA=0): per k_chain workgroup 6.48 M against 5.18 M ticks of theta
// over 49 updates, bench 7.83 against 8.06 M evals/s (round 6).
// m is staged 8 at a time (16, with A's rows XOR-swizzled instead of padded -- half the barriers,
// twice the loads in flight per step -- measured slower: 41.9 against 39.3 ms per k_chain launch)
constexpr int kThetaCh = 8;
constexpr int kThetaAPitch = 9;
constexpr int kThetaLds = 2 * 32 * kThetaAPitch + 2 * kThetaCh * 33;  // complex per sub-group
static_assert(4 * kThetaLds * 16 <= kChainLdsBytes, "theta staging exceeds the chain's LDS");
[[maybe_unused]] __device__ __forceinline__ void chain_theta(const TwoSiteJob& j) {
  extern __shared__ double2 xbuf[];
  const int tid = fresh_tid(), sg = tid >> 8, lt = tid & 255;
  constexpr int KCH = kThetaCh;
  cplx* base = xbuf + sg * kThetaLds;
  cplx (*As)[32][kThetaAPitch] = reinterpret_cast<cplx (*)[32][kThetaAPitch]>(base);
  cplx (*Bs)[KCH][33] = reinterpret_cast<cplx (*)[KCH][33]>(base + 2 * 32 * kThetaAPitch);
  const int chl = j.dims[0], chm = j.dims[1], chr = j.dims[2];
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  const int M = 2 * chl;
  const int l0 = 32 * (sg >> 1), r0 = 32 * (sg & 1);
  const bool active = l0 < chl && r0 < chr;
  const int ty = lt >> 4, tx = lt & 15;
  // the operand pointers held in SGPRs across the m loop: left to the compiler they were re-read
  // from the job (s_load) every step, and each step's global loads waited on lgkmcnt(0) first
  const cplx* gp = j.gp;
  const cplx* gq = j.gq;
  const double* llp = j.ll;
  const double* lmp = j.lm;
  const double* lrp = j.lr;
  asm volatile("" : "+s"(gp), "+s"(gq), "+s"(llp), "+s"(lmp), "+s"(lrp));
  // the gate to the LDS (visible after the m loop's first barrier): read by the epilogue, where
  // scalar loads of it waited out one scalar-cache round trip per 8 entries
  __shared__ cplx sG[16];
  if (tid < 16) sG[tid] = aqc::ldg(j.G + tid);
  cplx acc[4][2][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[q][i][jj] = aqc::cmk(0, 0);
  for (int m0 = 0; m0 < chm; m0 += KCH) {
#pragma unroll
    for (int u = 0; u < KCH / 4; ++u) {
      const int e = lt + 256 * u, s = e / (32 * KCH);
      {  // A: KCH consecutive m of one row per KCH lanes
        const int row = (e / KCH) & 31, mm = e % KCH, l = l0 + row, m = m0 + mm;
        cplx a = aqc::cmk(0, 0);
        if (active && l < chl && m < chm)
          a = aqc::cscale(aqc::ldg(gp + s * half + (size_t)l * cap + m), aqc::ldg(llp + l) * aqc::ldg(lmp + m));
        As[s][row][mm] = a;
      }
      {  // B: 32 consecutive r of one row per 32 lanes
        const int mm = (e >> 5) % KCH, col = e & 31, m = m0 + mm, r = r0 + col;
        cplx b = aqc::cmk(0, 0);
        if (active && m < chm && r < chr) b = aqc::cscale(aqc::ldg(gq + s * half + (size_t)m * cap + r), aqc::ldg(lrp + r));
        Bs[s][mm][col] = b;
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll 2
      for (int mm = 0; mm < KCH; ++mm) {
        cplx av[2][2], bv[2][2];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            av[s][i] = As[s][tx + 16 * i][mm];
            bv[s][i] = Bs[s][mm][ty + 16 * i];
          }
#pragma unroll
        for (int s1 = 0; s1 < 2; ++s1)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int jj = 0; jj < 2; ++jj)
                acc[2 * s1 + s2][i][jj] = aqc::cfma(av[s1][i], bv[s2][jj], acc[2 * s1 + s2][i][jj]);
      }
    }
    __syncthreads();
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int l = l0 + tx + 16 * i, r = r0 + ty + 16 * jj;
        if (l < chl && r < chr) {
#pragma unroll
          for (int o = 0; o < 4; ++o) {
            cplx v = aqc::cmul(sG[o * 4 + 0], acc[0][i][jj]);
            v = aqc::cfma(sG[o * 4 + 1], acc[1][i][jj], v);
            v = aqc::cfma(sG[o * 4 + 2], acc[2][i][jj], v);
            v = aqc::cfma(sG[o * 4 + 3], acc[3][i][jj], v);
            aqc::stg(j.theta + (size_t)((o & 1) * chr + r) * M + (o >> 1) * chl + l, v);  // GLOBAL, not FLAT
          }
        }
      }
  }
}
#ifndef AQC_THETA_MFMA
#define AQC_THETA_MFMA 1
#endif
// theta in the chain on the FP64 matrix cores (round 6): wave w owns the 16 x 16 output tile
// (r0, l0) = 16 (w >> 2, w & 3) of all four P_{s1 s2}, computed transposed -- P^T[r][l] = sum_m
// B_{s2}[m][r] A_{s1}[l][m] (A operand: B_{s2} from the LDS, lane l: row r0 + l % 16, k = l / 16;
// B operand: A_{s1}) -- so the accumulator rows run along r and its columns along l, and the theta
// stores (column-major, l fastest) go out as 256-byte runs.  A complex product is four real MFMAs
// into two accumulators (4 P's: 64 VGPRs of accumulators, the VALU form's 16 complex).  m is staged
// 8 at a time for the whole workgroup (A: 2 x 64 x 8, B: 2 x 8 x 64 complex, double-buffered, one
// barrier per chunk), the next chunk's global loads in flight during the current chunk's MFMAs.
constexpr int kThetaMfmaAP = 9;   // As row pitch (complex): [s1][l][m]
constexpr int kThetaMfmaBP = 65;  // Bs row pitch: [s2][m][r]
constexpr int kThetaMfmaBuf = 2 * 64 * kThetaMfmaAP + 2 * 8 * kThetaMfmaBP;  // complex per buffer
static_assert(2 * kThetaMfmaBuf * 16 <= kChainLdsBytes, "theta staging exceeds the chain's LDS");
__device__ __forceinline__ void chain_theta_mfma(const TwoSiteJob& j) {
  extern __shared__ double2 xbuf[];
  const int tid = fresh_tid(), wave = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int chl = j.dims[0], chm = j.dims[1], chr = j.dims[2];
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  const int M = 2 * chl;
  const int r0 = 16 * (wave >> 2), l0 = 16 * (wave & 3);
  const bool active = r0 < chr && l0 < chl;  // (uniform per wave)
  const cplx* gp = j.gp;
  const cplx* gq = j.gq;
  const double* llp = j.ll;
  const double* lmp = j.lm;
  const double* lrp = j.lr;
  asm volatile("" : "+s"(gp), "+s"(gq), "+s"(llp), "+s"(lmp), "+s"(lrp));
  __shared__ cplx sG[16];
  if (tid < 16) sG[tid] = aqc::ldg(j.G + tid);
  // this thread's staging element: A[s1 = e >> 9][l = (e >> 3) & 63][m = e & 7],
  // B[s2 = e >> 9][m = (e >> 6) & 7][r = e & 63]
  const int as1 = tid >> 9, al = (tid >> 3) & 63, am = tid & 7;
  const int bs2 = tid >> 9, bm = (tid >> 6) & 7, br = tid & 63;
  auto fetch = [&](int m0, cplx& a, cplx& b) {
    const int ma = m0 + am, mb = m0 + bm;
    a = (al < chl && ma < chm) ? aqc::cscale(aqc::ldg(gp + as1 * half + (size_t)al * cap + ma), aqc::ldg(llp + al) * aqc::ldg(lmp + ma))
                               : aqc::cmk(0, 0);
    b = (mb < chm && br < chr) ? aqc::cscale(aqc::ldg(gq + bs2 * half + (size_t)mb * cap + br), aqc::ldg(lrp + br)) : aqc::cmk(0, 0);
  };
  auto stash = [&](int buf, cplx a, cplx b) {
    cplx* base = xbuf + buf * kThetaMfmaBuf;
    base[(as1 * 64 + al) * kThetaMfmaAP + am] = a;
    base[2 * 64 * kThetaMfmaAP + (bs2 * 8 + bm) * kThetaMfmaBP + br] = b;
  };
  aqc::d4_t cr[2][2], ci[2][2];
#pragma unroll
  for (int s1 = 0; s1 < 2; ++s1)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) cr[s1][s2] = aqc::d4_t{0, 0, 0, 0}, ci[s1][s2] = aqc::d4_t{0, 0, 0, 0};
  const int nch = (chm + 7) >> 3;
  {
    cplx a, b;
    fetch(0, a, b);
    stash(0, a, b);
  }
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    cplx na = aqc::cmk(0, 0), nb = aqc::cmk(0, 0);
    if (more) fetch(8 * (c + 1), na, nb);
    if (active) {
      const cplx* base = xbuf + (c & 1) * kThetaMfmaBuf;
      const cplx* As = base;
      const cplx* Bs = base + 2 * 64 * kThetaMfmaAP;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int mm = 4 * ks + lk;
        cplx x[2], y[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          x[s] = Bs[(s * 8 + mm) * kThetaMfmaBP + r0 + li];     // B_{s2}[m][r0 + li]
          y[s] = As[(s * 64 + l0 + li) * kThetaMfmaAP + mm];    // A_{s1}[l0 + li][m]
        }
#pragma unroll
        for (int s1 = 0; s1 < 2; ++s1)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2) {
            cr[s1][s2] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s2].x, y[s1].x, cr[s1][s2], 0, 0, 0);
            cr[s1][s2] = __builtin_amdgcn_mfma_f64_16x16x4f64(-x[s2].y, y[s1].y, cr[s1][s2], 0, 0, 0);
            ci[s1][s2] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s2].x, y[s1].y, ci[s1][s2], 0, 0, 0);
            ci[s1][s2] = __builtin_amdgcn_mfma_f64_16x16x4f64(x[s2].y, y[s1].x, ci[s1][s2], 0, 0, 0);
          }
      }
    }
    if (more) stash((c + 1) & 1, na, nb);
    __syncthreads();
  }
  if (active) {
    const int l = l0 + li;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + lk + 4 * q;
      if (l < chl && r < chr) {
        const cplx p0 = aqc::cmk(cr[0][0][q], ci[0][0][q]), p1 = aqc::cmk(cr[0][1][q], ci[0][1][q]);
        const cplx p2 = aqc::cmk(cr[1][0][q], ci[1][0][q]), p3 = aqc::cmk(cr[1][1][q], ci[1][1][q]);
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          cplx v = aqc::cmul(sG[o * 4 + 0], p0);
          v = aqc::cfma(sG[o * 4 + 1], p1, v);
          v = aqc::cfma(sG[o * 4 + 2], p2, v);
          v = aqc::cfma(sG[o * 4 + 3], p3, v);
          aqc::stg(j.theta + (size_t)((o & 1) * chr + r) * M + (o >> 1) * chl + l, v);  // GLOBAL, not FLAT
        }
      }
    }
  }
}

// the register Jacobi is the chain's fallback (Gram path off or refused): a real call, so that
// its register allocation stays out of k_chain's
__device__ __noinline__ void chain_jacobi_fallback(const TwoSiteJob& j) { jacobi_reg_body<128, 8, 16>(j); }
__device__ __forceinline__ void chain_jacobi(const TwoSiteJob& j) {
  if (j.gram) {
    const int g = gram_svd_body(j);
    if (g == 1) return;
    __syncthreads();
    if (g == 2 && gram_certified(j)) return;
  }
  chain_jacobi_fallback(j);
}
__device__ __forceinline__ void chain_rank(const TwoSiteJob& j) { rank_body<1024, 128>(j); }
// The split GEMM in the chain: its output (k x N, or M x k) is two 64 x 64 blocks, so the four
// sub-groups split the contraction length L in halves -- sub-group sg computes block sg >> 1 over
// half sg & 1 -- and the second halves' accumulators meet the first halves' through the LDS.
__device__ __forceinline__ void split_gemm_chain(const TwoSiteJob& j, int tid) {
  extern __shared__ double2 xbuf[];
  const int sg = tid >> 8, lt = tid & 255, blk = sg >> 1, h = sg & 1;
  const int chl = j.dims[0], k = j.dims[1], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = (M < N) != (j.qr != 0);
  const int L = tr ? N : M;
  const int cap = j.cap;
  const size_t half = (size_t)cap * cap;
  const double* ss = j.sig + kSigMax;
  const int rows = tr ? M : k, cols = tr ? k : N;
  const int r0 = tr ? 64 * blk : 0, c0 = tr ? 0 : 64 * blk;
  const bool active = r0 < rows && c0 < cols;
  const int mb = active ? min(64, rows - r0) : 64, nb = active ? min(64, cols - c0) : 64;
  const int kh = ((L + 1) / 2 + 15) & ~15, klo = h * kh;  // both halves run kh (barriers pair up)
  const cplx* W = j.work;
  const int* perm = j.perm;
  const cplx* th = j.theta;
  aqc::GemmLds& lds = reinterpret_cast<aqc::GemmLds*>(xbuf)[sg];
  aqc::d4_t cr[2][2], ci[2][2];
  if (!tr) {
    aqc::block_cgemm_tile<true, true, false>(
        mb, nb, kh, 0, 0,
        [&](int kk, int R) {
          return klo + R < L ? aqc::cconj(aqc::ldg(W + (size_t)perm[r0 + kk] * L + klo + R)) : aqc::cmk(0, 0);
        },
        [&](int R, int c) { return klo + R < L ? aqc::ldg(th + (size_t)(c0 + c) * M + klo + R) : aqc::cmk(0, 0); }, lds, lt,
        active, cr, ci);
  } else {
    aqc::block_cgemm_tile<false, true, false>(
        mb, nb, kh, 0, 0,
        [&](int R, int c) { return klo + c < L ? aqc::ldg(th + (size_t)(klo + c) * M + r0 + R) : aqc::cmk(0, 0); },
        [&](int c, int kk) { return klo + c < L ? aqc::ldg(W + (size_t)perm[c0 + kk] * L + klo + c) : aqc::cmk(0, 0); }, lds,
        lt, active, cr, ci);
  }
  // (block_cgemm_tile ends on a barrier: the staging LDS is free)
  cplx* part = xbuf + blk * (64 * 64);
  const int wave = lt >> 6, lane = lt & 63;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32, li = lane & 15, lk = lane >> 4;
  if (active && h == 1) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          part[(wr + 16 * r + lk + 4 * q) * 64 + wc + 16 * c + li] = aqc::cmk(cr[r][c][q], ci[r][c][q]);
  }
  __syncthreads();
  if (active && h == 0) {
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = wr + 16 * r + lk + 4 * q, jj = wc + 16 * c + li;
          if (i < mb && jj < nb) {
            const cplx o = part[i * 64 + jj];
            const cplx v = aqc::cmk(cr[r][c][q] + o.x, ci[r][c][q] + o.y);
            if (!tr) {  // Gq'[s2][kq][r] = Vh / sig^2 / lr[r]
              const int kq = r0 + i, cc = c0 + jj, s2 = cc / chr, rr = cc % chr;
              const double sk = aqc::ldg(ss + kq), d = sk * sk * aqc::ldg(j.lr + rr);
              aqc::stg(j.gq + s2 * half + (size_t)kq * cap + rr, d != 0.0 ? aqc::cscale(v, 1.0 / d) : aqc::cmk(0, 0));
            } else {  // Gp'[s1][l][kq] = U / sig^2 / ll[l]
              const int Rr = r0 + i, kq = c0 + jj, s1 = Rr / chl, l = Rr % chl;
              const double sk = aqc::ldg(ss + kq), d = sk * sk * aqc::ldg(j.ll + l);
              aqc::stg(j.gp + s1 * half + (size_t)l * cap + kq, d != 0.0 ? aqc::cscale(v, 1.0 / d) : aqc::cmk(0, 0));
            }
          }
        }
  }
}
__device__ __forceinline__ void chain_split(const TwoSiteJob& j) {
  const int tid = fresh_tid();
  split_copy_body(j, tid, 1024);
  split_gemm_chain(j, tid);
}

__global__ __launch_bounds__(1024) void k_chain(const ChainJob* __restrict__ chains, const TwoSiteJob* __restrict__ two,
                                                const OneSiteJob* __restrict__ one) {
  const ChainJob& c = chains[blockIdx.x];
  const int tid = fresh_tid();
  // shader-clock ticks of the phases (thread 0 of each workgroup; aqc_mps_chain_ticks), kept in
  // LDS so that no VGPR stays live across the phases
  __shared__ unsigned long long tk[6];  // 5 phase totals, last tick
  if (tid == 0) tk[0] = tk[1] = tk[2] = tk[3] = tk[4] = tk[5] = 0;
  auto tick = [&](int ph) {
    if (tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (ph >= 0) tk[ph] += t - tk[5];
      tk[5] = t;
    }
  };
  tick(-1);
  for (int o = 0; o < c.nops; ++o) {
    // wave-uniform (SGPR) op code, so the job's fields are scalar loads and hold no VGPRs
    const int code = __builtin_amdgcn_readfirstlane(c.ops[o]);
    if (code < 0) {
      one_site_body(one[-code - 1], tid, 1024);
      __syncthreads();
      tick(4);
      continue;
    }
    const TwoSiteJob& j = two[code];
#if AQC_THETA_MFMA
    chain_theta_mfma(j);
#else
    chain_theta(j);
#endif
    __syncthreads();
    tick(0);
    chain_jacobi(j);
    __syncthreads();
    tick(1);
    chain_rank(j);
    __syncthreads();
    tick(2);
    chain_split(j);
    __syncthreads();
    tick(3);
  }
  if (tid == 0)
    for (int ph = 0; ph < 5; ++ph) atomicAdd(&g_chain_ticks[ph], tk[ph]);
}

// ---- measurements -------------------------------------------------------------------------
struct MeasJob {
  const cplx* gam;
  const double* lam;
  const int* dims;
  int n;
  int cap;
  cplx* out;
  cplx* vec;   // zero-chain scratch (2*(n+1)*cap)
  cplx* env;   // env scratch
  cplx* tmp;   // 2*cap*cap
};

__device__ __forceinline__ cplx site_a(const cplx* gam, const double* lam, int cap, int i, int s, int l,
                                        int r) {
  // A_i[s][l][r] = Gamma_i[s][l][r] * lambda_{i+1}[r]  (aqc_research _preprocess_mps)
  const size_t ss = (size_t)2 * cap * cap;
  return aqc::cscale(gam[(size_t)i * ss + (size_t)s * cap * cap + (size_t)l * cap + r],
                     lam[(size_t)(i + 1) * cap + r]);
}

// <0...0|psi>: v <- v A_i[0] from the left.  One workgroup per state.
// The running vectors in dynamic LDS sized by the batch's largest capacity (vc complex each): at
// capacity-1024 static arrays (48 KB) three of the bench's four workgroups per CU fit and its 1024
// states ran in two rounds (483 -> 761 us a launch).
__global__ __launch_bounds__(kT) void k_overlap_zero(const MeasJob* __restrict__ jobs, int vc) {
  const MeasJob& j = jobs[blockIdx.x];
  extern __shared__ cplx ovz_lds[];
  
  __shared__ cplx part[4][256];
  const int tid = fresh_tid();
  if (tid == 0) ovz_lds[0] = aqc::cmk(1.0, 0.0);
  __syncthreads();
  int cur = 0;
  const int q = tid >> 6, lane = tid & 63;
  for (int i = 0; i < j.n; ++i) {
    const int cl = j.dims[i], cr = j.dims[i + 1];
    for (int r0 = 0; r0 < cr; r0 += 64) {
      const int r = r0 + lane;
      cplx acc = aqc::cmk(0, 0);
      if (r < cr)
        for (int l = q; l < cl; l += 4) acc = aqc::cfma(ovz_lds[cur * vc + l], site_a(j.gam, j.lam, j.cap, i, 0, l, r), acc);
      part[q][lane + 0] = acc;
      __syncthreads();
      if (q == 0 && r < cr)
        ovz_lds[(cur ^ 1) * vc + r] = aqc::cadd(aqc::cadd(part[0][lane], part[1][lane]), aqc::cadd(part[2][lane], part[3][lane]));
      __syncthreads();
    }
    cur ^= 1;
  }
  if (tid == 0) j.out[0] = ovz_lds[cur * vc];
}

// Zero chains: vec[b] (left, bond b) = <0..0| A_0..A_{b-1};  vec[(n+1)+b] (right) = A_b..A_{n-1}|0..0>.
// blockIdx.y = 0 -> left chain, 1 -> right chain.  The running vector in the LDS; the left chain as
// k_overlap_zero (lanes along r, the four waves splitting l), the right one with lanes along r too
// (coalesced rows of A) and one wave sum per output row.  (Round 6: one thread per output entry
// with the whole dot product and the vector in global memory, columns of A read with a cap stride,
// made the softened-cost batch's HW-1 amplitudes ~2 ms a call.)
__global__ __launch_bounds__(kT) void k_zero_chains(const MeasJob* __restrict__ jobs, int vc) {
  const MeasJob& j = jobs[blockIdx.x];
  const int tid = fresh_tid(), q = tid >> 6, lane = tid & 63;
  const int cap = j.cap, n = j.n;
  cplx* L = j.vec;
  cplx* R = j.vec + (size_t)(n + 1) * cap;
  extern __shared__ cplx ovz_lds[];  // (as k_overlap_zero)
  
  __shared__ cplx part[4][64];
  if (tid == 0) ovz_lds[0] = aqc::cmk(1.0, 0.0);
  int cur = 0;
  if (blockIdx.y == 0) {
    if (tid == 0) L[0] = aqc::cmk(1.0, 0.0);
    __syncthreads();
    for (int i = 0; i < n; ++i) {
      const int cl = j.dims[i], cr = j.dims[i + 1];
      for (int r0 = 0; r0 < cr; r0 += 64) {
        const int r = r0 + lane;
        cplx acc = aqc::cmk(0, 0);
        if (r < cr)
          for (int l = q; l < cl; l += 4) acc = aqc::cfma(ovz_lds[cur * vc + l], site_a(j.gam, j.lam, cap, i, 0, l, r), acc);
        part[q][lane] = acc;
        __syncthreads();
        if (q == 0 && r < cr) {
          const cplx s = aqc::cadd(aqc::cadd(part[0][lane], part[1][lane]), aqc::cadd(part[2][lane], part[3][lane]));
          ovz_lds[(cur ^ 1) * vc + r] = s;
          L[(size_t)(i + 1) * cap + r] = s;
        }
        __syncthreads();
      }
      cur ^= 1;
    }
  } else {
    if (tid == 0) R[(size_t)n * cap] = aqc::cmk(1.0, 0.0);
    __syncthreads();
    for (int i = n - 1; i >= 0; --i) {
      const int cl = j.dims[i], cr = j.dims[i + 1];
      for (int l = q; l < cl; l += 4) {  // (uniform per wave)
        cplx acc = aqc::cmk(0, 0);
        for (int r = lane; r < cr; r += 64) acc = aqc::cfma(site_a(j.gam, j.lam, cap, i, 0, l, r), ovz_lds[cur * vc + r], acc);
        acc.x = wave_sum_d(acc.x);
        acc.y = wave_sum_d(acc.y);
        if (lane == 0) {
          ovz_lds[(cur ^ 1) * vc + l] = acc;
          R[(size_t)i * cap + l] = acc;
        }
      }
      __syncthreads();
      cur ^= 1;
    }
  }
}

// amp_i = <e_i|psi> = L[i] A_i[1] R[i+1].  blockIdx.x = site, blockIdx.y = job.
__global__ __launch_bounds__(kT) void k_hw1(const MeasJob* __restrict__ jobs) {
  const MeasJob& j = jobs[blockIdx.y];
  const int i = blockIdx.x;
  const int cap = j.cap, n = j.n;
  if (i >= n) return;
  const cplx* L = j.vec + (size_t)i * cap;
  const cplx* R = j.vec + (size_t)(n + 1) * cap + (size_t)(i + 1) * cap;
  const int cl = j.dims[i], cr = j.dims[i + 1];
  __shared__ double red[2][kT];
  cplx acc = aqc::cmk(0, 0);
  for (int e = threadIdx.x; e < cl * cr; e += kT) {
    const int l = e / cr, r = e % cr;
    acc = aqc::cfma(aqc::cmul(L[l], site_a(j.gam, j.lam, cap, i, 1, l, r)), R[r], acc);
  }
  red[0][threadIdx.x] = acc.x;
  red[1][threadIdx.x] = acc.y;
  __syncthreads();
  for (int s = kT / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) j.out[i] = aqc::cmk(red[0][0], red[1][0]);
}

// ---- zero and Hamming-weight-1 amplitudes through a window (round 6) --------------------------
// The global cost's <0|psi> and the softened cost's <e_i|psi> (aer_mps_backend.py:49-70, 88-93)
// are linear in every site tensor.  Rows from the left, per bond b: row 0 = <0..0| A_0 .. A_{b-1}
// (all sites on 0), row 1 + k = the same with site k < b on 1; from the right: row 0 =
// A_b .. A_{n-1} |0..0>, row 1 + k = with site k >= b on 1.  A Rotoselect candidate differs from
// the prefix only on the sites lo..hi it rewrote, so with the prefix's left rows at bond lo (Ml) and
// right rows at bond hi + 1 (Nr), cached on the prefix handle, and the candidate's own row-0
// vectors through the window, u_b (from Ml[0], bonds lo .. hi + 1) and y_b (from Nr[0], bonds
// hi + 1 .. lo):
//   <0|psi> = u_b . y_b (any window bond: the two chains meet in the middle when only it is asked)
//   amp_k   = Ml[1 + k] . y_lo (k < lo),  u_k A_k[1] y_{k+1} (lo <= k <= hi),  u_{hi+1} . Nr[1 + k] (k > hi)
// -- w small vector steps per candidate instead of two n-step chains and n closings.
//
// One vector step for up to kHwR vectors at once (the same site): left out_r[c] = sum_l v_r[l] A_t[l][c],
// right out_r[l] = sum_c A_t[l][c] v_r[c].  The four waves split the contraction, lanes run over
// 64 outputs, partial sums meet in the LDS (two barriers per 64 outputs); t = 1 for the rows
// flagged in newmask (the flipped site), A_0 otherwise.  src(r, k), dst(r, x, value).
constexpr int kHwR = 8;
template <typename FS, typename FD>
__device__ __forceinline__ void hw_step(const cplx* gam, const double* lam, int cap, int i, bool right, int nrows,
                                        unsigned newmask, int ke, int m2, FS src, FD dst, cplx (*part)[kHwR][64]) {
  const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t cc = (size_t)cap * cap;
  const cplx* g = gam + (size_t)i * 2 * cc;
  const double* lm = lam + (size_t)(i + 1) * cap;
  for (int x0 = 0; x0 < m2; x0 += 64) {
    const int x = x0 + lane;
    cplx acc[kHwR];
#pragma unroll
    for (int r = 0; r < kHwR; ++r) acc[r] = aqc::cmk(0, 0);
    if (x < m2) {
      for (int k = q; k < ke; k += 4) {
        // A_t[l][c] = Gamma_t[l][c] lambda_{i+1}[c]: left (l, c) = (k, x), right (x, k)
        const size_t o = right ? (size_t)x * cap + k : (size_t)k * cap + x;
        const double lv = lm[right ? k : x];
        const cplx a0 = aqc::cscale(g[o], lv);
        const cplx a1 = newmask ? aqc::cscale(g[cc + o], lv) : a0;
#pragma unroll
        for (int r = 0; r < kHwR; ++r)
          if (r < nrows) acc[r] = aqc::cfma(src(r, k), (newmask >> r) & 1 ? a1 : a0, acc[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < kHwR; ++r)
      if (r < nrows) part[q][r][lane] = acc[r];
    __syncthreads();
    for (int e = threadIdx.x; e < nrows * 64; e += kT) {
      const int r = e >> 6, ln = e & 63;
      if (x0 + ln < m2)
        dst(r, x0 + ln, aqc::cadd(aqc::cadd(part[0][r][ln], part[1][r][ln]), aqc::cadd(part[2][r][ln], part[3][r][ln])));
    }
    __syncthreads();
  }
}

struct HwRowsJob {
  const cplx* gam;
  const double* lam;
  const int* dims;
  int n, cap;
  int dir, first, nsteps;  // left: sites first .. first + nsteps - 1; right: first down
  int full;                // every row, or row 0 only
  cplx* rows;              // bond b's (n + 1) x cap block at rows + b (n + 1) cap
};

// The prefix's rows.  grid (directions, G): with `full`, workgroup g owns the flip rows 1 + k with
// k % G == g (each an independent chain once created) and every workgroup carries row 0 itself
// (workgroup 0 stores it), so the workgroups never wait on each other.  Every bond has its own
// block, written once per launch and read by the next step only (no stale L1 line); row 0 is also
// kept in the LDS.
constexpr int kHwRowsG = 8;
__global__ __launch_bounds__(kT) void k_hw_rows(const HwRowsJob* __restrict__ jobs) {
  const HwRowsJob& j = jobs[blockIdx.x];
  const int n = j.n, cap = j.cap, g = blockIdx.y, G = gridDim.y;
  const size_t blk = (size_t)(n + 1) * cap;
  extern __shared__ cplx hw_lds[];
  cplx* v0[2] = {hw_lds, hw_lds + cap};  // row 0, this workgroup's copy
  cplx (*part)[kHwR][64] = reinterpret_cast<cplx (*)[kHwR][64]>(hw_lds + 2 * cap);
  {
    const int b = j.dir == 0 ? j.first : j.first + 1, d = j.dims[b];
    for (int e = threadIdx.x; e < d; e += kT) v0[0][e] = j.rows[(size_t)b * blk + e];
  }
  __syncthreads();
  for (int s = 0; s < j.nsteps; ++s) {
    const int i = j.dir == 0 ? j.first + s : j.first - s;
    const bool right = j.dir != 0;
    const int ke = right ? j.dims[i + 1] : j.dims[i], m2 = right ? j.dims[i] : j.dims[i + 1];
    const cplx* M = j.rows + (size_t)(right ? i + 1 : i) * blk;
    cplx* O = j.rows + (size_t)(right ? i : i + 1) * blk;
    const cplx* v = v0[s & 1];
    cplx* vn = v0[(s + 1) & 1];
    // this workgroup's rows: 0; the old flip rows k (left: k < i, right: k > i) with k % G == g;
    // the new row 1 + i (from row 0 with the site on 1) when i % G == g
    int k0 = 0, nold = 0;
    if (j.full) {
      if (!right) nold = i > g ? (i - g + G - 1) / G : 0, k0 = g;
      else {
        k0 = i + 1 + ((g - (i + 1) % G) % G + G) % G;
        nold = k0 < n ? (n - 1 - k0) / G + 1 : 0;
      }
    }
    const int nnew = j.full && i % G == g ? 1 : 0, nr = 1 + nold + nnew;
    // row list position p: 0 = row 0, 1 .. nold = old rows, nold + 1 = the new row
    auto row_of = [&](int p) { return p == 0 ? 0 : (p <= nold ? 1 + k0 + G * (p - 1) : 1 + i); };
    for (int p0 = 0; p0 < nr; p0 += kHwR) {
      const int cnt = min(kHwR, nr - p0);
      const unsigned nm = (nnew && nr - 1 >= p0 && nr - 1 < p0 + cnt) ? 1u << (nr - 1 - p0) : 0u;
      hw_step(
          j.gam, j.lam, cap, i, right, cnt, nm, ke, m2,
          [&](int r, int k) {
            const int p = p0 + r;
            return (p == 0 || p == nold + 1) ? v[k] : M[(size_t)row_of(p) * cap + k];
          },
          [&](int r, int x, cplx val) {
            const int p = p0 + r;
            if (p == 0) vn[x] = val;
            if (p != 0 || g == 0) O[(size_t)row_of(p) * cap + x] = val;
          },
          part);
    }
  }
}

struct HwWinJob {
  const cplx* gam;
  const double* lam;
  const int* dims;
  int n, cap, lo, hi;
  const cplx* ml;  // prefix's left rows at bond lo
  const cplx* nr;  // prefix's right rows at bond hi + 1
  cplx* ov;        // <0..0|psi> (the amplitude; the host conjugates for mps_dot(psi, zero))
  cplx* amps;      // n amplitudes, or nullptr
  cplx* uy;        // with amps: u_b at uy + (b - lo) cap, y_b at uy + (w + 1 + b - lo) cap
  cplx* fin;       // the two chains' last vectors (2 cap): u at fin, y at fin + cap
  int* cnt;        // the job's hand-off counter (0 at launch)
  int pad;
};

// Vectors handed between the two chains' workgroups (possibly on different XCDs): agent-scope
// stores and loads, as the environment chains' hand-offs (ent.hip)
typedef __attribute__((address_space(1))) double win_gdbl;
__device__ __forceinline__ void win_st(cplx* p, cplx v) {
  win_gdbl* q = (win_gdbl*)(double*)p;
  __hip_atomic_store(q, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ cplx win_ld(const cplx* p) {
  win_gdbl* q = (win_gdbl*)(double*)p;
  return aqc::cmk(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                  __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// One window step with the running vector v in the LDS (out in the LDS too, and to `store` when
// not null).  Left (site i, bond i -> i + 1): out[x] = sum_k v[k] A_i[0][k][x] -- lanes along x
// (coalesced rows of Gamma), the four waves splitting k, partial sums through the LDS.  Right (bond
// i + 1 -> i): out[x] = sum_k A_i[0][x][k] v[k] -- lanes along k (coalesced rows again), four
// outputs per wave in flight, wave sums.  A = Gamma lambda_{i+1}.
__device__ __forceinline__ void win_step(const cplx* __restrict__ gam, const double* __restrict__ lam, int cap, int i,
                                         bool right, int ke, int m2, const cplx* v, cplx* out, cplx* store,
                                         cplx (*part)[64]) {
  const int q = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const cplx* g = gam + (size_t)i * 2 * cap * cap;
  const double* lm = lam + (size_t)(i + 1) * cap;
  if (!right) {
    for (int x0 = 0; x0 < m2; x0 += 64) {
      const int x = x0 + lane;
      cplx acc = aqc::cmk(0, 0);
      if (x < m2) {
        int k = q;
        for (; k + 12 < ke; k += 16) {  // four rows' loads issued together
          cplx a[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) a[t] = g[(size_t)(k + 4 * t) * cap + x];
#pragma unroll
          for (int t = 0; t < 4; ++t) acc = aqc::cfma(v[k + 4 * t], a[t], acc);
        }
        for (; k < ke; k += 4) acc = aqc::cfma(v[k], g[(size_t)k * cap + x], acc);
        acc = aqc::cscale(acc, lm[x]);
      }
      part[q][lane] = acc;
      __syncthreads();
      if (q == 0 && x < m2) {
        const cplx r = aqc::cadd(aqc::cadd(part[0][lane], part[1][lane]), aqc::cadd(part[2][lane], part[3][lane]));
        out[x] = r;
        if (store) win_st(store + x, r);
      }
      __syncthreads();
    }
  } else {
    for (int x0 = 4 * q; x0 < m2; x0 += 16) {  // (uniform per wave)
      // (four named sums: as an array the compiler kept them in scratch)
      cplx c0 = aqc::cmk(0, 0), c1 = c0, c2 = c0, c3 = c0;
      const bool h1 = x0 + 1 < m2, h2 = x0 + 2 < m2, h3 = x0 + 3 < m2;
      for (int k = lane; k < ke; k += 64) {
        const cplx vk = aqc::cscale(v[k], lm[k]);
        const cplx* gk = g + (size_t)x0 * cap + k;
        c0 = aqc::cfma(gk[0], vk, c0);
        if (h1) c1 = aqc::cfma(gk[cap], vk, c1);
        if (h2) c2 = aqc::cfma(gk[2 * (size_t)cap], vk, c2);
        if (h3) c3 = aqc::cfma(gk[3 * (size_t)cap], vk, c3);
      }
      c0.x = wave_sum_d(c0.x), c0.y = wave_sum_d(c0.y);
      c1.x = wave_sum_d(c1.x), c1.y = wave_sum_d(c1.y);
      c2.x = wave_sum_d(c2.x), c2.y = wave_sum_d(c2.y);
      c3.x = wave_sum_d(c3.x), c3.y = wave_sum_d(c3.y);
      if (lane < 4 && x0 + lane < m2) {
        cplx r = c0;
        if (lane == 1) r = c1;
        if (lane == 2) r = c2;
        if (lane == 3) r = c3;
        out[x0 + lane] = r;
        if (store) win_st(store + x0 + lane, r);
      }
    }
    __syncthreads();
  }
}

// Two workgroups per state (blockIdx.y): the left chain u through sites lo .. lo + nl - 1 (bond lo
// -> lo + nl) and the right chain y through hi .. hi - ny + 1 (bond hi + 1 -> hi + 1 - ny) run side
// by side; without amplitudes they meet at bond lo + nl, with them both run the whole window.
// Each writes its last vector to fin; the second to finish (the job's counter) closes: <0|psi> =
// u . y and, with amps, the window's amplitudes from the bond vectors in uy (every vector written
// once to global memory before the hand-off, read after it).  Dynamic LDS: two vectors (2 cap)
// and the step partials.  (One workgroup running the two chains one step after the other: ~190 us
// a launch in the paper-setting layer, lanes strided by cap on the right chain's rows.)
__global__ __launch_bounds__(kT) void k_hw_win(const HwWinJob* __restrict__ jobs) {
  const HwWinJob& j = jobs[blockIdx.x];
  const int side = blockIdx.y;
  extern __shared__ cplx hw_lds[];
  const int cap = j.cap, n = j.n, lo = j.lo, hi = j.hi, w = hi - lo + 1;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  cplx (*part)[64] = reinterpret_cast<cplx (*)[64]>(hw_lds + 2 * cap);
  const bool amps = j.amps != nullptr;
  const int nl = amps ? w : (w + 1) / 2, ny = amps ? w : w - nl;
  cplx* U = j.uy;
  cplx* Y = j.uy + (size_t)(w + 1) * cap;
  const int steps = side == 0 ? nl : ny;
  {
    const int d0 = side == 0 ? j.dims[lo] : j.dims[hi + 1];
    const cplx* src = side == 0 ? j.ml : j.nr;
    cplx* st0 = amps ? (side == 0 ? U : Y + (size_t)w * cap) : nullptr;
    for (int e = tid; e < d0; e += kT) {
      hw_lds[e] = src[e];
      if (st0) win_st(st0 + e, src[e]);
    }
  }
  __syncthreads();
  if (cap <= 64) {
    // capacity <= 64: a step's whole 64 x 64 tile is 16 entries per thread, all loaded at once --
    // and the next step's issued before this step's products (the tiles do not depend on the
    // running vector), so a step waits on no global load.  Left: thread (q, x) holds A[q + 4t][x];
    // right: thread (q, k) holds A[q + 4t][k] (rows along the lanes either way: coalesced), its 16
    // products reduced over k through the LDS (red, 64 x 65).
    cplx (*red)[65] = reinterpret_cast<cplx (*)[65]>(hw_lds + 2 * cap + 4 * 64);
    auto site_of = [&](int s) { return side == 0 ? lo + s : hi - s; };
    auto fetch = [&](int s, cplx (&a)[16]) {
      const int i = site_of(s);
      const int rows = side == 0 ? j.dims[i] : j.dims[i];      // A's row count (left: k; right: x)
      const int cols = side == 0 ? j.dims[i + 1] : j.dims[i + 1];
      const cplx* g = j.gam + (size_t)i * 2 * cap * cap;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int r = wave + 4 * t;
        a[t] = (r < rows && lane < cols) ? g[(size_t)r * cap + lane] : aqc::cmk(0, 0);
      }
    };
    cplx a[16], an[16];
    if (steps > 0) fetch(0, a);
    for (int s = 0; s < steps; ++s) {
      if (s + 1 < steps) fetch(s + 1, an);
      const int i = site_of(s);
      const cplx* v = hw_lds + (s & 1) * cap;
      cplx* vn = hw_lds + ((s + 1) & 1) * cap;
      const double* lm = j.lam + (size_t)(i + 1) * cap;
      if (side == 0) {  // out[x] = lambda[x] sum_k v[k] A[k][x], x = lane
        const int ke = j.dims[i], m2 = j.dims[i + 1];
        cplx acc = aqc::cmk(0, 0);
#pragma unroll
        for (int t = 0; t < 16; ++t)
          if (wave + 4 * t < ke) acc = aqc::cfma(v[wave + 4 * t], a[t], acc);
        part[wave][lane] = acc;
        __syncthreads();
        if (wave == 0 && lane < m2) {
          const cplx r = aqc::cscale(aqc::cadd(aqc::cadd(part[0][lane], part[1][lane]), aqc::cadd(part[2][lane], part[3][lane])),
                                     lm[lane]);
          vn[lane] = r;
          if (amps) win_st(U + (size_t)(s + 1) * cap + lane, r);
        }
      } else {  // out[x] = sum_k A[x][k] lambda[k] v[k], k = lane
        const int ke = j.dims[i + 1], m2 = j.dims[i];
        const cplx vk = lane < ke ? aqc::cscale(v[lane], lm[lane]) : aqc::cmk(0, 0);
#pragma unroll
        for (int t = 0; t < 16; ++t) red[wave + 4 * t][lane] = aqc::cmul(a[t], vk);
        __syncthreads();
        {  // thread (x = tid / 4, quarter p = tid % 4): 16 k's, then the four quarters by shuffles
          const int x = tid >> 2, p = tid & 3;
          cplx acc = aqc::cmk(0, 0);
#pragma unroll
          for (int c = 0; c < 16; ++c) acc = aqc::cadd(acc, red[x][16 * p + c]);
          acc.x += __shfl_xor(acc.x, 1);
          acc.y += __shfl_xor(acc.y, 1);
          acc.x += __shfl_xor(acc.x, 2);
          acc.y += __shfl_xor(acc.y, 2);
          if (p == 0 && x < m2) {
            vn[x] = acc;
            if (amps) win_st(Y + (size_t)(i - lo) * cap + x, acc);
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < 16; ++t) a[t] = an[t];
    }
  } else
  for (int s = 0; s < steps; ++s) {
    const cplx* v = hw_lds + (s & 1) * cap;
    cplx* vn = hw_lds + ((s + 1) & 1) * cap;
    if (side == 0) {
      const int i = lo + s;
      win_step(j.gam, j.lam, cap, i, false, j.dims[i], j.dims[i + 1], v, vn, amps ? U + (size_t)(s + 1) * cap : nullptr,
               part);
    } else {
      const int i = hi - s;
      win_step(j.gam, j.lam, cap, i, true, j.dims[i + 1], j.dims[i], v, vn, amps ? Y + (size_t)(i - lo) * cap : nullptr,
               part);
    }
  }
  {
    const cplx* v = hw_lds + (steps & 1) * cap;
    const int d = side == 0 ? j.dims[lo + nl] : j.dims[hi + 1 - ny];
    for (int e = tid; e < d; e += kT) win_st(j.fin + (size_t)side * cap + e, v[e]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (tid == 0) last = __hip_atomic_fetch_add(j.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1;
  __syncthreads();
  if (!last) return;
  const cplx* u = j.fin;        // at bond lo + nl
  const cplx* y = j.fin + cap;  // at bond hi + 1 - ny
  const int dl = j.dims[lo], dr = j.dims[hi + 1];
  // closings, a wave per output, lanes along the bond: output 0 = <0|psi>, 1 + k = amp_k (with
  // amps; window sites as u_k A_k[1] y_{k+1}: lanes along the right index, a loop over the left)
  const int nout = amps ? n + 1 : 1;
  for (int o = wave; o < nout; o += kT / 64) {  // (uniform per wave)
    const int k = o - 1;
    cplx acc = aqc::cmk(0, 0);
    if (o == 0) {  // (with amps u is at bond hi + 1: against Nr[0]; else the chains' meeting bond)
      const cplx* yy = amps ? j.nr : y;
      const int d = j.dims[lo + nl];
      for (int c = lane; c < d; c += 64) acc = aqc::cfma(win_ld(u + c), amps ? yy[c] : win_ld(yy + c), acc);
    } else if (k < lo) {
      for (int c = lane; c < dl; c += 64) acc = aqc::cfma(j.ml[(size_t)(1 + k) * cap + c], win_ld(y + c), acc);
    } else if (k > hi) {
      for (int c = lane; c < dr; c += 64) acc = aqc::cfma(win_ld(u + c), j.nr[(size_t)(1 + k) * cap + c], acc);
    } else {
      const cplx* uk = U + (size_t)(k - lo) * cap;
      const cplx* yk = Y + (size_t)(k + 1 - lo) * cap;
      const int kl = j.dims[k], kr = j.dims[k + 1];
      for (int r = lane; r < kr; r += 64) {
        cplx t = aqc::cmk(0, 0);
        for (int l = 0; l < kl; ++l) t = aqc::cfma(win_ld(uk + l), site_a(j.gam, j.lam, cap, k, 1, l, r), t);
        acc = aqc::cfma(t, win_ld(yk + r), acc);
      }
    }
    acc.x = wave_sum_d(acc.x);
    acc.y = wave_sum_d(acc.y);
    if (lane == 0) {
      if (o == 0) j.ov[0] = acc;
      else j.amps[k] = acc;
    }
  }
}

// Transfer-matrix environments of <a|b> (one workgroup per chain):
//   left : E_{i+1}[ra][rb] = sum_s sum_{la,lb} conj(A_i[s][la][ra]) E_i[la][lb] B_i[s][lb][rb]
//   right: E_i[la][lb]     = sum_s sum_{ra,rb} conj(A_i[s][la][ra]) B_i[s][lb][rb] E_{i+1}[ra][rb]
// With keep_all, every bond's environment is stored (env + b*cap*cap), else only the final one.
struct EnvJob {
  const cplx* ga;
  const double* la;
  const int* da;
  const cplx* gb;
  const double* lb;
  const int* db;
  int n;
  int cap;
  cplx* env;  // (n+1) * cap * cap if keep_all, else 2 * cap*cap ping-pong
  cplx* tmp;  // 2 * cap * cap
  int keep_all;
  int right;
  cplx* out;
};

__global__ __launch_bounds__(kT) void k_env(const EnvJob* __restrict__ jobs) {
  const EnvJob& j = jobs[blockIdx.x];
  const int tid = fresh_tid();
  const int cap = j.cap, n = j.n;
  const size_t cc = (size_t)cap * cap;
  auto envp = [&](int b) -> cplx* { return j.keep_all ? j.env + (size_t)b * cc : j.env + (size_t)(b & 1) * cc; };
  if (!j.right) {
    if (tid == 0) envp(0)[0] = aqc::cmk(1.0, 0.0);
    __syncthreads();
    for (int i = 0; i < n; ++i) {
      const int la = j.da[i], ra = j.da[i + 1], lb = j.db[i], rb = j.db[i + 1];
      const cplx* E = envp(i);
      cplx* En = envp(i + 1);
      // X[s][la][rb] = sum_lb E[la][lb] B[s][lb][rb]   (X in tmp, ld = cap)
      for (int e = tid; e < 2 * la * rb; e += kT) {
        const int s = e / (la * rb), rem = e % (la * rb), a = rem / rb, c = rem % rb;
        cplx acc = aqc::cmk(0, 0);
        for (int b = 0; b < lb; ++b) acc = aqc::cfma(E[(size_t)a * cap + b], site_a(j.gb, j.lb, cap, i, s, b, c), acc);
        j.tmp[(size_t)s * cc + (size_t)a * cap + c] = acc;
      }
      __syncthreads();
      for (int e = tid; e < ra * rb; e += kT) {
        const int a = e / rb, c = e % rb;
        cplx acc = aqc::cmk(0, 0);
        for (int s = 0; s < 2; ++s)
          for (int x = 0; x < la; ++x)
            acc = aqc::cfmac(site_a(j.ga, j.la, cap, i, s, x, a), j.tmp[(size_t)s * cc + (size_t)x * cap + c], acc);
        En[(size_t)a * cap + c] = acc;
      }
      __syncthreads();
    }
    if (tid == 0 && j.out) j.out[0] = envp(n)[0];
  } else {
    if (tid == 0) envp(n)[0] = aqc::cmk(1.0, 0.0);
    __syncthreads();
    for (int i = n - 1; i >= 0; --i) {
      const int la = j.da[i], ra = j.da[i + 1], lb = j.db[i], rb = j.db[i + 1];
      const cplx* E = envp(i + 1);
      cplx* En = envp(i);
      // Y[s][lb][ra] = sum_rb B[s][lb][rb] E[ra][rb]
      for (int e = tid; e < 2 * lb * ra; e += kT) {
        const int s = e / (lb * ra), rem = e % (lb * ra), b = rem / ra, a = rem % ra;
        cplx acc = aqc::cmk(0, 0);
        for (int c = 0; c < rb; ++c) acc = aqc::cfma(site_a(j.gb, j.lb, cap, i, s, b, c), E[(size_t)a * cap + c], acc);
        j.tmp[(size_t)s * cc + (size_t)b * cap + a] = acc;
      }
      __syncthreads();
      for (int e = tid; e < la * lb; e += kT) {
        const int a = e / lb, b = e % lb;
        cplx acc = aqc::cmk(0, 0);
        for (int s = 0; s < 2; ++s)
          for (int x = 0; x < ra; ++x)
            acc = aqc::cfmac(site_a(j.ga, j.la, cap, i, s, a, x), j.tmp[(size_t)s * cc + (size_t)b * cap + x], acc);
        En[(size_t)a * cap + b] = acc;
      }
      __syncthreads();
    }
    if (tid == 0 && j.out) j.out[0] = envp(0)[0];
  }
}

// ---- host-side scheduling ---------------------------------------------------------------
struct DevOp {
  int kind;  // 1: one-site, 2: two-site (p, p+1)
  int p;
  cplx m[16];
};

inline cplx hc(double r, double i) { return aqc::cmk(r, i); }
// host complex arithmetic without fma(): the x86 host build has no FMA instructions enabled, so
// fma() is a libm call per operation
inline cplx hmul(cplx a, cplx b) { return aqc::cmk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
inline cplx hfma(cplx a, cplx b, cplx c) { return aqc::cmk(c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x); }

void mat2_mul(const cplx* a, const cplx* b, cplx* out) {  // out = a b (2x2)
  cplx t[4];
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 2; ++c)
      t[r * 2 + c] = hfma(a[r * 2 + 1], b[2 + c], hmul(a[r * 2], b[c]));
  std::memcpy(out, t, sizeof(t));
}

struct Scheduler {
  int n;
  std::vector<int>& order;
  std::vector<int>& loc;
  std::vector<cplx> pend;     // 4 per qubit
  std::vector<char> has;
  std::vector<DevOp>& out;

  Scheduler(int n_, std::vector<int>& o, std::vector<int>& l, std::vector<DevOp>& dst)
      : n(n_), order(o), loc(l), pend(4 * n_), has(n_, 0), out(dst) {}

  void swap_sites(int p) {
    DevOp d;
    std::memset(&d, 0, sizeof(d));
    d.kind = 2;
    d.p = p;
    // SWAP in site order: out (s1', s2') = in (s2, s1)
    for (int o = 0; o < 4; ++o) {
      const int s1 = o >> 1, s2 = o & 1;
      const int in = 2 * s2 + s1;
      d.m[o * 4 + in] = hc(1, 0);
    }
    out.push_back(d);
    const int qa = order[p], qb = order[p + 1];
    order[p] = qb;
    order[p + 1] = qa;
    loc[qa] = p + 1;
    loc[qb] = p;
  }

  void one(int q, const double* m) {
    cplx u[4];
    for (int e = 0; e < 4; ++e) u[e] = hc(m[2 * e], m[2 * e + 1]);
    if (!has[q]) {
      std::memcpy(&pend[4 * q], u, sizeof(u));
      has[q] = 1;
    } else {
      mat2_mul(u, &pend[4 * q], &pend[4 * q]);
    }
  }

  void two(int qa, int qb, const double* m) {
    const int pa = loc[qa], pb = loc[qb];
    const int low = std::min(pa, pb), high = std::max(pa, pb);
    for (int i = high; i > low + 1; --i) swap_sites(i - 1);  // change_position(high, low+1)
    cplx M4[16];
    for (int e = 0; e < 16; ++e) M4[e] = hc(m[2 * e], m[2 * e + 1]);
    // fold pending one-qubit gates: M' = M . kron(P_b, P_a)   (index 2*b1 + b0, b0 <-> qa)
    cplx Pa[4] = {hc(1, 0), hc(0, 0), hc(0, 0), hc(1, 0)}, Pb[4] = {hc(1, 0), hc(0, 0), hc(0, 0), hc(1, 0)};
    if (has[qa]) std::memcpy(Pa, &pend[4 * qa], sizeof(Pa));
    if (has[qb]) std::memcpy(Pb, &pend[4 * qb], sizeof(Pb));
    has[qa] = has[qb] = 0;
    cplx K[16];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) K[r * 4 + c] = hmul(Pb[(r >> 1) * 2 + (c >> 1)], Pa[(r & 1) * 2 + (c & 1)]);
    cplx Mf[16];
    for (int r = 0; r < 4; ++r)
      for (int c = 0; c < 4; ++c) {
        cplx acc = hc(0, 0);
        for (int t = 0; t < 4; ++t) acc = hfma(M4[r * 4 + t], K[t * 4 + c], acc);
        Mf[r * 4 + c] = acc;
      }
    // to site order: G[(2 s1' + s2')][(2 s1 + s2)]
    const bool a_low = loc[qa] == low;
    DevOp d;
    std::memset(&d, 0, sizeof(d));
    d.kind = 2;
    d.p = low;
    for (int so = 0; so < 4; ++so)
      for (int si = 0; si < 4; ++si) {
        const int s1o = so >> 1, s2o = so & 1, s1i = si >> 1, s2i = si & 1;
        int ro, ci;
        if (a_low) {  // b0 = s1 (qa), b1 = s2 (qb)
          ro = 2 * s2o + s1o;
          ci = 2 * s2i + s1i;
        } else {  // b0 = s2 (qa), b1 = s1 (qb)
          ro = 2 * s1o + s2o;
          ci = 2 * s1i + s2i;
        }
        d.m[so * 4 + si] = Mf[ro * 4 + ci];
      }
    out.push_back(d);
  }

  void flush() {
    for (int q = 0; q < n; ++q) {
      if (!has[q]) continue;
      DevOp d;
      std::memset(&d, 0, sizeof(d));
      d.kind = 1;
      d.p = loc[q];
      std::memcpy(d.m, &pend[4 * q], 4 * sizeof(cplx));
      out.push_back(d);
      has[q] = 0;
    }
  }

  void sort() {
    for (int left = 0; left < n; ++left) {
      const int pos = loc[left];
      for (int j = pos; j > left; --j) swap_sites(j - 1);
    }
  }
};

// Host-side per-state work (scheduling, job building), optionally over a few threads
// (AQC_HOST_THREADS; f(s) must touch only state s's data).  Default 1: on the MI355X box a batch of
// 1024 states took 0.5 ms to schedule and 0.4 ms to build on one thread, 0.9 + 0.9 ms on eight
// (thread start-up and allocator contention outweigh the ~1 ms of work; AQC_HOST_TIMING=1).
template <class F>
void parallel_states(int ns, F&& f) {
  static const int kThreads = [] {
    const char* e = std::getenv("AQC_HOST_THREADS");
    const int v = e ? std::atoi(e) : 1;
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }();
  const int nt = std::min(kThreads, ns / 32);
  if (nt <= 1) {
    for (int s = 0; s < ns; ++s) f(s);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (int t = 1; t < nt; ++t)
    th.emplace_back([&f, t, nt, ns] {
      for (int s = t; s < ns; s += nt) f(s);
    });
  for (int s = 0; s < ns; s += nt) f(s);
  for (auto& x : th) x.join();
}

bool distinct_handles(aqc_mps_t* hs, int ns) {
  std::unordered_set<const void*> seen;
  seen.reserve(2 * ns);
  for (int s = 0; s < ns; ++s)
    if (!seen.insert(hs[s]).second) return false;
  return true;
}

int validate_ops(aqc_mps_t h, const aqc_op_t* ops, int nops) {
  for (int i = 0; i < nops; ++i) {
    const aqc_op_t& o = ops[i];
    AQC_REQUIRE(o.nq == 1 || o.nq == 2, "aqc_mps_apply: only 1- and 2-qubit ops are supported");
    AQC_REQUIRE(o.q0 >= 0 && o.q0 < h->d.n, "aqc_mps_apply: qubit index out of range");
    if (o.nq == 2) AQC_REQUIRE(o.q1 >= 0 && o.q1 < h->d.n && o.q1 != o.q0, "aqc_mps_apply: bad second qubit");
  }
  return AQC_OK;
}

void schedule(aqc_mps_t h, const aqc_op_t* ops, int nops, bool sort_after, std::vector<DevOp>& out) {
  Scheduler s(h->d.n, h->order, h->loc, out);
  for (int i = 0; i < nops; ++i) {
    if (ops[i].nq == 1) s.one(ops[i].q0, ops[i].m);
    else s.two(ops[i].q0, ops[i].q1, ops[i].m);
  }
  s.flush();
  if (sort_after) s.sort();
}

// Device staging buffers for job arrays (grown on demand, reused across calls).
struct Staging {
  void* dev = nullptr;
  size_t cap = 0;
  void* host = nullptr;
  size_t hcap = 0;
};

int ensure_staging(Staging& st, size_t bytes) {
  if (bytes > st.cap) {
    if (st.dev) hipFree(st.dev);
    st.cap = std::max(bytes, st.cap * 2);
    AQC_HIP_CHECK(hipMalloc(&st.dev, st.cap));
  }
  if (bytes > st.hcap) {
    if (st.host) hipHostFree(st.host);
    st.hcap = std::max(bytes, st.hcap * 2);
    AQC_HIP_CHECK(hipHostMalloc(&st.host, st.hcap, hipHostMallocDefault));
  }
  return AQC_OK;
}

void free_staging(Staging& s) {
  if (s.dev) (void)hipFree(s.dev);
  if (s.host) (void)hipHostFree(s.host);
  s = Staging();
}
Staging g_staging[64];
void release_staging() {
  for (auto& s : g_staging) free_staging(s);
}
Staging& staging() {
  int dev = 0;
  hipGetDevice(&dev);
  aqc::on_finalize(release_staging);
  return g_staging[dev];
}

// Job staging for the gate-application launches: a ring of buffer sets per device, each with an
// event recorded after the launches that read it, so that building the next batch's jobs waits
// only for the set's previous use (four calls back) instead of draining the stream -- the host
// schedules while the GPU still runs the previous work.
struct StagingSet {
  Staging buf;
  hipEvent_t done = nullptr;
  bool pending = false;
};

// A lease on the next set of this device's ring.  It holds the device's staging mutex for its
// lifetime (several host threads may drive one device) and records the set's event on the stream
// on EVERY exit path -- an early error return included -- so the set is never handed out again
// while kernels queued before the error may still read it.
constexpr int kStagingRing = 4;
StagingSet g_stage_sets[64][kStagingRing];
void release_stage_sets() {
  for (auto& dev_sets : g_stage_sets)
    for (auto& s : dev_sets) {
      if (s.done) (void)hipEventDestroy(s.done);
      free_staging(s.buf);
      s.done = nullptr;
      s.pending = false;
    }
}
class StagingLease {
 public:
  explicit StagingLease(hipStream_t st) : st_(st), lk_(mutex_for(device())) {
    static int next[64] = {0};
    const int dev = device();
    aqc::on_finalize(release_stage_sets);
    ss_ = &g_stage_sets[dev][next[dev]];
    next[dev] = (next[dev] + 1) % kStagingRing;
    if (ss_->pending) {
      const hipError_t e = hipEventSynchronize(ss_->done);
      if (e != hipSuccess) {
        aqc::set_error(std::string("staging event wait: ") + hipGetErrorString(e));
        rc_ = AQC_ERR_HIP;
      }
      ss_->pending = false;
    }
  }
  ~StagingLease() {
    if (!ss_->done && hipEventCreateWithFlags(&ss_->done, hipEventDisableTiming) != hipSuccess) {
      hipStreamSynchronize(st_);  // no event: drain instead, so the next user finds the set idle
      return;
    }
    if (hipEventRecord(ss_->done, st_) == hipSuccess) ss_->pending = true;
    else hipStreamSynchronize(st_);
  }
  StagingLease(const StagingLease&) = delete;
  StagingLease& operator=(const StagingLease&) = delete;
  Staging& buf() { return ss_->buf; }
  int rc() const { return rc_; }

  // Sizes the leased set for `bytes`.  A set that must grow brings the whole ring to the new size
  // at once (waiting for the other sets' last uses): grown one set at a time, a workload whose
  // calls per step are not a multiple of the ring's length met a fresh (smaller) set in each of
  // its first four steps, and each growth's hipFree drained the device mid-step.
  int ensure(size_t bytes) {
    Staging& mine = ss_->buf;
    if (bytes <= mine.cap && bytes <= mine.hcap) return AQC_OK;
    const size_t want = std::max({bytes, mine.cap * 2, mine.hcap * 2});
    StagingSet* ring = g_stage_sets[device()];
    for (int i = 0; i < kStagingRing; ++i) {
      StagingSet& s = ring[i];
      if (&s != ss_ && s.pending) {
        AQC_HIP_CHECK(hipEventSynchronize(s.done));
        s.pending = false;
      }
      if (int rc = ensure_staging(s.buf, want)) return rc;
    }
    return AQC_OK;
  }

 private:
  static int device() {
    int dev = 0;
    hipGetDevice(&dev);
    return dev;
  }
  static std::mutex& mutex_for(int dev) {
    static std::mutex m[64];
    return m[dev];
  }
  hipStream_t st_;
  std::unique_lock<std::mutex> lk_;
  StagingSet* ss_ = nullptr;
  int rc_ = AQC_OK;
};

TwoSiteJob make_two(aqc_mps_t h, const DevOp& op, int slot = 0) {
  TwoSiteJob j;
  std::memset(&j, 0, sizeof(j));
  const int p = op.p;
  j.gp = h->d.site(p);
  j.gq = h->d.site(p + 1);
  j.ll = h->d.bond(p);
  j.lm = h->d.bond(p + 1);
  j.lr = h->d.bond(p + 2);
  j.dims = h->d.dims + p;
  if (slot == 0) {
    j.theta = h->d.theta;
    j.work = h->d.work;
    j.sig = h->d.sig;
    j.perm = h->d.perm;
  } else {
    const aqc_mps_s::Slot& sl = h->slots[slot - 1];
    j.theta = sl.theta;
    j.work = sl.work;
    j.sig = sl.sig;
    j.perm = sl.perm;
  }
  j.flags = h->d.flags;
  j.cap = h->d.cap;
  j.max_chi = h->max_chi;
  j.thr = h->thr;
  j.jtol = g_jacobi_tol_factor;
  j.jtiny = g_jacobi_tiny_t;
  j.jnoise = kJacobiNoise;
  j.gram = g_svd_gram;
  std::memcpy(j.G, op.m, sizeof(j.G));
  return j;
}

OneSiteJob make_one(aqc_mps_t h, const DevOp& op) {
  OneSiteJob j;
  std::memset(&j, 0, sizeof(j));
  j.g = h->d.site(op.p);
  j.dims = h->d.dims + op.p;
  j.cap = h->d.cap;
  std::memcpy(j.u, op.m, sizeof(j.u));
  return j;
}

// Run per-state device-op lists in lock-step waves on the MPS stream.
// Extra two-site workspace (theta, W, sigma, perm) of `h` for concurrent updates of one state;
// slot 0 is the handle's own workspace.
int ensure_slots(aqc_mps_t h, int nslots) {
  const size_t cap = h->d.cap;
  while ((int)h->slots.size() + 1 < nslots) {
    aqc_mps_s::Slot sl;
    sl.theta = (cplx*)aqc::dev_alloc(4 * cap * cap * sizeof(cplx));
    sl.work = (cplx*)aqc::dev_alloc(aqc::work_elems(cap) * sizeof(cplx));
    sl.sig = (double*)aqc::dev_alloc(kSigLen * sizeof(double));
    sl.perm = (int*)aqc::dev_alloc(kSigMax * sizeof(int));
    if (!sl.theta || !sl.work || !sl.sig || !sl.perm) {
      aqc::dev_free(sl.theta), aqc::dev_free(sl.work), aqc::dev_free(sl.sig), aqc::dev_free(sl.perm);
      aqc::set_error("ensure_slots: out of device memory");
      return AQC_ERR_NOMEM;
    }
    AQC_HIP_CHECK(hipMemsetAsync(sl.sig, 0, kSigLen * sizeof(double), aqc::mps_stream()));
    h->slots.push_back(sl);
  }
  return AQC_OK;
}

// Level each state's device-op list: an op goes one level after the last op touching one of its
// sites.  Two-site updates at p and q with |p - q| >= 2 touch disjoint sites and bonds (the update
// at p reads lambda_p, lambda_{p+1}, lambda_{p+2} and writes Gamma_p, Gamma_{p+1}, lambda_{p+1}),
// so they commute exactly -- truncation included -- and one brickwork layer becomes one wave.
std::vector<std::vector<const DevOp*>> level_ops(const std::vector<DevOp>& ops, int n) {
  std::vector<int> last(n + 1, -1);
  std::vector<std::vector<const DevOp*>> lv;
  for (const DevOp& op : ops) {
    int l;
    if (op.kind == 2) {
      l = std::max(last[op.p], last[op.p + 1]) + 1;
      last[op.p] = last[op.p + 1] = l;
    } else {
      l = last[op.p] + 1;
      last[op.p] = l;
    }
    if ((int)lv.size() <= l) lv.resize(l + 1);
    lv[l].push_back(&op);
  }
  return lv;
}

// Batches at 2 chi = 128: every state's op list runs in one k_chain workgroup (longest lists
// first, so that the short ones fill in behind them).
int run_chains(aqc_mps_t* hs, int ns, std::vector<std::vector<DevOp>>& lists, int cap_max) {
  hipStream_t st = aqc::mps_stream();
  // per-state job counts -> offsets, then every state's jobs written straight into the staging
  // buffer (states in parallel)
  std::vector<size_t> off2(ns + 1, 0), off1(ns + 1, 0), offc(ns + 1, 0);
  for (int s = 0; s < ns; ++s) {
    size_t n2 = 0;
    for (const DevOp& op : lists[s]) n2 += op.kind == 2;
    off2[s + 1] = off2[s] + n2;
    off1[s + 1] = off1[s] + (lists[s].size() - n2);
    offc[s + 1] = offc[s] + lists[s].size();
  }
  const size_t n_two = off2[ns], n_one = off1[ns], n_codes = offc[ns];
  if (n_codes == 0) return AQC_OK;
  std::vector<int> order(ns);
  for (int s = 0; s < ns; ++s) order[s] = s;
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return lists[a].size() > lists[b].size(); });
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_two = 0, o_one = al(o_two + n_two * sizeof(TwoSiteJob));
  const size_t o_codes = al(o_one + n_one * sizeof(OneSiteJob));
  const size_t o_chain = al(o_codes + n_codes * sizeof(int));
  const size_t total = o_chain + (size_t)ns * sizeof(ChainJob);
  StagingLease lease(st);
  if (lease.rc() != AQC_OK) return lease.rc();
  Staging& sg = lease.buf();
  int rc = lease.ensure(total);
  if (rc != AQC_OK) return rc;
  char* hb = (char*)sg.host;
  char* db = (char*)sg.dev;
  TwoSiteJob* h2 = (TwoSiteJob*)(hb + o_two);
  OneSiteJob* h1 = (OneSiteJob*)(hb + o_one);
  int* hcode = (int*)(hb + o_codes);
  parallel_states(ns, [&](int s) {
    size_t i2 = off2[s], i1 = off1[s], ic = offc[s];
    for (const DevOp& op : lists[s]) {
      if (op.kind == 2) {
        h2[i2] = make_two(hs[s], op, 0);
        h2[i2].qr = 1;
        hcode[ic++] = (int)i2++;
        std::vector<int>& ub = hs[s]->ub;  // the host bond bounds (run_waves)
        int nb = std::min(2 * std::min(ub[op.p], ub[op.p + 2]), hs[s]->d.cap);
        if (hs[s]->max_chi > 0) nb = std::min(nb, hs[s]->max_chi);
        ub[op.p + 1] = std::max(nb, 1);
      } else {
        h1[i1] = make_one(hs[s], op);
        hcode[ic++] = -(int)(++i1);
      }
    }
  });
  ChainJob* hc = (ChainJob*)(hb + o_chain);
  for (int k = 0; k < ns; ++k) {
    const int s = order[k];
    hc[k].ops = (const int*)(db + o_codes) + offc[s];
    hc[k].nops = (int)lists[s].size();
    hc[k].pad = 0;
  }
  if (int e = aqc::upload_async(sg.dev, sg.host, total, st)) return e;
  const double c = cap_max, nj = (double)n_two;
  // algorithmic: the two sites' Gammas in and out; nominal SVD + theta + split flops
  aqc::KernelTimer::begin(st, "mps_chain", nj * 8.0 * c * c * 16, nj * (84.0 * 8.0 + 64.0) * c * c * c);
  hipLaunchKernelGGL(k_chain, dim3(ns), dim3(1024), kChainLds, st, (const ChainJob*)(db + o_chain),
                     (const TwoSiteJob*)(db + o_two), (const OneSiteJob*)(db + o_one));
  aqc::KernelTimer::end(st);
  AQC_CHECK_LAUNCH();
  return AQC_OK;  // the lease records the set's event
}

int run_waves(aqc_mps_t* hs, int ns, std::vector<std::vector<DevOp>>& lists) {
  for (int s = 0; s < ns; ++s) {  // every Gamma these lists write (reload bookkeeping)
    int lo = 1 << 30, hi = -1;
    for (const DevOp& op : lists[s]) {
      lo = std::min(lo, op.p);
      hi = std::max(hi, op.kind == 2 ? op.p + 1 : op.p);
    }
    if (hi >= 0) hs[s]->changed(lo, hi);
  }
  {
    int cap_max = 0;
    for (int s = 0; s < ns; ++s) cap_max = std::max(cap_max, hs[s]->d.cap);
    if (g_fused_chain && ns >= g_chain_min_states && 2 * cap_max > 64 && 2 * cap_max <= 128)
      return run_chains(hs, ns, lists, cap_max);
  }
  hipStream_t st = aqc::mps_stream();
  std::vector<std::vector<std::vector<const DevOp*>>> lv(ns);
  size_t maxlen = 0;
  for (int s = 0; s < ns; ++s) {
    lv[s] = level_ops(lists[s], hs[s]->d.n);
    maxlen = std::max(maxlen, lv[s].size());
    int width = 1;
    for (auto& w : lv[s]) {
      int k = 0;
      for (const DevOp* op : w) k += op->kind == 2;
      width = std::max(width, k);
    }
    int rc = ensure_slots(hs[s], width);
    if (rc != AQC_OK) return rc;
  }
  if (maxlen == 0) return AQC_OK;
  // pre-build every wave's jobs into one staging buffer
  std::vector<TwoSiteJob> two;
  std::vector<OneSiteJob> one;
  std::vector<std::pair<size_t, size_t>> two_rng(maxlen), one_rng(maxlen);
  int cap_max = 0;
  for (int s = 0; s < ns; ++s) cap_max = std::max(cap_max, hs[s]->d.cap);
  // each wave's largest possible theta side (2 chi), from the host bond bounds advanced through
  // the lists in wave order: 2 chi <= 128 runs the register Jacobi with pivoted-QR
  // preconditioning (the Gram path in front of it at 2 chi = 128), larger the multi-workgroup
  // block Jacobi sized by the bound -- so a large-capacity state with small bonds (an unbounded
  // MPS early in a circuit) does not pay for its capacity
  // Each two-site job's SVD kernel class from its own largest possible theta side (2 chi): the
  // register Jacobi up to 128 (the Gram path in front of it at 128), the block Jacobi sized to the
  // next power of two above (at most 2 cap) -- so a large-capacity state with small bonds does not
  // pay for its capacity, and a job's kernel does not depend on the jobs it shares a wave with
  // (a batched wave equals the same updates applied one call at a time, bit for bit).  Capacities
  // <= 64 keep one class (2 cap): the lock-step path then matches the fused chain exactly.
  struct ClassRange {
    int cls;
    size_t first, count;
  };
  std::vector<std::vector<ClassRange>> wave_cls(maxlen);
  auto class_of = [&](int side) {
    if (2 * cap_max <= 128) return 2 * cap_max;
    if (side <= 32) return 32;
    if (side <= 64) return 64;
    if (side <= 128) return 128;
    int c = 256;
    while (c < side) c <<= 1;
    return std::min(c, 2 * cap_max);
  };
  std::vector<std::pair<int, TwoSiteJob>> wjobs;
  for (size_t w = 0; w < maxlen; ++w) {
    size_t t0 = two.size(), o0 = one.size();
    wjobs.clear();
    for (int s = 0; s < ns; ++s) {
      if (w >= lv[s].size()) continue;
      int slot = 0;
      std::vector<int>& ub = hs[s]->ub;
      for (const DevOp* op : lv[s][w]) {
        if (op->kind == 2) {
          const int p = op->p;
          const int cls = class_of(2 * std::max(ub[p], ub[p + 2]));
          wjobs.push_back({cls, make_two(hs[s], *op, slot++)});
          wjobs.back().second.qr = cls <= 128 ? 1 : 0;
          int nb = std::min(2 * std::min(ub[p], ub[p + 2]), hs[s]->d.cap);
          if (hs[s]->max_chi > 0) nb = std::min(nb, hs[s]->max_chi);
          ub[p + 1] = std::max(nb, 1);
        } else {
          one.push_back(make_one(hs[s], *op));
        }
      }
    }
    std::stable_sort(wjobs.begin(), wjobs.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (size_t k = 0; k < wjobs.size(); ++k) {
      if (k == 0 || wjobs[k].first != wjobs[k - 1].first) wave_cls[w].push_back({wjobs[k].first, two.size(), 0});
      wave_cls[w].back().count += 1;
      two.push_back(wjobs[k].second);
    }
    two_rng[w] = {t0, two.size() - t0};
    one_rng[w] = {o0, one.size() - o0};
  }
  const size_t tb = two.size() * sizeof(TwoSiteJob), ob = one.size() * sizeof(OneSiteJob);
  StagingLease lease(st);
  if (lease.rc() != AQC_OK) return lease.rc();
  Staging& sg = lease.buf();
  int rc = lease.ensure(tb + ob + 256);
  if (rc != AQC_OK) return rc;
  std::memcpy(sg.host, two.data(), tb);
  std::memcpy((char*)sg.host + tb, one.data(), ob);
  if (int e = aqc::upload_async(sg.dev, sg.host, tb + ob, st)) return e;
  const TwoSiteJob* dtwo = (const TwoSiteJob*)sg.dev;
  const OneSiteJob* done = (const OneSiteJob*)((char*)sg.dev + tb);
  const int tiles = ((cap_max + 15) / 16) * ((cap_max + 15) / 16);
  const int tiles32 = ((cap_max + 31) / 32) * ((cap_max + 31) / 32);
  const int blocks_split = ((2 * cap_max + 63) / 64) * ((2 * cap_max + 63) / 64);
  for (size_t w = 0; w < maxlen; ++w) {
    if (one_rng[w].second) {
      const int nj = (int)one_rng[w].second;
      hipLaunchKernelGGL(k_1q, dim3((cap_max * cap_max + kT - 1) / kT, nj), dim3(kT), 0, st,
                         done + one_rng[w].first);
      AQC_CHECK_LAUNCH();
    }
    if (two_rng[w].second) {
      const int nj = (int)two_rng[w].second;
      const TwoSiteJob* jp = dtwo + two_rng[w].first;
      const double c = cap_max;
      aqc::KernelTimer::begin(st, "mps_theta", nj * (6.0 * c * c * 16 + 4.0 * c * c * 16), nj * 4.0 * c * c * c * 8);
      if (tiles32 * nj >= 256)  // (enough 32 x 32 tiles to fill the GPU)
        hipLaunchKernelGGL(k_theta32, dim3(aqc::xcd_grid(tiles32, nj)), dim3(kT), 0, st, jp, nj);
      else
        hipLaunchKernelGGL(k_theta, dim3(aqc::xcd_grid(tiles, nj)), dim3(kT), 0, st, jp, nj);
      aqc::KernelTimer::end(st);
      AQC_CHECK_LAUNCH();
      aqc::KernelTimer::begin(st, "mps_svd", nj * 2.0 * (4.0 * c * c * 16), 0.0);
      for (const ClassRange& cr : wave_cls[w]) {
        const int side = cr.cls, nc = (int)cr.count;
        const TwoSiteJob* jc = dtwo + cr.first;
        if (side <= 128) {
          // register-resident kernel; column count padded to a power of two.  Dynamic LDS holds
          // the round exchange (kG x 16*MAXR) or the QR transpose (kG x (CP+1)), whichever is larger
          if (side <= 32)
            hipLaunchKernelGGL((k_jacobi_reg<32, 2>), dim3(nc), dim3(256), 16 * 33 * 16, st, jc);
          else if (side <= 64)
            hipLaunchKernelGGL((k_jacobi_reg<64, 4>), dim3(nc), dim3(512), 32 * 65 * 16, st, jc);
          else
            launch_jacobi_reg128(nc, st, jc);
        } else {
          // 2 chi > 128: the multi-workgroup Gram path (gram_big.hip), the block Jacobi
          // (bjacobi.hip) for the jobs it declines; sized by the class
          const int brc = aqc::big_svd(two.data() + cr.first, jc, nc, side, side / 2, st);
          if (brc != AQC_OK) return brc;
        }
      }
      aqc::KernelTimer::end(st);
      AQC_CHECK_LAUNCH();
      hipLaunchKernelGGL(k_rank, dim3(nj), dim3(kT), 0, st, jp);
      AQC_CHECK_LAUNCH();
      hipLaunchKernelGGL(k_split_copy, dim3(std::max(1, (4 * cap_max * cap_max + kT - 1) / kT), nj), dim3(kT), 0, st, jp);
      AQC_CHECK_LAUNCH();
      aqc::KernelTimer::begin(st, "mps_split", 0.0, nj * 2.0 * c * c * 2.0 * c * 8);
      hipLaunchKernelGGL(k_split_gemm, dim3(aqc::xcd_grid(blocks_split, nj)), dim3(aqc::kGemmThreads), 0, st, jp, nj);
      aqc::KernelTimer::end(st);
      AQC_CHECK_LAUNCH();
    }
  }
  return AQC_OK;  // the lease records the set's event
}

int check_flags(aqc_mps_t h) {
  int f[3] = {0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyAsync(f, h->d.flags, sizeof(f), hipMemcpyDeviceToHost, aqc::mps_stream()));
  AQC_HIP_CHECK(hipStreamSynchronize(aqc::mps_stream()));
  if (f[0]) {
    aqc::set_error("MPS bond capacity (chi_cap) exceeded: increase chi_cap or set max_chi");
    int z[3] = {0, 0, 0};
    hipMemcpy(h->d.flags, z, sizeof(z), hipMemcpyHostToDevice);
    return AQC_ERR_STATE;
  }
  if (f[1]) {
    aqc::set_error("one-sided Jacobi SVD did not converge");
    int z[3] = {0, 0, 0};
    hipMemcpy(h->d.flags, z, sizeof(z), hipMemcpyHostToDevice);
    return AQC_ERR_STATE;
  }
  return AQC_OK;
}

// Flags of many states with one gather launch and one read-back (instead of one synchronous
// copy per state); only states with a raised flag are then inspected and reset one by one.
__global__ void k_gather_flags(int* const* __restrict__ flags, int ns, int* __restrict__ out) {
  for (int s = blockIdx.x * blockDim.x + threadIdx.x; s < ns; s += gridDim.x * blockDim.x)
    out[s] = flags[s][0] | flags[s][1];
}

int check_flags_batch(aqc_mps_t* hs, int ns) {
  if (ns <= 0) return AQC_OK;
  if (ns == 1) return check_flags(hs[0]);
  struct FlagStage {
    void* dev = nullptr;
    size_t cap = 0;
    int* host = nullptr;
    size_t hcap = 0;
  };
  static FlagStage stages[64];
  static void (*release)() = [] {
    for (auto& f : stages) {
      if (f.dev) (void)hipFree(f.dev);
      if (f.host) (void)hipHostFree(f.host);
      f = FlagStage();
    }
  };
  aqc::on_finalize(release);
  int dev = 0;
  hipGetDevice(&dev);
  FlagStage& fs = stages[dev];
  const size_t bytes = (size_t)ns * (sizeof(int*) + sizeof(int));
  if (bytes > fs.cap) {
    if (fs.dev) hipFree(fs.dev);
    fs.cap = std::max(bytes, 2 * fs.cap);
    AQC_HIP_CHECK(hipMalloc(&fs.dev, fs.cap));
  }
  if (bytes > fs.hcap) {
    if (fs.host) hipHostFree(fs.host);
    fs.hcap = std::max(bytes, 2 * fs.hcap);
    AQC_HIP_CHECK(hipHostMalloc((void**)&fs.host, fs.hcap, hipHostMallocDefault));
  }
  hipStream_t st = aqc::mps_stream();
  int** hp = (int**)fs.host;
  for (int s = 0; s < ns; ++s) hp[s] = hs[s]->d.flags;
  int** dp = (int**)fs.dev;
  int* dout = (int*)((char*)fs.dev + (size_t)ns * sizeof(int*));
  AQC_HIP_CHECK(hipMemcpyAsync(dp, hp, (size_t)ns * sizeof(int*), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_gather_flags, dim3((ns + 255) / 256), dim3(256), 0, st, (int* const*)dp, ns, dout);
  AQC_CHECK_LAUNCH();
  int* hout = (int*)((char*)fs.host + (size_t)ns * sizeof(int*));
  AQC_HIP_CHECK(hipMemcpyAsync(hout, dout, (size_t)ns * sizeof(int), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  int first = AQC_OK;  // every raised flag is read and reset; the first error is reported
  for (int s = 0; s < ns; ++s) {
    if (hout[s]) {
      const int rc = check_flags(hs[s]);
      if (first == AQC_OK) first = rc;
    }
  }
  return first;
}

bool is_sorted_order(aqc_mps_t h) {
  for (int i = 0; i < h->d.n; ++i)
    if (h->order[i] != i) return false;
  return true;
}

// Moves every state to sorted qubit order; *moved = number of states that needed swaps.
int do_sort(aqc_mps_t* hs, int ns, int* moved = nullptr) {
  std::vector<aqc_mps_t> todo;
  for (int s = 0; s < ns; ++s)
    if (!is_sorted_order(hs[s])) todo.push_back(hs[s]);
  if (moved) *moved = (int)todo.size();
  if (todo.empty()) return AQC_OK;
  const int nt = (int)todo.size();
  std::vector<std::vector<DevOp>> lists(nt);
  for (int s = 0; s < nt; ++s) {
    Scheduler sc(todo[s]->d.n, todo[s]->order, todo[s]->loc, lists[s]);
    sc.sort();
  }
  return run_waves(todo.data(), nt, lists);
}

MeasJob make_meas(aqc_mps_t h, cplx* out) {
  MeasJob m;
  m.gam = h->d.gam;
  m.lam = h->d.lam;
  m.dims = h->d.dims;
  m.n = h->d.n;
  m.cap = h->d.cap;
  m.out = out;
  m.vec = h->d.vec;
  m.env = h->d.env;
  m.tmp = h->d.tmp;
  return m;
}

template <typename T>
int upload_jobs(const std::vector<T>& jobs, const T** dptr) {
  Staging& sg = staging();
  hipStream_t st = aqc::mps_stream();
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  const size_t b = jobs.size() * sizeof(T);
  int rc = ensure_staging(sg, b + 64);
  if (rc != AQC_OK) return rc;
  std::memcpy(sg.host, jobs.data(), b);
  if (int e = aqc::upload_async(sg.dev, sg.host, b, st)) return e;
  *dptr = (const T*)sg.dev;
  return AQC_OK;
}

}  // namespace

extern "C" {

int aqc_mps_create(int n, int chi_cap, double threshold, int max_chi, aqc_mps_t* out) {
  AQC_REQUIRE(out, "aqc_mps_create: null out");
  AQC_REQUIRE(n >= 1 && n <= 4096, "aqc_mps_create: bad n");
  AQC_REQUIRE(chi_cap >= 1 && chi_cap <= kMaxCap, "aqc_mps_create: chi_cap must be in [1, 1024]");
  auto* h = new aqc_mps_s();
  static std::atomic<unsigned long long> next_uid{1};
  h->uid = next_uid++;
  AQC_HIP_CHECK(hipGetDevice(&h->dev));
  h->d.n = n;
  h->d.cap = chi_cap;
  h->zr = h->hr = h->h0r = n;
  h->thr = threshold;
  h->max_chi = max_chi;
  h->order.resize(n);
  h->loc.resize(n);
  for (int i = 0; i < n; ++i) h->order[i] = h->loc[i] = i;
  h->ub.assign(n + 1, 1);
  const size_t cap = chi_cap;
  const size_t g = (size_t)n * 2 * cap * cap;
  hipStream_t st = aqc::mps_stream();
  // the fixed buffers carved from one cached device block (256-byte aligned pieces)
  {
    const size_t sz[11] = {g * sizeof(cplx), (size_t)(n + 1) * cap * sizeof(double), (size_t)(n + 1) * sizeof(int),
                           4 * cap * cap * sizeof(cplx), aqc::work_elems(cap) * sizeof(cplx), kSigLen * sizeof(double),
                           kSigMax * sizeof(int), 4 * sizeof(int), 2 * (size_t)(n + 1) * cap * sizeof(cplx),
                           2 * cap * cap * sizeof(cplx), (size_t)(2 * n + 8) * sizeof(cplx)};
    size_t off[11], total = 0;
    for (int i = 0; i < 11; ++i) {
      off[i] = total;
      total += (sz[i] + 255) & ~(size_t)255;
    }
    char* b = (char*)aqc::dev_alloc(total);
    if (!b) {
      delete h;
      aqc::set_error("aqc_mps_create: out of device memory");
      return AQC_ERR_NOMEM;
    }
    h->base = b;
    h->d.gam = (cplx*)(b + off[0]);
    h->d.lam = (double*)(b + off[1]);
    h->d.dims = (int*)(b + off[2]);
    h->d.theta = (cplx*)(b + off[3]);
    h->d.work = (cplx*)(b + off[4]);
    h->d.sig = (double*)(b + off[5]);
    h->d.perm = (int*)(b + off[6]);
    h->d.flags = (int*)(b + off[7]);
    h->d.vec = (cplx*)(b + off[8]);
    h->d.tmp = (cplx*)(b + off[9]);
    h->d.scal = (cplx*)(b + off[10]);
  }
  h->d.env = nullptr;  // allocated lazily for dot / z_all
  AQC_HIP_CHECK(hipMemsetAsync(h->d.gam, 0, g * sizeof(cplx), st));
  AQC_HIP_CHECK(hipMemsetAsync(h->d.lam, 0, (size_t)(n + 1) * cap * sizeof(double), st));
  AQC_HIP_CHECK(hipMemsetAsync(h->d.flags, 0, 4 * sizeof(int), st));
  AQC_HIP_CHECK(hipMemsetAsync(h->d.sig, 0, kSigLen * sizeof(double), st));
  hipLaunchKernelGGL(k_mps_zero, dim3(1 + n / 256), dim3(256), 0, st, h->d.gam, h->d.lam, h->d.dims, n, chi_cap);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  *out = h;
  return AQC_OK;
}

int aqc_mps_destroy(aqc_mps_t h) {
  if (!h) return AQC_OK;
  // drain the handle's own device's MPS stream (the caller may have switched devices since), and
  // do not create one: after aqc_finalize (interpreter teardown) no stream is left, nor any work
  if (hipStream_t st = aqc::mps_stream_if_any(h->dev)) {
    int cur = 0;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    if (!have || cur != h->dev) (void)hipSetDevice(h->dev);
    (void)hipStreamSynchronize(st);
    if (have && cur != h->dev) (void)hipSetDevice(cur);
  }
  aqc::dev_free(h->base);
  aqc::dev_free(h->d.env);
  aqc::dev_free(h->gw);
  aqc::dev_free(h->zenv);
  aqc::dev_free(h->hwenv);
  for (auto& sl : h->slots) {
    aqc::dev_free(sl.theta);
    aqc::dev_free(sl.work);
    aqc::dev_free(sl.sig);
    aqc::dev_free(sl.perm);
  }
  delete h;
  return AQC_OK;
}

int aqc_svd_debug(const double* theta, int m, int n, int variant, int stop_after_qr, double* w_out,
                  double* sig_out, int* perm_out, int* sweeps) {
  AQC_REQUIRE(theta && w_out && sig_out && sweeps, "aqc_svd_debug: null argument");
  AQC_REQUIRE(m >= 1 && n >= 1 && m % 2 == 0 && n % 2 == 0 && m <= 128 && n <= 128,
              "aqc_svd_debug: m, n must be even and <= 128");
  AQC_REQUIRE(stop_after_qr >= 0 && stop_after_qr <= 2, "aqc_svd_debug: stop_after_qr must be 0, 1 or 2");
  AQC_REQUIRE(variant == 2 || variant == 7, "aqc_svd_debug: variant must be 2 (register Jacobi) or 7 (Gram path)");
  AQC_REQUIRE(variant < 7 || (std::max(m, n) > 64 && stop_after_qr == 0),
              "aqc_svd_debug: variant 7 (Gram) needs 64 < max(m, n) <= 128 and no QR stop");
  hipStream_t st = aqc::mps_stream();
  const int cp = std::max(m, n) <= 32 ? 32 : (std::max(m, n) <= 64 ? 64 : 128);
  const size_t mat = (size_t)128 * 128 * sizeof(cplx), wmat = aqc::work_elems(64) * sizeof(cplx);
  char* buf = nullptr;
  AQC_HIP_CHECK(hipMalloc(&buf, mat + wmat + kSigLen * sizeof(double) + 512 * sizeof(int) + 8 * sizeof(int) +
                                    sizeof(TwoSiteJob)));
  cplx* th = (cplx*)buf;
  cplx* wk = (cplx*)(buf + mat);
  double* sg = (double*)(buf + mat + wmat);
  int* pm = (int*)(sg + kSigLen);
  int* dm = pm + 512;  // dims[3] + flags share this tail
  int* fl = dm + 4;
  TwoSiteJob* dj = (TwoSiteJob*)(fl + 4);
  TwoSiteJob j;
  std::memset(&j, 0, sizeof(j));
  j.dims = dm;
  j.theta = th;
  j.work = wk;
  j.sig = sg;
  j.perm = pm;
  j.flags = fl;
  j.jtol = g_jacobi_tol_factor;
  j.jtiny = g_jacobi_tiny_t;
  j.jnoise = kJacobiNoise;
  j.qr = 1;
  j.dbg = stop_after_qr;
  j.cap = 64;                     // the work buffer holds 128 x 128
  j.max_chi = g_debug_max_chi;    // Gram path: K = min(C, max_chi)
  j.gram = variant == 7;  // (stop_after_qr 1: stop after the QR phase; 2: also its ticks)
  int hd[8] = {m / 2, 0, n / 2, 0, 0, 0, 0, 0};  // dims, then zeroed flags
  AQC_HIP_CHECK(hipMemcpyAsync(th, theta, (size_t)m * n * sizeof(cplx), hipMemcpyHostToDevice, st));
  AQC_HIP_CHECK(hipMemcpyAsync(dm, hd, sizeof(hd), hipMemcpyHostToDevice, st));
  AQC_HIP_CHECK(hipMemcpyAsync(dj, &j, sizeof(j), hipMemcpyHostToDevice, st));
  AQC_HIP_CHECK(hipMemsetAsync(wk, 0, wmat, st));
  AQC_HIP_CHECK(hipMemsetAsync(sg, 0, kSigLen * sizeof(double), st));
  if (cp == 32) hipLaunchKernelGGL((k_jacobi_reg<32, 2>), dim3(1), dim3(256), 16 * 33 * 16, st, dj);
  else if (cp == 64) hipLaunchKernelGGL((k_jacobi_reg<64, 4>), dim3(1), dim3(512), 32 * 65 * 16, st, dj);
  else if (variant == 7)
    hipLaunchKernelGGL(k_svd_gram, dim3(1), dim3(1024), kChainLdsBytes, st, dj);
  else  // the register Jacobi itself (not the Gram path in front of it)
    hipLaunchKernelGGL((k_jacobi_reg<128, 8>), dim3(1), dim3(1024), 64 * 129 * 16, st, dj);
  AQC_CHECK_LAUNCH();
  const int L = std::max(m, n), C = std::min(m, n);
  const int Lw = j.qr ? C : L;
  AQC_HIP_CHECK(hipMemcpyAsync(w_out, wk, (size_t)C * Lw * sizeof(cplx), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipMemcpyAsync(sig_out, sg, (size_t)C * sizeof(double), hipMemcpyDeviceToHost, st));
  if (perm_out) AQC_HIP_CHECK(hipMemcpyAsync(perm_out, pm, (size_t)C * sizeof(int), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipMemcpyAsync(hd, fl, 4 * sizeof(int), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  *sweeps = hd[2];
  AQC_HIP_CHECK(hipFree(buf));
  return AQC_OK;
}

int aqc_mps_jacobi_stats(aqc_mps_t h, int* max_sweeps) {
  AQC_REQUIRE(h && max_sweeps, "aqc_mps_jacobi_stats: null argument");
  hipStream_t st = aqc::mps_stream();
  int f[3] = {0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyAsync(f, h->d.flags, sizeof(f), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  *max_sweeps = f[2];
  int z = 0;
  AQC_HIP_CHECK(hipMemcpy(h->d.flags + 2, &z, sizeof(int), hipMemcpyHostToDevice));
  return AQC_OK;
}

int aqc_mps_set_jacobi_tol(double factor) {
  AQC_REQUIRE(factor > 0, "aqc_mps_set_jacobi_tol: factor must be positive");
  g_jacobi_tol_factor = factor;
  return AQC_OK;
}

int aqc_svd_gram_ticks(double* out) {
  AQC_REQUIRE(out, "aqc_svd_gram_ticks: null argument");
  unsigned long long t[12];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_gram_ticks), sizeof(t)));
  for (int i = 0; i < 12; ++i) out[i] = (double)t[i];
  unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_gram_ticks), z, sizeof(z)));
  return AQC_OK;
}

int aqc_svd_gram_stats(double* out) {
  AQC_REQUIRE(out, "aqc_svd_gram_stats: null argument");
  unsigned long long t[6];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_gram_stats), sizeof(t)));
  for (int i = 0; i < 6; ++i) out[i] = (double)t[i];
  unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_gram_stats), z, sizeof(z)));
  return AQC_OK;
}

int aqc_mps_set_svd_path(int gram, int debug_max_chi) {
  AQC_REQUIRE(gram >= 0 && gram <= 1, "aqc_mps_set_svd_path: gram must be 0 or 1");
  g_svd_gram = gram;
  g_debug_max_chi = debug_max_chi;
  return AQC_OK;
}


int aqc_mps_set_jacobi_stop(double tiny_t) {
  AQC_REQUIRE(tiny_t < 1e-3, "aqc_mps_set_jacobi_stop: tiny_t must be < 1e-3 (<= 0 restores the default)");
  g_jacobi_tiny_t = tiny_t > 0 ? tiny_t : kDefaultTinyT;
  return AQC_OK;
}

int aqc_mps_chain_ticks(double* out) {
  AQC_REQUIRE(out, "aqc_mps_chain_ticks: null argument");
  unsigned long long t[5] = {0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipStreamSynchronize(aqc::mps_stream()));
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(g_chain_ticks), sizeof(t)));
  const unsigned long long z[5] = {0, 0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_chain_ticks), z, sizeof(z)));
  for (int i = 0; i < 5; ++i) out[i] = (double)t[i];
  return AQC_OK;
}

int aqc_mps_set_fused_chain(int on) {
  AQC_REQUIRE(on >= 0 && on <= 2, "aqc_mps_set_fused_chain: 0, 1 or 2");
  g_fused_chain = on != 0;
  g_chain_min_states = on == 2 ? 1 : 32;
  return AQC_OK;
}


int aqc_mps_set_truncation(aqc_mps_t h, double threshold, int max_chi) {
  AQC_REQUIRE(h, "aqc_mps_set_truncation: null handle");
  h->thr = threshold;
  h->max_chi = max_chi;
  return AQC_OK;
}

int aqc_mps_set_vidal(aqc_mps_t h, const int* dims, const double* gammas, const double* lambdas) {
  AQC_REQUIRE(h && dims && gammas && lambdas, "aqc_mps_set_vidal: null argument");
  const int n = h->d.n, cap = h->d.cap;
  AQC_REQUIRE(dims[0] == 1 && dims[n] == 1, "aqc_mps_set_vidal: dims[0] and dims[n] must be 1");
  for (int b = 0; b <= n; ++b) {
    if (dims[b] < 1 || dims[b] > cap) {
      aqc::set_error("aqc_mps_set_vidal: bond dimension exceeds chi_cap");
      return AQC_ERR_ARG;
    }
  }
  std::vector<cplx> g((size_t)n * 2 * cap * cap, aqc::cmk(0, 0));
  std::vector<double> l((size_t)(n + 1) * cap, 0.0);
  size_t off = 0;
  for (int i = 0; i < n; ++i)
    for (int s = 0; s < 2; ++s)
      for (int a = 0; a < dims[i]; ++a)
        for (int b = 0; b < dims[i + 1]; ++b, ++off)
          g[(size_t)i * 2 * cap * cap + (size_t)s * cap * cap + (size_t)a * cap + b] =
              aqc::cmk(gammas[2 * off], gammas[2 * off + 1]);
  l[0] = 1.0;
  l[(size_t)n * cap] = 1.0;
  size_t lo = 0;
  for (int b = 1; b < n; ++b)
    for (int k = 0; k < dims[b]; ++k) l[(size_t)b * cap + k] = lambdas[lo++];
  hipStream_t st = aqc::mps_stream();
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  AQC_HIP_CHECK(hipMemcpy(h->d.gam, g.data(), g.size() * sizeof(cplx), hipMemcpyHostToDevice));
  AQC_HIP_CHECK(hipMemcpy(h->d.lam, l.data(), l.size() * sizeof(double), hipMemcpyHostToDevice));
  AQC_HIP_CHECK(hipMemcpy(h->d.dims, dims, (n + 1) * sizeof(int), hipMemcpyHostToDevice));
  for (int i = 0; i < n; ++i) h->order[i] = h->loc[i] = i;
  h->ub.assign(dims, dims + n + 1);
  h->changed_all();
  return AQC_OK;
}

int aqc_mps_get_dims(aqc_mps_t h, int* dims) {
  AQC_REQUIRE(h && dims, "aqc_mps_get_dims: null argument");
  hipStream_t st = aqc::mps_stream();
  AQC_HIP_CHECK(hipMemcpyAsync(dims, h->d.dims, (h->d.n + 1) * sizeof(int), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  h->ub.assign(dims, dims + h->d.n + 1);  // exact again
  return AQC_OK;
}

int aqc_mps_sort(aqc_mps_t h) {
  AQC_REQUIRE(h, "aqc_mps_sort: null handle");
  if (is_sorted_order(h)) return AQC_OK;
  int rc = do_sort(&h, 1);
  if (rc != AQC_OK) return rc;
  return check_flags(h);
}

int aqc_mps_sort_batch(aqc_mps_t* hs, int ns) {
  AQC_REQUIRE(hs && ns >= 0, "aqc_mps_sort_batch: bad arguments");
  int moved = 0;
  int rc = do_sort(hs, ns, &moved);
  if (rc != AQC_OK) return rc;
  return moved ? check_flags_batch(hs, ns) : AQC_OK;  // (no update ran: no flag can have risen)
}

int aqc_mps_get_vidal(aqc_mps_t h, int* dims, double* gammas, double* lambdas) {
  AQC_REQUIRE(h && dims, "aqc_mps_get_vidal: null argument");
  int rc = aqc_mps_sort(h);
  if (rc != AQC_OK) return rc;
  rc = aqc_mps_get_dims(h, dims);
  if (rc != AQC_OK) return rc;
  if (!gammas || !lambdas) return AQC_OK;
  const int n = h->d.n, cap = h->d.cap;
  std::vector<cplx> g((size_t)n * 2 * cap * cap);
  std::vector<double> l((size_t)(n + 1) * cap);
  AQC_HIP_CHECK(hipMemcpy(g.data(), h->d.gam, g.size() * sizeof(cplx), hipMemcpyDeviceToHost));
  AQC_HIP_CHECK(hipMemcpy(l.data(), h->d.lam, l.size() * sizeof(double), hipMemcpyDeviceToHost));
  size_t off = 0;
  for (int i = 0; i < n; ++i)
    for (int s = 0; s < 2; ++s)
      for (int a = 0; a < dims[i]; ++a)
        for (int b = 0; b < dims[i + 1]; ++b, ++off) {
          const cplx v = g[(size_t)i * 2 * cap * cap + (size_t)s * cap * cap + (size_t)a * cap + b];
          gammas[2 * off] = v.x;
          gammas[2 * off + 1] = v.y;
        }
  size_t lo = 0;
  for (int b = 1; b < n; ++b)
    for (int k = 0; k < dims[b]; ++k) lambdas[lo++] = l[(size_t)b * cap + k];
  return AQC_OK;
}

// Batched reload of cached MPS (one launch instead of three copies per state): every state's
// gamma, lambda and dims blocks are contiguous, copied as 16-byte words, grid (chunks, states).
struct CopyJob {
  const double2* sg;
  double2* dg;
  size_t ng;  // double2 words of gamma
  const double* sl;
  double* dl;
  size_t nl;
  const int* sd;
  int* dd;
  int nd;
  int pad;
};

__global__ __launch_bounds__(kT) void k_copy_batch(const CopyJob* __restrict__ jobs) {
  const CopyJob& j = jobs[blockIdx.y];
  const size_t stride = (size_t)gridDim.x * kT;
  for (size_t e = (size_t)blockIdx.x * kT + threadIdx.x; e < j.ng; e += stride) j.dg[e] = j.sg[e];
  for (size_t e = (size_t)blockIdx.x * kT + threadIdx.x; e < j.nl; e += stride) j.dl[e] = j.sl[e];
  for (size_t e = (size_t)blockIdx.x * kT + threadIdx.x; e < (size_t)j.nd; e += stride) j.dd[e] = j.sd[e];
}

int aqc_mps_copy_batch(aqc_mps_t* dst, const aqc_mps_t* src, int ns) {
  AQC_REQUIRE(ns >= 0 && (ns == 0 || (dst && src)), "aqc_mps_copy_batch: null argument");
  if (ns == 0) return AQC_OK;
  std::vector<CopyJob> jobs(ns);
  for (int s = 0; s < ns; ++s) {
    AQC_REQUIRE(dst[s] && src[s] && dst[s]->d.n == src[s]->d.n && dst[s]->d.cap == src[s]->d.cap,
                "aqc_mps_copy_batch: handle mismatch");
    const size_t cap = src[s]->d.cap, n = src[s]->d.n;
    aqc_mps_s* d = dst[s];
    const aqc_mps_s* r = src[s];
    // Gamma sites to copy: all, or -- when dst was last copied from this source and the source
    // has not changed since -- only the sites dst has rewritten since then
    size_t lo = 0, cnt = n;
    if (d != r && d->synced_src == r->uid && d->synced_ver == r->version) {
      lo = d->dirty_hi >= d->dirty_lo ? (size_t)d->dirty_lo : 0;
      cnt = d->dirty_hi >= d->dirty_lo ? (size_t)(d->dirty_hi - d->dirty_lo + 1) : 0;
    }
    CopyJob& j = jobs[s];
    j.sg = r->d.gam + lo * 2 * cap * cap;
    j.dg = d->d.gam + lo * 2 * cap * cap;
    j.ng = cnt * 2 * cap * cap;
    j.sl = src[s]->d.lam;
    j.dl = dst[s]->d.lam;
    j.nl = (n + 1) * cap;
    j.sd = src[s]->d.dims;
    j.dd = dst[s]->d.dims;
    j.nd = (int)n + 1;
    j.pad = 0;
    d->order = r->order;
    d->loc = r->loc;
    d->ub = r->ub;
    d->synced_src = r->uid;
    d->synced_ver = r->version;
    d->dirty_lo = 1 << 30;
    d->dirty_hi = -1;
    ++d->version;
    d->zenv_stale();
  }
  hipStream_t st = aqc::mps_stream();
  StagingLease lease(st);  // (the ring: no wait for the stream's earlier work)
  if (lease.rc() != AQC_OK) return lease.rc();
  Staging& sg = lease.buf();
  const size_t bytes = jobs.size() * sizeof(CopyJob);
  int rc = lease.ensure(bytes);
  if (rc != AQC_OK) return rc;
  std::memcpy(sg.host, jobs.data(), bytes);
  if (int e = aqc::upload_async(sg.dev, sg.host, bytes, st)) return e;
  size_t words = jobs[0].nl / 2, moved = 0;
  for (const CopyJob& j : jobs) {
    words = std::max(words, j.ng);
    moved += j.ng * 16 + j.nl * 8;
  }
  const int chunks = (int)std::min<size_t>(64, (words + 8 * kT - 1) / (8 * kT));
  aqc::KernelTimer::begin(st, "mps_copy", 2.0 * (double)moved, 0.0);
  hipLaunchKernelGGL(k_copy_batch, dim3(std::max(chunks, 1), ns), dim3(kT), 0, st, (const CopyJob*)sg.dev);
  aqc::KernelTimer::end(st);
  AQC_CHECK_LAUNCH();
  return AQC_OK;
}

int aqc_stream_join(void* stream) {
  static std::mutex mu;
  static hipEvent_t ev[64] = {nullptr};
  static void (*release)() = [] {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
  };
  aqc::on_finalize(release);
  int dev = 0;
  AQC_HIP_CHECK(hipGetDevice(&dev));
  AQC_REQUIRE(dev >= 0 && dev < 64, "aqc_stream_join: device index out of range");
  std::lock_guard<std::mutex> lk(mu);
  if (!ev[dev]) AQC_HIP_CHECK(hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming));
  AQC_HIP_CHECK(hipEventRecord(ev[dev], aqc::mps_stream()));
  AQC_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, ev[dev], 0));
  return AQC_OK;
}

int aqc_stream_wait(void* stream) {
  static std::mutex mu;
  static hipEvent_t ev[64] = {nullptr};
  static void (*release)() = [] {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
  };
  aqc::on_finalize(release);
  int dev = 0;
  AQC_HIP_CHECK(hipGetDevice(&dev));
  AQC_REQUIRE(dev >= 0 && dev < 64, "aqc_stream_wait: device index out of range");
  std::lock_guard<std::mutex> lk(mu);
  if (!ev[dev]) AQC_HIP_CHECK(hipEventCreateWithFlags(&ev[dev], hipEventDisableTiming));
  AQC_HIP_CHECK(hipEventRecord(ev[dev], (hipStream_t)stream));
  AQC_HIP_CHECK(hipStreamWaitEvent(aqc::mps_stream(), ev[dev], 0));
  return AQC_OK;
}

int aqc_mps_copy(aqc_mps_t dst, const aqc_mps_t src) {
  AQC_REQUIRE(dst && src && dst->d.n == src->d.n && dst->d.cap == src->d.cap, "aqc_mps_copy: handle mismatch");
  hipStream_t st = aqc::mps_stream();
  const size_t cap = src->d.cap, n = src->d.n;
  AQC_HIP_CHECK(hipMemcpyAsync(dst->d.gam, src->d.gam, n * 2 * cap * cap * sizeof(cplx), hipMemcpyDeviceToDevice, st));
  AQC_HIP_CHECK(hipMemcpyAsync(dst->d.lam, src->d.lam, (n + 1) * cap * sizeof(double), hipMemcpyDeviceToDevice, st));
  AQC_HIP_CHECK(hipMemcpyAsync(dst->d.dims, src->d.dims, (n + 1) * sizeof(int), hipMemcpyDeviceToDevice, st));
  dst->order = src->order;
  dst->ub = src->ub;
  dst->loc = src->loc;
  if (dst != src) {
    dst->zenv_stale();
    dst->synced_src = src->uid;
    dst->synced_ver = src->version;
    dst->dirty_lo = 1 << 30;
    dst->dirty_hi = -1;
    ++dst->version;
  }
  return AQC_OK;
}

// AQC_HOST_TIMING=1: host-side phase times of each batched apply to stderr (lab diagnostics)
bool host_timing() {
  static const bool on = [] {
    const char* e = std::getenv("AQC_HOST_TIMING");
    return e && std::strcmp(e, "0") != 0;
  }();
  return on;
}
double host_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int apply_batch_impl(aqc_mps_t* hs, int ns, const aqc_op_t* const* ops, const int* nops, bool sort_after,
                     bool check = true) {
  AQC_REQUIRE(hs && ops && nops && ns >= 0, "aqc_mps_apply_batch: null argument");
  const double t0 = host_timing() ? host_ms() : 0.0;
  std::vector<std::vector<DevOp>> lists(ns);
  for (int s = 0; s < ns; ++s) {
    AQC_REQUIRE(hs[s], "aqc_mps_apply_batch: null handle");
    int rc = validate_ops(hs[s], ops[s], nops[s]);
    if (rc != AQC_OK) return rc;
  }
  const double t1 = host_timing() ? host_ms() : 0.0;
  if (distinct_handles(hs, ns)) {
    parallel_states(ns, [&](int s) { schedule(hs[s], ops[s], nops[s], sort_after, lists[s]); });
  } else {  // a state listed twice: its op lists apply in order
    for (int s = 0; s < ns; ++s) schedule(hs[s], ops[s], nops[s], sort_after, lists[s]);
  }
  const double t2 = host_timing() ? host_ms() : 0.0;
  int rc = run_waves(hs, ns, lists);
  if (host_timing())
    std::fprintf(stderr, "[aqc host] apply %d states: validate %.3f ms, schedule %.3f ms, jobs+launch %.3f ms\n", ns,
                 t1 - t0, t2 - t1, host_ms() - t2);
  if (rc != AQC_OK) return rc;
  return check ? check_flags_batch(hs, ns) : AQC_OK;
}

int aqc_mps_apply_batch(aqc_mps_t* hs, int ns, const aqc_op_t* const* ops, const int* nops) {
  return apply_batch_impl(hs, ns, ops, nops, false);
}

int aqc_mps_apply_sort_batch(aqc_mps_t* hs, int ns, const aqc_op_t* const* ops, const int* nops) {
  return apply_batch_impl(hs, ns, ops, nops, true);
}

int aqc_mps_apply_sort_batch_async(aqc_mps_t* hs, int ns, const aqc_op_t* const* ops, const int* nops) {
  return apply_batch_impl(hs, ns, ops, nops, true, false);
}

int aqc_mps_apply_batch_async(aqc_mps_t* hs, int ns, const aqc_op_t* const* ops, const int* nops) {
  return apply_batch_impl(hs, ns, ops, nops, false, false);
}

int aqc_mps_check_batch(aqc_mps_t* hs, int ns) {
  AQC_REQUIRE(hs && ns >= 0, "aqc_mps_check_batch: null argument");
  for (int s = 0; s < ns; ++s) AQC_REQUIRE(hs[s], "aqc_mps_check_batch: null handle");
  return check_flags_batch(hs, ns);
}

int aqc_mps_apply(aqc_mps_t h, const aqc_op_t* ops, int nops) {
  return aqc_mps_apply_batch(&h, 1, &ops, &nops);
}

int aqc_mps_overlap_zero_batch(aqc_mps_t* hs, int ns, double* out) {
  AQC_REQUIRE(hs && out && ns >= 0, "aqc_mps_overlap_zero_batch: null argument");
  if (ns == 0) return AQC_OK;
  int rc = aqc_mps_sort_batch(hs, ns);
  if (rc != AQC_OK) return rc;
  // results (ns complex) and the states' gathered error flags (ns ints) in one device buffer: one
  // read-back for both (the caller needs no aqc_mps_check_batch round trip after it)
  static char* dres[64] = {nullptr};
  static size_t dres_n[64] = {0};
  static void (*release)() = [] {
    for (int d = 0; d < 64; ++d)
      if (dres[d]) (void)hipFree(dres[d]), dres[d] = nullptr, dres_n[d] = 0;
  };
  aqc::on_finalize(release);
  int dev = 0;
  hipGetDevice(&dev);
  hipStream_t st = aqc::mps_stream();
  const size_t rbytes = (size_t)ns * sizeof(cplx), need = rbytes + (size_t)ns * sizeof(int);
  if (dres_n[dev] < need) {
    AQC_HIP_CHECK(hipStreamSynchronize(st));
    if (dres[dev]) hipFree(dres[dev]);
    dres_n[dev] = std::max(need, 2 * dres_n[dev]);
    AQC_HIP_CHECK(hipMalloc(&dres[dev], dres_n[dev]));
  }
  cplx* dr = (cplx*)dres[dev];
  int* dflags = (int*)(dres[dev] + rbytes);
  // the jobs and flag pointers through a pinned staging set of the ring: no wait for the stream's
  // earlier work (the chain that wrote the states) before these launches are queued
  StagingLease lease(st);
  if (lease.rc() != AQC_OK) return lease.rc();
  const size_t jb = ((ns * sizeof(MeasJob) + 255) / 256) * 256, fpb = (size_t)ns * sizeof(int*);
  rc = lease.ensure(jb + fpb);
  if (rc != AQC_OK) return rc;
  char* hj = (char*)lease.buf().host;
  char* dj = (char*)lease.buf().dev;
  MeasJob* hjobs = (MeasJob*)hj;
  int** hfp = (int**)(hj + jb);
  for (int s = 0; s < ns; ++s) {
    hjobs[s] = make_meas(hs[s], dr + s);  // one contiguous result array
    hfp[s] = hs[s]->d.flags;
  }
  if (int e = aqc::upload_async(dj, hj, jb + fpb, st)) return e;
  double bytes = 0;
  for (int s = 0; s < ns; ++s) bytes += (double)hs[s]->d.n * hs[s]->d.cap * hs[s]->d.cap * 16.0;
  aqc::KernelTimer::begin(st, "mps_overlap0", bytes, bytes / 2.0);
  int vc = 1;
  for (int s = 0; s < ns; ++s) vc = std::max(vc, hs[s]->d.cap);
  hipLaunchKernelGGL(k_overlap_zero, dim3(ns), dim3(kT), 2 * vc * sizeof(cplx), st, (const MeasJob*)dj, vc);
  aqc::KernelTimer::end(st);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_gather_flags, dim3((ns + 255) / 256), dim3(256), 0, st, (int* const*)(dj + jb), ns, dflags);
  AQC_CHECK_LAUNCH();
  std::vector<char> hv(need);
  AQC_HIP_CHECK(hipMemcpyAsync(hv.data(), dres[dev], need, hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  const cplx* v = (const cplx*)hv.data();
  const int* hf = (const int*)(hv.data() + rbytes);
  int first = AQC_OK;  // (every raised flag reset; the first error reported)
  for (int s = 0; s < ns; ++s)
    if (hf[s]) {
      const int frc = check_flags(hs[s]);
      if (first == AQC_OK) first = frc;
    }
  if (first != AQC_OK) return first;
  for (int s = 0; s < ns; ++s) {
    // mps_dot(psi, zero) = <psi|0..0> = conj(amplitude of |0..0>)
    out[2 * s] = v[s].x;
    out[2 * s + 1] = -v[s].y;
  }
  return AQC_OK;
}

int aqc_mps_overlap_zero(aqc_mps_t h, double* re, double* im) {
  AQC_REQUIRE(re && im, "aqc_mps_overlap_zero: null argument");
  double o[2];
  int rc = aqc_mps_overlap_zero_batch(&h, 1, o);
  *re = o[0];
  *im = o[1];
  return rc;
}

int aqc_mps_amps_hw1_batch(aqc_mps_t* hs, int ns, double* out) {
  AQC_REQUIRE(hs && ns >= 0 && (out || ns == 0), "aqc_mps_amps_hw1_batch: null argument");
  if (ns == 0) return AQC_OK;
  const int n = hs[0]->d.n;
  for (int s = 0; s < ns; ++s) AQC_REQUIRE(hs[s] && hs[s]->d.n == n, "aqc_mps_amps_hw1_batch: all states need the same n");
  int rc = aqc_mps_sort_batch(hs, ns);
  if (rc != AQC_OK) return rc;
  static cplx* dres[64] = {nullptr};
  static size_t dres_n[64] = {0};
  static void (*release)() = [] {
    for (int d = 0; d < 64; ++d)
      if (dres[d]) (void)hipFree(dres[d]), dres[d] = nullptr, dres_n[d] = 0;
  };
  aqc::on_finalize(release);
  int dev = 0;
  hipGetDevice(&dev);
  hipStream_t st = aqc::mps_stream();
  const size_t need = (size_t)ns * n;
  if (dres_n[dev] < need) {
    AQC_HIP_CHECK(hipStreamSynchronize(st));
    if (dres[dev]) hipFree(dres[dev]);
    dres_n[dev] = std::max(need, 2 * dres_n[dev]);
    AQC_HIP_CHECK(hipMalloc(&dres[dev], dres_n[dev] * sizeof(cplx)));
  }
  std::vector<MeasJob> jobs(ns);
  for (int s = 0; s < ns; ++s) jobs[s] = make_meas(hs[s], dres[dev] + (size_t)s * n);
  const MeasJob* dj = nullptr;
  rc = upload_jobs(jobs, &dj);
  if (rc != AQC_OK) return rc;
  int vc = 1;
  for (int s = 0; s < ns; ++s) vc = std::max(vc, hs[s]->d.cap);
  hipLaunchKernelGGL(k_zero_chains, dim3(ns, 2), dim3(kT), 2 * vc * sizeof(cplx), st, dj, vc);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_hw1, dim3(n, ns), dim3(kT), 0, st, dj);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipMemcpyAsync(out, dres[dev], need * sizeof(cplx), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  return AQC_OK;
}

/* <psi|0..0> (out_ov, 2 doubles per state, as aqc_mps_overlap_zero_batch) and, when out_amps is
   not null, the amplitudes <e_i|psi> (2 n doubles per state, as aqc_mps_amps_hw1_batch) of every
   state (sorted first): a state copied from `base` while base has not changed since contracts only
   the sites it rewrote against rows cached on base; any other state (or a window too wide for the
   LDS) takes the full chains. */
int aqc_mps_zero_hw1_batch(aqc_mps_t base, aqc_mps_t* hs, int ns, double* out_ov, double* out_amps) {
  AQC_REQUIRE(base && hs && ns >= 0 && (out_ov || ns == 0), "aqc_mps_zero_hw1_batch: bad arguments");
  if (ns == 0) return AQC_OK;
  const int n = base->d.n, cap = base->d.cap;
  for (int s = 0; s < ns; ++s)
    AQC_REQUIRE(hs[s] && hs[s] != base && hs[s]->d.n == n && hs[s]->d.cap == cap,
                "aqc_mps_zero_hw1_batch: every state needs base's n and capacity (and is not base)");
  int rc = aqc_mps_sort_batch(hs, ns);
  if (rc != AQC_OK) return rc;
  std::vector<int> win, lo(ns), hi(ns), fb;
  int need_l = 0, need_r = n;
  for (int s = 0; s < ns; ++s) {
    const aqc_mps_s* h = hs[s];
    const bool ok = h->synced_src == base->uid && h->synced_ver == base->version;
    lo[s] = h->dirty_hi >= h->dirty_lo ? h->dirty_lo : 0;
    hi[s] = h->dirty_hi >= h->dirty_lo ? h->dirty_hi : 0;
    if (!ok) {
      fb.push_back(s);
      continue;
    }
    need_l = std::max(need_l, lo[s]);
    need_r = std::min(need_r, hi[s] + 1);
    win.push_back(s);
  }
  hipStream_t st = aqc::mps_stream();
  const size_t blk = (size_t)(n + 1) * cap;
  if (!win.empty()) {
    if (!base->hwenv) {
      base->hwenv = (cplx*)aqc::dev_alloc(2 * (size_t)(n + 1) * blk * sizeof(cplx));
      AQC_REQUIRE(base->hwenv, "aqc_mps_zero_hw1_batch: out of device memory");
      AQC_HIP_CHECK(hipMemsetAsync(base->hwenv, 0, 2 * (size_t)(n + 1) * blk * sizeof(cplx), st));
      const double one = 1.0;
      AQC_HIP_CHECK(hipMemcpyAsync(base->hwenv, &one, sizeof(double), hipMemcpyHostToDevice, st));
      AQC_HIP_CHECK(hipMemcpyAsync(base->hwenv + (size_t)(n + 1) * blk + (size_t)n * blk, &one, sizeof(double),
                                   hipMemcpyHostToDevice, st));
      AQC_HIP_CHECK(hipStreamSynchronize(st));  // (the host constant's copies)
      base->hl = base->h0l = 0;
      base->hr = base->h0r = n;
    }
    cplx* HL = base->hwenv;
    cplx* HR = base->hwenv + (size_t)(n + 1) * blk;
    std::vector<HwRowsJob> rj;
    const int full = out_amps ? 1 : 0;
    auto rows_job = [&](int dir, int first, int nsteps, cplx* rows) {
      HwRowsJob j;
      j.gam = base->d.gam;
      j.lam = base->d.lam;
      j.dims = base->d.dims;
      j.n = n;
      j.cap = cap;
      j.dir = dir;
      j.first = first;
      j.nsteps = nsteps;
      j.full = full;
      j.rows = rows;
      rj.push_back(j);
    };
    // (the amplitudes need every row; the overlap alone row 0)
    const int hl = full ? base->hl : base->h0l, hr = full ? base->hr : base->h0r;
    if (need_l > hl) rows_job(0, hl, need_l - hl, HL);
    if (need_r < hr) rows_job(1, hr - 1, hr - need_r, HR);
    std::vector<HwWinJob> wj;
    const size_t jb = ((rj.size() * sizeof(HwRowsJob) + 255) / 256) * 256;
    const size_t wb = ((win.size() * sizeof(HwWinJob) + 255) / 256) * 256;
    const size_t rb = (((size_t)win.size() * (n + 1) * sizeof(cplx)) + 255) / 256 * 256;
    const size_t fnb = (size_t)win.size() * 2 * cap * sizeof(cplx);  // the chains' last vectors
    const size_t cb = ((win.size() * sizeof(int) + 255) / 256) * 256;  // hand-off counters
    size_t uyb = 0;  // with amps: each state's window vectors (2 (w + 1) cap)
    if (out_amps)
      for (int s : win) uyb += 2 * (size_t)(hi[s] - lo[s] + 2) * cap * sizeof(cplx);
    // the states' and base's error flags are gathered beside the results (one read-back: the
    // caller needs no separate aqc_mps_check_batch round trip)
    const size_t flb = (((size_t)ns + 1) * sizeof(int) + 255) / 256 * 256;
    char* d = (char*)aqc::dev_alloc(rb + flb + fnb + uyb + 256);
    AQC_REQUIRE(d, "aqc_mps_zero_hw1_batch: out of device memory");
    cplx* res = (cplx*)d;
    int* dflags = (int*)(d + rb);
    cplx* fin = (cplx*)(d + rb + flb);
    cplx* uy = (cplx*)(d + rb + flb + fnb);
    for (size_t k = 0; k < win.size(); ++k) {
      const int s = win[k];
      HwWinJob j;
      j.gam = hs[s]->d.gam;
      j.lam = hs[s]->d.lam;
      j.dims = hs[s]->d.dims;
      j.n = n;
      j.cap = cap;
      j.lo = lo[s];
      j.hi = hi[s];
      j.ml = HL + (size_t)lo[s] * blk;
      j.nr = HR + (size_t)(hi[s] + 1) * blk;
      j.ov = res + k * (n + 1);
      j.amps = out_amps ? res + k * (n + 1) + 1 : nullptr;
      j.uy = out_amps ? uy : nullptr;
      if (out_amps) uy += 2 * (size_t)(hi[s] - lo[s] + 2) * cap;
      j.fin = fin + k * 2 * (size_t)cap;
      j.cnt = nullptr;  // (set below: in the staging buffer)
      j.pad = 0;
      wj.push_back(j);
    }
    // (capacity <= 64: plus the right steps' 64 x 65 reduction tile)
    const size_t lds_win = (2 * (size_t)cap + 4 * 64 + (cap <= 64 ? 64 * 65 : 0)) * sizeof(cplx);
    const size_t lds_rows = (2 * (size_t)cap + 4 * kHwR * 64) * sizeof(cplx);
    // the job arrays through a pinned staging set of the ring (pageable copies were a host round
    // trip each, between the candidates' replay and these kernels)
    StagingLease lease(st);
    if (lease.rc() != AQC_OK) {
      aqc::dev_free(d);
      return lease.rc();
    }
    const size_t fpb = ((size_t)ns + 1) * sizeof(int*);
    rc = lease.ensure(jb + wb + cb + fpb);
    if (rc != AQC_OK) {
      aqc::dev_free(d);
      return rc;
    }
    char* hj = (char*)lease.buf().host;
    char* dj = (char*)lease.buf().dev;
    for (size_t k = 0; k < wj.size(); ++k) wj[k].cnt = (int*)(dj + jb + wb) + k;
    if (!rj.empty()) std::memcpy(hj, rj.data(), rj.size() * sizeof(HwRowsJob));
    std::memcpy(hj + jb, wj.data(), wj.size() * sizeof(HwWinJob));
    std::memset(hj + jb + wb, 0, cb);
    int** hfp = (int**)(hj + jb + wb + cb);
    for (int s = 0; s < ns; ++s) hfp[s] = hs[s]->d.flags;
    hfp[ns] = base->d.flags;
    if (int e = aqc::upload_async(dj, hj, jb + wb + cb + fpb, st)) {
      aqc::dev_free(d);
      return e;
    }
    static bool attr = false;
    if (!attr) {  // (up to 98 KB at capacity 1024)
      AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_hw_win, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
      AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_hw_rows, hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024));
      attr = true;
    }
    if (!rj.empty()) {
      hipLaunchKernelGGL(k_hw_rows, dim3((unsigned)rj.size(), full ? kHwRowsG : 1), dim3(kT), lds_rows, st,
                         (const HwRowsJob*)dj);
      AQC_CHECK_LAUNCH();
    }
    aqc::KernelTimer::begin(st, "mps_zero_hw1", 0.0, 0.0);
    hipLaunchKernelGGL(k_hw_win, dim3((unsigned)win.size(), 2), dim3(kT), lds_win, st, (const HwWinJob*)(dj + jb));
    aqc::KernelTimer::end(st);
    AQC_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_gather_flags, dim3(1), dim3(256), 0, st, (int* const*)(dj + jb + wb + cb), ns + 1, dflags);
    AQC_CHECK_LAUNCH();
    std::vector<cplx> h(rb / sizeof(cplx) + flb / sizeof(cplx));
    AQC_HIP_CHECK(hipMemcpyAsync(h.data(), res, rb + flb, hipMemcpyDeviceToHost, st));
    AQC_HIP_CHECK(hipStreamSynchronize(st));
    aqc::dev_free(d);
    {
      const int* hf = (const int*)((const char*)h.data() + rb);
      int first = AQC_OK;  // (every raised flag reset; the first error reported)
      for (int s = 0; s <= ns; ++s)
        if (hf[s]) {
          const int frc = check_flags(s < ns ? hs[s] : base);
          if (first == AQC_OK) first = frc;
        }
      if (first != AQC_OK) return first;
    }
    base->h0l = std::max(base->h0l, need_l);
    base->h0r = std::min(base->h0r, need_r);
    if (full) {
      base->hl = std::max(hl, need_l);
      base->hr = std::min(hr, need_r);
    }
    for (size_t k = 0; k < win.size(); ++k) {
      const int s = win[k];
      const cplx* v = h.data() + k * (n + 1);
      out_ov[2 * s] = v[0].x;  // mps_dot(psi, zero) = conj(amplitude of |0..0>)
      out_ov[2 * s + 1] = -v[0].y;
      if (out_amps)
        for (int q = 0; q < n; ++q) {
          out_amps[((size_t)s * n + q) * 2] = v[1 + q].x;
          out_amps[((size_t)s * n + q) * 2 + 1] = v[1 + q].y;
        }
    }
  }
  if (!fb.empty()) {  // the full chains
    std::vector<aqc_mps_t> fh;
    for (int s : fb) fh.push_back(hs[s]);
    std::vector<double> o(2 * fb.size()), a(out_amps ? 2 * fb.size() * n : 0);
    rc = aqc_mps_overlap_zero_batch(fh.data(), (int)fh.size(), o.data());
    if (rc != AQC_OK) return rc;
    if (out_amps) {
      rc = aqc_mps_amps_hw1_batch(fh.data(), (int)fh.size(), a.data());
      if (rc != AQC_OK) return rc;
    }
    fh.push_back(base);  // (their error flags and base's, as on the window path)
    rc = check_flags_batch(fh.data(), (int)fh.size());
    if (rc != AQC_OK) return rc;
    for (size_t k = 0; k < fb.size(); ++k) {
      const int s = fb[k];
      out_ov[2 * s] = o[2 * k];
      out_ov[2 * s + 1] = o[2 * k + 1];
      if (out_amps) std::memcpy(out_amps + (size_t)s * 2 * n, a.data() + k * 2 * n, 2 * n * sizeof(double));
    }
  }
  return AQC_OK;
}

int aqc_mps_amps_hw1(aqc_mps_t h, double* out) {
  AQC_REQUIRE(h && out, "aqc_mps_amps_hw1: null argument");
  int rc = aqc_mps_sort(h);
  if (rc != AQC_OK) return rc;
  std::vector<MeasJob> jobs(1, make_meas(h, h->d.scal));
  const MeasJob* dj = nullptr;
  rc = upload_jobs(jobs, &dj);
  if (rc != AQC_OK) return rc;
  hipStream_t st = aqc::mps_stream();
  hipLaunchKernelGGL(k_zero_chains, dim3(1, 2), dim3(kT), 2 * h->d.cap * sizeof(cplx), st, dj, h->d.cap);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_hw1, dim3(h->d.n, 1), dim3(kT), 0, st, dj);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipMemcpyAsync(out, h->d.scal, 2 * h->d.n * sizeof(double), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  return AQC_OK;
}

static int ensure_env(aqc_mps_t h) {
  if (h->d.env) return AQC_OK;
  const size_t cap = h->d.cap;
  h->d.env = (cplx*)aqc::dev_alloc(2 * (size_t)(h->d.n + 1) * cap * cap * sizeof(cplx));
  if (!h->d.env) {
    aqc::set_error("aqc_mps: out of device memory (environments)");
    return AQC_ERR_NOMEM;
  }
  return AQC_OK;
}

int aqc_mps_dot(aqc_mps_t a, aqc_mps_t b, double* re, double* im) {
  AQC_REQUIRE(a && b && re && im && a->d.n == b->d.n, "aqc_mps_dot: bad arguments");
  int rc = aqc_mps_sort(a);
  if (rc != AQC_OK) return rc;
  rc = aqc_mps_sort(b);
  if (rc != AQC_OK) return rc;
  rc = ensure_env(a);
  if (rc != AQC_OK) return rc;
  // env scratch sized for max(cap)
  const int cap = std::max(a->d.cap, b->d.cap);
  EnvJob j;
  std::memset(&j, 0, sizeof(j));
  if (a->d.cap != b->d.cap) {
    aqc::set_error("aqc_mps_dot: both MPS must share chi_cap");
    return AQC_ERR_ARG;
  }
  j.ga = a->d.gam;
  j.la = a->d.lam;
  j.da = a->d.dims;
  j.gb = b->d.gam;
  j.lb = b->d.lam;
  j.db = b->d.dims;
  j.n = a->d.n;
  j.cap = cap;
  j.env = a->d.env;
  j.tmp = a->d.tmp;
  j.keep_all = 0;
  j.right = 0;
  j.out = a->d.scal;
  std::vector<EnvJob> jobs(1, j);
  const EnvJob* dj = nullptr;
  rc = upload_jobs(jobs, &dj);
  if (rc != AQC_OK) return rc;
  hipStream_t st = aqc::mps_stream();
  hipLaunchKernelGGL(k_env, dim3(1), dim3(kT), 0, st, dj);
  AQC_CHECK_LAUNCH();
  cplx v;
  AQC_HIP_CHECK(hipMemcpyAsync(&v, a->d.scal, sizeof(cplx), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  *re = v.x;
  *im = v.y;
  return AQC_OK;
}

int aqc_mps_z_all(aqc_mps_t h, double* out) {
  AQC_REQUIRE(h && out, "aqc_mps_z_all: null argument");
  // the batched path (ent.hip: left / right environment chains over several workgroups on the
  // matrix cores, P_b per site, one trace each): O(n chi^3).  The per-site kernel used until round
  // 6 contracted L A R for each output entry, O(chi^4) per site -- 83 s for one 21-qubit state at
  // bond 512 (profiles/r6_zall_cap1024_kernel_stats.csv).
  return aqc_mps_z_all_batch(&h, 1, out);
}

}  // extern "C"
