// MPS engine internals shared by mps.hip (gate application, measurements) and grad.hip
// (candidate sweep).
#pragma once

#include <vector>

#include "aqc_internal.h"

namespace aqc {

// Device layout of one MPS (Vidal form, as Aer's MPS simulator keeps it):
//   gam : n sites x [2][cap][cap] complex, row-major [s][l][r]; site i uses l < dims[i],
//         r < dims[i+1].
//   lam : (n+1) bonds x cap doubles; bond b sits left of site b; lam[0] = lam[n] = {1}.
//   dims: (n+1) ints on device, dims[0] = dims[n] = 1.
// The qubit permutation created by Aer's swap routing lives on the host (order / loc).
// Largest two-site column count 2 chi (bond capacity <= 1024): the singular-value buffer holds the
// raw column norms at [0, kSigMax) and the sorted values at [kSigMax, 2 kSigMax).  sig[kSigTail]:
// the part of the reduce_zeros tail sum that an SVD path which decides the kept count itself (the
// Gram paths, svd_gram.h / gram_big.hip) has already removed -- it writes the kept singular values
// and zeros, and the rank step's tail rule continues from this sum (then resets it to 0).
constexpr int kSigMax = 2048;
constexpr int kMaxCap = kSigMax / 2;
constexpr int kSigTail = 2 * kSigMax;
constexpr int kSigLen = 2 * kSigMax + 2;  // doubles
// Two-site work buffer (complex elements): 4 cap^2 (the Jacobi's working columns), and at least what
// the 2 chi = 128 Gram path lays out in it (svd_gram.h: reflectors, W, the compact-WY factors and the
// inverse-iteration scratch of more than 64 kept vectors)
constexpr size_t kGramWorkElems = 36864;
inline size_t work_elems(size_t cap) { return 4 * cap * cap > kGramWorkElems ? 4 * cap * cap : kGramWorkElems; }

struct MpsDev {
  int n = 0;
  int cap = 0;
  cplx* gam = nullptr;
  double* lam = nullptr;
  int* dims = nullptr;
  // two-site workspace
  cplx* theta = nullptr;  // (2cap)^2, column-major M x N
  cplx* work = nullptr;   // work_elems(cap): Jacobi working columns / Gram-path scratch
  double* sig = nullptr;  // kSigLen: column norms, then the sorted values, then the removed tail
  int* perm = nullptr;    // kSigMax sorted -> column index
  int* flags = nullptr;   // [0] capacity overflow, [1] jacobi non-convergence, [2] max sweeps used
  // measurement workspace
  cplx* env = nullptr;    // 2 * (n+1) * cap * cap  (left and right environments)
  cplx* tmp = nullptr;    // 2 * cap * cap
  cplx* vec = nullptr;    // 2 * (n+1) * cap  (left / right zero-chains)
  cplx* scal = nullptr;   // scratch results (2n + 8 complex)

  size_t site_stride() const { return (size_t)2 * cap * cap; }
  cplx* site(int i) const { return gam + (size_t)i * site_stride(); }
  double* bond(int b) const { return lam + (size_t)b * cap; }
};

// One two-site update of one state (k_theta -> SVD -> k_rank -> k_split_*), see mps.hip.
struct TwoSiteJob {
  cplx* gp;
  cplx* gq;
  const double* ll;
  double* lm;
  const double* lr;
  int* dims;  // &dims[p] : dims[0] = chi_l, dims[1] = chi_m, dims[2] = chi_r
  cplx* theta;
  cplx* work;
  double* sig;
  int* perm;
  int* flags;
  int cap;
  int max_chi;
  double thr;
  double jtol;  // Jacobi rotation threshold factor
  double jtiny; // sweep stop: a sweep whose counted rotations all had |t| <= jtiny is the last
  int qr;      // 1: Jacobi ran on R^H of a pivoted QR -> W holds the other side (see k_jacobi_reg)
  int dbg;      // diagnostics (aqc_svd_debug): 1 = stop after the QR phase, write X unpermuted
  int gram;     // 1: try the Gram / tridiagonal SVD first (svd_gram.h), the Jacobi as fallback
  int pad_;
  double jnoise;  // Jacobi dot-product noise floor, in units of eps ||W|| (|a| + |b|) (0: off)
  cplx G[16];  // row = 2*s1'+s2' (out), col = 2*s1+s2 (in)
};

// Squared dot-product noise floor factor of the Jacobi rotations: a pair rotates only if
// |g|^2 > jacobi_noise2(j, ||W||^2) (|a|^2 + |b|^2) (mps.hip, jacobi_reg_body).
__device__ __forceinline__ double jacobi_noise2(const TwoSiteJob& j, double fro2) {
  const double e = j.jnoise * 2.220446049250313e-16;
  return 2.0 * e * e * fro2;
}

// Rotation parameters of the pair (alpha, beta, gamma = gx + i gy): t = sgn(zeta) /
// (|zeta| + sqrt(1 + zeta^2)), zeta = (beta - alpha) / (2|gamma|), c = 1/sqrt(1 + t^2) and
// s e = c t gamma / |gamma|.  v_rsq_f64 / v_rcp_f64 seeds with two Newton steps each (full double
// precision) instead of the IEEE sqrt / divide sequences: this chain is serial per round.
__device__ __forceinline__ void jacobi_params(double al, double be, double gx, double gy, double g2, double& c,
                                              double& ex, double& ey) {
  double rg = __builtin_amdgcn_rsq(g2);  // 1 / |gamma|
  rg = rg * fma(-0.5 * g2 * rg, rg, 1.5);
  rg = rg * fma(-0.5 * g2 * rg, rg, 1.5);
  const double zeta = 0.5 * (be - al) * rg;
  const double q = fma(zeta, zeta, 1.0);
  double rq = __builtin_amdgcn_rsq(q);
  rq = rq * fma(-0.5 * q * rq, rq, 1.5);
  rq = rq * fma(-0.5 * q * rq, rq, 1.5);
  const double den = fabs(zeta) + q * rq;  // |zeta| + sqrt(1 + zeta^2)
  double inv = __builtin_amdgcn_rcp(den);
  inv = inv * fma(-den, inv, 2.0);
  inv = inv * fma(-den, inv, 2.0);
  const double t = zeta >= 0 ? inv : -inv;
  const double p = fma(t, t, 1.0);
  double cc = __builtin_amdgcn_rsq(p);
  cc = cc * fma(-0.5 * p * cc, cc, 1.5);
  cc = cc * fma(-0.5 * p * cc, cc, 1.5);
  c = cc;
  const double sc = cc * t * rg;
  ex = gx * sc;
  ey = gy * sc;
}

// Jacobi rotation of the pair (alpha = |a|^2, beta = |b|^2, |g|^2 = |a^H b|^2): t = sgn(zeta) /
// (|zeta| + sqrt(1 + zeta^2)), zeta = (beta - alpha) / (2|g|), c = 1 / sqrt(p), p = 1 + t^2,
// rg = 1 / |g| (rsq / rcp seeds with two Newton steps each: full double precision).
__device__ __forceinline__ void jacobi_tc(double al, double be, double g2, double& t, double& c, double& p,
                                          double& rg) {
  double r = __builtin_amdgcn_rsq(g2);
  r = r * fma(-0.5 * g2 * r, r, 1.5);
  r = r * fma(-0.5 * g2 * r, r, 1.5);
  rg = r;
  const double zeta = 0.5 * (be - al) * r;
  const double q = fma(zeta, zeta, 1.0);
  double rq = __builtin_amdgcn_rsq(q);
  rq = rq * fma(-0.5 * q * rq, rq, 1.5);
  rq = rq * fma(-0.5 * q * rq, rq, 1.5);
  const double den = fabs(zeta) + q * rq;
  double inv = __builtin_amdgcn_rcp(den);
  inv = inv * fma(-den, inv, 2.0);
  inv = inv * fma(-den, inv, 2.0);
  t = zeta >= 0 ? inv : -inv;
  p = fma(t, t, 1.0);
  double cc = __builtin_amdgcn_rsq(p);
  cc = cc * fma(-0.5 * p * cc, cc, 1.5);
  cc = cc * fma(-0.5 * p * cc, cc, 1.5);
  c = cc;
}

// The same rotation without |g|: with h = (beta - alpha) / 2, t / |g| = sgn(h) / (|h| + sqrt(h^2 +
// |g|^2)) =: te, so t e = te g, t |g| = te |g|^2 and p = 1 + t^2 = 1 + te^2 |g|^2.  One rsq and
// one rcp, each with a single Newton step (their ~2^-23 seeds -> ~2^-46: the angle needs no more,
// as long as c = 1 / sqrt(p) is exact for the t actually applied -- two Newton steps there).
__device__ __forceinline__ void jacobi_te(double al, double be, double g2, double& te, double& c, double& p) {
  const double h = 0.5 * (be - al);
  const double q = fma(h, h, g2);
  double rq = __builtin_amdgcn_rsq(q);
  rq = rq * fma(-0.5 * q * rq, rq, 1.5);
  const double den = fabs(h) + q * rq;
  double inv = __builtin_amdgcn_rcp(den);
  inv = inv * fma(-den, inv, 2.0);
  te = h >= 0 ? inv : -inv;
  p = fma(te * te, g2, 1.0);
  double cc = __builtin_amdgcn_rsq(p);
  cc = cc * fma(-0.5 * p * cc, cc, 1.5);
  cc = cc * fma(-0.5 * p * cc, cc, 1.5);
  c = cc;
}

constexpr double kReduceChop = 1e-16;  // reduce_zeros' CHOP on sigma^2 (mps.hip kChop)

// reduce_zeros (oracle/mps.py truncation_rank: Aer's rule as the reference drives it,
// aer_mps_backend.py:27-42) on the top KE eigenvalues lam (descending, = sigma^2) of G, each known to
// +-err: CHOP (sigma^2 > 1e-16), the max_chi cap, then the tail rule (drop the smallest while the
// dropped sum stays below thr).  Every comparison must hold for any values inside the error bars --
// err is the multisection bracket, plus the noise of forming and reducing G (16 C eps ||T||) -- and
// the kept values must clear the Gram path's floor (lambda_K > floor lambda_1, 1e-9); otherwise -1 (the
// caller declines and the Jacobi decides).  An eigenvalue whose CHOP decision is open may still be
// dropped by the tail rule from either start, which then decides nothing: it enters the tail as
// [0, lam + err].  Returns the kept count K, and in tail_out the dropped tail sum (handed to
// rank_body through sig[kSigTail], whose own tail rule then keeps all K).
// cert (optional): where that fails only because of values in the CHOP's open band -- a rank-deficient
// theta', whose numerically zero eigenvalues come out of G as +-(noise) -- the decision that they all
// fall below the CHOP, with *cert = 1: valid if the caller then shows ||X - X V V^H||_F^2 < CHOP / 2
// for the K kept right vectors V (every dropped sigma^2 is then below it; gram_big.hip k_gb_cert).
[[maybe_unused]] static __device__ __noinline__ int gram_keep(const double* lam, const double* err, int KE, int C, int max_chi,
                                             double thr, double tn, double floor, double& tail_out,
                                             int* cert = nullptr) {
  const double noise = 16.0 * C * 2.220446049250313e-16 * tn;
  int k_lo = 0, k_hi = 0;  // counts surely / possibly above the CHOP (lam descending)
  for (int i = 0; i < KE; ++i) {
    const double e = err[i] + noise;
    if (lam[i] - e > kReduceChop) k_lo = i + 1;
    if (lam[i] + e > kReduceChop) k_hi = i + 1;
  }
  if (cert) *cert = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    // attempt 0: the open values as [0, lam + err]; attempt 1 (cert): the open values chopped
    if (attempt == 1 && !(cert && k_hi > k_lo)) return -1;
    int k = attempt == 0 ? k_hi : k_lo;
    if (k < 1) k = 1;
    if (max_chi > 0 && k > max_chi) k = max_chi;
    double tail = 0.0, unc = 0.0;
    bool ok = true;
    while (k > 1) {
      const int i = k - 1;
      const double e = err[i] + noise;
      double v = lam[i], ev = e;
      if (i >= k_lo) {  // CHOP open: contributes anything in [0, lam + e] if dropped
        v = 0.5 * (lam[i] + e);
        ev = v;
      }
      const double sum = tail + v, m = unc + ev;
      if (fabs(sum - thr) <= m) {  // the comparison is open
        ok = false;
        break;
      }
      if (sum >= thr) break;
      if (attempt == 1) {  // (a surely-kept value dropped: the certificate cannot tell them apart)
        ok = false;
        break;
      }
      tail = sum;
      unc = m;
      --k;
    }
    if (!ok) continue;
    if (k > k_lo) continue;  // a kept value whose CHOP is open (also far below the floor)
    if (!(lam[0] > 0.0) || !(lam[k - 1] > floor * lam[0])) return -1;
    tail_out = tail;
    if (attempt == 1) *cert = !(max_chi > 0 && k_lo >= max_chi);
    return k;
  }
  return -1;
}

// Multi-workgroup block one-sided Jacobi SVD for 2 * chi > 128 (bjacobi.hip): factors the nj
// two-site thetas of `jobs` (device array) into the k_jacobi output contract (W columns = U sigma,
// sig = column norms, qr = 0).  Enqueued on `st`; synchronises the host once per sweep (from the
// third on) to stop when every decomposition has converged.
int block_jacobi(const TwoSiteJob* jobs, int nj, int cap_max, hipStream_t st);

// Two-site SVDs at 2 chi = side in (128, 2048] (gram_big.hip): the multi-workgroup Gram path
// (G = X^H X of the C x C side, C = min(2 chi_l, 2 chi_r) <= 1024; tridiagonalisation over several
// workgroups per job, inverse iteration, V = Q Z; output contract qr = 1, written into the device
// job), the block Jacobi for the jobs it declines (and for C > 1024).
// hjobs: host copies of the device jobs (qr = 0).  Synchronises the host once.
int big_svd(const TwoSiteJob* hjobs, const TwoSiteJob* jobs, int nj, int side, int cap_max, hipStream_t st);

hipStream_t mps_stream();
hipStream_t mps_stream_if_any(int dev);

}  // namespace aqc

struct aqc_mps_s {
  aqc::MpsDev d;
  double thr = 1e-16;
  int max_chi = 0;
  int dev = 0;  // the device the handle's buffers live on (aqc_mps_create's current device)
  std::vector<int> order;  // site -> qubit
  // host upper bounds of the bond dimensions (n + 1; exact after a load or a dims read-back, then
  // advanced per two-site update as min(2 chi_l, 2 chi_r, cap, max_chi)): the lock-step path picks
  // each wave's SVD kernel by the largest theta the wave can hold, not by the capacity
  std::vector<int> ub;
  std::vector<int> loc;    // qubit -> site
  // Reload bookkeeping (aqc_mps_copy_batch): `version` changes with every change of the device
  // contents; after a copy from the handle with id `synced_src` at its version `synced_ver`, the
  // Gamma sites changed since are [dirty_lo, dirty_hi], so a reload from the same, unchanged
  // source rewrites only those (lambdas and dims in full): the result is that of a full copy.
  unsigned long long uid = 0;
  unsigned long long version = 0;
  unsigned long long synced_src = 0;
  unsigned long long synced_ver = 0;
  int dirty_lo = 1 << 30, dirty_hi = -1;
  // Cached Z-sum environments (ent.hip, aqc_mps_z_sum_batch): zenv holds, per bond b, the left pair
  // (L_b, LZ_b) and the right pair (R_b, RZ_b); left pairs are current for bonds <= zl, right pairs
  // for bonds >= zr.  A rewrite of Gamma sites lo..hi (and the lambdas between them) leaves the left
  // environments up to bond lo and the right ones from bond hi + 1 as they were.
  aqc::cplx* zenv = nullptr;
  int zl = 0, zr = 1 << 30;
  // Cached zero / Hamming-weight-1 rows (mps.hip, aqc_mps_zero_hw1_batch), per bond b: from the
  // left <0..0| A_0 .. A_{b-1} (row 0) and the same with site k < b flipped (row 1 + k); from the
  // right A_b .. A_{n-1} |0..0> (row 0) and with site k >= b flipped (row 1 + k).  Every row is
  // current for bonds <= hl (left) and >= hr (right), row 0 for bonds <= h0l / >= h0r.
  aqc::cplx* hwenv = nullptr;
  int hl = 0, hr = 1 << 30, h0l = 0, h0r = 1 << 30;
  void changed(int lo, int hi) {  // Gamma sites lo..hi rewritten
    ++version;
    dirty_lo = lo < dirty_lo ? lo : dirty_lo;
    dirty_hi = hi > dirty_hi ? hi : dirty_hi;
    zl = lo < zl ? lo : zl;
    zr = hi + 1 > zr ? hi + 1 : zr;
    hl = lo < hl ? lo : hl;
    hr = hi + 1 > hr ? hi + 1 : hr;
    h0l = lo < h0l ? lo : h0l;
    h0r = hi + 1 > h0r ? hi + 1 : h0r;
  }
  void changed_all() {
    ++version;
    synced_src = 0;
    zenv_stale();
  }
  void zenv_stale() {  // every cached environment and row past the boundaries
    zl = hl = h0l = 0;
    zr = hr = h0r = d.n;
  }
  // the one device block the handle's fixed buffers are carved from (aqc::dev_alloc)
  void* base = nullptr;
  // scratch for the candidate sweep (grad.hip), allocated lazily
  aqc::cplx* gw = nullptr;
  size_t gw_bytes = 0;
  // extra two-site workspaces for concurrent updates of disjoint bonds (mps.hip run_waves)
  struct Slot {
    aqc::cplx* theta = nullptr;
    aqc::cplx* work = nullptr;
    double* sig = nullptr;
    int* perm = nullptr;
  };
  std::vector<Slot> slots;
};
