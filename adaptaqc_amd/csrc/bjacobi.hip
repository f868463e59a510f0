// Multi-workgroup block one-sided Jacobi SVD for the large two-site updates (2 chi > 128:
// chi = 128 and the 100-qubit chi = 256 MPS preparation of BASELINE config 5).
//
// The single-workgroup kernels of mps.hip keep a whole 2chi x 2chi theta in one CU (VGPRs for
// chi <= 64).  A 512 x 512 complex theta is 4 MB: it lives in HBM / L2 here, and the cyclic
// one-sided Jacobi is spread over many CUs by column blocks (Hestenes block-Jacobi):
//   * W (L rows x C columns, column-major, ld = L) is cut into nb blocks of kB = 16 columns;
//   * one sweep = one "intra" launch (every block orthogonalises its own 16 columns, one
//     workgroup per block, round-robin in LDS) + nb - 1 block-pair launches (round-robin
//     tournament over the blocks: nb / 2 workgroups, each orthogonalising block I against block J
//     through their 32 x 32 Gram matrix on the matrix cores, k_bj_pair below);
//   * launch boundaries are the only inter-workgroup synchronisation (no grid barrier, no
//     cross-XCD coherence assumptions).
// Rotation rule, thresholds and stop test are those of k_jacobi_reg (mps.hip): relative
// threshold L eps (and the dot-product noise floor jnoise eps ||W|| (|a| + |b|)), squared-norm floor
// ||W||^2 1e-24, a sweep without rotations above 4x the
// threshold -- or with only rotations moving <= j.jtiny^2 of the norms (t|g|) -- is the last.  Output: W's columns = U sigma,
// sig = their norms (the k_jacobi contract consumed by k_rank / k_split_*, qr = 0).
#include <cstdlib>

#include "mps_internal.h"

namespace aqc {
namespace {

constexpr int kB = 16;        // columns per block
constexpr int kMaxSweepsBJ = 40;

struct BJState {
  double fro;   // ||W||_F^2
  int rot;      // rotations above noise in this sweep
  int big;      // rotations with |t| > jtiny in this sweep
  int done;     // converged (later launches return at once)
  int sweeps;   // sweeps run
  int pad[2];
};

// Sum over the 64 lanes of a wave, result in every lane: DPP row sums, then a two-step
// ds_bpermute butterfly across the rows (the row_bcast15/31 + readlane form stalled on the
// VALU -> SGPR -> VALU hazards).
__device__ __forceinline__ double wave_sum(double v) {
  v = row_sum16(v);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ void job_shape(const TwoSiteJob& j, int& L, int& C, bool& tr) {
  const int M = 2 * j.dims[0], N = 2 * j.dims[2];
  tr = M < N;
  L = tr ? N : M;
  C = tr ? M : N;
}

// round-robin tournament on c (even) players: position 0 fixed, the others rotate
__device__ __forceinline__ int rr(int pos, int r, int c) { return pos == 0 ? 0 : ((pos - 1 + r) % (c - 1)) + 1; }

// W <- theta (or theta^H when M < N) with the columns in descending norm order, ||W||_F^2 into
// st.fro.  One workgroup per job.  The column order of W is free (k_rank sorts the singular
// values, k_split recovers the other side from theta), and a one-sided Jacobi started on
// norm-sorted columns converges in fewer sweeps (de Rijk).  grid (nj), 1024 threads.
// (up to kInitCols = 2048 columns: bond capacity 1024; two sort entries per thread)
constexpr int kInitCols = 2048;
__global__ __launch_bounds__(1024) void k_bj_init(const TwoSiteJob* __restrict__ jobs, BJState* __restrict__ st) {
  const TwoSiteJob& j = jobs[blockIdx.x];
  int L, C;
  bool tr;
  job_shape(j, L, C, tr);
  const int M = 2 * j.dims[0];
  __shared__ double key[kInitCols];
  __shared__ int idx[kInitCols];
  __shared__ double red[16];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  auto elem = [&](int row, int col) -> cplx {
    return tr ? cconj(j.theta[(size_t)row * M + col]) : j.theta[(size_t)col * M + row];
  };
  int P = 1024;  // sort length: 1024, or the columns rounded up to a power of two above it
  while (P < C) P <<= 1;
  double f = 0.0;
  for (int c = w; c < P; c += 16) {  // column norms, one wave per column
    double x = 0.0;
    if (c < C)
      for (int r = lane; r < L; r += 64) {
        const cplx v = elem(r, c);
        x = fma(v.x, v.x, fma(v.y, v.y, x));
      }
    x = wave_sum(x);
    f += x;
    if (lane == 0) key[c] = c < C ? x : -1.0, idx[c] = c;
  }
  if (lane == 0) red[w] = f;
  __syncthreads();
  // bitonic sort of P (key, idx), descending key (padding keys -1 sink to the end)
  for (int k = 2; k <= P; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = threadIdx.x; i < P; i += 1024) {
        const int l = i ^ jj;
        if (l > i) {
          const bool desc = (i & k) == 0;
          const double a = key[i], b = key[l];
          if (desc ? (a < b) : (a > b)) {
            key[i] = b, key[l] = a;
            const int t = idx[i];
            idx[i] = idx[l], idx[l] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int c = w; c < C; c += 16) {
    const int src = idx[c];
    for (int r = lane; r < L; r += 64) j.work[(size_t)c * L + r] = elem(r, src);
  }
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int q = 0; q < 16; ++q) t += red[q];
    st[blockIdx.x].fro = t;
  }
}

// One pair rotation of scaled columns a = da * (sr, si), b = db * (mr, mi) with tracked squared
// norms na, nb (the scheme of k_jacobi_reg, mps.hip: v_a' = v_a - mu v_b, v_b' = v_b + nu v_a,
// d' = c d, n_a' = n_a - t|g|, n_b' = n_b + t|g|, exact recompute on a 1e6 drop).  MAXR rows per
// lane, 64 lanes.  Returns whether the pair was rotated; rot / big collect the stop-test flags.
// With bcol != nullptr the new b goes straight to that LDS column (row lane + 64 i) instead of
// back into mr / mi.
template <int MAXR>
__device__ __forceinline__ bool rotate_pair(double (&sr)[MAXR], double (&si)[MAXR], double (&mr)[MAXR],
                                            double (&mi)[MAXR], double& na, double& da, double& ida, double& nb,
                                            double& db, double& idb, double tol2, double nfl2, double floor2,
                                            double tiny2, int& rot, int& big,
                                            double2* bcol = nullptr) {
  double gx = 0, gy = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    gx = fma(sr[i], mr[i], fma(si[i], mi[i], gx));  // conj(a) * b
    gy = fma(sr[i], mi[i], fma(-si[i], mr[i], gy));
  }
  const double dd = da * db;
  gx = wave_sum(gx) * dd;
  gy = wave_sum(gy) * dd;
  const double g2 = gx * gx + gy * gy;
  // relative threshold, and the dot-product noise floor of columns with ~eps ||W|| absolute error
  // (mps.hip, jacobi_reg_body): nfl2 = 2 (jnoise eps)^2 ||W||^2
  const double thr = fmax(tol2 * na * nb, nfl2 * (na + nb));
  if (!(g2 > thr && na > floor2 && nb > floor2)) return false;
  double te, c, p;  // te = t / |g|, p = 1 + t^2
  jacobi_te(na, nb, g2, te, c, p);
  if (g2 > 16.0 * thr) {
    rot = 1;
    if (fabs(te) * g2 > tiny2 * (na + nb)) big = 1;  // t|g| above jtiny^2 of the norms (jacobi_reg_body)
  }
  const double ra = db * ida, ira = da * idb;
  const double mux = te * gx * ra, muy = -te * gy * ra;
  const double nux = te * gx * ira, nuy = te * gy * ira;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const double ar = sr[i], ai = si[i], br = mr[i], bi = mi[i];
    sr[i] = fma(-mux, br, fma(muy, bi, ar));
    si[i] = fma(-mux, bi, fma(-muy, br, ai));
    const double nr = fma(nux, ar, fma(-nuy, ai, br)), ni = fma(nux, ai, fma(nuy, ar, bi));
    if (bcol) {
      bcol[lane_id() + 64 * i] = make_double2(nr, ni);
    } else {
      mr[i] = nr;
      mi[i] = ni;
    }
  }
  const double ic = p * c;
  da *= c, ida *= ic, db *= c, idb *= ic;
  const double tg = te * g2;
  double na2 = na - tg, nb2 = nb + tg;
  if (na2 < 1e-6 * na || nb2 < 1e-6 * nb) {
    double x = 0, y = 0;
    if (bcol) asm volatile("" ::: "memory");  // re-read b from LDS (own lanes' writes: in order)
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
      x = fma(sr[i], sr[i], fma(si[i], si[i], x));
      const double2 v = bcol ? bcol[lane_id() + 64 * i] : make_double2(mr[i], mi[i]);
      y = fma(v.x, v.x, fma(v.y, v.y, y));
    }
    na2 = wave_sum(x) * da * da;
    nb2 = wave_sum(y) * db * db;
  }
  na = na2, nb = nb2;
  return true;
}

template <int MAXR>
__device__ __forceinline__ double col_norm2(const double (&r)[MAXR], const double (&i_)[MAXR]) {
  double x = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) x = fma(r[i], r[i], fma(i_[i], i_[i], x));
  return wave_sum(x);
}

__device__ __forceinline__ double tol_sq(const TwoSiteJob& j, int L) {
  const double tol = j.jtol * (double)L * 2.220446049250313e-16;
  return tol * tol;
}

// Intra-block visits: one workgroup (8 waves) per block; the block's 16 columns in LDS, 15
// round-robin rounds of 8 pairs.  grid (nb, nj).
template <int MAXR>
__global__ __launch_bounds__(512) void k_bj_intra(const TwoSiteJob* __restrict__ jobs, BJState* __restrict__ st) {
  BJState& s = st[blockIdx.y];
  if (s.done) return;
  const TwoSiteJob& j = jobs[blockIdx.y];
  int L, C;
  bool tr;
  job_shape(j, L, C, tr);
  const int c0 = blockIdx.x * kB;
  if (c0 >= C) return;
  const int nc = min(kB, C - c0);
  extern __shared__ double2 cols[];  // kB x (64 MAXR)
  constexpr int ldl = 64 * MAXR;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  cplx* W = j.work + (size_t)c0 * L;
  for (int k = w; k < kB; k += 8) {
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
      const int row = lane + 64 * i;
      cols[k * ldl + row] = (k < nc && row < L) ? W[(size_t)k * L + row] : make_double2(0, 0);
    }
  }
  __syncthreads();
  __shared__ double cn[kB], cd[kB], cid[kB];  // tracked norms and scales of the 16 columns
  for (int k = w; k < kB; k += 8) {
    double x = 0;
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
      const double2 v = cols[k * ldl + lane + 64 * i];
      x = fma(v.x, v.x, fma(v.y, v.y, x));
    }
    x = wave_sum(x);
    if (lane == 0) cn[k] = x, cd[k] = 1.0, cid[k] = 1.0;
  }
  __syncthreads();
  const double tol2 = tol_sq(j, L), floor2 = s.fro * 1e-24;
  int rot = 0, big = 0;
  for (int r = 0; r < kB - 1; ++r) {
    const int a = rr(w, r, kB), b = rr(kB - 1 - w, r, kB);
    double sr[MAXR], si[MAXR], mr[MAXR], mi[MAXR];
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
      const double2 x = cols[a * ldl + lane + 64 * i], y = cols[b * ldl + lane + 64 * i];
      sr[i] = x.x, si[i] = x.y, mr[i] = y.x, mi[i] = y.y;
    }
    double na = cn[a], da = cd[a], ida = cid[a], nb = cn[b], db = cd[b], idb = cid[b];
    if (rotate_pair<MAXR>(sr, si, mr, mi, na, da, ida, nb, db, idb, tol2, jacobi_noise2(j, s.fro), floor2,
                          j.jtiny * j.jtiny, rot, big)) {
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        cols[a * ldl + lane + 64 * i] = make_double2(sr[i], si[i]);
        cols[b * ldl + lane + 64 * i] = make_double2(mr[i], mi[i]);
      }
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) cn[a] = na, cd[a] = da, cid[a] = ida, cn[b] = nb, cd[b] = db, cid[b] = idb;
    }
    __syncthreads();
  }
  for (int k = w; k < nc; k += 8) {
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
      const int row = lane + 64 * i;
      if (row < L) {
        const double2 v = cols[k * ldl + row];
        W[(size_t)k * L + row] = make_double2(v.x * cd[k], v.y * cd[k]);
      }
    }
  }
  if (lane == 0 && rot) atomicOr(&s.rot, 1);
  if (lane == 0 && big) atomicOr(&s.big, 1);
}

// Block-pair visit of tournament round `round` (after each sweep's intra launch): workgroup p orthogonalises the 32 columns of blocks I = rr(p) and
// J = rr(nb-1-p) together through their Gram matrix -- Hestenes block Jacobi with one inner sweep:
//   1. G = A^H A (A = [W_I W_J], L x 32) on the matrix cores: wave w takes a quarter of the rows,
//      three 16 x 16 tiles (G is Hermitian), partial sums through the LDS;
//   2. one cyclic Jacobi sweep on G: 31 rounds of 16 disjoint rotations (round-robin), each round
//      G <- J^H G J and V <- V J computed elementwise from the previous round's copies (double-
//      buffered LDS), the pair's own 2 x 2 block set exactly (a - t|g|, b + t|g|, 0); rotation rule,
//      thresholds and stop flags those of rotate_pair on the Gram entries;
//   3. A <- A V on the matrix cores as A'^T = V^T A^T (a lane group reads and writes 16
//      consecutive rows of one column).
// FULL = false (2 chi <= 512): the blocks' own Gram blocks are taken as diagonal (each sweep's
// intra launch has just orthogonalised them; norms only) and the visit rotates the 16 x 16 cross
// pairs in 16 rounds.  FULL = true (2 chi up to 1024, where the intra launch's block would not fit
// the LDS; 2 chi = 2048 too, bond capacity 1024): the visit forms all of G and rotates every pair of
// the 32 columns (31 round-robin rounds), so no intra launch is needed.  grid (nb / 2, nj), 256 threads.
typedef double __attribute__((ext_vector_type(4))) d4_t;
constexpr int kPairCols = 2 * kB;  // 32
struct PairLds {
  cplx G[2][kPairCols][kPairCols + 1];
  cplx V[2][kPairCols][kPairCols + 1];
  double rc[kB], rtg[kB];
  cplx rus[kB];
};
constexpr size_t kPairLdsBytes = sizeof(PairLds);  // dynamic LDS (> 64 KB of static)

// shader-clock ticks of the pair visits' phases summed over workgroups (thread 0): Gram, Jacobi,
// A V, visits (aqc_bj_ticks)
__device__ unsigned long long g_bj_ticks[4];

template <int MAXR, bool kPairFullGram>
__global__ __launch_bounds__(256, 2) void k_bj_pair(const TwoSiteJob* __restrict__ jobs, BJState* __restrict__ st,
                                                 int round, int nb) {
  BJState& s = st[blockIdx.y];
  if (s.done) return;
  const TwoSiteJob& j = jobs[blockIdx.y];
  int L, C;
  bool tr;
  job_shape(j, L, C, tr);
  const int I = rr(blockIdx.x, round, nb), J = rr(nb - 1 - blockIdx.x, round, nb);
  const int cI = I * kB, cJ = J * kB;
  if (cI >= C && cJ >= C) return;
  const int nI = max(0, min(kB, C - cI)), nJ = max(0, min(kB, C - cJ));
  extern __shared__ double2 pair_raw[];
  PairLds& sm = *reinterpret_cast<PairLds*>(pair_raw);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  // local column c (0..31) -> W column, or -1 (padding: zero)
  auto wcol = [&](int c) { return c < kB ? (c < nI ? cI + c : -1) : (c - kB < nJ ? cJ + c - kB : -1); };
  const cplx* W = j.work;
  unsigned long long t0 = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull, t1 = 0, t2 = 0;
  constexpr int RW = 16 * MAXR;  // rows per wave
  const int r0 = w * RW;
  // ---- 1: G = A^H A ----
  {
    d4_t gr[3], gi[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) gr[t] = d4_t{0, 0, 0, 0}, gi[t] = d4_t{0, 0, 0, 0};
    double n0 = 0.0, n1 = 0.0;
    const int ca = wcol(li), cb = wcol(kB + li);
    // loads kPf k steps ahead of the MFMAs (W streams from the Infinity Cache)
    constexpr int kPf = 4;
    cplx pa[kPf], pb[kPf];
    auto ld = [&](int ks, cplx& x, cplx& y) {
      const int row = r0 + 4 * ks + lk;
      x = (ca >= 0 && row < L) ? ldg(W + (size_t)ca * L + row) : cmk(0, 0);
      y = (cb >= 0 && row < L) ? ldg(W + (size_t)cb * L + row) : cmk(0, 0);
    };
#pragma unroll
    for (int u = 0; u < kPf; ++u) ld(u, pa[u], pb[u]);
#pragma unroll kPf
    for (int ks = 0; ks < RW / 4; ++ks) {
      const cplx a0 = pa[ks % kPf], a1 = pb[ks % kPf];
      if (ks + kPf < RW / 4) ld(ks + kPf, pa[ks % kPf], pb[ks % kPf]);
      // conj(x) y: Re += xr yr + xi yi, Im += xr yi - xi yr
      auto acc = [&](int t, cplx x, cplx y) {
        gr[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.x, gr[t], 0, 0, 0);
        gr[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x.y, y.y, gr[t], 0, 0, 0);
        gi[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.y, gi[t], 0, 0, 0);
        gi[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-x.y, y.x, gi[t], 0, 0, 0);
      };
      if constexpr (kPairFullGram) {
        acc(0, a0, a0);
        acc(2, a1, a1);
      } else {  // the blocks' own Gram entries: column norms only (intra launch orthogonalises them)
        n0 = fma(a0.x, a0.x, fma(a0.y, a0.y, n0));
        n1 = fma(a1.x, a1.x, fma(a1.y, a1.y, n1));
      }
      acc(1, a0, a1);
    }
    if constexpr (!kPairFullGram) {  // norms of columns li (block I) and 16 + li (J) in tiles 0, 2
      n0 += __shfl_xor(n0, 16);
      n0 += __shfl_xor(n0, 32);
      n1 += __shfl_xor(n1, 16);
      n1 += __shfl_xor(n1, 32);
      // accumulator entry (row lk + 4q, col li): the diagonal sits at lk + 4q == li
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool dg = lk + 4 * q == li;
        gr[0][q] = dg ? n0 : 0.0, gi[0][q] = 0.0;
        gr[2][q] = dg ? n1 : 0.0, gi[2][q] = 0.0;
      }
    }
    // partials: wave w's tile t entry (row lk + 4q, col li) at V[0..1] as scratch
    cplx* part = &sm.G[0][0][0];  // 4 waves x 3 tiles x 256 over G[0..1] and V[0..1]
    static_assert(4 * 3 * 256 <= 4 * kPairCols * (kPairCols + 1), "partial scratch");
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) part[(w * 3 + t) * 256 + (lk + 4 * q) * 16 + li] = cmk(gr[t][q], gi[t][q]);
    __syncthreads();
    cplx gsum[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int e = tid + 256 * m, i = e >> 5, k = e & 31;
      int t, a, b;
      bool cj = false;
      if (i < kB && k < kB) t = 0, a = i, b = k;
      else if (i >= kB && k >= kB) t = 2, a = i - kB, b = k - kB;
      else if (i < kB) t = 1, a = i, b = k - kB;
      else t = 1, a = k, b = i - kB, cj = true;  // G[i][k] = conj(G[k][i])
      cplx v = cmk(0, 0);
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        const cplx x = part[(ww * 3 + t) * 256 + a * 16 + b];
        v.x += x.x, v.y += x.y;
      }
      if (cj) v.y = -v.y;
      if (i == k) v.y = 0.0;
      gsum[m] = v;
    }
    __syncthreads();  // partials read
#pragma unroll
    for (int m = 0; m < 4; ++m) sm.G[0][(tid >> 5) + 8 * m][tid & 31] = gsum[m];
    for (int e = tid; e < kPairCols * kPairCols; e += 256) {
      const int i = e >> 5, k = e & 31;
      sm.V[0][i][k] = cmk(i == k ? 1.0 : 0.0, 0.0);
    }
  }
  if (tid == 0) t1 = __builtin_amdgcn_s_memtime();
  // ---- 2: one cyclic Jacobi sweep on G ----
  // Thread (P, Q) = (tid / 16, tid % 16) owns the 2 x 2 blocks of G and V at the rows of pair P and
  // the columns of pair Q, and computes both pairs' rotations itself (redundantly across the 16
  // threads sharing a pair): one barrier per round.  J[p][p] = J[q][q] = c, J[p][q] = us,
  // J[q][p] = -conj(us); G' = J^H G J and V' = V J on the block; the diagonal blocks exact.
  const double tol2 = tol_sq(j, L), floor2 = s.fro * 1e-24, nfl2 = jacobi_noise2(j, s.fro),
               tiny2 = j.jtiny * j.jtiny;
  const int P = tid >> 4, Q = tid & 15;
  int rot = 0, big = 0, any = 0;
  int cur = 0;
  auto rrf = [](int pos, int r) {  // rr(pos, r, 32) without the division
    if (pos == 0) return 0;
    int v = pos - 1 + r;
    if (v >= kPairCols - 1) v -= kPairCols - 1;
    return v + 1;
  };
  (void)rrf;
  constexpr int kRounds = kPairFullGram ? kPairCols - 1 : kB;
  for (int r = 0; r < kRounds; ++r) {
    __syncthreads();  // G[cur] / V[cur] complete
    // FULL: every pair of the 32 columns, 31 round-robin rounds of 16 disjoint pairs; otherwise
    // cross pairs only (block I column k with block J column (k + r) mod 16): 16 rounds of 16
    // disjoint pairs; the blocks' own pairs are the intra launch's
    int pP, qP, pQ, qQ;
    if constexpr (kPairFullGram) {
      pP = rrf(P, r), qP = rrf(kPairCols - 1 - P, r), pQ = rrf(Q, r), qQ = rrf(kPairCols - 1 - Q, r);
    } else {
      pP = P, qP = kB + ((P + r) & (kB - 1)), pQ = Q, qQ = kB + ((Q + r) & (kB - 1));
    }
    auto rotation = [&](int p, int q, double& c, cplx& us, double& tg, int& flag_rot, int& flag_big) {
      const double a = sm.G[cur][p][p].x, b = sm.G[cur][q][q].x;
      const cplx g = sm.G[cur][p][q];
      const double g2 = g.x * g.x + g.y * g.y;
      const double thr = fmax(tol2 * a * b, nfl2 * (a + b));
      c = 1.0, tg = 0.0, us = cmk(0, 0), flag_rot = 0, flag_big = 0;
      if (g2 > thr && a > floor2 && b > floor2) {
        double te, pp;
        jacobi_te(a, b, g2, te, c, pp);
        us = cmk(c * te * g.x, c * te * g.y);  // u s = c t g / |g|
        tg = te * g2;                           // t |g|
        if (g2 > 16.0 * thr) {
          flag_rot = 1;
          if (fabs(te) * g2 > tiny2 * (a + b)) flag_big = 1;
        }
        return true;
      }
      return false;
    };
    // each lane computes pair Q's rotation (Q = lane % 16); pair P's comes from the lane of its
    // own row that holds Q = P (same wave: lane 16 (lane / 16) + P)
    double cQ, tgQ;
    cplx usQ;
    int frQ, fbQ;
    const bool didQ = rotation(pQ, qQ, cQ, usQ, tgQ, frQ, fbQ);
    const int src = 16 * (lane >> 4) + P;
    const double cP = __shfl(cQ, src), tgP = __shfl(tgQ, src);
    const cplx usP = cmk(__shfl(usQ.x, src), __shfl(usQ.y, src));
    const bool didP = __shfl((int)didQ, src) != 0;
    const int frP = frQ, fbP = fbQ;  // used only where P == Q (src == lane)
    const int nxt = cur ^ 1;
    const cplx m_pp = sm.G[cur][pP][pQ], m_pq = sm.G[cur][pP][qQ], m_qp = sm.G[cur][qP][pQ], m_qq = sm.G[cur][qP][qQ];
    cplx n_pp, n_pq, n_qp, n_qq;
    if (P == Q) {
      if (didP) {
        n_pp = cmk(m_pp.x - tgP, 0.0), n_qq = cmk(m_qq.x + tgP, 0.0), n_pq = n_qp = cmk(0, 0);
        any = 1, rot |= frP, big |= fbP;
      } else {
        n_pp = m_pp, n_pq = m_pq, n_qp = m_qp, n_qq = m_qq;
      }
    } else {
      // T = M JQ (columns), then JP^H T (rows)
      const cplx mus = cmk(-usQ.x, usQ.y);  // -conj(usQ) = J[q][p]
      const cplx t_pp = cfma(m_pq, mus, cscale(m_pp, cQ)), t_pq = cfma(m_pp, usQ, cscale(m_pq, cQ));
      const cplx t_qp = cfma(m_qq, mus, cscale(m_qp, cQ)), t_qq = cfma(m_qp, usQ, cscale(m_qq, cQ));
      // conj(J[x][i]): i = p: conj(J[p][p]) = cP, conj(J[q][p]) = -usP; i = q: conj(J[p][q]) = conj(usP), cP
      const cplx nus = cmk(-usP.x, -usP.y);
      n_pp = cfma(nus, t_qp, cscale(t_pp, cP));
      n_pq = cfma(nus, t_qq, cscale(t_pq, cP));
      n_qp = cfmac(usP, t_pp, cscale(t_qp, cP));
      n_qq = cfmac(usP, t_pq, cscale(t_qq, cP));
    }
    sm.G[nxt][pP][pQ] = n_pp, sm.G[nxt][pP][qQ] = n_pq, sm.G[nxt][qP][pQ] = n_qp, sm.G[nxt][qP][qQ] = n_qq;
    {
      const cplx mus = cmk(-usQ.x, usQ.y);
      const cplx v_pp = sm.V[cur][pP][pQ], v_pq = sm.V[cur][pP][qQ], v_qp = sm.V[cur][qP][pQ], v_qq = sm.V[cur][qP][qQ];
      sm.V[nxt][pP][pQ] = cfma(v_pq, mus, cscale(v_pp, cQ));
      sm.V[nxt][pP][qQ] = cfma(v_pp, usQ, cscale(v_pq, cQ));
      sm.V[nxt][qP][pQ] = cfma(v_qq, mus, cscale(v_qp, cQ));
      sm.V[nxt][qP][qQ] = cfma(v_qp, usQ, cscale(v_qq, cQ));
    }
    (void)didQ;
    cur = nxt;
  }
  if (tid == 0) t2 = __builtin_amdgcn_s_memtime();
  // ---- 3: A <- A V (skipped when nothing rotated: uniform via the LDS flag) ----
  __shared__ int s_any;
  if (tid == 0) s_any = 0;
  __syncthreads();
  if (any) s_any = 1;
  __syncthreads();
  if (s_any) {
    // V^T operands (A_op[i][k] = V[k][i]): jt output tile, ks k step; lane holds i = li, k = lk
    cplx vt[2][8];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) vt[jt][ks] = sm.V[cur][4 * ks + lk][16 * jt + li];
    int colk[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) colk[ks] = wcol(4 * ks + lk);
    cplx* Wm = j.work;
    // row tile rt + 1's loads in flight while rt's MFMAs run
    cplx bn[8];
    auto ldt = [&](int rt, cplx (&b)[8]) {
      const int row = r0 + 16 * rt + li;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) b[ks] = (colk[ks] >= 0 && row < L) ? ldg(Wm + (size_t)colk[ks] * L + row) : cmk(0, 0);
    };
    ldt(0, bn);
#pragma unroll 2
    for (int rt = 0; rt < MAXR; ++rt) {
      const int row = r0 + 16 * rt + li;
      cplx b[8];
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) b[ks] = bn[ks];
      if (rt + 1 < MAXR) ldt(rt + 1, bn);
      d4_t orr[2], oi[2];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        orr[jt] = d4_t{0, 0, 0, 0}, oi[jt] = d4_t{0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const cplx x = vt[jt][ks], y = b[ks];
          orr[jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.x, orr[jt], 0, 0, 0);
          orr[jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(-x.y, y.y, orr[jt], 0, 0, 0);
          oi[jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(x.x, y.y, oi[jt], 0, 0, 0);
          oi[jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(x.y, y.x, oi[jt], 0, 0, 0);
        }
      }
      // every wave has read its rows' 32 columns before any lane writes them (the MFMA results
      // depend on all the loads)
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cc = wcol(16 * jt + lk + 4 * q);
          if (cc >= 0 && row < L) Wm[(size_t)cc * L + row] = cmk(orr[jt][q], oi[jt][q]);
        }
    }
  }
  if (rot) atomicOr(&s.rot, 1);
  if (big) atomicOr(&s.big, 1);
  if (tid == 0) {
    const unsigned long long t3 = __builtin_amdgcn_s_memtime();
    atomicAdd(&g_bj_ticks[0], t1 - t0);
    atomicAdd(&g_bj_ticks[1], t2 - t1);
    atomicAdd(&g_bj_ticks[2], t3 - t2);
    atomicAdd(&g_bj_ticks[3], 1ull);
  }
}

// End of sweep: decide convergence, reset the sweep flags, count converged jobs.  grid (nj).
__global__ void k_bj_sweep_end(BJState* __restrict__ st, int* __restrict__ ndone) {
  if (threadIdx.x != 0) return;
  BJState& s = st[blockIdx.x];
  if (s.done) return;
  s.sweeps += 1;
  if (s.rot == 0 || s.big == 0 || s.sweeps >= kMaxSweepsBJ) {
    s.done = 1;
    atomicAdd(ndone, 1);
  }
  s.rot = 0;
  s.big = 0;
}

// sig = column norms (one wave per column), flags.  grid (ceil(C / 16), nj), 16 waves.
template <int MAXR>
__global__ __launch_bounds__(1024) void k_bj_final(const TwoSiteJob* __restrict__ jobs, const BJState* __restrict__ st) {
  const TwoSiteJob& j = jobs[blockIdx.y];
  const BJState& s = st[blockIdx.y];
  int L, C;
  bool tr;
  job_shape(j, L, C, tr);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = blockIdx.x * kB + w;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (s.sweeps >= kMaxSweepsBJ) atomicOr(&j.flags[1], 1);
    atomicMax(&j.flags[2], s.sweeps);
  }
  if (col >= C) return;
  double n2 = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + 64 * i;
    if (row < L) {
      const double2 v = j.work[(size_t)col * L + row];
      n2 = fma(v.x, v.x, fma(v.y, v.y, n2));
    }
  }
  n2 = wave_sum(n2);
  if (lane == 0) j.sig[col] = sqrt(n2);
}

struct BJBuffers {
  BJState* st = nullptr;
  int* ndone = nullptr;  // device counter
  int* host = nullptr;   // pinned read-back
  int cap = 0;
};

BJBuffers g_bj_buffers;
void release_bj_buffers() {
  BJBuffers& b = g_bj_buffers;
  if (b.st) (void)hipFree(b.st);
  if (b.ndone) (void)hipFree(b.ndone);
  if (b.host) (void)hipHostFree(b.host);
  b = BJBuffers();
}
BJBuffers& bj_buffers() {
  aqc::on_finalize(release_bj_buffers);
  return g_bj_buffers;
}

template <int MAXR>
int run_block_jacobi(const TwoSiteJob* jobs, int nj, int cap_max, hipStream_t stream) {
  BJBuffers& b = bj_buffers();
  if (b.cap < nj) {
    AQC_HIP_CHECK(hipStreamSynchronize(stream));
    if (b.st) hipFree(b.st);
    if (b.ndone) hipFree(b.ndone);
    if (b.host) hipHostFree(b.host);
    b.st = nullptr, b.ndone = nullptr, b.host = nullptr, b.cap = 0;
    AQC_HIP_CHECK(hipMalloc(&b.st, sizeof(BJState) * nj));
    AQC_HIP_CHECK(hipMalloc(&b.ndone, sizeof(int)));
    AQC_HIP_CHECK(hipHostMalloc(&b.host, sizeof(int)));
    b.cap = nj;
  }
  AQC_HIP_CHECK(hipMemsetAsync(b.st, 0, sizeof(BJState) * nj, stream));
  AQC_HIP_CHECK(hipMemsetAsync(b.ndone, 0, sizeof(int), stream));
  const int L = 2 * cap_max;
  int nb = (L + kB - 1) / kB;
  nb += nb & 1;
  const size_t lds = MAXR > 8 ? 0 : (size_t)kB * 64 * MAXR * sizeof(double2);
  hipLaunchKernelGGL(k_bj_init, dim3(nj), dim3(1024), 0, stream, jobs, b.st);
  AQC_CHECK_LAUNCH();
  for (int sweep = 0; sweep < kMaxSweepsBJ; ++sweep) {
    constexpr bool kFull = MAXR > 8;  // 2 chi > 512: the intra block would not fit the LDS
    if constexpr (!kFull) {
      hipLaunchKernelGGL((k_bj_intra<MAXR>), dim3(nb, nj), dim3(512), lds, stream, jobs, b.st);
      AQC_CHECK_LAUNCH();
    }
    for (int r = 0; r < nb - 1; ++r) {
      hipLaunchKernelGGL((k_bj_pair<MAXR, kFull>), dim3(nb / 2, nj), dim3(256), kPairLdsBytes, stream, jobs, b.st, r,
                         nb);
      AQC_CHECK_LAUNCH();
    }
    hipLaunchKernelGGL(k_bj_sweep_end, dim3(nj), dim3(64), 0, stream, b.st, b.ndone);
    AQC_CHECK_LAUNCH();
    if (sweep >= 2) {
      AQC_HIP_CHECK(hipMemcpyAsync(b.host, b.ndone, sizeof(int), hipMemcpyDeviceToHost, stream));
      AQC_HIP_CHECK(hipStreamSynchronize(stream));
      if (*b.host >= nj) break;
    }
  }
  hipLaunchKernelGGL((k_bj_final<MAXR>), dim3(nb, nj), dim3(1024), 0, stream, jobs, b.st);
  AQC_CHECK_LAUNCH();
  return AQC_OK;
}

}  // namespace

int block_jacobi(const TwoSiteJob* jobs, int nj, int cap_max, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    // 128 KB of dynamic LDS (block J's 16 columns of 512 rows)
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_bj_intra<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_bj_intra<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_bj_pair<8, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kPairLdsBytes));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_bj_pair<4, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kPairLdsBytes));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_bj_pair<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kPairLdsBytes));
    AQC_HIP_CHECK(hipFuncSetAttribute((const void*)k_bj_pair<32, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)kPairLdsBytes));
    attr = true;
  }
  AQC_REQUIRE(2 * cap_max <= 2048, "block Jacobi supports 2 * chi_cap <= 2048");
  if (2 * cap_max <= 256) return run_block_jacobi<4>(jobs, nj, cap_max, st);
  if (2 * cap_max <= 512) return run_block_jacobi<8>(jobs, nj, cap_max, st);
  if (2 * cap_max <= 1024) return run_block_jacobi<16>(jobs, nj, cap_max, st);
  return run_block_jacobi<32>(jobs, nj, cap_max, st);
}

}  // namespace aqc

extern "C" int aqc_bj_ticks(double* out) {
  AQC_REQUIRE(out, "aqc_bj_ticks: null argument");
  unsigned long long t[4];
  AQC_HIP_CHECK(hipMemcpyFromSymbol(t, HIP_SYMBOL(aqc::g_bj_ticks), sizeof(t)));
  for (int i = 0; i < 4; ++i) out[i] = (double)t[i];
  unsigned long long z[4] = {0, 0, 0, 0};
  AQC_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(aqc::g_bj_ticks), z, sizeof(z)));
  return AQC_OK;
}
