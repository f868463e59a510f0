// Candidate sweep: replaces adaptaqc/utils/gradients.py:23-124 (general_grad_of_pairs).
//
// The reference builds, for every coupling-map pair (c, t) and every generator G_k, the MPS of
// G_k^dag|s> through Aer and takes a whole-psi dot.  With a product starting state |s> every
// such overlap factorises through a 4-vector per pair:
//   T_ab[sa, sb] = <s_{not a,b}, sa sb | psi>,   <s|O|psi> = sum (s_c (x) s_t)^dag O T_ct,
// so one sweep over psi yields every pair's overlaps:
//   M_i = sum_s conj(s_i[s]) A_i[s]            (k_sweep_M)
//   l_b = M_0 .. M_{b-1},  r_b = M_b .. M_{n-1}  (k_sweep_lr)
//   w_b[s] = A_b[s] r_{b+1},  v_a[s] = l_a A_a[s] (k_sweep_w)
//   for each a: T_ab = v . w_b, v <- v M_b      (k_sweep_chain, one workgroup per a)
//   g_p = sqrt(sum_k deg_k (-Im(<s|G_k|psi> <psi|U0^dag|s>))^2)  (k_sweep_grad)
// Work per state: sum_a (n-a) vector-matrix products, O(n^2 chi^2), instead of the reference's
// O(n^2 * n_gen) MPS builds and O(n^3 chi^2 n_gen) dot work.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "aqc_gemm.h"
#include "mps_internal.h"

using aqc::cplx;

namespace {

constexpr int kT = 256;
// k_sweep_w splits each contraction over two halves of kT / 2 = 128 threads (part[2])
static_assert(kT == 256, "k_sweep_w assumes 4 waves of 64 lanes per workgroup");

struct SweepJob {
  const cplx* gam;
  const double* lam;
  const int* dims;
  int n;
  int cap;
  cplx* M;      // n * cap * cap
  cplx* lv;     // (n+1) * cap
  cplx* rv;     // (n+1) * cap
  cplx* w;      // n * 2 * cap
  cplx* v0;     // n * 2 * cap
  cplx* T;      // n * n * 4
  double* out;  // npairs
};

struct SweepConst {
  int npairs;
  int ngen;
  const int* pairs;      // 2 * npairs
  const cplx* svec;      // n * 2
  const cplx* u0;        // 16
  const cplx* gens;      // ngen * 16
  const double* degs;    // ngen
};

__device__ __forceinline__ cplx site_a(const SweepJob& j, int i, int s, int l, int r) {
  const size_t ss = (size_t)2 * j.cap * j.cap;
  return aqc::cscale(j.gam[(size_t)i * ss + (size_t)s * j.cap * j.cap + (size_t)l * j.cap + r],
                     j.lam[(size_t)(i + 1) * j.cap + r]);
}

// blockIdx.x: site, blockIdx.y: job
__global__ __launch_bounds__(kT) void k_sweep_M(const SweepJob* __restrict__ jobs, const cplx* __restrict__ svec) {
  const SweepJob& j = jobs[blockIdx.y];
  const int i = blockIdx.x;
  const int cl = j.dims[i], cr = j.dims[i + 1];
  const cplx s0 = aqc::cconj(svec[2 * i]), s1 = aqc::cconj(svec[2 * i + 1]);
  cplx* Mi = j.M + (size_t)i * j.cap * j.cap;
  // the whole cap x cap block, zeros outside chi_l x chi_r: the chains read it without masks
  // (blockIdx.z splits a site over several workgroups when few states are swept)
  for (int e = blockIdx.z * kT + threadIdx.x; e < j.cap * j.cap; e += kT * gridDim.z) {
    const int l = e / j.cap, r = e % j.cap;
    Mi[e] = (l < cl && r < cr) ? aqc::cfma(s1, site_a(j, i, 1, l, r), aqc::cmul(s0, site_a(j, i, 0, l, r)))
                               : aqc::cmk(0, 0);
  }
}

// blockIdx.x: job, blockIdx.y: 0 left / 1 right.  A chain of n dependent vector-matrix products
// (l_{i+1} = l_i M_i, r_i = M_i r_{i+1}) in one 1024-thread workgroup: thread t owns output
// o = t >> 3 (+ 128 per pass) and the contraction indices k = (t & 7) + 8 kk, so each group of 8
// lanes reads 8 consecutive complex of one matrix row (128-byte segments for both orientations)
// and sums through DPP (row_sum8); the running vector sits in LDS, double-buffered, one barrier
// per step.  The matrices do not depend on the vector: with cap <= 128 the next step's 16 values
// per thread are loaded while the current step computes, so the chain runs at the matrices'
// streaming rate instead of one memory latency per step.
__device__ __forceinline__ void lds_barrier() {
  // LDS-only barrier: the workgroup fence of __syncthreads would also drain the prefetch loads
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// CAP: 64, 128 or 256 >= the bond capacity; EXACT: the capacity equals CAP (mask-free loads,
// compile-time strides), otherwise out-of-block elements are clamped and zeroed.
template <int CAP, bool EXACT>
__global__ __launch_bounds__(1024) void k_sweep_lr(const SweepJob* __restrict__ jobs) {
  static_assert(CAP == 64 || CAP == 128 || CAP == 256, "k_sweep_lr: capacity 64, 128 or 256");
  constexpr int NP = CAP > 128 ? 2 : 1;   // output passes of 128
  constexpr int NC = CAP > 128 ? 2 : 1;   // k chunks of 128 (8 lanes x NK)
  constexpr int NK = CAP < 128 ? 8 : 16;  // elements per thread per chunk
  constexpr bool PF = CAP <= 128;         // register prefetch of the next step
  const SweepJob& j = jobs[blockIdx.x];
  const int n = j.n;
  const int cap = EXACT ? CAP : j.cap;
  const int t = threadIdx.x, o0 = t >> 3, ks = t & 7;
  __shared__ cplx vec[2][CAP];
  const bool left = blockIdx.y == 0;
  cplx* out = left ? j.lv : j.rv;
  if (t < CAP) vec[0][t] = aqc::cmk(t == 0 ? 1.0 : 0.0, 0.0);
  if (t == 0) out[(size_t)(left ? 0 : n) * cap] = aqc::cmk(1, 0);
  // NK elements (k, o) of step `step`'s matrix (zero-padded to CAP x CAP by k_sweep_M, so no
  // masks) for output pass `pass`, k chunk `kc`: left out[o] = sum_k vec[k] M[k][o], right
  // out[o] = sum_k M[o][k] vec[k]
  auto load = [&](int step, int pass, int kc, cplx (&m)[NK]) {
    const int i = left ? step : n - 1 - step;
    const cplx* Mi = j.M + (size_t)i * cap * cap;
    // the lane's offset laundered per call: hoisted out of the step loop, the per-element
    // addresses would stay live across it (and spill)
    int o = o0 + 128 * pass, kq = ks + 128 * kc;
    asm volatile("" : "+v"(o), "+v"(kq));
    if constexpr (EXACT) {
      // one lane offset, the element stride as the uniform offset
      const auto rs = aqc::make_rsrc(Mi, CAP * CAP * 16);
      const unsigned voff = 16u * (left ? (unsigned)(kq * CAP + o) : (unsigned)(o * CAP + kq));
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) m[kk] = aqc::buf_ld(rs, voff, 16u * kk * (left ? 8 * CAP : 8));
    } else {
      const bool ov = o < cap;
      const int oc = ov ? o : 0;
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const int k = kq + 8 * kk;
        const bool ok = ov && k < cap;
        const int kc2 = ok ? k : 0;
        const cplx v = aqc::ldg(Mi + (left ? kc2 * cap + oc : oc * cap + kc2));
        m[kk] = aqc::cmk(ok ? v.x : 0.0, ok ? v.y : 0.0);
      }
    }
  };
  const bool oact = o0 < CAP;  // CAP 64: waves 8..15 only join the barriers (uniform per wave)
  cplx mc[NK];
  if constexpr (PF) {
    if (oact) load(0, 0, 0, mc);
  }
  __syncthreads();
  int cur = 0;
  for (int step = 0; step < n; ++step) {
    const int i = left ? step : n - 1 - step;
    const int nout = left ? j.dims[i + 1] : j.dims[i];
    if (oact) {
#pragma unroll
      for (int pass = 0; pass < NP; ++pass) {
        cplx acc = aqc::cmk(0, 0);
#pragma unroll
        for (int kc = 0; kc < NC; ++kc) {
          cplx m[NK];
          if constexpr (PF) {
#pragma unroll
            for (int kk = 0; kk < NK; ++kk) m[kk] = mc[kk];
            if (step + 1 < n) load(step + 1, 0, 0, mc);
          } else {
            load(step, pass, kc, m);
          }
#pragma unroll
          for (int kk = 0; kk < NK; ++kk) {
            acc = aqc::cfma(vec[cur][128 * kc + ks + 8 * kk], m[kk], acc);
            if ((kk & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // LDS reads in groups of 4
          }
        }
        acc.x = aqc::row_sum8(acc.x);
        acc.y = aqc::row_sum8(acc.y);
        const int o = o0 + 128 * pass;
        if (ks == 0) {
          // M's zero padding makes acc = 0 beyond nout: the next step's vector stays clean
          vec[cur ^ 1][o] = acc;
          if (o < nout) out[(size_t)(left ? i + 1 : i) * cap + o] = acc;
        }
      }
    }
    lds_barrier();
    cur ^= 1;
  }
}

// The same chain for the exact capacities 64 and 128 with the whole next step's matrix share in
// flight while the current one computes: 8 CAP threads, thread t owns output o = t / 8 and
// k = (t % 8) + 8 kk (CAP / 8 elements), two register sets with the step loop unrolled by two
// (a register copy of an in-flight load would wait for it; a spill reload would wait for every
// older load, the prefetch included).
template <int CAP>
__global__ __launch_bounds__(CAP * 8) void k_sweep_lr_pf(const SweepJob* __restrict__ jobs) {
  static_assert(CAP == 64 || CAP == 128, "k_sweep_lr_pf: capacity 64 or 128");
  constexpr int LPO = 8, NK = CAP / LPO;
  const SweepJob& j = jobs[blockIdx.x];
  const int n = j.n;
  const int t = threadIdx.x, o = t / LPO, ks = t % LPO;
  __shared__ cplx vec[2][CAP];
  const bool left = blockIdx.y == 0;
  cplx* out = left ? j.lv : j.rv;
  if (t < CAP) vec[0][t] = aqc::cmk(t == 0 ? 1.0 : 0.0, 0.0);
  if (t == 0) out[(size_t)(left ? 0 : n) * CAP] = aqc::cmk(1, 0);
  // left out[o] = sum_k vec[k] M[k][o], right out[o] = sum_k M[o][k] vec[k] (zero-padded M)
  const unsigned voff = 16u * (left ? (unsigned)(ks * CAP + o) : (unsigned)(o * CAP + ks));
  constexpr unsigned kstep_l = 16u * LPO * CAP, kstep_r = 16u * LPO;
  auto load = [&](int step, cplx (&m)[NK]) {
    const int i = left ? step : n - 1 - step;
    const auto rs = aqc::make_rsrc(j.M + (size_t)i * CAP * CAP, CAP * CAP * 16);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) m[kk] = aqc::buf_ld(rs, voff, kk * (left ? kstep_l : kstep_r));
  };
  // rolling pipeline: element kk of step s + 1 is requested right after element kk of step s has
  // been consumed, so NK loads are always in flight and each has a whole step to land
  cplx m[NK];
  load(0, m);
  __syncthreads();
  int cur = 0;
  for (int step = 0; step < n; ++step) {
    const int i = left ? step : n - 1 - step;
    const int nout = left ? j.dims[i + 1] : j.dims[i];
    const int inext = left ? min(step + 1, n - 1) : max(n - 2 - step, 0);
    const auto rs = aqc::make_rsrc(j.M + (size_t)inext * CAP * CAP, CAP * CAP * 16);
    cplx acc = aqc::cmk(0, 0);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      acc = aqc::cfma(vec[cur][ks + LPO * kk], m[kk], acc);
      m[kk] = aqc::buf_ld(rs, voff, kk * (left ? kstep_l : kstep_r));
    }
    acc.x = aqc::group_sum<LPO>(acc.x);
    acc.y = aqc::group_sum<LPO>(acc.y);
    if (ks == 0) {
      vec[cur ^ 1][o] = acc;  // zero beyond nout (M's padding)
      if (o < nout) out[(size_t)(left ? i + 1 : i) * CAP + o] = acc;
    }
    lds_barrier();
    cur ^= 1;
  }
}

// One chain per workgroup (the latency form, for a single state) at the exact capacities 64 and
// 128: 8 CAP threads in the k_sweep_lr_pf layout propagate both row vectors v[sa] through M_b
// (one load of each M element for the two rows), with M_{b+1} in flight during step b.
template <int CAP>
__global__ __launch_bounds__(CAP * 8) void k_sweep_chain_pf(const SweepJob* __restrict__ jobs,
                                                            const int* __restrict__ alist) {
  static_assert(CAP == 64 || CAP == 128, "k_sweep_chain_pf: capacity 64 or 128");
  constexpr int LPO = 8, NK = CAP / LPO, NT = CAP * 8;
  const SweepJob& j = jobs[blockIdx.y];
  const int a = alist[blockIdx.x];
  const int n = j.n;
  if (a >= n - 1) return;
  const int t = threadIdx.x, o = t / LPO, ks = t % LPO, wave = t >> 6, lane = t & 63;
  __shared__ cplx v[2][2][CAP];
  {
    const int d0 = j.dims[a + 1];
    for (int e = t; e < 2 * CAP; e += NT) {
      const int sa = e / CAP, k = e % CAP;
      v[0][sa][k] = k < d0 ? j.v0[((size_t)a * 2 + sa) * CAP + k] : aqc::cmk(0, 0);
    }
  }
  const unsigned voff = 16u * (unsigned)(ks * CAP + o);
  constexpr unsigned kstep = 16u * LPO * CAP;
  auto load = [&](int b, cplx (&m)[NK]) {
    const auto rs = aqc::make_rsrc(j.M + (size_t)b * CAP * CAP, CAP * CAP * 16);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) m[kk] = aqc::buf_ld(rs, voff, kk * kstep);
  };
  // rolling pipeline (k_sweep_lr_pf)
  cplx m[NK];
  load(a + 1, m);
  __syncthreads();
  int cur = 0;
  for (int b = a + 1; b < n; ++b) {
    const int db = j.dims[b];
    // T_ab[sa][sb] = sum_k v[sa][k] w_b[sb][k]: wave w < 4 -> (sa, sb) = (w >> 1, w & 1)
    if (wave < 4) {
      const int sa = wave >> 1, sb = wave & 1;
      const cplx* wb = j.w + ((size_t)b * 2 + sb) * CAP;
      cplx acc = aqc::cmk(0, 0);
      for (int k = lane; k < db; k += 64) acc = aqc::cfma(v[cur][sa][k], wb[k], acc);
      acc.x = aqc::row_sum16(acc.x);
      acc.y = aqc::row_sum16(acc.y);
      acc.x += __shfl_xor(acc.x, 16);
      acc.y += __shfl_xor(acc.y, 16);
      acc.x += __shfl_xor(acc.x, 32);
      acc.y += __shfl_xor(acc.y, 32);
      if (lane == 0) j.T[((size_t)a * n + b) * 4 + wave] = acc;
    }
    if (b == n - 1) break;
    const auto rs = aqc::make_rsrc(j.M + (size_t)min(b + 1, n - 1) * CAP * CAP, CAP * CAP * 16);
    cplx a0 = aqc::cmk(0, 0), a1 = aqc::cmk(0, 0);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const int k = ks + LPO * kk;
      a0 = aqc::cfma(v[cur][0][k], m[kk], a0);
      a1 = aqc::cfma(v[cur][1][k], m[kk], a1);
      m[kk] = aqc::buf_ld(rs, voff, kk * kstep);
    }
    a0.x = aqc::group_sum<LPO>(a0.x);
    a0.y = aqc::group_sum<LPO>(a0.y);
    a1.x = aqc::group_sum<LPO>(a1.x);
    a1.y = aqc::group_sum<LPO>(a1.y);
    if (ks == 0) {
      v[cur ^ 1][0][o] = a0;
      v[cur ^ 1][1][o] = a1;
    }
    lds_barrier();
    cur ^= 1;
  }
}

// blockIdx.x: site, blockIdx.y: job.  w_b[s][l] = sum_r Gamma_b[s][l][r] x[r] with
// x[r] = lambda_{b+1}[r] rv[b+1][r] (in LDS): rows (s, l) 8 lanes each, the lanes along r (one
// 128-byte segment per row and instruction), summed through DPP; v0_a[s][r] = lambda_{a+1}[r]
// sum_l lv[a][l] Gamma_a[s][l][r], only at chain starts (start[a]: the first qubits of this rank's
// pair shard): a thread per (s, r), the lanes along r.
__global__ __launch_bounds__(kT) void k_sweep_w(const SweepJob* __restrict__ jobs, const int* __restrict__ start) {
  const SweepJob& j = jobs[blockIdx.y];
  const int i = blockIdx.x, cap = j.cap;
  const int cl = j.dims[i], cr = j.dims[i + 1];
  const int tid = threadIdx.x;
  __shared__ cplx x[256];
  const cplx* G = j.gam + (size_t)i * 2 * cap * cap;
  const double* lamr = j.lam + (size_t)(i + 1) * cap;
  for (int r = tid; r < cr; r += kT) x[r] = aqc::cscale(j.rv[(size_t)(i + 1) * cap + r], lamr[r]);
  __syncthreads();
  {
    const int ks = tid & 7;
    for (int row0 = blockIdx.z * (kT / 8); row0 < 2 * cl; row0 += (kT / 8) * gridDim.z) {
      const int row = row0 + (tid >> 3);  // (s, l) = (row / cl, row % cl)
      const bool ok = row < 2 * cl;
      const int sr = ok ? row / cl : 0, lr = ok ? row % cl : 0;
      const cplx* g = G + ((size_t)sr * cap + lr) * cap;
      cplx acc = aqc::cmk(0, 0);
      if (ok)
        for (int r = ks; r < cr; r += 8) acc = aqc::cfma(aqc::ldg(g + r), x[r], acc);
      acc.x = aqc::row_sum8(acc.x);
      acc.y = aqc::row_sum8(acc.y);
      if (ok && ks == 0) j.w[((size_t)i * 2 + sr) * cap + lr] = acc;
    }
  }
  if (!start[i]) return;  // uniform in the workgroup
  __syncthreads();
  for (int l = tid; l < cl; l += kT) x[l] = j.lv[(size_t)i * cap + l];
  __syncthreads();
  for (int e = blockIdx.z * kT + tid; e < 2 * cap; e += kT * gridDim.z) {
    const int sr = e / cap, r = e % cap;
    if (r >= cr) continue;
    const cplx* g = G + (size_t)sr * cap * cap + r;
    cplx acc = aqc::cmk(0, 0);
    for (int l = 0; l < cl; ++l) acc = aqc::cfma(x[l], aqc::ldg(g + (size_t)l * cap), acc);
    j.v0[((size_t)i * 2 + sr) * cap + r] = aqc::cscale(acc, lamr[r]);
  }
}

// One workgroup per (a, job): propagate the two row vectors v[sa] through M_b, emitting T_ab.
__global__ __launch_bounds__(kT) void k_sweep_chain(const SweepJob* __restrict__ jobs, const int* __restrict__ alist) {
  const SweepJob& j = jobs[blockIdx.y];
  const int a = alist[blockIdx.x];
  const int n = j.n, cap = j.cap;
  if (a >= n - 1) return;
  __shared__ cplx v[2][2][256];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int d0 = j.dims[a + 1];
  for (int e = tid; e < 2 * d0; e += kT) v[0][e / d0][e % d0] = j.v0[((size_t)a * 2 + e / d0) * cap + e % d0];
  __syncthreads();
  int cur = 0;
  for (int b = a + 1; b < n; ++b) {
    const int db = j.dims[b], dn = j.dims[b + 1];
    // T_ab[sa][sb] = sum_k v[sa][k] w_b[sb][k] : wave w -> (sa, sb) = (w >> 1, w & 1)
    {
      const int sa = wave >> 1, sb = wave & 1;
      const cplx* wb = j.w + ((size_t)b * 2 + sb) * cap;
      cplx acc = aqc::cmk(0, 0);
      for (int k = lane; k < db; k += 64) acc = aqc::cfma(v[cur][sa][k], wb[k], acc);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        acc.x += __shfl_xor(acc.x, off);
        acc.y += __shfl_xor(acc.y, off);
      }
      if (lane == 0) j.T[((size_t)a * n + b) * 4 + wave] = acc;
    }
    if (b == n - 1) break;
    // v[s] <- v[s] M_b
    const cplx* Mb = j.M + (size_t)b * cap * cap;
    for (int e = tid; e < 2 * dn; e += kT) {
      const int s = e / dn, r = e % dn;
      cplx acc = aqc::cmk(0, 0);
      for (int k = 0; k < db; ++k) acc = aqc::cfma(v[cur][s][k], Mb[(size_t)k * cap + r], acc);
      v[cur ^ 1][s][r] = acc;
    }
    __syncthreads();
    cur ^= 1;
  }
}

// Grouped chains (the sweep batched over first qubits, one GEMM per site): one
// 512-thread workgroup per (group of up to 8 consecutive first qubits of alist, job), capacity
// 128.  The group's 16 row vectors (row 2c + sa: chain c, first-qubit value sa) advance through
// M_b together as a 16 x 128 by 128 x 128 complex product on the FP64 matrix cores, so M_b is read
// once per group instead of once per chain.  Wave w owns output columns 16w .. 16w + 15 (one
// 16 x 16 tile of v_mfma_f64_16x16x4f64, four real products per complex one, split over two
// accumulator pairs so that consecutive MFMAs are independent; A operand: lane l holds
// A[l & 15][k = l >> 4], B: B[k = l >> 4][l & 15], D: row (l >> 4) + 4 q, column l & 15).  The
// lane's 32 B elements of M_{b+1} are requested one by one as those of M_b are consumed (a
// rolling pipeline: a whole step to land), under LDS-only barriers.  Rows of chains not yet
// started (a >= b) keep v0_a.  M is zero-padded, so no masks.
template <int CAP>
constexpr int kChain8Ld = CAP + 4;  // V row stride (complex)

// G first qubits per workgroup: 8 (default), or 16 (round-4 experiment: M_b read once per 16
// chains, each MFMA step's B operands serving two row tiles -- measured slower, sweep_group())
template <int CAP, int G>
__global__ __launch_bounds__(4 * CAP) void k_sweep_chain8(const SweepJob* __restrict__ jobs, const int* __restrict__ alist,
                                                          int nal, int ns) {
  constexpr int NQ = CAP / 4, NT = 4 * CAP;  // CAP / 16 waves, one 16-column tile each
  constexpr int R = 2 * G, RT = R / 16;      // rows (chain c, first-qubit value sa: 2c + sa), row tiles
  static_assert(G == 8 || G == 16, "8 or 16 chains per workgroup");
  // 1-D grid over (state slot, group): linear id = state + nsp group with nsp = ns rounded up to 8,
  // so a state's groups -- which read the same M_b matrices at about the same time -- share one XCD
  // (and its L2) under the dispatcher's round-robin placement (a speed matter only)
  const int nsp = (ns + 7) & ~7, sj = (int)blockIdx.x % nsp;
  if (sj >= ns) return;  // (padding: whole workgroups)
  const SweepJob& j = jobs[sj];
  const int g0 = ((int)blockIdx.x / nsp) * G;
  const int n = j.n;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  __shared__ cplx V[2][R][kChain8Ld<CAP>];
  __shared__ int s_a[G];
  if (tid < G) s_a[tid] = g0 + tid < nal ? alist[g0 + tid] : n;  // n: never active
  __syncthreads();
  const int amin = s_a[0];  // alist is ascending
  if (amin >= n - 1) return;  // uniform
  for (int e = tid; e < R * CAP; e += NT) {
    const int row = e / CAP, k = e % CAP, a = s_a[row >> 1];
    cplx v = aqc::cmk(0, 0);
    if (a < n - 1 && k < j.dims[a + 1]) v = j.v0[((size_t)a * 2 + (row & 1)) * CAP + k];
    V[0][row][k] = v;
  }
  const int li = lane & 15, lk = lane >> 4, col = 16 * wave + li;
  const unsigned voff = 16u * (unsigned)(lk * CAP + col);
  constexpr unsigned qstep = 16u * 4 * CAP;
  cplx bq[NQ];
  {
    const auto rs = aqc::make_rsrc(j.M + (size_t)(amin + 1) * CAP * CAP, CAP * CAP * 16);
#pragma unroll
    for (int q = 0; q < NQ; ++q) bq[q] = aqc::buf_ld(rs, voff, q * qstep);
  }
  __syncthreads();
  int cur = 0;
  for (int b = amin + 1; b < n; ++b) {
    const int db = j.dims[b];
    // T_ab[sa][sb] = sum_k v[sa][k] w_b[sb][k]: 16 lanes per row
    for (int base = 0; base < 16 * R; base += NT) {
      const int t = base + tid;
      if (t < 16 * R) {
        const int row = t >> 4, sub = t & 15, a = s_a[row >> 1];
        const cplx* w0 = j.w + ((size_t)b * 2) * CAP;
        cplx t0 = aqc::cmk(0, 0), t1 = aqc::cmk(0, 0);
        for (int k = sub; k < db; k += 16) {
          const cplx v = V[cur][row][k];
          t0 = aqc::cfma(v, w0[k], t0);
          t1 = aqc::cfma(v, w0[CAP + k], t1);
        }
        t0.x = aqc::row_sum16(t0.x);
        t0.y = aqc::row_sum16(t0.y);
        t1.x = aqc::row_sum16(t1.x);
        t1.y = aqc::row_sum16(t1.y);
        if (sub == 0 && a < b) {
          cplx* T = j.T + ((size_t)a * n + b) * 4 + 2 * (row & 1);
          T[0] = t0;
          T[1] = t1;
        }
      }
    }
    if (b == n - 1) break;
    const auto rs = aqc::make_rsrc(j.M + (size_t)min(b + 1, n - 1) * CAP * CAP, CAP * CAP * 16);
    aqc::d4_t cr0[RT], ci0[RT], cr1[RT], ci1[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) cr0[rt] = ci0[rt] = cr1[rt] = ci1[rt] = aqc::d4_t{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const cplx bv = bq[q];
      cplx av[RT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) av[rt] = V[cur][16 * rt + li][4 * q + lk];
      bq[q] = aqc::buf_ld(rs, voff, q * qstep);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        cr0[rt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[rt].x, bv.x, cr0[rt], 0, 0, 0);
        ci0[rt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[rt].x, bv.y, ci0[rt], 0, 0, 0);
        cr1[rt] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av[rt].y, bv.y, cr1[rt], 0, 0, 0);
        ci1[rt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[rt].y, bv.x, ci1[rt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * rt + lk + 4 * q;
        const bool act = s_a[row >> 1] < b;
        V[cur ^ 1][row][col] = act ? aqc::cmk(cr0[rt][q] + cr1[rt][q], ci0[rt][q] + ci1[rt][q]) : V[cur][row][col];
      }
    }
    lds_barrier();
    cur ^= 1;
  }
}

// One thread per pair.
__global__ void k_sweep_grad(const SweepJob* __restrict__ jobs, SweepConst c) {
  const SweepJob& j = jobs[blockIdx.y];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= c.npairs) return;
  const int qc = c.pairs[2 * p], qt = c.pairs[2 * p + 1];
  const int a = qc < qt ? qc : qt, b = qc < qt ? qt : qc;
  const cplx* tab = j.T + ((size_t)a * j.n + b) * 4;  // [sa][sb]
  cplx vec[4];  // little-endian over (c, t): index 2*st + sc
#pragma unroll
  for (int sa = 0; sa < 2; ++sa)
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const int sc = qc == a ? sa : sb, st = qc == a ? sb : sa;
      vec[2 * st + sc] = tab[2 * sa + sb];
    }
  cplx s4[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) s4[x] = aqc::cconj(aqc::cmul(c.svec[2 * qt + (x >> 1)], c.svec[2 * qc + (x & 1)]));
  auto bra_op_ket = [&](const cplx* O) {
    cplx acc = aqc::cmk(0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cplx ov = aqc::cmk(0, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) ov = aqc::cfma(O[4 * r + k], vec[k], ov);
      acc = aqc::cfma(s4[r], ov, acc);
    }
    return acc;
  };
  const cplx z = aqc::cconj(bra_op_ket(c.u0));  // <psi|U0^dag|s>
  double g = 0.0;
  for (int k = 0; k < c.ngen; ++k) {
    const cplx ov = bra_op_ket(c.gens + 16 * k);  // <s|G_k|psi>
    const double gg = -aqc::cmul(ov, z).y;
    g += gg * gg * c.degs[k];
  }
  j.out[p] = sqrt(g);  // out is per job (make_job)
}

// np.argmax(s * prio) over one row in one 256-thread workgroup: the first maximum (lowest index on
// ties), NaN winning as in numpy.  Thread 0 gets (index, value).
__device__ void argmax_row(const double* s, const double* prio, int count, int& best, double& val) {
  __shared__ double bv[256];
  __shared__ int bi[256];
  double v = -1.0 / 0.0;
  int idx = 0x7fffffff;
  for (int i = threadIdx.x; i < count; i += blockDim.x) {
    const double x = s[i] * prio[i];
    if (x > v || (x == v && i < idx) || (x != x && v == v)) {  // NaN wins like np.argmax
      v = x;
      idx = i;
    }
  }
  bv[threadIdx.x] = v;
  bi[threadIdx.x] = idx;
  __syncthreads();
  for (int st = blockDim.x / 2; st > 0; st >>= 1) {
    if (threadIdx.x < st) {
      const double o = bv[threadIdx.x + st];
      const int oi = bi[threadIdx.x + st];
      const double m = bv[threadIdx.x];
      const int mi = bi[threadIdx.x];
      const bool on = o != o, mn = m != m;
      bool take;
      if (on || mn) take = on && (!mn || oi < mi);
      else take = (o > m) || (o == m && oi < mi);
      if (take) {
        bv[threadIdx.x] = o;
        bi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  best = bi[0];
  val = bv[0];
}

__global__ __launch_bounds__(256) void k_argmax(const double* s, const double* prio, int count, int* best) {
  int b;
  double v;
  argmax_row(s, prio, count, b, v);
  if (threadIdx.x == 0) *best = b;
}

// one row (state) per workgroup: out[r] = its arg-max index (as a double), out[nrows + r] = the
// scaled score there -- the [2][nrows] block the state-sharded sweep all-gathers (sharding.gather_best)
__global__ __launch_bounds__(256) void k_argmax_rows(const double* __restrict__ s, int ld, const double* __restrict__ prio,
                                                     int count, int nrows, double* __restrict__ out) {
  int b;
  double v;
  argmax_row(s + (size_t)blockIdx.x * ld, prio, count, b, v);
  if (threadIdx.x == 0) {
    out[blockIdx.x] = (double)b;
    out[nrows + blockIdx.x] = v;
  }
}

// ---- chi = 1 variational compression (tenpy_product_state, approximate_compiler.py:222-242) ----
// The best product-state approximation |s> = (x) s_i of psi by alternating two-site updates: with
// every other site fixed, <s|psi> = sum_ab conj(s_i[a]) conj(s_{i+1}[b]) F[a][b], F[a][b] =
// l_i A_i[a] A_{i+1}[b] r_{i+2}, is maximised by the top singular pair of the 2 x 2 F (s_i = u_1,
// s_{i+1} = conj(v_1), |<s|psi>| = sigma_1).  One sweep = a left-to-right pass (right
// environments r from the current s, left ones carried along) and a right-to-left pass.  One
// workgroup per state; the chains are O(n chi^2) and sequential.
struct FitJob {
  const cplx* gam;
  const double* lam;
  const int* dims;
  int n;
  int cap;
  cplx* svec;   // n x 2 (in: initial guess unless guess_from_gamma, out: result)
  cplx* Lv;     // (n + 1) x cap left environments
  cplx* Rv;     // (n + 1) x cap right environments
  double* out;  // [0] fidelity |<s|psi>|^2, [1] sweeps, [2] fidelity after each sweep (max_sweeps)
  int guess_from_gamma;
  int min_sweeps;
  int max_sweeps;
  double tol;
};

__device__ __forceinline__ cplx fit_a(const FitJob& j, int i, int s, int l, int r) {
  const size_t ss = (size_t)2 * j.cap * j.cap;
  return aqc::cscale(j.gam[(size_t)i * ss + (size_t)s * j.cap * j.cap + (size_t)l * j.cap + r],
                     j.lam[(size_t)(i + 1) * j.cap + r]);
}

// top singular pair of the 2 x 2 complex F (row a, column b): F v = sigma u
__device__ void top_pair_2x2(const cplx F[4], cplx u[2], cplx v[2], double& sigma) {
  const double h00 = F[0].x * F[0].x + F[0].y * F[0].y + F[2].x * F[2].x + F[2].y * F[2].y;
  const double h11 = F[1].x * F[1].x + F[1].y * F[1].y + F[3].x * F[3].x + F[3].y * F[3].y;
  const cplx h01 = aqc::cadd(aqc::cmul(aqc::cconj(F[0]), F[1]), aqc::cmul(aqc::cconj(F[2]), F[3]));
  const double hm = 0.5 * (h00 + h11), hd = 0.5 * (h00 - h11);
  const double lam = hm + sqrt(hd * hd + h01.x * h01.x + h01.y * h01.y);
  cplx v0, v1;
  if (h00 >= h11) {
    v0 = aqc::cmk(lam - h11, 0.0);
    v1 = aqc::cconj(h01);
  } else {
    v0 = h01;
    v1 = aqc::cmk(lam - h00, 0.0);
  }
  double nv = sqrt(v0.x * v0.x + v0.y * v0.y + v1.x * v1.x + v1.y * v1.y);
  if (!(nv > 0.0)) {
    v0 = aqc::cmk(1, 0);
    v1 = aqc::cmk(0, 0);
    nv = 1.0;
  }
  v[0] = aqc::cscale(v0, 1.0 / nv);
  v[1] = aqc::cscale(v1, 1.0 / nv);
  const cplx a0 = aqc::cfma(F[1], v[1], aqc::cmul(F[0], v[0]));
  const cplx a1 = aqc::cfma(F[3], v[1], aqc::cmul(F[2], v[0]));
  sigma = sqrt(a0.x * a0.x + a0.y * a0.y + a1.x * a1.x + a1.y * a1.y);
  if (sigma > 0.0) {
    u[0] = aqc::cscale(a0, 1.0 / sigma);
    u[1] = aqc::cscale(a1, 1.0 / sigma);
  } else {
    u[0] = aqc::cmk(1, 0);
    u[1] = aqc::cmk(0, 0);
  }
}

// largest bond capacity of the chi = 1 fit (its running vectors sit in the dynamic LDS: 5 cap complex)
constexpr int kFitMaxCap = 1024;

__global__ __launch_bounds__(kT) void k_product_fit(const FitJob* __restrict__ jobs) {
  const FitJob& j = jobs[blockIdx.x];
  const int n = j.n, cap = j.cap, tid = threadIdx.x;
  // dynamic LDS (5 cap complex): the running l (left-to-right) or r (right-to-left), then u[s][m],
  // w[s][m]
  extern __shared__ cplx fit_lds[];
  cplx* vec = fit_lds;
  cplx* fit_uw = fit_lds + cap;
  __shared__ cplx part[4][kT / 64];
  __shared__ cplx sv[2][2];       // the updated pair
  __shared__ double fid_s;
  if (j.guess_from_gamma && tid == 0) {
    // chi = 1 truncation of the canonical form: keep the largest Schmidt value on every bond
    for (int i = 0; i < n; ++i) {
      const size_t ss = (size_t)2 * cap * cap;
      cplx a = j.gam[(size_t)i * ss], b = j.gam[(size_t)i * ss + (size_t)cap * cap];
      const double nn = sqrt(a.x * a.x + a.y * a.y + b.x * b.x + b.y * b.y);
      if (nn > 0.0) {
        a = aqc::cscale(a, 1.0 / nn);
        b = aqc::cscale(b, 1.0 / nn);
      } else {
        a = aqc::cmk(1, 0);
        b = aqc::cmk(0, 0);
      }
      j.svec[2 * i] = a;
      j.svec[2 * i + 1] = b;
    }
  }
  __syncthreads();
  // r_k = M_k r_{k+1} for k = n-1 .. lo (M_k = sum_s conj(s_k[s]) A_k[s]); l_{k+1} = l_k M_k for k < hi
  auto right_envs = [&]() {
    if (tid == 0) j.Rv[(size_t)n * cap] = aqc::cmk(1, 0);
    __syncthreads();
    for (int k = n - 1; k >= 0; --k) {
      const int cl = j.dims[k], cr = j.dims[k + 1];
      const cplx c0 = aqc::cconj(j.svec[2 * k]), c1 = aqc::cconj(j.svec[2 * k + 1]);
      const cplx* rn = j.Rv + (size_t)(k + 1) * cap;
      for (int l = tid; l < cl; l += kT) {
        cplx a0 = aqc::cmk(0, 0), a1 = aqc::cmk(0, 0);
        for (int r = 0; r < cr; ++r) {
          a0 = aqc::cfma(fit_a(j, k, 0, l, r), rn[r], a0);
          a1 = aqc::cfma(fit_a(j, k, 1, l, r), rn[r], a1);
        }
        j.Rv[(size_t)k * cap + l] = aqc::cfma(c1, a1, aqc::cmul(c0, a0));
      }
      __syncthreads();
    }
  };
  auto left_envs = [&]() {
    if (tid == 0) j.Lv[0] = aqc::cmk(1, 0);
    __syncthreads();
    for (int k = 0; k < n; ++k) {
      const int cl = j.dims[k], cr = j.dims[k + 1];
      const cplx c0 = aqc::cconj(j.svec[2 * k]), c1 = aqc::cconj(j.svec[2 * k + 1]);
      const cplx* lp = j.Lv + (size_t)k * cap;
      for (int r = tid; r < cr; r += kT) {
        cplx a0 = aqc::cmk(0, 0), a1 = aqc::cmk(0, 0);
        for (int l = 0; l < cl; ++l) {
          a0 = aqc::cfma(lp[l], fit_a(j, k, 0, l, r), a0);
          a1 = aqc::cfma(lp[l], fit_a(j, k, 1, l, r), a1);
        }
        j.Lv[(size_t)(k + 1) * cap + r] = aqc::cfma(c1, a1, aqc::cmul(c0, a0));
      }
      __syncthreads();
    }
  };
  // u[s][m] = sum_l lv[l] A_i[s][l][m], w[s][m] = sum_r A_{i+1}[s][m][r] rv[r]; F; update of (i, i+1)
  auto update = [&](int i, const cplx* lv, const cplx* rv) {
    const int cl = j.dims[i], cm = j.dims[i + 1], cr = j.dims[i + 2];
    for (int e = tid; e < 2 * cm; e += kT) {
      const int s = e / cm, m = e % cm;
      cplx a = aqc::cmk(0, 0), b = aqc::cmk(0, 0);
      for (int l = 0; l < cl; ++l) a = aqc::cfma(lv[l], fit_a(j, i, s, l, m), a);
      for (int r = 0; r < cr; ++r) b = aqc::cfma(fit_a(j, i + 1, s, m, r), rv[r], b);
      fit_uw[((0) * 2 + (s)) * cap + (m)] = a;
      fit_uw[((1) * 2 + (s)) * cap + (m)] = b;
    }
    __syncthreads();
    // F[a][b] = sum_m u[a][m] w[b][m]: wave q -> entry q
    {
      const int q = tid >> 6, lane = tid & 63;
      const int a = q >> 1, b = q & 1;
      cplx acc = aqc::cmk(0, 0);
      for (int m = lane; m < cm; m += 64) acc = aqc::cfma(fit_uw[((0) * 2 + (a)) * cap + (m)], fit_uw[((1) * 2 + (b)) * cap + (m)], acc);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        acc.x += __shfl_xor(acc.x, off);
        acc.y += __shfl_xor(acc.y, off);
      }
      if (lane == 0) part[q][0] = acc;
    }
    __syncthreads();
    if (tid == 0) {
      const cplx F[4] = {part[0][0], part[1][0], part[2][0], part[3][0]};
      cplx u[2], v[2];
      double sg;
      top_pair_2x2(F, u, v, sg);
      sv[0][0] = u[0];
      sv[0][1] = u[1];
      sv[1][0] = aqc::cconj(v[0]);
      sv[1][1] = aqc::cconj(v[1]);
      j.svec[2 * i] = sv[0][0];
      j.svec[2 * i + 1] = sv[0][1];
      j.svec[2 * (i + 1)] = sv[1][0];
      j.svec[2 * (i + 1) + 1] = sv[1][1];
      fid_s = sg * sg;
    }
    __syncthreads();
  };
  double prev = -1.0;
  int sweep = 0;
  if (n == 1) {  // a single site: s = psi itself
    if (tid == 0) {
      cplx a = fit_a(j, 0, 0, 0, 0), b = fit_a(j, 0, 1, 0, 0);
      const double nn = sqrt(a.x * a.x + a.y * a.y + b.x * b.x + b.y * b.y);
      j.svec[0] = aqc::cscale(a, 1.0 / nn);
      j.svec[1] = aqc::cscale(b, 1.0 / nn);
      j.out[0] = nn * nn;
      j.out[1] = 0;
    }
    return;
  }
  for (sweep = 0; sweep < j.max_sweeps; ++sweep) {
    // left to right
    right_envs();
    if (tid == 0) vec[0] = aqc::cmk(1, 0);
    __syncthreads();
    for (int i = 0; i < n - 1; ++i) {
      update(i, vec, j.Rv + (size_t)(i + 2) * cap);
      const int cm = j.dims[i + 1];
      for (int m = tid; m < cm; m += kT)
        vec[m] = aqc::cfma(aqc::cconj(sv[0][1]), fit_uw[((0) * 2 + (1)) * cap + (m)], aqc::cmul(aqc::cconj(sv[0][0]), fit_uw[((0) * 2 + (0)) * cap + (m)]));
      __syncthreads();
    }
    // right to left
    left_envs();
    if (tid == 0) vec[0] = aqc::cmk(1, 0);
    __syncthreads();
    for (int i = n - 2; i >= 0; --i) {
      update(i, j.Lv + (size_t)i * cap, vec);
      const int cm = j.dims[i + 1];
      for (int m = tid; m < cm; m += kT)
        vec[m] = aqc::cfma(aqc::cconj(sv[1][1]), fit_uw[((1) * 2 + (1)) * cap + (m)], aqc::cmul(aqc::cconj(sv[1][0]), fit_uw[((1) * 2 + (0)) * cap + (m)]));
      __syncthreads();
    }
    const double f = fid_s;
    if (tid == 0) j.out[2 + sweep] = f;
    if (sweep + 1 >= j.min_sweeps && prev >= 0.0 && fabs(f - prev) <= j.tol * f) {
      ++sweep;
      break;
    }
    prev = f;
  }
  if (tid == 0) {
    j.out[0] = fid_s;
    j.out[1] = (double)sweep;
  }
}

// Per-device staging for the sweep's jobs and constants: a ring of two (pinned host, device)
// buffer pairs, each guarded by an event recorded after the launches that read it, so a call
// packs its constants into one pinned buffer and issues ONE asynchronous copy instead of draining
// the stream and issuing blocking hipMemcpys.
struct GradBuffers {
  void* dev = nullptr;
  size_t cap = 0;
  char* host = nullptr;
  size_t hcap = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
};

struct GradRing {
  std::mutex mu;
  GradBuffers b[2];
  int next = 0;
};

GradRing g_gring[64];
void release_gring() {
  for (auto& r : g_gring)
    for (auto& b : r.b) {
      if (b.done) (void)hipEventDestroy(b.done);
      if (b.dev) (void)hipFree(b.dev);
      if (b.host) (void)hipHostFree(b.host);
      b.done = nullptr, b.dev = nullptr, b.host = nullptr;
      b.cap = b.hcap = 0;
      b.pending = false;
    }
}
GradRing& gring() {
  int dev = 0;
  hipGetDevice(&dev);
  aqc::on_finalize(release_gring);
  return g_gring[dev];
}

int grad_buffers(GradBuffers& gb, size_t need) {
  if (gb.pending) {
    AQC_HIP_CHECK(hipEventSynchronize(gb.done));
    gb.pending = false;
  }
  if (need > gb.cap) {
    if (gb.dev) hipFree(gb.dev);
    gb.dev = nullptr;
    gb.cap = std::max(need, 2 * gb.cap);
    AQC_HIP_CHECK(hipMalloc(&gb.dev, gb.cap));
  }
  if (need > gb.hcap) {
    if (gb.host) hipHostFree(gb.host);
    gb.host = nullptr;
    gb.hcap = std::max(need, 2 * gb.hcap);
    AQC_HIP_CHECK(hipHostMalloc((void**)&gb.host, gb.hcap, hipHostMallocDefault));
  }
  if (!gb.done) AQC_HIP_CHECK(hipEventCreateWithFlags(&gb.done, hipEventDisableTiming));
  return AQC_OK;
}

int ensure_gw(aqc_mps_t h) {
  const size_t cap = h->d.cap, n = h->d.n;
  const size_t need = (n * cap * cap + 2 * (n + 1) * cap + 4 * n * cap + n * n * 4) * sizeof(cplx);
  if (h->gw_bytes >= need) return AQC_OK;
  if (h->gw) {  // (queued sweeps may still read the old block: the pool reuses it at once)
    AQC_HIP_CHECK(hipStreamSynchronize(aqc::mps_stream()));
    aqc::dev_free(h->gw);
  }
  h->gw = (cplx*)aqc::dev_alloc(need);
  if (!h->gw) {
    h->gw_bytes = 0;
    aqc::set_error("ensure_gw: out of device memory");
    return AQC_ERR_NOMEM;
  }
  h->gw_bytes = need;
  return AQC_OK;
}

#include "sweep_seg.h"

// 0: automatic (grouped chains for batches of states at cap 128, one chain per workgroup for a
// single state, where the per-step latency of 2 rows beats the 16-row group's), 1: one chain per
// workgroup, 2: grouped, 3: the segmented single-state sweep (sweep_seg.h) whenever one state is
// swept (aqc_sweep_set_chain_mode).  Auto picks the segmented form for one state above cap 64:
// 0.41 vs 0.92 ms at chi = 128 (50 qubits, 1225 pairs), 0.43 vs 0.41 ms at chi = 64
// (tools/single_sweep_timing.py).
int g_chain_mode = 0;
bool use_segments(int cap, int ns) {
  if (cap > 256) return true;  // (one state: aqc_pair_grads_batch splits larger batches)
  return ns == 1 && cap >= 16 && (g_chain_mode == 3 || (g_chain_mode == 0 && cap > 64));
}
bool use_chain8(int cap, int ns) {
  if ((cap != 128 && cap != 64) || g_chain_mode == 1) return false;
  return g_chain_mode == 2 || ns >= 2;
}
// first qubits per grouped-chain workgroup: 8 (16 measured slower: config 4 34.3-34.8 M against
// 35.9-36.8 M evals/s, profiles/r4_sweep_group16_ab.json; 16 chains hold 135 KB of LDS at CAP = 128,
// one workgroup per CU, and a group's later chains idle through more of its sites)
constexpr int kSweepGroup = 8;

SweepJob make_job(aqc_mps_t h, double* out) {
  SweepJob j;
  const size_t cap = h->d.cap, n = h->d.n;
  j.gam = h->d.gam;
  j.lam = h->d.lam;
  j.dims = h->d.dims;
  j.n = (int)n;
  j.cap = (int)cap;
  cplx* p = h->gw;
  j.M = p;
  p += n * cap * cap;
  j.lv = p;
  p += (n + 1) * cap;
  j.rv = p;
  p += (n + 1) * cap;
  j.w = p;
  p += 2 * n * cap;
  j.v0 = p;
  p += 2 * n * cap;
  j.T = p;
  j.out = out;
  return j;
}

}  // namespace

extern "C" {

int aqc_pair_grads_batch(aqc_mps_t* psis, int ns, const double* svec, const int* pairs, int npairs,
                         const double* u0, const double* gens, const double* degs, int ngen, double* out,
                         int out_is_device) {
  AQC_REQUIRE(psis && ns > 0 && svec && pairs && u0 && out && npairs >= 0 && ngen >= 0,
              "aqc_pair_grads_batch: bad arguments");
  AQC_REQUIRE(ngen == 0 || (gens && degs), "aqc_pair_grads_batch: null generators");
  const int n = psis[0]->d.n;
  for (int s = 0; s < ns; ++s) AQC_REQUIRE(psis[s] && psis[s]->d.n == n, "aqc_pair_grads_batch: all states need n qubits");
  for (int s = 0; s < ns; ++s)
    AQC_REQUIRE(psis[s]->d.cap == psis[0]->d.cap, "aqc_pair_grads_batch: states need one bond capacity");
  if (psis[0]->d.cap > 256 && ns > 1) {
    // capacities above 256 (the unbounded MPS of aer_mps_backend.py:27-42 grows to 512): the chain
    // kernels hold a row vector per lane group up to 256 only, the segmented single-state sweep is
    // capacity-agnostic -- one state at a time through it
    for (int s = 0; s < ns; ++s) {
      const int rc = aqc_pair_grads_batch(psis + s, 1, svec, pairs, npairs, u0, gens, degs, ngen,
                                          out + (size_t)s * npairs, out_is_device);
      if (rc != AQC_OK) return rc;
    }
    return AQC_OK;
  }
  for (int p = 0; p < npairs; ++p) {
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    AQC_REQUIRE(a >= 0 && a < n && b >= 0 && b < n && a != b, "aqc_pair_grads_batch: bad pair");
  }
  int rc = aqc_mps_sort_batch(psis, ns);
  if (rc != AQC_OK) return rc;
  for (int s = 0; s < ns; ++s) {
    rc = ensure_gw(psis[s]);
    if (rc != AQC_OK) return rc;
  }
  hipStream_t st = aqc::mps_stream();
  // constants + jobs + (host-out) result buffer: one pinned image, one asynchronous copy
  const size_t jb = ns * sizeof(SweepJob);
  // chains are needed only for the first qubits present in `pairs` (pair sharding across ranks)
  std::vector<int> alist;
  {
    std::vector<char> need(n, 0);
    for (int p = 0; p < npairs; ++p) need[std::min(pairs[2 * p], pairs[2 * p + 1])] = 1;
    for (int a = 0; a < n - 1; ++a)
      if (need[a]) alist.push_back(a);
  }
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_jobs = 0;
  const size_t o_pairs = al(o_jobs + jb);
  const size_t o_svec = al(o_pairs + 2 * (size_t)npairs * sizeof(int));
  const size_t o_u0 = o_svec + 2 * (size_t)n * sizeof(cplx);
  const size_t o_gens = o_u0 + 16 * sizeof(cplx);
  const size_t o_degs = o_gens + 16 * (size_t)ngen * sizeof(cplx);
  const size_t o_alist = al(o_degs + (size_t)ngen * sizeof(double));
  const size_t o_start = al(o_alist + (alist.size() + 4) * sizeof(int));
  const size_t o_out = al(o_start + (size_t)n * sizeof(int));
  const size_t image = o_out;  // bytes copied host -> device
  const size_t need = o_out + (out_is_device ? 0 : (size_t)ns * npairs * sizeof(double)) + 256;
  GradRing& ring = gring();
  std::lock_guard<std::mutex> lk(ring.mu);
  GradBuffers& gb = ring.b[ring.next];
  ring.next ^= 1;
  rc = grad_buffers(gb, need);
  if (rc != AQC_OK) return rc;
  char* base = (char*)gb.dev;
  char* hbase = gb.host;
  SweepJob* djobs = (SweepJob*)(base + o_jobs);
  int* dpairs = (int*)(base + o_pairs);
  cplx* dsvec = (cplx*)(base + o_svec);
  cplx* du0 = (cplx*)(base + o_u0);
  cplx* dgens = (cplx*)(base + o_gens);
  double* ddegs = (double*)(base + o_degs);
  int* dalist = (int*)(base + o_alist);
  int* dstart = (int*)(base + o_start);  // n flags: chain start (v0 needed) at this qubit
  double* dout = out_is_device ? out : (double*)(base + o_out);
  {
    SweepJob* hj = (SweepJob*)(hbase + o_jobs);
    for (int s = 0; s < ns; ++s) hj[s] = make_job(psis[s], dout + (size_t)s * npairs);
    if (npairs) std::memcpy(hbase + o_pairs, pairs, 2 * (size_t)npairs * sizeof(int));
    std::memcpy(hbase + o_svec, svec, 2 * (size_t)n * sizeof(cplx));
    std::memcpy(hbase + o_u0, u0, 16 * sizeof(cplx));
    if (ngen) {
      std::memcpy(hbase + o_gens, gens, 16 * (size_t)ngen * sizeof(cplx));
      std::memcpy(hbase + o_degs, degs, (size_t)ngen * sizeof(double));
    }
    if (!alist.empty()) std::memcpy(hbase + o_alist, alist.data(), alist.size() * sizeof(int));
    int* hstart = (int*)(hbase + o_start);
    for (int a = 0; a < n; ++a) hstart[a] = 0;
    for (int a : alist) hstart[a] = 1;
  }
  if (int e = aqc::upload_async(base, hbase, image, st)) return e;
  const int cap = psis[0]->d.cap;
  // few states: each site's M over several workgroups (the chains / GEMMs that follow are the
  // single sweep's critical path)
  const unsigned zsplit = ns >= 8 ? 1u : 8u;
  hipLaunchKernelGGL(k_sweep_M, dim3(n, ns, zsplit), dim3(kT), 0, st, djobs, dsvec);
  AQC_CHECK_LAUNCH();
  if (use_segments(cap, ns)) {
    const SweepJob* hj0 = (const SweepJob*)(hbase + o_jobs);
    aqc::KernelTimer::begin(st, "grad_seg", 0.0, 2.0 * n * 8.0 * (double)cap * cap * cap);
    rc = run_segment_sweep(*hj0, djobs, pairs, dpairs, npairs, dstart, st);
    aqc::KernelTimer::end(st);
    if (rc != AQC_OK) return rc;
  } else {
  {
    const dim3 g(ns, 2), b(1024);
    if (cap == 64) hipLaunchKernelGGL((k_sweep_lr_pf<64>), g, dim3(512), 0, st, djobs);
    else if (cap == 128) hipLaunchKernelGGL((k_sweep_lr_pf<128>), g, dim3(1024), 0, st, djobs);
    else if (cap == 256) hipLaunchKernelGGL((k_sweep_lr<256, true>), g, b, 0, st, djobs);
    else if (cap < 64) hipLaunchKernelGGL((k_sweep_lr<64, false>), g, b, 0, st, djobs);
    else if (cap < 128) hipLaunchKernelGGL((k_sweep_lr<128, false>), g, b, 0, st, djobs);
    else hipLaunchKernelGGL((k_sweep_lr<256, false>), g, b, 0, st, djobs);
  }
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_sweep_w, dim3(n, ns, zsplit), dim3(kT), 0, st, djobs, (const int*)dstart);
  AQC_CHECK_LAUNCH();
  {
    // algorithmic work of the chain: sum_a (n-a-1) steps of a 2 x chi x chi complex vec-mat
    const double c = cap;
    double steps = 0.0;
    for (int a : alist) steps += (double)(n - 1 - a);
    if (!alist.empty()) {
      aqc::KernelTimer::begin(st, "grad_chain", ns * steps * c * c * 16.0, ns * steps * 2.0 * c * c * 8.0);
      const unsigned ng = (unsigned)(alist.size() + kSweepGroup - 1) / kSweepGroup;
      if (use_chain8(cap, ns) && cap == 128) {
        hipLaunchKernelGGL((k_sweep_chain8<128, kSweepGroup>), dim3(ng * ((ns + 7) & ~7)), dim3(512), 0, st, djobs,
                           (const int*)dalist, (int)alist.size(), ns);
      } else if (use_chain8(cap, ns)) {
        hipLaunchKernelGGL((k_sweep_chain8<64, kSweepGroup>), dim3(ng * ((ns + 7) & ~7)), dim3(256), 0, st, djobs,
                           (const int*)dalist, (int)alist.size(), ns);
      }
      else
        if (cap == 128)
          hipLaunchKernelGGL(k_sweep_chain_pf<128>, dim3((unsigned)alist.size(), ns), dim3(1024), 0, st, djobs,
                             (const int*)dalist);
        else if (cap == 64)
          hipLaunchKernelGGL(k_sweep_chain_pf<64>, dim3((unsigned)alist.size(), ns), dim3(512), 0, st, djobs,
                             (const int*)dalist);
        else
          hipLaunchKernelGGL(k_sweep_chain, dim3((unsigned)alist.size(), ns), dim3(kT), 0, st, djobs, dalist);
      aqc::KernelTimer::end(st);
      AQC_CHECK_LAUNCH();
    }
  }
  }  // chain form
  if (npairs) {
    SweepConst c;
    c.npairs = npairs;
    c.ngen = ngen;
    c.pairs = dpairs;
    c.svec = dsvec;
    c.u0 = du0;
    c.gens = dgens;
    c.degs = ddegs;
    hipLaunchKernelGGL(k_sweep_grad, dim3((npairs + 127) / 128, ns), dim3(128), 0, st, djobs, c);
    AQC_CHECK_LAUNCH();
  }
  AQC_HIP_CHECK(hipEventRecord(gb.done, st));
  gb.pending = true;
  // a host result is complete on return (one wait at the end, none before the launches); a
  // device result is complete on this stream -- the caller joins its own (aqc_stream_join)
  if (!out_is_device && npairs) {
    AQC_HIP_CHECK(hipMemcpyAsync(out, dout, (size_t)ns * npairs * sizeof(double), hipMemcpyDeviceToHost, st));
    AQC_HIP_CHECK(hipStreamSynchronize(st));
  }
  return AQC_OK;
}

int aqc_sweep_set_chain_mode(int mode) {
  AQC_REQUIRE(mode >= 0 && mode <= 3, "aqc_sweep_set_chain_mode: mode 0, 1, 2 or 3");
  g_chain_mode = mode;
  return AQC_OK;
}

int aqc_pair_grads(aqc_mps_t psi, const double* svec, const int* pairs, int npairs, const double* u0,
                   const double* gens, const double* degs, int ngen, double* out, int out_is_device) {
  return aqc_pair_grads_batch(&psi, 1, svec, pairs, npairs, u0, gens, degs, ngen, out, out_is_device);
}

int aqc_mps_product_fit(aqc_mps_t psi, double* svec, int guess_from_gamma, int min_sweeps, int max_sweeps,
                        double tol, double* fidelity, int* sweeps) {
  AQC_REQUIRE(psi && svec && max_sweeps >= 1 && min_sweeps >= 0 && tol >= 0.0, "aqc_mps_product_fit: bad arguments");
  AQC_REQUIRE(psi->d.cap <= kFitMaxCap, "aqc_mps_product_fit: bond capacity above 1024");
  int rc = aqc_mps_sort(psi);  // the fit runs in qubit order
  if (rc != AQC_OK) return rc;
  rc = ensure_gw(psi);
  if (rc != AQC_OK) return rc;
  const int n = psi->d.n, cap = psi->d.cap;
  hipStream_t st = aqc::mps_stream();
  // device scratch: the sweep workspace (gw) holds n cap^2 >= 2 (n + 1) cap complex for the
  // environments; svec, the job and the outputs in a small allocation of their own
  cplx* Lv = psi->gw;
  cplx* Rv = Lv + (size_t)(n + 1) * cap;
  const size_t ob = (2 + (size_t)max_sweeps) * sizeof(double);
  const size_t bytes = 2 * (size_t)n * sizeof(cplx) + sizeof(FitJob) + ob + 512;
  char* d = nullptr;
  AQC_HIP_CHECK(hipMalloc(&d, bytes));
  cplx* dsv = (cplx*)d;
  FitJob* dj = (FitJob*)(d + ((2 * (size_t)n * sizeof(cplx) + 255) & ~(size_t)255));
  double* dout = (double*)((char*)dj + ((sizeof(FitJob) + 255) & ~(size_t)255));
  FitJob j;
  j.gam = psi->d.gam;
  j.lam = psi->d.lam;
  j.dims = psi->d.dims;
  j.n = n;
  j.cap = cap;
  j.svec = dsv;
  j.Lv = Lv;
  j.Rv = Rv;
  j.out = dout;
  j.guess_from_gamma = guess_from_gamma ? 1 : 0;
  j.min_sweeps = min_sweeps;
  j.max_sweeps = max_sweeps;
  j.tol = tol;
  int err = AQC_OK;
  std::vector<double> hout(2 + max_sweeps, 0.0);
  do {
    if (hipMemcpyAsync(dsv, svec, 2 * (size_t)n * sizeof(cplx), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(dj, &j, sizeof(FitJob), hipMemcpyHostToDevice, st) != hipSuccess) {
      err = AQC_ERR_HIP;
      break;
    }
    const size_t lds = 5 * (size_t)psi->d.cap * sizeof(cplx);  // (80 KB at capacity 1024)
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)k_product_fit, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(5 * kFitMaxCap * sizeof(cplx)));
      attr = true;
    }
    hipLaunchKernelGGL(k_product_fit, dim3(1), dim3(kT), lds, st, (const FitJob*)dj);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(svec, dsv, 2 * (size_t)n * sizeof(cplx), hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(hout.data(), dout, ob, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      err = AQC_ERR_HIP;
      break;
    }
  } while (false);
  hipFree(d);
  if (err != AQC_OK) {
    aqc::set_error("aqc_mps_product_fit: HIP failure");
    return err;
  }
  if (fidelity) *fidelity = hout[0];
  if (sweeps) *sweeps = (int)hout[1];
  return AQC_OK;
}

int aqc_argmax_scaled(const double* scores, const double* prio, int count, int scores_is_device, int* best) {
  AQC_REQUIRE(scores && prio && best && count > 0, "aqc_argmax_scaled: bad arguments");
  hipStream_t st = aqc::mps_stream();
  // cached per-device (pinned host, device) pair: no allocation per call, one copy each way
  struct ArgmaxBuf {
    std::mutex mu;
    double* dev = nullptr;
    double* host = nullptr;
    size_t cap = 0;  // doubles
  };
  static ArgmaxBuf bufs[64];
  static void (*release)() = [] {
    for (auto& b : bufs) {
      if (b.dev) (void)hipFree(b.dev);
      if (b.host) (void)hipHostFree(b.host);
      b.dev = nullptr, b.host = nullptr, b.cap = 0;
    }
  };
  aqc::on_finalize(release);
  int devi = 0;
  hipGetDevice(&devi);
  ArgmaxBuf& ab = bufs[devi];
  std::lock_guard<std::mutex> lk(ab.mu);
  const size_t need = 2 * (size_t)count + 4;
  if (need > ab.cap) {
    if (ab.dev) hipFree(ab.dev);
    if (ab.host) hipHostFree(ab.host);
    ab.dev = nullptr;
    ab.host = nullptr;
    ab.cap = std::max(need, 2 * ab.cap);
    AQC_HIP_CHECK(hipMalloc(&ab.dev, ab.cap * sizeof(double)));
    AQC_HIP_CHECK(hipHostMalloc((void**)&ab.host, ab.cap * sizeof(double), hipHostMallocDefault));
  }
  double* dp = ab.dev;
  double* ds = ab.dev + count;
  int* db = (int*)(ab.dev + 2 * (size_t)count);
  std::memcpy(ab.host, prio, count * sizeof(double));
  if (!scores_is_device) std::memcpy(ab.host + count, scores, count * sizeof(double));
  if (int e = aqc::upload_async(dp, ab.host, (scores_is_device ? 1 : 2) * (size_t)count * sizeof(double), st))
    return e;
  hipLaunchKernelGGL(k_argmax, dim3(1), dim3(256), 0, st, scores_is_device ? scores : ds, dp, count, db);
  AQC_CHECK_LAUNCH();
  int* hb = (int*)(ab.host + 2 * (size_t)count);
  AQC_HIP_CHECK(hipMemcpyAsync(hb, db, sizeof(int), hipMemcpyDeviceToHost, st));
  AQC_HIP_CHECK(hipStreamSynchronize(st));
  *best = *hb;
  return AQC_OK;
}

int aqc_argmax_scaled_batch(const double* scores, int ld, const double* prio, int count, int nrows, double* out) {
  AQC_REQUIRE(scores && prio && out && count > 0 && nrows > 0 && ld >= count, "aqc_argmax_scaled_batch: bad arguments");
  hipLaunchKernelGGL(k_argmax_rows, dim3(nrows), dim3(256), 0, aqc::mps_stream(), scores, ld, prio, count, nrows, out);
  AQC_CHECK_LAUNCH();
  return AQC_OK;
}

}  // extern "C"
