// Microbenchmark lab for the register-resident one-sided Jacobi round (not part of the library).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/jacobi_lab tools/jacobi_lab.hip
// Run on an MI355X: ./tools/jacobi_lab [blocks] [sweeps]
// Variants are template switches so every phase can be timed in isolation:
//   RED 0 = __shfl_xor reductions (ds_bpermute), 1 = DPP row reductions
//   XCH 0 = ring shift through LDS, 1 = Gray-code pairing (xor 16/32 lanes in registers, LDS
//           only for xor >= 4 groups), 2 = no exchange (timing only, wrong result)
//   ROT false = skip the column update (timing only)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__constant__ double c_tolf = 1.0;
constexpr int MAXR = 8, CP = 128, kG = CP / 2, kThreads = kG * 16, ld = 16 * MAXR;

__device__ __forceinline__ double dpp_sum16(double v) {
  v += __builtin_amdgcn_update_dpp(0.0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0.0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0.0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v += __builtin_amdgcn_update_dpp(0.0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

// value held by lane ^ 16 (D = 16) or lane ^ 32 (D = 32) of this wave
template <int D>
__device__ __forceinline__ double xor_lanes(double v, bool upper) {
  const long long b = __double_as_longlong(v);
  int lo = (int)b, hi = (int)(b >> 32);
  if constexpr (D == 16) {
    auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    auto c = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    lo = upper ? a[0] : a[1];
    hi = upper ? c[0] : c[1];
  } else {
    auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    auto c = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    lo = upper ? a[0] : a[1];
    hi = upper ? c[0] : c[1];
  }
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int RED, int XCH, bool ROT>
__global__ __launch_bounds__(kThreads) void k_lab(const double2* __restrict__ A, double2* __restrict__ W,
                                                  double* __restrict__ sig, int* __restrict__ sweeps_out,
                                                  int fixed_sweeps) {
  extern __shared__ double2 xbuf[];
  __shared__ double fred[kThreads / 64];
  __shared__ int xid[kG];
  __shared__ int rot;
  const int L = CP, C = CP;
  const double2* a = A + (size_t)blockIdx.x * L * C;
  const int tid = threadIdx.x, g = tid >> 4, lane = tid & 15;
  double sr[MAXR], si[MAXR], mr[MAXR], mi[MAXR];
  int sid = g, mid = g + kG;
  double f = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = lane + 16 * i;
    const double2 x = a[(size_t)sid * L + r], y = a[(size_t)mid * L + r];
    sr[i] = x.x, si[i] = x.y, mr[i] = y.x, mi[i] = y.y;
    f += x.x * x.x + x.y * x.y + y.x * y.x + y.y * y.y;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) f += __shfl_xor(f, off);
  if ((tid & 63) == 0) fred[tid >> 6] = f;
  __syncthreads();
  double fro = 0;
  for (int w = 0; w < kThreads / 64; ++w) fro += fred[w];
  const double floor2 = fro * 1e-24, tol = c_tolf * L * 2.220446049250313e-16, tol2 = tol * tol;
  const bool up16 = (tid & 16) != 0, up32 = (tid & 32) != 0;
  int sweeps = 0;
  for (sweeps = 0; sweeps < 40; ++sweeps) {
    if (tid == 0) rot = 0;
    __syncthreads();
    int my_rot = 0;
    for (int m = kG; m >= 1; m >>= 1) {
      const int li = g & (m - 1), base = g - li;
      for (int r = 0; r < m; ++r) {
        double al = 0, be = 0, gx = 0, gy = 0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          al = fma(sr[i], sr[i], fma(si[i], si[i], al));
          be = fma(mr[i], mr[i], fma(mi[i], mi[i], be));
          gx = fma(sr[i], mr[i], fma(si[i], mi[i], gx));
          gy = fma(sr[i], mi[i], fma(-si[i], mr[i], gy));
        }
        if constexpr (RED == 0) {
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) {
            al += __shfl_xor(al, off, 16);
            be += __shfl_xor(be, off, 16);
            gx += __shfl_xor(gx, off, 16);
            gy += __shfl_xor(gy, off, 16);
          }
        } else {  // RED 1, 2
          al = dpp_sum16(al);
          be = dpp_sum16(be);
          gx = dpp_sum16(gx);
          gy = dpp_sum16(gy);
        }
        const double g2 = gx * gx + gy * gy;
        if (g2 > tol2 * al * be && al > floor2 && be > floor2) {
          double c, ex, ey;
          if constexpr (RED == 2) {
            // rsq + Newton steps instead of IEEE sqrt / div sequences
            double rg = __builtin_amdgcn_rsq(g2);            // ~1/|g|
            rg = rg * fma(-0.5 * g2 * rg, rg, 1.5);
            rg = rg * fma(-0.5 * g2 * rg, rg, 1.5);
            const double zeta = 0.5 * (be - al) * rg;
            const double q = fma(zeta, zeta, 1.0);
            double rq = __builtin_amdgcn_rsq(q);
            rq = rq * fma(-0.5 * q * rq, rq, 1.5);
            rq = rq * fma(-0.5 * q * rq, rq, 1.5);
            const double den = fabs(zeta) + q * rq;            // |zeta| + sqrt(1 + zeta^2)
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
            ex = gx * sc, ey = gy * sc;
          } else {
            const double gg = sqrt(g2);
            const double zeta = (be - al) / (2.0 * gg);
            const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
            c = 1.0 / sqrt(1.0 + t * t);
            const double sc = c * t / gg;
            ex = gx * sc, ey = gy * sc;
          }
          if constexpr (ROT) {
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {
              const double ar = sr[i], ai = si[i], br = mr[i], bi = mi[i];
              sr[i] = fma(c, ar, -fma(ex, br, ey * bi));
              si[i] = fma(c, ai, -fma(ex, bi, -ey * br));
              mr[i] = fma(c, br, fma(ex, ar, -ey * ai));
              mi[i] = fma(c, bi, fma(ex, ai, ey * ar));
            }
          } else {
            sr[0] += ex * 1e-300;
          }
          my_rot = 1;
        }
        if (r == m - 1) break;
        if constexpr (XCH == 3) {
#pragma unroll
          for (int i = 0; i < MAXR; ++i) xbuf[g * ld + lane + 16 * i] = make_double2(mr[i], mi[i]);
          const int src = base + ((li + 1) & (m - 1));
#pragma unroll
          for (int i = 0; i < MAXR; ++i) {
            const double2 v = xbuf[src * ld + lane + 16 * i];
            mr[i] = v.x, mi[i] = v.y;
          }
        }
        if constexpr (XCH == 0) {
#pragma unroll
          for (int i = 0; i < MAXR; ++i) xbuf[g * ld + lane + 16 * i] = make_double2(mr[i], mi[i]);
          if (lane == 0) xid[g] = mid;
          __syncthreads();
          const int src = base + ((li + 1) & (m - 1));
#pragma unroll
          for (int i = 0; i < MAXR; ++i) {
            const double2 v = xbuf[src * ld + lane + 16 * i];
            mr[i] = v.x, mi[i] = v.y;
          }
          mid = xid[src];
          __syncthreads();
        } else if constexpr (XCH == 1) {
          const int d = 1 << __builtin_ctz(r + 1);  // Gray code: partner = g ^ d
          if (d == 1) {
#pragma unroll
            for (int i = 0; i < MAXR; ++i) mr[i] = xor_lanes<16>(mr[i], up16), mi[i] = xor_lanes<16>(mi[i], up16);
            mid = __shfl_xor(mid, 16);
          } else if (d == 2) {
#pragma unroll
            for (int i = 0; i < MAXR; ++i) mr[i] = xor_lanes<32>(mr[i], up32), mi[i] = xor_lanes<32>(mi[i], up32);
            mid = __shfl_xor(mid, 32);
          } else {
#pragma unroll
            for (int i = 0; i < MAXR; ++i) xbuf[g * ld + lane + 16 * i] = make_double2(mr[i], mi[i]);
            if (lane == 0) xid[g] = mid;
            __syncthreads();
            const int src = g ^ d;
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {
              const double2 v = xbuf[src * ld + lane + 16 * i];
              mr[i] = v.x, mi[i] = v.y;
            }
            mid = xid[src];
            __syncthreads();
          }
        }
      }
      if (m == 1) break;
      const int h = m >> 1;
      const bool lowh = li < h;
      if constexpr (XCH == 2) continue;
      if (XCH == 1 && h <= 2) {
        double tr_[MAXR], ti_[MAXR];
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          tr_[i] = lowh ? mr[i] : sr[i];
          ti_[i] = lowh ? mi[i] : si[i];
          if (h == 1) tr_[i] = xor_lanes<16>(tr_[i], up16), ti_[i] = xor_lanes<16>(ti_[i], up16);
          else tr_[i] = xor_lanes<32>(tr_[i], up32), ti_[i] = xor_lanes<32>(ti_[i], up32);
          mr[i] = lowh ? tr_[i] : mr[i];
          mi[i] = lowh ? ti_[i] : mi[i];
          sr[i] = lowh ? sr[i] : tr_[i];
          si[i] = lowh ? si[i] : ti_[i];
        }
        const int send = lowh ? mid : sid;
        const int pid = h == 1 ? __shfl_xor(send, 16) : __shfl_xor(send, 32);
        mid = lowh ? pid : mid;
        sid = lowh ? sid : pid;
        continue;
      }
#pragma unroll
      for (int i = 0; i < MAXR; ++i)
        xbuf[g * ld + lane + 16 * i] = lowh ? make_double2(mr[i], mi[i]) : make_double2(sr[i], si[i]);
      if (lane == 0) xid[g] = lowh ? mid : sid;
      __syncthreads();
      const int partner = lowh ? g + h : g - h;
      const int pid = xid[partner];
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        const double2 v = xbuf[partner * ld + lane + 16 * i];
        mr[i] = lowh ? v.x : mr[i];
        mi[i] = lowh ? v.y : mi[i];
        sr[i] = lowh ? sr[i] : v.x;
        si[i] = lowh ? si[i] : v.y;
      }
      mid = lowh ? pid : mid;
      sid = lowh ? sid : pid;
      __syncthreads();
    }
    if (my_rot && lane == 0) atomicAdd(&rot, 1);
    __syncthreads();
    const bool done = fixed_sweeps > 0 ? sweeps + 1 >= fixed_sweeps : rot == 0;
    if (done) break;
    __syncthreads();
  }
  double2* w = W + (size_t)blockIdx.x * L * C;
  double ns = 0, nm = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + 16 * i;
    w[(size_t)sid * L + row] = make_double2(sr[i], si[i]);
    w[(size_t)mid * L + row] = make_double2(mr[i], mi[i]);
    ns = fma(sr[i], sr[i], fma(si[i], si[i], ns));
    nm = fma(mr[i], mr[i], fma(mi[i], mi[i], nm));
  }
  ns = dpp_sum16(ns);
  nm = dpp_sum16(nm);
  if (lane == 0) {
    sig[blockIdx.x * C + sid] = sqrt(ns);
    sig[blockIdx.x * C + mid] = sqrt(nm);
  }
  if (tid == 0) sweeps_out[blockIdx.x] = sweeps + 1;
}


// ---- block variant: one wave = one S block + one M block of 4 columns each -------------------
// Lane l holds rows l + 64 r (r < R) of its wave's 8 columns.  A block-round pairs the S block
// with the M block in 4 register-only sub-steps of 4 independent rotations; only the M block
// crosses LDS, between block-rounds (4x fewer exchanges than the column kernel).
__device__ __forceinline__ double dsum(unsigned a_lo, unsigned a_hi, unsigned b_lo, unsigned b_hi) {
  return __longlong_as_double(((long long)a_hi << 32) | a_lo) + __longlong_as_double(((long long)b_hi << 32) | b_lo);
}
// reduce-scatter step across the two 32-lane halves: low lanes get a(low)+a(high), high lanes b(low)+b(high)
__device__ __forceinline__ double rs32(double a, double b) {
  const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)y, false, false);
  auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
  return dsum(lo[0], hi[0], lo[1], hi[1]);
}
// same across row pairs (0,1) and (2,3): even rows get a(even)+a(odd), odd rows b(even)+b(odd)
__device__ __forceinline__ double rs16(double a, double b) {
  const long long x = __double_as_longlong(a), y = __double_as_longlong(b);
  auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)y, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(y >> 32), false, false);
  return dsum(lo[0], hi[0], lo[1], hi[1]);
}
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) { return __longlong_as_double(((long long)hi << 32) | lo); }
// all-gather of one double per row: returns (value of row 0|2, value of row 1|3) in (e, o)
__device__ __forceinline__ void ag16(double v, double& e, double& o) {
  const long long x = __double_as_longlong(v);
  auto lo = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
  auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
  e = mkd(lo[0], hi[0]);
  o = mkd(lo[1], hi[1]);
}
// (value of the low half, value of the high half)
__device__ __forceinline__ void ag32(double v, double& l, double& h) {
  const long long x = __double_as_longlong(v);
  auto lo = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
  auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(x >> 32), (unsigned)(x >> 32), false, false);
  l = mkd(lo[0], hi[0]);
  h = mkd(lo[1], hi[1]);
}

template <int R>
__device__ __forceinline__ void bj_dots(const double (&xr)[8][R], const double (&xi)[8][R], int pa, int pb, double* v) {
  double al = 0, be = 0, gx = 0, gy = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double ar = xr[pa][r], ai = xi[pa][r], br = xr[pb][r], bi = xi[pb][r];
    al = fma(ar, ar, fma(ai, ai, al));
    be = fma(br, br, fma(bi, bi, be));
    gx = fma(ar, br, fma(ai, bi, gx));
    gy = fma(ar, bi, fma(-ai, br, gy));
  }
  v[0] = al, v[1] = be, v[2] = gx, v[3] = gy;
}
__device__ __forceinline__ double bcast(double x, int srclane) {
  const long long b = __double_as_longlong(x);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, srclane);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), srclane);
  return mkd(lo, hi);
}

// rotations (a_k, b_k), k < 4, all independent.  Row q of the wave finishes rotation q's
// reduction and parameters; readlane broadcasts them (wave-uniform, so they live in SGPRs).
template <int R, int BC>
__device__ __forceinline__ void bj_substep(double (&xr)[8][R], double (&xi)[8][R], int a0, int b0, int a1, int b1,
                                           int a2, int b2, int a3, int b3, double tol2, double floor2, int& any) {
  const int pa[4] = {a0, a1, a2, a3}, pb[4] = {b0, b1, b2, b3};
  double u[4], w[4];
  {
    double v0[4], v2[4];
    bj_dots<R>(xr, xi, a0, b0, v0);
    bj_dots<R>(xr, xi, a2, b2, v2);
#pragma unroll
    for (int j = 0; j < 4; ++j) u[j] = rs32(v0[j], v2[j]);  // low half: rot 0, high half: rot 2
  }
  {
    double v1[4], v3[4];
    bj_dots<R>(xr, xi, a1, b1, v1);
    bj_dots<R>(xr, xi, a3, b3, v3);
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = rs32(v1[j], v3[j]);  // low half: rot 1, high half: rot 3
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = dpp_sum16(rs16(u[j], w[j]));  // row q: rotation q
  double c = 1.0, ex = 0.0, ey = 0.0;
  {
    const double al = u[0], be = u[1], gx = u[2], gy = u[3];
    const double g2 = gx * gx + gy * gy;
    if (g2 > tol2 * al * be && al > floor2 && be > floor2) {
      const double gg = sqrt(g2);
      const double zeta = (be - al) / (2.0 * gg);
      const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
      c = 1.0 / sqrt(1.0 + t * t);
      const double sc = c * t / gg;
      ex = gx * sc, ey = gy * sc;
      any = 1;
    }
  }
  double pc[4], px[4], py[4];
  if constexpr (BC == 1) {
    double ce, co, xe, xo, ye, yo;
    ag16(c, ce, co);
    ag16(ex, xe, xo);
    ag16(ey, ye, yo);
    ag32(ce, pc[0], pc[2]);
    ag32(co, pc[1], pc[3]);
    ag32(xe, px[0], px[2]);
    ag32(xo, px[1], px[3]);
    ag32(ye, py[0], py[2]);
    ag32(yo, py[1], py[3]);
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) pc[k] = bcast(c, 16 * k), px[k] = bcast(ex, 16 * k), py[k] = bcast(ey, 16 * k);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double cc = pc[k], sx = px[k], sy = py[k];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const double ar = xr[pa[k]][r], ai = xi[pa[k]][r], br = xr[pb[k]][r], bi = xi[pb[k]][r];
      xr[pa[k]][r] = fma(cc, ar, -fma(sx, br, sy * bi));
      xi[pa[k]][r] = fma(cc, ai, -fma(sx, bi, -sy * br));
      xr[pb[k]][r] = fma(cc, br, fma(sx, ar, -sy * ai));
      xi[pb[k]][r] = fma(cc, bi, fma(sx, ai, sy * ar));
    }
  }
}

template <int R>
__device__ __forceinline__ void rotate_m(double (&xr)[8][R], double (&xi)[8][R], int (&id)[8]) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double tr = xr[4][r], ti = xi[4][r];
    xr[4][r] = xr[5][r], xi[4][r] = xi[5][r];
    xr[5][r] = xr[6][r], xi[5][r] = xi[6][r];
    xr[6][r] = xr[7][r], xi[6][r] = xi[7][r];
    xr[7][r] = tr, xi[7][r] = ti;
  }
  const int t = id[4];
  id[4] = id[5], id[5] = id[6], id[6] = id[7], id[7] = t;
}

template <int NW, int R, int BC>
__global__ __launch_bounds__(NW * 64) void k_bj(const double2* __restrict__ A, double2* __restrict__ W,
                                                double* __restrict__ sig, int* __restrict__ sweeps_out,
                                                int fixed_sweeps) {
  constexpr int LR = 64 * R;           // padded rows
  extern __shared__ double2 xbuf[];    // NW * 4 * LR
  __shared__ double fred[NW];
  __shared__ int xid[NW * 4];
  __shared__ int rot;
  const int L = CP, C = CP;
  const double2* a = A + (size_t)blockIdx.x * L * C;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: ids and branches in SGPRs
  double xr[8][R], xi[8][R];
  int id[8];
  double f = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    id[k] = k < 4 ? 4 * w + k : 4 * (NW + w) + k - 4;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = lane + 64 * r;
      double2 x = make_double2(0, 0);
      if (row < L && id[k] < C) x = a[(size_t)id[k] * L + row];
      xr[k][r] = x.x, xi[k][r] = x.y;
      f += x.x * x.x + x.y * x.y;
    }
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) f += __shfl_xor(f, off);
  if (lane == 0) fred[w] = f;
  __syncthreads();
  double fro = 0;
  for (int k = 0; k < NW; ++k) fro += fred[k];
  const double floor2 = fro * 1e-24, tol = c_tolf * L * 2.220446049250313e-16, tol2 = tol * tol;
  int sweeps;
  for (sweeps = 0; sweeps < 40; ++sweeps) {
    if (tid == 0) rot = 0;
    __syncthreads();
    int any = 0;
    bj_substep<R, BC>(xr, xi, 0, 1, 2, 3, 4, 5, 6, 7, tol2, floor2, any);
    bj_substep<R, BC>(xr, xi, 0, 2, 1, 3, 4, 6, 5, 7, tol2, floor2, any);
    bj_substep<R, BC>(xr, xi, 0, 3, 1, 2, 4, 7, 5, 6, tol2, floor2, any);
    for (int m = NW; m >= 1; m >>= 1) {
      const int li = w & (m - 1), base = w - li;
      for (int r = 0; r < m; ++r) {
#pragma unroll 1
        for (int t = 0; t < 4; ++t) {
          bj_substep<R, BC>(xr, xi, 0, 4, 1, 5, 2, 6, 3, 7, tol2, floor2, any);
          rotate_m<R>(xr, xi, id);
        }
        if (r == m - 1) break;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int q = 0; q < R; ++q) xbuf[(w * 4 + k) * LR + lane + 64 * q] = make_double2(xr[4 + k][q], xi[4 + k][q]);
        if (lane == 0) {
#pragma unroll
          for (int k = 0; k < 4; ++k) xid[w * 4 + k] = id[4 + k];
        }
        __syncthreads();
        const int src = base + ((li + 1) & (m - 1));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
          for (int q = 0; q < R; ++q) {
            const double2 v = xbuf[(src * 4 + k) * LR + lane + 64 * q];
            xr[4 + k][q] = v.x, xi[4 + k][q] = v.y;
          }
          id[4 + k] = __builtin_amdgcn_readfirstlane(xid[src * 4 + k]);
        }
        __syncthreads();
      }
      if (m == 1) break;
      const int h = m >> 1;
      const bool lowh = li < h;
      const int off = lowh ? 4 : 0;  // lower half sends M, upper half sends S
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int q = 0; q < R; ++q)
          xbuf[(w * 4 + k) * LR + lane + 64 * q] =
              lowh ? make_double2(xr[4 + k][q], xi[4 + k][q]) : make_double2(xr[k][q], xi[k][q]);
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) xid[w * 4 + k] = lowh ? id[4 + k] : id[k];
      }
      __syncthreads();
      const int partner = lowh ? w + h : w - h;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
          const double2 v = xbuf[(partner * 4 + k) * LR + lane + 64 * q];
          if (lowh) xr[4 + k][q] = v.x, xi[4 + k][q] = v.y;
          else xr[k][q] = v.x, xi[k][q] = v.y;
        }
        const int pid = __builtin_amdgcn_readfirstlane(xid[partner * 4 + k]);
        if (lowh) id[4 + k] = pid;
        else id[k] = pid;
      }
      (void)off;
      __syncthreads();
    }
    if (any) atomicAdd(&rot, 1);
    __syncthreads();
    const bool done = fixed_sweeps > 0 ? sweeps + 1 >= fixed_sweeps : rot == 0;
    if (done) break;
    __syncthreads();
  }
  double2* wo = W + (size_t)blockIdx.x * L * C;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    double n2 = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = lane + 64 * r;
      if (row < L && id[k] < C) wo[(size_t)id[k] * L + row] = make_double2(xr[k][r], xi[k][r]);
      n2 = fma(xr[k][r], xr[k][r], fma(xi[k][r], xi[k][r], n2));
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) n2 += __shfl_xor(n2, off);
    if (lane == 0 && id[k] < C) sig[blockIdx.x * C + id[k]] = sqrt(n2);
  }
  if (tid == 0) sweeps_out[blockIdx.x] = sweeps + 1;
}


// ---- LDS-resident M variant: S columns in VGPRs, the M half in 64 LDS slots --------------------
// Round r of a level with sub-blocks of m groups: group g (li = g - base) pairs S_g with slot
// base + (li + r) mod m -- the "shift" is addressing only.  A slot is written back only when
// its column was rotated (rare in late sweeps).  Level split: the upper half swaps its S with
// slot g - h (that slot then holds an upper S for the lower half).  One barrier per round.
template <int RED>
__global__ __launch_bounds__(kThreads) void k_slot(const double2* __restrict__ A, double2* __restrict__ W,
                                                  double* __restrict__ sig, int* __restrict__ sweeps_out,
                                                  int fixed_sweeps) {
  extern __shared__ double2 xbuf[];  // kG slots x ld
  __shared__ double fred[kThreads / 64];
  __shared__ int xid[kG];
  __shared__ int rot;
  const int L = CP, C = CP;
  const double2* a = A + (size_t)blockIdx.x * L * C;
  const int tid = threadIdx.x, g = tid >> 4, lane = tid & 15;
  double sr[MAXR], si[MAXR];
  int sid = g;
  double f = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = lane + 16 * i;
    const double2 x = a[(size_t)sid * L + r], y = a[(size_t)(g + kG) * L + r];
    sr[i] = x.x, si[i] = x.y;
    xbuf[g * ld + r] = y;
    f += x.x * x.x + x.y * x.y + y.x * y.x + y.y * y.y;
  }
  if (lane == 0) xid[g] = g + kG;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) f += __shfl_xor(f, off);
  if ((tid & 63) == 0) fred[tid >> 6] = f;
  __syncthreads();
  double fro = 0;
  for (int w = 0; w < kThreads / 64; ++w) fro += fred[w];
  const double floor2 = fro * 1e-24, tol = c_tolf * L * 2.220446049250313e-16, tol2 = tol * tol;
  int sweeps;
  for (sweeps = 0; sweeps < 40; ++sweeps) {
    if (tid == 0) rot = 0;
    __syncthreads();
    int my_rot = 0;
    for (int m = kG; m >= 1; m >>= 1) {
      const int li = g & (m - 1), base = g - li;
      for (int r = 0; r < m; ++r) {
        const int slot = base + ((li + r) & (m - 1));
        double2* col = xbuf + slot * ld;
        double mr[MAXR], mi[MAXR];
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const double2 v = col[lane + 16 * i];
          mr[i] = v.x, mi[i] = v.y;
        }
        double al = 0, be = 0, gx = 0, gy = 0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          al = fma(sr[i], sr[i], fma(si[i], si[i], al));
          be = fma(mr[i], mr[i], fma(mi[i], mi[i], be));
          gx = fma(sr[i], mr[i], fma(si[i], mi[i], gx));
          gy = fma(sr[i], mi[i], fma(-si[i], mr[i], gy));
        }
        al = dpp_sum16(al);
        be = dpp_sum16(be);
        gx = dpp_sum16(gx);
        gy = dpp_sum16(gy);
        const double g2 = gx * gx + gy * gy;
        if (g2 > tol2 * al * be && al > floor2 && be > floor2) {
          if (g2 > 16.0 * tol2 * al * be) my_rot = 1;
          double c, ex, ey;
          if constexpr (RED == 2) {
            double rg = __builtin_amdgcn_rsq(g2);
            rg = rg * fma(-0.5 * g2 * rg, rg, 1.5);
            rg = rg * fma(-0.5 * g2 * rg, rg, 1.5);
            const double zeta = 0.5 * (be - al) * rg;
            const double q = fma(zeta, zeta, 1.0);
            double rq = __builtin_amdgcn_rsq(q);
            rq = rq * fma(-0.5 * q * rq, rq, 1.5);
            rq = rq * fma(-0.5 * q * rq, rq, 1.5);
            const double den = fabs(zeta) + q * rq;
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
            ex = gx * sc, ey = gy * sc;
          } else {
            const double gg = sqrt(g2);
            const double zeta = (be - al) / (2.0 * gg);
            const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
            c = 1.0 / sqrt(1.0 + t * t);
            const double sc = c * t / gg;
            ex = gx * sc, ey = gy * sc;
          }
#pragma unroll
          for (int i = 0; i < MAXR; ++i) {
            const double ar = sr[i], ai = si[i], br = mr[i], bi = mi[i];
            sr[i] = fma(c, ar, -fma(ex, br, ey * bi));
            si[i] = fma(c, ai, -fma(ex, bi, -ey * br));
            col[lane + 16 * i] = make_double2(fma(c, br, fma(ex, ar, -ey * ai)), fma(c, bi, fma(ex, ai, ey * ar)));
          }
        }
        __syncthreads();
      }
      if (m == 1) break;
      const int h = m >> 1;
      if (li >= h) {  // upper half: S <-> slot g - h
        double2* col = xbuf + (g - h) * ld;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const double2 v = col[lane + 16 * i];
          col[lane + 16 * i] = make_double2(sr[i], si[i]);
          sr[i] = v.x, si[i] = v.y;
        }
        const int pid = xid[g - h];
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) xid[g - h] = sid;
        sid = pid;
      }
      __syncthreads();
    }
    if (my_rot && lane == 0) atomicAdd(&rot, 1);
    __syncthreads();
    const bool done = fixed_sweeps > 0 ? sweeps + 1 >= fixed_sweeps : rot == 0;
    if (done) break;
    __syncthreads();
  }
  double2* wo = W + (size_t)blockIdx.x * L * C;
  const int mid = xid[g];
  double ns = 0, nm = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + 16 * i;
    const double2 mv = xbuf[g * ld + row];
    wo[(size_t)sid * L + row] = make_double2(sr[i], si[i]);
    wo[(size_t)mid * L + row] = mv;
    ns = fma(sr[i], sr[i], fma(si[i], si[i], ns));
    nm = fma(mv.x, mv.x, fma(mv.y, mv.y, nm));
  }
  ns = dpp_sum16(ns);
  nm = dpp_sum16(nm);
  if (lane == 0) {
    sig[blockIdx.x * C + sid] = sqrt(ns);
    sig[blockIdx.x * C + mid] = sqrt(nm);
  }
  if (tid == 0) sweeps_out[blockIdx.x] = sweeps + 1;
}

struct Out {
  std::vector<double> sig;
  std::vector<double2> W;
  std::vector<int> sw;
};

template <int RED, int XCH, bool ROT>
static float run(const char* name, const double2* dA, double2* dW, double* dS, int* dSw, int B, int fixed, Out* o) {
  auto k = k_lab<RED, XCH, ROT>;
  const size_t lds = (size_t)kG * ld * 16;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(B), dim3(kThreads), lds, 0, dA, dW, dS, dSw, fixed);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(B), dim3(kThreads), lds, 0, dA, dW, dS, dSw, fixed);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  o->sig.resize((size_t)B * CP);
  o->sw.resize(B);
  o->W.resize((size_t)B * CP * CP);
  CK(hipMemcpy(o->sig.data(), dS, o->sig.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o->sw.data(), dSw, B * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o->W.data(), dW, o->W.size() * 16, hipMemcpyDeviceToHost));
  int swmax = *std::max_element(o->sw.begin(), o->sw.end());
  printf("%-34s %8.3f ms  (%.3f CU-ms/SVD, sweeps max %d, %.2f us/round)\n", name, best, best * 256.0 / B, swmax,
         1e3 * best / swmax / (CP - 1) / std::max(1, (B + 255) / 256));
  return best;
}


template <int NW, int R, int BC = 0>
static float run_bj(const char* name, const double2* dA, double2* dW, double* dS, int* dSw, int B, int fixed, Out* o) {
  auto k = k_bj<NW, R, BC>;
  const size_t lds = (size_t)NW * 4 * 64 * R * 16;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(B), dim3(NW * 64), lds, 0, dA, dW, dS, dSw, fixed);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(B), dim3(NW * 64), lds, 0, dA, dW, dS, dSw, fixed);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  o->sig.resize((size_t)B * CP);
  o->sw.resize(B);
  o->W.resize((size_t)B * CP * CP);
  CK(hipMemcpy(o->sig.data(), dS, o->sig.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o->sw.data(), dSw, B * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o->W.data(), dW, o->W.size() * 16, hipMemcpyDeviceToHost));
  int swmax = *std::max_element(o->sw.begin(), o->sw.end());
  printf("%-34s %8.3f ms  (%.3f CU-ms/SVD, sweeps max %d, %.2f us/substep)\n", name, best, best * 256.0 / B, swmax,
         1e3 * best / swmax / (CP - 1) / std::max(1, (B + 255) / 256));
  int hist[64] = {0};
  for (int x : o->sw) hist[std::min(x, 63)]++;
  printf("    sweeps histogram:");
  for (int i = 0; i < 64; ++i) if (hist[i]) printf(" %d:%d", i, hist[i]);
  printf("\n");
  return best;
}


template <int RED>
static float run_slot(const char* name, const double2* dA, double2* dW, double* dS, int* dSw, int B, int fixed, Out* o) {
  auto k = k_slot<RED>;
  const size_t lds = (size_t)kG * ld * 16;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(B), dim3(kThreads), lds, 0, dA, dW, dS, dSw, fixed);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(B), dim3(kThreads), lds, 0, dA, dW, dS, dSw, fixed);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
  }
  o->sig.resize((size_t)B * CP);
  o->sw.resize(B);
  o->W.resize((size_t)B * CP * CP);
  CK(hipMemcpy(o->sig.data(), dS, o->sig.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o->sw.data(), dSw, B * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o->W.data(), dW, o->W.size() * 16, hipMemcpyDeviceToHost));
  int swmax = *std::max_element(o->sw.begin(), o->sw.end());
  printf("%-34s %8.3f ms  (%.3f CU-ms/SVD, sweeps max %d, %.2f us/round)\n", name, best, best * 256.0 / B, swmax,
         1e3 * best / swmax / (CP - 1) / std::max(1, (B + 255) / 256));
  return best;
}

// max relative difference of sorted singular values vs ref; max column non-orthogonality of block 0
static void check(const Out& o, const Out& ref, int B) {
  double dmax = 0;
  for (int b = 0; b < B; ++b) {
    std::vector<double> x(o.sig.begin() + b * CP, o.sig.begin() + (b + 1) * CP), y(ref.sig.begin() + b * CP, ref.sig.begin() + (b + 1) * CP);
    std::sort(x.begin(), x.end());
    std::sort(y.begin(), y.end());
    for (int i = 0; i < CP; ++i) dmax = std::max(dmax, std::fabs(x[i] - y[i]) / y[CP - 1]);
  }
  double omax = 0;
  for (int p = 0; p < CP; ++p)
    for (int q = p + 1; q < CP; ++q) {
      double gr = 0, gi = 0, np = 0, nq = 0;
      for (int r = 0; r < CP; ++r) {
        const double2 a = o.W[(size_t)p * CP + r], b = o.W[(size_t)q * CP + r];
        gr += a.x * b.x + a.y * b.y;
        gi += a.x * b.y - a.y * b.x;
        np += a.x * a.x + a.y * a.y;
        nq += b.x * b.x + b.y * b.y;
      }
      if (np > 1e-20 && nq > 1e-20) omax = std::max(omax, std::sqrt(gr * gr + gi * gi) / std::sqrt(np * nq));
    }
  printf("    sigma diff vs ref %.2e, max |cos| block0 %.2e\n", dmax, omax);
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 256;
  const int fixed = argc > 2 ? atoi(argv[2]) : 0;
  std::vector<double2> h((size_t)B * CP * CP);
  std::mt19937_64 rng(1234);
  std::normal_distribution<double> nd;
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < CP; ++c) {
      const double scale = 1.0 / (1.0 + 0.15 * c);  // graded columns, like lambda-weighted theta
      for (int r = 0; r < CP; ++r) h[((size_t)b * CP + c) * CP + r] = make_double2(nd(rng) * scale, nd(rng) * scale);
    }
  double2 *dA, *dW;
  double* dS;
  int* dSw;
  CK(hipMalloc(&dA, h.size() * 16));
  CK(hipMalloc(&dW, h.size() * 16));
  CK(hipMalloc(&dS, (size_t)B * CP * 8));
  CK(hipMalloc(&dSw, B * 4));
  CK(hipMemcpy(dA, h.data(), h.size() * 16, hipMemcpyHostToDevice));
  printf("blocks %d, fixed sweeps %d (0 = converge)\n", B, fixed);
  Out ref, o;
  run<1, 0, true>("dpp + ring LDS (library)", dA, dW, dS, dSw, B, fixed, &ref);
  run<2, 0, true>("dpp + fast params + ring LDS", dA, dW, dS, dSw, B, fixed, &o);
  check(o, ref, B);
  run_slot<1>("LDS-resident M slots", dA, dW, dS, dSw, B, fixed, &o);
  check(o, ref, B);
  run_slot<2>("LDS-resident M + fast params", dA, dW, dS, dSw, B, fixed, &o);
  check(o, ref, B);
  const int fs = fixed > 0 ? fixed : 14;
  run<1, 2, true>("dpp + no exchange [timing]", dA, dW, dS, dSw, B, fs, &o);
  run<2, 2, true>("dpp + fast params, no exch [timing]", dA, dW, dS, dSw, B, fs, &o);
  return 0;
}
