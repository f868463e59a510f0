// FP32 register Jacobi for the two-site SVD: the same algorithm as jacobi_reg_body (mps.hip) --
// pivoted Householder QR, then one-sided Jacobi on R^H with scaled rotations and tracked norms --
// with the columns, reflectors and rotation parameters in single precision.  On gfx950 an FP32
// FMA issues in half the cycles of an FP64 one and a 16-lane DPP sum is one fused v_add_f32_dpp
// per step instead of two moves and an add, so a round costs about half the FP64 round.  Its
// result is only a preconditioner: the FP64 stage (mixed-precision pipeline, mps.hip) re-orthogonalises
// the right singular vectors it implies and finishes with FP64 sweeps.
//
// Included into mps.hip's anonymous namespace (needs TwoSiteJob, kMaxSweeps, pivot_key).
#pragma once

typedef float2 fcplx;

template <int CTRL>
__device__ __forceinline__ float dpp_perm_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

template <int LPG>
__device__ __forceinline__ float group_sum_f(float v) {
  v += dpp_perm_f<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_perm_f<0x4E>(v);  // quad_perm [2,3,0,1]
  if constexpr (LPG == 8) {
    v += dpp_perm_f<0x141>(v);  // row_half_mirror
  } else if constexpr (LPG == 16) {
    v += dpp_perm_f<0x124>(v);  // row_ror:4
    v += dpp_perm_f<0x128>(v);  // row_ror:8
  }
  return v;
}

// rotation parameters without |g| (jacobi_te), single precision: v_rsq_f32 / v_rcp_f32 are
// accurate to about 1 ulp, no Newton steps
__device__ __forceinline__ void jacobi_te_f(float al, float be, float g2, float& te, float& c, float& p) {
  const float h = 0.5f * (be - al);
  const float q = fmaf(h, h, g2);
  const float den = fabsf(h) + q * __builtin_amdgcn_rsqf(q);
  const float inv = __builtin_amdgcn_rcpf(den);
  te = h >= 0.f ? inv : -inv;
  p = fmaf(te * te, g2, 1.0f);
  c = __builtin_amdgcn_rsqf(p);
}

template <int MAXR, int LPG>
__device__ __forceinline__ void qr_reflector_f(float (&xr)[MAXR], float (&xi)[MAXR], int k, int lane, fcplx* vb,
                                               fcplx* tb) {
  const int kr = k / LPG;
  float ar = 0, ai = 0, s2p[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + LPG * i;
    if (i == kr) ar = xr[i], ai = xi[i];
    const float w = row > k ? 1.0f : 0.0f;
    s2p[i & 1] = fmaf(w, fmaf(xr[i], xr[i], xi[i] * xi[i]), s2p[i & 1]);
  }
  ar = __shfl(ar, k % LPG, LPG);
  ai = __shfl(ai, k % LPG, LPG);
  const float s2 = group_sum_f<LPG>(s2p[0] + s2p[1]);
  float beta, tr_, ti_, cr = 0, ci = 0;
  if (s2 == 0.0f && ai == 0.0f) {
    beta = ar, tr_ = 0.0f, ti_ = 0.0f;
  } else {
    const float x = fmaf(ar, ar, fmaf(ai, ai, s2));
    const float r = __builtin_amdgcn_rsqf(x);
    const float nrm = x * r;
    beta = ar >= 0.0f ? -nrm : nrm;
    const float ib = ar >= 0.0f ? -r : r;
    tr_ = (beta - ar) * ib;
    ti_ = -ai * ib;
    const float dr = ar - beta, di = ai, d2 = fmaf(dr, dr, di * di);
    const float id2 = __builtin_amdgcn_rcpf(d2);
    cr = dr * id2, ci = -di * id2;
  }
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + LPG * i;
    fcplx v = make_float2(0, 0);
    if (row > k) v = make_float2(xr[i] * cr - xi[i] * ci, xr[i] * ci + xi[i] * cr);
    if (row == k) v = make_float2(1.0f, 0.0f);
    vb[row] = v;
    const float nr = row == k ? beta : (row > k ? 0.0f : xr[i]);
    const float ni = row >= k ? 0.0f : xi[i];
    xr[i] = nr, xi[i] = ni;
  }
  if (lane == 0) *tb = make_float2(tr_, ti_);
}

// One 2chi x 2chi theta (CP = 128: 64 groups of LPG = 16 lanes, MAXR = 8 rows per lane).  Output:
// j.work column c (length C, FP64) = the right singular vector of theta' for the c-th Jacobi
// column scaled by its singular value (rows in theta's column order: the pivot order is undone),
// j.sig[c] its norm -- the k_jacobi_reg variant-2 contract, at FP32 accuracy.  `tiny` ends the
// sweeps after one whose rotations all had |t| <= tiny.
template <int CP, int MAXR, int LPG = 16>
__device__ __forceinline__ void jacobi32_body(const TwoSiteJob& j, float tiny) {
  static_assert(LPG * MAXR == CP, "LPG lanes x MAXR rows must cover the CP rows of a column");
  constexpr int kG = CP / 2;
  constexpr int kThreads = kG * LPG;
  constexpr int ld = LPG * MAXR + (LPG < 16 ? LPG : 0);
  constexpr int ldt = CP + 1;
  extern __shared__ double2 xbuf_raw[];
  fcplx* xbuf = reinterpret_cast<fcplx*>(xbuf_raw);
  __shared__ float fred[kThreads / 64];
  __shared__ int xid[kG];
  __shared__ int rot, big;
  __shared__ unsigned long long pkey[2];
  __shared__ fcplx vb[2][CP];
  __shared__ fcplx tb[2];
  __shared__ int perm_s[CP];
  const int chl = j.dims[0], chr = j.dims[2];
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = M < N;
  const int L = tr ? N : M;
  const int C = tr ? M : N;
  const int tid = threadIdx.x;
  const int g = tid / LPG, lane = tid % LPG;
  float sr[MAXR], si[MAXR], mr[MAXR], mi[MAXR];
  int sid = g, mid = g + kG;
  float f = 0.0f;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int r = lane + LPG * i;
    const int cs = g, cm = g + kG;
    double2 a = make_double2(0, 0), b = make_double2(0, 0);
    if (r < L && cs < C) a = tr ? aqc::cconj(j.theta[(size_t)r * M + cs]) : j.theta[(size_t)cs * M + r];
    if (r < L && cm < C) b = tr ? aqc::cconj(j.theta[(size_t)r * M + cm]) : j.theta[(size_t)cm * M + r];
    sr[i] = (float)a.x;
    si[i] = (float)a.y;
    mr[i] = (float)b.x;
    mi[i] = (float)b.y;
    f += sr[i] * sr[i] + si[i] * si[i] + mr[i] * mr[i] + mi[i] * mi[i];
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) f += __shfl_xor(f, off);
  if ((tid & 63) == 0) fred[tid >> 6] = f;
  if (tid == 0) pkey[0] = pkey[1] = 0ull;
  __syncthreads();
  if (tid == 0) {
    float s = 0.0f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += fred[w];
    fred[0] = s;
  }
  {  // pivoted Householder QR (as jacobi_reg_body)
    int ks = -1, km = -1;
    float ns = 0, nm = 0, nsr = 0, nmr = 0;
    for (int k = 0; k < C; ++k) {
      const int b = k & 1;
      bool exact = k == 0;
      if (k > 0) {
        const int kr = (k - 1) / LPG, kl = (k - 1) % LPG;
        float xsr = 0, xsi = 0, xmr = 0, xmi = 0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          if (i == kr) xsr = sr[i], xsi = si[i], xmr = mr[i], xmi = mi[i];
        }
        ns -= __shfl(fmaf(xsr, xsr, xsi * xsi), kl, LPG);
        nm -= __shfl(fmaf(xmr, xmr, xmi * xmi), kl, LPG);
        exact = ns <= 3e-4f * nsr || nm <= 3e-4f * nmr;  // sqrt(eps32) of the last exact value
      }
      if (exact) {
        ns = 0, nm = 0;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const float w = (lane + LPG * i) >= k ? 1.0f : 0.0f;
          ns = fmaf(w, fmaf(sr[i], sr[i], si[i] * si[i]), ns);
          nm = fmaf(w, fmaf(mr[i], mr[i], mi[i] * mi[i]), nm);
        }
        ns = group_sum_f<LPG>(ns);
        nm = group_sum_f<LPG>(nm);
        nsr = ns, nmr = nm;
      }
      const unsigned long long ka = (ks < 0 && sid < C) ? pivot_key((double)fmaxf(ns, 0.f), sid) : 0ull;
      const unsigned long long kb = (km < 0 && mid < C) ? pivot_key((double)fmaxf(nm, 0.f), mid) : 0ull;
      if (lane == 0) atomicMax(&pkey[b], ka > kb ? ka : kb);
      __syncthreads();
      const int p = 255 - (int)(pkey[b] & 255ull);
      if (tid == 0) pkey[b ^ 1] = 0ull;
      if (sid == p) {
        qr_reflector_f<MAXR, LPG>(sr, si, k, lane, vb[b], &tb[b]);
        ks = k;
      } else if (mid == p) {
        qr_reflector_f<MAXR, LPG>(mr, mi, k, lane, vb[b], &tb[b]);
        km = k;
      }
      if (tid == 0) perm_s[k] = p;
      __syncthreads();
      const fcplx tau = tb[b];
      float wsr = 0, wsi = 0, wmr = 0, wmi = 0;
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        const fcplx v = vb[b][lane + LPG * i];
        wsr = fmaf(v.x, sr[i], fmaf(v.y, si[i], wsr));
        wsi = fmaf(v.x, si[i], fmaf(-v.y, sr[i], wsi));
        wmr = fmaf(v.x, mr[i], fmaf(v.y, mi[i], wmr));
        wmi = fmaf(v.x, mi[i], fmaf(-v.y, mr[i], wmi));
      }
      wsr = group_sum_f<LPG>(wsr);
      wsi = group_sum_f<LPG>(wsi);
      wmr = group_sum_f<LPG>(wmr);
      wmi = group_sum_f<LPG>(wmi);
      const float as = ks < 0 ? 1.0f : 0.0f, am = km < 0 ? 1.0f : 0.0f;
      const float fsr = as * (tau.x * wsr + tau.y * wsi), fsi = as * (tau.x * wsi - tau.y * wsr);
      const float fmr = am * (tau.x * wmr + tau.y * wmi), fmi = am * (tau.x * wmi - tau.y * wmr);
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        const fcplx v = vb[b][lane + LPG * i];
        sr[i] = fmaf(-v.x, fsr, fmaf(v.y, fsi, sr[i]));
        si[i] = fmaf(-v.x, fsi, fmaf(-v.y, fsr, si[i]));
        mr[i] = fmaf(-v.x, fmr, fmaf(v.y, fmi, mr[i]));
        mi[i] = fmaf(-v.x, fmi, fmaf(-v.y, fmr, mi[i]));
      }
    }
    // X = R^H through the LDS transpose (as jacobi_reg_body)
    constexpr int H = MAXR / 2;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int i = h * H; i < (h + 1) * H; ++i) {
        const int jx = lane + LPG * (i - h * H);
        if (ks >= 0) xbuf[jx * ldt + ks] = make_float2(sr[i], -si[i]);
        if (km >= 0) xbuf[jx * ldt + km] = make_float2(mr[i], -mi[i]);
      }
      __syncthreads();
      const bool real_col = g + h * kG < C;
#pragma unroll
      for (int i = h * H; i < (h + 1) * H; ++i) {
        const int ra = lane + LPG * (i - h * H), rb = ra + kG;
        fcplx va = make_float2(0, 0), vb2 = make_float2(0, 0);
        if (real_col && ra < C) va = xbuf[g * ldt + ra];
        if (real_col && rb < C) vb2 = xbuf[g * ldt + rb];
        sr[i] = va.x, si[i] = va.y;
        mr[i] = vb2.x, mi[i] = vb2.y;
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const float tr0 = mr[i], ti0 = mi[i];
      mr[i] = sr[i + H], mi[i] = si[i + H];
      sr[i + H] = tr0, si[i + H] = ti0;
    }
  }
  const int Lj = C;
  __syncthreads();
  const float floor2 = fred[0] * 1e-14f;
  const float tol = (float)j.jtol * (float)Lj * 1.1920929e-7f;
  const float tol2 = tol * tol;
  __shared__ float xnrm[kG], xscl[kG], xisc[kG];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < MAXR; ++i) xbuf[g * ld + lane + LPG * i] = make_float2(mr[i], mi[i]);
  if (lane == 0) {
    xid[g] = mid;
    xscl[g] = 1.0f;
  }
  const float tiny2 = tiny * tiny;
  float sd = 1.0f, sn = 0.0f;
  int sweeps = 0;
  for (sweeps = 0; sweeps < kMaxSweeps; ++sweeps) {
    {
      fcplx* own = xbuf + g * ld;
      const float od = xscl[g];
      float a = 0, b = 0;
#pragma unroll
      for (int i = 0; i < MAXR; ++i) {
        sr[i] *= sd;
        si[i] *= sd;
        fcplx v = own[lane + LPG * i];
        v.x *= od;
        v.y *= od;
        own[lane + LPG * i] = v;
        a = fmaf(sr[i], sr[i], fmaf(si[i], si[i], a));
        b = fmaf(v.x, v.x, fmaf(v.y, v.y, b));
      }
      a = group_sum_f<LPG>(a);
      b = group_sum_f<LPG>(b);
      sd = 1.0f;
      sn = a;
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        xscl[g] = 1.0f;
        xisc[g] = 1.0f;
        xnrm[g] = b;
      }
      if (tid == 0) rot = big = 0;
    }
    __syncthreads();
    float isd = 1.0f;
    int my_rot = 0, my_big = 0;
    for (int m = kG; m >= 1; m >>= 1) {
      const int li = g & (m - 1), base = g - li;
      for (int r = 0; r < m; ++r) {
        const int slot = base + ((li + r) & (m - 1));
        fcplx* col = xbuf + slot * ld;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const fcplx v = col[lane + LPG * i];
          mr[i] = v.x;
          mi[i] = v.y;
        }
        const float mn = xnrm[slot], md = xscl[slot], imd = xisc[slot];
        float gx = 0.f, gy = 0.f;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          gx = fmaf(sr[i], mr[i], fmaf(si[i], mi[i], gx));
          gy = fmaf(sr[i], mi[i], fmaf(-si[i], mr[i], gy));
        }
        gx = group_sum_f<LPG>(gx);
        gy = group_sum_f<LPG>(gy);
        const float dd = sd * md;
        gx *= dd;
        gy *= dd;
        const float g2 = gx * gx + gy * gy;
        const float ab = sn * mn;
        if (g2 > tol2 * ab && sn > floor2 && mn > floor2) {
          float te, c, p;
          jacobi_te_f(sn, mn, g2, te, c, p);
          if (g2 > 16.0f * tol2 * ab) {
            my_rot = 1;
            if (p - 1.0f > tiny2) my_big = 1;
          }
          const float ra = md * isd, ira = sd * imd;
          const float mux = te * gx * ra, muy = -te * gy * ra;
          const float nux = te * gx * ira, nuy = te * gy * ira;
#pragma unroll
          for (int i = 0; i < MAXR; ++i) {
            const float ar = sr[i], ai = si[i], br = mr[i], bi = mi[i];
            sr[i] = fmaf(-mux, br, fmaf(muy, bi, ar));
            si[i] = fmaf(-mux, bi, fmaf(-muy, br, ai));
            col[lane + LPG * i] = make_float2(fmaf(nux, ar, fmaf(-nuy, ai, br)), fmaf(nux, ai, fmaf(nuy, ar, bi)));
          }
          const float ic = p * c;
          sd *= c;
          isd *= ic;
          const float md2 = md * c, imd2 = imd * ic;
          const float tg = te * g2;
          float sn2 = sn - tg, mn2 = mn + tg;
          if (sn2 < 1e-3f * sn || mn2 < 1e-3f * mn) {
            float a = 0, b = 0;
            asm volatile("" ::: "memory");
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {
              const fcplx v = col[lane + LPG * i];
              a = fmaf(sr[i], sr[i], fmaf(si[i], si[i], a));
              b = fmaf(v.x, v.x, fmaf(v.y, v.y, b));
            }
            sn2 = group_sum_f<LPG>(a) * sd * sd;
            mn2 = group_sum_f<LPG>(b) * md2 * md2;
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
      if (li >= h) {
        fcplx* col = xbuf + (g - h) * ld;
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const fcplx v = col[lane + LPG * i];
          col[lane + LPG * i] = make_float2(sr[i], si[i]);
          sr[i] = v.x;
          si[i] = v.y;
        }
        const int pid = xid[g - h];
        const float pn = xnrm[g - h], pd = xscl[g - h], pi = xisc[g - h];
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
  // columns (scaled) to their slots with the rows mapped back through the pivot order, FP64
  double2* W = j.work;
  const int mid_out = xid[g];
  const float od = xscl[g];
  float ns = 0, nm = 0;
#pragma unroll
  for (int i = 0; i < MAXR; ++i) {
    const int row = lane + LPG * i;
    fcplx mv = xbuf[g * ld + row];
    mv.x *= od;
    mv.y *= od;
    const float ar = sr[i] * sd, ai = si[i] * sd;
    if (row < Lj) {
      const int orow = perm_s[row];
      if (sid < C) W[(size_t)sid * Lj + orow] = make_double2(ar, ai);
      if (mid_out < C) W[(size_t)mid_out * Lj + orow] = make_double2(mv.x, mv.y);
    }
    ns = fmaf(ar, ar, fmaf(ai, ai, ns));
    nm = fmaf(mv.x, mv.x, fmaf(mv.y, mv.y, nm));
  }
  ns = group_sum_f<LPG>(ns);
  nm = group_sum_f<LPG>(nm);
  if (lane == 0) {
    if (sid < C) j.sig[sid] = sqrt((double)ns);
    if (mid_out < C) j.sig[mid_out] = sqrt((double)nm);
  }
  if (tid == 0) {
    if (sweeps >= kMaxSweeps) atomicOr(&j.flags[1], 1);
    atomicMax(&j.flags[2], sweeps + 1);
  }
}

template <int CP, int MAXR, int LPG = 16>
__global__ __launch_bounds__(CP / 2 * LPG) void k_jacobi32(const TwoSiteJob* __restrict__ jobs, float tiny) {
  jacobi32_body<CP, MAXR, LPG>(jobs[blockIdx.x], tiny);
}
