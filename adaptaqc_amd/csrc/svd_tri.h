// Two-site SVD at 2 chi = 128 for the two-states-per-CU chain (k_chain256): the Gram path of
// svd_gram.h (G = X^H X, Householder tridiagonalisation, Sturm multisection, inverse iteration,
// back-transformation) re-laid-out for a 256-thread workgroup with at most ~76 KB of LDS, so that
// two states' workgroups share a CU and each one's serial per-column chain and barriers are covered
// by the other's issue.
//
// What changes against the 1024-thread body:
//   * G is held as its LOWER TRIANGLE ONLY (8256 of 16384 entries, 128 VGPRs per lane): the
//     1024-thread body keeps the whole Hermitian matrix (256 KB of registers = the CU's whole file
//     with the rest of the workgroup), which is what held it to one state per CU.  Thread t owns
//     one TR x 2TR tile (R, Cb) of the strictly lower part, tiles dealt in order of their death
//     column (Cb ascending) so that waves retire as the trailing block shrinks; the even diagonal
//     TR x TR blocks are spread one element per lane (a 16-lane group per block, wave 3 holding two
//     for the last four blocks), the odd ones sit in the right half of the "half tiles"
//     (R = 2 Cb + 1) whose left half is the strictly lower block beside them.  A stored element
//     contributes to y = G x twice: g x_c to its row and conj(g) x_r to its column (diagonal blocks,
//     stored whole, only to their rows).
//   * Three stages, repacked through global scratch when the trailing block halves: tiles of 4 x 8
//     (trailing 128, columns 0..63), 2 x 4 (trailing 64, columns 64..95), 1 x 2 (trailing 32): a
//     lane's work per column falls with the trailing block instead of the last live tiles keeping a
//     wave's full tile pass going to the end.
//   * Per column two barriers, no single-wave phase B: the pass writes per-tile partial products
//     into a grid of per-row contribution lists, two (four, eight) threads per row sum a row and
//     form reflector k's p, v, z (zlarfg's scalars by wave 0 after its own pass).
//   * S5 (inverse iteration) in two batches of 32 vectors (LDS), S6 on four waves, each owning 16
//     columns of V whole (no cross-wave partial sums for Y^H V).
// A declined decomposition (shape, eigenvalue floor) returns false: k_chain256 then hands the rest
// of that state's list to the 1024-thread chain, which runs the register Jacobi.
//
// Included into mps.hip's anonymous namespace after svd_gram.h (shares its helpers and counters).
#pragma once

namespace tri {

constexpr int kThreads = 256;
// dynamic LDS map (complex units)
constexpr int kGrid = 0;        // S3: the partial-product grid, 784 x TR entries (<= 3136)
constexpr int kVec = 3136;      // S3: {v, p, z} of the last reflector, 136 rows (128.. zero)
constexpr int kGk1 = 3544;      // S3: G^(k)[r][k + 1]
constexpr int kScal = 3672;     // S3: reflector k's 1 / (alpha - beta), tau / (alpha - beta)
constexpr int kKtp = 3676;      // S3: p^H v per wave
// live from S3 to the end of S6
constexpr int kD = 4096;        // 128 doubles: d_k
constexpr int kE = 4160;        // 128 doubles: e_k = beta_k
constexpr int kE2 = 4224;       // 128 doubles: e_k^2
constexpr int kDE = 4288;       // 128 double2: Sturm rows (d_i, e_{i-1}^2) / ||T||
constexpr int kLam = 4416;      // 64 doubles
constexpr int kSig2 = 4448;     // 64 doubles
constexpr int kTau = 4480;      // 130 complex: tau_k at kTau + 1 + k (tau_{-1} = 0)
constexpr int kMisc = 4610;     // lo, hi, tn
constexpr int kLdsComplex = 4616;
constexpr int kLdsBytes = kLdsComplex * 16;
constexpr size_t kScratch = 8192;  // complex offset of the global scratch in j.work (reflectors below)

// (TriLds, the LDS map per workgroup size: svd_gram.h)
static_assert(TriLds<256>::kVec == kVec && TriLds<256>::kD == kD && TriLds<256>::kE == kE && TriLds<256>::kTau == kTau,
              "the 256-thread LDS map");
// grid sizes: TR x tri_off<NB>(NB) entries (NB - R / 2 per row block R) -- 4 x 784 at 256 threads,
// 2 x 3104 at 1024 -- below each map's vectors; the 1024-thread map inside the chain's dynamic LDS
static_assert(4 * (2 * 32 * 16 - 16 * 15) <= TriLds<256>::kVec, "256-thread grid");
static_assert(2 * (2 * 64 * 32 - 32 * 31) <= TriLds<1024>::kVec, "1024-thread grid");
static_assert(TriLds<1024>::kVec + 3 * 136 <= TriLds<1024>::kGk1 && TriLds<1024>::kGk1 + 128 <= TriLds<1024>::kScal &&
                  TriLds<1024>::kKtp + 16 <= TriLds<1024>::kD && TriLds<1024>::kD + 64 <= TriLds<1024>::kE &&
                  TriLds<1024>::kE + 64 <= TriLds<1024>::kTau && TriLds<1024>::kEnd * 16 <= kChainLdsBytes,
              "1024-thread LDS map");

#if defined(__HIP_DEVICE_COMPILE__)
using lcplx = __attribute__((address_space(3))) cplx;
using ldbl = __attribute__((address_space(3))) double;
using ldbl2 = __attribute__((address_space(3))) double2;
using lint = __attribute__((address_space(3))) int;
#else
using lcplx = cplx;
using ldbl = double;
using ldbl2 = double2;
using lint = int;
#endif

// NB row blocks of height TR over the trailing S = NB TR rows (NB = 32 at 256 threads, 64 at
// 1024): column block c (width 2 TR) holds tiles R = 2c + 1 .. NB - 1
template <int NB>
__device__ __forceinline__ int tri_cum(int c) { return c * (NB - c); }
// first grid entry of row block R (entries of TR complex): NB - R / 2 entries per row block
template <int NB>
__device__ __forceinline__ int tri_off(int R) {
  const int m = R >> 1, e = R & 1;
  return 2 * NB * m - m * (m - 1) + e * (NB - m);
}

// Lane t's work in a stage of tile height TR (width 2 TR, trailing size NB TR) on NT threads:
// tile (R, Cb) and up to two elements of the even diagonal blocks (local row / col, -1: none);
// last = the lane's last live stage-local column.
template <int TR, int NT>
__device__ __forceinline__ void tri_map(int t, int& R, int& Cb, int (&dr)[2], int (&dc)[2], int& last) {
  constexpr int TC = 2 * TR, Q = TR * TR, NB = NT == 256 ? 32 : 64;
  int c = 0;
  while (c < NB / 2 - 1 && tri_cum<NB>(c + 1) <= t) ++c;
  Cb = c;
  R = 2 * c + 1 + (t - tri_cum<NB>(c));
  last = TC * Cb + TC - 1;  // (a half tile's right half is the odd diagonal block: live to its last column)
  dr[0] = dc[0] = dr[1] = dc[1] = -1;
  int prev = -Q, ovf = 0;
  for (int B = 0; B < NB / 2; ++B) {
    int a = (tri_cum<NB>(B) + Q - 1) / Q * Q;
    a = a > prev + Q ? a : prev + Q;
    int slot = 0;
    if (a + Q > NT) {  // no room left among the tiles that outlive it: the last wave's second slot
      a = NT - 64 + Q * ovf++;
      slot = 1;
    } else {
      prev = a;
    }
    if (t >= a && t < a + Q) {
      const int u = t - a;
      dr[slot] = 2 * B * TR + u / TR;
      dc[slot] = 2 * B * TR + u % TR;
      const int dl = 2 * B * TR + TR - 1;
      last = last > dl ? last : dl;
    }
  }
}

// sum over aligned groups of N lanes (N = 1, 2, 4, 8, 16)
template <int N>
__device__ __forceinline__ double group_sum_n(double v) {
  static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16, "group size");
  if constexpr (N == 2) return v + aqc::dpp_perm<0xB1>(v);
  else if constexpr (N == 4) return aqc::row_sum4(v);
  else if constexpr (N == 8) return aqc::row_sum8(v);
  else if constexpr (N == 16) return aqc::row_sum16(v);
  else return v;
}

// wave-uniform maximum of an int
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
  return __builtin_amdgcn_readfirstlane(v);
}

// sum of the NW waves' p^H v partials (LDS broadcasts)
template <int NW>
__device__ __forceinline__ cplx ktp_sum(const lcplx* ktp) {
  cplx t[4] = {aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0)};
#pragma unroll
  for (int w = 0; w < NW; ++w) t[w & 3] = aqc::cadd(t[w & 3], ktp[w]);
  return aqc::cadd(aqc::cadd(t[0], t[1]), aqc::cadd(t[2], t[3]));
}

// (S3Ctx: svd_gram.h, where gram_svd_body<true> calls the stages at 1024 threads)

// G[a][b] (a <= b) in gram_svd_body's packed LDS copy of the upper triangle (its S2): block (0, 1)
// square (row stride 65), then the packed upper triangles of the diagonal 64 x 64 blocks
__device__ __forceinline__ int gsq_index(int a, int b) {
  if (b < 64) return 64 * 65 + b * (b + 1) / 2 + a;
  if (a >= 64) return 64 * 65 + 2080 + (b - 64) * (b - 63) / 2 + (a - 64);
  return a * 65 + (b - 64);
}

// One stage of the tridiagonalisation on NT threads: columns k0 .. k1 - 1 with tiles of height TR
// over the trailing NB TR rows.  mode 0 (256 threads): the tiles are formed from X (S1); 1: loaded
// from the repack scratch (trailing block from 128 - NB TR); 2 (1024 threads, the first stage):
// from gram_svd_body's packed LDS copy of G (gsq_index).  If k1 < C - 1 the stage ends by writing
// the next stage's trailing block to the scratch; otherwise it forms d_{C-1}.
template <int TR, int NT>
__device__ __noinline__ void s3_stage(const S3Ctx& cx_in, int k0, int k1, int mode) {
  // (arguments arrive in VGPRs: the uniform ones back to SGPRs, so the column loop and its tests
  // are scalar)
  S3Ctx cx;
  cx.C = __builtin_amdgcn_readfirstlane(cx_in.C);
  cx.hh = uniform_ptr(cx_in.hh);
  cx.scratch = uniform_ptr(cx_in.scratch);
  cx.th = uniform_ptr(cx_in.th);
  cx.M = __builtin_amdgcn_readfirstlane(cx_in.M);
  cx.L = __builtin_amdgcn_readfirstlane(cx_in.L);
  cx.tr = __builtin_amdgcn_readfirstlane(cx_in.tr);
  k0 = __builtin_amdgcn_readfirstlane(k0);
  k1 = __builtin_amdgcn_readfirstlane(k1);
  mode = __builtin_amdgcn_readfirstlane(mode);
  constexpr int NB = NT == 256 ? 32 : 64, NW = NT / 64;
  constexpr int TC = 2 * TR, S = NB * TR, GPR = NT / S;
  using Map = TriLds<NT>;
  extern __shared__ double2 xbuf[];
  lcplx* lb = (lcplx*)xbuf;
  asm volatile("" : "+s"(lb));
  lcplx* grid = lb + Map::kGrid;
  lcplx* vec = lb + Map::kVec;
  lcplx* gk1b = lb + Map::kGk1;
  lcplx* scal = lb + Map::kScal;
  lcplx* ktp = lb + Map::kKtp;
  ldbl* dS = (ldbl*)(lb + Map::kD);
  ldbl* eS = (ldbl*)(lb + Map::kE);
  lcplx* tauS = lb + Map::kTau + 1;  // tauS[-1] = 0
  const int C = cx.C;
  const int base = 128 - S;
  const int tid = fresh_tid(), lane = tid & 63, wave = tid >> 6;
  int R, Cb, dr[2], dc[2], last;
  tri_map<TR, NT>(tid, R, Cb, dr, dc, last);
  const int wlast = wave_max_i(last);  // (uniform)
  const bool half = R == 2 * Cb + 1;
  const int rl0 = base + TR * R, cl0 = base + TC * Cb;  // global first row / column of the tile
  // the grid entries this lane writes (complex units)
  const int o_row = TR * (tri_off<NB>(R) + Cb);
  const int o_clo = TR * (tri_off<NB>(2 * Cb) + R - Cb - 1);
  const int o_chi = TR * (tri_off<NB>(2 * Cb + 1) + R - Cb);
  int o_d[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int B = dr[s] >= 0 ? dr[s] / (2 * TR) : 0;
    o_d[s] = dr[s] >= 0 ? TR * (tri_off<NB>(2 * B) + NB - 1 - B) + (dr[s] - 2 * B * TR) : 0;
  }
  const int gdr0 = base + dr[0], gdc0 = base + dc[0], gdr1 = base + dr[1], gdc1 = base + dc[1];
  cplx g[TR][TC];
  cplx gd[2] = {aqc::cmk(0, 0), aqc::cmk(0, 0)};
  // phase ticks of thread 0 (summed into g_gram_ticks: [6] pass + zlarfg + barrier A, [7] row sums
  // + p / v / z + barrier B, [9] S1, [10] the stage's entry load / exit repack)
  unsigned long long t_pa = 0, t_pb = 0, t_m = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
  auto lap = [&](unsigned long long& acc) {
    if (tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc += t - t_m;
      t_m = t;
    }
  };
  unsigned long long t_s1 = 0, t_io = 0;
  if (mode != 1) {
    if constexpr (NT == 256) {
      if (mode == 0) {
    // ---- S1: G = X^H X into the tiles and diagonal elements: X staged through the LDS in chunks
    // of 8 rows, column c at position (c & 3) 32 + (c >> 2) (lanes with consecutive R read
    // consecutive complex), double-buffered with the next chunk's global loads in flight
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int jj = 0; jj < TC; ++jj) g[i][jj] = aqc::cmk(0, 0);
    constexpr int KC = 8;
    auto pos = [](int c) { return (c & 3) * 32 + (c >> 2); };
    const int nch = (cx.L + KC - 1) / KC;
    // element e of a chunk: (row kk, column c), lanes along theta's contiguous index
    auto elem = [&](int e, int& kk, int& c) {
      kk = cx.tr ? e >> 7 : e & 7;
      c = cx.tr ? e & 127 : e >> 3;
    };
    auto fetch = [&](int ch, cplx (&x)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int kk, c;
        elem(tid + 256 * u, kk, c);
        kk += ch * KC;
        cplx v = aqc::cmk(0, 0);
        if (kk < cx.L && c < C) v = cx.tr ? aqc::ldg(cx.th + (size_t)kk * cx.M + c) : aqc::ldg(cx.th + (size_t)c * cx.M + kk);
        x[u] = v;
      }
    };
    auto stash = [&](int buf, const cplx (&x)[4]) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int kk, c;
        elem(tid + 256 * u, kk, c);
        cplx v = x[u];
        if (cx.tr) v.y = -v.y;
        lb[buf * 1024 + kk * 128 + pos(c)] = v;
      }
    };
    cplx xn[4];
    fetch(0, xn);
    stash(0, xn);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      const bool more = ch + 1 < nch;
      if (more) fetch(ch + 1, xn);
      const lcplx* cb = lb + (ch & 1) * 1024;
      for (int l = 0; l < KC; ++l) {
        const lcplx* row = cb + l * 128;
        cplx xr[TR];
#pragma unroll
        for (int i = 0; i < TR; ++i) xr[i] = row[pos(rl0 + i)];
#pragma unroll
        for (int jj = 0; jj < TC; ++jj) {
          const cplx xc = row[pos(cl0 + jj)];
#pragma unroll
          for (int i = 0; i < TR; ++i) g[i][jj] = aqc::cfmac(xr[i], xc, g[i][jj]);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (dr[s] >= 0) {  // (lane-dependent: two loads, one fma)
            const int a = s ? gdr1 : gdr0, b = s ? gdc1 : gdc0;
            gd[s] = aqc::cfmac(row[pos(a)], row[pos(b)], gd[s]);
          }
        }
      }
      if (more) stash((ch + 1) & 1, xn);
      __syncthreads();
    }
      }
    }
    if (mode == 2) {
      // ---- G from gram_svd_body's packed LDS copy of its upper triangle (trailing block = all of G)
      auto ldq = [&](int r, int c) {
        cplx v = aqc::cmk(0, 0);
        if (r < C && c < C) {
          v = lb[r <= c ? gsq_index(r, c) : gsq_index(c, r)];
          if (r > c) v.y = -v.y;
        }
        return v;
      };
#pragma unroll
      for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int jj = 0; jj < TC; ++jj) g[i][jj] = ldq(rl0 + i, cl0 + jj);
      if (dr[0] >= 0) gd[0] = ldq(gdr0, gdc0);
      if (dr[1] >= 0) gd[1] = ldq(gdr1, gdc1);
      __syncthreads();  // (the vectors below overwrite the packed G)
    }
    // VEC: zeros, then "reflector -1": z = column 0 below the diagonal
    for (int e = tid; e < 3 * 136; e += NT) vec[e] = aqc::cmk(0, 0);
    if (tid < NW) ktp[tid] = aqc::cmk(0, 0);
    if (tid == 0) tauS[-1] = aqc::cmk(0, 0);
    __syncthreads();
    if (cl0 == 0) {
#pragma unroll
      for (int i = 0; i < TR; ++i)
        if (rl0 + i > 0) vec[3 * (rl0 + i) + 2] = g[i][0];
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int a = s ? gdr1 : gdr0, b = s ? gdc1 : gdc0;
      if (dr[s] >= 0 && b == 0 && a > 0) vec[3 * a + 2] = gd[s];
    }
    lap(t_s1);
  } else {
    // ---- the trailing block from the scratch (lower triangle, row-major S x S) ----
    auto ld = [&](int r, int c) {  // global indices >= base
      const int a = r - base, b = c - base;
      return r >= c ? aqc::ldg(cx.scratch + (size_t)a * S + b) : aqc::cconj(aqc::ldg(cx.scratch + (size_t)b * S + a));
    };
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int jj = 0; jj < TC; ++jj) g[i][jj] = ld(rl0 + i, cl0 + jj);
    if (dr[0] >= 0) gd[0] = ld(gdr0, gdc0);
    if (dr[1] >= 0) gd[1] = ld(gdr1, gdc1);
  }
  __syncthreads();
  lap(mode != 1 ? t_s1 : t_io);
  // ---- the columns ----
  for (int k = k0; k < k1; ++k) {
    const int kl = k - base;
    // reflector k - 1's a2 and s (every wave, uniform: LDS broadcasts)
    cplx a2, s;
    {
      const cplx kt = ktp_sum<NW>(ktp);
      a2 = aqc::cscale(aqc::cmul(tauS[k - 1], kt), -0.5);
      const cplx pk = vec[3 * k + 1];
      s = aqc::cmk(pk.x + 2.0 * a2.x, -pk.y);
      a2.x = uniform_d(a2.x);
      s.x = uniform_d(s.x);
      s.y = uniform_d(s.y);
    }
    if (kl <= wlast + 1) {  // (one extra column: a retiring wave writes its zero partials once)
      const double a2r2 = 2.0 * a2.x;
      // pass 1 (columns streamed): the rank-2 update of reflector k - 1 and the row products g x_c
      // (rows' v and w held; x_r is formed in pass 2, when they are dead -- held together with the
      // tile they spilled)
      cplx yr[TR];
      {
        cplx vr[TR], wr[TR];
#pragma unroll
        for (int i = 0; i < TR; ++i) {
          const int r = rl0 + i;
          const cplx v = vec[3 * r], p = vec[3 * r + 1];
          vr[i] = v;
          wr[i] = aqc::cmk(fma(a2r2, v.x, p.x), fma(a2r2, v.y, p.y));
          yr[i] = aqc::cmk(0, 0);
        }
#pragma unroll
        for (int jj = 0; jj < TC; ++jj) {
          const int c = cl0 + jj;
          const cplx vc = vec[3 * c], pc = vec[3 * c + 1], zc = vec[3 * c + 2];
          const cplx xq = aqc::cfma(aqc::cmk(-s.x, -s.y), vc, zc);
          const cplx xc = c > k ? xq : aqc::cmk(0, 0);
#pragma unroll
          for (int i = 0; i < TR; ++i) {
            // g -= v_r conj(p_c) + w_r conj(v_c)
            cplx t = g[i][jj];
            t.x = fma(-vr[i].x, pc.x, fma(-vr[i].y, pc.y, fma(-wr[i].x, vc.x, fma(-wr[i].y, vc.y, t.x))));
            t.y = fma(-vr[i].y, pc.x, fma(vr[i].x, pc.y, fma(-wr[i].y, vc.x, fma(wr[i].x, vc.y, t.y))));
            g[i][jj] = t;
            yr[i] = aqc::cfma(t, xc, yr[i]);
          }
          if (c == k + 1) {
#pragma unroll
            for (int i = 0; i < TR; ++i)
              if (rl0 + i >= k + 1) gk1b[rl0 + i] = g[i][jj];
          }
          if (jj >= TR && c == k) {  // (the odd diagonal block of a half tile)
#pragma unroll
            for (int i = 0; i < TR; ++i)
              if (rl0 + i == k) dS[k] = g[i][jj].x;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < TR; ++i) grid[o_row + i] = yr[i];
      // pass 2: the column products conj(g) x_r (the strictly lower part's upper mirror)
      {
        cplx xr[TR];
#pragma unroll
        for (int i = 0; i < TR; ++i) {
          const int r = rl0 + i;
          const cplx x = aqc::cfma(aqc::cmk(-s.x, -s.y), vec[3 * r], vec[3 * r + 2]);
          xr[i] = r > k ? x : aqc::cmk(0, 0);
        }
#pragma unroll
        for (int jj = 0; jj < TC; ++jj) {
          cplx yc = aqc::cmk(0, 0);
#pragma unroll
          for (int i = 0; i < TR; ++i) yc = aqc::cfmac(g[i][jj], xr[i], yc);
          if (jj < TR) grid[o_clo + jj] = yc;
          else grid[o_chi + jj - TR] = half ? aqc::cmk(0, 0) : yc;
        }
      }
      // the even diagonal blocks: one or two elements, row products summed over the TR lanes of a row
#pragma unroll
      for (int sl = 0; sl < 2; ++sl) {
        if (sl == 1 && wave != NW - 1) continue;  // (uniform: the second slot exists in the last wave only)
        const bool act = dr[sl] >= 0;
        const int rd = act ? (sl ? gdr1 : gdr0) : 128, cd = act ? (sl ? gdc1 : gdc0) : 128;
        const cplx v = vec[3 * rd], p = vec[3 * rd + 1];
        const cplx w = aqc::cmk(fma(a2r2, v.x, p.x), fma(a2r2, v.y, p.y));
        const cplx vc = vec[3 * cd], pc = vec[3 * cd + 1], zc = vec[3 * cd + 2];
        const cplx xq = aqc::cfma(aqc::cmk(-s.x, -s.y), vc, zc);
        const cplx xc = cd > k ? xq : aqc::cmk(0, 0);
        cplx t = gd[sl];
        t.x = fma(-v.x, pc.x, fma(-v.y, pc.y, fma(-w.x, vc.x, fma(-w.y, vc.y, t.x))));
        t.y = fma(-v.y, pc.x, fma(v.x, pc.y, fma(-w.y, vc.x, fma(w.x, vc.y, t.y))));
        gd[sl] = t;
        cplx pr = aqc::cmul(t, xc);
        pr.x = group_sum_n<TR>(pr.x);
        pr.y = group_sum_n<TR>(pr.y);
        if (act) {
          if (cd == k + 1 && rd >= k + 1) gk1b[rd] = t;
          if (rd == k && cd == k) dS[k] = t.x;
          if (cd % TR == 0) grid[o_d[sl]] = pr;  // the row's first lane
        }
      }
    }
    if (wave == 0) {
      // reflector k's zlarfg scalars: x = column k of G^(k) below the diagonal = z - s v (rows > k)
      if (AQC_S3_PRIO) __builtin_amdgcn_s_setprio(3);
      double xn2;
      {
        const cplx z0 = vec[3 * lane + 2], z1 = vec[3 * (lane + 64) + 2];
        const cplx v0 = vec[3 * lane], v1 = vec[3 * (lane + 64)];
        const cplx x0 = aqc::cfma(aqc::cmk(-s.x, -s.y), v0, z0), x1 = aqc::cfma(aqc::cmk(-s.x, -s.y), v1, z1);
        const double n0 = lane > k + 1 ? aqc::cnorm2(x0) : 0.0, n1 = lane + 64 > k + 1 ? aqc::cnorm2(x1) : 0.0;
        xn2 = wave_sum_dpp(n0 + n1);
      }
      const cplx alpha = aqc::cfma(aqc::cmk(-s.x, -s.y), vec[3 * (k + 1)], vec[3 * (k + 1) + 2]);
      const double x2 = fma(alpha.x, alpha.x, fma(alpha.y, alpha.y, xn2));
      double rs = __builtin_amdgcn_rsq(x2);
      rs = rs * fma(-0.5 * x2 * rs, rs, 1.5);
      rs = rs * fma(-0.5 * x2 * rs, rs, 1.5);
      const double nn = x2 * rs;
      const bool triv = xn2 == 0.0 && alpha.y == 0.0;  // H = I
      const double beta = triv ? alpha.x : (alpha.x >= 0.0 ? -nn : nn);
      const double ib = alpha.x >= 0.0 ? -rs : rs;  // 1 / beta
      const double drr = alpha.x - beta, di = alpha.y, id2 = rcp_nr(fma(drr, drr, di * di));
      const cplx tau = triv ? aqc::cmk(0, 0) : aqc::cmk((beta - alpha.x) * ib, -alpha.y * ib);
      const cplx scl = triv ? aqc::cmk(0, 0) : aqc::cmk(drr * id2, -di * id2);  // 1 / (alpha - beta)
      if (lane == 0) {
        tauS[k] = tau;
        eS[k] = beta;
        scal[0] = scl;
        scal[1] = aqc::cmul(tau, scl);
      }
      if (AQC_S3_PRIO) __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();  // A: partials, gk1b, reflector k's scalars
    lap(t_pa);
    {
      // rows of the stage: GPR threads each, a row's sum over its contribution list
      int t = tid;
      asm volatile("" : "+v"(t));
      const int rloc = t / GPR, h = t % GPR;
      const int Rr = rloc / TR, ir = rloc % TR, n = NB - (Rr >> 1);
      const lcplx* gl = grid + TR * tri_off<NB>(Rr) + ir;
      // (a fixed count of independent loads, clamped and masked: issued together instead of one
      // LDS round trip per contribution)
      constexpr int NO = (NB + GPR - 1) / GPR;
      cplx part[4] = {aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0)};
#pragma unroll
      for (int u = 0; u < NO; ++u) {
        const int o = h + GPR * u;
        const cplx v = gl[TR * (o < n ? o : n - 1)];
        if (o < n) part[u & 3] = aqc::cadd(part[u & 3], v);
      }
      cplx y = aqc::cadd(aqc::cadd(part[0], part[1]), aqc::cadd(part[2], part[3]));
      y.x = group_sum_n<GPR>(y.x);
      y.y = group_sum_n<GPR>(y.y);
      const int r = base + rloc;
      const double beta = eS[k];
      const cplx ts = scal[1], scl = scal[0];
      const cplx g1 = gk1b[r];
      cplx sum = y;
      sum.x = fma(-beta, g1.x, sum.x);  // x_{k+1} = alpha where reflector k has alpha - beta
      sum.y = fma(-beta, g1.y, sum.y);
      const bool rowact = r > k && r < C, below = r > k + 1 && r < C;
      cplx p = aqc::cmul(ts, sum);
      if (!rowact) p = aqc::cmk(0, 0);
      const cplx vo = vec[3 * r], zo = vec[3 * r + 2];
      cplx v = aqc::cmul(aqc::cfma(aqc::cmk(-s.x, -s.y), vo, zo), scl);
      if (!below) v = aqc::cmk(r == k + 1 ? 1.0 : 0.0, 0.0);
      const cplx z = below ? aqc::csub(g1, p) : aqc::cmk(0, 0);
      const bool own = h == 0;
      if (own) {
        vec[3 * r] = v;
        vec[3 * r + 1] = p;
        vec[3 * r + 2] = z;
        if (rowact) aqc::stg(cx.hh + (size_t)k * (2 * C - k - 1) / 2 + (r - k - 1), v);
      }
      const double px = own ? fma(p.x, v.x, p.y * v.y) : 0.0, py = own ? fma(p.x, v.y, -p.y * v.x) : 0.0;
      const double ktx = wave_sum_dpp(px), kty = wave_sum_dpp(py);
      if (lane == 0) ktp[wave] = aqc::cmk(ktx, kty);
    }
    __syncthreads();  // B: reflector k's p, v, z and p^H v
    lap(t_pb);
  }
  if (k1 < C - 1) {
    // ---- repack: the next stage's trailing block (rows / columns >= nb) to the scratch ----
    const int nb = base + S / 2, SN = S / 2;
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int jj = 0; jj < TC; ++jj) {
        const int r = rl0 + i, c = cl0 + jj;
        if (c >= nb && r >= c) aqc::stg(cx.scratch + (size_t)(r - nb) * SN + (c - nb), g[i][jj]);
      }
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int r = sl ? gdr1 : gdr0, c = sl ? gdc1 : gdc0;
      if (dr[sl] >= 0 && c >= nb && r >= c) aqc::stg(cx.scratch + (size_t)(r - nb) * SN + (c - nb), gd[sl]);
    }
    __syncthreads();
  } else {
    // d_{C-1}: reflector C - 2's update of the last diagonal entry, by its owner
    const int kk = C - 1;
    cplx a2;
    {
      const cplx kt = ktp_sum<NW>(ktp);
      a2 = aqc::cscale(aqc::cmul(tauS[kk - 1], kt), -0.5);
    }
    const cplx v = vec[3 * kk], p = vec[3 * kk + 1];
    const cplx w = aqc::cfma(a2, v, p);
    const double upd = 2.0 * (v.x * w.x + v.y * w.y);  // Re(v conj(w) + w conj(v))
#pragma unroll
    for (int i = 0; i < TR; ++i)
#pragma unroll
      for (int jj = TR; jj < TC; ++jj)
        if (rl0 + i == kk && cl0 + jj == kk) dS[kk] = g[i][jj].x - upd;
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      const int r = sl ? gdr1 : gdr0, c = sl ? gdc1 : gdc0;
      if (dr[sl] >= 0 && r == kk && c == kk) dS[kk] = gd[sl].x - upd;
    }
    __syncthreads();
  }
  lap(t_io);
  if (tid == 0) {
    atomicAdd(&g_gram_ticks[6], t_pa);
    atomicAdd(&g_gram_ticks[7], t_pb);
    atomicAdd(&g_gram_ticks[9], t_s1);
    atomicAdd(&g_gram_ticks[10], t_io);
  }
}

// Gram-path SVD of one theta' on 256 threads: the contract of gram_svd_body (work columns =
// right singular vectors x sigma, sig, j.flags[2]); false when it declines (nothing written
// beyond scratch: the caller reruns the update on the 1024-thread chain).
__device__ __noinline__ bool gram256_body(const TwoSiteJob& j) {
  extern __shared__ double2 xbuf[];
  // (uniform values in SGPRs: dims are read through a generic pointer)
  const int chl = __builtin_amdgcn_readfirstlane(j.dims[0]), chr = __builtin_amdgcn_readfirstlane(j.dims[2]);
  const int M = 2 * chl, N = 2 * chr;
  const bool tr = M < N;
  const int L = tr ? N : M, C = tr ? M : N;
  int K = C;
  const int mx = __builtin_amdgcn_readfirstlane(j.max_chi);
  if (mx > 0 && mx < K) K = mx;
  if (K > kGramMaxK || C < 4 || C > 128 || L > 128 || __builtin_amdgcn_readfirstlane(j.cap) != 64) return false;
  const int tid = fresh_tid(), lane = tid & 63, wave = tid >> 6;
  unsigned long long t_last = tid == 0 ? __builtin_amdgcn_s_memtime() : 0ull;
  auto tick = [&](int ph) {
    if (tid == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      atomicAdd(&g_gram_ticks[ph], t - t_last);
      t_last = t;
    }
  };
  lcplx* lb = (lcplx*)xbuf;
  asm volatile("" : "+s"(lb));
  ldbl* s_d = (ldbl*)(lb + kD);
  ldbl* s_e = (ldbl*)(lb + kE);
  ldbl* s_e2 = (ldbl*)(lb + kE2);
  ldbl2* s_de = (ldbl2*)(lb + kDE);
  ldbl* s_lam = (ldbl*)(lb + kLam);
  ldbl* s_sig2 = (ldbl*)(lb + kSig2);
  lcplx* s_tau = lb + kTau + 1;
  ldbl* misc = (ldbl*)(lb + kMisc);  // lo, hi, tn
  // ---- S1 + S3 ----
  S3Ctx cx;
  cx.C = C;
  cx.hh = uniform_ptr(j.work);
  cx.scratch = uniform_ptr(j.work + kScratch);
  cx.th = j.theta;
  cx.M = M;
  cx.L = L;
  cx.tr = tr;
  const int kend = C - 1;
  s3_stage<4, 256>(cx, 0, kend < 64 ? kend : 64, 0);
  if (kend > 64) s3_stage<2, 256>(cx, 64, kend < 96 ? kend : 96, 1);
  if (kend > 96) s3_stage<1, 256>(cx, 96, kend, 1);
  tick(1);
  // ---- S4: top-K eigenvalues of T by multisection (as gram_svd_body) ----
  if (wave == 0) {
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
      misc[0] = lo - 1e-12 * span;
      misc[1] = hi + 1e-12 * span;
      misc[2] = tn;
    }
    const double itn = 1.0 / fmax(tn, 1e-300);
    for (int i = lane; i < C; i += 64) {
      const double2 de = s_de[i];
      s_de[i] = make_double2(de.x * itn, de.y * itn * itn);
    }
  }
  __syncthreads();
  const double s_lo = misc[0], s_hi = misc[1], s_tn = misc[2];
  {
    constexpr int kG = 4, kFirst = 256, kRounds = 12;
    const int eid = tid / kG, sub = tid % kG;
    const int a = C - 1 - eid;
    lint* cntb = (lint*)lb;
    const double lo0 = s_lo, span0 = s_hi - s_lo;
    const double itn = 1.0 / fmax(s_tn, 1e-300);
    constexpr double kInvF = 1.0 / (kFirst + 1), kInvG = 1.0 / (kG + 1);
    const double2* de = (const double2*)s_de;
    cntb[tid] = sturm_count_poly(de, C, (lo0 + span0 * (double)(tid + 1) * kInvF) * itn);
    __syncthreads();
    double lo, hi;
    {
      int l = 0, h = kFirst;
      while (l < h) {
        const int m = (l + h) >> 1;
        if (cntb[m] >= a + 1) h = m;
        else l = m + 1;
      }
      lo = l > 0 ? lo0 + span0 * (double)l * kInvF : s_lo;
      hi = l < kFirst ? lo0 + span0 * (double)(l + 1) * kInvF : s_hi;
    }
    for (int round = 0; round < kRounds; ++round) {
      const double x = lo + (hi - lo) * (double)(sub + 1) * kInvG;
      const int cnt = sturm_count_poly(de, C, x * itn);
      const unsigned long long bal = __ballot(cnt >= a + 1);
      const unsigned int gm = (unsigned int)(bal >> (lane & ~(kG - 1))) & ((1u << kG) - 1u);
      const int f = gm ? __builtin_ctz(gm) : kG;
      const double nhi = f < kG ? lo + (hi - lo) * (double)(f + 1) * kInvG : hi;
      const double nlo = f > 0 ? lo + (hi - lo) * (double)f * kInvG : lo;
      lo = nlo;
      hi = nhi;
    }
    if (eid < K && sub == 0) s_lam[eid] = 0.5 * (lo + hi);
  }
  __syncthreads();
  tick(2);
  if (!(s_lam[0] > 0.0) || !(s_lam[K - 1] > kGramRelFloor * s_lam[0])) return false;  // uniform
  // ---- S5: inverse iteration in two batches of 32 vectors (z and 1 / D of a batch: 64 KB of
  // LDS), each batch's vectors to the global scratch; then all of Z back into the LDS ----
  double* zs = (double*)(j.work + kScratch);  // zs[row * 64 + i]
  for (int bt = 0; bt < 2; ++bt) {
    ldbl* zb = (ldbl*)lb;             // zb[row * 32 + i]
    ldbl* Db = zb + 128 * 32;         // 1 / D_row of vector i
    const int i = lane, vi = 32 * bt + lane;
    if (wave == 0 && lane < 32 && vi < K) {
      const double lam = s_lam[vi];
      for (int row = 0; row < C; ++row) {
        unsigned int hsh = (unsigned int)(row * 2654435761u) ^ (unsigned int)((vi + 1) * 40503u);
        hsh ^= hsh >> 13;
        hsh *= 0x5bd1e995u;
        hsh ^= hsh >> 15;
        zb[row * 32 + i] = (double)(hsh & 0xFFFFFu) * (2.0 / 1048576.0) - 1.0;
      }
      constexpr int U = 8;
      const double itn = 1.0 / fmax(s_tn, 1e-300), lamn = lam * itn;
      double p0 = 0.0, p1 = 1.0;
      auto fac_row = [&](int row, double d, double e2) {
        const double dmx = fma(d, itn, -lamn), t = (e2 * itn * itn) * p0;
        const double lim = 2.220446049250313e-16 * fabs(p1);
        double p = fma(dmx, p1, -t);
        p = fabs(p) < lim ? copysign(lim, p) : p;
        Db[row * 32 + i] = p1 * rcp_nr(p) * itn;
        p0 = p1;
        p1 = p;
      };
      {
        int r0 = 0;
        for (; r0 + U <= C; r0 += U) {
          double dd[U], ee[U];
#pragma unroll
          for (int u = 0; u < U; ++u) dd[u] = s_d[r0 + u], ee[u] = s_e2[max(r0 + u - 1, 0)];
#pragma unroll
          for (int u = 0; u < U; ++u) fac_row(r0 + u, dd[u], ee[u]);
          const int ex = max(__builtin_amdgcn_frexp_exp(p0), __builtin_amdgcn_frexp_exp(p1));
          p0 = __builtin_amdgcn_ldexp(p0, -ex);
          p1 = __builtin_amdgcn_ldexp(p1, -ex);
        }
        for (; r0 < C; ++r0) fac_row(r0, s_d[r0], s_e2[max(r0 - 1, 0)]);
      }
      double sc = 1.0;
      for (int it = 0; it < AQC_S5_ITERS; ++it) {
        double yp = 0.0;
        auto fwd_row = [&](int row, double z, double e, double dp) {
          const double y = fma(-e * dp, yp, z * sc);
          zb[row * 32 + i] = y;
          yp = y;
        };
        int r0 = 0;
        for (; r0 + U <= C; r0 += U) {
          double zz[U], ee[U], dp[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int rm = max(r0 + u - 1, 0);
            zz[u] = zb[(r0 + u) * 32 + i], ee[u] = s_e[rm], dp[u] = Db[rm * 32 + i];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) fwd_row(r0 + u, zz[u], ee[u], dp[u]);
        }
        for (; r0 < C; ++r0) {
          const int rm = max(r0 - 1, 0);
          fwd_row(r0, zb[r0 * 32 + i], s_e[rm], Db[rm * 32 + i]);
        }
        double zn = 0.0, n2 = 0.0;
        auto bwd_row = [&](int row, double y, double e, double d) {
          zn = fma(-e * d, zn, y * d);
          zb[row * 32 + i] = zn;
          n2 = fma(zn, zn, n2);
        };
        int r1 = C - 1;
        for (; r1 - U + 1 >= 0; r1 -= U) {
          double yy[U], ee[U], dd[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int row = r1 - u;
            yy[u] = zb[row * 32 + i], ee[u] = s_e[min(row, C - 2)], dd[u] = Db[row * 32 + i];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) bwd_row(r1 - u, yy[u], ee[u], dd[u]);
        }
        for (; r1 >= 0; --r1) bwd_row(r1, zb[r1 * 32 + i], s_e[min(r1, C - 2)], Db[r1 * 32 + i]);
        const double rs = __builtin_amdgcn_rsq(n2);
        sc = rs * fma(-0.5 * n2 * rs, rs, 1.5);
      }
      for (int row = 0; row < C; ++row) aqc::stg(zs + (size_t)row * 64 + vi, zb[row * 32 + i] * sc);
    }
  }
  __syncthreads();
  ldbl* zb = (ldbl*)lb;  // zb[row * 64 + i], all K vectors
  for (int e = tid; e < 128 * 64; e += 256) {
    const int row = e >> 6, i = e & 63;
    zb[e] = (row < C && i < K) ? aqc::ldg(zs + e) : 0.0;
  }
  __syncthreads();
  if (wave == 0) {  // Gram-Schmidt inside clusters
    const double ortol = 1e-7 * s_tn;
    int start = 0;
    for (int i = 1; i < K; ++i) {
      if (s_lam[i - 1] - s_lam[i] >= ortol) {
        start = i;
        continue;
      }
      for (int jj = start; jj < i; ++jj) {
        double dp = 0.0;
        for (int row = lane; row < C; row += 64) dp = fma(zb[row * 64 + i], zb[row * 64 + jj], dp);
        dp = wave_sum_d(dp);
        for (int row = lane; row < C; row += 64) zb[row * 64 + i] = fma(-dp, zb[row * 64 + jj], zb[row * 64 + i]);
      }
      double n2 = 0.0;
      for (int row = lane; row < C; row += 64) n2 = fma(zb[row * 64 + i], zb[row * 64 + i], n2);
      n2 = wave_sum_d(n2);
      const double sc = 1.0 / sqrt(n2);
      for (int row = lane; row < C; row += 64) zb[row * 64 + i] *= sc;
    }
  }
  __syncthreads();
  if (tid < K) {  // sigma^2 = z^T T z
    const int i = tid;
    double s2a = 0.0, s2b = 0.0;
    for (int r0 = 0; r0 < C; ++r0) {
      const double z = zb[r0 * 64 + i];
      s2a = fma(s_d[r0] * z, z, s2a);
      if (r0 < C - 1) s2b = fma(2.0 * s_e[r0] * z, zb[(r0 + 1) * 64 + i], s2b);
    }
    const double s2 = s2a + s2b;
    s_sig2[i] = s2 > 0.0 ? s2 : 0.0;
  }
  __syncthreads();
  tick(3);
  // ---- S6: V = Q Z on the matrix cores, blocks of 16 reflectors in compact WY form.  Wave w owns
  // the 16 columns 16 w .. 16 w + 15 of V whole (8 row tiles in the accumulator layout: lane l
  // column l & 15, rows 16 t + (l >> 4) + 4 q), so Y^H V needs no cross-wave sums; S = Y^H Y from
  // four 32-row partials, T by zlarft in wave 0, W2 = T (Y^H V) per wave in its own LDS slice. ----
  cplx* hh = uniform_ptr(j.work);
  const int wv = __builtin_amdgcn_readfirstlane(wave);  // (uniform: an SGPR)
  const int li = lane & 15, lk = lane >> 4, nt = wave;
  aqc::d4_t vre[8], vim[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = 16 * t + lk + 4 * q, col = 16 * nt + li;
      vre[t][q] = zb[row * 64 + col];  // (zero for row >= C or col >= K: filled so above)
      vim[t][q] = 0.0;
    }
  }
  // LDS: Y [128][16] (column swizzled by row & 15), four partials of S (then T [16][17]), four
  // waves' Y^H V / W2 slices, S [16][16] over d, e (dead after S5; s_lam, s_sig2, s_tau live on)
  lcplx* Yl = lb;
  lcplx* Sp = lb + 2048;
  lcplx* Wl = lb + 3072;
  lcplx* Ss = lb + kD;
  static_assert(kD + 256 <= kLam, "S6's S overlaps the eigenvalues");
  auto fetch_y = [&](int kb0, int nb, cplx (&y)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u, row = e >> 4, i = e & 15, k = kb0 + i;
      y[u] = (i < nb && row > k && row < C) ? aqc::ldg(hh + (size_t)k * (2 * C - k - 1) / 2 + (row - k - 1))
                                            : aqc::cmk(0, 0);
    }
  };
  __syncthreads();  // V's initial values read from zb: the LDS is free
  lcplx* Tl = Sp;   // [16][17] after wave 0 summed the partials
  for (int k1 = C - 1; k1 > 0; k1 -= 16) {
    const int kb0 = k1 > 16 ? k1 - 16 : 0, nb = k1 - kb0;
    {
      cplx ynx[8];
      fetch_y(kb0, nb, ynx);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = tid + 256 * u, row = e >> 4, i = e & 15;
        Yl[row * 16 + (i ^ (row & 15))] = ynx[u];
      }
    }
    __syncthreads();  // B1: Y
    // W1 = Y^H V over all rows (rows <= kb0 of Y are zero); S partial over rows 32 w .. 32 w + 31
    aqc::d4_t wr = {0, 0, 0, 0}, wi = {0, 0, 0, 0}, sr = {0, 0, 0, 0}, si = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (16 * t + 15 > kb0) {  // uniform
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
          const int row = 16 * t + 4 * sb + lk;
          const cplx y = Yl[row * 16 + (li ^ (row & 15))];
          wr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, vre[t][sb], wr, 0, 0, 0);
          wr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, vim[t][sb], wr, 0, 0, 0);
          wi = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, vim[t][sb], wi, 0, 0, 0);
          wi = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, vre[t][sb], wi, 0, 0, 0);
          if ((t >> 1) == wv) {
            sr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, y.x, sr, 0, 0, 0);
            sr = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, y.y, sr, 0, 0, 0);
            si = __builtin_amdgcn_mfma_f64_16x16x4f64(y.x, y.y, si, 0, 0, 0);
            si = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, y.x, si, 0, 0, 0);
          }
        }
      }
    }
    // (S: the A operand conj(Y[row][m = li]) and the B operand Y[row][n = li] are the same lane value)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      Wl[wv * 256 + (lk + 4 * q) * 16 + li] = aqc::cmk(wr[q], wi[q]);
      Sp[wv * 256 + (lk + 4 * q) * 16 + li] = aqc::cmk(sr[q], si[q]);
    }
    __syncthreads();  // B2: partials
    if (wv == 0) {  // S, then T (zlarft: T[a][i] = -tau_i sum_{a <= b < i} T[a][b] S[b][i])
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int b = lk + 4 * q;
        cplx sv = Sp[b * 16 + li];
#pragma unroll
        for (int m = 1; m < 4; ++m) sv = aqc::cadd(sv, Sp[m * 256 + b * 16 + li]);
        Ss[b * 16 + li] = sv;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      {
        const int fl = fresh_lane(), a = fl >> 2, gq = fl & 3;
        cplx tq[4] = {aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0)};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const cplx tau = i < nb ? s_tau[kb0 + i] : aqc::cmk(0, 0);
          cplx acc = aqc::cmk(0, 0);
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            if (4 * m < i) {
              const int bb = gq + 4 * m;
              const cplx sv = bb < i ? Ss[bb * 16 + i] : aqc::cmk(0, 0);
              acc = aqc::cfma(tq[m], sv, acc);
            }
          }
          acc.x = aqc::row_sum4(acc.x);
          acc.y = aqc::row_sum4(acc.y);
          const cplx ti = aqc::cmul(tau, acc);
          const cplx val = a < i ? aqc::cmk(-ti.x, -ti.y) : (a == i ? tau : aqc::cmk(0, 0));
          if (gq == (i & 3)) tq[i >> 2] = val;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) Tl[a * 17 + gq + 4 * m] = tq[m];
      }
    }
    __syncthreads();  // B3: T
    {  // W2 = T W1 in this wave's slice: lane (q4, n) rows q4 + 4 m (all reads before the writes)
      const int fl = fresh_lane(), q4 = fl >> 4, n = fl & 15;
      lcplx* W = Wl + wv * 256;
      cplx o[4] = {aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0)};
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const cplx w1 = W[b * 16 + n];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int i = q4 + 4 * m;
          if (b >= 4 * m) {  // (T is upper triangular: rows i <= b)
            const cplx tv = i <= b ? Tl[i * 17 + b] : aqc::cmk(0, 0);
            o[m] = aqc::cfma(tv, w1, o[m]);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int m = 0; m < 4; ++m) W[(q4 + 4 * m) * 16 + n] = o[m];
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    {  // V -= Y W2: A[m = row][k = b] = Y[row][b], B[k = b][n] = W2[b][n]
      const int vl_ = fresh_lane(), vli = vl_ & 15, vlk = vl_ >> 4;
      const lcplx* W = Wl + wv * 256;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (16 * t + 15 > kb0) {
          const int row = 16 * t + vli;
#pragma unroll
          for (int sb = 0; sb < 4; ++sb) {
            const int b = 4 * sb + vlk;
            const cplx y = Yl[row * 16 + (b ^ (row & 15))];
            const cplx w = W[b * 16 + vli];
            vre[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.x, w.x, vre[t], 0, 0, 0);
            vre[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(y.y, w.y, vre[t], 0, 0, 0);
            vim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.x, w.y, vim[t], 0, 0, 0);
            vim[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(-y.y, w.x, vim[t], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // B4: Y, T, S are overwritten next block
  }
  tick(4);
  {  // the reflectors are dead: W = V Sigma over them
    const int col = 16 * nt + li;
    if (col < K) {
      const double sg = sqrt(s_sig2[col]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = 16 * t + lk + 4 * q;
          if (row < C) aqc::stg(j.work + (size_t)col * C + row, aqc::cmk(vre[t][q] * sg, vim[t][q] * sg));
        }
      }
    }
  }
  for (int c = tid; c < C; c += 256) aqc::stg(j.sig + c, c < K ? sqrt(s_sig2[c]) : 0.0);
  if (tid == 0) {
    atomicMax(&j.flags[2], 1);
    atomicAdd(&g_gram_stats[0], 1ull);
    atomicAdd(&g_gram_stats[1], 1ull);
  }
  tick(5);
  return true;
}

}  // namespace tri
