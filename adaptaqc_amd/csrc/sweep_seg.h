// Segmented candidate sweep for ONE state: the same T_ab as the chain kernels (k_sweep_chain*),
// reorganised so that its dependent depth is O(sqrt(n)) small GEMMs instead of O(n) streamed
// vector-matrix steps.  The chain form walks l_b = l_0 M_0 .. M_{b-1}, r_b and every first qubit's
// row vectors through up to n - 1 dependent products, each one workgroup streaming a chi x chi
// matrix from the Infinity Cache (~7.7 us at chi = 128): ~1.1 ms for one chi = 128, n = 50 sweep,
// with one CU busy.  Here the sites are cut into S segments of m ~ sqrt(n) sites:
//   1. prefix / suffix products inside every segment, P(i) = M_{s_q} .. M_i and Q(i) = M_i ..
//      M_{e_q - 1} (m - 1 steps of 2 S batched GEMMs), the segment products F_q = P(e_q - 1);
//   2. the environments at the segment boundaries, L_{q+1} = L_q F_q and R_q = F_{q+1} R_{q+1}
//      (S - 1 steps, written straight into lv[s_q] / rv[e_q]);
//   3. every site's environments in one step: l_a = L_q P(a - 1), r_{b+1} = Q(b + 1) R_q;
//   4. v0_a, w_b as the chain form (k_sweep_w);
//   5. pairs inside a segment: V_a^(t) = V_a^(t-1) M_{a+t} (t <= m - 2); pairs across segments:
//      U_a^(q_a+1) = v0_a Q(a + 1), U_a^(q+1) = U_a^(q) F_q, and y_b = w_b P(b - 1)^T -- all in the
//      same max(m - 2, S - 1) batched launches;
//   6. T_ab = V_a^(b-a-1) w_b^T or U_a^(q_b) y_b^T, one wave per pair.
// Every product is a batched complex GEMM on the FP64 matrix cores (k_cgemm16: one workgroup per
// 16 x 16 output tile), so each step spreads over hundreds of CUs.  ~2.5x the chain form's flops
// (n chi^3 products against n^2 chi^2 vector steps) for ~10x less depth: the single-sweep path,
// while batches of states keep the grouped chain kernel (k_sweep_chain8), whose throughput is
// higher.  Reference: gradients.py:81-122 (one sweep per layer, adapt_compiler.py:839-856).
//
// Included into grad.hip's anonymous namespace.
#pragma once

struct CgemmJob {
  const cplx* A;  // m x k, row-major (lda)
  const cplx* B;  // k x n, row-major (ldb); tb: B is stored n x k (B[j][kk] at j * ldb + kk)
  cplx* C;        // m x n, row-major (ldc)
  int m, n, k;
  int lda, ldb, ldc;
  int tb;
  int tiles_n;
};

// C = A B (complex) for a batch of jobs; one 256-thread workgroup per 16 x 16 output tile, grid
// (tiles, jobs).  The four waves split the contraction: wave w takes k steps w, w + 4, ... (4 k
// values each), issues all of its operand loads at once (8 steps in flight; the operands stream
// from L2 / the Infinity Cache), and the partial tiles meet in the LDS -- each launch is one
// latency-bound step of the single sweep's dependent chain.  v_mfma_f64_16x16x4f64 operand
// layout: A[m = lane & 15][k = lane >> 4], B[k = lane >> 4][n = lane & 15], D[m = (lane >> 4) +
// 4 q][n = lane & 15]; a complex product is four real ones into two accumulators.
__global__ __launch_bounds__(256) void k_cgemm16(const CgemmJob* __restrict__ jobs) {
  const CgemmJob& jb = jobs[blockIdx.y];
  const int tm = blockIdx.x / jb.tiles_n, tn = blockIdx.x % jb.tiles_n;
  const int i0 = tm * 16, j0 = tn * 16;
  if (i0 >= jb.m) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const int ia = i0 + li, jc = j0 + li;
  const bool arow = ia < jb.m, bcol = jc < jb.n;
  typedef double __attribute__((ext_vector_type(4))) d4;
  d4 cr = {0, 0, 0, 0}, ci = {0, 0, 0, 0};
  const int K = jb.k;
  constexpr int CS = 8;  // k steps per wave per pass
  for (int base = 0; base < K; base += 4 * 4 * CS) {
    cplx a[CS], b[CS];
#pragma unroll
    for (int s = 0; s < CS; ++s) {
      const int kk = base + 4 * (4 * s + wave) + lk;
      const bool kin = kk < K;
      a[s] = (arow && kin) ? aqc::ldg(jb.A + (size_t)ia * jb.lda + kk) : aqc::cmk(0, 0);
      b[s] = (bcol && kin) ? aqc::ldg(jb.B + (jb.tb ? (size_t)jc * jb.ldb + kk : (size_t)kk * jb.ldb + jc))
                           : aqc::cmk(0, 0);
    }
#pragma unroll
    for (int s = 0; s < CS; ++s) {
      cr = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s].x, b[s].x, cr, 0, 0, 0);
      ci = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s].x, b[s].y, ci, 0, 0, 0);
      cr = __builtin_amdgcn_mfma_f64_16x16x4f64(-a[s].y, b[s].y, cr, 0, 0, 0);
      ci = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s].y, b[s].x, ci, 0, 0, 0);
    }
  }
  __shared__ double part[3][8][64];
  if (wave > 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) part[wave - 1][q][lane] = cr[q], part[wave - 1][4 + q][lane] = ci[q];
  }
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double re = cr[q] + part[0][q][lane] + part[1][q][lane] + part[2][q][lane];
    const double im = ci[q] + part[0][4 + q][lane] + part[1][4 + q][lane] + part[2][4 + q][lane];
    const int row = i0 + lk + 4 * q;
    if (row < jb.m && bcol) jb.C[(size_t)row * jb.ldc + jc] = aqc::cmk(re, im);
  }
}

// T_ab[sa][sb] = sum_x X_p[sa][x] Y_p[sb][x] for pair p (a < b), X / Y two rows of cap complex;
// one wave per pair, four per workgroup.
__global__ __launch_bounds__(256) void k_seg_pairs(const cplx* const* __restrict__ X, const cplx* const* __restrict__ Y,
                                                   const int* __restrict__ pairs, int npairs, int n, int cap,
                                                   cplx* __restrict__ T) {
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (p >= npairs) return;
  const int c = pairs[2 * p], t = pairs[2 * p + 1];
  const int a = min(c, t), b = max(c, t);
  const cplx* x = X[p];
  const cplx* y = Y[p];
  cplx acc[4] = {aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0), aqc::cmk(0, 0)};
  for (int k = lane; k < cap; k += 64) {
    const cplx x0 = x[k], x1 = x[cap + k], y0 = y[k], y1 = y[cap + k];
    acc[0] = aqc::cfma(x0, y0, acc[0]);
    acc[1] = aqc::cfma(x0, y1, acc[1]);
    acc[2] = aqc::cfma(x1, y0, acc[2]);
    acc[3] = aqc::cfma(x1, y1, acc[3]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      acc[u].x += __shfl_xor(acc[u].x, off);
      acc[u].y += __shfl_xor(acc[u].y, off);
    }
  }
  if (lane < 4) T[((size_t)a * n + b) * 4 + lane] = acc[lane];
}

// Boundary vectors e_0 of lv[0] (L_0) and rv[n] (R_{S-1}) and the zero padding the pair
// products rely on (v0 / w beyond the bond dimensions).
__global__ void k_seg_init(cplx* lv0, cplx* rvn, cplx* w, cplx* v0, int cap, size_t wlen) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (size_t)cap) {
    lv0[t] = aqc::cmk(t == 0 ? 1.0 : 0.0, 0.0);
    rvn[t] = aqc::cmk(t == 0 ? 1.0 : 0.0, 0.0);
  }
  for (size_t e = t; e < wlen; e += (size_t)gridDim.x * blockDim.x) {
    w[e] = aqc::cmk(0, 0);
    v0[e] = aqc::cmk(0, 0);
  }
}

// Host plan and launches of the segmented sweep (steps 1-6 above) for one state whose M_i the
// caller's k_sweep_M has queued; T written for `pairs`; k_sweep_w launched here with `dstart`.
struct SegScratch {
  cplx* dev = nullptr;
  size_t bytes = 0;
  char* host = nullptr;
  size_t hbytes = 0;
  hipEvent_t done = nullptr;
  bool pending = false;
  // the last plan (its job / pointer tables stay on the device): reused while the state's buffers
  // and the pair list are the same -- the per-layer call repeats both
  std::vector<unsigned long long> key;
  std::vector<std::pair<size_t, size_t>> launches;
  std::vector<int> ltiles;
  size_t env_launches = 0, tbl_bytes = 0;
};

SegScratch g_seg_scratch[64];
void release_seg_scratch() {
  for (auto& s : g_seg_scratch) {
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.dev) (void)hipFree(s.dev);
    if (s.host) (void)hipHostFree(s.host);
    s = SegScratch();
  }
}
SegScratch& seg_scratch() {
  int dev = 0;
  hipGetDevice(&dev);
  aqc::on_finalize(release_seg_scratch);
  return g_seg_scratch[dev];
}

int run_segment_sweep(const SweepJob& hj, const SweepJob* djob, const int* pairs, const int* dpairs, int npairs,
                      const int* dstart, hipStream_t st) {
  const int n = hj.n, cap = hj.cap;
  const size_t cc = (size_t)cap * cap;
  int m = 1;
  while (m * m < n) ++m;  // segment length ~ sqrt(n)
  const int S = (n + m - 1) / m;
  auto seg = [&](int i) { return i / m; };
  auto s_of = [&](int q) { return q * m; };
  auto e_of = [&](int q) { return std::min(n, (q + 1) * m); };
  const int Tv = std::max(m - 2, 0);  // within-segment hop vectors per first qubit
  // device scratch: P and Q (n matrices each; P(s_q), Q(e_q - 1) alias M), V (n x Tv x 2 cap),
  // U (n x S x 2 cap), y (n x 2 cap), then the job tables
  const size_t oP = 0, oQ = oP + (size_t)n * cc, oV = oQ + (size_t)n * cc;
  const size_t oU = oV + (size_t)n * Tv * 2 * cap, oY = oU + (size_t)n * S * 2 * cap;
  const size_t oEnd = oY + (size_t)n * 2 * cap;  // complex units
  cplx* Mb = hj.M;
  auto Mi = [&](int i) { return Mb + (size_t)i * cc; };
  std::vector<CgemmJob> jobs;
  std::vector<std::pair<size_t, size_t>> launches;  // (first job, count)
  std::vector<int> ltiles;
  SegScratch& sc = seg_scratch();
  // (pointers into the device scratch are formed from its base after sizing; plan with offsets)
  const size_t table_off_bytes = oEnd * sizeof(cplx);
  // plan once with a null base to count, then with the real base
  auto plan = [&](cplx* base) {
    jobs.clear();
    launches.clear();
    ltiles.clear();
    auto Pp = [&](int i) -> const cplx* { return i == s_of(seg(i)) ? Mi(i) : base + oP + (size_t)i * cc; };
    auto Pw = [&](int i) { return base + oP + (size_t)i * cc; };
    auto Qp = [&](int i) -> const cplx* { return i == e_of(seg(i)) - 1 ? Mi(i) : base + oQ + (size_t)i * cc; };
    auto Qw = [&](int i) { return base + oQ + (size_t)i * cc; };
    auto Vp = [&](int a, int t) -> cplx* { return base + oV + ((size_t)a * Tv + (t - 1)) * 2 * cap; };
    auto Up = [&](int a, int q) -> cplx* { return base + oU + ((size_t)a * S + q) * 2 * cap; };
    auto Yp = [&](int b) -> cplx* { return base + oY + (size_t)b * 2 * cap; };
    auto add = [&](const cplx* A, const cplx* B, cplx* C, int mm, int nn, int kk, int lda, int ldb, int ldc,
                   int tb) {
      CgemmJob j;
      j.A = A, j.B = B, j.C = C, j.m = mm, j.n = nn, j.k = kk, j.lda = lda, j.ldb = ldb, j.ldc = ldc, j.tb = tb;
      j.tiles_n = (nn + 15) / 16;
      jobs.push_back(j);
    };
    auto close = [&](size_t first) {
      if (jobs.size() > first) {
        launches.push_back({first, jobs.size() - first});
        int tmax = 0;
        for (size_t k = first; k < jobs.size(); ++k)
          tmax = std::max(tmax, ((jobs[k].m + 15) / 16) * jobs[k].tiles_n);
        ltiles.push_back(tmax);
      }
    };
    // 1. prefix / suffix products inside the segments
    for (int t = 1; t < m; ++t) {
      const size_t f = jobs.size();
      for (int q = 0; q < S; ++q) {
        const int s = s_of(q), e = e_of(q);
        if (s + t < e) add(Pp(s + t - 1), Mi(s + t), Pw(s + t), cap, cap, cap, cap, cap, cap, 0);
        if (e - 1 - t >= s) add(Mi(e - 1 - t), Qp(e - t), Qw(e - 1 - t), cap, cap, cap, cap, cap, cap, 0);
      }
      close(f);
    }
    // 2. boundary environments: L_{q+1} = L_q F_q (row), R_{q} = F_{q+1} R_{q+1} (column)
    for (int k = 0; k + 1 < S; ++k) {
      const size_t f = jobs.size();
      add(hj.lv + (size_t)s_of(k) * cap, Pp(e_of(k) - 1), hj.lv + (size_t)s_of(k + 1) * cap, 1, cap, cap, cap, cap,
          cap, 0);
      const int qr = S - 2 - k;  // R_qr = F_{qr+1} R_{qr+1}
      add(Pp(e_of(qr + 1) - 1), hj.rv + (size_t)e_of(qr + 1) * cap, hj.rv + (size_t)e_of(qr) * cap, cap, 1, cap, cap,
          1, 1, 0);
      close(f);
    }
    // 3. every site's environments
    {
      const size_t f = jobs.size();
      for (int a = 0; a < n; ++a) {
        const int q = seg(a), s = s_of(q), e = e_of(q);
        if (a > s) add(hj.lv + (size_t)s * cap, Pp(a - 1), hj.lv + (size_t)a * cap, 1, cap, cap, cap, cap, cap, 0);
        if (a + 1 < e) add(Qp(a + 1), hj.rv + (size_t)e * cap, hj.rv + (size_t)(a + 1) * cap, cap, 1, cap, cap, 1, 1, 0);
      }
      close(f);
    }
    const size_t env_launches = launches.size();
    // 5. hops (after k_sweep_w): within-segment V, across-segment U, and y
    const int H = std::max(Tv, S - 1);
    for (int c = 0; c < H; ++c) {
      const size_t f = jobs.size();
      for (int a = 0; a < n - 1; ++a) {
        const int q = seg(a), e = e_of(q);
        const cplx* v0a = hj.v0 + (size_t)a * 2 * cap;
        const int t = c + 1;  // within: V_a^(t) for b = a + t + 1 inside the segment
        if (t <= Tv && a + t + 1 <= e - 1)
          add(t == 1 ? v0a : Vp(a, t - 1), Mi(a + t), Vp(a, t), 2, cap, cap, cap, cap, cap, 0);
        if (q + 1 + c <= S - 1) {  // across: U_a^(q+1+c)
          if (c == 0) {
            if (a + 1 < e) add(v0a, Qp(a + 1), Up(a, q + 1), 2, cap, cap, cap, cap, cap, 0);
          } else {
            const cplx* src = (c == 1 && a + 1 == e) ? v0a : Up(a, q + c);
            add(src, Pp(e_of(q + c) - 1), Up(a, q + 1 + c), 2, cap, cap, cap, cap, cap, 0);
          }
        }
      }
      if (c == 0)
        for (int b = 1; b < n; ++b)
          if (seg(b) > 0 && b > s_of(seg(b)))
            add(hj.w + (size_t)b * 2 * cap, Pp(b - 1), Yp(b), 2, cap, cap, cap, cap, cap, 1);
      close(f);
    }
    return env_launches;
  };
  // the plan's identity: shapes, the state's buffers, the pair list
  std::vector<unsigned long long> key = {(unsigned long long)n, (unsigned long long)cap, (unsigned long long)npairs,
                                         (unsigned long long)(uintptr_t)hj.M, (unsigned long long)(uintptr_t)hj.lv,
                                         (unsigned long long)(uintptr_t)hj.rv, (unsigned long long)(uintptr_t)hj.w,
                                         (unsigned long long)(uintptr_t)hj.v0, (unsigned long long)(uintptr_t)hj.T};
  {
    unsigned long long h = 1469598103934665603ull;
    for (int i = 0; i < 2 * npairs; ++i) h = (h ^ (unsigned long long)(unsigned)pairs[i]) * 1099511628211ull;
    key.push_back(h);
  }
  const bool reuse = sc.dev && key == sc.key;
  if (reuse) {
    launches = sc.launches;
    ltiles = sc.ltiles;
  }
  // size the scratch: data + job table + pair pointer tables
  size_t env_launches = reuse ? sc.env_launches : plan(nullptr);
  const size_t tbl_bytes = reuse ? sc.tbl_bytes : jobs.size() * sizeof(CgemmJob);
  const size_t ptr_bytes = 2 * (size_t)npairs * sizeof(cplx*);
  const size_t need = table_off_bytes + tbl_bytes + ptr_bytes + 256;
  if (sc.pending && !reuse) {  // the last call's host staging may still be in flight
    AQC_HIP_CHECK(hipEventSynchronize(sc.done));
    sc.pending = false;
  }
  if (need > sc.bytes) {
    if (sc.dev) hipFree(sc.dev);
    sc.dev = nullptr;
    sc.bytes = 0;
    sc.key.clear();
    AQC_HIP_CHECK(hipMalloc(&sc.dev, need));
    sc.bytes = need;
  }
  const size_t hneed = tbl_bytes + ptr_bytes + 256;
  if (hneed > sc.hbytes) {
    if (sc.host) hipHostFree(sc.host);
    sc.host = nullptr;
    sc.hbytes = 0;
    AQC_HIP_CHECK(hipHostMalloc((void**)&sc.host, hneed, hipHostMallocDefault));
    sc.hbytes = hneed;
  }
  if (!sc.done) AQC_HIP_CHECK(hipEventCreateWithFlags(&sc.done, hipEventDisableTiming));
  cplx* base = sc.dev;
  char* dtab = reinterpret_cast<char*>(base) + table_off_bytes;
  if (!reuse) {
  env_launches = plan(base);
  // pair operand pointers (step 6)
  auto Vp = [&](int a, int t) -> const cplx* { return base + oV + ((size_t)a * Tv + (t - 1)) * 2 * cap; };
  auto Up = [&](int a, int q) -> const cplx* { return base + oU + ((size_t)a * S + q) * 2 * cap; };
  auto Yp = [&](int b) -> const cplx* { return base + oY + (size_t)b * 2 * cap; };
  const cplx** hx = reinterpret_cast<const cplx**>(sc.host + tbl_bytes);
  const cplx** hy = hx + npairs;
  for (int p = 0; p < npairs; ++p) {
    const int a = std::min(pairs[2 * p], pairs[2 * p + 1]), b = std::max(pairs[2 * p], pairs[2 * p + 1]);
    const int qa = seg(a), qb = seg(b);
    const cplx* v0a = hj.v0 + (size_t)a * 2 * cap;
    const cplx* wb = hj.w + (size_t)b * 2 * cap;
    if (qa == qb) {
      const int t = b - a - 1;
      hx[p] = t == 0 ? v0a : Vp(a, t);
      hy[p] = wb;
    } else {
      hx[p] = (qb == qa + 1 && a + 1 == e_of(qa)) ? v0a : Up(a, qb);
      hy[p] = b == s_of(qb) ? wb : Yp(b);
    }
  }
  std::memcpy(sc.host, jobs.data(), tbl_bytes);
  AQC_HIP_CHECK(hipMemcpyAsync(dtab, sc.host, tbl_bytes + ptr_bytes, hipMemcpyHostToDevice, st));
  sc.key = key;
  sc.launches = launches;
  sc.ltiles = ltiles;
  sc.env_launches = env_launches;
  sc.tbl_bytes = tbl_bytes;
  }
  const CgemmJob* djobs = reinterpret_cast<const CgemmJob*>(dtab);
  const cplx* const* dx = reinterpret_cast<const cplx* const*>(dtab + tbl_bytes);
  const cplx* const* dy = dx + npairs;
  // boundary vectors and zero padding, then steps 1-3
  const size_t wlen = (size_t)2 * n * cap;
  hipLaunchKernelGGL(k_seg_init, dim3(64), dim3(256), 0, st, hj.lv, hj.rv + (size_t)n * cap, hj.w, hj.v0, cap, wlen);
  AQC_CHECK_LAUNCH();
  for (size_t l = 0; l < env_launches; ++l) {
    hipLaunchKernelGGL(k_cgemm16, dim3(ltiles[l], (unsigned)launches[l].second), dim3(256), 0, st,
                       djobs + launches[l].first);
    AQC_CHECK_LAUNCH();
  }
  // 4. v0, w
  hipLaunchKernelGGL(k_sweep_w, dim3(n, 1, 8), dim3(kT), 0, st, djob, dstart);
  AQC_CHECK_LAUNCH();
  // 5. hops
  for (size_t l = env_launches; l < launches.size(); ++l) {
    hipLaunchKernelGGL(k_cgemm16, dim3(ltiles[l], (unsigned)launches[l].second), dim3(256), 0, st,
                       djobs + launches[l].first);
    AQC_CHECK_LAUNCH();
  }
  // 6. pair values
  if (npairs) {
    hipLaunchKernelGGL(k_seg_pairs, dim3((npairs + 3) / 4), dim3(256), 0, st, dx, dy, dpairs, npairs, n, cap, hj.T);
    AQC_CHECK_LAUNCH();
  }
  AQC_HIP_CHECK(hipEventRecord(sc.done, st));
  sc.pending = true;
  return AQC_OK;
}
