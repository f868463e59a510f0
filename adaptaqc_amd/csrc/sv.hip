// Statevector engine: replaces Aer's statevector_simulator as driven by
// adaptaqc/backends/aer_sv_backend.py:37-59.
//
// Layout: 2^n interleaved complex128 amplitudes, little-endian (qubit q = bit q of the index).
// Gates are fused on the host into "segments": a run of gates (reordered only across gates on
// disjoint qubits) whose qubits fit in a K-bit tile.  One launch per segment: each workgroup
// gathers the 2^K amplitudes of one tile (tile bits = segment qubits padded with the lowest
// free bits, so global reads are contiguous runs), applies every gate of the segment in LDS,
// and writes the tile back.  A segment therefore costs one HBM/MALL pass (32 * 2^n bytes)
// regardless of how many gates it holds.
#include <algorithm>
#include <array>
#include <cstring>

#include "aqc_internal.h"

using aqc::cplx;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxTileBits = 12;
constexpr int kGateChunk = 48;  // gates staged in LDS per chunk (48 x 272 B = 12.75 KB)

struct SegGate {
  int32_t nq;  // 1 or 2
  int32_t t0;  // local bit of q0
  int32_t t1;  // local bit of q1 (2q only)
  int32_t pad;
  cplx m[16];
};

struct SegHeader {
  int32_t tilebits[kMaxTileBits];  // ascending global bit positions
  int32_t gate_off;                // index into gate array
  int32_t ngates;
  int32_t pad[2];
};

__device__ __forceinline__ uint64_t insert_zero(uint64_t v, int b) {
  uint64_t lo = v & ((1ull << b) - 1ull);
  return ((v >> b) << (b + 1)) | lo;
}

template <int K>
__global__ __launch_bounds__(kThreads) void k_sv_segment(cplx* __restrict__ state, int n,
                                                         const SegHeader* __restrict__ hdr,
                                                         const SegGate* __restrict__ gates) {
  __shared__ cplx tile[1 << K];
  constexpr int kPer = (1 << K) / kThreads > 0 ? (1 << K) / kThreads : 1;
  const int tid = threadIdx.x;
  int tb[K];
#pragma unroll
  for (int j = 0; j < K; ++j) tb[j] = hdr->tilebits[j];
  // base index: blockIdx bits scattered into the non-tile positions
  uint64_t base = blockIdx.x;
#pragma unroll
  for (int j = 0; j < K; ++j) base = insert_zero(base, tb[j]);
  uint64_t gidx[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    int x = tid + r * kThreads;
    uint64_t g = base;
#pragma unroll
    for (int j = 0; j < K; ++j) g |= (uint64_t)((x >> j) & 1) << tb[j];
    gidx[r] = g;
    if (x < (1 << K)) tile[x] = state[g];
  }
  const int ng = hdr->ngates;
  const SegGate* gp = gates + hdr->gate_off;
  // The segment's gates are staged into LDS in chunks with vector loads, so a gate costs one
  // barrier and LDS broadcast reads: read through the scalar cache, each gate was a chain of six
  // dependent s_load round trips (kind, bits, four matrix rows) standing between two barriers.
  __shared__ SegGate gl[kGateChunk];
  for (int c0 = 0; c0 < ng; c0 += kGateChunk) {
    const int nc = min(kGateChunk, ng - c0);
    __syncthreads();  // the previous chunk's last gate has been applied
    constexpr int kWords = (int)(sizeof(SegGate) / sizeof(double2));
    for (int w = tid; w < nc * kWords; w += kThreads)
      reinterpret_cast<double2*>(gl)[w] = reinterpret_cast<const double2*>(gp + c0)[w];
    for (int gi = 0; gi < nc; ++gi) {
      const SegGate& g_s = gl[gi];
      __syncthreads();
      if (g_s.nq == 1) {
        const int t = g_s.t0;
        const cplx m00 = g_s.m[0], m01 = g_s.m[1], m10 = g_s.m[2], m11 = g_s.m[3];
        for (int p = tid; p < (1 << (K - 1)); p += kThreads) {
          int i0 = (int)insert_zero((uint64_t)p, t);
          int i1 = i0 | (1 << t);
          cplx a0 = tile[i0], a1 = tile[i1];
          tile[i0] = aqc::cfma(m01, a1, aqc::cmul(m00, a0));
          tile[i1] = aqc::cfma(m11, a1, aqc::cmul(m10, a0));
        }
      } else if constexpr (K >= 2) {
        const int t0 = g_s.t0, t1 = g_s.t1;
        const int lo = t0 < t1 ? t0 : t1, hi = t0 < t1 ? t1 : t0;
        cplx m[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) m[e] = g_s.m[e];
        for (int p = tid; p < (1 << (K - 2)); p += kThreads) {
          int b = (int)insert_zero(insert_zero((uint64_t)p, lo), hi);
          int idx[4];
          cplx v[4];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            idx[s] = b | ((s & 1) << t0) | ((s >> 1) << t1);
            v[s] = tile[idx[s]];
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            cplx acc = aqc::cmul(m[4 * r], v[0]);
            acc = aqc::cfma(m[4 * r + 1], v[1], acc);
            acc = aqc::cfma(m[4 * r + 2], v[2], acc);
            acc = aqc::cfma(m[4 * r + 3], v[3], acc);
            tile[idx[r]] = acc;
          }
        }
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    int x = tid + r * kThreads;
    if (x < (1 << K)) state[gidx[r]] = tile[x];
  }
}

// Per-workgroup partial probabilities: out[wg * (n+1) + i] = sum |a|^2 over amplitudes of this
// workgroup with bit i set (i < n); out[wg*(n+1)+n] = total.
constexpr int kZChunk = 16;  // amplitudes per thread
__global__ __launch_bounds__(kThreads) void k_sv_zpartial(const cplx* __restrict__ state, int n,
                                                          double* __restrict__ out) {
  __shared__ double red[kThreads];
  const int tid = threadIdx.x;
  const uint64_t dim = 1ull << n;
  const uint64_t base = (uint64_t)blockIdx.x * (kThreads * kZChunk);
  double tot = 0.0;
  double pj[kZChunk];
#pragma unroll
  for (int j = 0; j < kZChunk; ++j) {
    uint64_t x = base + tid + (uint64_t)j * kThreads;
    double p = 0.0;
    if (x < dim) p = aqc::cnorm2(state[x]);
    pj[j] = p;
    tot += p;
  }
  // bits 8..11 vary with j (kThreads = 256 = 2^8)
  double hi4[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    double s = 0;
#pragma unroll
    for (int j = 0; j < kZChunk; ++j)
      if ((j >> b) & 1) s += pj[j];
    hi4[b] = s;
  }
  for (int i = 0; i <= n; ++i) {
    double c;
    if (i == n) {
      c = tot;
    } else if (i < 8) {
      c = ((tid >> i) & 1) ? tot : 0.0;
    } else if (i < 12) {
      c = hi4[i - 8];
    } else {
      c = ((base >> i) & 1ull) ? tot : 0.0;
    }
    red[tid] = c;
    __syncthreads();
    for (int s = kThreads / 2; s > 0; s >>= 1) {
      if (tid < s) red[tid] += red[tid + s];
      __syncthreads();
    }
    if (tid == 0) out[(uint64_t)blockIdx.x * (n + 1) + i] = red[0];
    __syncthreads();
  }
}

__global__ void k_sv_zfinal(const double* __restrict__ part, int nwg, int n, double* __restrict__ z) {
  const int i = threadIdx.x;
  if (i > n) return;
  double s = 0.0, t = 0.0;
  for (int w = 0; w < nwg; ++w) {
    s += part[(uint64_t)w * (n + 1) + i];
    t += part[(uint64_t)w * (n + 1) + n];
  }
  if (i < n) z[i] = t - 2.0 * s;  // p0 - p1 with p0 = total - p1
}

__global__ void k_sv_reset(cplx* state, uint64_t dim) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < dim; i += (uint64_t)gridDim.x * blockDim.x) state[i] = aqc::cmk(i == 0 ? 1.0 : 0.0, 0.0);
}

// ---- host-side segmentation -------------------------------------------------------------
struct HostSeg {
  std::vector<int> gates;  // indices into op list, in application order
  uint64_t qmask = 0;
};

std::vector<HostSeg> build_segments(const aqc_op_t* ops, int nops, int K, int n) {
  std::vector<HostSeg> segs;
  std::vector<char> done(nops, 0);
  int remaining = nops;
  int first = 0;
  while (remaining > 0) {
    while (first < nops && done[first]) ++first;
    HostSeg seg;
    uint64_t blocked = 0;
    for (int i = first; i < nops; ++i) {
      if (done[i]) continue;
      uint64_t gm = (1ull << ops[i].q0);
      if (ops[i].nq == 2) gm |= (1ull << ops[i].q1);
      if (gm & blocked) {
        blocked |= gm;
      } else {
        uint64_t u = seg.qmask | gm;
        if (__builtin_popcountll(u) <= K) {
          seg.qmask = u;
          seg.gates.push_back(i);
          done[i] = 1;
          --remaining;
        } else {
          blocked |= gm;
        }
      }
      if (__builtin_popcountll(blocked) >= n) break;
    }
    segs.push_back(std::move(seg));
  }
  return segs;
}

// ---- host-side gate fusion inside a segment -------------------------------------------------
// Every 1-qubit gate is multiplied into the last fused op on its qubit (1- or 2-qubit), or into
// the next 2-qubit gate on it when that gate comes first; consecutive 2-qubit gates on the same
// pair become one 4x4.  Valid because the merged ops are adjacent on their qubits (everything in
// between acts on other qubits and commutes).  Aer fuses too (fusion_enable at >= 14 qubits);
// here every tile pass saves one LDS sweep and one barrier per absorbed gate.  Brickwork: 3 ops
// per pair and layer become 1.
typedef std::array<cplx, 16> Mat4;

static Mat4 mat4_mul(const Mat4& a, const Mat4& b) {  // a b
  Mat4 c;
  for (int r = 0; r < 4; ++r)
    for (int k = 0; k < 4; ++k) {
      cplx acc = aqc::cmk(0, 0);
      for (int j = 0; j < 4; ++j) acc = aqc::cfma(a[4 * r + j], b[4 * j + k], acc);
      c[4 * r + k] = acc;
    }
  return c;
}

// 1-qubit u on bit `which` (0: the op's t0, 1: its t1) of a 4x4 (index 2 b1 + b0)
static Mat4 embed1(const cplx* u, int which) {
  Mat4 m;
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) {
      const int r0 = r & 1, r1 = r >> 1, c0 = c & 1, c1 = c >> 1;
      cplx v = aqc::cmk(0, 0);
      if (which == 0 && r1 == c1) v = u[2 * r0 + c0];
      if (which == 1 && r0 == c0) v = u[2 * r1 + c1];
      m[4 * r + c] = v;
    }
  return m;
}

static Mat4 swap_bits(const Mat4& a) {  // the same operator with t0 and t1 exchanged
  Mat4 m;
  auto sw = [](int x) { return ((x & 1) << 1) | (x >> 1); };
  for (int r = 0; r < 4; ++r)
    for (int c = 0; c < 4; ++c) m[4 * sw(r) + sw(c)] = a[4 * r + c];
  return m;
}

std::vector<SegGate> fuse_segment(const aqc_op_t* ops, const std::vector<int>& idx, const int* local_of) {
  struct F {
    int nq, t0, t1;
    Mat4 m;  // nq == 1: m[0..3] = 2x2
    bool dead = false;
  };
  std::vector<F> f;
  int last[64];
  for (int q = 0; q < 64; ++q) last[q] = -1;
  for (int gi : idx) {
    const aqc_op_t& o = ops[gi];
    cplx u[16];
    const int nel = o.nq == 1 ? 4 : 16;
    for (int e = 0; e < nel; ++e) u[e] = aqc::cmk(o.m[2 * e], o.m[2 * e + 1]);
    if (o.nq == 1) {
      const int q = local_of[o.q0];
      const int k = last[q];
      if (k >= 0 && f[k].nq == 1) {  // 2x2 product u * m
        Mat4 c = f[k].m;
        for (int r = 0; r < 2; ++r)
          for (int cc = 0; cc < 2; ++cc) c[2 * r + cc] = aqc::cfma(u[2 * r + 1], f[k].m[2 + cc], aqc::cmul(u[2 * r], f[k].m[cc]));
        f[k].m = c;
      } else if (k >= 0) {
        f[k].m = mat4_mul(embed1(u, f[k].t0 == q ? 0 : 1), f[k].m);
      } else {
        F n;
        n.nq = 1, n.t0 = q, n.t1 = 0;
        n.m = Mat4{};
        for (int e = 0; e < 4; ++e) n.m[e] = u[e];
        f.push_back(n);
        last[q] = (int)f.size() - 1;
      }
      continue;
    }
    const int a = local_of[o.q0], b = local_of[o.q1];
    Mat4 g;
    for (int e = 0; e < 16; ++e) g[e] = u[e];
    const int ka = last[a], kb = last[b];
    if (ka >= 0 && ka == kb && f[ka].nq == 2) {  // same pair again
      f[ka].m = mat4_mul(f[ka].t0 == a ? g : swap_bits(g), f[ka].m);
      continue;
    }
    // absorb pending single-qubit ops on a / b (their last op, nothing after them on that qubit)
    Mat4 m = g;
    if (ka >= 0 && f[ka].nq == 1) {
      m = mat4_mul(m, embed1(f[ka].m.data(), 0));
      f[ka].dead = true;
    }
    if (kb >= 0 && f[kb].nq == 1) {
      m = mat4_mul(m, embed1(f[kb].m.data(), 1));
      f[kb].dead = true;
    }
    F n;
    n.nq = 2, n.t0 = a, n.t1 = b, n.m = m;
    f.push_back(n);
    last[a] = last[b] = (int)f.size() - 1;
  }
  std::vector<SegGate> out;
  for (const F& x : f) {
    if (x.dead) continue;
    SegGate g;
    std::memset(&g, 0, sizeof(g));
    g.nq = x.nq, g.t0 = x.t0, g.t1 = x.t1;
    for (int e = 0; e < (x.nq == 1 ? 4 : 16); ++e) g.m[e] = x.m[e];
    out.push_back(g);
  }
  return out;
}

}  // namespace

// ---- two-qubit reduced density matrices (ISL, entanglement_measures.py:326-340) ------------
// rho_ab[x][x'] = sum_rest psi[rest, x] conj(psi[rest, x']), x = 2*bit(hi) + bit(lo).  Each
// workgroup reduces one chunk of the 2^(n-2) "rest" indices of one pair into the 16 real
// numbers of the Hermitian 4x4 (upper triangle); a second pass sums the chunks (deterministic).
__device__ __forceinline__ size_t insert_zero_bit(size_t x, int pos) {
  return ((x >> pos) << (pos + 1)) | (x & ((size_t(1) << pos) - 1));
}

__global__ __launch_bounds__(kThreads) void k_sv_rdm_partial(const cplx* __restrict__ psi, int n,
                                                            const int* __restrict__ pairs,
                                                            double* __restrict__ partial) {
  const int p = blockIdx.y, chunks = gridDim.x;
  const int lo = min(pairs[2 * p], pairs[2 * p + 1]), hi = max(pairs[2 * p], pairs[2 * p + 1]);
  const size_t rest = size_t(1) << (n - 2);
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0;
  for (size_t r = (size_t)blockIdx.x * kThreads + threadIdx.x; r < rest; r += (size_t)chunks * kThreads) {
    const size_t base = insert_zero_bit(insert_zero_bit(r, lo), hi);
    cplx v[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) v[x] = psi[base | ((size_t)(x & 1) << lo) | ((size_t)(x >> 1) << hi)];
    int q = 0;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      acc[q++] += aqc::cnorm2(v[x]);
#pragma unroll
      for (int y = x + 1; y < 4; ++y) {
        const cplx m = aqc::cmul(v[x], aqc::cconj(v[y]));
        acc[q++] += m.x;
        acc[q++] += m.y;
      }
    }
  }
  __shared__ double red[16][kThreads];
#pragma unroll
  for (int q = 0; q < 16; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int h = kThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
#pragma unroll
      for (int q = 0; q < 16; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x < 16) partial[((size_t)p * chunks + blockIdx.x) * 16 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_sv_rdm_final(const double* __restrict__ partial, int chunks, int npairs, cplx* __restrict__ out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  double s[16];
  for (int q = 0; q < 16; ++q) s[q] = 0.0;
  for (int c = 0; c < chunks; ++c)
    for (int q = 0; q < 16; ++q) s[q] += partial[((size_t)p * chunks + c) * 16 + q];
  cplx* rho = out + (size_t)p * 16;
  int q = 0;
  for (int x = 0; x < 4; ++x) {
    rho[x * 4 + x] = aqc::cmk(s[q++], 0.0);
    for (int y = x + 1; y < 4; ++y) {
      const cplx m = aqc::cmk(s[q], s[q + 1]);
      q += 2;
      rho[x * 4 + y] = m;
      rho[y * 4 + x] = aqc::cconj(m);
    }
  }
}

// ---- transition matrix for cached Rotoselect / Rotosolve -------------------------------------
// T[a][b] = <chi| (|a><b|)_q |phi> = sum_rest conj(chi[rest, q=a]) phi[rest, q=b]: with phi the
// prefix state and chi = S^dag|0> the undone suffix, <0|S V P|0> = sum_ab V[a][b] T[a][b] for
// every single-qubit gate V at that position (cost_minimiser.py:344-368 evaluates 3 of them by
// full simulations).  Partial sums per workgroup, deterministic final pass.
__global__ __launch_bounds__(kThreads) void k_sv_transition_partial(const cplx* __restrict__ chi,
                                                                   const cplx* __restrict__ phi, int n, int q,
                                                                   double* __restrict__ partial) {
  const size_t half = size_t(1) << (n - 1);
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t r = (size_t)blockIdx.x * kThreads + threadIdx.x; r < half; r += (size_t)gridDim.x * kThreads) {
    const size_t i0 = insert_zero_bit(r, q), i1 = i0 | (size_t(1) << q);
    const cplx c0 = chi[i0], c1 = chi[i1], p0 = phi[i0], p1 = phi[i1];
    const cplx t00 = aqc::cconjmul(c0, p0), t01 = aqc::cconjmul(c0, p1), t10 = aqc::cconjmul(c1, p0),
               t11 = aqc::cconjmul(c1, p1);
    acc[0] += t00.x, acc[1] += t00.y, acc[2] += t01.x, acc[3] += t01.y;
    acc[4] += t10.x, acc[5] += t10.y, acc[6] += t11.x, acc[7] += t11.y;
  }
  __shared__ double red[8][kThreads];
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  for (int h = kThreads / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
#pragma unroll
      for (int k = 0; k < 8; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x < 8) partial[(size_t)blockIdx.x * 8 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void k_sv_transition_final(const double* __restrict__ partial, int chunks, double* __restrict__ out) {
  const int k = threadIdx.x;
  if (k >= 8) return;
  double s = 0.0;
  for (int c = 0; c < chunks; ++c) s += partial[(size_t)c * 8 + k];
  out[k] = s;
}

struct aqc_sv_s {
  int n = 0;
  int K = 0;
  cplx* state = nullptr;
  hipStream_t stream = nullptr;
  SegHeader* d_hdr = nullptr;
  size_t hdr_cap = 0;
  SegGate* d_gates = nullptr;
  size_t gate_cap = 0;
  double* d_zpart = nullptr;
  double* d_z = nullptr;
  int zwg = 0;
  cplx* h_pinned = nullptr;
  char* d_scratch = nullptr;  // grow-only workspace of the reduction kernels (RDMs, transition)
  size_t scratch_cap = 0;
};

static int sv_scratch(aqc_sv_t h, size_t bytes, char** out) {
  if (bytes > h->scratch_cap) {
    AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
    if (h->d_scratch) AQC_HIP_CHECK(hipFree(h->d_scratch));
    h->scratch_cap = std::max(bytes, 2 * h->scratch_cap);
    AQC_HIP_CHECK(hipMalloc(&h->d_scratch, h->scratch_cap));
  }
  *out = h->d_scratch;
  return AQC_OK;
}

static int sv_launch_segment(aqc_sv_t h, const SegHeader* dh, const SegGate* dg, int nblocks) {
  const double bytes = 32.0 * (double)(1ull << h->n);
  aqc::KernelTimer::begin(h->stream, "sv_segment", bytes, 0.0);
  switch (h->K) {
#define AQC_SEG_CASE(KK)                                                                   \
  case KK:                                                                                 \
    hipLaunchKernelGGL(k_sv_segment<KK>, dim3(nblocks), dim3(kThreads), 0, h->stream,      \
                       h->state, h->n, dh, dg);                                            \
    break;
    AQC_SEG_CASE(1)
    AQC_SEG_CASE(2)
    AQC_SEG_CASE(3)
    AQC_SEG_CASE(4)
    AQC_SEG_CASE(5)
    AQC_SEG_CASE(6)
    AQC_SEG_CASE(7)
    AQC_SEG_CASE(8)
    AQC_SEG_CASE(9)
    AQC_SEG_CASE(10)
    AQC_SEG_CASE(11)
#undef AQC_SEG_CASE
    default:
      aqc::set_error("sv: unsupported tile size");
      return AQC_ERR_UNSUPPORTED;
  }
  aqc::KernelTimer::end(h->stream);
  AQC_CHECK_LAUNCH();
  return AQC_OK;
}

extern "C" {

int aqc_sv_create(int n, aqc_sv_t* out) {
  AQC_REQUIRE(out != nullptr, "aqc_sv_create: null out");
  AQC_REQUIRE(n >= 1 && n <= 34, "aqc_sv_create: n must be in [1, 34]");
  auto* h = new aqc_sv_s();
  h->n = n;
  h->K = n < 10 ? n : 10;
  const uint64_t dim = 1ull << n;
  hipError_t e = hipMalloc(&h->state, dim * sizeof(cplx));
  if (e != hipSuccess) {
    delete h;
    aqc::set_error(std::string("aqc_sv_create: hipMalloc state: ") + hipGetErrorString(e));
    return AQC_ERR_NOMEM;
  }
  AQC_HIP_CHECK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  h->zwg = (int)((dim + kThreads * kZChunk - 1) / (kThreads * kZChunk));
  AQC_HIP_CHECK(hipMalloc(&h->d_zpart, sizeof(double) * (size_t)h->zwg * (n + 1)));
  AQC_HIP_CHECK(hipMalloc(&h->d_z, sizeof(double) * (n + 1)));
  AQC_HIP_CHECK(hipHostMalloc(&h->h_pinned, sizeof(cplx) * 64, hipHostMallocDefault));
  *out = h;
  return aqc_sv_reset(h);
}

int aqc_sv_destroy(aqc_sv_t h) {
  if (!h) return AQC_OK;
  if (h->stream) hipStreamSynchronize(h->stream);
  hipFree(h->state);
  hipFree(h->d_hdr);
  hipFree(h->d_gates);
  hipFree(h->d_zpart);
  hipFree(h->d_z);
  if (h->d_scratch) hipFree(h->d_scratch);
  if (h->h_pinned) hipHostFree(h->h_pinned);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return AQC_OK;
}

int aqc_sv_reset(aqc_sv_t h) {
  AQC_REQUIRE(h, "aqc_sv_reset: null handle");
  const uint64_t dim = 1ull << h->n;
  unsigned grid = (unsigned)std::min<uint64_t>((dim + 255) / 256, 65536);
  hipLaunchKernelGGL(k_sv_reset, dim3(grid), dim3(256), 0, h->stream, h->state, dim);
  AQC_CHECK_LAUNCH();
  return AQC_OK;
}

int aqc_sv_copy(aqc_sv_t dst, const aqc_sv_t src) {
  AQC_REQUIRE(dst && src && dst->n == src->n, "aqc_sv_copy: handle mismatch");
  AQC_HIP_CHECK(hipStreamSynchronize(src->stream));
  AQC_HIP_CHECK(hipMemcpyAsync(dst->state, src->state, sizeof(cplx) << dst->n,
                               hipMemcpyDeviceToDevice, dst->stream));
  return AQC_OK;
}

int aqc_sv_apply(aqc_sv_t h, const aqc_op_t* ops, int nops) {
  AQC_REQUIRE(h, "aqc_sv_apply: null handle");
  if (nops <= 0) return AQC_OK;
  AQC_REQUIRE(ops, "aqc_sv_apply: null ops");
  for (int i = 0; i < nops; ++i) {
    const aqc_op_t& o = ops[i];
    AQC_REQUIRE(o.nq == 1 || o.nq == 2, "aqc_sv_apply: only 1- and 2-qubit ops are supported");
    AQC_REQUIRE(o.q0 >= 0 && o.q0 < h->n, "aqc_sv_apply: qubit index out of range");
    if (o.nq == 2) {
      AQC_REQUIRE(o.q1 >= 0 && o.q1 < h->n && o.q1 != o.q0, "aqc_sv_apply: bad second qubit");
    }
  }
  const int K = h->K;
  std::vector<HostSeg> segs = build_segments(ops, nops, K, h->n);
  std::vector<SegHeader> hdr(segs.size());
  std::vector<SegGate> gts;
  gts.reserve(nops);
  for (size_t s = 0; s < segs.size(); ++s) {
    // tile bits: segment qubits + lowest free bits up to K
    uint64_t mask = segs[s].qmask;
    for (int b = 0; b < h->n && __builtin_popcountll(mask) < K; ++b) mask |= (1ull << b);
    int pos[64];
    int cnt = 0;
    for (int b = 0; b < h->n; ++b)
      if ((mask >> b) & 1ull) pos[cnt++] = b;
    std::memset(&hdr[s], 0, sizeof(SegHeader));
    int local_of[64];
    for (int j = 0; j < cnt; ++j) {
      hdr[s].tilebits[j] = pos[j];
      local_of[pos[j]] = j;
    }
    hdr[s].gate_off = (int)gts.size();
    const std::vector<SegGate> fused = fuse_segment(ops, segs[s].gates, local_of);
    hdr[s].ngates = (int)fused.size();
    gts.insert(gts.end(), fused.begin(), fused.end());
  }
  if (hdr.size() > h->hdr_cap) {
    AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
    hipFree(h->d_hdr);
    h->hdr_cap = hdr.size() * 2;
    AQC_HIP_CHECK(hipMalloc(&h->d_hdr, sizeof(SegHeader) * h->hdr_cap));
  }
  if (gts.size() > h->gate_cap) {
    AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
    hipFree(h->d_gates);
    h->gate_cap = gts.size() * 2;
    AQC_HIP_CHECK(hipMalloc(&h->d_gates, sizeof(SegGate) * h->gate_cap));
  }
  // The previous call's launches may still read these buffers: order the copy on the stream.
  AQC_HIP_CHECK(hipMemcpyAsync(h->d_hdr, hdr.data(), sizeof(SegHeader) * hdr.size(),
                               hipMemcpyHostToDevice, h->stream));
  AQC_HIP_CHECK(hipMemcpyAsync(h->d_gates, gts.data(), sizeof(SegGate) * gts.size(),
                               hipMemcpyHostToDevice, h->stream));
  // hipMemcpyAsync from pageable memory is staged before returning, so hdr/gts may go out
  // of scope; synchronising keeps that guarantee explicit.
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  const int nblocks = (int)(1ull << (h->n - K));
  for (size_t s = 0; s < hdr.size(); ++s) {
    int rc = sv_launch_segment(h, h->d_hdr + s, h->d_gates, nblocks);
    if (rc != AQC_OK) return rc;
  }
  return AQC_OK;
}

int aqc_sv_amp0(aqc_sv_t h, double* re, double* im) {
  AQC_REQUIRE(h && re && im, "aqc_sv_amp0: null argument");
  AQC_HIP_CHECK(hipMemcpyAsync(h->h_pinned, h->state, sizeof(cplx), hipMemcpyDeviceToHost, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  *re = h->h_pinned[0].x;
  *im = h->h_pinned[0].y;
  return AQC_OK;
}

int aqc_sv_z_all(aqc_sv_t h, double* out) {
  AQC_REQUIRE(h && out, "aqc_sv_z_all: null argument");
  aqc::KernelTimer::begin(h->stream, "sv_zall", 16.0 * (double)(1ull << h->n), 0.0);
  hipLaunchKernelGGL(k_sv_zpartial, dim3(h->zwg), dim3(kThreads), 0, h->stream, h->state, h->n,
                     h->d_zpart);
  aqc::KernelTimer::end(h->stream);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_sv_zfinal, dim3(1), dim3(64), 0, h->stream, h->d_zpart, h->zwg, h->n, h->d_z);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipMemcpyAsync(out, h->d_z, sizeof(double) * h->n, hipMemcpyDeviceToHost, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  return AQC_OK;
}

int aqc_sv_pair_rdms(aqc_sv_t h, const int* pairs, int npairs, double* out) {
  AQC_REQUIRE(h && pairs && out && npairs >= 0, "aqc_sv_pair_rdms: bad arguments");
  AQC_REQUIRE(h->n >= 2, "aqc_sv_pair_rdms: needs at least 2 qubits");
  for (int p = 0; p < npairs; ++p) {
    const int a = pairs[2 * p], b = pairs[2 * p + 1];
    AQC_REQUIRE(a >= 0 && a < h->n && b >= 0 && b < h->n && a != b, "aqc_sv_pair_rdms: bad pair");
  }
  if (npairs == 0) return AQC_OK;
  const size_t rest = size_t(1) << (h->n - 2);
  // about 2048 workgroups in total, at least 4 rest indices per thread
  const size_t per_pair = std::max<size_t>(1, std::min<size_t>(rest / (4 * kThreads), (2048 + npairs - 1) / npairs));
  const int chunks = (int)per_pair;
  char* buf = nullptr;
  const size_t pb = ((size_t)2 * npairs * sizeof(int) + 255) / 256 * 256;
  const size_t qb = (size_t)npairs * chunks * 16 * sizeof(double);
  const size_t ob = (size_t)npairs * 16 * sizeof(cplx);
  int rc = sv_scratch(h, pb + qb + ob, &buf);
  if (rc != AQC_OK) return rc;
  int* dpairs = (int*)buf;
  double* dpart = (double*)(buf + pb);
  cplx* dout = (cplx*)(buf + pb + qb);
  AQC_HIP_CHECK(hipMemcpyAsync(dpairs, pairs, 2 * npairs * sizeof(int), hipMemcpyHostToDevice, h->stream));
  aqc::KernelTimer::begin(h->stream, "sv_rdm", (double)npairs * 16.0 * (double)(1ull << h->n), 0.0);
  hipLaunchKernelGGL(k_sv_rdm_partial, dim3(chunks, npairs), dim3(kThreads), 0, h->stream, h->state, h->n, dpairs,
                     dpart);
  aqc::KernelTimer::end(h->stream);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_sv_rdm_final, dim3((npairs + 63) / 64), dim3(64), 0, h->stream, dpart, chunks, npairs, dout);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  return AQC_OK;
}

int aqc_sv_transition(aqc_sv_t bra, aqc_sv_t ket, int q, double* out) {
  AQC_REQUIRE(bra && ket && out, "aqc_sv_transition: null argument");
  AQC_REQUIRE(bra->n == ket->n && q >= 0 && q < bra->n, "aqc_sv_transition: bad qubit or size mismatch");
  const int n = bra->n;
  // ket and bra live on their own streams: order the reads after both states' pending work
  AQC_HIP_CHECK(hipStreamSynchronize(bra->stream));
  const size_t half = size_t(1) << (n - 1);
  const int chunks = (int)std::max<size_t>(1, std::min<size_t>(1024, half / (4 * kThreads)));
  char* raw = nullptr;
  int rc = sv_scratch(ket, ((size_t)chunks * 8 + 8) * sizeof(double), &raw);
  if (rc != AQC_OK) return rc;
  double* buf = (double*)raw;
  hipLaunchKernelGGL(k_sv_transition_partial, dim3(chunks), dim3(kThreads), 0, ket->stream, bra->state, ket->state, n,
                     q, buf);
  AQC_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_sv_transition_final, dim3(1), dim3(64), 0, ket->stream, buf, chunks, buf + (size_t)chunks * 8);
  AQC_CHECK_LAUNCH();
  AQC_HIP_CHECK(hipMemcpyAsync(out, buf + (size_t)chunks * 8, 8 * sizeof(double), hipMemcpyDeviceToHost, ket->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(ket->stream));
  return AQC_OK;
}

int aqc_sv_get(aqc_sv_t h, double* out) {
  AQC_REQUIRE(h && out, "aqc_sv_get: null argument");
  AQC_HIP_CHECK(hipMemcpyAsync(out, h->state, sizeof(cplx) << h->n, hipMemcpyDeviceToHost, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  return AQC_OK;
}

int aqc_sv_set(aqc_sv_t h, const double* in) {
  AQC_REQUIRE(h && in, "aqc_sv_set: null argument");
  AQC_HIP_CHECK(hipMemcpyAsync(h->state, in, sizeof(cplx) << h->n, hipMemcpyHostToDevice, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  return AQC_OK;
}

}  // extern "C"
