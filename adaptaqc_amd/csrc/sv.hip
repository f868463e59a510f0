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
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <atomic>

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

// ---- register-resident tile passes (n >= kRegMinQubits) -------------------------------------
// A 4096-amplitude tile per workgroup.  The segment's fused gates are grouped on the host into
// "phases" whose gates all act inside one set of NS tile bits (the phase's slots).  In a phase
// every thread holds the 2^NS amplitudes that differ only in those slot bits in registers, applies
// all of the phase's gates there (fully unrolled per slot pattern), and writes them back: one LDS
// round trip and one barrier per phase instead of per gate, and 2^NS independent LDS reads per
// thread in flight instead of 2 or 4 dependent ones.  Gate matrices of phase p+1 are staged into
// LDS (double buffer) while phase p computes.  NS = 4: 256 threads x 16 amplitudes (one wave per
// SIMD at n = 20, where there are 256 tiles).  (NS = 3, 512 threads x 8 amplitudes and two waves per
// SIMD, measured 4% slower at 1.7x the phases; removed from the library in round 5.)
constexpr int kSlots = 4;
constexpr int kRegTileBits = 12;   // 4096 amplitudes (64 KB LDS)
constexpr int kRegMinQubits = 14;  // below: the per-gate kernel (too few tiles)
constexpr int kPhaseMaxGates = 16;
constexpr int kRegLowBits = 4;     // global bits 0..3 always in the tile (256-byte runs)
static_assert(kRegTileBits <= kMaxTileBits, "tile header too small");

struct PhaseHdr {
  int32_t slotmask;  // the phase's NS tile bits (+ the direct-I/O flags below)
  int32_t gate_off;  // into the segment gate array (SegGate: t0 < t1 are slot indices 0..NS-1)
  int32_t ngates;
  int32_t pad;
  uint64_t lanemap;  // thread bit j -> tile bit (lanemap >> 4j) & 15 (the 12 - NS non-slot bits)
};

// LDS layout: amplitude e of the tile lives at e ^ swz(e), where swz XORs a column of kSwzCol
// into the low 4 bits per set bit of e >> 4.  With the 12 columns of the map e -> (e ^ swz(e)) & 15
// distinct and non-zero (bits 0-3: 1, 2, 4, 8), any 8 of them span GF(2)^4, so for every slot set
// the host can order the non-slot bits over the lanes (PhaseHdr::lanemap) such that each 16-lane
// group of a ds_read_b128 (the cosets of lanes {1, 2, 12, 20}) and each 8-lane group of a
// ds_write_b128 touches distinct 16-byte bank slots: conflict-free phases.  A linear layout puts
// the 16 lanes of a phase whose slots are tile bits 0-3 on one bank slot (16-way).
constexpr int kSwzCol[8] = {3, 6, 12, 9, 5, 10, 7, 14};
__host__ __device__ __forceinline__ int swz_bits(int e) {
  int v = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b)
    if ((e >> (4 + b)) & 1) v ^= kSwzCol[b];
  return v;
}
__host__ __device__ __forceinline__ int swz(int e) { return e ^ swz_bits(e); }

template <int S, int NA>
__device__ __forceinline__ void reg_apply1(cplx (&a)[NA], const SegGate& g) {
  const cplx m00 = g.m[0], m01 = g.m[1], m10 = g.m[2], m11 = g.m[3];
#pragma unroll
  for (int r = 0; r < NA; ++r) {
    if ((r >> S) & 1) continue;
    const int r1 = r | (1 << S);
    const cplx a0 = a[r], a1 = a[r1];
    a[r] = aqc::cfma(m01, a1, aqc::cmul(m00, a0));
    a[r1] = aqc::cfma(m11, a1, aqc::cmul(m10, a0));
  }
}

template <int S0, int S1, int NA>
__device__ __forceinline__ void reg_apply2(cplx (&a)[NA], const SegGate& g) {
  cplx m[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) m[e] = g.m[e];
#pragma unroll
  for (int r = 0; r < NA; ++r) {
    if (((r >> S0) & 1) || ((r >> S1) & 1)) continue;
    int idx[4];
    cplx v[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      idx[s] = r | ((s & 1) << S0) | ((s >> 1) << S1);
      v[s] = a[idx[s]];
    }
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      cplx acc = aqc::cmul(m[4 * o], v[0]);
      acc = aqc::cfma(m[4 * o + 1], v[1], acc);
      acc = aqc::cfma(m[4 * o + 2], v[2], acc);
      acc = aqc::cfma(m[4 * o + 3], v[3], acc);
      a[idx[o]] = acc;
    }
  }
}

template <int NS>
__device__ __forceinline__ void reg_apply(cplx (&a)[1 << NS], const SegGate& g) {
  // wave-uniform dispatch on the slot pattern (t0 < t1 for 2-qubit gates, host-normalised)
  constexpr int NA = 1 << NS;
  const int code = __builtin_amdgcn_readfirstlane(g.nq == 1 ? g.t0 : 4 + 4 * g.t0 + g.t1);
  switch (code) {
    case 0: reg_apply1<0, NA>(a, g); break;
    case 1: reg_apply1<1, NA>(a, g); break;
    case 2: reg_apply1<2, NA>(a, g); break;
    case 4 + 1: reg_apply2<0, 1, NA>(a, g); break;
    case 4 + 2: reg_apply2<0, 2, NA>(a, g); break;
    case 4 + 6: reg_apply2<1, 2, NA>(a, g); break;
    default:
      if constexpr (NS == 4) {
        switch (code) {
          case 3: reg_apply1<3, NA>(a, g); break;
          case 4 + 3: reg_apply2<0, 3, NA>(a, g); break;
          case 4 + 7: reg_apply2<1, 3, NA>(a, g); break;
          case 4 + 11: reg_apply2<2, 3, NA>(a, g); break;
          default: break;
        }
      }
      break;
  }
}

// Phase flags in PhaseHdr::slotmask above the tile bits: the segment's first phase reads its
// registers straight from global memory, its last phase writes them straight back (no LDS round
// trip, no barrier).  The host sets them when the phase's lane map can put thread bits 0-3 on tile
// bits 0-3 (no low slot bit): a wave then reads / writes 16 runs of 256 contiguous bytes.
constexpr int kPhaseDirectIn = 1 << 30, kPhaseDirectOut = 1 << 29, kPhaseSlotBits = (1 << kRegTileBits) - 1;

template <int NS>
__global__ __launch_bounds__(4096 >> NS) void k_sv_tile_reg(cplx* __restrict__ state, const SegHeader* __restrict__ hdr,
                                                           const PhaseHdr* __restrict__ phases,
                                                           const SegGate* __restrict__ gates, int from_zero,
                                                           cplx* __restrict__ amp0_out) {
  constexpr int K = kRegTileBits, kThr = 4096 >> NS, kTB = K - NS, NA = 1 << NS;
  __shared__ cplx tile[1 << K];
  __shared__ SegGate gl[2][kPhaseMaxGates];
  const int tid = threadIdx.x;
  int tb[K];
#pragma unroll
  for (int j = 0; j < K; ++j) tb[j] = hdr->tilebits[j];
  uint64_t base = blockIdx.x;
#pragma unroll
  for (int j = 0; j < K; ++j) base = insert_zero(base, tb[j]);
  auto gidx = [&](int x) {
    uint64_t g = base;
#pragma unroll
    for (int j = 0; j < K; ++j) g |= (uint64_t)((x >> j) & 1) << tb[j];
    return g;
  };
  constexpr int kPer = (1 << K) / kThr;
  if (from_zero && blockIdx.x != 0) {
    // a deferred aqc_sv_reset: every tile but tile 0 (which holds index 0) is zero in and out --
    // the segment's gates act inside the tile -- so it is written without loads or gates
#pragma unroll
    for (int r = 0; r < kPer; ++r) aqc::stg(state + gidx(tid + r * kThr), aqc::cmk(0.0, 0.0));
    return;
  }
  const int np = hdr->ngates;
  const PhaseHdr* ph = phases + hdr->gate_off;
  const bool d_in = np > 0 && (ph[0].slotmask & kPhaseDirectIn);
  const bool d_out = np > 0 && (ph[np - 1].slotmask & kPhaseDirectOut);
  if (!d_in) {
    cplx v[kPer];
    if (from_zero) {
#pragma unroll
      for (int r = 0; r < kPer; ++r) v[r] = aqc::cmk(tid + r * kThr == 0 ? 1.0 : 0.0, 0.0);
    } else {
#pragma unroll
      for (int r = 0; r < kPer; ++r) v[r] = aqc::ldg(state + gidx(tid + r * kThr));
    }
#pragma unroll
    for (int r = 0; r < kPer; ++r) tile[swz(tid + r * kThr)] = v[r];
  }
  constexpr int kWords = (int)(sizeof(SegGate) / sizeof(double2));
  auto stage = [&](int p) {
    const int ng = ph[p].ngates;
    const double2* src = reinterpret_cast<const double2*>(gates + ph[p].gate_off);
    double2* dst = reinterpret_cast<double2*>(gl[p & 1]);
    for (int w = tid; w < ng * kWords; w += kThr) dst[w] = src[w];
  };
  if (np > 0) stage(0);
  __syncthreads();
  for (int p = 0; p < np; ++p) {
    if (p + 1 < np) stage(p + 1);  // the other buffer: its last readers passed the barrier below
    const int sm = __builtin_amdgcn_readfirstlane(ph[p].slotmask) & kPhaseSlotBits;
    const uint64_t lm = ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(ph[p].lanemap >> 32)) << 32) |
                        (unsigned)__builtin_amdgcn_readfirstlane((int)ph[p].lanemap);
    // thread bits placed on the non-slot tile bits by the lane map, slot bits from r; the swizzle
    // is linear, so the LDS address is swz(thread part) ^ swz(slot part), and the global index
    // is the OR of the two parts' scattered bits
    int lraw = 0;
#pragma unroll
    for (int j = 0; j < kTB; ++j) lraw |= ((tid >> j) & 1) << ((int)(lm >> (4 * j)) & 15);
    // the NS slot bits, lowest first (the host pads every phase to exactly NS), and their global
    // bits (no per-lane indexing: the arrays stay in registers)
    int sraw[4] = {0, 0, 0, 0};
    uint64_t sg[4] = {0, 0, 0, 0};
    {
      int m = sm;
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        sraw[i] = m & -m;
        m ^= sraw[i];
        sg[i] = gidx(sraw[i]) ^ base;
      }
    }
    const bool in_g = p == 0 && d_in, out_g = p == np - 1 && d_out;
    const int lb = swz(lraw);
    int off[NA];
#pragma unroll
    for (int r = 0; r < NA; ++r)
      off[r] = lb ^ ((r & 1) ? swz(sraw[0]) : 0) ^ ((r & 2) ? swz(sraw[1]) : 0) ^ ((r & 4) ? swz(sraw[2]) : 0) ^
               ((r & 8) ? swz(sraw[3]) : 0);
    auto gaddr = [&](int r) {
      return state + (gidx(lraw) | ((r & 1) ? sg[0] : 0) | ((r & 2) ? sg[1] : 0) | ((r & 4) ? sg[2] : 0) |
                      ((r & 8) ? sg[3] : 0));
    };
    cplx a[NA];
    if (in_g) {
      if (from_zero) {
#pragma unroll
        for (int r = 0; r < NA; ++r) {
          const int x = lraw | ((r & 1) ? sraw[0] : 0) | ((r & 2) ? sraw[1] : 0) | ((r & 4) ? sraw[2] : 0) |
                        ((r & 8) ? sraw[3] : 0);
          a[r] = aqc::cmk(x == 0 ? 1.0 : 0.0, 0.0);
        }
      } else {
#pragma unroll
        for (int r = 0; r < NA; ++r) a[r] = aqc::ldg(gaddr(r));
      }
    } else {
#pragma unroll
      for (int r = 0; r < NA; ++r) a[r] = tile[off[r]];
    }
    const int ng = ph[p].ngates;
    for (int gi = 0; gi < ng; ++gi) reg_apply<NS>(a, gl[p & 1][gi]);
    if (out_g) {
#pragma unroll
      for (int r = 0; r < NA; ++r) aqc::stg(gaddr(r), a[r]);
      // the apply's last pass hands <0...0|psi> (tile 0, thread 0, r = 0: global index 0) straight
      // to the pinned host buffer, so aqc_sv_amp0 needs no copy of its own
      if (amp0_out && blockIdx.x == 0 && tid == 0) *amp0_out = a[0];
    } else {
#pragma unroll
      for (int r = 0; r < NA; ++r) tile[off[r]] = a[r];
      __syncthreads();
    }
  }
  if (!d_out) {
#pragma unroll
    for (int r = 0; r < kPer; ++r) aqc::stg(state + gidx(tid + r * kThr), tile[swz(tid + r * kThr)]);
    if (amp0_out && blockIdx.x == 0 && tid == 0) *amp0_out = tile[swz(0)];
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

// Greedy segmentation, one segment per next(): a segment takes every not-yet-placed op, in order,
// whose qubits fit in the K tile bits and that no skipped op on its qubits precedes.  Produced one
// at a time so that aqc_sv_apply launches the first segment before the rest are formed.
struct SegBuilder {
  const aqc_op_t* ops;
  int nops, K, n;
  uint64_t reserve;
  std::vector<char> done;
  int remaining, first = 0;
  SegBuilder(const aqc_op_t* o, int no, int k, int nq, uint64_t res)
      : ops(o), nops(no), K(k), n(nq), reserve(res), done(no, 0), remaining(no) {}
  bool next(HostSeg& seg) {
    seg.gates.clear();
    seg.qmask = 0;
    if (remaining <= 0) return false;
    while (first < nops && done[first]) ++first;
    uint64_t blocked = 0;
    for (int i = first; i < nops; ++i) {
      if (done[i]) continue;
      uint64_t gm = (1ull << ops[i].q0);
      if (ops[i].nq == 2) gm |= (1ull << ops[i].q1);
      if (gm & blocked) {
        blocked |= gm;
      } else {
        uint64_t u = seg.qmask | gm;
        if (__builtin_popcountll(u | reserve) <= K) {
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
    return true;
  }
};

std::vector<HostSeg> build_segments(const aqc_op_t* ops, int nops, int K, int n, uint64_t reserve = 0) {
  std::vector<HostSeg> segs;
  SegBuilder b(ops, nops, K, n, reserve);
  HostSeg seg;
  while (b.next(seg)) segs.push_back(seg);
  return segs;
}

// ---- host-side gate fusion inside a segment -------------------------------------------------
// Every 1-qubit gate is multiplied into the last fused op on its qubit (1- or 2-qubit), or into
// the next 2-qubit gate on it when that gate comes first; consecutive 2-qubit gates on the same
// pair become one 4x4.  Valid because the merged ops are adjacent on their qubits (everything in
// between acts on other qubits and commutes).  Aer fuses too (fusion_enable at >= 14 qubits);
// here every tile pass saves one LDS sweep and one barrier per absorbed gate.  Brickwork: 3 ops
// per pair and layer become 1.
// Host arithmetic on a plain {re, im} pair: HIP's vector type kept the fusion from optimising
// (0.13 us per gate, 88 us of a 20-qubit evaluation's ~140 us host plan), and no fma() -- the x86
// host build has no FMA instructions enabled, so fma() is a libm call per operation.
struct hc {
  double r, i;
};
typedef std::array<hc, 16> Mat4;
static inline hc hmul(hc a, hc b) { return {a.r * b.r - a.i * b.i, a.r * b.i + a.i * b.r}; }
static inline hc hfma(hc a, hc b, hc c) { return {c.r + a.r * b.r - a.i * b.i, c.i + a.r * b.i + a.i * b.r}; }

static Mat4 mat4_mul(const Mat4& a, const Mat4& b) {  // a b
  Mat4 c;
  for (int r = 0; r < 4; ++r)
    for (int k = 0; k < 4; ++k) {
      hc acc = {0.0, 0.0};
      for (int j = 0; j < 4; ++j) acc = hfma(a[4 * r + j], b[4 * j + k], acc);
      c[4 * r + k] = acc;
    }
  return c;
}

// E m and m E for E = the 1-qubit u on bit `which` (0: the op's t0, 1: its t1) of a 4x4 (index
// 2 b1 + b0), without forming E: 32 complex products instead of 64
static void left1(const hc* u, int which, Mat4& m) {
  const int bit = 1 << which;
  for (int r0 = 0; r0 < 4; ++r0) {
    if (r0 & bit) continue;
    const int r1 = r0 | bit;
    for (int c = 0; c < 4; ++c) {
      const hc a = m[4 * r0 + c], b = m[4 * r1 + c];
      m[4 * r0 + c] = hfma(u[1], b, hmul(u[0], a));
      m[4 * r1 + c] = hfma(u[3], b, hmul(u[2], a));
    }
  }
}
static void right1(Mat4& m, const hc* u, int which) {
  const int bit = 1 << which;
  for (int c0 = 0; c0 < 4; ++c0) {
    if (c0 & bit) continue;
    const int c1 = c0 | bit;
    for (int r = 0; r < 4; ++r) {
      const hc a = m[4 * r + c0], b = m[4 * r + c1];
      m[4 * r + c0] = hfma(b, u[2], hmul(a, u[0]));
      m[4 * r + c1] = hfma(b, u[3], hmul(a, u[1]));
    }
  }
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
    bool dead;
    Mat4 m;  // nq == 1: m[0..3] = 2x2
  };
  thread_local std::vector<F> f;  // (reused: one allocation per thread, not per segment)
  f.clear();
  f.reserve(idx.size());
  int last[64];
  for (int q = 0; q < 64; ++q) last[q] = -1;
  for (int gi : idx) {
    const aqc_op_t& o = ops[gi];
    const hc* u = reinterpret_cast<const hc*>(o.m);  // (re, im) pairs, row-major
    if (o.nq == 1) {
      const int q = local_of[o.q0];
      const int k = last[q];
      if (k >= 0 && f[k].nq == 1) {  // 2x2 product u * m
        Mat4& m = f[k].m;
        const hc m0 = m[0], m1 = m[1], m2 = m[2], m3 = m[3];
        m[0] = hfma(u[1], m2, hmul(u[0], m0));
        m[1] = hfma(u[1], m3, hmul(u[0], m1));
        m[2] = hfma(u[3], m2, hmul(u[2], m0));
        m[3] = hfma(u[3], m3, hmul(u[2], m1));
      } else if (k >= 0) {
        left1(u, f[k].t0 == q ? 0 : 1, f[k].m);
      } else {
        f.emplace_back();
        F& n = f.back();
        n.nq = 1, n.t0 = q, n.t1 = 0, n.dead = false;
        for (int e = 0; e < 4; ++e) n.m[e] = u[e];
        last[q] = (int)f.size() - 1;
      }
      continue;
    }
    const int a = local_of[o.q0], b = local_of[o.q1];
    const int ka = last[a], kb = last[b];
    if (ka >= 0 && ka == kb && f[ka].nq == 2) {  // same pair again
      Mat4 g;
      for (int e = 0; e < 16; ++e) g[e] = u[e];
      f[ka].m = mat4_mul(f[ka].t0 == a ? g : swap_bits(g), f[ka].m);
      continue;
    }
    // absorb pending single-qubit ops on a / b (their last op, nothing after them on that qubit)
    f.emplace_back();
    F& n = f.back();
    n.nq = 2, n.t0 = a, n.t1 = b, n.dead = false;
    for (int e = 0; e < 16; ++e) n.m[e] = u[e];
    if (ka >= 0 && f[ka].nq == 1) {
      right1(n.m, f[ka].m.data(), 0);
      f[ka].dead = true;
    }
    if (kb >= 0 && f[kb].nq == 1) {
      right1(n.m, f[kb].m.data(), 1);
      f[kb].dead = true;
    }
    last[a] = last[b] = (int)f.size() - 1;
  }
  std::vector<SegGate> out;
  out.reserve(f.size());
  for (const F& x : f) {
    if (x.dead) continue;
    out.emplace_back();
    SegGate& g = out.back();
    std::memset(&g, 0, sizeof(g));
    g.nq = x.nq, g.t0 = x.t0, g.t1 = x.t1;
    for (int e = 0; e < (x.nq == 1 ? 4 : 16); ++e) g.m[e] = aqc::cmk(x.m[e].r, x.m[e].i);
  }
  return out;
}

// Phases of a fused segment (k_sv_tile_reg): greedy in application order, a gate joins the
// current phase when its tile bits fit in the phase's NS slots and it acts on no bit of a gate
// left for a later phase (gates on disjoint bits commute).  Gate bits become slot indices (t0 < t1,
// the 4x4 re-indexed when the order flips).
// Lane map of a slot set: an order of the 12 - NS non-slot tile bits over the thread bits whose
// first six (the wave's lanes) give conflict-free LDS groups under swz (checked by counting bank
// slots over the 64 lanes of a wave; the first order with no conflict, else the one with the
// fewest extra cycles).  Cached per slot set.
uint64_t lane_map(uint32_t S, int NS) {
  // cached per (NS, slot set): bit 63 marks a computed entry (lock-free reads; a race computes
  // the same value twice)
  static std::array<std::atomic<uint64_t>, 2 << kRegTileBits> cache{};
  std::atomic<uint64_t>& slot_entry = cache[(NS == 3 ? (1 << kRegTileBits) : 0) + S];
  const uint64_t c = slot_entry.load(std::memory_order_acquire);
  if (c >> 63) return c & ~(1ull << 63);
  const int TB = kRegTileBits - NS;
  int ns[9], nn = 0;
  for (int b = 0; b < kRegTileBits; ++b)
    if (!((S >> b) & 1u) && nn < 9) ns[nn++] = b;
  auto cost = [&](const int* pos) {
    int e[64];
    for (int l = 0; l < 64; ++l) {
      int v = 0;
      for (int j = 0; j < 6; ++j) v |= ((l >> j) & 1) << pos[j];
      e[l] = swz(v);
    }
    int c = 0;
    static const int g128[16] = {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27};
    for (int base : {0, 4, 32, 36}) {  // the four cosets of the b128 read group
      int cnt[16] = {};
      int mx = 0;
      for (int k = 0; k < 16; ++k) mx = std::max(mx, ++cnt[e[base ^ g128[k]] & 15]);
      c += mx - 1;
    }
    for (int g = 0; g < 64; g += 8) {  // b128 writes: 8 contiguous lanes, 8 bank slots
      int cnt[8] = {};
      int mx = 0;
      for (int k = 0; k < 8; ++k) mx = std::max(mx, ++cnt[e[g + k] & 7]);
      c += mx - 1;
    }
    return c;
  };
  int best[9], bc = 1 << 30;
  int perm[9];
  for (int i = 0; i < TB; ++i) perm[i] = i;
  // the first six positions decide the wave's banks; the rest (threads across waves) follow
  do {
    int pos[9];
    for (int i = 0; i < TB; ++i) pos[i] = ns[perm[i]];
    const int c = cost(pos);
    if (c < bc) {
      bc = c;
      std::memcpy(best, pos, sizeof(int) * TB);
      if (c == 0) break;
    }
    std::reverse(perm + 6, perm + TB);  // skip orders that differ only past the sixth position
  } while (std::next_permutation(perm, perm + TB));
  uint64_t m = 0;
  for (int j = 0; j < TB; ++j) m |= (uint64_t)best[j] << (4 * j);
  slot_entry.store((1ull << 63) | m, std::memory_order_release);
  return m;
}

// The segment's first / last phase: non-slot tile bits in ascending order over the thread bits,
// flagged for direct global reads / writes (k_sv_tile_reg) when no slot is a low tile bit
uint64_t lane_map_coalesced(uint32_t S) {
  uint64_t m = 0;
  int j = 0;
  for (int b = 0; b < kRegTileBits; ++b)
    if (!((S >> b) & 1u)) m |= (uint64_t)b << (4 * j++);
  return m;
}

void mark_direct_phases(PhaseHdr* first, PhaseHdr* last) {
  if ((first->slotmask & 15) == 0) {
    first->lanemap = lane_map_coalesced((uint32_t)first->slotmask);
    first->slotmask |= kPhaseDirectIn;
  }
  if (((last->slotmask & kPhaseSlotBits) & 15) == 0) {
    if (last != first) last->lanemap = lane_map_coalesced((uint32_t)(last->slotmask & kPhaseSlotBits));
    last->slotmask |= kPhaseDirectOut;
  }
}

void build_phases(const std::vector<SegGate>& fused, int K, int NS, std::vector<PhaseHdr>& ph,
                  std::vector<SegGate>& out) {
  std::vector<char> done(fused.size(), 0);
  size_t remaining = fused.size(), first = 0;
  while (remaining > 0) {
    while (done[first]) ++first;
    uint32_t S = 0, blocked = 0;
    size_t members[kPhaseMaxGates];
    int nm = 0;
    for (size_t i = first; i < fused.size() && nm < kPhaseMaxGates; ++i) {
      if (done[i]) continue;
      const uint32_t gm = (1u << fused[i].t0) | (fused[i].nq == 2 ? (1u << fused[i].t1) : 0u);
      if (gm & blocked) {
        blocked |= gm;
      } else if (__builtin_popcount(S | gm) <= NS) {
        S |= gm;
        members[nm++] = i;
        done[i] = 1;
        --remaining;
      } else {
        blocked |= gm;
      }
      if (__builtin_popcount(blocked) >= K) break;
    }
    for (int b = 0; b < K && __builtin_popcount(S) < NS; ++b) S |= 1u << b;
    auto slot = [&](int b) { return __builtin_popcount(S & ((1u << b) - 1u)); };
    PhaseHdr h;
    h.slotmask = (int32_t)S;
    h.gate_off = (int32_t)out.size();
    h.ngates = (int32_t)nm;
    h.pad = 0;
    h.lanemap = lane_map(S, NS);
    ph.push_back(h);
    for (int mi = 0; mi < nm; ++mi) {
      SegGate g = fused[members[mi]];
      if (g.nq == 1) {
        g.t0 = slot(g.t0);
      } else {
        const int s0 = slot(g.t0), s1 = slot(g.t1);
        if (s0 > s1) {
          Mat4 m;
          for (int e = 0; e < 16; ++e) m[e] = {g.m[e].x, g.m[e].y};
          m = swap_bits(m);
          for (int e = 0; e < 16; ++e) g.m[e] = aqc::cmk(m[e].r, m[e].i);
        }
        g.t0 = s0 < s1 ? s0 : s1;
        g.t1 = s0 < s1 ? s1 : s0;
      }
      out.push_back(g);
    }
  }
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
  char* d_plan = nullptr;  // [segment headers | phases | gates] of the last aqc_sv_apply
  char* h_plan = nullptr;  // pinned staging copy
  size_t plan_cap = 0;
  hipEvent_t plan_ev = nullptr;
  bool reg_tiles = false;
  double* d_zpart = nullptr;
  double* d_z = nullptr;
  int zwg = 0;
  cplx* h_pinned = nullptr;
  char* d_scratch = nullptr;  // grow-only workspace of the reduction kernels (RDMs, transition)
  size_t scratch_cap = 0;
  // aqc_sv_reset on the register-tile path is deferred: the next aqc_sv_apply's first pass forms
  // |0...0> in its tiles instead of reading the state (no reset kernel, one 2^n read less); any
  // other reader materialises it first (sv_materialize)
  bool zero_pending = false;
  // the last aqc_sv_apply's final pass wrote amp 0 to h_pinned[0] (valid once the stream is drained)
  bool amp0_ready = false;
  // plans of an apply's second and later batches go over on this stream while the previous batch's
  // passes run; the state's stream waits on the batch's event before its first pass
  hipStream_t up_stream = nullptr;
  hipEvent_t up_ev[2] = {nullptr, nullptr};
  // recorded on this state's stream after a copy that reads another state (aqc_sv_copy): the
  // source's stream waits on it, so the source is neither rewritten nor freed (and its pooled block
  // handed out again) while the copy still reads it
  hipEvent_t read_ev = nullptr;
};

static int sv_materialize(aqc_sv_t h) {
  if (!h->zero_pending) return AQC_OK;
  const uint64_t dim = 1ull << h->n;
  unsigned grid = (unsigned)std::min<uint64_t>((dim + 255) / 256, 65536);
  hipLaunchKernelGGL(k_sv_reset, dim3(grid), dim3(256), 0, h->stream, h->state, dim);
  AQC_CHECK_LAUNCH();
  h->zero_pending = false;
  return AQC_OK;
}

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

// register tiles keep the lowest global bits in every tile (runs of 2^low contiguous amplitudes
// per lane group: a tile of high qubits only reads 16-byte pieces scattered 4 KB apart)
static uint64_t sv_reserved_bits(bool reg_tiles) {
  if (!reg_tiles) return 0;
  return (1ull << kRegLowBits) - 1ull;
}

static std::vector<HostSeg> sv_plan_segments(int n, int K, bool reg_tiles, const aqc_op_t* ops, int nops) {
  return build_segments(ops, nops, K, n, sv_reserved_bits(reg_tiles));
}

// Segment s of the plan: its header (hdr[s], sized by the caller), its fused gates and phases
// appended to gts / phs (gate_off indexes the whole list).
static void sv_plan_one(int n, int K, bool reg_tiles, const aqc_op_t* ops, const HostSeg& seg, size_t s,
                        std::vector<SegHeader>& hdr, std::vector<SegGate>& gts, std::vector<PhaseHdr>& phs,
                        std::vector<double>* seg_flops) {
  // tile bits: segment qubits + lowest free bits up to K
  uint64_t mask = seg.qmask;
  for (int b = 0; b < n && __builtin_popcountll(mask) < K; ++b) mask |= (1ull << b);
  int pos[64];
  int cnt = 0;
  for (int b = 0; b < n; ++b)
    if ((mask >> b) & 1ull) pos[cnt++] = b;
  std::memset(&hdr[s], 0, sizeof(SegHeader));
  int local_of[64];
  for (int j = 0; j < cnt; ++j) {
    hdr[s].tilebits[j] = pos[j];
    local_of[pos[j]] = j;
  }
  const std::vector<SegGate> fused = fuse_segment(ops, seg.gates, local_of);
  if (seg_flops) {  // real flops of the fused gates: 1q 2, 2q 4 complex MACs (8 flops) per amplitude
    double f = 0.0;
    for (const SegGate& g : fused) f += (g.nq == 1 ? 16.0 : 32.0) * std::ldexp(1.0, n);
    seg_flops->push_back(f);
  }
  if (reg_tiles) {  // gate_off / ngates index the phase list
    hdr[s].gate_off = (int)phs.size();
    const size_t before = phs.size();
    build_phases(fused, K, kSlots, phs, gts);
    hdr[s].ngates = (int)(phs.size() - before);
    if (phs.size() > before) mark_direct_phases(&phs[before], &phs.back());
  } else {
    hdr[s].gate_off = (int)gts.size();
    hdr[s].ngates = (int)fused.size();
    gts.insert(gts.end(), fused.begin(), fused.end());
  }
}

// Host planning of one aqc_sv_apply: segments (tile bits + fused gates), and the phases of the
// register-tile path.
static void sv_plan(int n, int K, bool reg_tiles, const aqc_op_t* ops, int nops, std::vector<SegHeader>& hdr,
                    std::vector<SegGate>& gts, std::vector<PhaseHdr>& phs, std::vector<double>* seg_flops = nullptr) {
  const std::vector<HostSeg> segs = sv_plan_segments(n, K, reg_tiles, ops, nops);
  hdr.assign(segs.size(), SegHeader{});
  gts.reserve(nops);
  for (size_t s = 0; s < segs.size(); ++s) sv_plan_one(n, K, reg_tiles, ops, segs[s], s, hdr, gts, phs, seg_flops);
}

static bool sv_reg_tiles(int n) {
  // register-resident 4096-amplitude tiles from kRegMinQubits qubits (below: the per-gate LDS kernel;
  // AQC_SV_TILE=lds keeps it above too, which the tests use to check one kernel against the other)
  const char* tile_env = std::getenv("AQC_SV_TILE");
  return n >= kRegMinQubits && !(tile_env && std::strcmp(tile_env, "lds") == 0);
}

static int sv_launch_segment(aqc_sv_t h, const SegHeader* dh, const PhaseHdr* dp, const SegGate* dg, int nblocks, cplx* amp0_out,
                             double flops) {
  const int from_zero = h->zero_pending ? 1 : 0;
  const double bytes = (from_zero ? 16.0 : 32.0) * (double)(1ull << h->n);
  aqc::KernelTimer::begin(h->stream, "sv_segment", bytes, flops);
  if (h->reg_tiles) {
    hipLaunchKernelGGL(k_sv_tile_reg<kSlots>, dim3(nblocks), dim3(4096 >> kSlots), 0, h->stream, h->state, dh, dp, dg,
                       from_zero, amp0_out);
    h->zero_pending = false;
    aqc::KernelTimer::end(h->stream);
    AQC_CHECK_LAUNCH();
    return AQC_OK;
  }
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
  h->reg_tiles = sv_reg_tiles(n);
  h->K = h->reg_tiles ? kRegTileBits : (n < 10 ? n : 10);
  const uint64_t dim = 1ull << n;
  h->state = (cplx*)aqc::dev_alloc(dim * sizeof(cplx));
  if (!h->state) {
    delete h;
    aqc::set_error("aqc_sv_create: out of device memory for the state");
    return AQC_ERR_NOMEM;
  }
  AQC_HIP_CHECK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
  AQC_HIP_CHECK(hipEventCreateWithFlags(&h->plan_ev, hipEventDisableTiming));
  AQC_HIP_CHECK(hipStreamCreateWithFlags(&h->up_stream, hipStreamNonBlocking));
  for (auto& e : h->up_ev) AQC_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  AQC_HIP_CHECK(hipEventCreateWithFlags(&h->read_ev, hipEventDisableTiming));
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
  aqc::dev_free(h->state);
  if (h->d_plan) hipFree(h->d_plan);
  if (h->h_plan) hipHostFree(h->h_plan);
  if (h->plan_ev) hipEventDestroy(h->plan_ev);
  hipFree(h->d_zpart);
  hipFree(h->d_z);
  if (h->d_scratch) hipFree(h->d_scratch);
  if (h->h_pinned) hipHostFree(h->h_pinned);
  if (h->up_stream) hipStreamSynchronize(h->up_stream), hipStreamDestroy(h->up_stream);
  for (hipEvent_t e : h->up_ev)
    if (e) hipEventDestroy(e);
  if (h->read_ev) hipEventDestroy(h->read_ev);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return AQC_OK;
}

int aqc_sv_reset(aqc_sv_t h) {
  AQC_REQUIRE(h, "aqc_sv_reset: null handle");
  h->zero_pending = true;
  h->amp0_ready = false;
  return h->reg_tiles ? AQC_OK : sv_materialize(h);
}

int aqc_sv_copy(aqc_sv_t dst, const aqc_sv_t src) {
  AQC_REQUIRE(dst && src && dst->n == src->n, "aqc_sv_copy: handle mismatch");
  if (dst == src) return sv_materialize(src);
  int rc = sv_materialize(src);
  if (rc != AQC_OK) return rc;
  dst->zero_pending = false;  // overwritten below
  dst->amp0_ready = false;
  AQC_HIP_CHECK(hipStreamSynchronize(src->stream));
  AQC_HIP_CHECK(hipMemcpyAsync(dst->state, src->state, sizeof(cplx) << dst->n,
                               hipMemcpyDeviceToDevice, dst->stream));
  // the copy reads src on dst's stream: later work on src's stream (an apply that rewrites it,
  // or the synchronisation in aqc_sv_destroy before its block returns to the pool) waits for it
  AQC_HIP_CHECK(hipEventRecord(dst->read_ev, dst->stream));
  AQC_HIP_CHECK(hipStreamWaitEvent(src->stream, dst->read_ev, 0));
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
  h->amp0_ready = false;
  // Planned and launched in batches of 1, 2, 4, ... segments, each segment formed as it is needed
  // (SegBuilder): the host plans the next batch while the GPU runs the previous one, and the first
  // pass starts after one segment's planning (planned whole, the GPU waited out the ~150 us of host
  // segmentation and fusion of a 20-qubit evaluation).  One pinned staging buffer; each batch
  // appends its [headers | phases | gates] contiguously (offsets relative to the batch) and goes
  // over in ONE copy -- a small H2D copy is a ~4 us blit on the stream, three per batch had cost
  // ~40 us per evaluation.  The previous call's copies have finished reading the staging buffer
  // once plan_ev has completed.
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  constexpr size_t kMaxBatches = 40;  // batch sizes double: 2^40 segments
  const size_t cap = sizeof(SegHeader) * (size_t)nops + sizeof(PhaseHdr) * (size_t)nops +
                     sizeof(SegGate) * (size_t)nops + 3 * 256 * kMaxBatches;
  if (cap > h->plan_cap) {
    AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
    if (h->d_plan) AQC_HIP_CHECK(hipFree(h->d_plan));
    if (h->h_plan) AQC_HIP_CHECK(hipHostFree(h->h_plan));
    h->d_plan = nullptr, h->h_plan = nullptr;
    h->plan_cap = std::max(cap, 2 * h->plan_cap);
    AQC_HIP_CHECK(hipMalloc(&h->d_plan, h->plan_cap));
    AQC_HIP_CHECK(hipHostMalloc(&h->h_plan, h->plan_cap, hipHostMallocDefault));
  }
  AQC_HIP_CHECK(hipEventSynchronize(h->plan_ev));
  const int nblocks = (int)(1ull << (h->n - K));
  SegBuilder sb(ops, nops, K, h->n, sv_reserved_bits(h->reg_tiles));
  std::vector<HostSeg> segs;
  std::vector<SegHeader> hdr;
  std::vector<SegGate> gts;
  std::vector<PhaseHdr> phs;
  std::vector<double> flops;
  gts.reserve(nops);
  phs.reserve(nops);
  size_t off = 0;
  int rc = AQC_OK;
  for (size_t batch = 1, nb_done = 0; rc == AQC_OK; batch *= 2, ++nb_done) {
    segs.clear();
    HostSeg seg;
    while (segs.size() < batch && sb.next(seg)) segs.push_back(seg);
    if (segs.empty()) break;
    const size_t nb = segs.size();
    hdr.assign(nb, SegHeader{});
    gts.clear();
    phs.clear();
    flops.clear();
    for (size_t s = 0; s < nb; ++s) sv_plan_one(h->n, K, h->reg_tiles, ops, segs[s], s, hdr, gts, phs, &flops);
    const size_t o_h = off, o_p = al(o_h + sizeof(SegHeader) * nb), o_g = al(o_p + sizeof(PhaseHdr) * phs.size());
    const size_t end = o_g + sizeof(SegGate) * gts.size();
    if (end > h->plan_cap || nb_done >= kMaxBatches) {
      aqc::set_error("aqc_sv_apply: plan exceeds its staging bound");
      rc = AQC_ERR_STATE;
      break;
    }
    std::memcpy(h->h_plan + o_h, hdr.data(), sizeof(SegHeader) * nb);
    if (!phs.empty()) std::memcpy(h->h_plan + o_p, phs.data(), sizeof(PhaseHdr) * phs.size());
    if (!gts.empty()) std::memcpy(h->h_plan + o_g, gts.data(), sizeof(SegGate) * gts.size());
    // (by a copy kernel, aqc::upload_async: the SDMA transfers hipMemcpyAsync used for the larger
    // batches cost ~10-25 us of idle GPU each in the config-2 timeline)
    if (nb_done > 0) {
      // (the batch's plan region is fresh: no pass reads it before the event below)
      hipEvent_t ev = h->up_ev[nb_done & 1];
      AQC_HIP_CHECK(hipMemcpyAsync(h->d_plan + o_h, h->h_plan + o_h, end - o_h, hipMemcpyHostToDevice, h->up_stream));
      AQC_HIP_CHECK(hipEventRecord(ev, h->up_stream));
      AQC_HIP_CHECK(hipStreamWaitEvent(h->stream, ev, 0));
    } else {
      rc = aqc::upload_async(h->d_plan + o_h, h->h_plan + o_h, end - o_h, h->stream);
      if (rc != AQC_OK) break;
    }
    const SegHeader* dh = reinterpret_cast<const SegHeader*>(h->d_plan + o_h);
    const PhaseHdr* dp = reinterpret_cast<const PhaseHdr*>(h->d_plan + o_p);
    const SegGate* dg = reinterpret_cast<const SegGate*>(h->d_plan + o_g);
    // the apply's final segment (no op left to place) hands amp 0 to the pinned buffer
    const bool final_batch = sb.remaining == 0 && h->reg_tiles;
    for (size_t s = 0; s < nb && rc == AQC_OK; ++s) {
      cplx* a0 = final_batch && s + 1 == nb ? h->h_pinned : nullptr;
      rc = sv_launch_segment(h, dh + s, dp, dg, nblocks, a0, flops[s]);
      if (rc == AQC_OK && a0) h->amp0_ready = true;
    }
    off = al(end);
  }
  // (recorded on every path, so the next call never reuses the staging buffer under a live copy)
  AQC_HIP_CHECK(hipEventRecord(h->plan_ev, h->stream));
  return rc;
}

int aqc_sv_plan(int n, const aqc_op_t* ops, int nops, int* out) {
  AQC_REQUIRE(out && n >= 1 && n <= 34 && nops >= 0 && (ops || nops == 0), "aqc_sv_plan: bad arguments");
  for (int i = 0; i < nops; ++i)
    AQC_REQUIRE((ops[i].nq == 1 || ops[i].nq == 2) && ops[i].q0 >= 0 && ops[i].q0 < n &&
                    (ops[i].nq == 1 || (ops[i].q1 >= 0 && ops[i].q1 < n && ops[i].q1 != ops[i].q0)),
                "aqc_sv_plan: bad op");
  const bool reg = sv_reg_tiles(n);
  const int K = reg ? kRegTileBits : (n < 10 ? n : 10);
  std::vector<SegHeader> hdr;
  std::vector<SegGate> gts;
  std::vector<PhaseHdr> phs;
  if (nops > 0) sv_plan(n, K, reg, ops, nops, hdr, gts, phs);
  out[0] = (int)hdr.size();
  out[1] = (int)phs.size();
  out[2] = (int)gts.size();
  out[3] = K;
  return AQC_OK;
}

int aqc_sv_amp0(aqc_sv_t h, double* re, double* im) {
  AQC_REQUIRE(h && re && im, "aqc_sv_amp0: null argument");
  if (int rc = sv_materialize(h)) return rc;
  // after an apply the final pass already wrote it (amp0_ready); otherwise one small copy
  if (!h->amp0_ready)
    AQC_HIP_CHECK(hipMemcpyAsync(h->h_pinned, h->state, sizeof(cplx), hipMemcpyDeviceToHost, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  *re = h->h_pinned[0].x;
  *im = h->h_pinned[0].y;
  return AQC_OK;
}

int aqc_sv_z_all(aqc_sv_t h, double* out) {
  AQC_REQUIRE(h && out, "aqc_sv_z_all: null argument");
  if (int rc = sv_materialize(h)) return rc;
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
  if (int rc = sv_materialize(h)) return rc;
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
  if (int rc = sv_materialize(bra)) return rc;
  if (int rc = sv_materialize(ket)) return rc;
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
  if (int rc = sv_materialize(h)) return rc;
  AQC_HIP_CHECK(hipMemcpyAsync(out, h->state, sizeof(cplx) << h->n, hipMemcpyDeviceToHost, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  return AQC_OK;
}

int aqc_sv_set(aqc_sv_t h, const double* in) {
  AQC_REQUIRE(h && in, "aqc_sv_set: null argument");
  h->zero_pending = false;  // overwritten
  h->amp0_ready = false;
  AQC_HIP_CHECK(hipMemcpyAsync(h->state, in, sizeof(cplx) << h->n, hipMemcpyHostToDevice, h->stream));
  AQC_HIP_CHECK(hipStreamSynchronize(h->stream));
  return AQC_OK;
}

}  // extern "C"
