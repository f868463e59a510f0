// Internal helpers shared by the libaqchip translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/aqc_hip.h"
#include "../../include/aqc_hip_diag.h"

namespace aqc {

void set_error(const std::string& msg);

#define AQC_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) {                                                              \
      ::aqc::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));               \
      return AQC_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define AQC_CHECK_LAUNCH()                                                               \
  do {                                                                                   \
    hipError_t _e = hipGetLastError();                                                   \
    if (_e != hipSuccess) {                                                              \
      ::aqc::set_error(std::string("kernel launch: ") + hipGetErrorString(_e));          \
      return AQC_ERR_HIP;                                                                \
    }                                                                                    \
  } while (0)

#define AQC_REQUIRE(cond, msg)                                                           \
  do {                                                                                   \
    if (!(cond)) {                                                                       \
      ::aqc::set_error(msg);                                                             \
      return AQC_ERR_ARG;                                                                \
    }                                                                                    \
  } while (0)

// ---- complex double helpers ----------------------------------------------------------
typedef double2 cplx;

__host__ __device__ __forceinline__ cplx cmk(double r, double i) { return make_double2(r, i); }
__host__ __device__ __forceinline__ cplx cadd(cplx a, cplx b) { return cmk(a.x + b.x, a.y + b.y); }
__host__ __device__ __forceinline__ cplx csub(cplx a, cplx b) { return cmk(a.x - b.x, a.y - b.y); }
__host__ __device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return cmk(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// a * conj(b)
__host__ __device__ __forceinline__ cplx cmulc(cplx a, cplx b) {
  return cmk(fma(a.x, b.x, a.y * b.y), fma(a.y, b.x, -a.x * b.y));
}
// conj(a) * b
__host__ __device__ __forceinline__ cplx cconjmul(cplx a, cplx b) {
  return cmk(fma(a.x, b.x, a.y * b.y), fma(a.x, b.y, -a.y * b.x));
}
// acc += a*b
__host__ __device__ __forceinline__ cplx cfma(cplx a, cplx b, cplx acc) {
  return cmk(fma(a.x, b.x, fma(-a.y, b.y, acc.x)), fma(a.x, b.y, fma(a.y, b.x, acc.y)));
}
// acc += conj(a)*b
__host__ __device__ __forceinline__ cplx cfmac(cplx a, cplx b, cplx acc) {
  return cmk(fma(a.x, b.x, fma(a.y, b.y, acc.x)), fma(a.x, b.y, fma(-a.y, b.x, acc.y)));
}
__host__ __device__ __forceinline__ cplx cscale(cplx a, double s) { return cmk(a.x * s, a.y * s); }
__host__ __device__ __forceinline__ cplx cconj(cplx a) { return cmk(a.x, -a.y); }
__host__ __device__ __forceinline__ double cnorm2(cplx a) { return fma(a.x, a.x, a.y * a.y); }

// Lane permutation of a double within DPP rows (CTRL: quad_perm / row_ror), as two 32-bit
// v_mov_b32_dpp with no "old" operand (every lane of these patterns reads a valid source).
template <int CTRL>
__device__ __forceinline__ double dpp_perm(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// Loads through a pointer known to address global memory.  Pointers read out of job structs
// are generic, so the compiler emits FLAT loads, which also count on LGKM_CNT: every LDS wait
// (and every barrier) then drains them too, and a prefetch issued ahead of a barrier stalls
// there.  GLOBAL loads count on VM_CNT only.
// (through double pointers: a cast of the HIP vector type's pointer is lost again in its copy
// constructor, which takes a generic reference)
typedef __attribute__((address_space(1))) double gdouble;
__device__ __forceinline__ cplx ldg(const cplx* p) {
  const gdouble* q = (const gdouble*)(const double*)p;
  return cmk(q[0], q[1]);
}
__device__ __forceinline__ double ldg(const double* p) { return *(const gdouble*)p; }
__device__ __forceinline__ void stg(cplx* p, cplx v) {
  gdouble* q = (gdouble*)(double*)p;
  q[0] = v.x;
  q[1] = v.y;
}
__device__ __forceinline__ void stg(double* p, double v) { *(gdouble*)p = v; }

// Raw buffer loads: a uniform (SGPR) resource + one 32-bit lane offset + a uniform SGPR offset,
// so a run of loads at uniform strides holds one VGPR of addressing instead of a 64-bit address
// each.  Offsets past `bytes` (lane offset + instruction offset) read as zero.  0x00020000 is the
// gfx9 data-format word of the resource.
// Per-job grids laid out so that a job's workgroups share one XCD (and its L2) under the
// dispatcher's round-robin placement: a 1-D grid of nblk x njp blocks, block id = job + njp blk,
// njp = nj rounded up to 8.  With `fair` set, njp = nj itself below 8 jobs: a job's blocks then
// cycle over 8 / gcd(nj, 8) XCDs, its share of the chip -- for jobs of many more workgroups than
// one XCD has CUs (one pair-RDM state's 147 chains on one XCD ran 2.5x slower; the lock-step
// per-job kernels measured no better either way, profiles/r5_xcd_fair_ab.json, and keep the
// plain rule).  False for the padding's blocks (whole workgroups: return at once).  Placement
// is a speed matter only.
__host__ __device__ __forceinline__ int xcd_pad(int nj, bool fair = false) {
  return fair && nj < 8 ? nj : (nj + 7) & ~7;
}
__device__ __forceinline__ bool xcd_job_block(int nj, int& job, int& blk, bool fair = false) {
  const int njp = xcd_pad(nj, fair);
  job = (int)blockIdx.x % njp;
  blk = (int)blockIdx.x / njp;
  return job < nj;
}
inline unsigned xcd_grid(int nblk, int nj, bool fair = false) {
  return (unsigned)nblk * (unsigned)xcd_pad(nj, fair);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ cplx buf_ld(__amdgpu_buffer_rsrc_t r, unsigned lane_off, unsigned uni_off) {
  return __builtin_bit_cast(cplx, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, uni_off, 0));
}

// Sum over the 16 lanes of a DPP row, result in every lane of the row -- bit-identical in every
// lane: with quad sums Q0..Q3, row_ror:8 first gives {Q0+Q2, Q1+Q3} in every lane (up to the order
// of one commutative add) and row_ror:4 then their sum, whereas row_ror:4 first associates the
// quads differently in alternate quads.  Callers branch on the sum (the Jacobi's rotation sign
// for near-degenerate pairs), so lanes must agree.  Pure VALU (DPP quad_perm / row_ror), no LDS
// crossbar: ~2.5x cheaper than the ds_bpermute __shfl_xor path.
__device__ __forceinline__ double row_sum16(double v) {
  v += dpp_perm<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_perm<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_perm<0x128>(v);  // row_ror:8
  v += dpp_perm<0x124>(v);  // row_ror:4
  return v;
}

// Sums over aligned groups of 8 / 4 lanes: the quad steps, then row_half_mirror (lane i of a
// half-row reads lane 7 - i) joins the two quads of a half-row.
__device__ __forceinline__ double row_sum8(double v) {
  v += dpp_perm<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_perm<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_perm<0x141>(v);  // row_half_mirror
  return v;
}
__device__ __forceinline__ double row_sum4(double v) {
  v += dpp_perm<0xB1>(v);
  v += dpp_perm<0x4E>(v);
  return v;
}
// Sum over an aligned group of LPG (4, 8 or 16) lanes, result in every lane of the group.
template <int LPG>
__device__ __forceinline__ double group_sum(double v) {
  if constexpr (LPG == 4) return row_sum4(v);
  else if constexpr (LPG == 8) return row_sum8(v);
  else return row_sum16(v);
}

// ---- teardown ----------------------------------------------------------------------------
// Lazily created HIP objects (side streams, events, cached buffer sets) register a cleanup here
// when they are first created; aqc_finalize synchronises every device the library touched, runs
// the cleanups (newest first) and forgets them, so the objects are recreated on next use.  The
// Python loader calls aqc_finalize from atexit, before the HIP runtime's own teardown.
void on_finalize(void (*fn)());
void note_device(int dev);

// Host -> device copy of a pinned (hipHostMalloc) staging buffer on `st`, done by a kernel that
// reads the host memory over the bus: the stream's next kernel then depends on a kernel, not on a
// copy-engine transfer (each of those cost ~10-25 us of idle GPU in the measured timelines,
// profiles/r4_cfg2_timeline_gaps.json).  hipMemcpyAsync below AQC_UPLOAD_MIN_KB (16) and for
// unaligned pointers; AQC_UPLOAD=memcpy selects it everywhere (A/B).
int upload_async(void* dst, const void* pinned_src, size_t bytes, hipStream_t st);

// ---- cached device memory ------------------------------------------------------------------
// Blocks freed by the library go to a per-device free list keyed by size (4 KB granules) and are
// handed out again to the next request of that size: handle creation and destruction (a batched
// Rotoselect gate creates and drops its candidate states) cost a list lookup instead of hipMalloc /
// hipFree, whose implicit device synchronisation took ~0.25 ms per MPS handle.  Unlike hipFree,
// dev_free does not synchronise: the caller frees only memory that no queued work on any stream
// still uses.  Each handle's destroy drains its own stream first, and every kernel or copy that
// reads a handle's buffers on another stream (aqc_sv_copy) makes the owner's stream wait on an
// event recorded after it, so that drain covers the reader too.  The cache holds at most
// AQC_POOL_MB (default 8192) MB; an allocation that fails first releases the cache and retries.
// aqc_finalize returns every cached block to the runtime.
void* dev_alloc(size_t bytes);
void dev_free(void* p);

// ---- kernel timing (HIP events on the launching stream) ------------------------------
struct KernelTimer {
  // Begin/End bracket one launch on `stream` when timing is enabled.
  static void begin(hipStream_t stream, const char* family, double bytes, double flops);
  static void end(hipStream_t stream);
};

}  // namespace aqc
