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
struct MpsDev {
  int n = 0;
  int cap = 0;
  cplx* gam = nullptr;
  double* lam = nullptr;
  int* dims = nullptr;
  // two-site workspace
  cplx* theta = nullptr;  // (2cap)^2, column-major M x N
  cplx* work = nullptr;   // (2cap)^2, Jacobi working columns
  double* sig = nullptr;  // 2cap column norms
  int* perm = nullptr;    // 2cap sorted -> column index
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

hipStream_t mps_stream();

}  // namespace aqc

struct aqc_mps_s {
  aqc::MpsDev d;
  double thr = 1e-16;
  int max_chi = 0;
  std::vector<int> order;  // site -> qubit
  std::vector<int> loc;    // qubit -> site
  // scratch for the candidate sweep (grad.hip), allocated lazily
  aqc::cplx* gw = nullptr;
  size_t gw_bytes = 0;
};
