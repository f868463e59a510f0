/*
 * aqc_hip_diag.h -- diagnostics, lab switches and test hooks of libaqchip.so.
 *
 * Not part of the drop-in boundary (aqc_hip.h): path selection for A/B measurements, per-phase
 * shader-clock ticks, the fast paths' acceptance counters (reported by bench.py), a CU-holding test
 * load, and single-kernel entry points the tests drive against numpy.  Same conventions as
 * aqc_hip.h (AQC_OK / AQC_ERR_*, aqc_last_error()).
 */
#ifndef AQC_HIP_DIAG_H
#define AQC_HIP_DIAG_H

#include "aqc_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostics: largest Jacobi sweep count since the last call (then reset). */
int aqc_mps_jacobi_stats(aqc_mps_t h, int* max_sweeps);
/* Jacobi rotation threshold |a^H b| > factor * L * eps * |a||b| (default factor 1). */
int aqc_mps_set_jacobi_tol(double factor);
/* Jacobi sweep stop: after a sweep whose counted rotations all moved at most tiny_t^2 of their
   pair's squared norms (t |g| <= tiny_t^2 (|a|^2 + |b|^2); |t| <= tiny_t for separated pairs) the
   decomposition ends (default 1e-6; tiny_t <= 0 restores it; must be < 1e-3). */
int aqc_mps_set_jacobi_stop(double tiny_t);
/* Two-site SVD at 2 chi = 128: gram = 1 (default) tries the Gram / tridiagonal path first (G = X^H X
   on the matrix cores, Householder tridiagonalisation, multisection, inverse iteration; taken when
   the kept count K = min(2 chi, max_chi) <= 64 and lambda_K > 1e-9 lambda_1, else the register
   Jacobi runs), gram = 0 the register Jacobi only.  Also AQC_SVD_PATH at load.  debug_max_chi:
   max_chi of aqc_svd_debug. */
int aqc_mps_set_svd_path(int gram, int debug_max_chi);
/* Diagnostics: shader-clock ticks of the Gram path's phases since the last call (then reset);
   out[12]: Gram GEMM, tridiagonalisation, eigenvalues, eigenvectors, back-transformation, output,
   then the tridiagonalisation's column steps, the inverse iteration, the steps' phase A (out[9..11]
   unused, 0). */
int aqc_svd_gram_ticks(double* out);
/* Gram-path counters since the last call (then reset): out[0] two-site SVDs that tried the Gram
   path, out[1] taken, out[2] declined by shape (2 chi != 128), out[3] declined at the
   eigenvalue floor (lambda_K <= 1e-9 lambda_1; the register Jacobi ran instead) or with a
   reduce_zeros decision the eigenvalues' error bars leave open, or with a failed certificate;
   K follows reduce_zeros on the eigenvalues (aqc::gram_keep, up to the whole side).  out[4]
   rank-deficiency certificates run (values in CHOP's error band assumed chopped, then
   ||X - X V V^H||_F^2 < CHOP / 2 checked), out[5] passed.  out[6]. */
int aqc_svd_gram_stats(double* out);
/* The four-workgroup environment chains (z_all / pair RDMs at capacities in multiples of 64):
   shader-clock ticks of one workgroup summed over its steps since the last call -- out[0] the
   T product, out[1] its columns of the new environment, out[2] the hand-off -- and out[3] the
   steps counted.  Resets. */
int aqc_env_ticks(double* out);
/* Environment launches (z_all / pair RDMs) whose split chains timed out on a hand-off -- their
   workgroups were not all resident together -- and were re-run with one workgroup per chain
   (k_rdm_env), since the last call (then reset). */
int aqc_env_fallbacks(long long* out);
/* on = 1: every environment chain on one workgroup (k_rdm_env, any capacity); 0: the default, the
   split chains at capacities 64, 128, 256 and 512. */
int aqc_env_set_single(int on);
/* Hand-off wait limit of the split environment chains in microseconds (< 0: the default, 2 s); 0
   makes every wait not already satisfied a timeout, which re-runs the call on single chains (tests). */
int aqc_env_set_spin_limit(double us);
/* Block Jacobi pair visits (2 chi > 128), shader-clock ticks summed over workgroups since the
 * last call: out[0] Gram, out[1] inner Jacobi sweep, out[2] A V, out[3] visits.  Resets. */
int aqc_bj_ticks(double* out);
/* Two-site SVDs at 2 chi in (128, 1024] (gram_big.hip; replaces the block Jacobi of the reference's
   Aer MPS truncation for chi = 128 ... 512, aer_mps_backend.py:76-78 via qiskit-aer's MPS two-site
   SVD): counters since the last call (then reset): out[0] jobs that entered the multi-workgroup
   Gram path, out[1] taken, out[2] declined (Gram path off for the job, or 2 chi < 4), out[3]
   declined at the eigenvalue floor (lambda_K <= 1e-9 lambda_1), out[4] exchange timeouts (the
   tridiagonalisation's workgroups did not all run together); declined jobs ran the block Jacobi.
   out[3] also counts kept-count decisions that the eigenvalues' error bars leave open (the kept
   count follows reduce_zeros on them: aqc::gram_keep).  out[5] rank-deficient decisions that needed
   the certificate ||X - X V V^H||_F^2 < CHOP / 2, out[6] certified, out[7] not (declined).  out[8].
   The environment variable AQC_BIG_GRAM=0 selects the block Jacobi alone. */
int aqc_svd_gram_big_stats(double* out);
/* Diagnostics of the same path: shader-clock ticks summed over calls (then reset): out[0..4] the
   tridiagonalisation's per-column phases on job 0's first workgroup (register pass + row sums,
   publish, counter wait, reads + p^H v, w / new row / partial norms), out[5] k_gb_eig (job 0),
   out[6] k_gb_back (job 0, first block), out[7] k_gb_inv (job 0, lane 0), out[8] the next
   reflector's zlarfg (per column, job 0's first workgroup). */
int aqc_svd_gram_big_ticks(double* out);
/* Counter-wait limit of the same path's tridiagonalisation in microseconds (< 0: default 100 ms);
   a job whose workgroups wait longer declines to the block Jacobi (out[4] above).  0 forces the
   decline wherever a wait is not already satisfied (tests). */
int aqc_gb_set_spin_limit(double us);
/* The same tridiagonalisation's last 128 columns: in one workgroup (on = 1, the default: the
   trailing block goes to the job's first workgroup, which finishes without the per-column
   exchange), or over all of the job's workgroups to the end (on = 0).  AQC_GB_TAIL=0 also selects 0. */
int aqc_gb_set_tail(int on);
/* With the tail at 2 chi = 512: columns 0 .. 255 over the job's 16 workgroups, then 256 .. 383 over
   4 (n = 2, the default: a round's second stage runs beside the next round's first), or 0 .. 383
   over 16 (n = 1).  AQC_GB_STAGES=1 also selects 1. */
int aqc_gb_set_stages(int n);
/* Test load: nblocks 256-thread workgroups on a private stream, block b spinning (b % 16 + 1) / 16
   of `ms` milliseconds, so work queued on other streams starts one CU at a time.  Asynchronous. */
int aqc_debug_hog(int nblocks, double ms);
/* Device-memory cache of the library (MPS / SV handle buffers): out[0] bytes cached (freed, kept
   for reuse), out[1] bytes handed out, out[2] blocks handed out, out[3] requests served from the
   cache, out[4] requests that went to hipMalloc.  Limit: AQC_POOL_MB (default 8192). */
int aqc_pool_stats(double* out);
/* Batched applies of >= 32 states at 2*chi = 128 run every state's whole op list in
   one fused workgroup (theta, Jacobi, truncation, split per update: no grid-wide step between
   updates); on = 0 selects the lock-step launches per update, on = 2 the fused chain for batches
   of any size (lab: single evaluations).  Default 1. */
int aqc_mps_set_fused_chain(int on);
/* Diagnostics: shader-clock ticks spent by the fused chain's workgroups (thread 0) in theta,
   Jacobi, rank, split and one-site ops since the last call (then reset); out[5]. */
int aqc_mps_chain_ticks(double* out);
/* Diagnostics: one register-resident Jacobi launch with pivoted-QR preconditioning (variant 2)
   on theta (m x n column-major complex, m, n even <= 128, as the two-site update builds it), or
   the Gram / tridiagonal path (variant 7; Jacobi fallback inside the kernel; same output contract).
   w_out receives min(m,n) columns of length min(m,n); sig_out their
   norms; perm_out (optional) the pivot order when stop_after_qr (then w_out holds X = R^H
   unsorted).  stop_after_qr = 2 also writes the QR phase's shader-clock ticks to sig_out[0..3]
   (downdate + pivot key, pivot barrier, reflector + barrier, update; 128 x 128 only).  For tests
   and tools only: allocates and frees device memory per call. */
int aqc_svd_debug(const double* theta, int m, int n, int variant, int stop_after_qr, double* w_out,
                  double* sig_out, int* perm_out, int* sweeps);
/* Chain kernel of the sweep: 0 = automatic (first qubits in groups of 8 advancing together on the
 * matrix cores for batches of states at bond capacity 64 or 128; for a single state the segmented
 * sweep above capacity 64, else one chain per workgroup), 1 = one chain per workgroup, 2 = grouped
 * whenever the capacity allows, 3 = the segmented sweep (prefix / suffix products of the site
 * matrices over ~sqrt(n) segments as batched MFMA GEMMs) for every single state.  Results are the
 * same up to floating-point summation order. */
int aqc_sweep_set_chain_mode(int mode);
#ifdef __cplusplus
}
#endif
#endif /* AQC_HIP_DIAG_H */
