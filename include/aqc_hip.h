/*
 * aqc_hip.h -- C ABI of libaqchip.so, the MI355X (gfx950) engine behind the
 * adaptaqc_amd backends.
 *
 * Every entry point replaces a specific reference call site (qiskit-community/adapt-aqc,
 * paths relative to the reference root); the arithmetic those call sites delegated to
 * qiskit-aer ~=0.16.0 and aqc_research.mps_operations runs here in hand-written HIP.
 *
 * Conventions
 *   - return value: AQC_OK (0) or a negative AQC_ERR_*; aqc_last_error() gives a
 *     thread-local message for the last failure.
 *   - complex numbers are interleaved (re, im) doubles; matrices are row-major.
 *   - gate matrices follow Qiskit: for an op on qubits (q0, q1) the row/column index is
 *     2*b1 + b0 (b0 = bit of q0).
 *   - handles own their device memory and one HIP stream; a handle is not re-entrant.
 *   - *_batch entry points take arrays of handles and run them in lock-step launches
 *     (one kernel launch serves every handle), so independent evaluations fill the GPU.
 */
#ifndef AQC_HIP_H
#define AQC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AQC_OK 0
#define AQC_ERR_ARG (-1)
#define AQC_ERR_HIP (-2)
#define AQC_ERR_STATE (-3)
#define AQC_ERR_UNSUPPORTED (-4)
#define AQC_ERR_NOMEM (-5)

/* One gate.  nq = 1: m[0..7] holds the 2x2 matrix; nq = 2: m[0..31] the 4x4 matrix. */
typedef struct aqc_op {
  int32_t nq;
  int32_t q0;
  int32_t q1;
  int32_t flags; /* reserved, 0 */
  double m[32];
} aqc_op_t;

typedef struct aqc_sv_s* aqc_sv_t;
typedef struct aqc_mps_s* aqc_mps_t;
typedef struct aqc_comm_s* aqc_comm_t;

/* ---- library -------------------------------------------------------------------- */
const char* aqc_last_error(void);
int aqc_version(void);
/* Select the HIP device used by handles created afterwards (hipSetDevice). */
int aqc_init(int device);
int aqc_finalize(void);
/* Kernel-time instrumentation: accumulate HIP-event time of the named kernel family
 * ("sv_segment", "mps_svd", "grad_chain", ...) issued after the call. */
int aqc_timing_enable(int on);
int aqc_timing_query(const char* name, double* total_ms, int64_t* launches, double* bytes,
                     double* flops);
int aqc_timing_reset(void);

/* ---- statevector: replaces aer_sv_backend.py:37-59 ---------------------------- */
/* Allocate |0...0> on n qubits (Aer statevector_simulator state). */
int aqc_sv_create(int n, aqc_sv_t* out);
int aqc_sv_destroy(aqc_sv_t h);
int aqc_sv_reset(aqc_sv_t h);
int aqc_sv_copy(aqc_sv_t dst, const aqc_sv_t src);
/* Apply ops in order (aer_sv_backend.py:42-47 simulator.run(full_circuit)).  Gates are
 * fused on the host into qubit-local segments: 10-bit LDS tiles below 14 qubits, 12-bit
 * register-resident tiles (4-bit phases) from 14 qubits. */
int aqc_sv_apply(aqc_sv_t h, const aqc_op_t* ops, int nops);
/* Host planning of aqc_sv_apply only (no GPU): out[0] segments (= launches), out[1] phases
 * (register-tile path; 0 otherwise), out[2] fused gates, out[3] tile bits. */
int aqc_sv_plan(int n, const aqc_op_t* ops, int nops, int* out);
/* Slots per phase of the register-tile kernel (n >= 14): 4 (default; 256 threads x 16 amplitudes
   per 4096-amplitude tile) or 3 (512 threads x 8: two waves per SIMD at n = 20, more phases).
   Also AQC_SV_SLOTS at first use.  Results equal up to summation order. */
int aqc_sv_set_slots(int slots);
/* sv[0] (aer_sv_backend.py:29). */
int aqc_sv_amp0(aqc_sv_t h, double* re, double* im);
/* <Z_i> = p0 - p1 for all i (aer_sv_backend.py:49-59), out[n]. */
int aqc_sv_z_all(aqc_sv_t h, double* out);
/* Host copies of the full state (2^n interleaved complex). */
int aqc_sv_get(aqc_sv_t h, double* out);
int aqc_sv_set(aqc_sv_t h, const double* in);

/* ---- MPS: replaces aer_mps_backend.py:27-93 and aqc_research.mps_operations ----- */
/* |0...0> on n qubits, bond capacity chi_cap; truncation as mps_sim_with_args
 * (aer_mps_backend.py:27-42): threshold on the discarded tail sum of s^2, max_chi <= 0
 * means unlimited (bounded by chi_cap). */
int aqc_mps_create(int n, int chi_cap, double threshold, int max_chi, aqc_mps_t* out);
int aqc_mps_destroy(aqc_mps_t h);
int aqc_mps_set_truncation(aqc_mps_t h, double threshold, int max_chi);
/* Load Aer-format Vidal MPS (set_matrix_product_state, approximate_compiler.py:180-204):
 * dims[n+1] bond dims (dims[0] = dims[n] = 1); gammas: for site i, 2*dims[i]*dims[i+1]
 * complex laid out [s][l][r]; lambdas: for bond i < n-1, dims[i+1] doubles. */
int aqc_mps_set_vidal(aqc_mps_t h, const int* dims, const double* gammas, const double* lambdas);
/* Export (save_matrix_product_state): sorts qubits first.  Pass NULL to query dims. */
int aqc_mps_get_vidal(aqc_mps_t h, int* dims, double* gammas, double* lambdas);
int aqc_mps_get_dims(aqc_mps_t h, int* dims);
int aqc_mps_copy(aqc_mps_t dst, const aqc_mps_t src);
/* Batched aqc_mps_copy (dst[s] <- src[s], same n and capacity): one launch for every state --
   the per-evaluation reload of the cached MPS (reference: every cost evaluation re-runs
   full_circuit, whose first instruction is set_matrix_product_state, aer_mps_backend.py:76-78;
   the instruction is built at approximate_compiler.py:181-184). */
int aqc_mps_copy_batch(aqc_mps_t* dst, const aqc_mps_t* src, int nstates);
/* Apply ops with Aer MPS semantics (swap-left routing, lazy qubit order, two-site SVD with
 * reduce_zeros truncation) -- the replay inside mps_from_circuit (aer_mps_backend.py:76-78). */
int aqc_mps_apply(aqc_mps_t h, const aqc_op_t* ops, int nops);
int aqc_mps_apply_batch(aqc_mps_t* hs, int nstates, const aqc_op_t* const* ops, const int* nops);
/* As aqc_mps_apply_batch, then move every state back to sorted qubit order in the same schedule
   -- one evaluation's replay + save of mps_from_circuit (aer_mps_backend.py:76-78), so that a
   state's swaps back run in the same fused chain as its gates. */
int aqc_mps_apply_sort_batch(aqc_mps_t* hs, int nstates, const aqc_op_t* const* ops, const int* nops);
/* As aqc_mps_apply_sort_batch, but returns once the work is queued: the states' error flags
   (capacity, Jacobi sweep limit) are not read back -- call aqc_mps_check_batch before using the
   results.  Lets the host prepare further work (the candidate sweep) while the chain runs. */
int aqc_mps_apply_sort_batch_async(aqc_mps_t* hs, int nstates, const aqc_op_t* const* ops, const int* nops);
/* Wait for the states' queued work and report their error flags (AQC_ERR_STATE etc.). */
int aqc_mps_check_batch(aqc_mps_t* hs, int nstates);
/* Diagnostics: largest Jacobi sweep count since the last call (then reset). */
int aqc_mps_jacobi_stats(aqc_mps_t h, int* max_sweeps);
/* Jacobi rotation threshold |a^H b| > factor * L * eps * |a||b| (default factor 1). */
/* Register / block Jacobi: dot-product noise floor of the rotations in units of eps ||W|| (|a| + |b|)
 * (default 0: the relative threshold alone). */
int aqc_mps_set_jacobi_noise(double factor);
int aqc_mps_set_jacobi_tol(double factor);
/* Jacobi sweep stop: after a sweep whose counted rotations all moved at most tiny_t^2 of their
   pair's squared norms (t |g| <= tiny_t^2 (|a|^2 + |b|^2); |t| <= tiny_t for separated pairs) the
   decomposition ends (default 1e-6; tiny_t <= 0 restores it; must be < 1e-3). */
int aqc_mps_set_jacobi_stop(double tiny_t);
/* Two-site SVD at 2 chi = 128: gram = 1 (default) tries the Gram / tridiagonal path first (G = X^H X
   on the matrix cores, Householder tridiagonalisation, multisection, inverse iteration; taken when
   the kept count K = min(2 chi, max_chi) <= 64 and lambda_K > 1e-9 lambda_1, else the register
   Jacobi runs), gram = 0 the register Jacobi only, gram = 2 the Gram path with the lower-triangle
   tridiagonalisation (svd_tri.h's stages on the 1024-thread workgroup).  debug_max_chi: max_chi of
   aqc_svd_debug. */
int aqc_mps_set_svd_path(int gram, int debug_max_chi);
/* Diagnostics: shader-clock ticks of the Gram path's phases since the last call (then reset);
   out[12]: Gram GEMM, tridiagonalisation, eigenvalues, eigenvectors, back-transformation, output,
   then the tridiagonalisation's column steps, the inverse iteration, the steps' phase A, and two
   diagnostics of a build with AQC_S3_DIAG (else 0). */
int aqc_svd_gram_ticks(double* out);
/* Gram-path counters since the last call (then reset): out[0] two-site SVDs that tried the Gram
   path, out[1] taken, out[2] declined by shape (K > 64, 2 chi != 128), out[3] declined at the
   eigenvalue floor (lambda_K <= 1e-9 lambda_1; the register Jacobi ran instead).  out[4]. */
int aqc_svd_gram_stats(double* out);
/* Block Jacobi pair visits (2 chi > 128), shader-clock ticks summed over workgroups since the
 * last call: out[0] Gram, out[1] inner Jacobi sweep, out[2] A V, out[3] visits.  Resets. */
int aqc_bj_ticks(double* out);
/* Two-site SVDs at 2 chi in (128, 1024] (gram_big.hip; replaces the block Jacobi of the reference's
   Aer MPS truncation for chi = 128 ... 512, aer_mps_backend.py:76-78 via qiskit-aer's MPS two-site
   SVD): counters since the last call (then reset): out[0] jobs that entered the multi-workgroup
   Gram path, out[1] taken, out[2] declined (Gram path off for the job, or 2 chi < 4), out[3]
   declined at the eigenvalue floor (lambda_K <= 1e-9 lambda_1), out[4] exchange timeouts (the
   tridiagonalisation's workgroups did not all run together); declined jobs ran the block Jacobi.
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
/* The fused chain's workgroup: 1024 threads, one state per CU (k_chain, default), or 256 threads,
   two states per CU (k_chain256: lower-triangle Gram SVD; a state whose Gram path declines finishes
   its list on k_chain).  Also AQC_CHAIN=256 at load.  Other values: AQC_ERR_ARG. */
int aqc_mps_set_chain_threads(int threads);
/* Diagnostics: shader-clock ticks spent by the fused chain's workgroups (thread 0) in theta,
   Jacobi, rank, split and one-site ops since the last call (then reset); out[5]. */
int aqc_mps_chain_ticks(double* out);
/* ---- ISL entanglement sweep (adapt_compiler.py:955-976 -> entanglement_measures.py:39-98) ----
   Two-qubit reduced density matrices for npairs pairs (pairs[2p], pairs[2p+1]), out = npairs x
   4 x 4 complex (row-major), row index 2*bit(max) + bit(min) as qiskit's partial_trace orders
   the remaining qubits.  SV: entanglement_measures.py:326-340.  MPS: the contraction of
   aqc_research.mps_operations.partial_trace (sorts qubits first); the batch version writes
   nstates x npairs x 16 complex, to device memory when out_is_device. */
int aqc_sv_pair_rdms(aqc_sv_t h, const int* pairs, int npairs, double* out);
int aqc_mps_pair_rdms(aqc_mps_t h, const int* pairs, int npairs, double* out);
int aqc_mps_pair_rdms_batch(aqc_mps_t* hs, int nstates, const int* pairs, int npairs, double* out,
                            int out_is_device);
/* Cached Rotoselect / Rotosolve (replaces the 3-7 full simulations per gate of
   cost_minimiser.py:318-368): out = 2x2 complex T[a][b] = <bra| (|a><b|)_q |ket>, so that
   <bra|V_q|ket> = sum_ab V[a][b] T[a][b] for any single-qubit V. */
int aqc_sv_transition(aqc_sv_t bra, aqc_sv_t ket, int q, double* out);
/* Measures of count 4x4 density matrices (entanglement_measures.py:245-306): method 0 =
   concurrence (EM_TOMOGRAPHY_CONCURRENCE), 1 = entanglement of formation, 2 = negativity,
   3 = log-negativity.  rdms / out in device memory when on_device. */
int aqc_entanglement_measures(const double* rdms, int count, int method, double* out, int on_device);

/* Diagnostics: one register-resident Jacobi launch with pivoted-QR preconditioning (variant 2)
   on theta (m x n column-major complex, m, n even <= 128, as the two-site update builds it), or
   the Gram / tridiagonal path (variant 7; Jacobi fallback inside the kernel; same output contract;
   variant 8: its 256-thread form, declines reported in the flags; variant 9: the 1024-thread form
   with the lower-triangle tridiagonalisation).
   w_out receives min(m,n) columns of length min(m,n); sig_out their
   norms; perm_out (optional) the pivot order when stop_after_qr (then w_out holds X = R^H
   unsorted).  stop_after_qr = 2 also writes the QR phase's shader-clock ticks to sig_out[0..3]
   (downdate + pivot key, pivot barrier, reflector + barrier, update; 128 x 128 only).  For tests
   and tools only: allocates and frees device memory per call. */
int aqc_svd_debug(const double* theta, int m, int n, int variant, int stop_after_qr, double* w_out,
                  double* sig_out, int* perm_out, int* sweeps);
/* move_all_qubits_to_sorted_ordering (done implicitly by every measurement below). */
int aqc_mps_sort(aqc_mps_t h);
int aqc_mps_sort_batch(aqc_mps_t* hs, int nstates);
/* mps_dot(psi, zero_mps) = <psi|0...0> (aer_mps_backend.py:49-57). */
int aqc_mps_overlap_zero(aqc_mps_t h, double* re, double* im);
int aqc_mps_overlap_zero_batch(aqc_mps_t* hs, int nstates, double* out /* 2*nstates */);
/* mps_dot(a, b) = <a|b>, conjugating a. */
int aqc_mps_dot(aqc_mps_t a, aqc_mps_t b, double* re, double* im);
/* mps_expectation(psi, "Z", i) for all i (aer_mps_backend.py:80-86), out[n]. */
int aqc_mps_z_all(aqc_mps_t h, double* out);
/* extract_amplitude(psi, 2**i) for all i (aer_mps_backend.py:88-93), out[2n]. */
int aqc_mps_amps_hw1(aqc_mps_t h, double* out);

/* ---- candidate sweep: replaces gradients.py:23-124 ------------------------------ */
/* For every pair (pairs[2p], pairs[2p+1]) = (control, target):
 *   g_p = sqrt( sum_k degs[k] * ( -Im( <s|G_k|psi> <psi|U0^dag|s> ) )^2 )
 * |s> is the product state with per-qubit 2-vectors svec[n][2] (complex); u0 and gens are
 * 4x4 (little-endian over (control, target)) matrices of U0 and G_k (NOT their inverses).
 * out: npairs doubles; out_is_device != 0 means `out` is a device pointer (for RCCL).
 * With a host `out` the call returns when the scores are there; with a device `out` it returns
 * once the work is queued on the library's stream: aqc_stream_join orders another stream (the
 * caller's, e.g. the all-gather's) after it, and aqc_stream_wait (called before) orders the sweep
 * after the caller's earlier work on `out`. */
int aqc_pair_grads(aqc_mps_t psi, const double* svec, const int* pairs, int npairs,
                   const double* u0, const double* gens, const double* degs, int ngen,
                   double* out, int out_is_device);
int aqc_pair_grads_batch(aqc_mps_t* psis, int nstates, const double* svec, const int* pairs,
                         int npairs, const double* u0, const double* gens, const double* degs,
                         int ngen, double* out /* nstates*npairs */, int out_is_device);
/* Chain kernel of the sweep: 0 = automatic (first qubits in groups of 8 advancing together on the
 * matrix cores for batches of states at bond capacity 64 or 128; for a single state the segmented
 * sweep above capacity 64, else one chain per workgroup), 1 = one chain per workgroup, 2 = grouped
 * whenever the capacity allows, 3 = the segmented sweep (prefix / suffix products of the site
 * matrices over ~sqrt(n) segments as batched MFMA GEMMs) for every single state.  Results are the
 * same up to floating-point summation order. */
int aqc_sweep_set_chain_mode(int mode);
/* Orders `stream` (a hipStream_t of the current device; NULL = the legacy default stream) after
   everything queued so far on the library's stream of that device, without a host wait. */
int aqc_stream_join(void* stream);
/* The reverse order: the library's stream of the current device waits for everything queued so far
 * on `stream`, without a host wait.  A device-output sweep (out_is_device) is ordered both ways by
 * calling aqc_stream_wait(caller) before it -- so the sweep's writes to `out` follow the caller's
 * earlier kernels on that buffer (a fill, the previous step's reads) -- and aqc_stream_join(caller)
 * after it, so the caller's later kernels see the scores. */
int aqc_stream_wait(void* stream);
/* Best product-state (chi = 1) approximation of psi: the starting circuit
 * starting_circuit="tenpy_product_state" (approximate_compiler.py:222-242, which compresses with
 * tenpy's variational method: trunc_params chi_max = 1, min_sweeps 10, max_sweeps 50).  Alternating
 * two-site updates maximise |<s|psi>| (each pair's optimum is the top singular pair of its 2 x 2
 * environment tensor); a sweep is a left-to-right and a right-to-left pass; the fit stops after
 * min_sweeps once a sweep changes the fidelity by <= tol (relative), or after max_sweeps.
 * svec: n x 2 complex per-qubit vectors (in: initial guess unless guess_from_gamma != 0, which
 * starts from the chi = 1 truncation of the canonical form; out: the fit).  fidelity = |<s|psi>|^2
 * (psi normalised). */
int aqc_mps_product_fit(aqc_mps_t psi, double* svec, int guess_from_gamma, int min_sweeps, int max_sweeps,
                        double tol, double* fidelity, int* sweeps);
/* np.argmax(scores * priorities) with lowest-index tie-break (adapt_compiler.py:832-837).  Device
 * scores are read on the library's stream: order it after their producer (aqc_stream_wait). */
int aqc_argmax_scaled(const double* scores, const double* prio, int count, int scores_is_device,
                      int* best);

/* ---- multi-GPU exchange over RCCL ---------------------------------------------
 * The candidate sweep shards the coupling-map pairs across ranks (one process per GPU); its one
 * exchange is an all-gather of the per-pair scores, after which every rank takes the same arg-max
 * (adapt_compiler.py:832-856 -- the reference has no collective: it runs on one host).  For
 * callers without torch.distributed.  aqc_comm_unique_id on one rank, its 128 bytes passed to
 * every rank by the caller's own channel, then aqc_comm_init(id, rank, world) on every rank
 * (collective; the current device, see aqc_init).  Collectives run on the library's stream:
 * aqc_allgather_f64 takes device buffers (send: count doubles, recv: world x count, rank order)
 * and returns once queued, ordered after the library's earlier work (a device-output sweep);
 * aqc_allgather_f64_host / aqc_allreduce_max_f64 take host memory and return complete. */
int aqc_comm_unique_id(char* out /* 128 bytes */);
int aqc_comm_init(const char* unique_id, int rank, int world, aqc_comm_t* out);
int aqc_comm_destroy(aqc_comm_t c);
int aqc_comm_rank(aqc_comm_t c, int* rank, int* world);
int aqc_allgather_f64(aqc_comm_t c, const double* send, double* recv, size_t count);
int aqc_allgather_f64_host(aqc_comm_t c, const double* send, double* recv, size_t count);
int aqc_allreduce_max_f64(aqc_comm_t c, double* value);

#ifdef __cplusplus
}
#endif
#endif /* AQC_HIP_H */
