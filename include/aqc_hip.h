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
/* sv[0] (aer_sv_backend.py:29). */
int aqc_sv_amp0(aqc_sv_t h, double* re, double* im);
/* <Z_i> = p0 - p1 for all i (aer_sv_backend.py:49-59), out[n]. */
int aqc_sv_z_all(aqc_sv_t h, double* out);
/* Host copies of the full state (2^n interleaved complex). */
int aqc_sv_get(aqc_sv_t h, double* out);
int aqc_sv_set(aqc_sv_t h, const double* in);

/* ---- MPS: replaces aer_mps_backend.py:27-93 and aqc_research.mps_operations ----- */
/* |0...0> on n qubits, bond capacity chi_cap (1 ... 1024); truncation as mps_sim_with_args
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
/* As aqc_mps_apply_batch (no sort), returning once the work is queued; flags as above.  The
   cached Rotoselect evaluator advances its prefix with it (one host wait per gate instead of three). */
int aqc_mps_apply_batch_async(aqc_mps_t* hs, int nstates, const aqc_op_t* const* ops, const int* nops);
/* Wait for the states' queued work and report their error flags (AQC_ERR_STATE etc.). */
int aqc_mps_check_batch(aqc_mps_t* hs, int nstates);
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

/* move_all_qubits_to_sorted_ordering (done implicitly by every measurement below). */
int aqc_mps_sort(aqc_mps_t h);
int aqc_mps_sort_batch(aqc_mps_t* hs, int nstates);
/* mps_dot(psi, zero_mps) = <psi|0...0> (aer_mps_backend.py:49-57).  The states' error flags are
   read with the result (AQC_ERR_STATE as aqc_mps_check_batch: work queued by the async applies). */
int aqc_mps_overlap_zero(aqc_mps_t h, double* re, double* im);
int aqc_mps_overlap_zero_batch(aqc_mps_t* hs, int nstates, double* out /* 2*nstates */);
/* mps_dot(a, b) = <a|b>, conjugating a. */
int aqc_mps_dot(aqc_mps_t a, aqc_mps_t b, double* re, double* im);
/* mps_expectation(psi, "Z", i) for all i (aer_mps_backend.py:80-86), out[n]. */
int aqc_mps_z_all(aqc_mps_t h, double* out);
/* extract_amplitude(psi, 2**i) for all i (aer_mps_backend.py:88-93), out[2n]. */
int aqc_mps_amps_hw1(aqc_mps_t h, double* out);
/* Batched forms for many states of the same n (and, for z_all, the same capacity): one set of
   launches for every state -- the softened global cost (aer_mps_backend.py:58-70) and the local cost
   (:72-74, 80-86) of a Rotoselect gate's candidates (cost_minimiser.py:318-368).  out: nstates x n
   doubles (<Z_i>) or nstates x 2n (complex amplitudes).  z_all_batch contracts the left / right
   environments as matrix products (the ISL RDM machinery) instead of aqc_mps_z_all's per-site
   chains; both are full contractions (no canonical form assumed). */
int aqc_mps_z_all_batch(aqc_mps_t* hs, int nstates, double* out);
int aqc_mps_amps_hw1_batch(aqc_mps_t* hs, int nstates, double* out);
/* out[s] = sum_i <Z_i> of hs[s] (sorted first, as z_all_batch) -- the local cost
   0.5 (1 - mean <Z_i>) (aer_mps_backend.py:72-74, 80-86) needs only the sum.  A state copied from
   `base` (aqc_mps_copy / aqc_mps_copy_batch) while base has not changed since contracts only the
   sites it rewrote, against environment pairs of the operator sum_i Z_i cached on base (extended
   as base changes: the Rotoselect prefix of cost_minimiser.py:318-368); any other state takes the
   full chains of z_all_batch.  base itself is not modified and must not be among hs. */
int aqc_mps_z_sum_batch(aqc_mps_t base, aqc_mps_t* hs, int nstates, double* out);
/* <psi|0..0> (out_ov: 2 doubles per state, as aqc_mps_overlap_zero_batch) and, when out_amps is not
   null, <e_i|psi> (2 n doubles per state, as aqc_mps_amps_hw1_batch) -- the global and softened
   costs (aer_mps_backend.py:49-70, 88-93) of a Rotoselect gate's candidates: a state copied from
   `base` while base has not changed since contracts only the sites it rewrote, against zero and
   Hamming-weight-1 rows cached on base; any other state takes the full chains.  base is not
   modified and must not be among hs.  The states' and base's error flags are read with the
   results (as aqc_mps_check_batch would: AQC_ERR_STATE on a capacity overflow of queued work). */
int aqc_mps_zero_hw1_batch(aqc_mps_t base, aqc_mps_t* hs, int nstates, double* out_ov, double* out_amps);

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
/* The same rule for each of nrows score rows at once (row r at scores + r * ld), all pointers on the
 * device, queued on the library's stream without a host wait (order it with aqc_stream_wait /
 * aqc_stream_join): out[r] = row r's arg-max index (as a double), out[nrows + r] = its scaled score
 * -- the per-state selection of a batch of sweeps, laid out for one all-gather. */
int aqc_argmax_scaled_batch(const double* scores, int ld, const double* prio, int count, int nrows,
                            double* out);

/* Diagnostics, lab switches and test hooks (path selection, phase ticks, path counters, a CU-holding
   test load, the SVD kernel on its own) are declared in aqc_hip_diag.h: they are not part of the
   drop-in boundary. */

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
