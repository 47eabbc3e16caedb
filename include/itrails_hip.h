/*
 * itrails_hip.h — C ABI of the MI355X (gfx950) coalescent-HMM decoding core.
 *
 * The reference (trails-phylogeny/itrails) has no FFI: its hot path is a Python call layer.
 * Every entry point below replaces one reference function; the host wrapper
 * (itrails_amd/hmm.py, itrails_amd/model.py) keeps the reference signatures and calls these
 * through ctypes.  Reference files are cited relative to /root/reference/src/itrails/.
 *
 * Conventions
 *  - Plain C types only: pointers + sizes; no torch / HIP types in the signatures.
 *  - `d_` pointers are DEVICE pointers (HBM-resident, e.g. torch.cuda tensors' data_ptr());
 *    `h_` pointers are host pointers.  `stream` is a hipStream_t passed as void* (NULL =
 *    the default stream of the current device).
 *  - Every function returns 0 on success and a non-zero ITR_E* code on failure; the message
 *    of the last failure on this thread is itr_last_error().  Nothing aborts the process.
 *  - Device selection follows the HIP current device of the calling thread (one process per
 *    GPU; multi-GPU sharding and the RCCL log-likelihood all-reduce live in the host layer,
 *    itrails_amd/distributed.py).
 *  - Observed columns are uint16 symbols 0..624 of the 625-letter alphabet of
 *    read_data.py:6-24 (0..255 = A/C/T/G^4 in species order, 256..624 contain N).
 *  - Hidden states: 1 <= N <= 192 (n_int up to 8+8; Viterbi back-pointers are uint8).
 */
#ifndef ITRAILS_HIP_H
#define ITRAILS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ITR_API __attribute__((visibility("default")))

#define ITR_OK 0
#define ITR_EINVAL 1   /* bad argument (shape, range, null pointer)           */
#define ITR_EHIP 2     /* HIP runtime error (allocation, launch, copy)         */
#define ITR_ESTATE 3   /* object used in the wrong state                       */
#define ITR_EDATA 4    /* input data outside the alphabet (the reference's ValueError) */

#define ITR_NOBS 625   /* observed alphabet size, read_data.py:6-24            */
#define ITR_MAX_STATES 192

typedef struct itr_model* itr_model_t; /* HMM tables resident on one device          */
typedef struct itr_plan* itr_plan_t;   /* block layout of one alignment + workspace   */
typedef struct itr_maf* itr_maf_t;     /* a parsed MAF file (host memory)              */

/* ---------------------------------------------------------------------------------- */
/* library                                                                             */
/* ---------------------------------------------------------------------------------- */
ITR_API int itr_version(void);               /* ABI version, currently 1             */
ITR_API const char* itr_last_error(void);    /* message of the last failure (thread) */
ITR_API int itr_device_count(int* n);

/* ---------------------------------------------------------------------------------- */
/* model tables                                                                        */
/*                                                                                     */
/* Replaces the (a, b, pi, order) argument group of optimizer.py:145-377.  The host     */
/* builds, with NumPy, exactly the per-column quantities the reference evaluates        */
/* (bit parity for Viterbi):                                                            */
/*   a        N x N      transition matrix (get_trans_emiss.py:166-168)                 */
/*   log_a    N x N      np.log(a)                          (optimizer.py:328)          */
/*   emit     625 x N    E[o] = b[:, order[o]].sum(axis=1)  (optimizer.py:182,186,329)  */
/*   log_emit 625 x N    np.log(E[o])                       (optimizer.py:329)          */
/*   pi_emit  625 x N    pi * E[o]                          (optimizer.py:182)          */
/*   log_pi_emit 625xN   np.log(pi * E[o])                  (optimizer.py:182,323)      */
/* all row-major float64 host arrays; they are copied to the current device.           */
/* ---------------------------------------------------------------------------------- */
ITR_API int itr_model_create(int n_states, const double* h_a, const double* h_log_a,
                             const double* h_emit, const double* h_log_emit,
                             const double* h_pi_emit, const double* h_log_pi_emit,
                             itr_model_t* out);
ITR_API int itr_model_destroy(itr_model_t model);
/* Build the model's Viterbi slot tables now (the one-block-per-wavefront layout's padded and
 * slot-ordered log-emission tables and per-slot bounds, N = 65..72 only; a no-op otherwise):
 * a host simulation of 2,048 columns plus blocking allocations and copies, a few ms.  A model
 * used for decoding should be prepared once after itr_model_create so that itr_viterbi /
 * itr_forward_viterbi stay allocation-free and asynchronous on their stream; an unprepared
 * model is prepared by its first Viterbi call, which then blocks the host for that time.  A
 * model used only for likelihoods (the optimizer's per-evaluation models) never needs it. */
ITR_API int itr_model_prepare_viterbi(itr_model_t model);
ITR_API int itr_model_n_states(itr_model_t model, int* n);

/* ---------------------------------------------------------------------------------- */
/* plans                                                                               */
/*                                                                                     */
/* A plan describes one alignment as n_blocks MAF blocks laid out back to back:        */
/* block k owns columns [h_block_off[k], h_block_off[k+1]) of the observation array    */
/* (the V_lst list of read_data.py:94-117, concatenated).  Empty blocks are allowed.   */
/* The plan uploads the offsets and a longest-first processing order and owns the      */
/* device workspace (Viterbi back-pointers, forward rows for posteriors).              */
/* ---------------------------------------------------------------------------------- */
ITR_API int itr_plan_create(const int64_t* h_block_off, int64_t n_blocks, itr_plan_t* out);
/* itr_plan_create with the work-decomposition knobs explicit (negative = default):
 *   split_frac       forward log-likelihood: blocks at least this share of the longest (and
 *                    >= 512 columns) run as two halves joined exactly (default 0.5; 0 = off)
 *   post_split_frac  posterior on few long blocks: blocks at least this share of the longest
 *                    get their backward sweep beside the forward one (default 0.25; 0 = off)
 * Results agree with the unsplit sweeps to rounding (log-likelihoods, posteriors) or bit for
 * bit (Viterbi paths). */
ITR_API int itr_plan_create_ex(const int64_t* h_block_off, int64_t n_blocks, double split_frac,
                               double post_split_frac, itr_plan_t* out);
ITR_API int itr_plan_destroy(itr_plan_t plan);
/* The per-wave Viterbi (N = 65..72) decodes a block with one of two steps that give the same
 * bits: a bound-pruned step (fewer instructions per column) for blocks shorter than a planned
 * length, a full scan (shorter dependent chain) for the others.  Blocks shorter than `len`
 * take the pruned step in every later call on this plan (0: never, INT64_MAX: always;
 * negative: back to the planned lengths, see itr_plan_partition_info). */
ITR_API int itr_plan_set_prune_len(itr_plan_t plan, int64_t len);
/* The plan's work placement on a device with `cus` compute units, host-side only (no device
 * needed): out[0..9] = forward+Viterbi long set (blocks, columns), its reserved CUs, the
 * forward's reserved CUs, per-wave layout on (1/0), the Viterbi-only call's long set, the
 * forward's VALU tasks, the mixed queue's entries, the block length below which the per-wave
 * Viterbi takes the bound-pruned step (forward+Viterbi call, Viterbi-only call).  For tests
 * and diagnostics. */
ITR_API int itr_plan_partition_info(const int64_t* h_block_off, int64_t n_blocks, int cus,
                                    int64_t* out);
ITR_API int itr_plan_total_columns(itr_plan_t plan, int64_t* total);
/* grow the workspace now (optional; the sweeps grow it on demand) */
ITR_API int itr_plan_reserve(itr_plan_t plan, int n_states, int for_posterior);

/* ---------------------------------------------------------------------------------- */
/* sweeps over device-resident observations                                            */
/* ---------------------------------------------------------------------------------- */

/* Per-block forward log-likelihood.
 * Replaces forward / forward_loglik (optimizer.py:145-188) for every block of the plan;
 * d_loglik[k] = log P(block k).  The host sums d_loglik in block order, as
 * loglik_wrapper does (optimizer.py:93-116). */
ITR_API int itr_forward_loglik(itr_model_t model, itr_plan_t plan, const uint16_t* d_obs,
                               double* d_loglik, void* stream);

/* Most likely hidden path of every block.
 * Replaces viterbi + backtrack_viterbi (optimizer.py:305-354) as called by viterbi_wrapper
 * (optimizer.py:357-377): d_path[c] = state index at column c (uint8; the reference returns
 * the same integers as float64).  Ties resolve to the lowest index, like np.argmax. */
ITR_API int itr_viterbi(itr_model_t model, itr_plan_t plan, const uint16_t* d_obs,
                        uint8_t* d_path, void* stream);

/* itr_forward_loglik and itr_viterbi in one call (the same paths bit for bit; the same
 * log-likelihoods to rounding: the forward may run in another layout), the forward sweep
 * overlapped with the Viterbi sweep's longest blocks on a disjoint set of CUs.
 * For a caller that needs both over the same alignment (e.g. scoring a model and decoding
 * with it: loglik_wrapper then viterbi_wrapper, optimizer.py:40-65, 357-377). */
ITR_API int itr_forward_viterbi(itr_model_t model, itr_plan_t plan, const uint16_t* d_obs,
                                double* d_loglik, uint8_t* d_path, void* stream);

/* Posterior decoding.
 * Replaces post_prob (optimizer.py:216-238) including the reference's backward recursion
 * beta_t = (beta_{t+1} * e_{t+1}) @ a (optimizer.py:207-212): d_post is (total_columns x N)
 * row-major float64, each row summing to 1. */
ITR_API int itr_posterior(itr_model_t model, itr_plan_t plan, const uint16_t* d_obs,
                          double* d_post, void* stream);

/* The drop-in host calls on the reference's own inputs: V_lst as n_blocks host int64 arrays
 * (blocks[k], lens[k] columns; read_data.py:94-117), which must match the plan's layout.
 * The blocks are packed and range-checked by host threads into a pinned buffer (ITR_EDATA
 * for a symbol outside the 625-letter alphabet, like the reference's IndexError), copied to
 * a device buffer kept by the calling thread (itr_release_staging frees both; so does the
 * thread's exit), and swept on the calling thread's own non-blocking stream, which first
 * waits for the work already queued on the null stream (so a sweep of the same plan queued
 * there finishes first).  Work on other streams that uses the same plan must be synchronised
 * by the caller.  The results are returned to host memory:
 *   itr_forward_loglik_blocks: h_loglik[k] = forward_loglik of block k (optimizer.py:145-162)
 *   itr_viterbi_blocks:        h_path[c]  = Viterbi state of column c as float64, the dtype
 *                              backtrack_viterbi returns (optimizer.py:336-377)
 * Both return when the results are on the host. */
ITR_API int itr_forward_loglik_blocks(itr_model_t model, itr_plan_t plan,
                                      const int64_t* const* blocks, const int64_t* lens,
                                      int64_t n_blocks, double* h_loglik);
ITR_API int itr_viterbi_blocks(itr_model_t model, itr_plan_t plan, const int64_t* const* blocks,
                               const int64_t* lens, int64_t n_blocks, double* h_path);

/* The reference's standalone sweep matrices of ONE block of T >= 1 columns, device pointers,
 * float64 row-major, on `stream`:
 *   kind 0  forward:  log alpha [T][N]                            (optimizer.py:165-188)
 *   kind 1  backward: log beta [T][N], the reference's (w * e) @ a (optimizer.py:191-213)
 *   kind 2  viterbi:  omega [T][N], and when d_prev is non-null the back-pointers
 *           [T-1][N] as float64 state indices (first maximum)    (optimizer.py:305-333)
 * omega and prev are exact; log alpha / log beta agree with the reference to rounding (its
 * matrix-vector sums go through numpy's BLAS).  API-sized: one workgroup per call. */
ITR_API int itr_block_rows(itr_model_t model, int kind, const uint16_t* d_obs, int64_t T,
                           double* d_rows, double* d_prev, void* stream);
/* backtrack_viterbi (optimizer.py:336-354): the path (float64 [T]) from omega [T][N] and
 * prev [T-1][N] (device pointers, on `stream`). */
ITR_API int itr_backtrack_rows(const double* d_omega, const double* d_prev, int64_t T, int n,
                               double* d_path, void* stream);

/* Packs the caller's per-block symbol arrays (the reference's V_lst: one int64 array per
 * MAF block, read_data.py:94-117, consumed by optimizer.py:40-116, 241-262, 357-377) into
 * the uint16 column array and int64 block offsets the sweeps take.  h_blocks[k] points at
 * h_lens[k] int64 symbols; h_obs holds sum(h_lens), h_block_off n_blocks + 1 entries.
 * A symbol outside [0, 625) fails with ITR_EDATA, naming the block and column
 * (the reference's fancy index would raise IndexError).  Host memory only, multi-threaded. */
ITR_API int itr_pack_symbols(const int64_t* const* h_blocks, const int64_t* h_lens,
                             int64_t n_blocks, uint16_t* h_obs, int64_t* h_block_off);

/* Host-buffer conveniences (synchronous; copy in, run, copy out). */
ITR_API int itr_forward_loglik_host(itr_model_t model, itr_plan_t plan,
                                    const uint16_t* h_obs, double* h_loglik);
ITR_API int itr_viterbi_host(itr_model_t model, itr_plan_t plan, const uint16_t* h_obs,
                             uint8_t* h_path);
ITR_API int itr_posterior_host(itr_model_t model, itr_plan_t plan, const uint16_t* h_obs,
                               double* h_post);
/* itr_posterior_host keeps two 128 MB pinned staging buffers (plus a stream and two events)
 * per calling thread for large copy-outs, bound to the thread's current device and
 * recreated when it changes; itr_vanloan_paths keeps a grow-only device workspace and a
 * pinned staging buffer per calling thread and device.  This frees the calling thread's
 * sets (after the thread's last Van Loan evaluation has finished on the device); another
 * thread's sets are untouched and are freed when that thread exits. */
ITR_API int itr_release_staging(void);
/* itr_viterbi / itr_forward_viterbi keep three CU-masked streams (and four events) per
 * calling thread and device; this destroys the calling thread's set. */
ITR_API int itr_release_streams(void);

/* Timing hook for benchmarks: average device duration (ms) of the dominant kernel of the
 * last sweep issued on this thread, measured with HIP events on the sweep's stream. */
ITR_API int itr_last_kernel_ms(const char* which, double* ms);

/* ---------------------------------------------------------------------------------- */
/* model build: batched matrix exponential                                             */
/* ---------------------------------------------------------------------------------- */

/* out[b] = expm(A[b]) for b < batch, each n x n row-major float64 (device pointers).
 * Replaces expm (expm.py:9-167): Higham's Pade 3/5/7/9/13 with scaling & squaring, the
 * branch chosen per matrix from its 1-norm exactly as expm.py:16-143, r = solve(V-U, V+U)
 * by LU with partial pivoting, then s squarings (np.linalg.matrix_power(r, 2**s)).  Used by
 * the Van Loan integrals (vanloan.py:392-425: expm of the block matrix, top-right block) and
 * every interval propagator of the CTMCs (get_joint_prob_mat.py:119-123,
 * run_markov_chain_AB.py:105-271, run_markov_chain_ABC.py:312-510,
 * get_emission_prob_mat.py:22-44).  Synchronises `stream` once (branch selection). */
ITR_API int itr_expm_batched(int n, int64_t batch, const double* d_A, double* d_out,
                             void* stream);
ITR_API int itr_expm_batched_host(int n, int64_t batch, const double* h_A, double* h_out);

/* The same for Van Loan matrices (vanloan.py:392-425): every member is block upper
 * triangular, n_blocks x n_blocks blocks of order n_block (n = n_block * n_blocks), with
 * all diagonal blocks equal (Q t).  Pade branch and scaling exactly as itr_expm_batched
 * (the 1-norm of the whole member); only the blocks on and above the diagonal are formed
 * (a product costs k(k+1)(k+2)/6 block GEMMs instead of k^3) and V - U is inverted through
 * its one diagonal block by block back substitution.  out's lower blocks are zero. */
ITR_API int itr_expm_blocktri_batched(int n_block, int n_blocks, int64_t batch,
                                      const double* d_A, double* d_out, void* stream);

/* Van Loan integrals of many omega paths at once (vanloan.py:392-425): for path p with
 * mask ids w_0 .. w_{L-1} (h_path_mask[h_path_off[p] .. h_path_off[p+1]), L >= 1) on interval
 * h_path_job[p] of length t = h_t[job], d_out[p] (n x n) = expm(C_p t)[0:n, -n:] with C_p
 * block bidiagonal: diagonal blocks h_Q (n x n), super-diagonal blocks
 * diag(m_{w_i}) h_Q diag(m_{w_{i+1}}), m_w = h_masks[w*n .. w*n+n) (0/1 bytes).  A path of
 * length 1 gives expm(Q t).  Every block of every Pade intermediate is formed once per
 * distinct (interval, sub-path) and shared by all paths containing it (vanloan.hip); one
 * Pade branch and scaling per interval, from the largest ||C_p t||_1 of its paths
 * (expm.py:16-143).  Host arrays are read before the call returns; the work is queued on
 * `stream` without host synchronisation.  Replaces the per-path vanloan calls of
 * run_markov_chain_ABC.py:407-490 (and the Van Loan integrals of the introgression chains). */
ITR_API int itr_vanloan_paths(int n, const double* h_Q, int n_jobs, const double* h_t,
                              int n_masks, const uint8_t* h_masks, int64_t n_paths,
                              const int32_t* h_path_job, const int64_t* h_path_off,
                              const int32_t* h_path_mask, double* d_out, void* stream);
/* The same with the Pade branch input given: interval j's branch and scaling come from
 * max(h_job_norm[j], the largest ||C_p t||_1 of the paths passed).  A rank-split model build
 * evaluates a subset of an interval's paths on each rank; handing every rank the norms of the
 * whole set (itr_vanloan_job_norms) makes each path's result identical to a single-rank
 * evaluation.  h_job_norm may be null (= itr_vanloan_paths). */
ITR_API int itr_vanloan_paths_ex(int n, const double* h_Q, int n_jobs, const double* h_t,
                                 int n_masks, const uint8_t* h_masks, int64_t n_paths,
                                 const int32_t* h_path_job, const int64_t* h_path_off,
                                 const int32_t* h_path_mask, const double* h_job_norm,
                                 double* d_out, void* stream);
/* Host only: h_job_norm[j] = the largest ||C_p t_j||_1 over the paths of interval j (0 for
 * an interval without paths), the quantity expm.py:16-143 chooses the Pade branch from. */
ITR_API int itr_vanloan_job_norms(int n, const double* h_Q, int n_jobs, const double* h_t,
                                  int n_masks, const uint8_t* h_masks, int64_t n_paths,
                                  const int32_t* h_path_job, const int64_t* h_path_off,
                                  const int32_t* h_path_mask, double* h_job_norm);

/* Solve M_b X_b = R_b for b < batch (M n x n, R n x nrhs, row-major, contiguous batches).
 * M is overwritten by its LU factors (partial pivoting, first maximum |.| like LAPACK
 * idamax), R by X.  Replaces np.linalg.inv in deepest_ti (deepest_ti.py:256: the last n
 * columns of C^-1 are solve(C, I[:, -n:])). */
ITR_API int itr_solve_batched(int n, int nrhs, int64_t batch, double* d_M, double* d_R,
                              void* stream);

/* d_out_b = d_M_b^-1 for every b (d_M untouched; d_out must not alias it).  n <= 208: one
 * workgroup per matrix, in-place Gauss-Jordan in registers with partial-pivoting pivots (a
 * pass without interchanges that checks the diagonal is the column maximum at every step,
 * and a pivoting pass for the matrices where it is not); larger n: the LU above against the
 * identity.  Replaces np.linalg.inv of the deepest-interval matrix (deepest_ti.py:256) and
 * the Pade denominator's inverse in the Van Loan evaluation (expm.py:141-160). */
ITR_API int itr_inverse_batched(int n, int64_t batch, const double* d_M, double* d_out,
                                void* stream);

/* C_b = alpha * A_b (m x k) @ B_b (k x n) + beta * C_b, contiguous row-major batches
 * (MFMA f64 16x16x4 tiles).  The contractions of the chain steps (prob @ (mask E mask),
 * run_markov_chain_ABC.py:9-14; deepest_ti.py:256 product with A_last). */
ITR_API int itr_gemm_batched(int m, int n, int k, int64_t batch, double alpha,
                             const double* d_A, const double* d_B, double beta, double* d_C,
                             void* stream);

/* One interval's chain-step products (run_markov_chain_ABC.py:13-33, 407-490): for group g
 * (0 <= g < n_groups) and row r < rmax, entry e = g * rmax + r (d_src[e] < 0: padding):
 *   d_out[d_dst[e]][:] = ((d_P[d_src[e]][cols] * d_F[d_oms[e]]) @ M_g) * d_F[d_ome[e]]
 * with M_g = d_M + g * k * k (k x k row-major), cols = d_cols (k column indices of P; NULL:
 * 0 .. k-1), d_oms / d_ome NULL for no mask.  Rows of d_P, d_F and d_out have strides ldp,
 * ldf, ldo.  One fused MFMA pass (gather, mask, product, mask, scatter); d_out must not alias
 * d_P.  Also the closing phase's per-task contractions (run_markov_chain_ABC.py:512-796). */
ITR_API int itr_chain_rows(int k, int n_groups, int rmax, const int32_t* d_src,
                           const int32_t* d_oms, const int32_t* d_ome, const int32_t* d_dst,
                           const int32_t* d_cols, const double* d_P, int64_t ldp,
                           const double* d_F, int64_t ldf, const double* d_M, double* d_out,
                           int64_t ldo, void* stream);

/* Path-group sums of one rebuild's Van Loan integrals (run_markov_chain_ABC.py:478-486:
 * the group's matrix S = S_0 + S_1 + ... over its paths, left to right):
 * d_M[g] = d_S[d_paths[d_off[g]]] + d_S[d_paths[d_off[g] + 1]] + ... for g < n_groups, every
 * matrix nn float64 values, each element summed in path order from 0.0 (bit-identical to
 * the sequential sum).  d_off: n_groups + 1 int32 offsets into d_paths (int32 matrix indices
 * of d_S); an empty group gives zeros. */
ITR_API int itr_group_sum(int64_t nn, int n_groups, const int32_t* d_off,
                          const int32_t* d_paths, const double* d_S, double* d_M, void* stream);

/* ---------------------------------------------------------------------------------- */
/* model build: emission rows                                                          */
/* ---------------------------------------------------------------------------------- */

/* Emission probabilities of n_states hidden states over the 256 N-free columns.
 * Replaces the per-state loops calc_emissions_single_JC69 / calc_emissions_double_JC69
 * (get_emission_prob_mat.py:585-698) and the topology re-keying (871-875, 897-901).
 * d_tables: n_states x 512 float64 per-state tables (layout in
 * itrails_amd/model/emissions.py: kind, re-keying, the 4x4 branch transition matrices, the
 * 4x4x4 single-coalescence and 4^4 double-coalescence integrals); d_out: n_states x 256. */
ITR_API int itr_emission_rows(int n_states, const double* d_tables, double* d_out,
                              void* stream);

/* ---------------------------------------------------------------------------------- */
/* MAF ingest (host)                                                                   */
/* ---------------------------------------------------------------------------------- */

/* Parse a MAF file into the concatenated observation layout of the plans.
 * Replaces maf_parser (read_data.py:94-117: blocks holding all 4 species of `species`,
 * '-' -> 'N', upper-cased, column symbol = index in the 625-letter alphabet; a letter
 * outside A/C/T/G/N fails with ITR_EDATA like the reference's list.index ValueError) and,
 * when `ref` is not NULL, parse_coordinates (read_data.py:150-220: per-column reference
 * positions, -9 for gaps / blocks without the reference).  The file is memory-mapped and
 * scanned once. */
ITR_API int itr_maf_open(const char* path, const char* const* species /* [4] */,
                         const char* ref, itr_maf_t* out);
ITR_API int itr_maf_sizes(itr_maf_t maf, int64_t* n_blocks, int64_t* n_columns,
                          int64_t* n_coord_blocks, int64_t* n_coords);
/* copy out: obs [n_columns], block_off [n_blocks+1], coords [n_coords],
 * coord_off [n_coord_blocks+1]; any pointer may be NULL */
ITR_API int itr_maf_copy(itr_maf_t maf, uint16_t* h_obs, int64_t* h_block_off,
                         int64_t* h_coords, int64_t* h_coord_off);
ITR_API int itr_maf_close(itr_maf_t maf);

/* ---------------------------------------------------------------------------------- */
/* result files (host)                                                                 */
/* ---------------------------------------------------------------------------------- */

/* Viterbi segments CSV, byte-identical to workflow_viterbi.py:690-743 (csv excel dialect):
 * one row per run of equal states per block; with h_coords (per-column reference
 * positions, -9 = gap; NULL = block-relative positions) the reference's gap handling.
 * n_coords must equal the decoded column count h_block_off[n_blocks] (ITR_EINVAL
 * otherwise; ignored when h_coords is NULL). */
ITR_API int itr_write_viterbi_csv(const char* path, const uint8_t* h_states,
                                  const int64_t* h_block_off, int64_t n_blocks,
                                  const int64_t* h_coords, int64_t n_coords);
/* Posterior CSV, byte-identical to workflow_posterior.py:697-716: one row per column,
 * probabilities printed like Python repr(float); formatted by `threads` threads.
 * n_coords as for itr_write_viterbi_csv. */
ITR_API int itr_write_posterior_csv(const char* path, const double* h_post, int n_states,
                                    const int64_t* h_block_off, int64_t n_blocks,
                                    const int64_t* h_coords, int64_t n_coords, int threads);
/* Python repr(float) of x into out (cap >= 33 bytes suffices). */
ITR_API int itr_format_float(double x, char* out, int cap);

#ifdef __cplusplus
}
#endif
#endif /* ITRAILS_HIP_H */
