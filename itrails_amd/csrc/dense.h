// dense.h — batched dense FP64 linear algebra for the model build (dense.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace itr {

// A batch of equally shaped row-major sub-matrices: member b starts at p + slot(b)*stride.
struct Mat {
  double* p;
  int64_t stride;  // elements between batch members
  int ld;          // elements between rows
};

// C = alpha * A(m x k) @ B(k x n) + beta * D + gamma * I   (D may be null; may alias C)
struct GemmArgs {
  int m, n, k;
  Mat A, B, C, D;
  double alpha, beta, gamma;
  const int* idx;  // batch member -> slot (null: member index)
};

hipError_t gemm_batched(const GemmArgs& g, int64_t batch, hipStream_t st);

// Chain-step rows (chain_rows_kernel): for the rows r < rmax of group g (entry e = g rmax + r,
// src[e] < 0: padding), out[dst[e]] = ((P[src[e]][cols] * F[oms[e]]) @ M[g]) * F[ome[e]]
// with M[g] k x k at M + g k k; cols (k entries) gathers P's columns (null: 0 .. k-1), oms /
// ome select rows of F (null: no mask).
struct ChainRowsArgs {
  int k, rmax;
  const int32_t *src, *oms, *ome, *dst, *cols;
  const double* P;
  int64_t ldp;
  const double* F;
  int64_t ldf;
  const double* M;
  double* out;
  int64_t ldo;
};
hipError_t chain_rows(const ChainRowsArgs& a, int ngroups, hipStream_t st);
hipError_t group_sum(int64_t nn, int ngroups, const int32_t* off, const int32_t* paths,
                     const double* S, double* M, hipStream_t st);

// Solve M X = R for every member (M n x n, R n x nrhs, both row-major, contiguous):
// M is overwritten by its LU factors (partial pivoting), R by X.  `piv` is a device
// workspace of batch * n ints.
hipError_t solve_batched(int n, int nrhs, int64_t batch, double* M, double* R, int* piv,
                         hipStream_t st);
// out_b = M_b^-1 (M untouched).  n <= 208: one workgroup per matrix (in-place Gauss-Jordan in
// registers, partial pivoting); larger n: the blocked LU against the identity, on `work`
// (batch n^2 doubles) with `piv` (batch n ints).
hipError_t inverse_batched(int n, int64_t batch, const double* M, double* out, int* piv,
                           double* work, hipStream_t st);
constexpr int kInverseRegMax = 208;

// out[b] = expm(A[b]) (expm.py:9-167).  Allocates its own workspace (stream-ordered).
hipError_t expm_batched(int n, int64_t batch, const double* A, double* out, hipStream_t st);
// The same for members that are block upper triangular (kb x kb blocks of order nb, all
// diagonal blocks equal; Van Loan matrices): only the blocks on and above the diagonal are
// formed, the result's lower blocks are zero.  Same Pade branch and scaling per member
// (the 1-norm of the whole matrix).
hipError_t expm_blocktri_batched(int nb, int kb, int64_t batch, const double* A, double* out,
                                 hipStream_t st);

// Van Loan integrals of many omega paths, shared sub-path evaluation (vanloan.hip; the
// arguments of itr_vanloan_paths)
hipError_t vanloan_paths(int nb, const double* h_Q, int njobs, const double* h_t, int nmasks,
                         const uint8_t* h_masks, int64_t npaths, const int32_t* h_job,
                         const int64_t* h_off, const int32_t* h_mask, const double* h_jnorm,
                         double* d_out, hipStream_t st);
// per interval, the largest ||C_p t||_1 over its paths (the Pade branch's input)
void vanloan_job_norms(int nb, const double* h_Q, int njobs, const double* h_t, int nmasks,
                       const uint8_t* h_masks, int64_t npaths, const int32_t* h_job,
                       const int64_t* h_off, const int32_t* h_mask, double* jnorm);
void release_vanloan_workspace();

// emission rows (emission.hip): tables [n_states x 512] -> out [n_states x 256]
hipError_t launch_emission(int n_states, const double* tables, double* out, hipStream_t st);

}  // namespace itr
