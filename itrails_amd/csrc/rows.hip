// rows.hip — the reference's per-column matrices of ONE block on MI355X (gfx950), for its
// standalone sweep functions: log alpha (optimizer.py:165-188), log beta (:191-213), the
// Viterbi omega and back-pointer matrices (:305-333) and the traceback of (omega, prev)
// (:336-354).  These materialise T x N rows, so they are API-sized paths (one block per call,
// one workgroup, one thread per state); the throughput paths (itr_forward_loglik,
// itr_viterbi, itr_posterior) never form these matrices.
//
// Arithmetic follows the reference expression by expression:
//   alpha_t[j] = log((exp(alpha_{t-1} - x) @ a)[j] * e_t[j]) + x,  x = max(alpha_{t-1})
//   beta_t[j]  = log(((exp(beta_{t+1} - x) * e_{t+1}) @ a)[j]) + x  (the reference's v @ a)
//   omega_t[j] = max_i (omega_{t-1}[i] + log a_ij) + log e_t[j], prev = first argmax over i
// The matrix-vector sums run in source order (numpy's BLAS order is not specified: alpha and
// beta agree to rounding); omega and prev are exact (max / argmax of identically rounded
// sums).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sweeps.h"

namespace itr {
namespace {

constexpr int kRowThreads = 256;  // >= ITR_MAX_STATES (192)

__device__ double block_max(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = kRowThreads / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmax(red[tid], red[tid + s]);
    __syncthreads();
  }
  const double m = red[0];
  __syncthreads();
  return m;
}

// kind 0: log alpha, 1: log beta, 2: omega (+ prev)
__global__ void __launch_bounds__(kRowThreads) rows_kernel(RowArgs p) {
  __shared__ double cur[kRowThreads];
  __shared__ double red[kRowThreads];
  const int j = threadIdx.x, n = p.n;
  const bool in = j < n;
  const int64_t T = p.T;
  auto sym = [&](int64_t t) { return (int)min((int)p.obs[t], 624); };
  if (p.kind == 0 || p.kind == 2) {
    double v = in ? p.lpie[(int64_t)sym(0) * n + j] : -INFINITY;
    if (in) p.rows[j] = v;
    cur[j] = v;
    __syncthreads();
    for (int64_t t = 1; t < T; ++t) {
      const int o = sym(t);
      if (p.kind == 0) {
        const double x = block_max(cur[j], red);
        double s = 0.0;
        if (in)
          for (int i = 0; i < n; ++i) s += exp(cur[i] - x) * p.a[(int64_t)i * n + j];
        v = in ? log(s * p.emit[(int64_t)o * n + j]) + x : -INFINITY;
      } else {
        double best = -INFINITY;
        int arg = 0;  // first maximum (np.argmax); a column of -inf -> 0
        if (in) {
          const double le = p.log_emit[(int64_t)o * n + j];
          for (int i = 0; i < n; ++i) {
            const double c = (cur[i] + p.log_a[(int64_t)i * n + j]) + le;
            if (c > best) {
              best = c;
              arg = i;
            }
          }
          if (p.prev) p.prev[(t - 1) * n + j] = (double)arg;
        }
        v = best;
      }
      __syncthreads();  // every thread's reads of cur precede the overwrite
      cur[j] = v;
      if (in) p.rows[t * n + j] = v;
      __syncthreads();
    }
  } else {
    double v = 0.0;
    if (in) p.rows[(T - 1) * n + j] = 0.0;
    cur[j] = in ? 0.0 : -INFINITY;
    __syncthreads();
    for (int64_t t = T - 2; t >= 0; --t) {
      const int o = sym(t + 1);
      const double x = block_max(cur[j], red);
      // w_i = exp(beta_{t+1}[i] - x) * e_{t+1}[i], then (w @ a)[j] = sum_i w_i a_ij
      red[j] = in ? exp(cur[j] - x) * p.emit[(int64_t)o * n + j] : 0.0;
      __syncthreads();
      double s = 0.0;
      if (in)
        for (int i = 0; i < n; ++i) s += red[i] * p.a[(int64_t)i * n + j];
      v = in ? log(s) + x : -INFINITY;
      __syncthreads();
      cur[j] = v;
      if (in) p.rows[t * n + j] = v;
      __syncthreads();
    }
  }
}

// S[T-1] = first argmax of omega[T-1], then S[t] = prev[t, S[t+1]]  (float64 like the reference)
__global__ void __launch_bounds__(64) backtrack_rows_kernel(const double* omega, const double* prev,
                                                             int64_t T, int n, double* path) {
  if (threadIdx.x != 0 || T <= 0) return;
  const double* last = omega + (T - 1) * n;
  int s = 0;
  for (int j = 1; j < n; ++j)
    if (last[j] > last[s]) s = j;
  path[T - 1] = (double)s;
  for (int64_t t = T - 2; t >= 0; --t) {
    const double b = prev[t * n + s];
    // NumPy's prev[i, int(s)]: truncation, negative indices wrap once; anything else (NaN,
    // +-inf, |s| >= n) is the reference's error: this and every earlier entry become NaN
    // (the wrapper raises) and no out-of-range row is read
    if (!(b > -(double)n - 1.0 && b < (double)n)) {
      for (int64_t u = t; u >= 0; --u) path[u] = __builtin_nan("");
      return;
    }
    s = (int)b;
    if (s < 0) s += n;
    if (s < 0 || s >= n) {
      for (int64_t u = t; u >= 0; --u) path[u] = __builtin_nan("");
      return;
    }
    path[t] = b;
  }
}

}  // namespace

hipError_t launch_rows(const RowArgs& p, hipStream_t st) {
  if (p.n < 1 || p.n > kRowThreads || p.T < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rows_kernel, dim3(1), dim3(kRowThreads), 0, st, p);
  return hipGetLastError();
}

hipError_t launch_backtrack_rows(const double* omega, const double* prev, int64_t T, int n,
                                 double* path, hipStream_t st) {
  hipLaunchKernelGGL(backtrack_rows_kernel, dim3(1), dim3(64), 0, st, omega, prev, T, n, path);
  return hipGetLastError();
}

}  // namespace itr
