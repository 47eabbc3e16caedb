/*
 * hmm_oracle.c — CPU restatement of the reference's HMM sweeps.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the
 * product path (itrails_amd/) never does.  It restates, in the reference's own operation
 * order and in log space, src/itrails/optimizer.py of trails-phylogeny/itrails:
 *
 *   forward           optimizer.py:165-188  alpha_0 = log(pi*e_0);
 *                                           alpha_t = log((exp(alpha_{t-1}-x) @ a) * e_t) + x
 *   forward_loglik    optimizer.py:145-162  x = max(alpha_T); log(sum(exp(alpha_T - x))) + x
 *   backward          optimizer.py:191-213  beta_t = log((exp(beta_{t+1}-x) * e_{t+1}) @ a) + x
 *   post_prob         optimizer.py:216-238  p = alpha+beta; exp(p - rowmax) / sum
 *   viterbi           optimizer.py:305-333  M_ij = (omega_i + log a_ij) + log e_j;
 *                                           prev_j = first argmax_i, omega_j = max_i
 *   backtrack_viterbi optimizer.py:336-354  last = first argmax(omega_T), follow prev
 *
 * The per-symbol quantities e = b[:, order[o]].sum(axis=1), log(e), pi*e, log(pi*e) and
 * log(a) are passed in as 625 x N / N x N tables built by NumPy exactly as the reference
 * evaluates them (itrails_amd/tables.py), so the Viterbi restatement is bit-exact.
 *
 * Parity pinning: tests/test_oracle.py checks this file against the golden vectors that
 * tests/golden/make_golden.py produced by running the reference itself.
 *
 * Blocks are independent; OpenMP distributes them over host cores (this is the
 * "cpu_baseline" of bench.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NOBS 625

static double vmax(const double* v, int n) {
  double m = v[0];
  for (int i = 1; i < n; ++i)
    if (v[i] > m) m = v[i];
  return m;
}

/* alpha: T x n, log space */
static void forward_block(int n, const double* a, const double* emit, const double* pi_emit,
                          const uint16_t* V, int64_t T, double* alpha, double* tmp) {
  for (int j = 0; j < n; ++j) alpha[j] = log(pi_emit[(int)V[0] * n + j]);
  for (int64_t t = 1; t < T; ++t) {
    const double* prev = alpha + (t - 1) * n;
    double* cur = alpha + t * n;
    const double x = vmax(prev, n);
    for (int i = 0; i < n; ++i) tmp[i] = exp(prev[i] - x);
    const double* e = emit + (int)V[t] * n;
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int i = 0; i < n; ++i) s += tmp[i] * a[(int64_t)i * n + j];
      cur[j] = log(s * e[j]) + x;
    }
  }
}

static double loglik_from_alpha(const double* last, int n) {
  const double x = vmax(last, n);
  double s = 0.0;
  for (int j = 0; j < n; ++j) s += exp(last[j] - x);
  return log(s) + x;
}

void oracle_forward_loglik(int n, const double* a, const double* emit, const double* pi_emit,
                           const uint16_t* obs, const int64_t* off, int64_t nblocks,
                           double* out) {
#pragma omp parallel
  {
    int64_t cap = 0;
    double* alpha = NULL;
    double* tmp = (double*)malloc(sizeof(double) * n);
#pragma omp for schedule(dynamic, 1)
    for (int64_t k = 0; k < nblocks; ++k) {
      const int64_t T = off[k + 1] - off[k];
      if (T <= 0) {
        out[k] = 0.0;
        continue;
      }
      /* only two rows are needed for the likelihood */
      if (cap < 2) {
        free(alpha);
        alpha = (double*)malloc(sizeof(double) * 2 * n);
        cap = 2;
      }
      const uint16_t* V = obs + off[k];
      for (int j = 0; j < n; ++j) alpha[j] = log(pi_emit[(int)V[0] * n + j]);
      for (int64_t t = 1; t < T; ++t) {
        double* prev = alpha + ((t - 1) & 1) * n;
        double* cur = alpha + (t & 1) * n;
        const double x = vmax(prev, n);
        for (int i = 0; i < n; ++i) tmp[i] = exp(prev[i] - x);
        const double* e = emit + (int)V[t] * n;
        for (int j = 0; j < n; ++j) {
          double s = 0.0;
          for (int i = 0; i < n; ++i) s += tmp[i] * a[(int64_t)i * n + j];
          cur[j] = log(s * e[j]) + x;
        }
      }
      out[k] = loglik_from_alpha(alpha + ((T - 1) & 1) * n, n);
    }
    free(alpha);
    free(tmp);
  }
}

void oracle_viterbi(int n, const double* log_a, const double* log_emit,
                    const double* log_pi_emit, const uint16_t* obs, const int64_t* off,
                    int64_t nblocks, int16_t* path) {
#pragma omp parallel
  {
    int64_t cap = 0;
    int16_t* prev = NULL;
    double* om = (double*)malloc(sizeof(double) * 2 * n);
#pragma omp for schedule(dynamic, 1)
    for (int64_t k = 0; k < nblocks; ++k) {
      const int64_t T = off[k + 1] - off[k];
      if (T <= 0) continue;
      if (T > cap) {
        free(prev);
        prev = (int16_t*)malloc(sizeof(int16_t) * T * n);
        cap = T;
      }
      const uint16_t* V = obs + off[k];
      for (int j = 0; j < n; ++j) om[j] = log_pi_emit[(int)V[0] * n + j];
      for (int64_t t = 1; t < T; ++t) {
        const double* o0 = om + ((t - 1) & 1) * n;
        double* o1 = om + (t & 1) * n;
        const double* le = log_emit + (int)V[t] * n;
        int16_t* pv = prev + t * n;
        for (int j = 0; j < n; ++j) {
          double best = (o0[0] + log_a[j]) + le[j];
          int arg = 0;
          for (int i = 1; i < n; ++i) {
            const double v = (o0[i] + log_a[(int64_t)i * n + j]) + le[j];
            if (v > best) {
              best = v;
              arg = i;
            }
          }
          o1[j] = best;
          pv[j] = (int16_t)arg;
        }
      }
      const double* last = om + ((T - 1) & 1) * n;
      int s = 0;
      for (int j = 1; j < n; ++j)
        if (last[j] > last[s]) s = j;
      int16_t* P = path + off[k];
      P[T - 1] = (int16_t)s;
      for (int64_t t = T - 1; t >= 1; --t) {
        s = prev[t * n + s];
        P[t - 1] = (int16_t)s;
      }
    }
    free(prev);
    free(om);
  }
}

void oracle_posterior(int n, const double* a, const double* emit, const double* pi_emit,
                      const uint16_t* obs, const int64_t* off, int64_t nblocks, double* post) {
#pragma omp parallel
  {
    int64_t cap = 0;
    double *alpha = NULL, *beta = NULL;
    double* tmp = (double*)malloc(sizeof(double) * n);
#pragma omp for schedule(dynamic, 1)
    for (int64_t k = 0; k < nblocks; ++k) {
      const int64_t T = off[k + 1] - off[k];
      if (T <= 0) continue;
      if (T > cap) {
        free(alpha);
        free(beta);
        alpha = (double*)malloc(sizeof(double) * T * n);
        beta = (double*)malloc(sizeof(double) * T * n);
        cap = T;
      }
      const uint16_t* V = obs + off[k];
      forward_block(n, a, emit, pi_emit, V, T, alpha, tmp);
      /* backward, optimizer.py:205-212: vector @ a */
      for (int j = 0; j < n; ++j) beta[(T - 1) * n + j] = 0.0;
      for (int64_t t = T - 2; t >= 0; --t) {
        const double* nx = beta + (t + 1) * n;
        double* cur = beta + t * n;
        const double x = vmax(nx, n);
        const double* e = emit + (int)V[t + 1] * n;
        for (int i = 0; i < n; ++i) tmp[i] = exp(nx[i] - x) * e[i];
        for (int j = 0; j < n; ++j) {
          double s = 0.0;
          for (int i = 0; i < n; ++i) s += tmp[i] * a[(int64_t)i * n + j];
          cur[j] = log(s) + x;
        }
      }
      double* P = post + off[k] * n;
      for (int64_t t = 0; t < T; ++t) {
        double* row = P + t * n;
        for (int j = 0; j < n; ++j) row[j] = alpha[t * n + j] + beta[t * n + j];
        const double mx = vmax(row, n);
        double s = 0.0;
        for (int j = 0; j < n; ++j) {
          row[j] = exp(row[j] - mx);
          s += row[j];
        }
        for (int j = 0; j < n; ++j) row[j] /= s;
      }
    }
    free(alpha);
    free(beta);
    free(tmp);
  }
}

/* threads of the OpenMP loops above (the CPU-baseline legs time 1 core and the job's share) */
#include <omp.h>
void oracle_set_threads(int k) { omp_set_num_threads(k > 0 ? k : 1); }
