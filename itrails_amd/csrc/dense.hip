// dense.hip — batched dense FP64 linear algebra for the iTRAILS model build on gfx950.
//
// The model build (get_joint_prob_mat.py, run_markov_chain_{AB,ABC}.py, vanloan.py:392-425,
// deepest_ti.py:215-256, get_emission_prob_mat.py:22-44) spends its time in matrix
// exponentials of CTMC rate matrices (n = 2, 4, 15, 203 and Van Loan block matrices of
// 406 … 1015) and in one inverse per deepest-interval task.  The reference evaluates them
// one at a time on the CPU (expm.py:9-167, numpy.linalg.solve / inv).  Here every distinct
// matrix of a rebuild is one member of a batch, and the batch runs as:
//
//   * gemm_kernel      — C = alpha A B + beta D + gamma I, one 64x64 output tile per
//                        workgroup (4 waves x 2x2 v_mfma_f64_16x16x4 tiles), K staged
//                        through LDS 16 at a time.  All Pade products, the LU trailing
//                        updates and the back-substitution updates run through it.
//   * norm1_kernel     — ||A||_1 (max column sum, rows summed in order like numpy's
//                        norm(ord=1)) selects the Pade branch per matrix (expm.py:26-140).
//   * LU with partial pivoting, blocked by 32 columns (getrf + getrs): panel_kernel (one
//                        workgroup per matrix, first-max |.| pivots like LAPACK idamax),
//                        swap_kernel, trsm_lower_kernel / trsm_upper_kernel (one thread per
//                        column, the 32x32 triangle in LDS) and gemm_kernel updates.
//   * lincomb_kernel   — the Pade polynomial sums (b_i A^i + b_0 I), V-U and V+U.
//
// Branch selection and scaling follow expm.py exactly: theta = 1.5e-2, 2.5e-1, 9.5e-1, 2.1
// select Pade 3/5/7/9; otherwise Pade 13 on A / 2^s with s = max(0, ceil(log2(norm/5.4)))
// evaluated as ceil(log(norm/5.4)/log(2)) like expm.py:141, then s squarings
// (np.linalg.matrix_power(r, 2**s) performs exactly s squarings).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "dense.h"

namespace itr {

typedef double dbl4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// GEMM
// ---------------------------------------------------------------------------------------
static constexpr int GBM = 64, GBN = 64, GBK = 16;

__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g) {
  __shared__ double As[GBK][GBM + 2];
  __shared__ double Bs[GBK][GBN + 2];
  const int tiles_n = (g.n + GBN - 1) / GBN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int64_t slot = g.idx ? g.idx[blockIdx.y] : (int64_t)blockIdx.y;
  const double* __restrict__ A = g.A.p + slot * g.A.stride;
  const double* __restrict__ B = g.B.p + slot * g.B.stride;
  const int row0 = tm * GBM, col0 = tn * GBN;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;  // this wave's 32x32 quadrant of the tile

  bool row_live[2], col_live[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    row_live[i] = row0 + wr * 32 + i * 16 < g.m;
    col_live[i] = col0 + wc * 32 + i * 16 < g.n;
  }
  dbl4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  const int ar = tid >> 2, ak = (tid & 3) * 4;   // A tile: row ar, k ak..ak+3
  const int bk = tid >> 4, bc = (tid & 15) * 4;  // B tile: k bk, cols bc..bc+3
  // the next K tile is fetched into registers while the current one is multiplied out of
  // LDS, so a tile's global-load latency hides behind the previous tile's MFMAs
  double ra[4], rb[4];
  auto fetch = [&](int k0) {
    const int gr = row0 + ar;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int gk = k0 + ak + e;
      ra[e] = (gr < g.m && gk < g.k) ? A[(int64_t)gr * g.A.ld + gk] : 0.0;
    }
    const int gk = k0 + bk;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int gc = col0 + bc + e;
      rb[e] = (gk < g.k && gc < g.n) ? B[(int64_t)gk * g.B.ld + gc] : 0.0;
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < g.k; k0 += GBK) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      As[ak + e][ar] = ra[e];
      Bs[bk][bc + e] = rb[e];
    }
    __syncthreads();
    if (k0 + GBK < g.k) fetch(k0 + GBK);
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 4) {
      // v_mfma_f64_16x16x4: lane l holds A[l&15][l>>4] and B[l>>4][l&15]
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk + (l >> 4)][wr * 32 + i * 16 + (l & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk + (l >> 4)][wc * 32 + j * 16 + (l & 15)];
      // 16 x 16 sub-tiles wholly outside C (the edge tiles of an order-203 block: 13 of 16
      // row and column groups are real) are skipped: a wave-uniform branch, the SIMD's
      // matrix pipe goes to the co-resident workgroups instead
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (row_live[i] && col_live[j])
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  double* __restrict__ C = g.C.p + slot * g.C.stride;
  const double* D = g.D.p ? g.D.p + slot * g.D.stride : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // f64 16x16x4 result: col = l & 15, row = (l >> 4) + 4 r
        const int row = row0 + wr * 32 + i * 16 + (l >> 4) + 4 * r;
        const int col = col0 + wc * 32 + j * 16 + (l & 15);
        if (row < g.m && col < g.n) {
          double v = g.alpha * acc[i][j][r];
          if (D) v += g.beta * D[(int64_t)row * g.D.ld + col];
          if (row == col) v += g.gamma;
          C[(int64_t)row * g.C.ld + col] = v;
        }
      }
}

hipError_t gemm_batched(const GemmArgs& g, int64_t batch, hipStream_t st) {
  if (batch <= 0 || g.m <= 0 || g.n <= 0) return hipSuccess;
  const int tiles = ((g.m + GBM - 1) / GBM) * ((g.n + GBN - 1) / GBN);
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {  // grid.y limit
    GemmArgs h = g;
    const int64_t nb = std::min<int64_t>(65535, batch - b0);
    if (h.idx) {
      h.idx = g.idx + b0;
    } else {
      h.A.p += b0 * g.A.stride;
      h.B.p += b0 * g.B.stride;
      h.C.p += b0 * g.C.stride;
      if (h.D.p) h.D.p += b0 * g.D.stride;
    }
    hipLaunchKernelGGL(gemm_kernel, dim3(tiles, (unsigned)nb), dim3(256), 0, st, h);
  }
  return hipGetLastError();
}

// Chain-step rows (run_markov_chain_ABC.py:13-33 products, :407-490 per interval): the
// gathered, masked row block of a group times the group's propagator, masked and scattered
// in one pass — gemm_kernel's 64 x 64 tile and MFMA loop with the gathers in the A-tile
// fetch and the mask and scatter in the epilogue (no V / result temporaries in HBM).
__global__ void __launch_bounds__(256) chain_rows_kernel(ChainRowsArgs g) {
  __shared__ double As[GBK][GBM + 2];
  __shared__ double Bs[GBK][GBN + 2];
  const int K = g.k;
  const int tiles_n = (K + GBN - 1) / GBN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int64_t e0 = (int64_t)blockIdx.y * g.rmax;
  const double* __restrict__ B = g.M + (int64_t)blockIdx.y * K * K;
  const int row0 = tm * GBM, col0 = tn * GBN;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;

  dbl4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  const int ar = tid >> 2, ak = (tid & 3) * 4;   // A tile: row ar, k ak..ak+3
  const int bk = tid >> 4, bc = (tid & 15) * 4;  // B tile: k bk, cols bc..bc+3
  const int arow = row0 + ar;
  const int asrc = arow < g.rmax ? g.src[e0 + arow] : -1;
  const double* prow = asrc >= 0 ? g.P + (int64_t)asrc * g.ldp : nullptr;
  const double* frow = (asrc >= 0 && g.oms) ? g.F + (int64_t)g.oms[e0 + arow] * g.ldf : nullptr;
  double ra[4], rb[4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int gk = k0 + ak + e;
      double v = 0.0;
      if (prow && gk < K) {
        v = prow[g.cols ? g.cols[gk] : gk];
        if (frow) v *= frow[gk];
      }
      ra[e] = v;
    }
    const int gk = k0 + bk;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int gc = col0 + bc + e;
      rb[e] = (gk < K && gc < K) ? B[(int64_t)gk * K + gc] : 0.0;
    }
  };
  fetch(0);
  for (int k0 = 0; k0 < K; k0 += GBK) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      As[ak + e][ar] = ra[e];
      Bs[bk][bc + e] = rb[e];
    }
    __syncthreads();
    if (k0 + GBK < K) fetch(k0 + GBK);
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk + (l >> 4)][wr * 32 + i * 16 + (l & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk + (l >> 4)][wc * 32 + j * 16 + (l & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = row0 + wr * 32 + i * 16 + (l >> 4) + 4 * r;
      if (row >= g.rmax) continue;
      const int64_t e = e0 + row;
      if (g.src[e] < 0) continue;
      double* orow = g.out + (int64_t)g.dst[e] * g.ldo;
      const double* mrow = g.ome ? g.F + (int64_t)g.ome[e] * g.ldf : nullptr;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = col0 + wc * 32 + j * 16 + (l & 15);
        if (col < K) orow[col] = mrow ? acc[i][j][r] * mrow[col] : acc[i][j][r];
      }
    }
}

// Path-group sums of the chain's Van Loan integrals: M[g] = S[p_g0] + S[p_g1] + ... for the
// paths of group g in order, every element summed one after another from 0.0 — the
// reference's left-to-right `S = S_0 + S_1 + ...` (run_markov_chain_ABC.py:478-486), one
// launch for all groups instead of one indexed add per path position.
__global__ void __launch_bounds__(256) group_sum_kernel(int64_t nn, const double* __restrict__ S,
                                                        const int32_t* __restrict__ off,
                                                        const int32_t* __restrict__ paths,
                                                        double* __restrict__ M) {
  const int g = blockIdx.y;
  const int k0 = off[g], k1 = off[g + 1];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn; e += (int64_t)gridDim.x * 256) {
    double acc = 0.0;
    for (int k = k0; k < k1; ++k) acc += S[(int64_t)paths[k] * nn + e];
    M[(int64_t)g * nn + e] = acc;
  }
}

hipError_t group_sum(int64_t nn, int ngroups, const int32_t* off, const int32_t* paths,
                     const double* S, double* M, hipStream_t st) {
  if (ngroups <= 0 || nn <= 0) return hipSuccess;
  const int gx = (int)std::min<int64_t>((nn + 255) / 256, 1024);
  hipLaunchKernelGGL(group_sum_kernel, dim3(gx, ngroups), dim3(256), 0, st, nn, S, off, paths, M);
  return hipGetLastError();
}

hipError_t chain_rows(const ChainRowsArgs& a, int ngroups, hipStream_t st) {
  if (ngroups <= 0 || a.rmax <= 0 || a.k <= 0) return hipSuccess;
  if (ngroups > 65535) return hipErrorInvalidValue;
  const int tiles = ((a.rmax + GBM - 1) / GBM) * ((a.k + GBN - 1) / GBN);
  hipLaunchKernelGGL(chain_rows_kernel, dim3(tiles, (unsigned)ngroups), dim3(256), 0, st, a);
  return hipGetLastError();
}

static hipError_t gemm(int m, int n, int k, Mat A, Mat B, Mat C, double alpha, Mat D,
                       double beta, double gamma, const int* idx, int64_t batch,
                       hipStream_t st) {
  GemmArgs g{m, n, k, A, B, C, D, alpha, beta, gamma, idx};
  return gemm_batched(g, batch, st);
}

// ---------------------------------------------------------------------------------------
// element-wise kernels
// ---------------------------------------------------------------------------------------
struct LinArgs {
  int64_t nn;         // elements per matrix (n*n)
  int n;              // order (for the identity term)
  double* out;        // out[g] = cI * I + sum_t c[t] * in[t][g]
  const double* in[4];
  double c[4];
  double cI;
};

__global__ void __launch_bounds__(256) lincomb_kernel(LinArgs a) {
  const int64_t g = blockIdx.y;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < a.nn;
       e += (int64_t)gridDim.x * 256) {
    double v = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (a.in[t]) v += a.c[t] * a.in[t][g * a.nn + e];
    if (e / a.n == e % a.n) v += a.cI;
    a.out[g * a.nn + e] = v;
  }
}

// out[g] = in[src[g]] * scale[g]
__global__ void __launch_bounds__(256) gather_scale_kernel(int64_t nn, const double* in,
                                                           const int* src,
                                                           const double* scale,
                                                           double* out) {
  const int64_t g = blockIdx.y;
  const double* s = in + (int64_t)src[g] * nn;
  const double f = scale[g];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn;
       e += (int64_t)gridDim.x * 256)
    out[g * nn + e] = s[e] * f;
}

// out[dst[g]] = in[sel[g]][g]   (sel picks one of two buffers per member)
__global__ void __launch_bounds__(256) scatter_kernel(int64_t nn, const double* in0,
                                                      const double* in1, const int* sel,
                                                      const int* dst, double* out) {
  const int64_t g = blockIdx.y;
  const double* s = (sel[g] ? in1 : in0) + g * nn;
  double* d = out + (int64_t)dst[g] * nn;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn;
       e += (int64_t)gridDim.x * 256)
    d[e] = s[e];
}

// out[g] (nb x nb, contiguous) = block (0, 0) of in[g] (row stride ld, member stride NN)
__global__ void __launch_bounds__(256) block00_kernel(int nb, int ld, int64_t NN, const double* in,
                                                      double* out) {
  const int64_t g = blockIdx.y;
  const int64_t nn = (int64_t)nb * nb;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn;
       e += (int64_t)gridDim.x * 256)
    out[g * nn + e] = in[g * NN + (e / nb) * ld + e % nb];
}

// zero the blocks (i > j) below the block diagonal of every member (kb x kb blocks of nb)
__global__ void __launch_bounds__(256) zero_lower_kernel(int nb, int kb, double* M) {
  const int64_t g = blockIdx.y;
  const int n = nb * kb;
  const int64_t NN = (int64_t)n * n;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < NN;
       e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / n), c = (int)(e % n);
    if (r / nb > c / nb) M[g * NN + e] = 0.0;
  }
}

// ||A||_1 = max_j sum_i |A_ij|, rows summed in order (numpy reduces axis 0 row by row)
__global__ void __launch_bounds__(256) norm1_kernel(int n, const double* A, double* out) {
  __shared__ double red[256];
  const double* M = A + (int64_t)blockIdx.x * n * n;
  double best = 0.0;
  for (int c = threadIdx.x; c < n; c += 256) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s += fabs(M[(int64_t)i * n + c]);
    best = fmax(best, s);
  }
  red[threadIdx.x] = best;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------------------
// LU with partial pivoting (blocked), then forward/back substitution on the right side
// ---------------------------------------------------------------------------------------
static constexpr int NB = 32;  // panel width

// Factor columns [k0, k0+kb) of rows [k0, n): unblocked right-looking LU on the panel.
__global__ void __launch_bounds__(256) panel_kernel(int n, double* Mb, int* pivb, int k0,
                                                    int kb) {
  __shared__ double rv[256];
  __shared__ int ri[256];
  double* M = Mb + (int64_t)blockIdx.x * n * n;
  int* piv = pivb + (int64_t)blockIdx.x * n;
  const int tid = threadIdx.x;
  for (int j = k0; j < k0 + kb; ++j) {
    // pivot: first row with the largest |M[i][j]|, i >= j
    double bv = -1.0;
    int bi = j;
    for (int i = j + tid; i < n; i += 256) {
      const double v = fabs(M[(int64_t)i * n + j]);
      if (v > bv) {
        bv = v;
        bi = i;
      }
    }
    rv[tid] = bv;
    ri[tid] = bi;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (tid < h) {
        const double o = rv[tid + h];
        const int oi = ri[tid + h];
        if (o > rv[tid] || (o == rv[tid] && oi < ri[tid])) {
          rv[tid] = o;
          ri[tid] = oi;
        }
      }
      __syncthreads();
    }
    const int p = ri[0];
    if (tid == 0) piv[j] = p;
    if (p != j && tid < kb) {
      const int c = k0 + tid;
      const double t = M[(int64_t)j * n + c];
      M[(int64_t)j * n + c] = M[(int64_t)p * n + c];
      M[(int64_t)p * n + c] = t;
    }
    __syncthreads();
    const double d = M[(int64_t)j * n + j];
    const double rd = 1.0 / d;
    for (int i = j + 1 + tid; i < n; i += 256) {
      double* row = M + (int64_t)i * n;
      const double lij = row[j] * rd;
      row[j] = lij;
      for (int c = j + 1; c < k0 + kb; ++c) row[c] -= lij * M[(int64_t)j * n + c];
    }
    __syncthreads();
  }
}

// panel_kernel with the panel (rows [k0, n) x kb columns) held in LDS for the whole
// factorisation: one global read and one write of the panel instead of a global round trip
// per column step (the (5,5) build's single LU of Q, n = 201: the column steps are latency-
// bound).  Same operations in the same order as panel_kernel: bit-identical factors.
constexpr int kPanelLdsBytes = 60 * 1024;
__global__ void __launch_bounds__(256) panel_lds_kernel(int n, double* Mb, int* pivb, int k0,
                                                        int kb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
  __shared__ double rv[256];
  __shared__ int ri[256];
  double* P = reinterpret_cast<double*>(psm);  // [n - k0][kb]
  double* M = Mb + (int64_t)blockIdx.x * n * n;
  int* piv = pivb + (int64_t)blockIdx.x * n;
  const int tid = threadIdx.x;
  const int rows = n - k0;
  for (int e = tid; e < rows * kb; e += 256) {
    const int r = e / kb, c = e % kb;
    P[e] = M[(int64_t)(k0 + r) * n + k0 + c];
  }
  __syncthreads();
  for (int jj = 0; jj < kb; ++jj) {
    const int j = k0 + jj;
    double bv = -1.0;
    int bi = j;
    for (int i = j + tid; i < n; i += 256) {
      const double v = fabs(P[(i - k0) * kb + jj]);
      if (v > bv) {
        bv = v;
        bi = i;
      }
    }
    rv[tid] = bv;
    ri[tid] = bi;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (tid < h) {
        const double o = rv[tid + h];
        const int oi = ri[tid + h];
        if (o > rv[tid] || (o == rv[tid] && oi < ri[tid])) {
          rv[tid] = o;
          ri[tid] = oi;
        }
      }
      __syncthreads();
    }
    const int p = ri[0];
    if (tid == 0) piv[j] = p;
    if (p != j && tid < kb) {
      const double t = P[jj * kb + tid];
      P[jj * kb + tid] = P[(p - k0) * kb + tid];
      P[(p - k0) * kb + tid] = t;
    }
    __syncthreads();
    const double rd = 1.0 / P[jj * kb + jj];
    for (int i = j + 1 + tid; i < n; i += 256) {
      double* row = P + (i - k0) * kb;
      const double lij = row[jj] * rd;
      row[jj] = lij;
      for (int c = jj + 1; c < kb; ++c) row[c] -= lij * P[jj * kb + c];
    }
    __syncthreads();
  }
  for (int e = tid; e < rows * kb; e += 256) {
    const int r = e / kb, c = e % kb;
    M[(int64_t)(k0 + r) * n + k0 + c] = P[e];
  }
}

// panel_kernel with each panel row in the registers of one thread (panel-local row t in
// thread t; at most 256 rows): per column one wave-level pivot reduction (shuffles, lowest
// index among equal maxima), one barrier to combine the four waves and hand over the pivot
// row, and the rank-1 update of the thread's own row in registers — instead of an LDS tree
// reduction with a barrier per level.  Same pivots, multipliers and update expressions in the
// same order as panel_kernel: bit-identical factors.
template <int CTRL>
__device__ __forceinline__ double dpp_mov_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}
template <int KB>
__global__ void __launch_bounds__(256) panel_reg_kernel(int n, double* Mb, int* pivb, int k0,
                                                        int kb) {
  __shared__ double prow[KB], xrow[KB];
  __shared__ double wv[4];
  __shared__ int wi[4];
  double* M = Mb + (int64_t)blockIdx.x * n * n;
  int* piv = pivb + (int64_t)blockIdx.x * n;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int rows = n - k0;
  const bool own = t < rows;
  double x[KB];
#pragma unroll
  for (int c = 0; c < KB; ++c) x[c] = (own && c < kb) ? M[(int64_t)(k0 + t) * n + k0 + c] : 0.0;
#pragma clang loop unroll(full)
  for (int jj = 0; jj < KB; ++jj) {
    if (jj >= kb) continue;  // (uniform; keeps the loop unrolled and x in registers)
    const double v = (own && t >= jj) ? fabs(x[jj]) : -1.0;
    // the wave's maximum by DPP moves within 16-lane rows and lane reads across them, then
    // its lowest lane holding it (ballot): the first maximum, as the sequential scan finds
    double mv = fmax(v, dpp_mov_f64<0xB1>(v));  // quad_perm [1,0,3,2]
    mv = fmax(mv, dpp_mov_f64<0x4E>(mv));       // quad_perm [2,3,0,1]
    mv = fmax(mv, dpp_mov_f64<0x141>(mv));      // row_half_mirror
    mv = fmax(mv, dpp_mov_f64<0x128>(mv));      // row_ror:8
    mv = fmax(fmax(readlane_f64(mv, 0), readlane_f64(mv, 16)),
              fmax(readlane_f64(mv, 32), readlane_f64(mv, 48)));
    const uint64_t hit = __ballot(v == mv);
    if (lane == 0) {
      wv[w] = mv;
      wi[w] = w * 64 + __ffsll((unsigned long long)hit) - 1;
    }
    __syncthreads();
    double bv = wv[0];
    int p = wi[0];
#pragma unroll
    for (int u = 1; u < 4; ++u)
      if (wv[u] > bv || (wv[u] == bv && wi[u] < p)) {
        bv = wv[u];
        p = wi[u];
      }
    if (t == 0) piv[k0 + jj] = k0 + p;
    if (t == p) {
#pragma unroll
      for (int c = 0; c < KB; ++c) prow[c] = x[c];
    }
    if (t == jj && p != jj) {
#pragma unroll
      for (int c = 0; c < KB; ++c) xrow[c] = x[c];
    }
    __syncthreads();
    if (p != jj && (t == jj || t == p)) {
#pragma unroll
      for (int c = 0; c < KB; ++c) x[c] = t == jj ? prow[c] : xrow[c];
    }
    const double rd = 1.0 / prow[jj];
    if (own && t > jj) {
      const double lij = x[jj] * rd;
      x[jj] = lij;
#pragma unroll
      for (int c = jj + 1; c < KB; ++c)
        if (c < kb) x[c] -= lij * prow[c];
    }
    __syncthreads();  // (prow / xrow / wv are rewritten for the next column)
  }
  if (own) {
#pragma unroll
    for (int c = 0; c < KB; ++c)
      if (c < kb) M[(int64_t)(k0 + t) * n + k0 + c] = x[c];
  }
}

// Apply the panel's row interchanges to every column outside the panel (and to R).
__global__ void __launch_bounds__(256) swap_kernel(int n, int nrhs, double* Mb, double* Rb,
                                                   const int* pivb, int k0, int kb) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n + nrhs || (c >= k0 && c < k0 + kb)) return;
  const int* piv = pivb + (int64_t)blockIdx.y * n;
  double* base;
  int ld, col;
  if (c < n) {
    base = Mb + (int64_t)blockIdx.y * n * n;
    ld = n;
    col = c;
  } else {
    base = Rb + (int64_t)blockIdx.y * n * nrhs;
    ld = nrhs;
    col = c - n;
  }
  for (int j = k0; j < k0 + kb; ++j) {
    const int p = piv[j];
    if (p != j) {
      const double t = base[(int64_t)j * ld + col];
      base[(int64_t)j * ld + col] = base[(int64_t)p * ld + col];
      base[(int64_t)p * ld + col] = t;
    }
  }
}

// rows [k0, k0+kb) of the columns right of the panel and of R: X <- L11^{-1} X
__global__ void __launch_bounds__(256) trsm_lower_kernel(int n, int nrhs, const double* Mb,
                                                         double* Mw, double* Rb, int k0,
                                                         int kb) {
  __shared__ double L[NB][NB];
  const double* M = Mb + (int64_t)blockIdx.y * n * n;
  for (int e = threadIdx.x; e < NB * NB; e += 256) {
    const int r = e / NB, c = e % NB;
    L[r][c] = (r < kb && c < kb) ? M[(int64_t)(k0 + r) * n + k0 + c] : 0.0;
  }
  __syncthreads();
  const int right = n - (k0 + kb);
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= right + nrhs) return;
  double* base;
  int ld, col;
  if (c < right) {
    base = Mw + (int64_t)blockIdx.y * n * n;
    ld = n;
    col = k0 + kb + c;
  } else {
    base = Rb + (int64_t)blockIdx.y * n * nrhs;
    ld = nrhs;
    col = c - right;
  }
  double x[NB];
#pragma unroll
  for (int a = 0; a < NB; ++a) x[a] = a < kb ? base[(int64_t)(k0 + a) * ld + col] : 0.0;
#pragma unroll
  for (int a = 0; a < NB; ++a) {
    if (a < kb) {  // rows b >= kb of L are zero-filled and their x is never stored
#pragma unroll
      for (int b = a + 1; b < NB; ++b) x[b] -= L[b][a] * x[a];
    }
  }
#pragma unroll
  for (int a = 0; a < NB; ++a)
    if (a < kb) base[(int64_t)(k0 + a) * ld + col] = x[a];
}

// rows [k0, k0+kb) of R: X <- U11^{-1} X
__global__ void __launch_bounds__(256) trsm_upper_kernel(int n, int nrhs, const double* Mb,
                                                         double* Rb, int k0, int kb) {
  __shared__ double U[NB][NB];
  const double* M = Mb + (int64_t)blockIdx.y * n * n;
  for (int e = threadIdx.x; e < NB * NB; e += 256) {
    const int r = e / NB, c = e % NB;
    U[r][c] = (r < kb && c < kb) ? M[(int64_t)(k0 + r) * n + k0 + c] : 0.0;
  }
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= nrhs) return;
  double* R = Rb + (int64_t)blockIdx.y * n * nrhs;
  double x[NB];
#pragma unroll
  for (int a = 0; a < NB; ++a) x[a] = a < kb ? R[(int64_t)(k0 + a) * nrhs + c] : 0.0;
#pragma unroll
  for (int a = NB - 1; a >= 0; --a) {
    if (a < kb) {
      x[a] /= U[a][a];
#pragma unroll
      for (int b = 0; b < a; ++b) x[b] -= U[b][a] * x[a];
    }
  }
#pragma unroll
  for (int a = 0; a < NB; ++a)
    if (a < kb) R[(int64_t)(k0 + a) * nrhs + c] = x[a];
}

hipError_t solve_batched(int n, int nrhs, int64_t batch, double* M, double* R, int* piv,
                         hipStream_t st) {
  if (batch <= 0 || n <= 0) return hipSuccess;
  const int64_t nn = (int64_t)n * n, nr = (int64_t)n * nrhs;
  for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = (int)std::min<int64_t>(65535, batch - b0);
    double* Mc = M + b0 * nn;
    double* Rc = R + b0 * nr;
    int* pc = piv + b0 * n;
    for (int k0 = 0; k0 < n; k0 += NB) {
      const int kb = std::min(NB, n - k0), k1 = k0 + kb;
      const size_t pbytes = (size_t)(n - k0) * kb * sizeof(double);
      if (n - k0 <= 256)
        hipLaunchKernelGGL(panel_reg_kernel<NB>, dim3(nb), dim3(256), 0, st, n, Mc, pc, k0, kb);
      else if (pbytes <= (size_t)kPanelLdsBytes)
        hipLaunchKernelGGL(panel_lds_kernel, dim3(nb), dim3(256), pbytes, st, n, Mc, pc, k0, kb);
      else
        hipLaunchKernelGGL(panel_kernel, dim3(nb), dim3(256), 0, st, n, Mc, pc, k0, kb);
      hipLaunchKernelGGL(swap_kernel, dim3((n + nrhs + 255) / 256, nb), dim3(256), 0, st, n,
                         nrhs, Mc, Rc, pc, k0, kb);
      const int right = n - k1;
      hipLaunchKernelGGL(trsm_lower_kernel, dim3((right + nrhs + 255) / 256, nb), dim3(256),
                         0, st, n, nrhs, Mc, Mc, Rc, k0, kb);
      if (right > 0) {
        // A22 -= L21 U12 ; R2 -= L21 R1
        Mat L21{Mc + (int64_t)k1 * n + k0, nn, n};
        Mat U12{Mc + (int64_t)k0 * n + k1, nn, n};
        Mat A22{Mc + (int64_t)k1 * n + k1, nn, n};
        if (hipError_t e = gemm(right, right, kb, L21, U12, A22, -1.0, A22, 1.0, 0.0, nullptr,
                                nb, st))
          return e;
        Mat R1{Rc + (int64_t)k0 * nrhs, nr, nrhs};
        Mat R2{Rc + (int64_t)k1 * nrhs, nr, nrhs};
        if (hipError_t e = gemm(right, nrhs, kb, L21, R1, R2, -1.0, R2, 1.0, 0.0, nullptr, nb,
                                st))
          return e;
      }
    }
    const int last = ((n - 1) / NB) * NB;
    for (int k0 = last; k0 >= 0; k0 -= NB) {
      const int kb = std::min(NB, n - k0);
      hipLaunchKernelGGL(trsm_upper_kernel, dim3((nrhs + 255) / 256, nb), dim3(256), 0, st, n,
                         nrhs, Mc, Rc, k0, kb);
      if (k0 > 0) {  // R[0:k0] -= U[0:k0, k0:k1] X[k0:k1]
        Mat U01{Mc + k0, nn, n};
        Mat X1{Rc + (int64_t)k0 * nrhs, nr, nrhs};
        Mat R0{Rc, nr, nrhs};
        if (hipError_t e = gemm(k0, nrhs, kb, U01, X1, R0, -1.0, R0, 1.0, 0.0, nullptr, nb,
                                st))
          return e;
      }
    }
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Inverse of an n x n matrix (n <= kGjMax) in one workgroup: in-place Gauss-Jordan
// ---------------------------------------------------------------------------------------
// The two inverses of a model build — Q^-1 of the deepest intervals (201 x 201 at (5,5)) and
// the Pade denominator's diagonal block of the Van Loan evaluation (203 x 203) — ran as the
// blocked LU above: ~50 dependent launches, ~0.55 ms each.  Here one workgroup holds the whole
// matrix in registers (512 threads; thread (r, c) owns rows r + 32 mr and columns c + 16 mc)
// and runs the n Gauss-Jordan steps with one barrier each: the pivot row and column go through
// LDS, then every thread applies the rank-1 update to its 7 x 13 elements.
//
// Pivots follow partial pivoting (the first maximum |a_ik|, i >= k, like LAPACK's idamax).
// Pass 1 takes the diagonal and checks at every step that no entry below it is larger in
// magnitude — then partial pivoting would have chosen the same pivots, with no interchange
// (the case for both matrices of the build).  If the check fails anywhere the workgroup
// reloads the matrix and runs pass 2: a pivot search per step, row interchanges, and the
// column interchanges of the in-place form in reverse order at the end.  The result is the
// inverse of the matrix under that pivot sequence (rounding differs from getrf + getrs).
constexpr int kGjR = 7, kGjC = 13;         // registers: rows r + 32 mr, columns c + 16 mc
constexpr int kGjMax = 16 * kGjC;          // 208
constexpr int kGjThreads = 512;

struct GjShared {
  double prow[2][kGjMax];  // the raw pivot row, by step parity
  double pcol[2][32 * kGjR];  // the multipliers (pivot column; -1 at the pivot row)
  double sw[2][32 * kGjR]; // row / column interchange buffers (pass 2; rows r + 32 mr <= 223)
  double dk[2];            // the pivot, by step parity
  double cval[32];
  int cidx[32];
  int piv[kGjMax];
  int viol;
};

// a[m][*] / a[*][m] for a workgroup-uniform register index m (the pivoting pass only)
template <int NR, int NC>
__device__ __forceinline__ void gj_row_out(const double (&a)[NR][NC], int m, double* dst, int c) {
#pragma unroll
  for (int mm = 0; mm < NR; ++mm)
    if (mm == m) {
#pragma unroll
      for (int mc = 0; mc < NC; ++mc) dst[c + 16 * mc] = a[mm][mc];
    }
}
template <int NR, int NC>
__device__ __forceinline__ void gj_row_in(double (&a)[NR][NC], int m, const double* src, int c) {
#pragma unroll
  for (int mm = 0; mm < NR; ++mm)
    if (mm == m) {
#pragma unroll
      for (int mc = 0; mc < NC; ++mc) a[mm][mc] = src[c + 16 * mc];
    }
}
template <int NR, int NC>
__device__ __forceinline__ void gj_col_out(const double (&a)[NR][NC], int m, double* dst, int r) {
#pragma unroll
  for (int mc = 0; mc < NC; ++mc)
    if (mc == m) {
#pragma unroll
      for (int mr = 0; mr < NR; ++mr) dst[r + 32 * mr] = a[mr][mc];
    }
}
template <int NR, int NC>
__device__ __forceinline__ void gj_col_in(double (&a)[NR][NC], int m, const double* src, int r) {
#pragma unroll
  for (int mc = 0; mc < NC; ++mc)
    if (mc == m) {
#pragma unroll
      for (int mr = 0; mr < NR; ++mr) a[mr][mc] = src[r + 32 * mr];
    }
}

// Step k of the elimination; MR = k >> 5 and MC = k >> 4 are compile-time register indices.
// a_ij <- (j == k ? 0 : a_ij) - f_i P_j with f_i = a_ik (-1 at i = k) and P_j = a_kj / a_kk
// (1 / a_kk at j = k): the pivot row becomes row / a_kk, the pivot column -a_ik / a_kk, the
// pivot 1 / a_kk, every other entry a_ij - a_ik a_kj / a_kk.  (P_j = a_kj * (1 / a_kk): the
// reciprocal multiplied, as LAPACK's getf2 scales its column.)
template <int MR, int MC>
__device__ __forceinline__ void gj_step(double (&a)[kGjR][kGjC], int k, int r, int c,
                                        GjShared& sh, bool check) {
  double* prow = sh.prow[k & 1];
  double* pcol = sh.pcol[k & 1];
  const bool own_row = r == (k & 31), own_col = c == (k & 15);
  if (own_row) {  // the pivot itself goes to dk, its slot in prow holds 1 (P_k = 1 / a_kk)
#pragma unroll
    for (int mc = 0; mc < kGjC; ++mc) prow[c + 16 * mc] = c + 16 * mc == k ? 1.0 : a[MR][mc];
    if (own_col) sh.dk[k & 1] = a[MR][MC];
  }
  if (own_col) {
#pragma unroll
    for (int mr = 0; mr < kGjR; ++mr) pcol[r + 32 * mr] = (r + 32 * mr == k) ? -1.0 : a[mr][MC];
  }
  __syncthreads();
  const double d = sh.dk[k & 1];
  const double inv = 1.0 / d;
  if (own_col) {
    if (check) {
      bool bad = false;
#pragma unroll
      for (int mr = 0; mr < kGjR; ++mr) bad |= (r + 32 * mr > k) && fabs(a[mr][MC]) > fabs(d);
      if (bad) sh.viol = 1;
    }
#pragma unroll
    for (int mr = 0; mr < kGjR; ++mr) a[mr][MC] = 0.0;
  }
  if (own_row) {
#pragma unroll
    for (int mc = 0; mc < kGjC; ++mc) a[MR][mc] = 0.0;
  }
  double P[kGjC];
#pragma unroll
  for (int mc = 0; mc < kGjC; ++mc) P[mc] = prow[c + 16 * mc] * inv;
#pragma unroll
  for (int mr = 0; mr < kGjR; ++mr) {
    const double f = pcol[r + 32 * mr];
#pragma unroll
    for (int mc = 0; mc < kGjC; ++mc) a[mr][mc] = fma(-f, P[mc], a[mr][mc]);
  }
}

// pass 2's row interchange before step k (pivot search over column k, rows >= k)
template <int MR, int MC>
__device__ __forceinline__ void gj_pivot(double (&a)[kGjR][kGjC], int n, int k, int r, int c,
                                         GjShared& sh) {
  if (c == (k & 15)) {
    double best = -1.0;
    int bi = 0x7fffffff;
#pragma unroll
    for (int mr = 0; mr < kGjR; ++mr) {  // rows ascend with mr: strict > keeps the first
      const int i = r + 32 * mr;
      const double v = fabs(a[mr][MC]);
      if (i >= k && i < n && v > best) {
        best = v;
        bi = i;
      }
    }
    sh.cval[r] = best;
    sh.cidx[r] = bi;
  }
  __syncthreads();
  double best = -1.0;
  int p = k;
  for (int u = 0; u < 32; ++u) {
    const double v = sh.cval[u];
    const int i = sh.cidx[u];
    if (v > best || (v == best && i < p)) {
      best = v;
      p = i;
    }
  }
  p = __builtin_amdgcn_readfirstlane(p);
  if (threadIdx.x == 0) sh.piv[k] = p;
  if (p != k) {
    if (r == (k & 31)) gj_row_out(a, MR, sh.sw[0], c);
    if (r == (p & 31)) gj_row_out(a, p >> 5, sh.sw[1], c);
    __syncthreads();
    if (r == (k & 31)) gj_row_in(a, MR, sh.sw[1], c);
    if (r == (p & 31)) gj_row_in(a, p >> 5, sh.sw[0], c);
  }
  __syncthreads();  // (cval / sw are rewritten by the next step)
}

// steps 16 MC .. 16 MC + 15 (register indices MR = MC / 2, MC), then the next 16
template <int MC, bool PIVOT>
__device__ __forceinline__ void gj_sweep(double (&a)[kGjR][kGjC], int n, int r, int c,
                                         GjShared& sh) {
  if constexpr (MC < kGjC) {
    for (int k = 16 * MC; k < 16 * MC + 16 && k < n; ++k) {
      if (PIVOT) gj_pivot<MC / 2, MC>(a, n, k, r, c, sh);
      gj_step<MC / 2, MC>(a, k, r, c, sh, !PIVOT);
    }
    gj_sweep<MC + 1, PIVOT>(a, n, r, c, sh);
  }
}

// PIVOT = false: pass 1, flag[b] = 1 where partial pivoting would interchange rows;
// PIVOT = true: pass 2 for the flagged matrices only (a launch of its own, so that its
// run-time register indices — the interchanged rows and columns — do not push pass 1's
// matrix out of registers; the flagged case does not occur in the model build)
template <bool PIVOT>
__global__ void __launch_bounds__(kGjThreads) gj_inverse_kernel(int n, const double* Mb,
                                                                double* Ob, int* flag) {
  __shared__ GjShared sh;
  if (PIVOT && flag[blockIdx.x] == 0) return;
  const double* M = Mb + (int64_t)blockIdx.x * n * n;
  double* O = Ob + (int64_t)blockIdx.x * n * n;
  const int r = threadIdx.x & 31, c = threadIdx.x >> 5;
  double a[kGjR][kGjC];
#pragma unroll
  for (int mr = 0; mr < kGjR; ++mr)
#pragma unroll
    for (int mc = 0; mc < kGjC; ++mc) {
      const int i = r + 32 * mr, j = c + 16 * mc;
      a[mr][mc] = (i < n && j < n) ? M[(int64_t)i * n + j] : 0.0;
    }
  if (threadIdx.x == 0) sh.viol = 0;
  __syncthreads();
  gj_sweep<0, PIVOT>(a, n, r, c, sh);
  __syncthreads();
  if (!PIVOT) {
    if (threadIdx.x == 0) flag[blockIdx.x] = sh.viol;
  } else {
    for (int k = n - 1; k >= 0; --k) {  // X P: column interchanges in reverse order
      const int p = sh.piv[k];
      if (p == k) continue;
      if (c == (k & 15)) gj_col_out(a, k >> 4, sh.sw[0], r);
      if (c == (p & 15)) gj_col_out(a, p >> 4, sh.sw[1], r);
      __syncthreads();
      if (c == (k & 15)) gj_col_in(a, k >> 4, sh.sw[1], r);
      if (c == (p & 15)) gj_col_in(a, p >> 4, sh.sw[0], r);
      __syncthreads();
    }
  }
#pragma unroll
  for (int mr = 0; mr < kGjR; ++mr)
#pragma unroll
    for (int mc = 0; mc < kGjC; ++mc) {
      const int i = r + 32 * mr, j = c + 16 * mc;
      if (i < n && j < n) O[(int64_t)i * n + j] = a[mr][mc];
    }
}

__global__ void __launch_bounds__(256) identity_kernel(int n, int64_t batch, double* R) {
  const int64_t nn = (int64_t)n * n;
  for (int64_t e = blockIdx.x * 256 + threadIdx.x; e < batch * nn; e += (int64_t)gridDim.x * 256) {
    const int64_t q = e % nn;
    R[e] = (q / n == q % n) ? 1.0 : 0.0;
  }
}

hipError_t inverse_batched(int n, int64_t batch, const double* M, double* out, int* piv,
                           double* work, hipStream_t st) {
  if (batch <= 0 || n <= 0) return hipSuccess;
  if (n <= kGjMax) {  // piv: one flag per matrix
    for (int64_t b0 = 0; b0 < batch; b0 += 65535) {
      const int nb = (int)std::min<int64_t>(65535, batch - b0);
      hipLaunchKernelGGL(gj_inverse_kernel<false>, dim3(nb), dim3(kGjThreads), 0, st, n,
                         M + b0 * n * n, out + b0 * n * n, piv + b0);
      hipLaunchKernelGGL(gj_inverse_kernel<true>, dim3(nb), dim3(kGjThreads), 0, st, n,
                         M + b0 * n * n, out + b0 * n * n, piv + b0);
    }
    return hipGetLastError();
  }
  // larger orders: the blocked LU on a copy, against the identity
  if (hipError_t e = hipMemcpyAsync(work, M, (size_t)batch * n * n * sizeof(double),
                                    hipMemcpyDeviceToDevice, st))
    return e;
  hipLaunchKernelGGL(identity_kernel, dim3(1024), dim3(256), 0, st, n, batch, out);
  return solve_batched(n, n, batch, work, out, piv, st);
}

// ---------------------------------------------------------------------------------------
// expm
// ---------------------------------------------------------------------------------------
// Pade coefficients b_0 .. b_m (Higham 2008, Alg. 10.20; the values of expm.py:29-140)
static const double kB3[] = {120, 60, 12, 1};
static const double kB5[] = {30240, 15120, 3360, 420, 30, 1};
static const double kB7[] = {17297280, 8648640, 1995840, 277200, 25200, 1512, 56, 1};
static const double kB9[] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0,
                             30270240.0,    2162160.0,    110880.0,     3960.0,
                             90.0,          1.0};
static const double kB13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                              1187353796428800.0,  129060195264000.0,   10559470521600.0,
                              670442572800.0,      33522128640.0,       1323241920.0,
                              40840800.0,          960960.0,            16380.0,
                              182.0,               1.0};

static hipError_t lincomb(int n, int64_t g, double* out, std::initializer_list<const double*> in,
                          std::initializer_list<double> c, double cI, hipStream_t st) {
  LinArgs a{};
  a.nn = (int64_t)n * n;
  a.n = n;
  a.out = out;
  int t = 0;
  auto ci = c.begin();
  for (const double* p : in) {
    a.in[t] = p;
    a.c[t] = *ci++;
    ++t;
  }
  a.cI = cI;
  const int bx = (int)std::min<int64_t>((a.nn + 255) / 256, 64);
  for (int64_t b0 = 0; b0 < g; b0 += 65535) {
    LinArgs h = a;
    const int64_t off = b0 * a.nn;
    h.out += off;
    for (int u = 0; u < 4; ++u)
      if (h.in[u]) h.in[u] += off;
    hipLaunchKernelGGL(lincomb_kernel, dim3(bx, (unsigned)std::min<int64_t>(65535, g - b0)),
                       dim3(256), 0, st, h);
  }
  return hipGetLastError();
}

// Products and solves of the Pade evaluation.  kb == 1: dense n x n members.  kb > 1: every
// member is block upper triangular with kb x kb blocks of order nb (n = kb nb) and all its
// diagonal blocks equal — the Van Loan matrices of vanloan.py:392-425 (diagonal blocks Q t,
// super-diagonal blocks diag(m) Q diag(m') t).  Every polynomial of such a matrix, and the
// Pade quotient, has the same structure, so only the blocks i <= j are formed: a product
// costs kb(kb+1)(kb+2)/6 block GEMMs instead of kb^3, and (V - U) R = V + U is solved by
// block back substitution with the inverse of the one diagonal block instead of an LU of
// order n.  Blocks below the diagonal of the work buffers are never read.
struct PadeOps {
  int n, nb, kb;
  hipStream_t st;
  double* inv;  // kb > 1: [G][nb][nb] inverse of the diagonal block of V - U
  double* tmp;  // kb > 1: [G][nb][nb] its LU copy
  int* piv;

  Mat blk(double* base, int i, int j) const {
    const int64_t NN = (int64_t)n * n;
    return Mat{base + (int64_t)i * nb * n + (int64_t)j * nb, NN, n};
  }
  // Z = alpha X Y + beta D + gamma I  (members selected by idx when given)
  hipError_t mul(double* X, double* Y, double* Z, double alpha, double* D, double beta,
                 double gamma, const int* idx, int64_t G) const {
    const int64_t NN = (int64_t)n * n;
    const Mat none{nullptr, 0, 0};
    if (kb == 1)
      return gemm(n, n, n, Mat{X, NN, n}, Mat{Y, NN, n}, Mat{Z, NN, n}, alpha,
                  D ? Mat{D, NN, n} : none, beta, gamma, idx, G, st);
    hipError_t e = hipSuccess;
    for (int i = 0; i < kb && !e; ++i)
      for (int j = i; j < kb && !e; ++j)
        for (int l = i; l <= j && !e; ++l) {
          const bool first = l == i;  // later terms accumulate into Z_ij
          e = gemm(nb, nb, nb, blk(X, i, l), blk(Y, l, j), blk(Z, i, j), alpha,
                   first ? (D ? blk(D, i, j) : none) : blk(Z, i, j), first ? beta : 1.0,
                   (first && i == j) ? gamma : 0.0, idx, G, st);
        }
    return e;
  }
  // M R = N for every member; R returned in `R` (kb == 1: R == N, overwritten; M
  // overwritten by its LU factors)
  hipError_t solve(double* M, double* N, double* R, int64_t G) const {
    if (kb == 1) return solve_batched(n, n, G, M, N, piv, st);
    const int64_t NN = (int64_t)n * n, bnn = (int64_t)nb * nb;
    const Mat none{nullptr, 0, 0};
    hipError_t e = hipSuccess;
    const int bx = (int)std::min<int64_t>((bnn + 255) / 256, 64);
    for (int64_t g0 = 0; !e && g0 < G; g0 += 65535) {
      hipLaunchKernelGGL(block00_kernel, dim3(bx, (unsigned)std::min<int64_t>(65535, G - g0)),
                         dim3(256), 0, st, nb, n, NN, M + g0 * NN, tmp + g0 * bnn);
      e = hipGetLastError();
    }
    if (!e) e = lincomb(nb, G, inv, {}, {}, 1.0, st);       // identity
    if (!e) e = solve_batched(nb, nb, G, tmp, inv, piv, st);  // inverse of the diagonal block
    for (int j = 0; j < kb && !e; ++j)
      for (int i = j; i >= 0 && !e; --i) {
        // N_ij -= sum_{l > i} M_il R_lj, then R_ij = inv N_ij
        for (int l = i + 1; l <= j && !e; ++l)
          e = gemm(nb, nb, nb, blk(M, i, l), blk(R, l, j), blk(N, i, j), -1.0, blk(N, i, j),
                   1.0, 0.0, nullptr, G, st);
        if (!e)
          e = gemm(nb, nb, nb, Mat{inv, bnn, nb}, blk(N, i, j), blk(R, i, j), 1.0, none, 0.0,
                   0.0, nullptr, G, st);
      }
    return e;
  }
};

// one Pade branch for a chunk of G members, already gathered + scaled into W[0]; result
// (before squaring) in W[2]
static hipError_t pade_chunk(const PadeOps& O, int64_t G, int m, double* const W[8]) {
  const int n = O.n;
  hipError_t e;
#define TRY(x)                   \
  if ((e = (x)) != hipSuccess) { \
    return e;                    \
  }
  // A2 = A @ A
  TRY(O.mul(W[0], W[0], W[1], 1.0, nullptr, 0.0, 0.0, nullptr, G));
  if (m == 13) {
    const double* b = kB13;
    TRY(O.mul(W[1], W[1], W[2], 1.0, nullptr, 0.0, 0.0, nullptr, G));  // A4
    TRY(O.mul(W[1], W[2], W[3], 1.0, nullptr, 0.0, 0.0, nullptr, G));  // A6 = A2 A4
    // U = A (A6 (b13 A6 + b11 A4 + b9 A2) + b7 A6 + b5 A4 + b3 A2 + b1 I)
    TRY(lincomb(n, G, W[4], {W[3], W[2], W[1]}, {b[13], b[11], b[9]}, 0.0, O.st));
    TRY(lincomb(n, G, W[5], {W[3], W[2], W[1]}, {b[7], b[5], b[3]}, b[1], O.st));
    TRY(O.mul(W[3], W[4], W[6], 1.0, W[5], 1.0, 0.0, nullptr, G));
    TRY(O.mul(W[0], W[6], W[7], 1.0, nullptr, 0.0, 0.0, nullptr, G));  // U -> W7
    // V = A6 (b12 A6 + b10 A4 + b8 A2) + b6 A6 + b4 A4 + b2 A2 + b0 I
    TRY(lincomb(n, G, W[4], {W[3], W[2], W[1]}, {b[12], b[10], b[8]}, 0.0, O.st));
    TRY(lincomb(n, G, W[5], {W[3], W[2], W[1]}, {b[6], b[4], b[2]}, b[0], O.st));
    TRY(O.mul(W[3], W[4], W[6], 1.0, W[5], 1.0, 0.0, nullptr, G));  // V -> W6
  } else {
    const double* b = m == 3 ? kB3 : m == 5 ? kB5 : m == 7 ? kB7 : kB9;
    const int np = m / 2;  // powers A2 .. A^(2 np) in W1 .. W(np)  (A2n = A2n @ A2)
    for (int p = 2; p <= np; ++p)
      TRY(O.mul(W[p - 1], W[1], W[p], 1.0, nullptr, 0.0, 0.0, nullptr, G));
    // U = A (b1 I + b3 A2 + ...), V = b0 I + b2 A2 + ...
    const double* P[4] = {W[1], np >= 2 ? W[2] : nullptr, np >= 3 ? W[3] : nullptr,
                          np >= 4 ? W[4] : nullptr};
    TRY(lincomb(n, G, W[5], {P[0], P[1], P[2], P[3]},
                {b[3], np >= 2 ? b[5] : 0.0, np >= 3 ? b[7] : 0.0, np >= 4 ? b[9] : 0.0},
                b[1], O.st));
    TRY(O.mul(W[0], W[5], W[7], 1.0, nullptr, 0.0, 0.0, nullptr, G));  // U -> W7
    TRY(lincomb(n, G, W[6], {P[0], P[1], P[2], P[3]},
                {b[2], np >= 2 ? b[4] : 0.0, np >= 3 ? b[6] : 0.0, np >= 4 ? b[8] : 0.0},
                b[0], O.st));  // V -> W6
  }
  // r = solve(V - U, V + U)  (expm.py:53,166)
  TRY(lincomb(n, G, W[1], {W[6], W[7]}, {1.0, -1.0}, 0.0, O.st));
  TRY(lincomb(n, G, W[2], {W[6], W[7]}, {1.0, 1.0}, 0.0, O.st));
  if (O.kb == 1) {
    TRY(O.solve(W[1], W[2], W[2], G));
  } else {  // R in W3, then back to W2 where the squarings start
    TRY(O.solve(W[1], W[2], W[3], G));
    TRY(hipMemcpyAsync(W[2], W[3], (size_t)G * n * n * sizeof(double),
                       hipMemcpyDeviceToDevice, O.st));
  }
#undef TRY
  return hipSuccess;
}

static void branch_of(double norm, int* m, int* s) {
  *s = 0;
  if (norm < 1.5e-2) *m = 3;
  else if (norm < 2.5e-1) *m = 5;
  else if (norm < 9.5e-1) *m = 7;
  else if (norm < 2.1) *m = 9;
  else {
    *m = 13;
    const double v = ceil(log(norm / 5.4) / log(2.0));
    *s = v > 0.0 ? (int)v : 0;
  }
}

// ---- small matrices (n <= 16): the whole expm of one matrix inside one workgroup ---------
// The model build's small exponentials — the emission branch propagators (4 x 4, hundreds
// per build), the two-sequence chain (15 x 15) and the one-sequence chain (2 x 2) — are
// launch- and sync-bound on the batched path (a norm pass read back by the host, then ~20
// GEMM / LU / combination launches per branch).  Here one 256-thread workgroup per matrix
// holds every intermediate in LDS (thread t owns element (t / 16, t % 16)) and runs expm.py's
// algorithm start to finish: the 1-norm (column sums in row order), the branch and scaling,
// the Pade polynomials in the reference's order (A2n = A2n @ A2 accumulation for m <= 9,
// expm.py:37-47; the nested form for m = 13, :150-163), the solve of (V - U) R = V + U by
// elimination with first-max partial pivoting (LAPACK getrf/getrs: multipliers times the
// pivot's reciprocal, then the unit-lower and upper substitutions in order) and the s
// squarings (matrix_power(r, 2**s)).
constexpr int kSmallN = 16, kSL = kSmallN + 1;
__constant__ double cB3[] = {120, 60, 12, 1};
__constant__ double cB5[] = {30240, 15120, 3360, 420, 30, 1};
__constant__ double cB7[] = {17297280, 8648640, 1995840, 277200, 25200, 1512, 56, 1};
__constant__ double cB9[] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                             2162160.0,     110880.0,     3960.0,       90.0,        1.0};
__constant__ double cB13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                              1187353796428800.0,  129060195264000.0,   10559470521600.0,
                              670442572800.0,      33522128640.0,       1323241920.0,
                              40840800.0,          960960.0,            16380.0,
                              182.0,               1.0};
__device__ __forceinline__ void sm_mul(const double (*X)[kSL], const double (*Y)[kSL],
                                       double (*Z)[kSL], int n, int i, int j) {
  if (i < n && j < n) {
    double acc = 0.0;
    for (int k = 0; k < n; ++k) acc = fma(X[i][k], Y[k][j], acc);
    Z[i][j] = acc;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) small_expm_kernel(int n, const double* __restrict__ Ab,
                                                         double* __restrict__ outb) {
#pragma clang fp contract(off)  // (products and sums rounded separately, like NumPy's)
  __shared__ double A[kSmallN][kSL], P2[kSmallN][kSL], P4[kSmallN][kSL], P6[kSmallN][kSL],
      U[kSmallN][kSL], V[kSmallN][kSL], T[kSmallN][kSL], W[kSmallN][kSL];
  __shared__ double colsum[kSmallN];
  __shared__ int piv_s;
  const int t = threadIdx.x, i = t >> 4, j = t & 15;
  const bool act = i < n && j < n;
  const double* Ain = Ab + (int64_t)blockIdx.x * n * n;
  if (act) A[i][j] = Ain[i * n + j];
  __syncthreads();
  if (t < n) {  // np.linalg.norm(A, 1): max over columns of the column's |.| sum, rows in order
    double c = 0.0;
    for (int r = 0; r < n; ++r) c += fabs(A[r][t]);
    colsum[t] = c;
  }
  __syncthreads();
  double norm = 0.0;
  for (int c = 0; c < n; ++c) norm = fmax(norm, colsum[c]);
  int m, sq = 0;
  if (norm < 1.5e-2) m = 3;
  else if (norm < 2.5e-1) m = 5;
  else if (norm < 9.5e-1) m = 7;
  else if (norm < 2.1) m = 9;
  else {
    m = 13;
    const double v = ceil(log(norm / 5.4) / log(2.0));
    sq = v > 0.0 ? (int)v : 0;
  }
  const double id = (i == j) ? 1.0 : 0.0;
  if (m == 13) {
    if (sq > 0 && act) A[i][j] = A[i][j] / ldexp(1.0, sq);  // A /= 2**s (exact)
    __syncthreads();
    const double* b = cB13;
    sm_mul(A, A, P2, n, i, j);    // A2
    sm_mul(P2, P2, P4, n, i, j);  // A4
    sm_mul(P2, P4, P6, n, i, j);  // A6
    if (act) T[i][j] = (b[13] * P6[i][j] + b[11] * P4[i][j]) + b[9] * P2[i][j];
    __syncthreads();
    sm_mul(P6, T, W, n, i, j);
    if (act) T[i][j] = (((W[i][j] + b[7] * P6[i][j]) + b[5] * P4[i][j]) + b[3] * P2[i][j]) + b[1] * id;
    __syncthreads();
    sm_mul(A, T, U, n, i, j);  // U
    if (act) T[i][j] = (b[12] * P6[i][j] + b[10] * P4[i][j]) + b[8] * P2[i][j];
    __syncthreads();
    sm_mul(P6, T, W, n, i, j);
    if (act) V[i][j] = (((W[i][j] + b[6] * P6[i][j]) + b[4] * P4[i][j]) + b[2] * P2[i][j]) + b[0] * id;
    __syncthreads();
  } else {
    const double* b = m == 3 ? cB3 : m == 5 ? cB5 : m == 7 ? cB7 : cB9;
    // U = b1 I, V = b0 I; A2n = I; per i: A2n = A2n @ A2, U += b[2i+1] A2n, V += b[2i] A2n
    sm_mul(A, A, P2, n, i, j);  // A2
    double u = b[1] * id, v = b[0] * id;
    if (act) T[i][j] = id;  // A2n
    __syncthreads();
    double (*cur)[kSL] = T;
    double (*nxt)[kSL] = W;
    for (int p = 1; p <= m / 2; ++p) {
      sm_mul(cur, P2, nxt, n, i, j);
      if (act) {
        u += b[2 * p + 1] * nxt[i][j];
        v += b[2 * p] * nxt[i][j];
      }
      double (*x)[kSL] = cur;
      cur = nxt;
      nxt = x;
    }
    if (act) {
      P4[i][j] = u;
      V[i][j] = v;
    }
    __syncthreads();
    sm_mul(A, P4, U, n, i, j);  // U = A @ U
  }
  // (V - U) R = V + U: M in T, R in W
  if (act) {
    T[i][j] = V[i][j] - U[i][j];
    W[i][j] = V[i][j] + U[i][j];
  }
  __syncthreads();
  for (int c = 0; c < n; ++c) {
    if (t == 0) {  // first row with the largest |M[r][c]|, r >= c (idamax)
      int pr = c;
      double best = fabs(T[c][c]);
      for (int r = c + 1; r < n; ++r)
        if (fabs(T[r][c]) > best) {
          best = fabs(T[r][c]);
          pr = r;
        }
      piv_s = pr;
    }
    __syncthreads();
    const int pr = piv_s;
    if (pr != c && t < 2 * kSmallN && (t & 15) < n) {  // swap rows c and pr of M and R
      double (*X)[kSL] = t < kSmallN ? T : W;
      const int col = t & 15;
      const double x = X[c][col];
      X[c][col] = X[pr][col];
      X[pr][col] = x;
    }
    __syncthreads();
    if (t > c && t < n) T[t][c] = T[t][c] * (1.0 / T[c][c]);  // multipliers
    __syncthreads();
    if (i > c && i < n && j < n) {
      const double l = T[i][c];
      if (j > c) T[i][j] = T[i][j] - l * T[c][j];
      W[i][j] = W[i][j] - l * W[c][j];
    }
    __syncthreads();
  }
  for (int c = n - 1; c >= 0; --c) {  // upper substitution, column by column
    if (t < n) W[c][t] = W[c][t] / T[c][c];
    __syncthreads();
    if (i < c && j < n) W[i][j] = W[i][j] - T[i][c] * W[c][j];
    __syncthreads();
  }
  // s squarings: r^(2^s)
  double (*cur)[kSL] = W;
  double (*nxt)[kSL] = U;
  for (int k = 0; k < sq; ++k) {
    sm_mul(cur, cur, nxt, n, i, j);
    double (*x)[kSL] = cur;
    cur = nxt;
    nxt = x;
  }
  if (act) outb[(int64_t)blockIdx.x * n * n + i * n + j] = cur[i][j];
}

hipError_t expm_batched(int n, int64_t batch, const double* A, double* out, hipStream_t st) {
  if (n >= 1 && n <= kSmallN && batch > 0) {
    for (int64_t b0 = 0; b0 < batch; b0 += 65535)
      hipLaunchKernelGGL(small_expm_kernel, dim3((unsigned)std::min<int64_t>(65535, batch - b0)),
                         dim3(256), 0, st, n, A + b0 * n * n, out + b0 * n * n);
    return hipGetLastError();
  }
  return expm_blocktri_batched(n, 1, batch, A, out, st);
}

hipError_t expm_blocktri_batched(int nb, int kb, int64_t batch, const double* A, double* out,
                                 hipStream_t st) {
  if (batch <= 0) return hipSuccess;
  if (nb <= 0 || kb <= 0) return hipErrorInvalidValue;
  const int n = nb * kb;
  const int64_t nn = (int64_t)n * n;
  hipError_t e;
  double* d_norm = nullptr;
  if ((e = hipMallocAsync((void**)&d_norm, batch * sizeof(double), st))) return e;
  for (int64_t b0 = 0; b0 < batch; b0 += 65535)
    hipLaunchKernelGGL(norm1_kernel, dim3((unsigned)std::min<int64_t>(65535, batch - b0)),
                       dim3(256), 0, st, n, A + b0 * nn, d_norm + b0);
  std::vector<double> norm(batch);
  e = hipMemcpyAsync(norm.data(), d_norm, batch * sizeof(double), hipMemcpyDeviceToHost, st);
  if (!e) e = hipStreamSynchronize(st);
  (void)hipFreeAsync(d_norm, st);
  if (e) return e;

  std::vector<int> m(batch), s(batch);
  for (int64_t b = 0; b < batch; ++b) branch_of(norm[b], &m[b], &s[b]);

  // chunk size: 8 work matrices per member, at most ~4 GiB of workspace per chunk
  const int64_t bnn = (int64_t)nb * nb;
  const int64_t per = 8 * nn * (int64_t)sizeof(double) + n * (int64_t)sizeof(int) + 64 +
                      (kb > 1 ? 2 * bnn * (int64_t)sizeof(double) : 0);
  const int64_t cap = std::max<int64_t>(1, ((int64_t)4 << 30) / per);
  for (int mm : {3, 5, 7, 9, 13}) {
    std::vector<int> members;
    for (int64_t b = 0; b < batch; ++b)
      if (m[b] == mm) members.push_back((int)b);
    for (size_t c0 = 0; c0 < members.size(); c0 += cap) {
      const int64_t G = std::min<int64_t>(cap, members.size() - c0);
      // host staging of the chunk's index / scale tables
      std::vector<int> src(G), sel(G), act;
      std::vector<double> scale(G);
      int smax = 0;
      for (int64_t g = 0; g < G; ++g) {
        const int b = members[c0 + g];
        src[g] = b;
        scale[g] = ldexp(1.0, -s[b]);  // A /= 2**s (exact)
        sel[g] = 0;
        smax = std::max(smax, s[b]);
      }
      char* ws = nullptr;
      const size_t bytes = (size_t)(8 * G * nn) * sizeof(double) + (size_t)G * n * sizeof(int) +
                           (size_t)G * (3 * sizeof(int) + sizeof(double)) + 256 +
                           (kb > 1 ? (size_t)(2 * G * bnn) * sizeof(double) : 0);
      if ((e = hipMallocAsync((void**)&ws, bytes, st))) return e;
      double* W[8];
      for (int i = 0; i < 8; ++i) W[i] = (double*)ws + (int64_t)i * G * nn;
      int* piv = (int*)(W[7] + G * nn);
      int* d_src = piv + G * n;
      int* d_sel = d_src + G;
      int* d_act = d_sel + G;
      double* d_scale = (double*)(((uintptr_t)(d_act + G) + 15) & ~(uintptr_t)15);
      PadeOps O{n, nb, kb, st, kb > 1 ? d_scale + G : nullptr,
                kb > 1 ? d_scale + G + G * bnn : nullptr, piv};
      e = hipMemcpyAsync(d_src, src.data(), G * sizeof(int), hipMemcpyHostToDevice, st);
      if (!e)
        e = hipMemcpyAsync(d_scale, scale.data(), G * sizeof(double), hipMemcpyHostToDevice, st);
      const int bx = (int)std::min<int64_t>((nn + 255) / 256, 64);
      for (int64_t g0 = 0; !e && g0 < G; g0 += 65535) {
        hipLaunchKernelGGL(gather_scale_kernel,
                           dim3(bx, (unsigned)std::min<int64_t>(65535, G - g0)), dim3(256), 0,
                           st, nn, A, d_src + g0, d_scale + g0, W[0] + g0 * nn);
        e = hipGetLastError();
      }
      if (!e) e = pade_chunk(O, G, mm, W);
      // s squarings, in lock-step: after level k the members with s >= k hold r^(2^k) in
      // W[2 + (k & 1)]  (np.linalg.matrix_power(r, 2**s), expm.py:167)
      for (int lev = 1; !e && lev <= smax; ++lev) {
        act.clear();
        for (int64_t g = 0; g < G; ++g)
          if (s[members[c0 + g]] >= lev) act.push_back((int)g);
        e = hipMemcpyAsync(d_act, act.data(), act.size() * sizeof(int), hipMemcpyHostToDevice,
                           st);
        if (!e) e = hipStreamSynchronize(st);  // act is reused next level
        double* X = W[2 + ((lev - 1) & 1)];
        double* Y = W[2 + (lev & 1)];
        if (!e) e = O.mul(X, X, Y, 1.0, nullptr, 0.0, 0.0, d_act, (int64_t)act.size());
      }
      for (int64_t g = 0; g < G; ++g) sel[g] = s[members[c0 + g]] & 1;
      if (!e) e = hipMemcpyAsync(d_sel, sel.data(), G * sizeof(int), hipMemcpyHostToDevice, st);
      for (int64_t g0 = 0; !e && g0 < G; g0 += 65535) {
        hipLaunchKernelGGL(scatter_kernel, dim3(bx, (unsigned)std::min<int64_t>(65535, G - g0)),
                           dim3(256), 0, st, nn, W[2] + g0 * nn, W[3] + g0 * nn, d_sel + g0,
                           d_src + g0, out);
        e = hipGetLastError();
      }
      // host vectors must outlive the async copies
      hipError_t e2 = hipStreamSynchronize(st);
      (void)hipFreeAsync(ws, st);
      if (e) return e;
      if (e2) return e2;
    }
  }
  if (kb > 1) {  // the blocks below the block diagonal were never formed: they are zero
    const int bx = (int)std::min<int64_t>((nn + 255) / 256, 64);
    for (int64_t b0 = 0; b0 < batch; b0 += 65535)
      hipLaunchKernelGGL(zero_lower_kernel,
                         dim3(bx, (unsigned)std::min<int64_t>(65535, batch - b0)), dim3(256),
                         0, st, nb, kb, out + b0 * nn);
    if (hipError_t e = hipGetLastError()) return e;
  }
  return hipSuccess;
}

}  // namespace itr
