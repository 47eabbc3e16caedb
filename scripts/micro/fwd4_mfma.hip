// Prototype (not wired into the library): forward sweep of 4 HMM blocks in lock-step on
// v_mfma_f64_4x4x4_4b_f64, N <= 72 (K = 72 = 4 x 18, 80 target columns = 5 tiles of 16).
// Synthetic equal-length blocks; measures columns/s against the VALU sweep.
// Workgroup = 5 waves, wave w owns target tile w; lane: row r = l >> 4 (HMM block),
// target j = 16 w + 4 g + (l & 3) with g = (l >> 2) & 3, sources 18 (l >> 4) .. + 17.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

constexpr int NP = 72, NC = 80, KS = 18, W = 5;

__global__ void __launch_bounds__(64 * W) fwd4(const double* __restrict__ a,  // NP x NC
                                                const double* __restrict__ E,  // 625 x NC
                                                const uint16_t* __restrict__ sym,  // G x 4 x T
                                                int T, double* __restrict__ ll) {
  __shared__ double X[2][4][NP];
  __shared__ double RED[2][W][4];
  __shared__ int KR[4];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int g = (l >> 2) & 3;
  const int j = 16 * w + 4 * g + (l & 3);  // D column (target)
  const int r = l >> 4;                    // D row (block of the group)
  const int ra = l & 3;                    // A row
  const int k0 = 18 * (l >> 4);            // A/B source range
  double b[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) b[s] = a[(k0 + s) * NC + j];
  const uint16_t* sy = sym + ((size_t)blockIdx.x * 4 + r) * T;
  // column 0: alpha_0 = pi * e (synthetic: e only)
  double x = E[sy[0] * NC + j];
  if (j < NP) X[0][r][j] = x;
  int K = 0;
  __syncthreads();
  double en = E[sy[1] * NC + j];
  for (int t = 1; t < T; ++t) {
    const int buf = (t - 1) & 1;
    const double e = en;
    if (t + 1 < T) en = E[sy[t + 1] * NC + j];
    const double* xs = &X[buf][ra][k0];
    double acc0 = 0.0, acc1 = 0.0;
#pragma unroll
    for (int s = 0; s < KS; s += 2) {
      acc0 = __builtin_amdgcn_mfma_f64_4x4x4f64(xs[s], b[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_4x4x4f64(xs[s + 1], b[s + 1], acc1, 0, 0, 0);
    }
    double sc = 1.0;
    if ((t & 7) == 1 && t > 1) {  // maxima published one step earlier
      double M = RED[buf][0][r];
#pragma unroll
      for (int v = 1; v < W; ++v) M = fmax(M, RED[buf][v][r]);
      if (M > 0.0 && M < INFINITY) {
        const int ex = ilogb(M);
        sc = ldexp(1.0, -ex);
        K += ex;
      }
    }
    x = (acc0 + acc1) * e * sc;
    if (j < NP) X[buf ^ 1][r][j] = x;
    if ((t & 7) == 0) {  // row max over this wave's 16 targets
      double m = x;
      m = fmax(m, __shfl_xor(m, 1));
      m = fmax(m, __shfl_xor(m, 2));
      m = fmax(m, __shfl_xor(m, 4));
      m = fmax(m, __shfl_xor(m, 8));
      if ((l & 15) == 0) RED[buf ^ 1][w][r] = m;
    }
    __syncthreads();
  }
  // log-likelihood of each block: log(sum_j x_j) + K ln 2
  double v = (j < NP) ? x : 0.0;
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  if ((l & 15) == 0) RED[0][w][r] = v;
  if (w == 0 && (l & 15) == 0) KR[r] = K;  // the row's exponent (lanes 0..3 are all row 0)
  __syncthreads();
  if (threadIdx.x < 4) {
    double s = 0.0;
    for (int u = 0; u < W; ++u) s += RED[0][u][threadIdx.x];
    ll[blockIdx.x * 4 + threadIdx.x] = log(s) + KR[threadIdx.x] * 0.69314718055994530942;
  }
}

int main(int argc, char** argv) {
  const int n = 70, T = argc > 1 ? atoi(argv[1]) : 2000, G = argc > 2 ? atoi(argv[2]) : 1250;
  srand(1);
  std::vector<double> ha(NP * NC, 0.0), hE(625 * NC, 0.0);
  for (int i = 0; i < n; ++i) {
    double s = 0;
    for (int jj = 0; jj < n; ++jj) s += (ha[i * NC + jj] = (i == jj ? 50.0 : 1.0) * (1 + rand() % 7));
    for (int jj = 0; jj < n; ++jj) ha[i * NC + jj] /= s;
  }
  for (int o = 0; o < 625; ++o)
    for (int jj = 0; jj < n; ++jj) hE[o * NC + jj] = 0.01 + (rand() % 1000) * 1e-3;
  std::vector<uint16_t> hs((size_t)G * 4 * T);
  for (auto& v : hs) v = rand() % 625;
  double *da, *dE, *dl;
  uint16_t* ds;
  (void)hipMalloc(&da, ha.size() * 8);
  (void)hipMalloc(&dE, hE.size() * 8);
  (void)hipMalloc(&ds, hs.size() * 2);
  (void)hipMalloc(&dl, G * 4 * 8);
  (void)hipMemcpy(da, ha.data(), ha.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dE, hE.data(), hE.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, hs.data(), hs.size() * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(fwd4, dim3(G), dim3(64 * W), 0, 0, da, dE, ds, T, dl);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  // CPU check of group 0, block 0..3 (plain scaled forward)
  std::vector<double> hl(G * 4);
  (void)hipMemcpy(hl.data(), dl, hl.size() * 8, hipMemcpyDeviceToHost);
  double maxrel = 0;
  for (int bi = 0; bi < 8; ++bi) {
    const uint16_t* sy = hs.data() + (size_t)bi * T;
    std::vector<double> x(n), y(n);
    double lsum = 0;
    for (int jj = 0; jj < n; ++jj) x[jj] = hE[sy[0] * NC + jj];
    for (int t = 1; t < T; ++t) {
      double m = 0;
      for (int jj = 0; jj < n; ++jj) {
        double s = 0;
        for (int i = 0; i < n; ++i) s += x[i] * ha[i * NC + jj];
        y[jj] = s * hE[sy[t] * NC + jj];
        m = fmax(m, y[jj]);
      }
      for (int jj = 0; jj < n; ++jj) x[jj] = y[jj] / m;
      lsum += log(m);
    }
    double s = 0;
    for (int jj = 0; jj < n; ++jj) s += x[jj];
    const double ref = log(s) + lsum;
    maxrel = fmax(maxrel, fabs(hl[bi] - ref) / fabs(ref));
  }
  const double cols = (double)G * 4 * T;
  printf("fwd4 MFMA: G=%d groups x 4 blocks x T=%d: %.3f ms, %.1f M columns/s, "
         "%.1f CU-ns per column; max rel err vs CPU (8 blocks) %.2e\n",
         G, T, ms, cols / (ms * 1e-3) / 1e6, ms * 1e6 * 256 / cols, maxrel);
  return 0;
}
