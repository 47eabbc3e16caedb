// Microbenchmark: issue cost of FP64 VALU ops on gfx950 (cycles per wave-instruction),
// for 1..4 waves per SIMD.  Each wave runs 8 independent chains of the op.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int OP>
__global__ void __launch_bounds__(1024) kern(double* out, uint64_t* cyc, int iters, double seed) {
  double a[8];
  int idx[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed + threadIdx.x * 1e-3 + i; idx[i] = i; }
  const double b = seed * 0.5;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = a[i] + b;                       // v_add_f64
      if (OP == 1) a[i] = fmax(a[i], b + (double)it);     // v_max_f64 (+ add)
      if (OP == 2) { const bool g = a[i] > b; idx[i] = g ? it : idx[i]; a[i] = a[i] - 1e-9; }  // cmp + cndmask + add
      if (OP == 3) a[i] = fma(a[i], b, 1.0);              // v_fma_f64
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  double s = 0; int si = 0;
  for (int i = 0; i < 8; ++i) { s += a[i]; si += idx[i]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + si;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out; uint64_t* cyc;
  hipMalloc(&out, 1024 * 256 * sizeof(double));
  hipMalloc(&cyc, 256 * sizeof(uint64_t));
  const int iters = 4096;
  const char* names[] = {"add_f64", "add+max_f64", "cmp+cndmask+add", "fma_f64"};
  for (int op = 0; op < 4; ++op)
    for (int wps = 1; wps <= 4; ++wps) {
      const int threads = 64 * 4 * wps;  // one workgroup per CU, wps waves per SIMD
      for (int rep = 0; rep < 2; ++rep) {
        if (op == 0) hipLaunchKernelGGL(kern<0>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 1) hipLaunchKernelGGL(kern<1>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 2) hipLaunchKernelGGL(kern<2>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 3) hipLaunchKernelGGL(kern<3>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        hipDeviceSynchronize();
      }
      uint64_t c;
      hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
      // cycles per (wave-instruction-group of one chain step) per SIMD
      const double per = (double)c / (iters * 8.0) / wps;
      printf("%-16s waves/SIMD=%d  cycles per op-step per wave: %.2f (SIMD time per step %.2f)\n", names[op], wps, per * wps, per);
    }
  return 0;
}
