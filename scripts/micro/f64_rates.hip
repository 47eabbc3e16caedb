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
  double bb[8];
  for (int i = 0; i < 8; ++i) bb[i] = seed * 0.25 + threadIdx.x * 1e-4 + i;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = a[i] + b;                       // v_add_f64
      if (OP == 1) a[i] = fmax(a[i], b + (double)it);     // v_max_f64 (+ add)
      if (OP == 2) { const bool g = a[i] > b; idx[i] = g ? it : idx[i]; a[i] = a[i] - 1e-9; }  // cmp + cndmask + add
      if (OP == 3) a[i] = fma(a[i], b, 1.0);              // v_fma_f64
      if (OP == 4) asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                       : "+v"(a[i]) : "v"(bb[i]), "v"(b));  // v_fmac_f64_dpp row_newbcast
      if (OP == 5) a[i] = fma(bb[i], b, a[i]);            // v_fmac_f64 (same shape, no DPP)
      if (OP == 6 && i == 0) { a[0] = fma(a[0], b, 1.0); a[0] = fma(a[0], b, 1.0); a[0] = fma(a[0], b, 1.0); a[0] = fma(a[0], b, 1.0);
                               a[0] = fma(a[0], b, 1.0); a[0] = fma(a[0], b, 1.0); a[0] = fma(a[0], b, 1.0); a[0] = fma(a[0], b, 1.0); }  // ONE dependent chain
      if (OP == 7 && i == 0) { for (int u = 0; u < 8; ++u) { unsigned lo = __double2loint(a[0]), hi = __double2hiint(a[0]);
                               auto x = __builtin_amdgcn_permlane32_swap(lo, lo, false, false); auto y = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
                               a[0] = __hiloint2double(y[0], x[0]) + __hiloint2double(y[1], x[1]); } }  // dependent permlane32 + add
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
  const char* names[] = {"add_f64", "add+max_f64", "cmp+cndmask+add", "fma_f64", "fmac_f64_dpp", "fmac_f64", "fma dep chain", "permlane32+add dep"};
  for (int op = 0; op < 8; ++op)
    for (int wps = 1; wps <= 4; ++wps) {
      const int threads = 64 * 4 * wps;  // one workgroup per CU, wps waves per SIMD
      for (int rep = 0; rep < 2; ++rep) {
        if (op == 0) hipLaunchKernelGGL(kern<0>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 1) hipLaunchKernelGGL(kern<1>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 2) hipLaunchKernelGGL(kern<2>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 3) hipLaunchKernelGGL(kern<3>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 4) hipLaunchKernelGGL(kern<4>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 5) hipLaunchKernelGGL(kern<5>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 6) hipLaunchKernelGGL(kern<6>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
        if (op == 7) hipLaunchKernelGGL(kern<7>, dim3(256), dim3(threads), 0, 0, out, cyc, iters, 1.0);
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
