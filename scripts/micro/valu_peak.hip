// Chip-wide FP64 VALU throughput on MI355X (gfx950), measured with HIP events: the peak the
// sweeps' roofline is priced against (bench.py reads profiles/*_valu_peak.txt).
//   fma     : v_fma_f64 chains            (2 flop per lane per instruction)
//   add     : v_add_f64 chains            (1 op per lane per instruction)
//   add+max : v_add_f64 then v_max_f64    (the Viterbi pair: 2 ops per lane per pair)
// Every lane runs NCH independent chains (so issue, not latency, bounds a full CU); the grid
// puts `wps` waves on every SIMD of every CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int NCH = 8;
constexpr int ITERS = 4096;

template <int KIND>
__global__ void __launch_bounds__(256) valu(double* out, double a, double b, double c) {
  double x[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) x[k] = threadIdx.x * 1e-3 + k;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (KIND == 0) x[k] = fma(x[k], a, b);
      if (KIND == 1) x[k] = x[k] + b;
      if (KIND == 2) x[k] = fmax(x[k] + b, c);
    }
  }
  double s = 0;
#pragma unroll
  for (int k = 0; k < NCH; ++k) s += x[k];
  if (s == 12345.678) out[0] = s;  // keeps the chains alive
}

int main(int argc, char** argv) {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  double* out;
  (void)hipMalloc(&out, 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[3] = {"fma", "add", "add+max"};
  printf("CUs %d, %d chains per lane, %d iterations\n", cus, NCH, ITERS);
  for (int wps : {1, 2, 4, 8}) {
    // 256-thread workgroups = one wave per SIMD each; wps of them per CU, one round
    const int grid = cus * wps;
    for (int kind = 0; kind < 3; ++kind) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(e0);
        if (kind == 0) hipLaunchKernelGGL(valu<0>, dim3(grid), dim3(256), 0, 0, out, 0.999999, 1e-7, -1e300);
        if (kind == 1) hipLaunchKernelGGL(valu<1>, dim3(grid), dim3(256), 0, 0, out, 0.999999, 1e-7, -1e300);
        if (kind == 2) hipLaunchKernelGGL(valu<2>, dim3(grid), dim3(256), 0, 0, out, 0.999999, -1e-7, -1e300);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
      }
      const double lanes = (double)grid * 256;
      const double instr = lanes / 64 * ITERS * NCH * (kind == 2 ? 2 : 1);  // wave-instructions
      const double ops = lanes * ITERS * NCH * (kind == 1 ? 1 : 2);          // flop / ops
      printf("%-8s waves/SIMD %d: %8.3f ms  %7.2f T%s/s  %6.2f Tinstr/s (wave64)  "
             "%.2f cycles/instr/SIMD at 2.4 GHz\n",
             names[kind], wps, best, ops / (best * 1e-3) / 1e12, kind == 0 ? "FLOP" : "op",
             instr / (best * 1e-3) / 1e12, (double)cus * 4 * 2.4e9 / (instr / (best * 1e-3)));
    }
  }
  return 0;
}
