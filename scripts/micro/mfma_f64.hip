// Microbenchmark: v_mfma_f64_16x16x4_f64 and v_mfma_f64_4x4x4_4b_f64 on gfx950 — cycles per instruction for one
// dependent accumulator chain (latency) and for 4 independent chains per wave (issue rate),
// 1..4 waves per SIMD.  Evidence for DESIGN.md §3 "why the sweeps stay on the VALU".
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

// SMALL = 0: v_mfma_f64_16x16x4_f64 (one 16x16 output, K = 4);
// SMALL = 1: v_mfma_f64_4x4x4_4b_f64 (four independent 4x4x4 products, one C value per lane)
template <int CH, int SMALL>
__global__ void __launch_bounds__(1024) kern(double* out, uint64_t* cyc, int iters) {
  const double a = 1.0 + threadIdx.x * 1e-6, b = 0.5 - threadIdx.x * 1e-7;
  d4 c[CH];
  double c1[CH];
  for (int i = 0; i < CH; ++i) c[i] = d4{0.0 + i, 1.0, 2.0, 3.0};
  for (int i = 0; i < CH; ++i) c1[i] = 1.0 + i;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (SMALL) c1[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1[i], 0, 0, 0);
      else c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < CH; ++i) s += SMALL ? c1[i] : c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  uint64_t* cyc;
  hipMalloc(&out, 1024 * 256 * sizeof(double));
  hipMalloc(&cyc, 256 * sizeof(uint64_t));
  const int iters = 4096;
  for (int small : {0, 1})
  for (int ch : {1, 4})
    for (int wps = 1; wps <= 4; ++wps) {
      const int threads = 64 * 4 * wps;  // one workgroup per CU, wps waves per SIMD
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float ms = 0;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (ch == 1 && !small) hipLaunchKernelGGL((kern<1, 0>), dim3(256), dim3(threads), 0, 0, out, cyc, iters);
        if (ch == 4 && !small) hipLaunchKernelGGL((kern<4, 0>), dim3(256), dim3(threads), 0, 0, out, cyc, iters);
        if (ch == 1 && small) hipLaunchKernelGGL((kern<1, 1>), dim3(256), dim3(threads), 0, 0, out, cyc, iters);
        if (ch == 4 && small) hipLaunchKernelGGL((kern<4, 1>), dim3(256), dim3(threads), 0, 0, out, cyc, iters);
        hipEventRecord(e1);
        hipDeviceSynchronize();
        hipEventElapsedTime(&ms, e0, e1);
      }
      uint64_t c;
      hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
      const double per_wave = (double)c / (iters * (double)ch);  // cycles per MFMA per wave
      // 16x16x4: 16*16*4*2 = 2048 flop; 4x4x4_4b: four 4x4x4 blocks = 512 flop (one C
      // element per lane)
      const double flops = 256.0 * threads / 64 * iters * ch * (small ? 512 : 2048);
      printf("%s chains=%d waves/SIMD=%d  cycles per mfma per wave %.2f  (SIMD %.2f)  "
             "%.1f TFLOP/s whole GPU (event %.3f ms)\n",
             small ? "4x4x4_4b" : "16x16x4 ", ch, wps, per_wave, per_wave / wps, flops / (ms * 1e-3) / 1e12, ms);
    }
  return 0;
}
