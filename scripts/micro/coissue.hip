// Microbenchmark: do the FP64 matrix pipe and the FP64 VALU run concurrently on one SIMD of
// MI355X (gfx950)?  One workgroup per CU; its first 4*NM waves ("M", NM per SIMD) issue
// back-to-back FP64 MFMAs on independent accumulators, the next 4*NV waves ("V", NV per SIMD)
// issue v_add_f64 + v_max_f64 pairs (the Viterbi max-plus pair) on 8 independent chains.
// A third form ("I") interleaves both kinds in ONE wave.  Printed: the kernel time (HIP
// events) and each kind's chip-wide rate, so "both" can be compared with "M only" and
// "V only" (sum = separate pipes, max = shared issue).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int MCH = 8;   // accumulator chains per M wave
constexpr int VCH = 8;   // add/max chains per V wave

// MK 0: v_mfma_f64_4x4x4_4b_f64, MK 1: v_mfma_f64_16x16x4_f64
template <int NM, int NV, int MK, int IL>
__global__ void __launch_bounds__(256 * (NM + NV)) kern(double* out, int iters, double b0,
                                                         double c0) {
  const int w = threadIdx.x >> 6;
  const double a = 1.0 + threadIdx.x * 1e-9, b = 0.5 - threadIdx.x * 1e-10;
  double s = 0.0;
  if (w < 4 * NM) {
    double c1[MCH];
    d4 c[MCH];
#pragma unroll
    for (int i = 0; i < MCH; ++i) {
      c1[i] = 1.0 + i;
      c[i] = d4{1.0 * i, 1.0, 2.0, 3.0};
    }
    double x[VCH];
#pragma unroll
    for (int k = 0; k < VCH; ++k) x[k] = threadIdx.x * 1e-3 + k;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < MCH; ++i) {
        if (MK == 0) c1[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1[i], 0, 0, 0);
        else c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
        if (IL) {  // IL add/max pairs per MFMA in the same wave
#pragma unroll
          for (int k = 0; k < IL; ++k) x[(i * IL + k) % VCH] = fmax(x[(i * IL + k) % VCH] + b0, c0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < MCH; ++i) s += MK == 0 ? c1[i] : c[i][0] + c[i][3];
#pragma unroll
    for (int k = 0; k < VCH; ++k) s += x[k];
  } else {
    double x[VCH];
#pragma unroll
    for (int k = 0; k < VCH; ++k) x[k] = threadIdx.x * 1e-3 + k;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < VCH; ++k) x[k] = fmax(x[k] + b0, c0);
    }
#pragma unroll
    for (int k = 0; k < VCH; ++k) s += x[k];
  }
  if (s == 12345.678) out[0] = s;
}

template <int NM, int NV, int MK, int IL>
void run(const char* name, int cus, double* out) {
  const int iters = 4096;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((kern<NM, NV, MK, IL>), dim3(cus), dim3(256 * (NM + NV)), 0, 0, out,
                       iters, -1e-7, -1e300);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  const double mflop = (double)cus * 4 * NM * 64 * iters * MCH * (MK == 0 ? 8.0 : 32.0);  // per lane: 4x4x4_4b 512/64, 16x16x4 2048/64
  const double vops = (double)cus * 4 * NV * 64 * iters * VCH * 2.0 +
                      (double)cus * 4 * NM * 64 * iters * MCH * IL * 2.0;
  printf("%-34s %8.3f ms   MFMA %6.2f TFLOP/s   VALU add+max %6.2f Tops/s\n", name, best,
         mflop / (best * 1e-3) / 1e12, vops / (best * 1e-3) / 1e12);
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  double* out;
  (void)hipMalloc(&out, 8);
  printf("CUs %d; M waves: %d MFMA chains, V waves: %d add+max chains, 4096 iterations\n", cus,
         MCH, VCH);
  run<1, 0, 0, 0>("4x4x4_4b: 1 M/SIMD", cus, out);
  run<0, 1, 0, 0>("V: 1 V/SIMD", cus, out);
  run<1, 1, 0, 0>("4x4x4_4b: 1 M + 1 V per SIMD", cus, out);
  run<0, 2, 0, 0>("V: 2 V/SIMD", cus, out);
  run<1, 2, 0, 0>("4x4x4_4b: 1 M + 2 V per SIMD", cus, out);
  run<2, 2, 0, 0>("4x4x4_4b: 2 M + 2 V per SIMD", cus, out);
  run<1, 0, 0, 1>("4x4x4_4b: 1 wave, 1 pair/MFMA", cus, out);
  run<1, 0, 0, 2>("4x4x4_4b: 1 wave, 2 pairs/MFMA", cus, out);
  run<1, 0, 0, 4>("4x4x4_4b: 1 wave, 4 pairs/MFMA", cus, out);
  run<1, 0, 1, 0>("16x16x4: 1 M/SIMD", cus, out);
  run<1, 1, 1, 0>("16x16x4: 1 M + 1 V per SIMD", cus, out);
  run<1, 2, 1, 0>("16x16x4: 1 M + 2 V per SIMD", cus, out);
  run<1, 0, 1, 2>("16x16x4: 1 wave, 2 pairs/MFMA", cus, out);
  run<1, 0, 1, 4>("16x16x4: 1 wave, 4 pairs/MFMA", cus, out);
  run<1, 0, 1, 8>("16x16x4: 1 wave, 8 pairs/MFMA", cus, out);
  return 0;
}
