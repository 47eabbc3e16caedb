// Latency microbenchmark for the lone-block step of the sweeps (MI355X, gfx950): cycles per
// iteration (s_memtime, one workgroup on an otherwise idle GPU) of
//   add_chain   dependent v_add_f64 chain, one wave
//   max_chain   dependent (v_add_f64, v_max_f64) pair chain (z = max(z, z + c)), one wave
//   dpp_max     one 64-bit DPP stage: two v_mov_b32_dpp + v_max_f64, dependent, one wave
//   lds_rt      ds_write_b64 -> ds_read_b64 of another lane's slot, dependent, one wave
//   bar_W       LDS publish + workgroup barrier (fence local) + read, W waves
//   bar_only_W  s_barrier alone, W waves
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int IT = 2048;

__device__ __forceinline__ double dppq1(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int KIND>
__global__ void kern(double* out, uint64_t* cyc, double c) {
  __shared__ double X[1024 + 64];
  const int tid = threadIdx.x, l = tid & 63;
  double z = tid * 1e-3;
  X[tid] = z;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < IT; ++it) {
    if (KIND == 0) {
      z = z + c;
    } else if (KIND == 1) {
      z = fmax(z, z + c);
    } else if (KIND == 2) {
      z = fmax(z, dppq1(z)) + c;
    } else if (KIND == 3) {
      X[l] = z;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
      z = X[l ^ 1] + c;
    } else if (KIND == 4) {
      X[(it & 1) * 512 + tid] = z;
      lds_barrier();
      z = X[(it & 1) * 512 + (tid ^ 64)] + c;
    } else if (KIND == 5) {
      __builtin_amdgcn_s_barrier();
      z = z + c;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + tid] = z;
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
void run(const char* name, int threads, double* out, uint64_t* cyc) {
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL(kern<KIND>, dim3(1), dim3(threads), 0, 0, out, cyc, 1e-9);
  (void)hipDeviceSynchronize();
  uint64_t c = 0;
  (void)hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
  printf("%-12s threads %4d  %8.1f cycles / iteration\n", name, threads, (double)c / IT);
}

int main() {
  double* out;
  uint64_t* cyc;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMalloc(&cyc, 4096);
  run<0>("add_chain", 64, out, cyc);
  run<1>("max_chain", 64, out, cyc);
  run<2>("dpp_max", 64, out, cyc);
  run<3>("lds_rt", 64, out, cyc);
  for (int w : {1, 2, 4, 5, 8, 9, 12, 16}) {
    char nm[32];
    snprintf(nm, sizeof nm, "bar_%d", w);
    run<4>(nm, 64 * w, out, cyc);
  }
  for (int w : {2, 4, 8, 9, 16}) {
    char nm[32];
    snprintf(nm, sizeof nm, "bar_only_%d", w);
    run<5>(nm, 64 * w, out, cyc);
  }
  return 0;
}
