// emission.hip — per-hidden-state emission rows of the iTRAILS HMM.
//
// get_emission_prob_mat.py:585-698 sums, for every hidden state and each of the 256
// observed columns (a0 b0 c0 d0 in A,C,T,G order), a product of seven small transition
// tables over the unobserved ancestral nucleotides: 4^6 terms for a state with the two
// coalescences in different intervals (calc_emissions_single_JC69) and 4^4 terms for both
// in one interval (calc_emissions_double_JC69).  The reference runs these loops in pure
// Python per state (~0.6 s/state).  Here one workgroup owns one state, one lane one
// observed column; the state's tables sit in LDS and every lane walks the internal
// nucleotides in the reference's loop order (same product and accumulation order), then
// writes its column at the position the state's topology maps it to (the species-swapped
// re-keying of get_emission_prob_mat.py:871-875, 897-901).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace itr {

// table layout per state (doubles), see itrails_amd/model/emissions.py
static constexpr int ET_STRIDE = 512;
enum { ET_KIND = 0, ET_PERM = 1, ET_A = 16, ET_B = 32, ET_C = 48, ET_D = 64, ET_AB = 80,
       ET_F = 96, ET_S = 160, ET_DD = 224 };

__global__ void __launch_bounds__(256) emission_kernel(const double* __restrict__ tables,
                                                       double* __restrict__ out) {
  __shared__ double T[ET_STRIDE];
  const double* src = tables + (int64_t)blockIdx.x * ET_STRIDE;
  for (int e = threadIdx.x; e < ET_STRIDE; e += 256) T[e] = src[e];
  __syncthreads();
  const int col = threadIdx.x;
  const int a0 = col >> 6, b0 = (col >> 4) & 3, c0 = (col >> 2) & 3, d0 = col & 3;
  const bool dbl = T[ET_KIND] != 0.0;
  const int perm = (int)T[ET_PERM];
  double acc = 0.0;
  if (!dbl) {
    for (int a1 = 0; a1 < 4; ++a1)
      for (int b1 = 0; b1 < 4; ++b1)
        for (int c1 = 0; c1 < 4; ++c1)
          for (int ab0 = 0; ab0 < 4; ++ab0)
            for (int ab1 = 0; ab1 < 4; ++ab1)
              for (int abc0 = 0; abc0 < 4; ++abc0) {
                double r = 1.0;
                r *= T[ET_A + a0 * 4 + a1];
                r *= T[ET_B + b1 * 4 + b0];
                r *= T[ET_F + (a1 * 4 + b1) * 4 + ab0];
                r *= T[ET_AB + ab0 * 4 + ab1];
                r *= T[ET_S + (ab1 * 4 + c1) * 4 + abc0];
                r *= T[ET_C + c1 * 4 + c0];
                r *= T[ET_D + abc0 * 4 + d0];
                acc += r;
              }
  } else {
    for (int a1 = 0; a1 < 4; ++a1)
      for (int b1 = 0; b1 < 4; ++b1)
        for (int c1 = 0; c1 < 4; ++c1)
          for (int abc0 = 0; abc0 < 4; ++abc0) {
            double r = 1.0;
            r *= T[ET_A + a0 * 4 + a1];
            r *= T[ET_B + b1 * 4 + b0];
            r *= T[ET_C + c1 * 4 + c0];
            r *= T[ET_DD + ((a1 * 4 + b1) * 4 + c1) * 4 + abc0];
            r *= T[ET_D + abc0 * 4 + d0];
            acc += r;
          }
  }
  // topology re-keying: 1 = (a, c, b, d), 2 = (c, a, b, d)
  int k0 = a0, k1 = b0, k2 = c0;
  if (perm == 1) {
    k1 = c0;
    k2 = b0;
  } else if (perm == 2) {
    k0 = c0;
    k1 = a0;
    k2 = b0;
  }
  out[(int64_t)blockIdx.x * 256 + k0 * 64 + k1 * 16 + k2 * 4 + d0] = acc / 4;
}

hipError_t launch_emission(int n_states, const double* tables, double* out, hipStream_t st) {
  if (n_states <= 0) return hipSuccess;
  hipLaunchKernelGGL(emission_kernel, dim3(n_states), dim3(256), 0, st, tables, out);
  return hipGetLastError();
}

}  // namespace itr
