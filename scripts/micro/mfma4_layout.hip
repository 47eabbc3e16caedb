// Layout probe for v_mfma_f64_4x4x4_4b_f64: for each lane p, A = e_p (1 in lane p only),
// B = lane + 1, C = 0.  The lanes of D that become nonzero and the B lanes they copy give
// the (block, row, k) of A's lane p and the (block, k, column) of B's lanes.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void probe(double* out) {
  const int l = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    const double a = (l == p) ? 1.0 : 0.0;
    const double b = l + 1.0;
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[p * 64 + l] = d;
  }
}

int main() {
  double* d;
  (void)hipMalloc(&d, 64 * 64 * sizeof(double));
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  double h[64 * 64];
  (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int p = 0; p < 64; ++p) {
    printf("A lane %2d ->", p);
    for (int l = 0; l < 64; ++l)
      if (h[p * 64 + l] != 0.0) printf(" D%d=B%d", l, (int)h[p * 64 + l] - 1);
    printf("\n");
  }
  return 0;
}
