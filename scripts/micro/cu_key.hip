// Census: is (XCC_ID, HW_ID.se_id, HW_ID.sh_id, HW_ID.cu_id) a unique CU key on gfx950?
// 256 x 4 workgroups, each holding 96 KB of LDS (one resident per CU at a time), record the
// key; the host counts distinct keys and workgroups per key.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <map>

__global__ void census(int* out) {
  extern __shared__ double pad[];
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg(0xF804);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(0xF814);  // HW_REG_XCC_ID
    const int cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    pad[0] = hw;
    out[blockIdx.x * 2] = ((((int)(xcc & 7) * 8 + se) * 2 + sh) * 16 + cu);
    out[blockIdx.x * 2 + 1] = (int)hw;
  }
  for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(10);
}

int main() {
  const int nb = 1024;
  int* d;
  (void)hipMalloc(&d, nb * 2 * sizeof(int));
  hipLaunchKernelGGL(census, dim3(nb), dim3(64), 96 * 1024, 0, d);
  (void)hipDeviceSynchronize();
  std::vector<int> h(nb * 2);
  (void)hipMemcpy(h.data(), d, h.size() * sizeof(int), hipMemcpyDeviceToHost);
  std::map<int, int> cnt;
  int kmax = 0;
  for (int i = 0; i < nb; ++i) {
    cnt[h[2 * i]]++;
    kmax = h[2 * i] > kmax ? h[2 * i] : kmax;
  }
  printf("distinct keys %zu (max key %d) over %d workgroups; sample HW_ID 0x%08x 0x%08x\n",
         cnt.size(), kmax, nb, h[1], h[3]);
  int mn = 1 << 30, mx = 0;
  for (auto& kv : cnt) {
    mn = kv.second < mn ? kv.second : mn;
    mx = kv.second > mx ? kv.second : mx;
  }
  printf("workgroups per key: min %d max %d\n", mn, mx);
  return 0;
}
