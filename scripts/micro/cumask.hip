// Which physical CUs does a CU-masked stream use?  For several masks over the 256 logical
// CU bits, launch 2048 short workgroups and record each one's (XCC, SE, SH, CU) hardware id;
// print the number of distinct CUs and how many workgroups ran at once per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <set>
#include <vector>

__global__ void who(uint32_t* out, int spin) {
  if (threadIdx.x == 0) {
    uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)); // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    const uint64_t t0 = __builtin_readcyclecounter();
    while (__builtin_readcyclecounter() - t0 < (uint64_t)spin) {}
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", cus);
  const int nwg = 2048;
  uint32_t* d;
  hipMalloc(&d, nwg * 2 * sizeof(uint32_t));
  std::vector<uint32_t> h(nwg * 2);
  struct M { const char* name; std::vector<uint32_t> m; };
  std::vector<M> masks;
  auto mk = [&](const char* name, auto pred) {
    std::vector<uint32_t> m((cus + 31) / 32, 0);
    int c = 0;
    for (int i = 0; i < cus; ++i)
      if (pred(i)) { m[i / 32] |= 1u << (i % 32); ++c; }
    masks.push_back({name, m});
    printf("mask %s: %d bits\n", name, c);
  };
  mk("all", [](int) { return true; });
  mk("first64", [](int i) { return i < 64; });
  mk("spread64", [&](int i) { for (int k = 0; k < 64; ++k) if (k * cus / 64 == i) return true; return false; });
  mk("spread100", [&](int i) { for (int k = 0; k < 100; ++k) if (k * cus / 100 == i) return true; return false; });
  mk("first100", [](int i) { return i < 100; });
  mk("even", [](int i) { return i % 2 == 0; });
  mk("mod8_0", [](int i) { return i % 8 == 0; });
  for (int b = 0; b < 16; ++b) {  // single logical bits: which physical CU is bit b?
    static char nm[16][16];
    snprintf(nm[b], 16, "bit%d", b * 17 % 256);
    const int bb = b * 17 % 256;
    mk(nm[b], [bb](int i) { return i == bb; });
  }
  for (int b = 0; b < 8; ++b) {
    static char nm2[8][16];
    snprintf(nm2[b], 16, "bit%d", b);
    mk(nm2[b], [b](int i) { return i == b; });
  }
  for (auto& M : masks) {
    hipStream_t s;
    hipExtStreamCreateWithCUMask(&s, (uint32_t)M.m.size() * 32, M.m.data());
    hipLaunchKernelGGL(who, dim3(nwg), dim3(64), 0, s, d, 20000);
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::set<uint64_t> cu;
    std::set<uint32_t> xcc;
    for (int i = 0; i < nwg; ++i) {
      const uint32_t hw = h[2 * i];
      const uint32_t cuid = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const uint32_t x = h[2 * i + 1] & 0xF;
      cu.insert(((uint64_t)x << 16) | (se << 8) | (sh << 4) | cuid);
      xcc.insert(x);
    }
    printf("%-10s distinct CUs %zu, XCCs %zu", M.name, cu.size(), xcc.size());
    if (cu.size() <= 2)
      for (uint64_t c : cu)
        printf("  [xcc %u se %u sh %u cu %u]", (unsigned)(c >> 16), (unsigned)((c >> 8) & 0xff),
               (unsigned)((c >> 4) & 0xf), (unsigned)(c & 0xf));
    printf("\n");
    hipStreamDestroy(s);
  }
  return 0;
}
