// CU-mask semantics on MI355X: which physical CUs (XCC, SE, SH, CU from HW_ID / XCC_ID) does a
// stream created with hipExtStreamCreateWithCUMask run on?  Masks with one logical bit per
// XCC under two hypotheses of the bit -> XCC mapping, and the reserved/bulk masks of the
// sweep partition.  Prints per mask: distinct CUs and CUs per XCC.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <map>
#include <set>
#include <string>
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
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("CUs %d\n", cus);
  const int nwg = 4096;
  uint32_t* d;
  (void)hipMalloc(&d, nwg * 2 * sizeof(uint32_t));
  std::vector<uint32_t> h(nwg * 2);
  std::vector<std::pair<std::string, std::vector<int>>> masks;
  auto add = [&](std::string name, std::vector<int> bits) { masks.push_back({name, bits}); };
  std::vector<int> v;
  for (int x = 0; x < 8; ++x) v.push_back(x);
  add("bits0-7", v);
  v.clear();
  for (int x = 0; x < 8; ++x) v.push_back(32 * x);
  add("bits32x", v);
  v.clear();
  for (int x = 0; x < 16; ++x) v.push_back(x);
  add("bits0-15", v);
  v.clear();
  for (int x = 8; x < 16; ++x) v.push_back(x);
  add("bits8-15", v);
  v.clear();
  for (int x = 0; x < 64; ++x) v.push_back(x);
  add("first64", v);
  v.clear();
  for (int k = 0; k < 64; ++k) v.push_back((int)((int64_t)k * cus / 64));
  add("every4th", v);
  v.clear();
  for (int i = 0; i < cus; ++i) if (i % 4 != 0) v.push_back(i);
  add("not4th", v);
  v.clear();
  for (int i = 0; i < cus; ++i) if ((i / 8) % 4 == 0) v.push_back(i);
  add("oct_of4", v);  // 8 consecutive bits out of every 32
  v.clear();
  for (int i = 0; i < cus; ++i) if ((i / 8) % 4 != 0) v.push_back(i);
  add("not_oct", v);
  for (int k = 0; k < cus / 8; ++k) {  // local CU index k in every XCC
    v.clear();
    for (int x = 0; x < 8; ++x) v.push_back(8 * k + x);
    char nm[16];
    snprintf(nm, sizeof nm, "local%d", k);
    add(nm, v);
  }
  for (auto& M : masks) {
    std::vector<uint32_t> m((cus + 31) / 32, 0);
    for (int b : M.second) m[b / 32] |= 1u << (b % 32);
    hipStream_t s;
    (void)hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size() * 32, m.data());
    hipLaunchKernelGGL(who, dim3(nwg), dim3(64), 0, s, d, 20000);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::set<uint64_t> cu;
    std::map<uint32_t, std::set<uint32_t>> per;
    for (int i = 0; i < nwg; ++i) {
      const uint32_t hw = h[2 * i];
      const uint32_t cuid = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
      const uint32_t x = h[2 * i + 1] & 0xF;
      const uint32_t local = (se << 8) | (sh << 4) | cuid;
      cu.insert(((uint64_t)x << 16) | local);
      per[x].insert(local);
    }
    printf("%-9s bits %3zu -> CUs %3zu  per XCC:", M.first.c_str(), M.second.size(), cu.size());
    for (auto& [x, s2] : per) printf(" %u:%zu", x, s2.size());
    if (cu.size() <= 16) {
      printf("  {");
      for (uint64_t c : cu)
        printf(" x%u.se%u.sh%u.cu%u", (unsigned)(c >> 16), (unsigned)((c >> 8) & 0xff),
               (unsigned)((c >> 4) & 0xf), (unsigned)(c & 0xf));
      printf(" }");
    }
    printf("\n");
    (void)hipStreamDestroy(s);
  }
  return 0;
}
