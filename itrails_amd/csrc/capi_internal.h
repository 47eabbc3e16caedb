// capi_internal.h — what the C ABI's translation units share (capi.cpp: models, sweeps,
// dense kernels; planner.cpp: plan creation and the CU partition; host_io.cpp: the host-buffer
// entry points, MAF ingest and result writers): error reporting, host threads, device
// allocation helpers and the two opaque handle types.  Host code only.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <deque>
#include <mutex>
#include <numeric>
#include <optional>
#include <atomic>
#include <string>
#include <chrono>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/itrails_hip.h"
#include "dense.h"
#include "maf.h"
#include "writers.h"
#include "sweeps.h"

namespace itr_host {

// records the message for itr_last_error() (thread-local) and returns `code`
int fail(int code, const char* fmt, ...);

// host threads of this job: OMP_NUM_THREADS when set (the GPU pool sets it to the job's CPU
// share), else the machine's cores; at most 16
inline int host_threads() {
  const char* e = getenv("OMP_NUM_THREADS");
  int n = e ? atoi(e) : 0;
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(16, n));
}
template <class F>
inline void parallel_for(int nt, F&& f) {
  std::vector<std::thread> th;
  for (int w = 1; w < nt; ++w) th.emplace_back(f, w);
  f(0);
  for (auto& t : th) t.join();
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(ITR_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),         \
                  __FILE__, __LINE__);                                                     \
  } while (0)


inline int cu_count() {
  int dev = 0, n = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    n = 256;
  return n > 0 ? n : 256;
}

template <class T>
int dev_alloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)));
  return 0;
}
template <class T>
void dev_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

struct DevBuf {  // a temporary device buffer freed with its scope
  void* p = nullptr;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace itr_host

struct itr_model {
  int device = 0;
  int n = 0;
  double *a = nullptr, *la = nullptr, *E = nullptr, *LE = nullptr, *PIE = nullptr,
         *LPIE = nullptr, *aT = nullptr;
  // the one-block-per-wave Viterbi (wave_tasks.h), when that layout serves this state count
  // (xrw = its slot count): log E padded to xrw columns (-inf) by state (the full-scan step)
  // and in the bound-pruned step's slot order, the state of every slot, max_{i != j} log a_ij
  // per slot; built on the model's first Viterbi call (vit_slot_tables) from host copies of
  // the tables kept until then
  double* LEW = nullptr;
  double* LEWP = nullptr;
  int32_t* VSLOT = nullptr;
  double* VMB = nullptr;
  double* MJ = nullptr;  // [n] max_{i != j} log a_ij (the bound-pruned Viterbi, prune_vit.hip)
  int xrw = 0;
  std::vector<double> h_a, h_la, h_LE, h_E, h_PIE;  // (E, PIE: the 256 N-free symbols)
  std::mutex vit_mu;  // (the first Viterbi calls of several threads)
  // E padded to the per-wave matrix-core forward's width (zero columns) plus a row of ones
  // (row 625), when that layout serves this state count (wave_tasks.h)
  double* EF = nullptr;
  int erf = 0;
};

struct itr_plan {
  int device = 0;
  int64_t nblocks = 0, total = 0;
  int64_t ntiles = 0;            // Viterbi tile records: sum over blocks of ceil(T / 16)
  int64_t* d_off = nullptr;
  int64_t* d_tile_off = nullptr;  // [nblocks+1] first tile record of every block
  // posterior split (launch_post_split): the first npsplit blocks of the order get their
  // backward sweep concurrently with the forward one; beta rows at d_boff[block]
  int64_t npsplit = 0, beta_rows = 0;
  int64_t* d_boff = nullptr;
  // hybrid posterior: per-block split column of the longest blocks (0: not split), for the
  // split set cached in sublo_key (nbeta, first split column fraction)
  int64_t* d_sublo = nullptr;
  std::pair<int64_t, double> sublo_key{-1, 0.0};
  int64_t* d_comb = nullptr;  // their combine tasks {block, t0, t1} (columns (lo, T))
  int64_t ncomb = 0;
  double* d_beta = nullptr;
  size_t beta_cap = 0;
  int32_t* d_order = nullptr;
  int* d_queue = nullptr;  // work counters: [0] fwd/bwd sweeps, [1] traceback, [2] Viterbi sweep,
                           // [3, 4] hybrid sweeps, [5, 6] Viterbi hybrid, [7] per-wave Viterbi,
                           // [8, 9] the idle loop of a split hybrid launch, [10] per-wave forward,
                           // [12] mixed launch, [13] the long blocks' traceback; the hybrid
                           // posterior: [3, 4] forward-store, [5, 6] backward, [7] combine
  double* d_sink = nullptr;  // write target of padded states (64 doubles per workgroup,
                             // itr::kSinkWgs of them)
  int prio_len = INT32_MAX;  // length of the ~CU-count-th longest block
  std::vector<int64_t> sorted_len;  // block lengths, longest first (processing order)
  std::vector<int64_t> h_off;       // block offsets (host copy: the host-block entry points)
  std::vector<int32_t> h_order;     // processing order (host copy of d_order)
  // forward log-likelihood tasks {block, split, slot} (split blocks: two halves) and the
  // split blocks' scratch
  int64_t ntasks = 0, nsplit = 0;
  int32_t *d_tasks = nullptr, *d_split_blk = nullptr;
  // hybrid (matrix-core) sweeps, see itr_plan_create: forward log-likelihood = VALU tasks
  // utasks + matrix-core groups of task ids into mtasks (split slots hsplit_blk); posterior =
  // VALU blocks order[0, nurg) + groups of four consecutive blocks of order[nurg, nblocks),
  // nurg chosen per call from the state count (MfmaGeometry.pfrac)
  // Viterbi placement (viterbi_impl): the vit_nlong longest blocks (vit_long_cols columns)
  // on the 9-wave layout; the combined call's mixed queue (wave_sweeps.hip): entries >= 0 =
  // Viterbi blocks, < 0 = forward groups of groups_ll, by expected duration; tasks at least
  // mix_prio_* long run at raised wave priority
  int64_t vit_nlong = 0, vit_long_cols = 0, nmix = 0;
  int64_t vit_nlong_v = 0;  // the Viterbi-only call's long set (plan_partition)
  // CU partition (plan_partition): reserved CUs for the long blocks' Viterbi and for the
  // forward's VALU halves; wave_ok = false when the long work cannot fit half the chip
  int vit_reserve = 0, fwd_reserve = 0;
  int long_per_cu = 1;  // long Viterbi blocks a reserved CU sweeps at a time
  int fwd_per_cu = 1;   // forward VALU halves a reserved CU sweeps at a time
  bool wave_ok = true;
  int32_t* d_mix = nullptr;
  int mix_prio_fwd = INT32_MAX, mix_prio_vit = INT32_MAX;
  // per-wave Viterbi: blocks shorter than this take the bound-pruned step (wave_tasks.h), in
  // the forward+Viterbi and the Viterbi-only call
  int vit_prune_len = 0, vit_prune_len_v = 0;
  int64_t prune_override = -1;  // itr_plan_set_prune_len (negative: the planned lengths)
  int64_t nutasks = 0, ngroups_ll = 0, nhsplit = 0;
  int32_t *d_utasks = nullptr, *d_mtasks = nullptr, *d_groups_ll = nullptr,
          *d_hsplit_blk = nullptr;
  double* d_svec = nullptr;
  int* d_sK = nullptr;
  // workspace (grown on demand): forward rows (posterior) or the Viterbi checkpoint rows,
  // and the Viterbi stay-flag words
  uint16_t* d_stay = nullptr;
  size_t stay_cap = 0;
  uint8_t* d_last = nullptr;
  double* d_alpha = nullptr;
  size_t alpha_cap = 0;
};

namespace itr_host {

inline int check_model(itr_model_t m) {
  if (!m) return fail(ITR_EINVAL, "null model");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev != m->device)
    return fail(ITR_ESTATE, "model lives on device %d, current device is %d", m->device, dev);
  return 0;
}
inline int check_plan(itr_plan_t p) {
  if (!p) return fail(ITR_EINVAL, "null plan");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev != p->device)
    return fail(ITR_ESTATE, "plan lives on device %d, current device is %d", p->device, dev);
  return 0;
}

}  // namespace itr_host

