// hmm_sweeps.hip — forward / backward+posterior / Viterbi sweeps of the iTRAILS HMM on
// MI355X (gfx950, CDNA4).  Written for this chip; not a translation of any CUDA code (the
// reference has none: its sweeps are numba/NumPy loops, optimizer.py:145-354).
//
// Work decomposition
// ------------------
// A MAF block is a strictly sequential recurrence over its columns: the only parallelism
// inside a block is the N x N state contraction of one column step, and the longest block
// bounds the makespan.  One WORKGROUP of W = ceil(N/8) wavefronts (one target state per
// lane: 2-3 waves interleave on each SIMD, and a lone wave would issue FP64 at only about
// half the SIMD's rate) owns one block at a time.  Blocks are pulled
// longest-first from a device work queue, and the longest ones run at raised wave priority
// (s_setprio) against the co-resident workgroups that work through the short ones.
//
//   * wave w produces target states j = 8*RJ*w + 8*r + jl (r < RJ slots per lane), lane
//     l = 8*jl + q;
//   * the 8 lanes q = 0..7 sharing a j split the source-state sum over i into 8 ranges of
//     IQ states, i = q*IQ + k.  The lane's IQ x RJ slice of the transition matrix lives in
//     VGPRs for the whole kernel (no LDS or HBM traffic for `a` in the step loop); every LDS
//     broadcast of x_i feeds RJ FMAs;
//   * the 8 partial results are combined with three DPP stages (quad_perm, quad_perm,
//     row_half_mirror): no LDS round trip, identical results in all 8 lanes;
//   * x_{t-1} (N doubles) is the only per-step exchange: published to LDS, one LDS-only
//     barrier, read back as 16-byte broadcasts.  Cross-wave scalars (rescale maxima, the
//     posterior row sum) go through one DPP row reduction + 16 LDS partials per step.
//   * per-column inputs (emission rows, for the posterior also the stored forward rows)
//     are staged into an LDS ring 16 columns at a time, so the step loop never waits on a
//     global load; observed symbols are staged 256 at a time.
//
// Numerics
// --------
// forward / backward run in the probability domain with exact power-of-two rescaling
// (ilogb / ldexp of the running maximum every 8 columns): mathematically identical to the
// reference's log-space max-shift recursion (optimizer.py:181-187, 205-212), no
// transcendental per state per column, and the rescaling itself is rounding-free.
// Viterbi is evaluated exactly as optimizer.py:325-330 rounds it — (omega_i + log a_ij)
// then + log e_j, IEEE adds only, first maximum wins — so paths are bit-identical for
// identical tables.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "sweeps.h"

#include "valu_sweep.h"
#include "trace.h"
#include "lane_groups.h"

namespace itr {

template <int QL, int WV, int RJN, int IQ, int MODE>
__global__ void __launch_bounds__(64 * WV, (Occ<QL, WV, RJN, IQ, MODE>::value))
    sweep_kernel(SweepArgs p) {
  sweep_device<QL, WV, RJN, IQ, MODE>(p);
}

// Viterbi on small lane groups per target (lane_groups.h); the register budget holds at least
// two waves per SIMD (four-wave workgroups: two per CU, the planner pairs long blocks on a
// reserved CU) and every wave of one workgroup
template <int G, int W, int S>
__global__ void __launch_bounds__(64 * W, ((W + 3) / 4 > 2 ? (W + 3) / 4 : 2))
    vit_group_kernel(SweepArgs p) {
  vit_group_device<G, W, S>(p);
}
template <int G, int W, int S>
__global__ void __launch_bounds__(64 * W, ((W + 3) / 4 > 2 ? (W + 3) / 4 : 2))
    fwd_group_kernel(SweepArgs p) {
  fwd_group_device<G, W, S>(p);
}

// ---------------------------------------------------------------------------------------
// Viterbi traceback (optimizer.py:336-354), trace.h: one wave per block, longest first from a
// work counter (the blocks the per-wave Viterbi task did not trace itself).
// ---------------------------------------------------------------------------------------
template <int G>  // state groups of 64 lanes: n <= 64 G
__global__ void __launch_bounds__(256) vit_trace_kernel(TraceArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int l = threadIdx.x & 63;
  // this wave's rows of one tile: row u = omega at column 16 * ctile + u
  double* rows = reinterpret_cast<double*>(smem) + (size_t)(threadIdx.x >> 6) * VIT_TILE * p.n;
  for (;;) {
    int bi = 0;
    if (l == 0) bi = atomicAdd(p.queue, 1);
    bi = uni(__shfl(bi, 0));
    if (bi >= p.nblocks) break;
    const int blk = uni(p.order[bi]);
    trace_block<G>(p, rows, blk, uni((int)p.last_state[blk]));
  }
}

// ---------------------------------------------------------------------------------------
// launch helpers: (RJN, IQ) configurations by state count
// ---------------------------------------------------------------------------------------
struct Cfg {
  int ql, w, rj, iq;  // lanes per target, waves, target states per lane, sources per lane
};                    // (ql < 0: Viterbi on lane groups of -ql lanes, lane_groups.h)
static constexpr Cfg kCfgs[] = {
    // eight lanes per target, four waves (one per SIMD), several targets per lane: fewest
    // LDS reads per column, several workgroups per CU
    {8, 4, 1, 4}, {8, 4, 2, 8}, {8, 4, 3, 9}, {8, 4, 3, 12}, {8, 4, 4, 16}, {8, 4, 5, 17},
    {8, 4, 6, 24},
    // eight lanes per target, one target per lane, W = ceil(N/8) waves
    {8, 4, 1, 4}, {8, 8, 1, 8}, {8, 9, 1, 9}, {8, 12, 1, 12}, {8, 16, 1, 16}, {8, 9, 2, 17},
    {8, 8, 3, 24},
    // four lanes per target: one DPP combine stage less and twice the pairs per lane
    {4, 4, 1, 16}, {4, 5, 1, 18}, {4, 6, 1, 24}, {4, 9, 1, 34}, {4, 3, 2, 24}, {4, 4, 2, 32},
    // eight lanes per target, three targets per lane, W = ceil(N / 24) waves
    {8, 3, 3, 9}, {8, 6, 3, 17},
    // Viterbi only, lane groups (lane_groups.h): three lanes per target and 20 targets per wave
    // (N <= 72), five lanes per target and 12 targets per wave (N <= 140 / 150)
    {-3, 4, 1, 24}, {-5, 12, 1, 28}, {-5, 12, 1, 30},
    // eight lanes per target, three targets per lane, six waves, 144 sources (N <= 144)
    {8, 6, 3, 18},
    // Viterbi only, lane groups of three, two waves (N <= 30)
    {-3, 2, 1, 10}};
static constexpr int kNarrow = 7;  // entries 0..6
[[maybe_unused]] static constexpr int kNumCfgs = (int)(sizeof kCfgs / sizeof kCfgs[0]);

static int cfg_xr(int c) {
  if (kCfgs[c].ql < 0) return 4 * (16 / -kCfgs[c].ql) * kCfgs[c].w;  // lane groups
  return (64 / kCfgs[c].ql) * kCfgs[c].w * kCfgs[c].rj;
}
static bool fits(int c, int n) {
  return cfg_xr(c) >= n && (kCfgs[c].ql < 0 ? -kCfgs[c].ql : kCfgs[c].ql) * kCfgs[c].iq >= n;
}

// Measured on the (5,5) model (N = 70), 10 Mbp: the forward log-likelihood
// sweep runs fastest on three waves with three targets per lane (configuration 20), the
// posterior sweeps too, Viterbi on the one-target-per-lane kernel (9); other sizes below.
static int pick_cfg(int n, int mode) {
#if defined(ITR_DIAG) || defined(ITR_EXPERIMENT)
  // diagnostic/experiment build only: force a configuration (ITR_VIT_CFG: Viterbi only)
  const char* force = (mode == MODE_VIT && getenv("ITR_VIT_CFG")) ? getenv("ITR_VIT_CFG")
                                                                  : getenv("ITR_SWEEP_CFG");
  if (force) {
    const int c = atoi(force);
    if (c >= 0 && c < kNumCfgs && fits(c, n)) return c;
  }
#endif
  int c = -1;
  // (posterior sweeps at N = 70 on configuration 20: 465 -> 496 M columns/s,
  // scripts/gpu_cfgsmall.sh)
  if (n > 64 && n <= 72) c = mode == MODE_VIT ? 22 : 20;
  // Viterbi at 32 < N <= 64 on eight waves, one target per lane ((4,4) model, N = 46:
  // 7.3 -> 6.2 ms)
  else if (n > 32 && n <= 64 && mode == MODE_VIT) c = 8;
  // measured on the (7,7) model (N = 133, 10 Mbp, scripts/gpu_cfg133.sh): six waves with
  // three targets per lane for the probability sweeps (posterior 146 -> 175 M columns/s);
  // Viterbi on lane groups of five, twelve waves (three per SIMD): 23.4 against 25.4 ms for
  // nine waves with four lanes per target (configuration 17: three waves on SIMD 0) and 27.6
  // for groups of three on seven waves (profiles/r6b_vit_layouts.txt)
  else if (n > 128 && n <= 144)
    c = mode == MODE_VIT ? (n <= 140 ? 23 : 24) : (n <= 136 ? 21 : 25);
  // introgression (5,5) model, N = 95 (scripts/gpu_cfg95.sh): Viterbi on six waves with four
  // lanes per target (11.9 -> 11.0 ms; 10.4 against 14.8 ms for lane groups of five on eight
  // waves, profiles/r6b_vit_layouts.txt); the probability sweeps keep configuration 3
  else if (n > 72 && n <= 96 && mode == MODE_VIT) c = 16;
  // every choice must cover the state count (targets and sources), else the generic ones
  if (c >= 0 && fits(c, n)) return c;
  for (int c = 0; c < kNarrow; ++c)
    if (fits(c, n)) return c;
  return -1;
}

static size_t lds_bytes(int cfg, int mode) {
  const int w = kCfgs[cfg].w, iq = kCfgs[cfg].iq;
  if (kCfgs[cfg].ql < 0)
    return (size_t)2 * (-kCfgs[cfg].ql * iq + 64) * sizeof(double) + 5 * 64 * sizeof(double) +
           (size_t)2 * VIT_TILE * cfg_xr(cfg) * sizeof(double) + 32 * sizeof(int) +
           (size_t)2 * 64 * w * sizeof(uint16_t);
  const int xs = kCfgs[cfg].ql * (iq + (iq & 1));
  const int xr = cfg_xr(cfg);
  const int tb = 64 * w;
  const int stages = (mode == MODE_BWD) ? 2 : 1;
  return (size_t)2 * (xs + 64) * sizeof(double) + 5 * 64 * sizeof(double) +
         (size_t)stages * 2 * tile_cols(mode, xr) * xr * sizeof(double) + 32 * sizeof(int) +
         (size_t)2 * tb * sizeof(uint16_t);
}

template <int QL, int WV, int RJN, int IQ, int MODE>
static hipError_t launch_one(const SweepArgs& a, int grid, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((sweep_kernel<QL, WV, RJN, IQ, MODE>), dim3(grid), dim3(64 * WV), lds, st,
                     a);
  return hipGetLastError();
}
template <int QL, int WV, int RJN, int IQ, int MODE>
static int occ_one(size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sweep_kernel<QL, WV, RJN, IQ, MODE>,
                                                   64 * WV, lds) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}

template <int G, int W, int S>
static hipError_t dispatch_group(bool launch, const SweepArgs* a, int grid, size_t lds,
                                 hipStream_t st, int* occ) {
  static_assert(VitGroupLayout<G, W, S>::XR > 0, "layout");
  if (launch) {
    hipLaunchKernelGGL((vit_group_kernel<G, W, S>), dim3(grid), dim3(64 * W), lds, st, *a);
    return hipGetLastError();
  }
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, vit_group_kernel<G, W, S>, 64 * W, lds) !=
      hipSuccess)
    nb = 1;
  *occ = nb > 0 ? nb : 1;
  return hipSuccess;
}

template <int MODE>
static hipError_t dispatch(int cfg, bool launch, const SweepArgs* a, int grid, size_t lds,
                           hipStream_t st, int* occ) {
  if (kCfgs[cfg].ql < 0 && MODE != MODE_VIT) return hipErrorInvalidValue;
  if constexpr (MODE == MODE_VIT) {
    switch (cfg) {
      case 22: return dispatch_group<3, 4, 24>(launch, a, grid, lds, st, occ);
      case 23: return dispatch_group<5, 12, 28>(launch, a, grid, lds, st, occ);
      case 24: return dispatch_group<5, 12, 30>(launch, a, grid, lds, st, occ);
      case 26: return dispatch_group<3, 2, 10>(launch, a, grid, lds, st, occ);
    }
  }
#define ITR_CFG(C, QL, WV, RJN, IQ)                                          \
  case C:                                                                    \
    if (launch) return launch_one<QL, WV, RJN, IQ, MODE>(*a, grid, lds, st); \
    *occ = occ_one<QL, WV, RJN, IQ, MODE>(lds);                              \
    return hipSuccess;
  switch (cfg) {
    ITR_CFG(0, 8, 4, 1, 4)
    ITR_CFG(1, 8, 4, 2, 8)
    ITR_CFG(2, 8, 4, 3, 9)
    ITR_CFG(3, 8, 4, 3, 12)
    ITR_CFG(4, 8, 4, 4, 16)
    ITR_CFG(5, 8, 4, 5, 17)
    ITR_CFG(6, 8, 4, 6, 24)
    ITR_CFG(7, 8, 4, 1, 4)
    ITR_CFG(8, 8, 8, 1, 8)
    ITR_CFG(9, 8, 9, 1, 9)
    ITR_CFG(10, 8, 12, 1, 12)
    ITR_CFG(11, 8, 16, 1, 16)
    ITR_CFG(12, 8, 9, 2, 17)
    ITR_CFG(13, 8, 8, 3, 24)
    ITR_CFG(14, 4, 4, 1, 16)
    ITR_CFG(15, 4, 5, 1, 18)
    ITR_CFG(16, 4, 6, 1, 24)
    ITR_CFG(17, 4, 9, 1, 34)
    ITR_CFG(18, 4, 3, 2, 24)
    ITR_CFG(19, 4, 4, 2, 32)
    ITR_CFG(20, 8, 3, 3, 9)
    ITR_CFG(21, 8, 6, 3, 17)
    ITR_CFG(25, 8, 6, 3, 18)
  }
#undef ITR_CFG
  return hipErrorInvalidValue;
}

static hipError_t dispatch_mode(int mode, int cfg, bool launch, const SweepArgs* a, int grid,
                                size_t lds, hipStream_t st, int* occ) {
  switch (mode) {
    case MODE_FWD_LL: return dispatch<MODE_FWD_LL>(cfg, launch, a, grid, lds, st, occ);
    case MODE_FWD_STORE: return dispatch<MODE_FWD_STORE>(cfg, launch, a, grid, lds, st, occ);
    case MODE_BWD: return dispatch<MODE_BWD>(cfg, launch, a, grid, lds, st, occ);
    case MODE_VIT: return dispatch<MODE_VIT>(cfg, launch, a, grid, lds, st, occ);
  }
  return hipErrorInvalidValue;
}

SweepGeometry sweep_geometry(int n, int mode) {
  SweepGeometry g{};
  g.iq = pick_cfg(n, mode);  // configuration index (negative: unsupported)
  g.xp = 0;
  if (g.iq < 0) return g;
  g.block = 64 * kCfgs[g.iq].w;
  g.lds = lds_bytes(g.iq, mode);
  int occ = 1;
  (void)dispatch_mode(mode, g.iq, false, nullptr, 0, g.lds, nullptr, &occ);
  g.per_cu = occ;
  // the three-wave forward kernel: one workgroup per CU beyond the occupancy API's count
  // (measured on the (5,5) model, 10 Mbp: 6.0 vs 6.8 ms)
  if (g.iq == 20 && mode == MODE_FWD_LL) g.per_cu = occ + 1;
#if defined(ITR_DIAG) || defined(ITR_EXPERIMENT)
  // diagnostic/experiment build only: resident workgroups per CU
  const char* pcu = (mode == MODE_VIT && getenv("ITR_VIT_PER_CU")) ? getenv("ITR_VIT_PER_CU")
                                                                   : getenv("ITR_PER_CU");
  if (pcu && atoi(pcu) > 0) g.per_cu = atoi(pcu);
#endif
  return g;
}

// the forward's VALU tasks on lane groups: N = 65..72 (groups of three, four waves, the
// hybrid forward's 80-wide split vectors)
FwdGroupGeometry fwd_group_geometry(int n) {
  FwdGroupGeometry g{};
  if (n < 65 || n > 72) return g;
  using L = VitGroupLayout<3, 4, 24>;
  g.block = L::TB;
  g.xr = L::XR;
  g.lds = L::lds_bytes;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fwd_group_kernel<3, 4, 24>, L::TB, g.lds) !=
      hipSuccess)
    nb = 1;
  g.per_cu = nb > 0 ? nb : 1;
  return g;
}

hipError_t launch_fwd_group(const FwdGroupGeometry& g, int grid, const SweepArgs& a,
                            hipStream_t st) {
  if (g.block != 256 || grid <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL((fwd_group_kernel<3, 4, 24>), dim3(grid), dim3(g.block), g.lds, st, a);
  return hipGetLastError();
}

hipError_t launch_sweep(int mode, const SweepGeometry& g, int grid, const SweepArgs& a,
                        hipStream_t st) {
  int occ = 0;
  return dispatch_mode(mode, g.iq, true, &a, grid, g.lds, st, &occ);
}

// ---------------------------------------------------------------------------------------
// Posterior of long blocks, forward and backward concurrently.  The posterior needs
// alpha_t and beta_t at every column; alpha depends only on the block's start and beta only
// on its end, so for the longest blocks the backward sweep need not wait for the forward
// one: one persistent launch takes the long blocks' backward sweeps (storing beta rows) and
// every block's forward sweep (storing alpha rows) from one queue, long backward tasks first;
// the short blocks' backward+posterior sweep follows as usual and post_combine_kernel forms
// the long blocks' posteriors from the two stored rows.  The critical path drops from 2 T
// to T + (the longest short block) for the longest block's T.
template <int QL, int WV, int RJN, int IQ>
__global__ void __launch_bounds__(64 * WV, (Occ<QL, WV, RJN, IQ, MODE_BWD>::value))
    post_split_kernel(SweepArgs f, SweepArgs b, int nlong) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot;
  for (;;) {
    if (threadIdx.x == 0) qslot = atomicAdd(f.queue, 1);
    lds_barrier();
    const int bi = uni(qslot);
    lds_barrier();
    if (bi < nlong) {
      sweep_task<QL, WV, RJN, IQ, MODE_BWD>(b, smem, bi);
    } else if (bi - nlong < f.nblocks) {
      sweep_task<QL, WV, RJN, IQ, MODE_FWD_STORE>(f, smem, bi - nlong);
    } else {
      break;
    }
  }
}

hipError_t launch_post_split(const SweepGeometry& g, int grid, const SweepArgs& f,
                             const SweepArgs& b, int nlong, hipStream_t st) {
#define ITR_PS(C, QL, WV, RJN, IQ)                                                           \
  case C:                                                                                    \
    hipLaunchKernelGGL((post_split_kernel<QL, WV, RJN, IQ>), dim3(grid), dim3(64 * WV), g.lds, \
                       st, f, b, nlong);                                                     \
    return hipGetLastError();
  switch (g.iq) {  // the configurations pick_cfg gives the probability sweeps
    ITR_PS(0, 8, 4, 1, 4)
    ITR_PS(1, 8, 4, 2, 8)
    ITR_PS(2, 8, 4, 3, 9)
    ITR_PS(3, 8, 4, 3, 12)
    ITR_PS(4, 8, 4, 4, 16)
    ITR_PS(5, 8, 4, 5, 17)
    ITR_PS(6, 8, 4, 6, 24)
    ITR_PS(20, 8, 3, 3, 9)
    ITR_PS(21, 8, 6, 3, 17)
  }
#undef ITR_PS
  return hipErrorInvalidValue;
}

// posteriors of the split blocks' columns: alpha_t * beta_t / sum_j alpha_t[j] beta_t[j]
// (the backward sweep's own expression, optimizer.py:228-238); one wave per column
__global__ void __launch_bounds__(256) post_combine_kernel(int n, int xr, const int32_t* order,
                                                           const int64_t* off,
                                                           const double* alpha,
                                                           const double* beta,
                                                           const int64_t* beta_off,
                                                           double* post,
                                                           const int64_t* sub_lo) {
  const int blk = order[blockIdx.y];
  const int64_t c0 = off[blk];
  const int64_t T = off[blk + 1] - c0;
  const int64_t lo = sub_lo ? sub_lo[blk] : 0;  // first column with a beta row
  const int64_t t = (sub_lo ? lo + 1 : 0) + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  post_combine_column(n, xr, alpha + (c0 + t) * xr, beta + (beta_off[blk] + t - lo) * xr,
                      post + (c0 + t) * n, threadIdx.x & 63);
}

hipError_t launch_post_combine(int n, int xr, int nlong, int64_t tmax, const int32_t* order,
                               const int64_t* off, const double* alpha, const double* beta,
                               const int64_t* beta_off, double* post, hipStream_t st,
                               const int64_t* sub_lo) {
  if (nlong <= 0 || tmax <= 0) return hipSuccess;
  if (n > 192) return hipErrorInvalidValue;
  hipLaunchKernelGGL(post_combine_kernel, dim3((unsigned)((tmax + 3) / 4), (unsigned)nlong),
                     dim3(256), 0, st, n, xr, order, off, alpha, beta, beta_off, post, sub_lo);
  return hipGetLastError();
}

int sweep_row_stride(int n, int mode) {  // padded target states: row stride of bp / alpha
  const int c = pick_cfg(n, mode);
  return c < 0 ? -1 : cfg_xr(c);
}

// log P of each split block from its two halves (one wave per block)
__global__ void fwd_split_combine_kernel(int n, int xr, int nsplit, const int32_t* split_blk,
                                         const double* svec, const int* sK, double* loglik) {
  const int wv = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int l = threadIdx.x & 63;
  if (wv >= nsplit) return;
  const double* a = svec + (int64_t)wv * 2 * xr;
  const double* b = a + xr;
  double part = 0.0;
  for (int j = l; j < n; j += 64) part += a[j] * b[j];
  part = wave_sum(part);
  if (l == 0) loglik[split_blk[wv]] = log(part) + (double)(sK[2 * wv] + sK[2 * wv + 1]) * LN2;
}

hipError_t launch_fwd_split_combine(int n, int xr, int nsplit, const int32_t* split_blk,
                                    const double* svec, const int* sK, double* loglik,
                                    hipStream_t st) {
  if (nsplit <= 0) return hipSuccess;
  hipLaunchKernelGGL(fwd_split_combine_kernel, dim3((nsplit + 3) / 4), dim3(256), 0, st, n, xr,
                     nsplit, split_blk, svec, sK, loglik);
  return hipGetLastError();
}

hipError_t launch_vit_traceback(const TraceArgs& a, int grid, hipStream_t st) {
  if (a.nblocks <= 0) return hipSuccess;
  const int g = (a.n + 63) / 64;
  const size_t lds = (size_t)4 * VIT_TILE * a.n * sizeof(double);  // 4 waves' tile rows
  switch (g) {
    case 1: hipLaunchKernelGGL(vit_trace_kernel<1>, dim3(grid), dim3(256), lds, st, a); break;
    case 2: hipLaunchKernelGGL(vit_trace_kernel<2>, dim3(grid), dim3(256), lds, st, a); break;
    case 3: hipLaunchKernelGGL(vit_trace_kernel<3>, dim3(grid), dim3(256), lds, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace itr
