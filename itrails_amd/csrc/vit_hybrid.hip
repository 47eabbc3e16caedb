// vit_hybrid.hip — the Viterbi sweep (optimizer.py:305-333) as one persistent launch with
// two kinds of tasks on MI355X (gfx950):
//
//  * the longest blocks, one per workgroup, on the latency-optimised VALU layout of
//    valu_sweep.h (8 lanes per target, one target per lane; the waves whose targets are all
//    padding skip the arithmetic), so the longest block runs at the lone-block step time;
//  * the bulk as groups of G blocks of similar length stepped in lock-step: two lanes per
//    (block, target), each taking the max-plus chain over half of the sources, one DPP
//    exchange to combine — a quarter of the combine and tail instructions per useful
//    add/max of the 8-lane layout, which is what bounds the bulk (VALU issue: round-1
//    instruction census).
//
// Both produce exactly the outputs of the VALU sweep — omega checkpoint rows every 16
// columns, 16-bit stay-flag words, the last column's first argmax — with the reference's
// rounding: omega_t[j] = max(yd, yo), yd = (omega_j + log a_jj) + log e_j,
// yo = max_{i != j}(omega_i + log a_ij) + log e_j (IEEE rounding is monotone), so the
// traceback (hmm_sweeps.hip) is shared and paths are bit-identical.
//
// Measured (1x MI355X, (5,5) model, 10 Mbp, scripts/gpu_vith.sh): 7.41 ms at the best urgent
// share (0.5) against 7.46 ms for the VALU-only sweep, and 7.31 ms on short blocks (mean 300
// columns) against 6.24 ms for the three-wave VALU configuration: the lock-step groups halve
// the VALU instructions per column but run one 12-wave workgroup per CU (the 36-value slice
// of log a per lane), which leaves every barrier and LDS burst exposed.  Not adopted: built
// into the experiment library only (ITR_EXPERIMENT, enabled by ITR_VIT_HYBRID=1).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {
#ifdef ITR_EXPERIMENT
namespace {

// LDS of a bulk group task: X[2][GM][XB] published omega vectors, Y[GM][XB] last rows
template <int W, int QL, int IQ>
struct VLds {
  static constexpr int XB = QL * IQ + (QL * IQ) % 2;
  static constexpr int GM = (64 * W) / (QL * (QL * (IQ - 1) + 1));  // blocks per group (max)
  static constexpr size_t bytes = (size_t)3 * GM * XB * 8;
};

// One bulk task: blocks grp[0 .. G) (-1: none) stepped in lock-step, QL lanes per (block,
// target), each taking the max-plus chain over IQ sources; G = (64 W) / (QL n).
template <int W, int QL, int IQ>
__device__ __forceinline__ void vit_group_task(const SweepArgs& p, unsigned char* smem,
                                               const int32_t* grp, int G, int xr) {
  constexpr int XB = VLds<W, QL, IQ>::XB;
  constexpr int GM = VLds<W, QL, IQ>::GM;
  constexpr int TB = 64 * W;
  constexpr int TE = 4;     // emission prefetch tile
  constexpr int NCH = 3;    // independent max chains per lane
  double* X = reinterpret_cast<double*>(smem);  // [2][GM][XB]
  double* Y = X + 2 * GM * XB;                  // [GM][XB]
  const int n = p.n;
  const int g = threadIdx.x;
  const int LB = QL * n;                          // lanes per block
  const int bq = g / LB;                          // block row of this lane (>= G: idle)
  const bool live = bq < G;
  const int b = live ? bq : 0;
  const int u = g - bq * LB;
  const int j = live ? u / QL : 0;                // target state
  const int q = u % QL;                           // source range
  const int blk = live ? grp[b] : -1;
  const int64_t c0 = blk >= 0 ? p.off[blk] : 0;
  const int T = blk >= 0 ? (int)(p.off[blk + 1] - c0) : 0;
  const bool act = blk >= 0 && T > 0;
  int Tmax = 0;
  for (int r = 0; r < G; ++r) {
    const int b2 = grp[r];
    if (b2 >= 0) Tmax = max(Tmax, (int)(p.off[b2 + 1] - p.off[b2]));
  }
  Tmax = uni(Tmax);
  const int64_t tk0 = blk >= 0 ? p.tile_off[blk] : 0;

  // this lane's IQ entries of column j of log a (the diagonal kept out of the chain, see
  // the VALU Viterbi in valu_sweep.h); sources beyond n read -inf from the padded vector
  double m[IQ];
#pragma unroll
  for (int k = 0; k < IQ; ++k) {
    const int i = q * IQ + k;
    m[k] = (act && i < n) ? (i == j ? -INFINITY : p.mat[(int64_t)i * n + j]) : 0.0;
  }
  const double ldiag = act ? p.mat[(int64_t)j * n + j] : 0.0;
  for (int i = g; i < 2 * GM * XB; i += TB) X[i] = -INFINITY;
  lds_barrier();

  auto sym = [&](int t) -> int {
    return act ? min((int)p.obs[c0 + min(t, T - 1)], 624) : 0;
  };
  double x = act ? p.init[sym(0) * n + j] : -INFINITY;
  double xfin = x;
  const bool pub = live && q == 0;
  if (pub) X[b * XB + j] = x;
  if (pub && act) p.alpha[tk0 * xr + j] = x;
  double enxt[TE];
  int snxt[TE];
#pragma unroll
  for (int v = 0; v < TE; ++v) {
    enxt[v] = act ? p.emit[sym(v) * n + j] : 0.0;
    snxt[v] = sym(TE + v);
  }
  wait_vmem_all();
  lds_barrier();
  for (int t0 = 0; t0 < Tmax; t0 += VIT_TILE) {
    const int64_t rec = (tk0 + t0 / VIT_TILE) * xr;  // this tile's checkpoint / flag record
    uint32_t bits = 0;
    double ecur[TE];
#pragma unroll
    for (int sub = 0; sub < VIT_TILE; ++sub) {
      if (sub % TE == 0) {  // the next prefetch tile: emissions loaded TE columns ago
#pragma unroll
        for (int v = 0; v < TE; ++v) ecur[v] = enxt[v];
#pragma unroll
        for (int v = 0; v < TE; ++v) {
          enxt[v] = act ? p.emit[snxt[v] * n + j] : 0.0;
          snxt[v] = sym(t0 + sub + 2 * TE + v);
        }
      }
      const int t = t0 + sub;
      if (t >= 1 && t < Tmax) {
        const int buf = (t - 1) & 1;
        const double* xs = X + (buf * GM + b) * XB + q * IQ;
        // sources in chunks of 8 with scheduling barriers between them, so at most one
        // chunk of the published vector is live in registers beside the slice of log a
        double bc[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) bc[c] = xs[c] + m[c];
#pragma unroll
        for (int k = NCH; k < IQ; ++k) {
          if (k % 8 == 0) __builtin_amdgcn_sched_barrier(0);
          bc[k % NCH] = fmax(bc[k % NCH], xs[k] + m[k]);
        }
        double zo = bc[0];
#pragma unroll
        for (int c = 1; c < NCH; ++c) zo = fmax(zo, bc[c]);
        // the other source ranges of this target: the QL lanes of a quad / pair
        zo = fmax(zo, dpp_f64<0xB1>(zo));                  // quad_perm [1,0,3,2]
        if constexpr (QL == 4) zo = fmax(zo, dpp_f64<0x4E>(zo));  // quad_perm [2,3,0,1]
        const double ec = ecur[sub % TE];
        const double yd = (x + ldiag) + ec;
        const double yo = zo + ec;
        bits |= (uint32_t)(yd > yo) << sub;
        x = fmax(yd, yo);
        if (pub && t < T) {
          if (sub == 0) p.alpha[rec + j] = x;  // the tile's checkpoint row
          if (sub == VIT_TILE - 1 || t == T - 1) p.stay[rec + j] = (uint16_t)bits;
        }
        if (t == T - 1) xfin = x;
        if (pub) X[((buf ^ 1) * GM + b) * XB + j] = x;
        lds_barrier();
      }
    }
  }
  // last state of every block = first argmax of its last omega row (optimizer.py:346)
  if (pub) Y[b * XB + j] = xfin;
  lds_barrier();
  if (g < G && grp[g] >= 0 && p.off[grp[g] + 1] > p.off[grp[g]]) {
    const double* yr = Y + g * XB;
    double bv = yr[0];
    int bj = 0;
    for (int i = 1; i < n; ++i)
      if (yr[i] > bv) {
        bv = yr[i];
        bj = i;
      }
    p.last_state[grp[g]] = (uint8_t)bj;
  }
  lds_barrier();
}

// v.order[0, nurg): the longest blocks as VALU tasks (8 lanes per target, IQV sources per
// lane: the configuration of the VALU-only sweep, so the record stride 8 W matches); then
// groups of G consecutive blocks of v.order[nurg, nblocks).  A workgroup on a CU whose
// cu_busy count is positive (another workgroup there decodes a long block) stops pulling
// bulk work.
template <int W, int QL, int IQ, int IQV, int WPS>
__global__ void __launch_bounds__(64 * W, WPS) vit_hybrid_kernel(SweepArgs v, int nurg, int G,
                                                                 int* cu_busy, int exit_busy) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot[2];
  constexpr int XR = 8 * W;  // record stride: the VALU task's padded targets
  const int64_t nb = v.nblocks;
  const int key = cu_key();
  for (;;) {
    if (threadIdx.x == 0) qslot[0] = atomicAdd(v.queue, 1);
    lds_barrier();
    const int bi = uni(qslot[0]);
    lds_barrier();
    if (bi >= nurg) break;
    if (threadIdx.x == 0 && exit_busy >= 0) atomicAdd(cu_busy + key, 1);
    sweep_task<8, W, 1, IQV, MODE_VIT>(v, smem, bi);
    if (threadIdx.x == 0 && exit_busy >= 0) atomicSub(cu_busy + key, 1);
  }
  __shared__ int32_t grp[16];
  const int64_t ngroups = (nb - nurg + G - 1) / G;
  for (;;) {
    if (threadIdx.x == 0) {
      // wait (asleep) while a long block is decoded on this CU; exit mode: leave instead
      while (__hip_atomic_load(cu_busy + key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0) {
        if (exit_busy) break;
        __builtin_amdgcn_s_sleep(64);
      }
      const bool busy =
          exit_busy && __hip_atomic_load(cu_busy + key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0;
      qslot[1] = busy ? (int)ngroups : atomicAdd(v.queue + 1, 1);
    }
    lds_barrier();
    const int gi = uni(qslot[1]);
    if (gi < ngroups && threadIdx.x < G) {
      const int64_t k = nurg + (int64_t)gi * G + threadIdx.x;
      grp[threadIdx.x] = k < nb ? v.order[k] : -1;
    }
    lds_barrier();
    if (gi >= ngroups) break;
    vit_group_task<W, QL, IQ>(v, smem, grp, G, XR);
  }
}

}  // namespace

// Configurations (64 < n <= 72): 9 waves (the VALU-only sweep's), record stride 72;
// cfg 0: four lanes per target, groups of 2 blocks, two workgroups per CU;
// cfg 1: two lanes per target, groups of 4 blocks, one workgroup per CU
VitHybridGeometry vit_hybrid_geometry(int n) {
  VitHybridGeometry g{};
  g.cfg = -1;
  if (!getenv("ITR_VIT_HYBRID")) return g;
  if (n > 64 && n <= 72) {
    g.cfg = atoi(getenv("ITR_VIT_HYBRID")) == 2 ? 1 : 0;
    g.exit_busy = getenv("ITR_VIT_EXIT") ? atoi(getenv("ITR_VIT_EXIT")) : 0;
    if (getenv("ITR_VIT_NOCU")) g.exit_busy = -1;
    g.block = 64 * 9;
    g.xr = 8 * 9;
    using V = ValuSweep<8, 9, 1, 9, MODE_VIT>;
    if (g.cfg == 0) {
      g.G = (64 * 9) / (4 * n);
      g.lds = std::max(VLds<9, 4, 18>::bytes, V::lds_bytes);
      g.per_cu = 2;
    } else {
      g.G = (64 * 9) / (2 * n);
      g.lds = std::max(VLds<9, 2, 36>::bytes, V::lds_bytes);
      g.per_cu = 1;
    }
  }
  return g;
}

hipError_t launch_vit_hybrid(const VitHybridGeometry& g, int grid, const SweepArgs& v, int nurg,
                             int* cu_busy, hipStream_t st) {
  switch (g.cfg) {
    case 0:
      hipLaunchKernelGGL((vit_hybrid_kernel<9, 4, 18, 9, 5>), dim3(grid), dim3(g.block), g.lds,
                         st, v, nurg, g.G, cu_busy, g.exit_busy);
      break;
    case 1:
      hipLaunchKernelGGL((vit_hybrid_kernel<9, 2, 36, 9, 3>), dim3(grid), dim3(g.block), g.lds,
                         st, v, nurg, g.G, cu_busy, g.exit_busy);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#else  // product library: the VALU-only Viterbi sweep (hmm_sweeps.hip)
VitHybridGeometry vit_hybrid_geometry(int) {
  VitHybridGeometry g{};
  g.cfg = -1;
  return g;
}
hipError_t launch_vit_hybrid(const VitHybridGeometry&, int, const SweepArgs&, int, int*,
                             hipStream_t) {
  return hipErrorInvalidValue;
}
#endif

}  // namespace itr
