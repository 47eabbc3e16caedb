// vit_hybrid.hip — EXPERIMENT (built into the experiment library only, ITR_EXPERIMENT,
// enabled by ITR_VIT_HYBRID=1|2): the Viterbi sweep (optimizer.py:305-333) as one persistent
// launch with two kinds of tasks on MI355X (gfx950):
//
//  * the longest blocks, one per workgroup, on the latency-optimised VALU layout of
//    valu_sweep.h (configuration 9: 8 lanes per target, 9 waves);
//  * the bulk as groups of G = 2 GL blocks stepped in lock-step, each lane (target j, source
//    quarter q) running the max-plus chain of its 18 sources for GL blocks, so the slice of
//    log a in registers serves GL blocks and the DPP combine / per-column tail cost a third
//    of the VALU instructions per useful add/max of the 8-lane layout.
//
// Both produce exactly the outputs of the VALU sweep — omega checkpoint rows every 16
// columns, 16-bit stay-flag words, the last column's first argmax — with the reference's
// rounding: omega_t[j] = max(yd, yo), yd = (omega_j + log a_jj) + log e_j,
// yo = max_{i != j}(omega_i + log a_ij) + log e_j (IEEE rounding is monotone), so the
// traceback (hmm_sweeps.hip) is shared and paths are bit-identical (parity tests green).
//
// Measured (1x MI355X, (5,5) model, chr10, scripts/gpu_vith4.sh, profiles/r2c_*): NOT
// adopted.  The lane groups run at one 9-wave workgroup per CU (168 VGPRs) and every step
// waits on the per-block emission loads (two columns of prefetch per block; the VALU
// sweep stages 16-column emission tiles through LDS, which G blocks cannot afford):
// 12.3 ms (GL 4, urgent share 0.3) .. 23 ms (share 0.7) against 7.5 ms for the VALU-only
// sweep.  Earlier variants (one block per lane, 2 or 4 lanes per target, groups of 2-4
// blocks, with and without CU-exclusive long blocks): 7.4-21 ms.  The VALU-only sweep is
// issue-bound at ~75% of the CU's VALU issue rate (~621 instructions per column over 9
// waves); the lone longest block (18377 columns) takes 5.97 ms by itself.
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

// One bulk task: G = 2 GL blocks stepped in lock-step by a 9-wave workgroup.  Lane
// (set s, target j, source quarter q): s = g / (4n), j, q from g mod 4n; set s owns blocks
// grp[s GL .. s GL + GL) and every lane runs the max-plus chain of ITS 18 sources for each of
// its GL blocks — the slice of log a in registers serves GL blocks, two DPP stages combine
// the four quarters of a target, and the per-column tail runs once per (lane, block).
template <int GL>
struct VLaneGroup {
  static constexpr int QLG = 4, IQ = 18, XB = 72, G = 2 * GL, TE = 2, NCH = 3;
  static constexpr size_t lds = (size_t)3 * G * XB * 8;
};

template <int GL>
__device__ __forceinline__ void vit_lane_group_task(const SweepArgs& p, unsigned char* smem,
                                                    const int32_t* grp, int xr) {
  using V = VLaneGroup<GL>;
  constexpr int IQ = V::IQ, XB = V::XB, G = V::G, TE = V::TE, NCH = V::NCH;
  double* X = reinterpret_cast<double*>(smem);  // [2][G][XB]
  double* Y = X + 2 * G * XB;                   // [G][XB]
  const int n = p.n;
  const int g = threadIdx.x;
  const int LS = V::QLG * n;
  const int s0 = g / LS;
  const bool live = s0 < 2;
  const int s = live ? s0 : 0;
  // idle lanes (g >= 8 n) carry -inf into the padding slot n of set 0
  const int j = live ? (g - s0 * LS) / V::QLG : n;
  const int jl = min(j, n - 1);  // row index for loads
  const int q = g & 3;
  const bool pub = live && q == 0;

  int T[GL];
  int64_t c0[GL], tk0[GL];
  int Tmax = 0;
#pragma unroll
  for (int k = 0; k < GL; ++k) {
    const int blk = grp[s * GL + k];
    c0[k] = blk >= 0 ? p.off[blk] : 0;
    T[k] = blk >= 0 ? (int)(p.off[blk + 1] - c0[k]) : 0;
    tk0[k] = blk >= 0 ? p.tile_off[blk] : 0;
  }
  for (int r = 0; r < G; ++r) {
    const int b2 = grp[r];
    if (b2 >= 0) Tmax = max(Tmax, (int)(p.off[b2 + 1] - p.off[b2]));
  }
  Tmax = uni(Tmax);

  // this lane's 18 entries of column j of log a (diagonal kept out of the chain); sources
  // beyond n read the -inf padding
  double m[IQ];
#pragma unroll
  for (int k = 0; k < IQ; ++k) {
    const int i = q * IQ + k;
    m[k] = !live ? -INFINITY : i >= n ? 0.0 : i == j ? -INFINITY : p.mat[(int64_t)i * n + j];
  }
  const double ldiag = live ? p.mat[(int64_t)j * n + j] : -INFINITY;
  for (int i = g; i < 2 * G * XB; i += 64 * 9) X[i] = -INFINITY;
  lds_barrier();

  // symbols of block k, clamped into the block (blocks of a group differ in length; the
  // columns past a block's end are stepped but never stored)
  auto sym = [&](int k, int t) -> int {
    return T[k] > 0 ? min((int)p.obs[c0[k] + min(t, T[k] - 1)], 624) : 0;
  };
  const double* emit = p.emit + jl;
  double x[GL], xfin[GL], ck[GL], enxt[GL][TE], ecur[GL][TE];
  int snxt[GL][TE];
  uint32_t bits[GL];
#pragma unroll
  for (int k = 0; k < GL; ++k) {
    x[k] = (live && T[k] > 0) ? p.init[sym(k, 0) * n + jl] : -INFINITY;
    xfin[k] = x[k];
    X[(s * GL + k) * XB + j] = x[k];
#pragma unroll
    for (int v = 0; v < TE; ++v) {
      enxt[k][v] = emit[sym(k, v) * n];
      snxt[k][v] = sym(k, TE + v);
    }
  }
  wait_vmem_all();
  lds_barrier();
  for (int t0 = 0; t0 < Tmax; t0 += VIT_TILE) {
#pragma unroll
    for (int k = 0; k < GL; ++k) {
      bits[k] = 0;
      ck[k] = x[k];  // column t0's omega row (t0 = 0: the initial row)
    }
#pragma unroll
    for (int sub = 0; sub < VIT_TILE; ++sub) {
      if (sub % TE == 0) {
#pragma unroll
        for (int k = 0; k < GL; ++k)
#pragma unroll
          for (int v = 0; v < TE; ++v) {
            ecur[k][v] = enxt[k][v];
            enxt[k][v] = emit[snxt[k][v] * n];
            snxt[k][v] = sym(k, t0 + sub + 2 * TE + v);
          }
      }
      const int t = t0 + sub;
      if (t >= 1 && t < Tmax) {
        const int buf = (t - 1) & 1;
#pragma unroll
        for (int k = 0; k < GL; ++k) {
          const double* xs = X + (buf * G + s * GL + k) * XB + q * IQ;
          double bc[NCH];
#pragma unroll
          for (int c = 0; c < NCH; ++c) bc[c] = xs[c] + m[c];
#pragma unroll
          for (int e = NCH; e < IQ; ++e) {
            if (e % 8 == 0) __builtin_amdgcn_sched_barrier(0);
            bc[e % NCH] = fmax(bc[e % NCH], xs[e] + m[e]);
          }
          double zo = fmax(fmax(bc[0], bc[1]), bc[2]);
          zo = fmax(zo, dpp_f64<0xB1>(zo));  // quad_perm [1,0,3,2]
          zo = fmax(zo, dpp_f64<0x4E>(zo));  // quad_perm [2,3,0,1]
          const double ec = ecur[k][sub % TE];
          const double yd = (x[k] + ldiag) + ec;
          const double yo = zo + ec;
          bits[k] |= (uint32_t)(yd > yo) << sub;
          x[k] = fmax(yd, yo);
          if (sub == 0) ck[k] = x[k];
          xfin[k] = t == T[k] - 1 ? x[k] : xfin[k];
          // the four lanes of a target hold the same value: all write it
          X[((buf ^ 1) * G + s * GL + k) * XB + j] = x[k];
        }
        lds_barrier();
      }
    }
    // the tile's checkpoint row and stay-flag word of every block that reaches it (flag
    // bits past a block's last column are never read by the traceback)
#pragma unroll
    for (int k = 0; k < GL; ++k)
      if (pub && t0 < T[k]) {
        const int64_t rec = (tk0[k] + t0 / VIT_TILE) * xr;
        p.alpha[rec + j] = ck[k];
        p.stay[rec + j] = (uint16_t)bits[k];
      }
  }
  // last state of every block = first argmax of its last omega row (optimizer.py:346)
#pragma unroll
  for (int k = 0; k < GL; ++k)
    if (pub) Y[(s * GL + k) * XB + j] = xfin[k];
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

// v.order[0, nurg): the longest blocks as VALU tasks (the VALU-only sweep's configuration 9:
// 8 lanes per target, 9 waves, record stride 72); then groups of G consecutive blocks of
// v.order[nurg, nblocks).
template <int GL, int WPS>
__global__ void __launch_bounds__(576, WPS) vit_hybrid_kernel(SweepArgs v, int nurg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot[2];
  constexpr int G = VLaneGroup<GL>::G;
  const int64_t nb = v.nblocks;
  for (;;) {
    if (threadIdx.x == 0) qslot[0] = atomicAdd(v.queue, 1);
    lds_barrier();
    const int bi = uni(qslot[0]);
    lds_barrier();
    if (bi >= nurg) break;
    sweep_task<8, 9, 1, 9, MODE_VIT>(v, smem, bi);
  }
  __shared__ int32_t grp[G];
  const int64_t ngroups = (nb - nurg + G - 1) / G;
  for (;;) {
    if (threadIdx.x == 0) qslot[1] = atomicAdd(v.queue + 1, 1);
    lds_barrier();
    const int gi = uni(qslot[1]);
    if (gi < ngroups && threadIdx.x < G) {
      const int64_t k = nurg + (int64_t)gi * G + threadIdx.x;
      grp[threadIdx.x] = k < nb ? v.order[k] : -1;
    }
    lds_barrier();
    if (gi >= ngroups) break;
    vit_lane_group_task<GL>(v, smem, grp, 72);
  }
}

}  // namespace

// Configurations (64 < n <= 72): 9 waves, record stride 72 (the VALU-only sweep's);
// cfg 0: GL = 4 (groups of 8 blocks), cfg 1: GL = 2 (groups of 4)
VitHybridGeometry vit_hybrid_geometry(int n) {
  VitHybridGeometry g{};
  g.cfg = -1;
  if (!getenv("ITR_VIT_HYBRID")) return g;
  if (n > 64 && n <= 72) {
    g.cfg = atoi(getenv("ITR_VIT_HYBRID")) == 2 ? 1 : 0;
    g.block = 576;
    g.xr = 72;
    using V = ValuSweep<8, 9, 1, 9, MODE_VIT>;
    g.G = g.cfg == 0 ? VLaneGroup<4>::G : VLaneGroup<2>::G;
    g.lds = std::max(g.cfg == 0 ? VLaneGroup<4>::lds : VLaneGroup<2>::lds, V::lds_bytes);
    g.per_cu = getenv("ITR_VIT_PER_CU") ? atoi(getenv("ITR_VIT_PER_CU")) : 1;
  }
  return g;
}

hipError_t launch_vit_hybrid(const VitHybridGeometry& g, int grid, const SweepArgs& v, int nurg,
                             int*, hipStream_t st) {
  switch (g.cfg) {
    case 0:
      hipLaunchKernelGGL((vit_hybrid_kernel<4, 3>), dim3(grid), dim3(g.block), g.lds, st, v,
                         nurg);
      break;
    case 1:
      hipLaunchKernelGGL((vit_hybrid_kernel<2, 5>), dim3(grid), dim3(g.block), g.lds, st, v,
                         nurg);
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
