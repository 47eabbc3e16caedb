// lane_groups.h — the Viterbi sweep of one block per workgroup with small lane groups per
// target state (G = 3 or 5 lanes inside a 16-lane row): the low-latency layout for the
// longest blocks.  Device code only; included by hmm_sweeps.hip.
//
// Why: a block's Viterbi step is a strictly sequential chain, so its time per
// column is set by the busiest SIMD's issue plus the step's latency.  The 9-wave layout (8
// lanes per target, 9 sources each, a 3-stage DPP butterfly) puts three waves on SIMD 0 —
// ~105 VALU instructions per column there against ~70 on the other SIMDs, and the barrier
// waits for SIMD 0.  Here lane l of wave w, row r = l >> 4, k = l & 15 belongs to group
// g = k / G (g < 16 / G; a row's leftover lanes hold no target) and source chunk q = k % G:
//   target  j = w * TPW + r * GPR + g      (GPR = 16 / G groups per row, TPW = 4 GPR per wave)
//   sources i = q * S .. q * S + S - 1     (G * S >= N)
// so W = ceil(N / TPW) waves cover the targets: at N = 70, G = 3, S = 24: four waves, ONE per
// SIMD (20 targets each), ~60 VALU instructions per column per wave.  The G partial maxima of
// a target meet in its last lane (q = G - 1) through row_shr DPP moves (two stages for G = 3:
// shr 1 and shr 2 of the same register, independent), which owns the target: it finalises
// omega, the stay flag and the checkpoint and publishes omega for the next column.  Other lanes'
// results are never used.
//
// Arithmetic, outputs and the traceback they feed are the 9-wave layout's (valu_sweep.h): the
// chain takes max over i != j of fl(omega_i + log a_ij) (the diagonal entry is -inf in the
// register slice), yd = fl(fl(omega_j + log a_jj) + log e_j), yo = fl(max + log e_j),
// omega = max(yd, yo), stay flag = yd > yo — bit-identical to optimizer.py:325-332 for any
// order of the max.  Per 16-column tile: the omega row of its first column (checkpoint) and one
// 16-bit flag word per state, at record stride p.xrec.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {

static constexpr int DPP_SHR1 = 0x111;  // row_shr:1 (lane x reads lane x - 1 of its row)
static constexpr int DPP_SHR2 = 0x112;
static constexpr int DPP_SHR3 = 0x113;
static constexpr int DPP_SHR4 = 0x114;

template <int G, int W, int S>
struct VitGroupLayout {
  static constexpr int GPR = 16 / G;       // groups per 16-lane row
  static constexpr int TPW = 4 * GPR;      // targets per wave
  static constexpr int XR = W * TPW;       // target slots (staged emission row width)
  static constexpr int XS = G * S;         // published vector length (padded sources)
  static constexpr int TE = VIT_TILE;      // columns per staged tile
  static constexpr int TB = 64 * W;
  static_assert(S % 2 == 0, "16-byte LDS reads of the source chunks");
  static constexpr size_t lds_bytes = (size_t)2 * (XS + 64) * 8 + 5 * 64 * 8 +
                                      (size_t)2 * TE * XR * 8 + 32 * 4 + (size_t)2 * TB * 2;
};

// max over the G lanes of the group ending at this lane (exact in lane q = G - 1 only)
template <int G>
__device__ __forceinline__ double group_max_last(double v) {
  static_assert(G == 3 || G == 5, "groups of 3 or 5 lanes");
  const double a = dpp_f64<DPP_SHR1>(v), b = dpp_f64<DPP_SHR2>(v);
  if constexpr (G == 3) {
    return fmax(fmax(v, a), b);
  } else {
    const double c = dpp_f64<DPP_SHR3>(v), d = dpp_f64<DPP_SHR4>(v);
    return fmax(fmax(fmax(v, a), b), fmax(c, d));
  }
}

template <int G, int W, int S>
__device__ __forceinline__ void vit_group_task(const SweepArgs& p, unsigned char* smem, int bi) {
  using Lay = VitGroupLayout<G, W, S>;
  constexpr int GPR = Lay::GPR, TPW = Lay::TPW, XR = Lay::XR, XS = Lay::XS, TE = Lay::TE;
  constexpr int TB = Lay::TB;
  constexpr int NCH = S >= 16 ? 4 : (S >= 6 ? 3 : 2);  // independent max chains per lane
  constexpr int C = 16;                                   // sources per LDS read piece
  constexpr int NPC = (S + C - 1) / C;
  const int n = p.n;
  const int tid = threadIdx.x;
  const int w = uni(tid >> 6);
  const int l = tid & 63;
  const int k16 = l & 15;
  const int gq = k16 / G;
  const bool lane_ok = gq < GPR;  // (the row's leftover lanes: no target)
  const int g = lane_ok ? gq : 0;
  const int q = lane_ok ? k16 - gq * G : 0;
  const int j = w * TPW + (l >> 4) * GPR + g;
  const bool jv = lane_ok && j < n;
  const bool owner = jv && q == G - 1;
  const int64_t xrec = p.xrec;

  double* X = reinterpret_cast<double*>(smem);  // [2][XS+64] published omega + write sinks
  double* RED = X + 2 * (XS + 64);              // [5][64]
  double* EST = RED + 5 * 64;                   // [2][TE][XR] staged log-emission rows
  int* SBLK = reinterpret_cast<int*>(EST + 2 * TE * XR);
  int* REDI = SBLK + 4;                                      // [16]
  uint16_t* OBS = reinterpret_cast<uint16_t*>(SBLK + 32);    // [2][TB]
  const int jx = owner ? j : XS + l;  // publish slot (non-owners: a sink nobody reads)

  // sources >= n keep -inf (never a maximum)
  for (int i = tid; i < 2 * (XS + 64); i += TB) X[i] = -INFINITY;
  lds_barrier();

  RowStage<W, XR, TE> est;
  DIAG_DECL
  {
    const int blk = uni(p.order[bi]);
    const int64_t c0 = p.off[blk];
    const int T = uni((int)(p.off[blk + 1] - c0));
    if (T > 0) {
      const bool urgent = T >= p.prio_len;
      if (urgent) __builtin_amdgcn_s_setprio(2);
      // this lane's slice of log a: rows i = q S + s of column j (-inf at i == j, outside the
      // model and on lanes without a target)
      double m[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int i = q * S + s;
        m[s] = (jv && i < n && i != j) ? p.mat[(int64_t)i * n + j] : -INFINITY;
      }
      const double ldiag = jv ? p.mat[(int64_t)j * n + j] : 0.0;
      ObsTiles ot{OBS, p.obs + c0, T, +1, TB, 0};
      ot.start(tid);
      lds_barrier();
      auto sym_row = [&](int s) -> int64_t { return s < T ? (int64_t)ot.get(s) : -1; };
      est.issue(p.emit, n, n, tid, 0, sym_row);
      est.commit(EST, tid);
      est.issue(p.emit, n, n, tid, TE, sym_row);
      auto staged = [&](int s, int jj) {
        return EST[((s / TE) & 1) * TE * XR + (s & (TE - 1)) * XR + jj];
      };
      lds_barrier();
      const int64_t tk0 = p.tile_off[blk];
      const int o0 = ot.get(0);
      double x = jv ? p.init[o0 * n + j] : -INFINITY;
      if (owner) p.alpha[tk0 * xrec + j] = x;
      wait_vmem_all();
      STAMP(-1);
      for (int t0 = 0; t0 < T; t0 += TE) {
        const int64_t rec = (tk0 + t0 / TE) * xrec;
        uint32_t bits = 0;
#pragma unroll
        for (int sub = 0; sub < TE; ++sub) {
          const int t = t0 + sub;
          if (t >= 1 && t < T) {
            DIAG_STEP();
            const int buf = sub & 1;  // t0 is even
            double* Xb = X + buf * (XS + 64);
            Xb[jx] = x;
            double ec = 0.0;
            if (sub != 0) ec = staged(t, j);
            if (sub == 0) {
              ot.advance(t, tid);
              if (t >= TE) est.commit(EST + ((t / TE) & 1) * TE * XR, tid);
            }
            STAMP(0);
            lds_barrier();
            STAMP(1);
            if (sub == 0) {
              if (t >= TE) est.issue(p.emit, n, n, tid, t + TE, sym_row);
              ec = staged(t, j);
            }
            if (w * TPW < n) {  // (waves whose targets are all padding skip: uniform)
              // The source chunk in pieces of C values, two pieces in flight: piece c + 2 is
              // requested when piece c has been consumed, so only the first piece's LDS latency
              // is exposed and at most three pieces hold registers (left to itself the
              // scheduler interleaves the reads two at a time and waits on each pair)
              const double* xs = Xb + q * S;
              double xv[S];
#pragma unroll
              for (int s = 0; s < S && s < 2 * C; ++s) xv[s] = xs[s];
              __builtin_amdgcn_sched_barrier(0);
              double bc[NCH];
#pragma unroll
              for (int c = 0; c < NCH; ++c) bc[c] = -INFINITY;
#pragma unroll
              for (int pc = 0; pc < NPC; ++pc) {
#pragma unroll
                for (int s = pc * C; s < S && s < (pc + 1) * C; ++s)
                  bc[s % NCH] = fmax(bc[s % NCH], xv[s] + m[s]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int s = (pc + 2) * C; s < S && s < (pc + 3) * C; ++s) xv[s] = xs[s];
                __builtin_amdgcn_sched_barrier(0);
              }
              double zo = bc[0];
#pragma unroll
              for (int c = 1; c < NCH; ++c) zo = fmax(zo, bc[c]);
              STAMP(2);
              zo = group_max_last<G>(zo);  // max over i != j (exact in the owner lane)
              STAMP(3);
              const double yd = (x + ldiag) + ec;
              const double yo = zo + ec;
              bits |= (uint32_t)(yd > yo) << sub;
              x = fmax(yd, yo);
            }
            STAMP(4);
            if (sub == 0 && owner) p.alpha[rec + j] = x;  // the tile's checkpoint (t = t0)
            STAMP(5);
          }
        }
        if (owner) p.stay[rec + j] = (uint16_t)bits;
      }
      // last state = first argmax of omega_{T-1}  (optimizer.py:346)
      double bv = owner ? x : -INFINITY;
      int bj = owner ? j : 0x7fffffff;
      wave_first_max(bv, bj);
      if (l == 0) {
        RED[256 + w] = bv;
        REDI[w] = bj;
      }
      lds_barrier();
      if (tid == 0) {
        double b = RED[256];
        int a = REDI[0];
#pragma unroll
        for (int v = 1; v < W; ++v) {
          const double c = RED[256 + v];
          if (c > b) {
            b = c;
            a = REDI[v];
          }
        }
        p.last_state[blk] = (uint8_t)a;
      }
      if (urgent) __builtin_amdgcn_s_setprio(0);
    }
    lds_barrier();
  }
  DIAG_FLUSH();
}

// sum over the G lanes of the group ending at this lane (exact in lane q = G - 1 only)
template <int G>
__device__ __forceinline__ double group_sum_last(double v) {
  static_assert(G == 3 || G == 5, "groups of 3 or 5 lanes");
  const double a = dpp_f64<DPP_SHR1>(v), b = dpp_f64<DPP_SHR2>(v);
  if constexpr (G == 3) {
    return (v + a) + b;
  } else {
    const double c = dpp_f64<DPP_SHR3>(v), d = dpp_f64<DPP_SHR4>(v);
    return ((v + a) + b) + (c + d);
  }
}
// maximum over the 16 lanes of a row, then over the wave's four rows: wave-uniform
__device__ __forceinline__ double wave_max_rows(double v) {
  v = fmax(v, dpp_f64<DPP_Q1>(v));
  v = fmax(v, dpp_f64<DPP_Q2>(v));
  v = fmax(v, dpp_f64<DPP_HM>(v));
  v = fmax(v, dpp_f64<DPP_R8>(v));
  return rows4_max(v);
}

// One forward log-likelihood task (MODE_FWD_LL, tasks {block, split, slot} as the VALU
// sweep's, valu_sweep.h) on the lane-group layout: the longest blocks' halves of the split
// forward (meet in the middle) at the lowest step latency.  x_t = (x_{t-1} @ a) * e_t in the
// probability domain with an exact power-of-two rescale every 8 columns (the exponents summed
// in K); a backward half (split < 0) runs the same step on a^T from its block's end, starting
// from e_{T-1} and ending with a row of ones.  Outputs as the VALU sweep's: the split halves'
// vectors (row stride XR, = the hybrid configuration's 16 x its waves) and exponents, or
// log P = log(sum_j x_j) + K ln 2 (optimizer.py:145-162).  (A forward-store form of this task,
// the posterior's longest blocks, measured slower in both placements tried: DESIGN.md §0.)
template <int G, int W, int S>
__device__ __forceinline__ void fwd_group_task(const SweepArgs& p, unsigned char* smem, int bi) {
  using Lay = VitGroupLayout<G, W, S>;
  constexpr int GPR = Lay::GPR, TPW = Lay::TPW, XR = Lay::XR, XS = Lay::XS, TE = Lay::TE;
  constexpr int TB = Lay::TB;
  constexpr int NCH = S >= 16 ? 4 : (S >= 6 ? 3 : 2);  // independent FMA chains per lane
  constexpr int C = 16;
  constexpr int NPC = (S + C - 1) / C;
  const int n = p.n;
  const int tid = threadIdx.x;
  const int w = uni(tid >> 6);
  const int l = tid & 63;
  const int k16 = l & 15;
  const int gq = k16 / G;
  const bool lane_ok = gq < GPR;
  const int g = lane_ok ? gq : 0;
  const int q = lane_ok ? k16 - gq * G : 0;
  const int j = w * TPW + (l >> 4) * GPR + g;
  const bool jv = lane_ok && j < n;
  const bool owner = jv && q == G - 1;

  double* X = reinterpret_cast<double*>(smem);  // [2][XS+64] published x + write sinks
  double* RED = X + 2 * (XS + 64);              // [5][64] rescale maxima, loglik partials
  double* EST = RED + 5 * 64;                   // [2][TE][XR] staged emission rows
  int* SBLK = reinterpret_cast<int*>(EST + 2 * TE * XR);
  uint16_t* OBS = reinterpret_cast<uint16_t*>(SBLK + 32);  // [2][TB]
  const int jx = owner ? j : XS + l;

  // sources >= n keep 0 (contribute nothing)
  for (int i = tid; i < 2 * (XS + 64); i += TB) X[i] = 0.0;
  lds_barrier();

  RowStage<W, XR, TE> est;
  {
    const int32_t* td = p.tasks + 3 * bi;
    const int blk = uni(td[0]);
    const int split = uni(td[1]);
    const int slot = uni(td[2]);
    const int64_t c0 = p.off[blk];
    const int Tb = uni((int)(p.off[blk + 1] - c0));
    const int T = split > 0 ? split : (split < 0 ? Tb + split + 1 : Tb);
    if (T <= 0) {  // empty block: log-likelihood of nothing is 0
      if (tid == 0) p.loglik[blk] = 0.0;
    } else {
      const bool urgent = T >= p.prio_len;
      if (urgent) __builtin_amdgcn_s_setprio(2);
      const double* mp = split < 0 ? p.matT : p.mat;
      double m[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const int i = q * S + s;
        m[s] = (jv && i < n) ? mp[(int64_t)i * n + j] : 0.0;
      }
      ObsTiles ot{OBS, p.obs + c0, Tb, split < 0 ? -1 : +1, TB, 0};
      ot.start(tid);
      lds_barrier();
      auto sym_row = [&](int s) -> int64_t {
        if (split < 0) return s < T - 1 ? (int64_t)ot.get(s) : (s == T - 1 ? -2 : -1);
        return s < T ? (int64_t)ot.get(s) : -1;
      };
      est.issue(p.emit, n, n, tid, 0, sym_row);
      est.commit(EST, tid);
      est.issue(p.emit, n, n, tid, TE, sym_row);
      auto staged = [&](int s, int jj) {
        return EST[((s / TE) & 1) * TE * XR + (s & (TE - 1)) * XR + jj];
      };
      lds_barrier();
      const int o0 = ot.get(0);
      const double* x0tab = split < 0 ? p.emit : p.init;
      double x = jv ? x0tab[o0 * n + j] : 0.0;
      int K = 0;  // sum of the power-of-two exponents divided out so far
      wait_vmem_all();
      for (int t0 = 0; t0 < T; t0 += TE) {
#pragma unroll
        for (int sub = 0; sub < TE; ++sub) {
          const int t = t0 + sub;
          if (t >= 1 && t < T) {
            const int buf = sub & 1;  // t0 is even
            double* Xb = X + buf * (XS + 64);
            Xb[jx] = x;
            const bool rescale = (sub & 7) == 1;
            if (rescale) {  // the wave's maximum of x_{t-1} (owners' values only)
              const double mx = wave_max_rows(owner ? x : 0.0);
              if (l == 0) RED[128 + buf * 64 + w] = mx;
            }
            double ec = 0.0;
            if (sub != 0) ec = staged(t, j);
            if (sub == 0) {
              ot.advance(t, tid);
              if (t >= TE) est.commit(EST + ((t / TE) & 1) * TE * XR, tid);
            }
            lds_barrier();
            if (sub == 0) {
              if (t >= TE) est.issue(p.emit, n, n, tid, t + TE, sym_row);
              ec = staged(t, j);
            }
            if (w * TPW < n) {
              const double* xs = Xb + q * S;
              double xv[S];
#pragma unroll
              for (int s = 0; s < S && s < 2 * C; ++s) xv[s] = xs[s];
              __builtin_amdgcn_sched_barrier(0);
              double acc[NCH];
#pragma unroll
              for (int c = 0; c < NCH; ++c) acc[c] = 0.0;
#pragma unroll
              for (int pc = 0; pc < NPC; ++pc) {
#pragma unroll
                for (int s = pc * C; s < S && s < (pc + 1) * C; ++s)
                  acc[s % NCH] = fma(xv[s], m[s], acc[s % NCH]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int s = (pc + 2) * C; s < S && s < (pc + 3) * C; ++s) xv[s] = xs[s];
                __builtin_amdgcn_sched_barrier(0);
              }
              if (rescale) {  // fold 2^-e into the emission factor (off the FMA chain)
                const double M = tree_max<W>(RED + 128 + buf * 64);
                const bool ok = M > 0.0 && M < INFINITY;
                const int e = ok ? ilogb(M) : 0;
                K += e;
                ec *= ldexp(1.0, -e);
              }
              double sum = acc[0];
#pragma unroll
              for (int c = 1; c < NCH; ++c) sum += acc[c];
              x = group_sum_last<G>(sum) * ec;
            }
          }
        }
      }
      if (split != 0) {  // half of a split block: the scaled vector and its exponent
        const int side = split < 0;
        if (owner) p.svec[((int64_t)slot * 2 + side) * XR + j] = x;
        if (tid == 0) p.sK[slot * 2 + side] = K;
      } else {  // log P = log(sum_j x_j) + K ln 2
        const double part = wave_sum(owner ? x : 0.0);
        if (l == 0) RED[256 + w] = part;
        lds_barrier();
        if (tid == 0) {
          double tot = 0.0;
#pragma unroll
          for (int v = 0; v < W; ++v) tot += RED[256 + v];
          p.loglik[blk] = log(tot) + (double)K * LN2;
        }
      }
      if (urgent) __builtin_amdgcn_s_setprio(0);
    }
    lds_barrier();
  }
}

// the persistent launch: every workgroup pulls blocks longest first
template <int G, int W, int S>
__device__ __forceinline__ void vit_group_device(const SweepArgs& p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot;
  for (;;) {
    if (threadIdx.x == 0) qslot = atomicAdd(p.queue, 1);
    lds_barrier();
    const int bi = uni(qslot);
    lds_barrier();
    if (bi >= p.nblocks) break;
    vit_group_task<G, W, S>(p, smem, bi);
  }
}
template <int G, int W, int S>
__device__ __forceinline__ void fwd_group_device(const SweepArgs& p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot;
  for (;;) {
    if (threadIdx.x == 0) qslot = atomicAdd(p.queue, 1);
    lds_barrier();
    const int bi = uni(qslot);
    lds_barrier();
    if (bi >= p.nblocks) break;
    fwd_group_task<G, W, S>(p, smem, bi);
  }
}

}  // namespace itr
