// wave_vit.hip — the Viterbi sweep (optimizer.py:305-333) with one MAF block per wavefront,
// for MI355X (gfx950).
//
// The 8-lanes-per-target layout of valu_sweep.h spends ~315 VALU instructions per column on
// the (5,5) model (N = 70): every lane ends with the full maximum of its target after a
// three-stage DPP all-reduce and runs the per-column tail redundantly, against 153 useful
// adds/maxes.  Here one wavefront decodes a whole block on its own (no workgroup barrier):
//
//   lane l = 8 g + q holds sources i in [IQ q, IQ q + IQ) x targets j in [IQ g, IQ g + IQ)
//   of log a in VGPRs (loaded once per wave), forms the IQ partial maxima
//   z_j = max_i (omega_i + log a_ij) over its sources (IQ^2 adds, IQ^2 - IQ maxes), writes
//   them to the wave's partial table P[j][q] in LDS, and then finalises ONE target j = l
//   (plus, for 8 IQ > 64, target 64 + (l & 7)) from the 8 partials of that target.
//
// ~181 VALU instructions per column at IQ = 9 (N <= 72).  All LDS traffic stays inside the
// wave (a wave's LDS instructions execute in order), so a step needs no barrier.  The
// emission rows are staged 8 columns at a time into the wave's LDS ring by direct-to-LDS
// loads from a log-emission table padded to 8 IQ columns.
//
// Two such waves share a SIMD (256 VGPRs each), so a block steps at ~640 ns per column
// (~1.7x the throughput of the 8-lane layout on short blocks, but ~2x its lone-step latency):
// itr_viterbi gives the longest blocks to the 9-wave VALU layout on a reserved set of CUs and
// this kernel the rest (capi.cpp); blocks at least p.prio_len long run at
// raised wave priority.
//
// Outputs are those of the VALU sweep — the omega row of every 16-column tile's first column,
// 16-bit stay-flag words, the last column's first argmax — from the identical arithmetic:
// omega_t[j] = max(yd, yo), yd = (omega_j + log a_jj) + log e_j,
// yo = max_{i != j}(omega_i + log a_ij) + log e_j (the max is exact and order-free), so the
// traceback (hmm_sweeps.hip) is shared and paths are bit-identical.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {
namespace {

template <int IQ>
struct WaveVit {
  static constexpr int XRW = 8 * IQ;                  // targets = sources of the layout
  static constexpr int NB = XRW > 64 ? XRW - 64 : 0;  // second targets: 64 + (l & 7)
  static_assert(NB <= 8, "at most 8 second targets");
  static constexpr int IQS = IQ + (IQ & 1);           // 16-byte aligned source chunks
  static constexpr int XN = 8 * IQS;                  // published vector slots
  static constexpr int PS = 10;  // partial row stride: 8 chunks + 2 (conflict-free b128 reads)
  static constexpr int HT = 8;   // columns per staged emission half-tile
  // a half-tile of emission rows [HT][XRW] arrives by NI direct-to-LDS loads of 16 bytes per
  // lane (1 KiB each); the buffer is rounded up to whole loads
  static constexpr int NI = (HT * XRW + 127) / 128, EB = 128 * NI;
  static_assert(XRW % 2 == 0, "16-byte pieces must not cross a row");
  // per-wave LDS (doubles): published vector + 64 sink slots, partials, emission ring [2],
  // symbol ring [2][64] (uint16)
  static constexpr int LX = XN + 64, LP = XRW * PS, LE = 2 * EB, LS = 2 * 64 / 4;
  static constexpr int WL = LX + LP + LE + LS;
};

constexpr int kWaves = 4;  // independent wavefronts per workgroup

template <int IQ>
__device__ __forceinline__ void wave_vit_blocks(const VitArgs& p, double* wl) {
  using C = WaveVit<IQ>;
  constexpr int XRW = C::XRW, NB = C::NB, IQS = C::IQS, XN = C::XN, PS = C::PS, HT = C::HT,
                NI = C::NI, EB = C::EB;
  const int l = threadIdx.x & 63, q = l & 7, g = l >> 3;
  const int n = p.n;
  const int64_t xr = p.xr;
  double* X = wl;
  double* P = X + C::LX;
  double* EST = P + C::LP;
  uint16_t* SYM = reinterpret_cast<uint16_t*>(EST + C::LE);

  // log a slice: rows IQ q + k, columns IQ g + r; the diagonal stays out of the max chain
  double m[IQ][IQ];
#pragma unroll
  for (int k = 0; k < IQ; ++k)
#pragma unroll
    for (int r = 0; r < IQ; ++r) {
      const int i = IQ * q + k, j = IQ * g + r;
      m[k][r] = (i < n && j < n && i != j) ? p.la[(int64_t)i * n + j] : -INFINITY;
    }
  // finalised targets: A = l (inside the layout), B = 64 + (l & 7) (NB > 0: formed by all 8
  // lanes of a group, stored by lane l < NB)
  const int A = l, B = 64 + (l & 7);
  const bool inA = A < XRW && A < n;
  const bool inB = NB > 0 && B < n;
  const bool ownB = inB && l < NB;
  const double ldA = inA ? p.la[(int64_t)A * n + A] : -INFINITY;
  const double ldB = inB ? p.la[(int64_t)B * n + B] : -INFINITY;
  const int sA = A < XRW ? (A / IQ) * IQS + A % IQ : XN + l;  // slot in X (or the sink)
  const int sB = (NB > 0 && l < NB) ? (B / IQ) * IQS + B % IQ : XN + l;
  const int rA = A < XRW ? A : 0, rB = NB > 0 ? B : 0;  // partial / emission rows
  for (int i = l; i < C::LX; i += 64) X[i] = -INFINITY;

  for (;;) {
    // every lane takes part in the atomic (lane 0 adds 1): with a lane-divergent
    // `if (l == 0)` at the loop head hipcc (ROCm 7.2) built a lane-divergent inner loop in
    // which lanes 1..63 re-read a stale block index and the wave never finished
    const int bi = uni(atomicAdd(p.queue, l == 0 ? 1 : 0));
    if (bi >= p.nblocks) break;
    const int blk = uni(p.order[bi]);
    const int64_t c0 = p.off[blk];
    const int T = uni((int)(p.off[blk + 1] - c0));
    if (T > 0) {  // (no `continue` in this loop, same reason)
      const bool urgent = T >= p.prio_len;
      if (urgent) __builtin_amdgcn_s_setprio(3);
      const uint16_t* ob = p.obs + c0;
      auto symg = [&](int s) -> int { return min((int)ob[min(s, T - 1)], 624); };
      // symbols: chunks of 64 columns, two resident in SYM, the next one in flight
      SYM[l] = (uint16_t)symg(l);
      SYM[64 + l] = (uint16_t)symg(64 + l);
      int sin = symg(128 + l);
      auto sym = [&](int s) -> int { return SYM[((s >> 6) & 1) * 64 + (s & 63)]; };
      // emission rows of half-tile h -> EST[h & 1] (row-major [HT][XRW]) by direct-to-LDS
      // loads; the compiler does not track them, so every read of a half-tile follows an
      // explicit vmcnt(0) (stage_wait) a half-tile after its loads were issued
      auto stage_issue = [&](int h) {
        double* d = EST + (h & 1) * EB;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int e = 128 * i + 2 * l;
          const double* src = p.lew;
          if (e < HT * XRW) src += (int64_t)sym(h * HT + e / XRW) * XRW + e % XRW;
          __builtin_amdgcn_global_load_lds(
              src, (__attribute__((address_space(3))) void*)(d + 128 * i), 16, 0, 0);
        }
      };
      auto stage_wait = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
      const int o0 = sym(0);
      double xA = inA ? p.lpie[o0 * n + A] : -INFINITY;
      double xB = inB ? p.lpie[o0 * n + B] : -INFINITY;
      X[sA] = xA;
      X[sB] = xB;
      const int64_t tk0 = p.tile_off[blk];
      if (inA) p.ckpt[tk0 * xr + A] = xA;
      if (ownB) p.ckpt[tk0 * xr + B] = xB;
      stage_issue(0);
      stage_wait();
      stage_issue(1);
      for (int t0 = 0; t0 < T; t0 += VIT_TILE) {
        const int64_t rec = (tk0 + t0 / VIT_TILE) * xr;
        uint32_t bA = 0, bB = 0;
#pragma unroll
        for (int sub = 0; sub < VIT_TILE; ++sub) {
          const int t = t0 + sub;
          if (t >= 1 && t < T) {
            if ((sub & (HT - 1)) == 0) {  // half-tile boundary (t >= 8)
              stage_wait();
              if ((t & 63) == 0) {  // next symbol chunk in, the one after requested
                SYM[(((t >> 6) + 1) & 1) * 64 + l] = (uint16_t)sin;
                sin = symg(t + 128 + l);
              }
              stage_issue(t / HT + 1);
            }
            const double* es = EST + ((t / HT) & 1) * EB + (t & (HT - 1)) * XRW;
            const double ecA = es[rA];
            const double ecB = es[rB];
            double xs[IQ];
#pragma unroll
            for (int k = 0; k < IQ; ++k) xs[k] = X[q * IQS + k];
            double z[IQ];
#pragma unroll
            for (int r = 0; r < IQ; ++r) z[r] = xs[0] + m[0][r];
#pragma unroll
            for (int k = 1; k < IQ; ++k)
#pragma unroll
              for (int r = 0; r < IQ; ++r) z[r] = fmax(z[r], xs[k] + m[k][r]);
#pragma unroll
            for (int r = 0; r < IQ; ++r) P[(IQ * g + r) * PS + q] = z[r];
            wave_lds_sync();  // partials of the other lanes visible
            // this lane's target(s): max over the 8 source chunks (exact, order-free)
            const double* pa = P + rA * PS;
            const double zoA = fmax(fmax(fmax(pa[0], pa[1]), fmax(pa[2], pa[3])),
                                    fmax(fmax(pa[4], pa[5]), fmax(pa[6], pa[7])));
            const double ydA = (xA + ldA) + ecA;
            const double yoA = zoA + ecA;
            bA |= (uint32_t)(ydA > yoA) << sub;
            xA = fmax(ydA, yoA);
            if constexpr (NB > 0) {
              const double* pb = P + rB * PS;
              const double zoB = fmax(fmax(fmax(pb[0], pb[1]), fmax(pb[2], pb[3])),
                                      fmax(fmax(pb[4], pb[5]), fmax(pb[6], pb[7])));
              const double ydB = (xB + ldB) + ecB;
              const double yoB = zoB + ecB;
              bB |= (uint32_t)(ydB > yoB) << sub;
              xB = fmax(ydB, yoB);
            }
            X[sA] = xA;
            X[sB] = xB;
            wave_lds_sync();  // omega_t visible to every lane for the next step
            if (sub == 0) {  // the tile's checkpoint row (t = t0 >= 16)
              if (inA) p.ckpt[rec + A] = xA;
              if (ownB) p.ckpt[rec + B] = xB;
            }
          }
        }
        if (inA) p.stay[rec + A] = (uint16_t)bA;  // the tile's flag words
        if (ownB) p.stay[rec + B] = (uint16_t)bB;
      }
      // last state = first argmax of omega_{T-1}  (optimizer.py:346)
      double bv = inA ? xA : -INFINITY;
      int bj = inA ? A : 0x7fffffff;
      if (ownB && xB > bv) {  // B > A: a tie keeps A
        bv = xB;
        bj = B;
      }
      wave_first_max(bv, bj);
      if (l == 0) p.last_state[blk] = (uint8_t)bj;
      if (urgent) __builtin_amdgcn_s_setprio(0);
    }
  }
}

// ---------------------------------------------------------------------------------------
// EXPERIMENT (ITR_EXPERIMENT builds, ITR_FV_WAVE_FWD=1): the forward log-likelihood sweep (optimizer.py:165-188) in the same one-task-per-wavefront
// layout: lane (g, q) holds the 9 x 9 slice of a (a^T for the backward half of a split
// block), forms 9 partial sums over its sources by FMA, writes them to P, and finalises one
// target (two for lanes 0-7) from the 8 partials: ~100 VALU instructions per column.  Tasks
// are the VALU sweep's (capi.cpp itr_plan_create: whole blocks, and the two halves of the
// blocks at least half as long as the longest: the forward over [0, m) and the textbook
// backward over [m, Tb) with x'_t = beta_t e_t, whose last step multiplies by a row of ones),
// the exact power-of-two rescale every 8 columns, the exponent kept as an integer, and the
// same outputs (log P of whole blocks; the split halves' vectors and exponents for
// fwd_split_combine).  Parity-green, but inside itr_forward_viterbi it made the step slower
// than the matrix-core forward split over the two CU sets (10.2 vs 9.7 ms at chr10,
// profiles/r2d_vit_layouts.txt): not adopted.
#ifdef ITR_EXPERIMENT
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = fmax(v, __shfl_xor(v, d));
  return v;
}

template <int IQ>
__device__ __forceinline__ void wave_fwd_tasks(const WaveFwdArgs& p, double* wl) {
  using C = WaveVit<IQ>;
  constexpr int XRW = C::XRW, NB = C::NB, IQS = C::IQS, XN = C::XN, PS = C::PS, HT = C::HT,
                NI = C::NI, EB = C::EB;
  const int l = threadIdx.x & 63, q = l & 7, g = l >> 3;
  const int n = p.n;
  double* X = wl;
  double* P = X + C::LX;
  double* EST = P + C::LP;
  uint16_t* SYM = reinterpret_cast<uint16_t*>(EST + C::LE);
  const int A = l, B = 64 + (l & 7);
  const bool inA = A < XRW && A < n;
  const bool inB = NB > 0 && B < n;
  const bool ownB = inB && l < NB;
  const int sA = A < XRW ? (A / IQ) * IQS + A % IQ : XN + l;
  const int sB = (NB > 0 && l < NB) ? (B / IQ) * IQS + B % IQ : XN + l;
  const int rA = A < XRW ? A : 0, rB = NB > 0 ? B : 0;
  for (int i = l; i < C::LX; i += 64) X[i] = 0.0;  // pad sources contribute nothing

  for (;;) {
    const int bi = uni(atomicAdd(p.queue, l == 0 ? 1 : 0));  // see wave_vit_blocks
    if (bi >= p.ntasks) break;
    const int32_t* td = p.tasks + 3 * bi;
    const int blk = uni(td[0]), split = uni(td[1]), slot = uni(td[2]);
    const int64_t c0 = p.off[blk];
    const int Tb = uni((int)(p.off[blk + 1] - c0));
    const int T = split > 0 ? split : (split < 0 ? Tb + split + 1 : Tb);
    if (T <= 0) {
      if (split == 0 && l == 0) p.loglik[blk] = 0.0;  // log-likelihood of nothing
    } else {
      const int dir = split < 0 ? -1 : 1;
      // the slice of a (a^T for a backward half), loaded per task: a few L2 loads against
      // thousands of steps
      double m[IQ][IQ];
      {
        const double* M = dir > 0 ? p.a : p.aT;
#pragma unroll
        for (int k = 0; k < IQ; ++k)
#pragma unroll
          for (int r = 0; r < IQ; ++r) {
            const int i = IQ * q + k, j = IQ * g + r;
            m[k][r] = (i < n && j < n) ? M[(int64_t)i * n + j] : 0.0;
          }
      }
      const bool urgent = T >= p.prio_len;
      if (urgent) __builtin_amdgcn_s_setprio(3);
      const uint16_t* ob = p.obs + c0;
      auto symg = [&](int s) -> int {
        const int s1 = min(s, Tb - 1);
        return min((int)ob[dir > 0 ? s1 : Tb - 1 - s1], 624);
      };
      SYM[l] = (uint16_t)symg(l);
      SYM[64 + l] = (uint16_t)symg(64 + l);
      int sin = symg(128 + l);
      // emission row of step s: the column's symbol; the backward half's last step: the row of
      // ones (row 625 of the padded table)
      auto srow = [&](int s) -> int {
        return (split < 0 && s == T - 1) ? 625 : (int)SYM[((s >> 6) & 1) * 64 + (s & 63)];
      };
      auto stage_issue = [&](int h) {
        double* d = EST + (h & 1) * EB;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int e = 128 * i + 2 * l;
          const double* src = p.ew;
          if (e < HT * XRW) src += (int64_t)srow(h * HT + e / XRW) * XRW + e % XRW;
          __builtin_amdgcn_global_load_lds(
              src, (__attribute__((address_space(3))) void*)(d + 128 * i), 16, 0, 0);
        }
      };
      auto stage_wait = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
      const int o0 = (int)SYM[0];
      const double* x0tab = dir < 0 ? p.emit : p.init;  // x'_{Tb-1} = e_{Tb-1}; alpha_0 = pi e_0
      double xA = inA ? x0tab[o0 * n + A] : 0.0;
      double xB = inB ? x0tab[o0 * n + B] : 0.0;
      X[sA] = xA;
      X[sB] = xB;
      int K = 0;  // sum of the power-of-two exponents divided out
      stage_issue(0);
      stage_wait();
      stage_issue(1);
      for (int t0 = 0; t0 < T; t0 += 16) {
#pragma unroll
        for (int sub = 0; sub < 16; ++sub) {
          const int t = t0 + sub;
          if (t >= 1 && t < T) {
            if ((sub & (HT - 1)) == 0) {  // half-tile boundary (t >= 8)
              stage_wait();
              if ((t & 63) == 0) {
                SYM[(((t >> 6) + 1) & 1) * 64 + l] = (uint16_t)sin;
                sin = symg(t + 128 + l);
              }
              stage_issue(t / HT + 1);
            }
            const double* es = EST + ((t / HT) & 1) * EB + (t & (HT - 1)) * XRW;
            double ecA = es[rA];
            double ecB = es[rB];
            if ((sub & 7) == 1) {  // exact 2^-e rescale by the max of x_{t-1}, into the factors
              const double Mx = wave_max(fmax(inA ? xA : 0.0, ownB ? xB : 0.0));
              const int e = (Mx > 0.0 && Mx < INFINITY) ? ilogb(Mx) : 0;
              const double sc = ldexp(1.0, -e);
              K += e;
              ecA *= sc;
              ecB *= sc;
            }
            double xs[IQ];
#pragma unroll
            for (int k = 0; k < IQ; ++k) xs[k] = X[q * IQS + k];
            double z[IQ];
#pragma unroll
            for (int r = 0; r < IQ; ++r) z[r] = xs[0] * m[0][r];
#pragma unroll
            for (int k = 1; k < IQ; ++k)
#pragma unroll
              for (int r = 0; r < IQ; ++r) z[r] = fma(xs[k], m[k][r], z[r]);
#pragma unroll
            for (int r = 0; r < IQ; ++r) P[(IQ * g + r) * PS + q] = z[r];
            const double* pa = P + rA * PS;
            xA = (((pa[0] + pa[1]) + (pa[2] + pa[3])) + ((pa[4] + pa[5]) + (pa[6] + pa[7]))) * ecA;
            if constexpr (NB > 0) {
              const double* pb = P + rB * PS;
              xB = (((pb[0] + pb[1]) + (pb[2] + pb[3])) + ((pb[4] + pb[5]) + (pb[6] + pb[7]))) *
                   ecB;
            }
            X[sA] = xA;
            X[sB] = xB;
          }
        }
      }
      if (split != 0) {  // half of a split block: the scaled vector and its exponent
        const int side = split < 0;
        double* sv = p.svec + ((int64_t)slot * 2 + side) * p.xr;
        if (inA) sv[A] = xA;
        if (ownB) sv[B] = xB;
        if (l == 0) p.sK[slot * 2 + side] = K;
      } else {  // log P = log(sum_j x_j) + K ln 2   (optimizer.py:160-162)
        const double tot = wave_sum((inA ? xA : 0.0) + (ownB ? xB : 0.0));
        if (l == 0) p.loglik[blk] = log(tot) + (double)K * LN2;
      }
      if (urgent) __builtin_amdgcn_s_setprio(0);
    }
  }
}

template <int IQ>
__global__ void __launch_bounds__(64 * kWaves, 2) wave_fwd_kernel(WaveFwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  wave_fwd_tasks<IQ>(p, reinterpret_cast<double*>(smem) +
                            (size_t)(threadIdx.x >> 6) * WaveVit<IQ>::WL);
}
#endif  // ITR_EXPERIMENT

template <int IQ>
__global__ void __launch_bounds__(64 * kWaves, 2) wave_vit_kernel(VitArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  wave_vit_blocks<IQ>(p, reinterpret_cast<double*>(smem) +
                             (size_t)(threadIdx.x >> 6) * WaveVit<IQ>::WL);
}

}  // namespace

WaveVitGeometry wave_vit_geometry(int n) {
  WaveVitGeometry g{};
  g.iq = -1;
  if (n > 64 && n <= 72) g.iq = 9;  // the (5,5) model, N = 70
  if (g.iq < 0) return g;
  g.block = 64 * kWaves;
  g.xr = 8 * g.iq;
  g.lds = (size_t)kWaves * WaveVit<9>::WL * sizeof(double);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, wave_vit_kernel<9>, g.block, g.lds) !=
          hipSuccess ||
      nb < 1)
    nb = 1;
  g.per_cu = nb;
  return g;
}

hipError_t launch_wave_fwd(const WaveVitGeometry& g, int grid, const WaveFwdArgs& p,
                           hipStream_t st) {
#ifndef ITR_EXPERIMENT
  (void)g, (void)grid, (void)p, (void)st;
  return hipErrorInvalidValue;
#else
  switch (g.iq) {
    case 9:
      hipLaunchKernelGGL(wave_fwd_kernel<9>, dim3(grid), dim3(g.block), g.lds, st, p);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
#endif
}

hipError_t launch_wave_vit(const WaveVitGeometry& g, int grid, const VitArgs& p,
                           hipStream_t st) {
  switch (g.iq) {
    case 9:
      hipLaunchKernelGGL(wave_vit_kernel<9>, dim3(grid), dim3(g.block), g.lds, st, p);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace itr
