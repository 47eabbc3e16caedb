// prune_vit.hip — Viterbi for the larger models (72 < N <= 140: the introgression (5,5)
// model, N = 95; the (7,7) model, N = 133) on MI355X (gfx950): one block per wavefront,
// log a in the workgroup's LDS (shared by every wave: all blocks decode with one model), the
// bound-pruned step of wave_tasks.h generalised to any N and made throughput-first.
//
// Why a separate layout.  At N = 65..72 the per-wave Viterbi keeps each lane's slice of log a
// in VGPRs (162 of them).  At N = 133 a slice of N^2 / 64 = 276 doubles per lane does not fit,
// so until round 5 these models ran the 9-wave workgroup layout (one block per CU, a barrier
// and an all-reduce per column, ~2N^2 / 64 VALU instructions per column of a block whatever
// the data).  Here the matrix lives once per CU in LDS (laT[j][i] = log a_ij, -inf on the
// diagonal: 142 KB at N = 133, 72 KB at N = 95), a wave's registers hold only its block's
// omega (lane l: states l, l + 64, l + 128), and per column:
//
//   1. Omega = max_i omega_i (DPP + lane reads), and for every target j the stay score
//      yd = fl(fl(omega_j + log a_jj) + log e_j) and the bound
//      B_j = fl(fl(Omega + M_j) + log e_j), M_j = max_{i != j} log a_ij.  Rounding is
//      monotone, so every other candidate fl(fl(omega_i + log a_ij) + log e_j) <= B_j: a
//      target with yd > B_j keeps its state, bit for bit what the full scan gives (the stay
//      flag is 1, omega_t[j] = yd).
//   2. The failing targets are ranked (ballot + mbcnt) into the wave's list and scanned
//      eight at a time: lane 8 k + q forms max over sources q S .. q S + S - 1 of
//      fl(omega_i + log a_ij) for the k-th listed target (S = ceil(N / 8) sources per lane,
//      rows of R = 8 S doubles; omega from the wave's LDS row, log a from laT), three DPP stages combine the eight lanes,
//      and lane q = 0 leaves the target's zo = max_{i != j} in the wave's result row.
//   3. The owner of a failing target: yo = fl(zo + log e_j), stay flag = yd > yo,
//      omega_t[j] = max(yd, yo) — the reference's max, its first argmax j exactly when
//      yd > yo (otherwise the traceback resolves the column exactly, trace.h).
//
// The outputs are those of every Viterbi sweep of this library (checkpoint rows of each
// 16-column tile's first column, 16-bit stay-flag words, the last column's first argmax),
// so the traceback (vit_trace_kernel) and the paths are shared and bit-identical.  A wave's
// LDS instructions execute in order, so a step needs no barrier; blocks come longest first
// from one device counter.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {
namespace {

constexpr int kPvQ = 8;       // lanes per scanned target
constexpr int kPvNmax = 144;  // S = 18 sources per scanning lane at most

__device__ __forceinline__ int pv_next(int* queue) {  // (every lane: see wave_sweeps.hip)
  return uni(atomicAdd(queue, (threadIdx.x & 63) == 0 ? 1 : 0));
}

// the wave's maximum of v (every lane gets it)
__device__ __forceinline__ double pv_wave_max(double v) {
  v = fmax(v, dpp_f64<DPP_Q1>(v));
  v = fmax(v, dpp_f64<DPP_Q2>(v));
  v = fmax(v, dpp_f64<DPP_HM>(v));
  v = fmax(v, dpp_f64<DPP_R8>(v));
  return fmax(fmax(lane_f64(v, 0), lane_f64(v, 16)), fmax(lane_f64(v, 32), lane_f64(v, 48)));
}

// lanes below this one with a bit set in `mask`
__device__ __forceinline__ int pv_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

template <int G, int S>  // state slots per lane (n <= 64 G), sources per scanning lane
__device__ __forceinline__ void pv_block(const PruneVitArgs& p, const double* laT, double* om,
                                         double* res, uint8_t* list, int blk) {
  const int l = threadIdx.x & 63;
  const int n = p.n;
  const int64_t c0 = p.off[blk];
  const int T = uni((int)(p.off[blk + 1] - c0));
  if (T <= 0) return;
  const int64_t tk0 = p.tile_off[blk];
  const uint16_t* obs = p.obs + c0;
  const int xr = p.xr;
  const bool urgent = T >= p.prio_len;
  if (urgent) __builtin_amdgcn_s_setprio(2);

  int jt[G];
  bool jv[G];
  double ld[G], mj[G];  // log a_jj and M_j = max_{i != j} log a_ij of this lane's targets
#pragma unroll
  for (int g = 0; g < G; ++g) {
    jt[g] = l + 64 * g;
    jv[g] = jt[g] < n;
    ld[g] = jv[g] ? p.la[(int64_t)jt[g] * n + jt[g]] : 0.0;
    mj[g] = jv[g] ? p.mj[jt[g]] : -INFINITY;
  }
  // symbols 64 columns at a time (lane c holds column 64 b + c); the step reads its own
  int symc = 0;
  int sym_next = l < T ? (int)obs[l] : 0;
  auto sym_at = [&](int t) -> int {  // t: the step's column; refills at multiples of 64
    return __builtin_amdgcn_readlane(symc, t & 63);
  };
  // omega_0 = log(pi * e_{o0})
  symc = sym_next;
  sym_next = 64 + l < T ? (int)obs[64 + l] : 0;
  double w[G];
  {
    const int o0 = min(sym_at(0), 624);
#pragma unroll
    for (int g = 0; g < G; ++g) w[g] = jv[g] ? p.lpie[(int64_t)o0 * n + jt[g]] : -INFINITY;
  }
  constexpr int R = kPvQ * S;  // row stride of laT and of the omega row
  // the padding of the omega row (sources n .. R - 1) stays -inf for the whole block
  for (int i = n + l; i < R; i += 64) om[i] = -INFINITY;
  // log e of the next column, loaded one step ahead
  double le[G];
  auto load_le = [&](int t, double (&dst)[G]) {
    const int o = t < T ? min(sym_at(t), 624) : 0;
#pragma unroll
    for (int g = 0; g < G; ++g) dst[g] = jv[g] ? p.log_e[(int64_t)o * n + jt[g]] : -INFINITY;
  };
  if (T > 1) load_le(1, le);
  uint32_t bits[G];
#pragma unroll
  for (int g = 0; g < G; ++g) bits[g] = 0;
  // the tile-0 checkpoint row: column 0
#pragma unroll
  for (int g = 0; g < G; ++g)
    if (jv[g]) p.ckpt[tk0 * xr + jt[g]] = w[g];
  wait_vmem_all();
  const int q = l & (kPvQ - 1), k8 = l >> 3;
#ifdef ITR_EXPERIMENT
  unsigned long long dg_f = 0, dg_p = 0;
#endif
  for (int t = 1; t < T; ++t) {
    const int sub = t & (VIT_TILE - 1);
    if ((t & 63) == 0) {  // next 64 symbols (the lanes' register already holds them)
      symc = sym_next;
      sym_next = t + 64 + l < T ? (int)obs[t + 64 + l] : 0;
    }
    double e[G];
#pragma unroll
    for (int g = 0; g < G; ++g) e[g] = le[g];
    if (t + 1 < T) {
      if (((t + 1) & 63) == 0) {  // (the next column's symbol is in the next batch)
        const int o = min(__builtin_amdgcn_readlane(sym_next, 0), 624);
#pragma unroll
        for (int g = 0; g < G; ++g) le[g] = jv[g] ? p.log_e[(int64_t)o * n + jt[g]] : -INFINITY;
      } else {
        load_le(t + 1, le);
      }
    }
    // publish omega_{t-1} for the scans (this wave's row; LDS is in order within a wave)
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (jv[g]) om[jt[g]] = w[g];
    double mx = w[0];
#pragma unroll
    for (int g = 1; g < G; ++g) mx = fmax(mx, w[g]);
    const double Om = pv_wave_max(mx);
    double yd[G];
    uint64_t fb[G];
    int base = 0;
    int rk[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      yd[g] = (w[g] + ld[g]) + e[g];
      const double bnd = (Om + mj[g]) + e[g];
      const bool fail = jv[g] && !(yd[g] > bnd);
      fb[g] = __ballot(fail);
      rk[g] = base + pv_rank(fb[g]);
      if (fail) list[rk[g]] = (uint8_t)jt[g];
      base += __builtin_popcountll(fb[g]);
    }
    const int nf = uni(base);
#ifdef ITR_EXPERIMENT
    dg_f += nf;
    dg_p += (nf + 7) / 8;
#endif
    wave_lds_sync();
    // scans of the failing targets, eight per pass
    for (int k0 = 0; k0 < nf; k0 += 8) {
      const int k = k0 + k8;
      const int j = k < nf ? (int)list[k] : 0;
      const double* ar = laT + (int64_t)j * R + q * S;
      const double* orow = om + q * S;
      double z0 = -INFINITY, z1 = -INFINITY, z2 = -INFINITY;  // three independent chains
#pragma unroll
      for (int s = 0; s < S; ++s) {
        const double v = orow[s] + ar[s];
        if (s % 3 == 0) z0 = fmax(z0, v);
        else if (s % 3 == 1) z1 = fmax(z1, v);
        else z2 = fmax(z2, v);
      }
      double z[1] = {fmax(fmax(z0, z1), z2)};
      combine_max<kPvQ, 1>(z);
      if (q == 0 && k < nf) res[k] = z[0];
    }
    wave_lds_sync();
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bool fail = (fb[g] >> l) & 1;
      double nw = yd[g];
      bool stay = true;
      if (fail) {
        const double yo = res[rk[g]] + e[g];
        stay = yd[g] > yo;
        nw = fmax(yd[g], yo);
      }
      w[g] = jv[g] ? nw : -INFINITY;
      bits[g] |= (uint32_t)stay << sub;
    }
    if (sub == 0) {  // the tile's checkpoint row (column t = 16 k)
      const int64_t rec = (tk0 + (t >> 4)) * xr;
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (jv[g]) p.ckpt[rec + jt[g]] = w[g];
    }
    if (sub == VIT_TILE - 1 || t == T - 1) {  // the tile's flag words
      const int64_t rec = (tk0 + (t >> 4)) * xr;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if (jv[g]) p.stay[rec + jt[g]] = (uint16_t)bits[g];
        bits[g] = 0;
      }
    }
  }
  if (T == 1) {  // (tile 0's flag word: no step, never read; written for determinism)
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (jv[g]) p.stay[tk0 * xr + jt[g]] = 0;
  }
  // last state = first argmax of omega_{T-1} (optimizer.py:346)
  double bv = w[0];
  int bj = jv[0] ? jt[0] : 0x7fffffff;
#pragma unroll
  for (int g = 1; g < G; ++g)
    if (jv[g] && w[g] > bv) {
      bv = w[g];
      bj = jt[g];
    }
  wave_first_max(bv, bj);
  if (l == 0) p.last_state[blk] = (uint8_t)bj;
#ifdef ITR_EXPERIMENT
  if (p.diag && l == 0) {
    atomicAdd(&p.diag[0], (unsigned long long)(T - 1));
    atomicAdd(&p.diag[1], dg_f);
    atomicAdd(&p.diag[2], dg_p);
  }
#endif
  if (urgent) __builtin_amdgcn_s_setprio(0);
  wave_lds_sync();
}

template <int G, int S>
__global__ void __launch_bounds__(1024) prune_vit_kernel(PruneVitArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int R = kPvQ * S;
  const int n = p.n;
  double* laT = reinterpret_cast<double*>(smem);  // [n][R]: laT[j][i] = log a_ij
  // log a transposed into LDS, -inf on the diagonal (the stay is scored apart) and in the
  // padding sources
  for (int e = threadIdx.x; e < n * R; e += blockDim.x) {
    const int j = e / R, i = e % R;
    laT[e] = (i < n && i != j) ? p.la[(int64_t)i * n + j] : -INFINITY;
  }
  const int w = threadIdx.x >> 6;
  double* om = laT + (size_t)n * R + (size_t)w * 2 * R;  // [R] omega row
  double* res = om + R;                                   // [R] scan results
  uint8_t* list = reinterpret_cast<uint8_t*>(laT + (size_t)n * R + (size_t)(blockDim.x >> 6) * 2 * R) +
                  (size_t)w * R;  // [R] failing targets
  __syncthreads();
  for (;;) {
    const int bi = pv_next(p.queue);
    if (bi >= p.nblocks) break;
    pv_block<G, S>(p, laT, om, res, list, uni(p.order[bi]));
  }
}

int pv_sources(int n) { return (n + kPvQ - 1) / kPvQ; }
size_t pv_lds(int n, int waves) {
  const int R = kPvQ * pv_sources(n);
  return (size_t)n * R * 8 + (size_t)waves * (2 * R * 8 + R);
}

}  // namespace

PruneVitGeometry prune_vit_geometry(int n) {
  PruneVitGeometry g{};
  g.waves = 0;
  // (N <= 72: the per-wave layouts of wave_tasks.h; this kernel on the (5,5) bulk measured
  // 13.2 vs 6.1 ms per itr_viterbi call, profiles/r5i_pv_bulk70_ab.txt)
  if (n <= 72 || n > kPvNmax) return g;
  // as many waves (blocks) per CU as the LDS holds beside the matrix, at most 16
  int waves = 16;
  while (waves > 1 && pv_lds(n, waves) > 160 * 1024) --waves;
  // N = 141..144: the matrix and one wave's rows exceed the 160 KiB of LDS (no layout)
  if (pv_lds(n, waves) > 160 * 1024) return g;
  g.waves = waves;
  g.block = 64 * waves;
  g.lds = pv_lds(n, waves);
  g.sources = pv_sources(n);
  return g;
}

hipError_t launch_prune_vit(const PruneVitGeometry& g, int grid, const PruneVitArgs& p,
                            hipStream_t st) {
  if (g.waves <= 0 || grid <= 0) return hipErrorInvalidValue;
#define ITR_PV(G, S)                                                                     \
  case S:                                                                                \
    hipLaunchKernelGGL((prune_vit_kernel<G, S>), dim3(grid), dim3(g.block), g.lds, st, p); \
    break;
  switch (g.sources) {  // (the launch bounds hold 16 waves: 128 VGPRs per lane at most)
    ITR_PV(2, 10)
    ITR_PV(2, 11)
    ITR_PV(2, 12)
    ITR_PV(2, 13)
    ITR_PV(2, 14)
    ITR_PV(2, 15)
    ITR_PV(2, 16)
    ITR_PV(3, 17)
    ITR_PV(3, 18)
    default:
      return hipErrorInvalidValue;
  }
#undef ITR_PV
  return hipGetLastError();
}

}  // namespace itr
