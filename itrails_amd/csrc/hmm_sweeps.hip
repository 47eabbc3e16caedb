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

namespace itr {

// QL (template parameter, 4 or 8): lanes splitting the i-sum of one target state
// columns per staged tile of per-column rows: 16, or 8 for the backward sweep of large
// models (it stages two tables; 8 keeps two workgroups' LDS within the CU's 160 KiB)
static constexpr int tile_cols(int mode, int xr) { return (mode == MODE_BWD && xr > 96) ? 8 : 16; }
static constexpr double LN2 = 0.69314718055994530942;

// Diagnostic build only (-DITR_DIAG, libitrails_hip_diag.so): one wave (ITR_DIAG_WAVE, 0) of every workgroup
// accumulates shader-clock cycles per step segment; never compiled into the product.
#ifdef ITR_DIAG
#define DIAG_DECL uint64_t dsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}; uint64_t dlast = 0; uint64_t dsteps = 0;
#define STAMP(i)                                                   \
  do {                                                             \
    __builtin_amdgcn_sched_barrier(0);                             \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();            \
    __builtin_amdgcn_sched_barrier(0);                             \
    if ((i) >= 0) dsum[(i) < 0 ? 0 : (i)] += now_ - dlast;         \
    dlast = now_;                                                  \
  } while (0)
#define DIAG_STEP() (++dsteps)
#define DIAG_FLUSH()                                                          \
  do {                                                                        \
    if (l == 0 && w == p.diag_wave && p.diag) {                               \
      for (int i_ = 0; i_ < 8; ++i_) atomicAdd((unsigned long long*)&p.diag[i_], \
                                               (unsigned long long)dsum[i_]);  \
      atomicAdd((unsigned long long*)&p.diag[8], (unsigned long long)dsteps);   \
    }                                                                         \
  } while (0)
#else
#define DIAG_DECL
#define STAMP(i)
#define DIAG_STEP()
#define DIAG_FLUSH()
#endif

// ---------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}
// first-maximum reduction over the wave: larger value wins, equal values -> lower index
__device__ __forceinline__ void wave_first_max(double& v, int& idx) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const double ov = __shfl_xor(v, d);
    const int oi = __shfl_xor(idx, d);
    const bool take = (ov > v) || (ov == v && oi < idx);
    v = take ? ov : v;
    idx = take ? oi : idx;
  }
}

// DPP cross-lane moves (a VALU operand modifier: a few cycles, no LDS round trip).
// Within the 8 lanes q = l & 7 of one target state: stage 1 pairs q with q^1, stage 2 with
// q^2 (quad_perm), stage 3 with 7-q (row_half_mirror).  Across the two target states of a
// 16-lane row: row_ror:8.
static constexpr int DPP_Q1 = 0xB1;   // quad_perm [1,0,3,2]
static constexpr int DPP_Q2 = 0x4E;   // quad_perm [2,3,0,1]
static constexpr int DPP_HM = 0x141;  // row_half_mirror
static constexpr int DPP_R8 = 0x128;  // row_ror:8
static constexpr int DPP_R4 = 0x124;  // row_ror:4
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = dpp_i32<CTRL>(__double2loint(v));
  const int hi = dpp_i32<CTRL>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
// after the three stages all 8 lanes hold ((a0+a1)+(a2+a3))+((a4+a5)+(a6+a7)): every
// addition is commutative, so the 8 copies are bit-identical
// (four lanes: stages 1 and 2 only)
template <int QL, int RJN>
__device__ __forceinline__ void combine_sum(double (&acc)[RJN]) {
#pragma unroll
  for (int r = 0; r < RJN; ++r) acc[r] += dpp_f64<DPP_Q1>(acc[r]);
#pragma unroll
  for (int r = 0; r < RJN; ++r) acc[r] += dpp_f64<DPP_Q2>(acc[r]);
  if constexpr (QL == 8) {
#pragma unroll
    for (int r = 0; r < RJN; ++r) acc[r] += dpp_f64<DPP_HM>(acc[r]);
  }
}
// Maximum over the QL lanes of a target state (fmax is exact and order-free, so all lanes
// end with the identical value).
template <int QL, int RJN>
__device__ __forceinline__ void combine_max(double (&v)[RJN]) {
#pragma unroll
  for (int r = 0; r < RJN; ++r) v[r] = fmax(v[r], dpp_f64<DPP_Q1>(v[r]));
#pragma unroll
  for (int r = 0; r < RJN; ++r) v[r] = fmax(v[r], dpp_f64<DPP_Q2>(v[r]));
  if constexpr (QL == 8) {
#pragma unroll
    for (int r = 0; r < RJN; ++r) v[r] = fmax(v[r], dpp_f64<DPP_HM>(v[r]));
  }
}
// Across the 16 / QL target groups of a 16-lane row (each group's lanes hold equal values)
template <int QL>
__device__ __forceinline__ double row_max(double v) {
  if constexpr (QL == 4) v = fmax(v, dpp_f64<DPP_R4>(v));
  return fmax(v, dpp_f64<DPP_R8>(v));
}
template <int QL>
__device__ __forceinline__ double row_sum(double v) {
  if constexpr (QL == 4) v += dpp_f64<DPP_R4>(v);
  return v + dpp_f64<DPP_R8>(v);
}

// s_waitcnt vmcnt(0) (expcnt/lgkmcnt untouched).  Issued once before each step loop so
// that no loop-carried register is the destination of a load in flight at loop entry:
// otherwise hipcc's waitcnt pass puts a vmcnt(0) INSIDE the loop at that register's first
// use, which then drains the staged-row and symbol loads every column.
__device__ __forceinline__ void wait_vmem_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup-scope fence
// over ALL address spaces, which on gfx950 drains vmcnt to 0 at every column: it would wait
// for the back-pointer / forward-row stores and the staged-row loads each step.  All
// inter-wave exchange in this kernel goes through LDS, so the fences are "local" only.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Observed symbols of the current block staged in LDS, one per thread per tile (forward:
// step s is column s; backward: column T-1-s).  Two tiles are resident and the next one is
// in flight in a register of every thread, so its global load is waited for a whole tile
// after it was issued.
struct ObsTiles {
  uint16_t* lds;      // [2][tb]
  const uint16_t* g;  // block's first column
  int T, dir;         // dir = +1 forward, -1 backward
  int tb;             // symbols per tile = threads per workgroup
  int inflight;       // this thread's element of the next tile to store

  __device__ __forceinline__ int col(int s) const { return dir > 0 ? s : T - 1 - s; }
  __device__ __forceinline__ int fetch(int s) const {
    return (s >= 0 && s < T) ? (int)g[col(s)] : 0;
  }
  // symbols outside the 625-letter alphabet are clamped (memory safety; the host wrappers
  // reject them before they reach the device)
  __device__ __forceinline__ static uint16_t clamp(int v) { return (uint16_t)min(v, 624); }
  __device__ __forceinline__ void start(int tid) {  // tiles 0, 1 in LDS; tile 2 in flight
    lds[tid] = clamp(fetch(tid));
    lds[tb + tid] = clamp(fetch(tb + tid));
    inflight = fetch(2 * tb + tid);
  }
  // at step s (before the step's barrier): when s starts tile k >= 1, tile k+1 replaces
  // tile k-1 and tile k+2 is requested
  __device__ __forceinline__ void advance(int s, int tid) {
    if (s >= tb && (s % tb) == 0) {
      const int k = s / tb;
      lds[((k + 1) & 1) * tb + tid] = clamp(inflight);
      inflight = fetch((k + 2) * tb + tid);
    }
  }
  __device__ __forceinline__ int get(int s) const {  // symbol at step s (LDS broadcast)
    return (s < T) ? (int)lds[((s / tb) & 1) * tb + (s % tb)] : 0;
  }
};

// Rows of a global row-major table (E / log E by observed symbol, or stored forward rows by
// column) for TE consecutive steps, loaded into registers one tile ahead and committed to an
// LDS ring [2][TE][XR] at the tile boundary.  Element idx = tid + e*TB of a tile is row
// idx / XR, target state idx % XR.
template <int WV, int XR, int TE>
struct RowStage {
  static constexpr int TB = 64 * WV;
  static constexpr int RS = TE * XR / TB;  // elements per thread
  static_assert(RS * TB == TE * XR, "tile must split evenly over the workgroup");
  double v[RS];
  template <class RowOf>
  __device__ __forceinline__ void issue(const double* __restrict__ g, int stride, int ncol,
                                        int tid, int s0, RowOf row_of) {
#pragma unroll
    for (int e = 0; e < RS; ++e) {
      const int idx = tid + e * TB;
      const int row = idx / XR, col = idx % XR;
      const int64_t src = row_of(s0 + row);
      // row -2: a row of ones (the backward half's last step, see the forward sweep)
      v[e] = (src >= 0 && col < ncol) ? g[src * stride + col] : (src == -2 ? 1.0 : 0.0);
    }
  }
  __device__ __forceinline__ void commit(double* lds_tile, int tid) const {
#pragma unroll
    for (int e = 0; e < RS; ++e) lds_tile[e * TB + tid] = v[e];
  }
};

// ---------------------------------------------------------------------------------------
// the sweep kernel: RJN target states per lane, IQ source states per lane
// ---------------------------------------------------------------------------------------
// co-resident workgroups per CU the register budget is sized for
template <int QL, int WV, int RJN, int IQ, int MODE>
struct Occ {
  // VGPRs a lane needs: its slice of the matrix, the source values it reads, working set
  static constexpr int need = 2 * RJN * IQ + 2 * IQ + 64;
  static constexpr int simd_waves = 512 / need;  // waves one SIMD's register file holds
  static constexpr int fit = simd_waves * 4 / WV;
  static constexpr int wide = fit > 3 ? 3 : (fit < 1 ? 1 : fit);
  // four-wave configurations: budget measured on the (5,5) model (N = 70)
  static constexpr int narrow = RJN * IQ <= 27 ? 3 : RJN * IQ <= 64 ? 2 : 1;
  static constexpr int base = (WV == 4 && QL == 8) ? narrow : wide;
  static constexpr int wgs = (MODE == MODE_BWD && base > 1) ? base - 1 : base;
  // launch_bounds' second argument is waves per SIMD.  A workgroup's waves are spread
  // round-robin over the 4 SIMDs starting at SIMD 0, so every co-resident workgroup puts
  // ceil(W/4) waves on SIMD 0: budget for that, not for the average.
  static constexpr int value = wgs * ((WV + 3) / 4);
};


template <int QL, int WV, int RJN, int IQ, int MODE>
__device__ __forceinline__ void sweep_device(const SweepArgs& p) {
  constexpr int W = WV;       // wavefronts per workgroup
  constexpr int TB = 64 * W;  // threads per workgroup
  constexpr int IQS = IQ + (IQ & 1);  // 16-byte aligned source ranges in LDS
  constexpr int XS = QL * IQS;        // published vector length
  constexpr int GW = 64 / QL;         // target groups per wave
  constexpr int JW = GW * RJN;        // target states per wave
  constexpr int XR = W * JW;          // padded target states per workgroup
  constexpr int TE = tile_cols(MODE, XR);
  constexpr int NCH = IQ >= 6 ? 3 : (IQ >= 2 ? 2 : 1);  // independent chains per target
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = p.n;
  const int tid = threadIdx.x;
  const int w = uni(tid >> 6);
  const int l = tid & 63;
  const int q = l & (QL - 1);
  const int jl = l / QL;
  const int row16 = w * 4 + (l >> 4);  // 16-lane row of the workgroup (0..4W-1)
  constexpr int NROW = 4 * W;
  const bool row_leader = (l & 15) == 0;

  double* X = reinterpret_cast<double*>(smem);  // [2][XS+64]    published vectors + a
                                                //               per-lane write sink
  double* RED = X + 2 * (XS + 64);              // [5][64]       row partials
  double* EST = RED + 5 * 64;                   // [2][TE][XR]   staged emission rows
  double* AST = EST + 2 * TE * XR;              // [2][TE][XR]   staged forward rows (BWD)
  int* SBLK = reinterpret_cast<int*>(AST + ((MODE == MODE_BWD) ? 2 * TE * XR : 0));
  int* REDI = SBLK + 4;                                      // [16]
  uint16_t* OBS = reinterpret_cast<uint16_t*>(SBLK + 32);    // [2][TB]

  // Publishing is branch-free: the one lane (q == 0) of a real target state writes its
  // slot, every other lane writes the same value into its own sink entry nobody reads.
  int jr[RJN], jx[RJN];
  bool jv[RJN];
#pragma unroll
  for (int r = 0; r < RJN; ++r) {
    jr[r] = w * JW + r * GW + jl;
    jv[r] = jr[r] < n;
    const bool pub = jv[r] && q == 0;
    jx[r] = pub ? (jr[r] / IQ) * IQS + jr[r] % IQ : XS + l;  // slot of state jr in X
  }

  // this lane's slice of a (or log a): rows i = q*IQ + k, columns jr[r].  Viterbi keeps the
  // self-transition log a_jj out of the max-plus chain (-inf there) and in ldiag instead:
  // the chain then yields max over i != j, which with the diagonal term decides whether
  // the first maximum is j itself (see the Viterbi sweep below).
  double m[IQ][RJN];
  double ldiag[RJN];
#pragma unroll
  for (int r = 0; r < RJN; ++r)
    ldiag[r] = (MODE == MODE_VIT && jv[r]) ? p.mat[(int64_t)jr[r] * n + jr[r]] : 0.0;
#pragma unroll
  for (int k = 0; k < (MODE == MODE_FWD_LL ? 0 : IQ); ++k) {  // FWD_LL: loaded per task
    const int i = q * IQ + k;
#pragma unroll
    for (int r = 0; r < RJN; ++r) {
      m[k][r] = (i < n && jv[r]) ? p.mat[(int64_t)i * n + jr[r]] : 0.0;
      if (MODE == MODE_VIT && i == jr[r]) m[k][r] = -INFINITY;
    }
  }

  // published entries of states >= n are never written: 0 for the probability sweeps
  // (contributes nothing), -inf for Viterbi (never a maximum)
  const double pad = (MODE == MODE_VIT) ? -INFINITY : 0.0;
  for (int i = tid; i < 2 * (XS + 64); i += TB) X[i] = pad;
  lds_barrier();

  RowStage<W, XR, TE> est;
  RowStage<W, XR, TE> ast;
  (void)ast;
  DIAG_DECL

  for (;;) {
    if (tid == 0) SBLK[0] = atomicAdd(p.queue, 1);
    lds_barrier();
    const int bi = uni(SBLK[0]);
    lds_barrier();
    if (bi >= p.nblocks) break;
    // forward log-likelihood tasks (itr_plan_create): {block, split, slot}; split 0 = the
    // whole block, +m = columns [0, m) forward, -m = the backward half (see below)
    const int32_t* td = (MODE == MODE_FWD_LL) ? p.tasks + 3 * bi : nullptr;
    const int blk = uni(td ? td[0] : p.order[bi]);
    const int split = td ? uni(td[1]) : 0;
    const int slot = td ? uni(td[2]) : 0;
    const int64_t c0 = p.off[blk];
    const int Tb = uni((int)(p.off[blk + 1] - c0));
    // steps + 1 of this task: the backward half runs Tb - m steps
    const int T = split > 0 ? split : (split < 0 ? Tb + split + 1 : Tb);
    // NOTE: no `continue` in this loop.  With a barrier in the body, hipcc (ROCm 7.2)
    // structurizes a `continue` back to the head's `if (tid == 0)` as a lane-divergent
    // inner loop around the barrier, which deadlocks the workgroup.
    if (T <= 0) {  // empty block: log-likelihood of nothing is 0, no other output
      if (MODE == MODE_FWD_LL && tid == 0) p.loglik[blk] = 0.0;
    } else {
      const bool urgent = T >= p.prio_len;
      if (urgent) __builtin_amdgcn_s_setprio(2);
      if constexpr (MODE == MODE_FWD_LL) {
        // the slice of a, or of a^T for a backward half, loaded for every task (a few L2
        // loads against thousands of steps; an unconditional load keeps m out of the
        // loop-carried state)
        const double* mp = split < 0 ? p.matT : p.mat;
#pragma unroll
        for (int k = 0; k < IQ; ++k) {
          const int i = q * IQ + k;
#pragma unroll
          for (int r = 0; r < RJN; ++r)
            m[k][r] = (i < n && jv[r]) ? mp[(int64_t)i * n + jr[r]] : 0.0;
        }
      }
      ObsTiles ot{OBS, p.obs + c0, Tb, (MODE == MODE_BWD || split < 0) ? -1 : +1, TB, 0};
      ot.start(tid);
      lds_barrier();
      auto sym_row = [&](int s) -> int64_t {
        if (split < 0) return s < T - 1 ? (int64_t)ot.get(s) : (s == T - 1 ? -2 : -1);
        return s < T ? (int64_t)ot.get(s) : -1;
      };
      auto fwd_row = [&](int s) -> int64_t { return s < T ? c0 + (T - 1 - s) : -1; };
      est.issue(p.emit, n, n, tid, 0, sym_row);
      est.commit(EST, tid);
      est.issue(p.emit, n, n, tid, TE, sym_row);
      if constexpr (MODE == MODE_BWD) {
        ast.issue(p.alpha, XR, XR, tid, 0, fwd_row);
        ast.commit(AST, tid);
        ast.issue(p.alpha, XR, XR, tid, TE, fwd_row);
      }
      // a new staged tile starts at step s: commit it before the step's barrier ...
      auto stage_commit = [&](int s) {
        if (s >= TE && (s & (TE - 1)) == 0) {
          const int slot = (s / TE) & 1;
          est.commit(EST + slot * TE * XR, tid);
          if constexpr (MODE == MODE_BWD) ast.commit(AST + slot * TE * XR, tid);
        }
      };
      // ... and request the one after it behind the barrier
      auto stage_issue = [&](int s) {
        if (s >= TE && (s & (TE - 1)) == 0) {
          est.issue(p.emit, n, n, tid, s + TE, sym_row);
          if constexpr (MODE == MODE_BWD) ast.issue(p.alpha, XR, XR, tid, s + TE, fwd_row);
        }
      };
      auto staged = [&](const double* base, int s, int j) {
        return base[((s / TE) & 1) * TE * XR + (s & (TE - 1)) * XR + j];
      };
      lds_barrier();

      if constexpr (MODE == MODE_FWD_LL || MODE == MODE_FWD_STORE) {
        // ------------- forward: alpha_t = (alpha_{t-1} @ a) * e_t  (optimizer.py:181-187)
        // Rows written to p.alpha (posterior workspace) have stride XR: every lane stores,
        // padded states store 0, duplicates store the same value (no branches).
        // Long blocks are split (meet in the middle, exact in real arithmetic):
        //   log P = log sum_j alpha_{m-1}[j] beta_{m-1}[j],  beta_{Tb-1} = 1,
        //   beta_{t-1} = a (e_t * beta_t)   (the textbook backward, not the reference's v @ a)
        // The forward half runs columns [0, m).  The backward half carries
        // x'_t = beta_t * e_t from x'_{Tb-1} = e_{Tb-1}: every step is "contract with a^T,
        // multiply by the next column's emission" — the forward step's shape — and its last
        // step multiplies by a row of ones, leaving beta_{m-1}.  Both halves run Tb/2 steps
        // on different workgroups; fwd_split_combine_kernel forms the dot product.
        const int o0 = ot.get(0);
        const double* x0tab = (MODE == MODE_FWD_LL && split < 0) ? p.emit : p.init;
        double x[RJN];
#pragma unroll
        for (int r = 0; r < RJN; ++r) x[r] = jv[r] ? x0tab[o0 * n + jr[r]] : 0.0;
        if constexpr (MODE == MODE_FWD_STORE) {
#pragma unroll
          for (int r = 0; r < RJN; ++r) p.alpha[c0 * XR + jr[r]] = x[r];
        }
        int K = 0;  // sum of the power-of-two exponents divided out so far
        wait_vmem_all();
        STAMP(-1);
        // steps in tiles of TE: the periodic work sits at compile-time positions of the
        // unrolled tile, so a normal step executes no taken branch
        for (int t0 = 0; t0 < T; t0 += TE) {
#pragma unroll
          for (int sub = 0; sub < TE; ++sub) {
            const int t = t0 + sub;
            if (t >= 1 && t < T) {
              DIAG_STEP();
              const int buf = sub & 1;  // t0 is even
              double* Xb = X + buf * (XS + 64);
#pragma unroll
              for (int r = 0; r < RJN; ++r) Xb[jx[r]] = x[r];
              const bool rescale = (sub & 7) == 1;
              if (rescale) {  // row maxima of x_{t-1} (padded states hold 0)
                double mx = x[0];
#pragma unroll
                for (int r = 1; r < RJN; ++r) mx = fmax(mx, x[r]);
                mx = row_max<QL>(mx);
                if (row_leader) RED[128 + buf * 64 + row16] = mx;
              }
              // emission factors of column t: staged at the start of this tile, so (except
              // on the tile's first step, which commits them) readable before the barrier
              double ec[RJN];
              if (sub != 0) {
#pragma unroll
                for (int r = 0; r < RJN; ++r) ec[r] = staged(EST, t, jr[r]);
              }
              if (sub == 0) {
                ot.advance(t, tid);
                stage_commit(t);
              }
              STAMP(0);
              lds_barrier();
              STAMP(1);
              if (sub == 0) {
                stage_issue(t);
#pragma unroll
                for (int r = 0; r < RJN; ++r) ec[r] = staged(EST, t, jr[r]);
              }
              const double* xs = Xb + q * IQS;
              // NCH independent partial sums per target (k = c mod NCH): the dependent
              // FP64 chain is ceil(IQ/NCH) long instead of IQ
              double acc[NCH][RJN];
#pragma unroll
              for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int r = 0; r < RJN; ++r) acc[c][r] = 0.0;
#pragma unroll
              for (int k = 0; k < IQ; ++k) {
                const double xi = xs[k];
#pragma unroll
                for (int r = 0; r < RJN; ++r) acc[k % NCH][r] = fma(xi, m[k][r], acc[k % NCH][r]);
              }
              if (rescale) {  // fold 2^-e into the emission factor (off the FMA chain)
                double M = RED[128 + buf * 64];
#pragma unroll
                for (int v = 1; v < NROW; ++v) M = fmax(M, RED[128 + buf * 64 + v]);
                const bool ok = M > 0.0 && M < INFINITY;
                const int e = ok ? ilogb(M) : 0;
                const double sc = ldexp(1.0, -e);
                K += e;
#pragma unroll
                for (int r = 0; r < RJN; ++r) ec[r] *= sc;
              }
              double sum[RJN];
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                sum[r] = acc[0][r];
#pragma unroll
                for (int c = 1; c < NCH; ++c) sum[r] += acc[c][r];
              }
              STAMP(2);
              combine_sum<QL>(sum);
              STAMP(3);
#pragma unroll
              for (int r = 0; r < RJN; ++r) x[r] = sum[r] * ec[r];
              STAMP(4);
              if constexpr (MODE == MODE_FWD_STORE) {
#pragma unroll
                for (int r = 0; r < RJN; ++r) p.alpha[(c0 + t) * XR + jr[r]] = x[r];
              }
              STAMP(5);
            }
          }
        }
        if (MODE == MODE_FWD_LL && split != 0) {
          // half of a split block: the scaled vector and its exponent
          const int side = split < 0;
          if (q == 0) {
#pragma unroll
            for (int r = 0; r < RJN; ++r)
              if (jv[r]) p.svec[((int64_t)slot * 2 + side) * XR + jr[r]] = x[r];
          }
          if (tid == 0) p.sK[slot * 2 + side] = K;
        } else if constexpr (MODE == MODE_FWD_LL) {
          // log P = log(sum_j x_j) + K ln 2   (optimizer.py:160-162)
          double part = 0.0;
          if (q == 0) {
#pragma unroll
            for (int r = 0; r < RJN; ++r) part += jv[r] ? x[r] : 0.0;
          }
          part = wave_sum(part);
          if (l == 0) RED[256 + w] = part;
          lds_barrier();
          if (tid == 0) {
            double tot = 0.0;
#pragma unroll
            for (int v = 0; v < W; ++v) tot += RED[256 + v];
            p.loglik[blk] = log(tot) + (double)K * LN2;
          }
        }
      } else if constexpr (MODE == MODE_BWD) {
        // ------------- backward + posterior (optimizer.py:191-238)
        //   beta_{T-1} = 1;  beta_{t-1} = (beta_t * e_t) @ a  (vector @ a: the reference's form)
        //   post_t = alpha_t * beta_t / sum_j(alpha_t * beta_t)
        // Step s handles column t = T-1-s.  Staged rows of step s are read BEFORE the step's
        // barrier, so each tile is committed on the last step of the previous tile; the
        // unrolled tile keeps the periodic work branch-free like the forward sweep.
        double bt[RJN];
#pragma unroll
        for (int r = 0; r < RJN; ++r) bt[r] = jv[r] ? 1.0 : 0.0;
        double* sink = p.sink + l;  // padded states store here (never read)
        wait_vmem_all();
        for (int s0 = 0; s0 < T; s0 += TE) {
#pragma unroll
          for (int sub = 0; sub < TE; ++sub) {
            const int s = s0 + sub;
            if (s < T) {
              const int t = T - 1 - s;
              const int buf = sub & 1;  // s0 is even
              double* Xb = X + buf * (XS + 64);
              double qv[RJN], v[RJN], ps = 0.0;
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                qv[r] = staged(AST, s, jr[r]) * bt[r];  // padded states: 0 * 0
                ps += qv[r];
                v[r] = bt[r] * staged(EST, s, jr[r]);
                Xb[jx[r]] = v[r];
              }
              ps = row_sum<QL>(ps);  // the row's target-state groups
              if (row_leader) RED[buf * 64 + row16] = ps;
              const bool rescale = (sub & 7) == 0;
              if (rescale) {
                double mx = v[0];
#pragma unroll
                for (int r = 1; r < RJN; ++r) mx = fmax(mx, v[r]);
                mx = row_max<QL>(mx);
                if (row_leader) RED[128 + buf * 64 + row16] = mx;
              }
              if (sub == 0) ot.advance(s, tid);
              if (sub == TE - 1) stage_commit(s + 1);
              lds_barrier();
              if (sub == TE - 1) stage_issue(s + 1);
              double S = 0.0;
#pragma unroll
              for (int u = 0; u < NROW; ++u) S += RED[buf * 64 + u];
              const double rS = 1.0 / S;
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                double* dst = jv[r] ? p.post + (c0 + t) * n + jr[r] : sink;
                *dst = qv[r] * rS;
              }
              double sc = 1.0;
              if (rescale) {
                double M = RED[128 + buf * 64];
#pragma unroll
                for (int u = 1; u < NROW; ++u) M = fmax(M, RED[128 + buf * 64 + u]);
                if (M > 0.0 && M < INFINITY) sc = ldexp(1.0, -ilogb(M));
              }
              const double* xs = Xb + q * IQS;
              double acc[NCH][RJN];
#pragma unroll
              for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int r = 0; r < RJN; ++r) acc[c][r] = 0.0;
#pragma unroll
              for (int k = 0; k < IQ; ++k) {
                const double xi = xs[k];
#pragma unroll
                for (int r = 0; r < RJN; ++r) acc[k % NCH][r] = fma(xi, m[k][r], acc[k % NCH][r]);
              }
              double sum[RJN];
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                sum[r] = acc[0][r];
#pragma unroll
                for (int c = 1; c < NCH; ++c) sum[r] += acc[c][r];
              }
              combine_sum<QL>(sum);
#pragma unroll
              for (int r = 0; r < RJN; ++r) bt[r] = sum[r] * sc;
            }
          }
        }
      } else {
        // ------------- Viterbi (optimizer.py:305-333)
        //   omega_t[j] = max_i (omega_{t-1}[i] + log a_ij) + log e_j,  bp = first argmax.
        // Rounding is monotone, so max_i fl(z_i + c) = fl(max_i z_i + c): the chain takes
        // the max of z_i = omega_i + log a_ij over i != j (one add + one max per pair), the
        // diagonal z_j = omega_j + log a_jj is formed separately, and
        //   yd = fl(z_j + c), yo = fl(max_{i != j} z_i + c), omega_t[j] = max(yd, yo)
        // is bit-identical to the reference's value.  yd > yo means j is the unique maximum,
        // so bp(t, j) = j for certain: that is the stay flag.  Otherwise (a switch, or a tie
        // the first-max rule must break) the traceback recomputes bp(t, j) exactly.
        // What is stored, per 16-column tile k of the block (tile record tk0 + k, row
        // stride XR): the omega row of the tile's first column (a checkpoint the traceback
        // recomputes the tile's later rows from) and one 16-bit word of stay flags per
        // state (bit u = column 16k + u), written once per tile by the q == 0 lane of each
        // real state.
        static_assert(TE == VIT_TILE, "Viterbi checkpoints are one per staged tile");
        const int64_t tk0 = p.tile_off[blk];
        const int o0 = ot.get(0);
        double x[RJN];
#pragma unroll
        for (int r = 0; r < RJN; ++r) {
          x[r] = jv[r] ? p.init[o0 * n + jr[r]] : -INFINITY;
          if (q == 0 && jv[r]) p.alpha[tk0 * XR + jr[r]] = x[r];
        }
        wait_vmem_all();
        STAMP(-1);
        for (int t0 = 0; t0 < T; t0 += TE) {
          const int64_t rec = (tk0 + t0 / TE) * XR;  // this tile's checkpoint / flag record
          uint32_t bits[RJN];
#pragma unroll
          for (int r = 0; r < RJN; ++r) bits[r] = 0;
#pragma unroll
          for (int sub = 0; sub < TE; ++sub) {
            const int t = t0 + sub;
            if (t >= 1 && t < T) {
              DIAG_STEP();
              const int buf = sub & 1;  // t0 is even
              double* Xb = X + buf * (XS + 64);
#pragma unroll
              for (int r = 0; r < RJN; ++r) Xb[jx[r]] = x[r];
              double ec[RJN];
              if (sub != 0) {
#pragma unroll
                for (int r = 0; r < RJN; ++r) ec[r] = staged(EST, t, jr[r]);
              }
              if (sub == 0) {
                ot.advance(t, tid);
                stage_commit(t);
              }
              STAMP(0);
              lds_barrier();
              STAMP(1);
              if (sub == 0) {
                stage_issue(t);
#pragma unroll
                for (int r = 0; r < RJN; ++r) ec[r] = staged(EST, t, jr[r]);
              }
              const double* xs = Xb + q * IQS;
              // NCH independent max chains per target (k = c mod NCH)
              double bc[NCH][RJN];
#pragma unroll
              for (int c = 0; c < NCH; ++c) {
                const double xc = xs[c];
#pragma unroll
                for (int r = 0; r < RJN; ++r) bc[c][r] = xc + m[c][r];
              }
#pragma unroll
              for (int k = NCH; k < IQ; ++k) {
                const double xi = xs[k];
#pragma unroll
                for (int r = 0; r < RJN; ++r) bc[k % NCH][r] = fmax(bc[k % NCH][r], xi + m[k][r]);
              }
              double zo[RJN];
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                zo[r] = bc[0][r];
#pragma unroll
                for (int c = 1; c < NCH; ++c) zo[r] = fmax(zo[r], bc[c][r]);
              }
              STAMP(2);
              combine_max<QL>(zo);  // max over i != j, identical in the 8 lanes
              STAMP(3);
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                const double yd = (x[r] + ldiag[r]) + ec[r];
                const double yo = zo[r] + ec[r];
                bits[r] |= (uint32_t)(yd > yo) << sub;
                x[r] = fmax(yd, yo);
              }
              STAMP(4);
              if (sub == 0 && q == 0) {  // the tile's checkpoint row (t = t0 >= 16)
#pragma unroll
                for (int r = 0; r < RJN; ++r)
                  if (jv[r]) p.alpha[rec + jr[r]] = x[r];
              }
              if ((sub == TE - 1 || t == T - 1) && q == 0) {  // the tile's flag words
#pragma unroll
                for (int r = 0; r < RJN; ++r)
                  if (jv[r]) p.stay[rec + jr[r]] = (uint16_t)bits[r];
              }
              STAMP(5);
            }
          }
        }
        // last state = first argmax of omega_{T-1}  (optimizer.py:346)
        double bv = jv[0] ? x[0] : -INFINITY;
        int bj = jv[0] ? jr[0] : 0x7fffffff;
#pragma unroll
        for (int r = 1; r < RJN; ++r) {
          if (jv[r] && (x[r] > bv || (x[r] == bv && jr[r] < bj))) {
            bv = x[r];
            bj = jr[r];
          }
        }
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
      }
      if (urgent) __builtin_amdgcn_s_setprio(0);
    }  // T > 0
    lds_barrier();
  }
  DIAG_FLUSH();
}

template <int QL, int WV, int RJN, int IQ, int MODE>
__global__ void __launch_bounds__(64 * WV, (Occ<QL, WV, RJN, IQ, MODE>::value))
    sweep_kernel(SweepArgs p) {
  sweep_device<QL, WV, RJN, IQ, MODE>(p);
}

// ---------------------------------------------------------------------------------------
// Viterbi traceback (optimizer.py:336-354) over the checkpoint rows and stay flags of
// MODE_VIT.  One wave per block (longest first from a work counter).  Walking down from the
// last column with the current state s, the path stays in s as long as stay(t, s) holds:
// lane l reads s's flag word of tile k - l, so one load covers 1,024 columns, and the
// highest clear bit of the highest tile with one is the next column u to resolve.  There
// bp(u, s) is the reference's first argmax over i of (omega_{u-1}[i] + log a_is) +
// log e_s(u) (lane i, +64, +128; first-max reduction).  omega_{u-1} is rebuilt from the
// checkpoint of its tile by at most 15 steps of the Viterbi recursion into the wave's LDS
// rows, each value max_i (omega[i] + log a_ij) + log e_j — bit-identical to the sweep's
// max(yd, yo) because IEEE rounding is monotone — and kept for further switches in the
// same tile.
// ---------------------------------------------------------------------------------------
// LDS hand-off between lanes of one wave (the region is private to the wave)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

template <int G>  // state groups of 64 lanes: n <= 64 G
__global__ void __launch_bounds__(256) vit_trace_kernel(TraceArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int l = threadIdx.x & 63;
  const int n = p.n;
  // this wave's rows of one tile: row u = omega at column 16 * ctile + u
  double* rows = reinterpret_cast<double*>(smem) + (size_t)(threadIdx.x >> 6) * VIT_TILE * n;
  for (;;) {
    int bi = 0;
    if (l == 0) bi = atomicAdd(p.queue, 1);
    bi = uni(__shfl(bi, 0));
    if (bi >= p.nblocks) break;
    const int blk = uni(p.order[bi]);
    const int64_t c0 = p.off[blk];
    const int T = uni((int)(p.off[blk + 1] - c0));
    if (T <= 0) continue;  // no barrier in this kernel: a wave-uniform continue is safe
    const int64_t tk0 = p.tile_off[blk];
    uint8_t* path = p.path + c0;
    int s = uni((int)p.last_state[blk]);
    if (l == 0) path[T - 1] = (uint8_t)s;
    int t = T - 1;             // column whose state (s) is known
    int ctile = -1, cupto = -1;  // LDS rows hold columns 16 ctile .. cupto
    while (t >= 1) {
      const int k = t >> 4;
      const int kt = k - l;
      const uint32_t w = kt >= 0 ? (uint32_t)p.stay[(tk0 + kt) * p.xr + s] : 0xFFFFu;
      uint32_t mask = l == 0 ? (2u << (t & 15)) - 1u : 0xFFFFu;  // columns <= t only
      if (kt == 0) mask &= ~1u;  // column 0 has no step
      const uint32_t clear = ~w & mask;
      const uint64_t hit = __ballot(clear != 0);
      int u;  // highest column <= t with a clear flag (or the window's lowest column - 1)
      if (hit) {
        const int lf = __builtin_ctzll(hit);
        const uint32_t cw = (uint32_t)__shfl((int)clear, lf);
        u = 16 * (k - lf) + (31 - __builtin_clz(cw));
      } else {
        u = max(1, 16 * (k - 63)) - 1;
      }
      for (int c = u + l; c < t; c += 64) path[c] = (uint8_t)s;  // columns u+1..t stay
      t = u;
      if (!hit) continue;
      // column u: a switch or a tie; bp(u, s) from omega_{u-1}
      const int cc = u - 1;
      const int tt = cc >> 4;
      if (tt != ctile || cc > cupto) {
        int start = cupto + 1;
        if (tt != ctile) {
          const double* ck = p.ckpt + (tk0 + tt) * p.xr;
          for (int j = l; j < n; j += 64) rows[j] = ck[j];
          start = 16 * tt + 1;
          ctile = tt;
        }
        wave_lds_sync();
        for (int c = start; c <= cc; ++c) {
          const int sym = min((int)p.obs[c0 + c], 624);
          const double* prev = rows + (c - 1 - 16 * tt) * n;
          double* cur = rows + (c - 16 * tt) * n;
          const double* le = p.log_e + (int64_t)sym * n;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const int j = l + 64 * g;
            if (j < n) {
              double m0 = -INFINITY, m1 = -INFINITY;
              int i = 0;
#pragma unroll 4
              for (; i + 1 < n; i += 2) {
                m0 = fmax(m0, prev[i] + p.log_a[(int64_t)i * n + j]);
                m1 = fmax(m1, prev[i + 1] + p.log_a[(int64_t)(i + 1) * n + j]);
              }
              if (i < n) m0 = fmax(m0, prev[i] + p.log_a[(int64_t)i * n + j]);
              cur[j] = fmax(m0, m1) + le[j];
            }
          }
          wave_lds_sync();
        }
        cupto = max(cupto, cc);
      }
      const double* prow = rows + (cc - 16 * tt) * n;
      const int sym = min((int)p.obs[c0 + u], 624);
      const double le = p.log_e[(int64_t)sym * n + s];
      double best = -INFINITY;
      int bidx = l;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int i = l + 64 * g;
        if (i < n) {
          const double y = (prow[i] + p.log_a[(int64_t)i * n + s]) + le;
          if (g == 0 || y > best) {
            best = y;
            bidx = i;
          }
        }
      }
      wave_first_max(best, bidx);
      s = uni(bidx);
      if (l == 0) path[u - 1] = (uint8_t)s;
      t = u - 1;
    }
  }
}

// ---------------------------------------------------------------------------------------
// launch helpers: (RJN, IQ) configurations by state count
// ---------------------------------------------------------------------------------------
struct Cfg {
  int ql, w, rj, iq;  // lanes per target, waves, target states per lane, sources per lane
};
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
    {8, 3, 3, 9}, {8, 6, 3, 17}};
static constexpr int kNarrow = 7;  // entries 0..6
[[maybe_unused]] static constexpr int kNumCfgs = (int)(sizeof kCfgs / sizeof kCfgs[0]);

static int cfg_xr(int c) { return (64 / kCfgs[c].ql) * kCfgs[c].w * kCfgs[c].rj; }
static bool fits(int c, int n) { return cfg_xr(c) >= n && kCfgs[c].ql * kCfgs[c].iq >= n; }

// Measured on the (5,5) model (N = 70), 10 Mbp: the forward log-likelihood
// sweep runs fastest on three waves with three targets per lane (configuration 20), the
// posterior sweeps too, Viterbi on the one-target-per-lane kernel (9); other sizes below.
static int pick_cfg(int n, int mode) {
#ifdef ITR_DIAG
  // diagnostic/experiment build only: force a configuration (ITR_VIT_CFG: Viterbi only)
  const char* force = (mode == MODE_VIT && getenv("ITR_VIT_CFG")) ? getenv("ITR_VIT_CFG")
                                                                  : getenv("ITR_SWEEP_CFG");
  if (force) {
    const int c = atoi(force);
    if (c >= 0 && c < kNumCfgs && fits(c, n)) return c;
  }
#endif
  // (posterior sweeps at N = 70 on configuration 20: 465 -> 496 M columns/s,
  // scripts/gpu_cfgsmall.sh)
  if (n > 64 && n <= 72) return mode == MODE_VIT ? 9 : 20;
  // Viterbi at 32 < N <= 64 on eight waves, one target per lane ((4,4) model, N = 46:
  // 7.3 -> 6.2 ms)
  if (n > 32 && n <= 64 && mode == MODE_VIT) return 8;
  // measured on the (7,7) model (N = 133, 10 Mbp, scripts/gpu_cfg133.sh): six waves with
  // three targets per lane for the probability sweeps (posterior 146 -> 175 M columns/s),
  // nine waves with four lanes per target for Viterbi (40.7 -> 26.0 ms)
  if (n > 128 && n <= 144) return mode == MODE_VIT ? 17 : 21;
  // introgression (5,5) model, N = 95 (scripts/gpu_cfg95.sh): Viterbi on six waves with four
  // lanes per target (11.9 -> 11.0 ms); the probability sweeps keep configuration 3
  if (n > 72 && n <= 96 && mode == MODE_VIT) return 16;
  for (int c = 0; c < kNarrow; ++c)
    if (fits(c, n)) return c;
  return -1;
}

static size_t lds_bytes(int cfg, int mode) {
  const int w = kCfgs[cfg].w, iq = kCfgs[cfg].iq;
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

template <int MODE>
static hipError_t dispatch(int cfg, bool launch, const SweepArgs* a, int grid, size_t lds,
                           hipStream_t st, int* occ) {
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
#ifdef ITR_DIAG
  // diagnostic/experiment build only: resident workgroups per CU
  const char* pcu = (mode == MODE_VIT && getenv("ITR_VIT_PER_CU")) ? getenv("ITR_VIT_PER_CU")
                                                                   : getenv("ITR_PER_CU");
  if (pcu && atoi(pcu) > 0) g.per_cu = atoi(pcu);
#endif
  return g;
}

hipError_t launch_sweep(int mode, const SweepGeometry& g, int grid, const SweepArgs& a,
                        hipStream_t st) {
  int occ = 0;
  return dispatch_mode(mode, g.iq, true, &a, grid, g.lds, st, &occ);
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
