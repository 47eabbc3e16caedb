// valu_sweep.h — the VALU (FP64 FMA / add-max) sweep tasks shared by the VALU-only kernels
// (hmm_sweeps.hip) and the matrix-core hybrid kernels (mfma_sweeps.hip).  Device code only.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

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
// a wave-uniform 64-bit value into scalar registers (a per-lane copy of a uniform offset
// makes every address built from it a 64-bit VGPR pair: register pressure and spills)
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

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

// Sum / maximum over the four 16-lane rows of a wave whose lanes hold their row's value:
// wave-uniform, from four lane reads (no LDS round trip)
__device__ __forceinline__ double lane_f64(double v, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), lane),
                          __builtin_amdgcn_readlane(__double2loint(v), lane));
}
__device__ __forceinline__ double rows4_sum(double v) {
  return (lane_f64(v, 0) + lane_f64(v, 16)) + (lane_f64(v, 32) + lane_f64(v, 48));
}
__device__ __forceinline__ double rows4_max(double v) {
  return fmax(fmax(lane_f64(v, 0), lane_f64(v, 16)), fmax(lane_f64(v, 32), lane_f64(v, 48)));
}
// 1 / s by the hardware reciprocal and one Newton step (a few ulps; the posterior's
// normalisation, whose bar is 1e-8 relative, instead of the ten-instruction IEEE division on
// the backward sweep's step)
__device__ __forceinline__ double recip_nr(double s) {
  const double r = __builtin_amdgcn_rcp(s);
  return fma(fma(-s, r, 1.0), r, r);
}
// pairwise sum / maximum of N consecutive values (independent LDS reads, log-depth chain)
template <int N>
__device__ __forceinline__ double tree_sum(const double* a) {
  if constexpr (N == 1) {
    return a[0];
  } else {
    return tree_sum<N / 2>(a) + tree_sum<N - N / 2>(a + N / 2);
  }
}
template <int N>
__device__ __forceinline__ double tree_max(const double* a) {
  if constexpr (N == 1) {
    return a[0];
  } else {
    return fmax(tree_max<N / 2>(a), tree_max<N - N / 2>(a + N / 2));
  }
}

// Stores through a wave-uniform base as a buffer resource (base and byte bound in SGPRs):
// the per-lane part is one 32-bit byte offset instead of a 64-bit address pair, and a lane
// whose offset is kOffNone (past the bound) stores nothing, without a branch.
constexpr uint32_t kOffNone = 0xFFFFFFF0u;
typedef unsigned int itr_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// voff: the lane's byte offset (VGPR); soff: a wave-uniform byte offset (SGPR)
__device__ __forceinline__ void buf_store_f64(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                              uint32_t soff, double v) {
  itr_u32x2 d;
  d.x = (unsigned)__double2loint(v);
  d.y = (unsigned)__double2hiint(v);
  __builtin_amdgcn_raw_buffer_store_b64(d, r, voff, soff, 0);
}
__device__ __forceinline__ void buf_store_u16(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                              uint32_t soff, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, r, voff, soff, 0);
}

// LDS hand-off between lanes of one wave (the region is private to the wave): a wave's LDS
// instructions execute in order, so this costs no instruction; it keeps the compiler from
// moving the reads above the writes or forwarding values around them
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// One posterior row from stored alpha and beta rows, by one wave (lane l: states l, l + 64,
// l + 128; n <= 192): alpha * beta / sum_j alpha_j beta_j, the backward sweep's expression
// (optimizer.py:228-238).  post_combine_kernel and the backward hybrid launch's combine tasks.
__device__ __forceinline__ void post_combine_column(int n, int xr, const double* a,
                                                    const double* b, double* dst, int l) {
  (void)xr;
  const double q0 = l < n ? a[l] * b[l] : 0.0;
  const double q1 = l + 64 < n ? a[l + 64] * b[l + 64] : 0.0;
  const double q2 = l + 128 < n ? a[l + 128] * b[l + 128] : 0.0;
  const double S = wave_sum((q0 + q1) + q2);
  const double rS = 1.0 / S;
  if (l < n) dst[l] = q0 * rS;
  if (l + 64 < n) dst[l + 64] = q1 * rS;
  if (l + 128 < n) dst[l + 128] = q2 * rS;
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


// LDS of one VALU task (sweep_task's carve below)
template <int QL, int WV, int RJN, int IQ, int MODE>
struct ValuSweep {
  static constexpr int IQS = IQ + (IQ & 1), XS = QL * IQS, XR = WV * (64 / QL) * RJN;
  static constexpr int TE = tile_cols(MODE, XR), TB = 64 * WV;
  static constexpr size_t lds_bytes = (size_t)2 * (XS + 64) * 8 + 5 * 64 * 8 +
                                      (size_t)(MODE == MODE_BWD ? 2 : 1) * 2 * TE * XR * 8 +
                                      32 * 4 + (size_t)2 * TB * 2;
};

// One task of the VALU sweep: a whole block, or (MODE_FWD_LL) half of a split block, run by
// the whole workgroup.  `bi` indexes p.tasks (MODE_FWD_LL) or p.order.  Every lane-dependent
// quantity, the matrix slice included, is set up per task, and the LDS region `smem` is
// (re)initialised per task: the matrix-core kernels (mfma_sweeps.hip) interleave these tasks
// with their own in the same workgroup and the same LDS.
template <int QL, int WV, int RJN, int IQ, int MODE>
__device__ __forceinline__ void sweep_task(const SweepArgs& p, unsigned char* smem, int bi) {
  constexpr int W = WV;       // wavefronts per workgroup
  constexpr int TB = 64 * W;  // threads per workgroup
  constexpr int IQS = IQ + (IQ & 1);  // 16-byte aligned source ranges in LDS
  constexpr int XS = QL * IQS;        // published vector length
  constexpr int GW = 64 / QL;         // target groups per wave
  constexpr int JW = GW * RJN;        // target states per wave
  constexpr int XR = W * JW;          // padded target states per workgroup
  constexpr int TE = tile_cols(MODE, XR);
  constexpr int NCH = IQ >= 6 ? 3 : (IQ >= 2 ? 2 : 1);  // independent chains per target
  const int n = p.n;
  const int tid = threadIdx.x;
  const int w = uni(tid >> 6);
  const int l = tid & 63;
  const int q = l & (QL - 1);
  const int jl = l / QL;

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

  // published entries of states >= n are never written: 0 for the probability sweeps
  // (contributes nothing), -inf for Viterbi (never a maximum)
  const double pad = (MODE == MODE_VIT) ? -INFINITY : 0.0;
  for (int i = tid; i < 2 * (XS + 64); i += TB) X[i] = pad;
  lds_barrier();

  RowStage<W, XR, TE> est;
  RowStage<W, XR, TE> ast;
  (void)ast;
  (void)SBLK;
  DIAG_DECL
  {
    // forward log-likelihood tasks (itr_plan_create): {block, split, slot}; split 0 = the
    // whole block, +m = columns [0, m) forward, -m = the backward half (see below)
    const int32_t* td = (MODE == MODE_FWD_LL) ? p.tasks + 3 * bi : nullptr;
    const int blk = uni(td ? td[0] : p.order[bi]);
    const int split = td ? uni(td[1]) : 0;
    const int slot = td ? uni(td[2]) : 0;
    int64_t c0 = p.off[blk];
    int Tb = uni((int)(p.off[blk + 1] - c0));
    // a block split at column lo (hybrid posterior, p.sub_lo): the beta task takes columns
    // [lo, T), the posterior task columns [0, lo] — each as a block of its own
    const int lo = ((MODE == MODE_BWD || MODE == MODE_BETA) && p.sub_lo)
                       ? uni((int)p.sub_lo[blk]) : 0;
    if (lo > 0) {
      if (MODE == MODE_BETA || p.beta) {
        c0 += lo;
        Tb -= lo;
      } else {
        Tb = lo + 1;
      }
    }
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
      {
        // the slice of a (log a for Viterbi; a^T for a backward half of a split forward
        // task), loaded for every task: a few L2 loads against thousands of steps
        const double* mp = (MODE == MODE_FWD_LL && split < 0) ? p.matT : p.mat;
#pragma unroll
        for (int k = 0; k < IQ; ++k) {
          const int i = q * IQ + k;
#pragma unroll
          for (int r = 0; r < RJN; ++r) {
            m[k][r] = (i < n && jv[r]) ? mp[(int64_t)i * n + jr[r]] : 0.0;
            if (MODE == MODE_VIT && i == jr[r]) m[k][r] = -INFINITY;
          }
        }
      }
      ObsTiles ot{OBS, p.obs + c0, Tb,
                  (MODE == MODE_BWD || MODE == MODE_BETA || split < 0) ? -1 : +1, TB, 0};
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
      // MODE_BWD with p.beta (the posterior's concurrent split) stores beta rows and needs no
      // forward rows
      const bool need_alpha = MODE == MODE_BWD && !p.beta;
      if (need_alpha) {
        ast.issue(p.alpha, XR, XR, tid, 0, fwd_row);
        ast.commit(AST, tid);
        ast.issue(p.alpha, XR, XR, tid, TE, fwd_row);
      }
      // a new staged tile starts at step s: commit it before the step's barrier ...
      auto stage_commit = [&](int s) {
        if (s >= TE && (s & (TE - 1)) == 0) {
          const int slot = (s / TE) & 1;
          est.commit(EST + slot * TE * XR, tid);
          if (need_alpha) ast.commit(AST + slot * TE * XR, tid);
        }
      };
      // ... and request the one after it behind the barrier
      auto stage_issue = [&](int s) {
        if (s >= TE && (s & (TE - 1)) == 0) {
          est.issue(p.emit, n, n, tid, s + TE, sym_row);
          if (need_alpha) ast.issue(p.alpha, XR, XR, tid, s + TE, fwd_row);
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
              if (rescale) {  // the wave's maximum of x_{t-1} (padded states hold 0)
                double mx = x[0];
#pragma unroll
                for (int r = 1; r < RJN; ++r) mx = fmax(mx, x[r]);
                mx = rows4_max(row_max<QL>(mx));
                if (l == 0) RED[128 + buf * 64 + w] = mx;
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
                const double M = tree_max<W>(RED + 128 + buf * 64);
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
      } else if constexpr (MODE == MODE_BWD || MODE == MODE_BETA) {
        // ------------- backward + posterior (optimizer.py:191-238)
        //   beta_{T-1} = 1;  beta_{t-1} = (beta_t * e_t) @ a  (vector @ a: the reference's form)
        //   post_t = alpha_t * beta_t / sum_j(alpha_t * beta_t)
        // Step s handles column t = T-1-s.  Staged rows of step s are read BEFORE the step's
        // barrier, so each tile is committed on the last step of the previous tile; the
        // unrolled tile keeps the periodic work branch-free like the forward sweep.
        double bt[RJN];
#pragma unroll
        for (int r = 0; r < RJN; ++r) {
          // a split block's posterior task starts from the stored beta_lo (rescaled like any
          // beta row: the posterior is invariant to a power-of-two factor per column)
          if (MODE == MODE_BWD && lo > 0 && !p.beta)
            bt[r] = jv[r] ? p.beta_in[p.beta_off[blk] * XR + jr[r]] : 0.0;
          else
            bt[r] = jv[r] ? 1.0 : 0.0;
        }
        // posterior rows through a buffer resource on the block's rows: lane offset = its
        // state (padded states: out of range, nothing stored), row offset in a scalar register
        // (blocks whose rows span 4 GiB or more store through 64-bit addresses instead)
        const bool wide = (int64_t)T * n * 8 >= (int64_t)kOffNone;
        const __amdgpu_buffer_rsrc_t rpost =
            buf_rsrc(p.post && !wide ? p.post + c0 * n : p.sink,
                     p.post && !wide ? (uint32_t)((int64_t)T * n * 8) : 0u);
        uint32_t voff[RJN];
#pragma unroll
        for (int r = 0; r < RJN; ++r) voff[r] = jv[r] ? (uint32_t)jr[r] * 8u : kOffNone;
        wait_vmem_all();
        // the staged emission / forward values of a step are read from LDS one step ahead
        // (after the previous step's barrier): the published vector v = beta * e needs them
        // before the barrier, where a read issued on the spot would stall the wave
        double ecur[RJN], acur[RJN];
#pragma unroll
        for (int r = 0; r < RJN; ++r) {
          ecur[r] = staged(EST, 0, jr[r]);
          acur[r] = need_alpha ? staged(AST, 0, jr[r]) : 0.0;
        }
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
                v[r] = bt[r] * ecur[r];
                Xb[jx[r]] = v[r];
              }
              // per-wave partials (the wave's four rows combined by lane reads): after the
              // barrier only W values are combined, by a log-depth tree, and after the
              // matrix product has been issued (a 4W-long chain of dependent LDS reads and
              // adds before it cost more than the product itself at N = 133)
              if (need_alpha) {
#pragma unroll
                for (int r = 0; r < RJN; ++r) {
                  qv[r] = acur[r] * bt[r];  // padded states: 0 * 0
                  ps += qv[r];
                }
                ps = rows4_sum(row_sum<QL>(ps));  // the wave's target states
                if (l == 0) RED[buf * 64 + w] = ps;
              }
              const bool rescale = (sub & 7) == 0;
              if (rescale) {
                double mx = v[0];
#pragma unroll
                for (int r = 1; r < RJN; ++r) mx = fmax(mx, v[r]);
                mx = rows4_max(row_max<QL>(mx));
                if (l == 0) RED[128 + buf * 64 + w] = mx;
              }
              if (sub == 0) ot.advance(s, tid);
              if (sub == TE - 1) stage_commit(s + 1);
              lds_barrier();
              if (sub == TE - 1) stage_issue(s + 1);
              // next step's staged values (its tile was committed before this barrier)
#pragma unroll
              for (int r = 0; r < RJN; ++r) {
                ecur[r] = staged(EST, s + 1, jr[r]);
                if (need_alpha) acur[r] = staged(AST, s + 1, jr[r]);
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
              if (MODE == MODE_BETA || p.beta) {
                // concurrent split (launch_post_split, the hybrid's beta tasks): this block's
                // forward rows are being written by another workgroup, so store beta_t for
                // post_combine instead
                const int64_t brow = (p.beta_off[blk] + t) * XR;
#pragma unroll
                for (int r = 0; r < RJN; ++r) p.beta[brow + jr[r]] = bt[r];
              } else {
                const double rS = recip_nr(tree_sum<W>(RED + buf * 64));
                if (!wide) {
                  const uint32_t row = (uint32_t)t * (uint32_t)n * 8u;
#pragma unroll
                  for (int r = 0; r < RJN; ++r) buf_store_f64(rpost, voff[r], row, qv[r] * rS);
                } else {
#pragma unroll
                  for (int r = 0; r < RJN; ++r)
                    if (jv[r]) p.post[(c0 + t) * n + jr[r]] = qv[r] * rS;
                }
              }
              double sc = 1.0;
              if (rescale) {
                const double M = tree_max<W>(RED + 128 + buf * 64);
                if (M > 0.0 && M < INFINITY) sc = ldexp(1.0, -ilogb(M));
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
              // waves whose targets are all padding (the Viterbi hybrid runs this task on a
              // wider workgroup than the block needs) skip the arithmetic: a uniform branch
              if (w * JW < n) {
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
              }  // w * JW < n
              STAMP(4);
              if (sub == 0 && q == 0) {  // the tile's checkpoint row (t = t0 >= 16)
#pragma unroll
                for (int r = 0; r < RJN; ++r)
                  if (jv[r]) p.alpha[rec + jr[r]] = x[r];
              }
              STAMP(5);
            }
          }
          // the tile's flag words, once per tile (bits of columns past the block's end are
          // never read by the traceback)
          if (q == 0) {
#pragma unroll
            for (int r = 0; r < RJN; ++r)
              if (jv[r]) p.stay[rec + jr[r]] = (uint16_t)bits[r];
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

// The VALU-only persistent sweep: every workgroup pulls tasks longest first.
template <int QL, int WV, int RJN, int IQ, int MODE>
__device__ __forceinline__ void sweep_device(const SweepArgs& p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot;
  for (;;) {
    if (threadIdx.x == 0) qslot = atomicAdd(p.queue, 1);
    lds_barrier();
    const int bi = uni(qslot);
    lds_barrier();
    if (bi >= p.nblocks) break;
    sweep_task<QL, WV, RJN, IQ, MODE>(p, smem, bi);
  }
}

}  // namespace itr
