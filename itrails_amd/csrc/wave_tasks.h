// wave_tasks.h — the per-wavefront sweep tasks of MI355X (gfx950): one Viterbi block per
// wavefront (vit_wave_task) and one group of four forward tasks per wavefront on the matrix
// cores (fwd_wave_task).  Device code only; kernels in wave_sweeps.hip run them from one
// queue each or from one mixed queue.  Each task sets up its own registers (matrix slice)
// and its wave's LDS region, so the two kinds interleave freely in one persistent launch.
//
// ---- Viterbi, one block per wavefront ----------------------------------------------------
//
// One wavefront decodes a whole block on its own (no workgroup barrier; a wave's LDS
// instructions execute in order), by one of two steps chosen per block (vit_wave_block):
//
// Full scan (vit_wave_task_full, blocks at least p.prune_len long): lane l = 8 q + g holds,
// in VGPRs, log a between sources IQ q .. IQ q + IQ - 1 and targets IQ g .. IQ g + IQ - 1,
// forms 9 partial maxima, writes them to the wave's partial table in LDS and finalises
// target l (and, lanes 0-7, 64 + l) from its 8 partials: ~181 VALU instructions per column,
// the shortest dependent chain — the step for the blocks whose latency sets the makespan.
//
// Bound-pruned step (vit_wave_task, the shorter blocks: fewer instructions per column, a
// longer chain).  The states are laid out in 8 IQ slots (IQ = 9: 72 slots for N = 65..72),
// slot s = IQ g + r holding the state VSLOT[s] (the model's slot order, capi.cpp
// vit_slot_tables).  Lane l = 8 g + q holds, in VGPRs, log a between the source slots of
// chunk q (IQ q .. IQ q + IQ - 1) and the target slots of group g, and owns target slot
// IQ g + q (A) and, for q = 0, target slot IQ g + IQ - 1 (B).
// With Omega = max_i omega_i (a wave-wide maximum) and
// M_j = max_{i != j} log a_ij (per model), rounding is monotone, so for every i != j
//   fl(fl(omega_i + log a_ij) + log e_j) <= fl(fl(Omega + M_j) + log e_j) =: B_j.
// A target whose stay score yd = fl(fl(omega_j + log a_jj) + log e_j) exceeds B_j has
// yd > yo = max_{i != j} fl(fl(omega_i + log a_ij) + log e_j): its stay flag is 1 and
// omega_t[j] = yd, bit for bit what the full scan gives.  Only the targets that fail the
// test need the scan over all sources: for each target column r in which any group has a
// failing target (a wave-uniform test on the ballot), the 8 lanes of every group form
// max_k(omega + log a) over their source chunk for target IQ g + r and combine it by three
// DPP steps; the owner takes its value.  On the (5,5) model, the bench workload (N = 70),
// 84 % of the (column, target) pairs pass and 43 % of the columns need no scan at all;
// with the slots ordered by how often a state fails (most often: column r = 0), a column
// scans 2.2 target columns on average instead of 9.
//
// Outputs are those of the VALU sweep — the omega row of every 16-column tile's first column,
// 16-bit stay-flag words, the last column's first argmax (by state index) — so the
// traceback (trace.h) is shared and paths are bit-identical whichever step ran.  The
// emission rows (padded to 8 IQ; slot order for the pruned step) are staged 8 columns at a
// time into the wave's LDS ring by direct-to-LDS loads.  Two waves share a SIMD; itr_viterbi
// gives the longest blocks to the 9-wave VALU layout on a reserved set of CUs and this
// kernel the rest (capi.cpp); blocks at least p.prio_len long run at raised
// wave priority.
//
// ---- forward log-likelihood, four tasks per wavefront on the matrix cores ----------------
//
// The workgroup-wide matrix-core sweep (mfma_sweeps.hip) spreads a group's target tiles over
// NT waves that meet at a workgroup barrier every column; here ONE wave owns the whole step:
// its lanes hold the complete transition matrix in the B-operand layout of
// v_mfma_f64_4x4x4_4b_f64 (NT x NK doubles per lane, 90 at N = 70), so a column step of four
// blocks is NT x NK MFMAs with NT independent accumulator chains and no barrier, and the
// vectors go through the wave's own LDS (in-order within a wave).  Two such waves per SIMD
// keep the matrix pipe fed while the partner runs its epilogue.  This is the throughput form
// for the bulk of short blocks (a group steps at ~1.5 us per column under full load); the
// longest blocks stay on the low-latency workgroup layouts.
//
// Operand layout (probed, scripts/micro/mfma4_layout.hip): sub-product g = (lane >> 2) & 3;
// A row lane & 3, k lane >> 4; B column lane & 3, k lane >> 4; D row lane >> 4, column lane & 3.
// Rows = the group's four blocks; MFMA (w, s) contracts sources i = (lane >> 4) NK + s with
// targets 16 w + (lane & 15): lane l ends a step holding x_t of block l >> 4 at the NT targets
// 16 w + (l & 15), and reads x_{t-1} of block l & 3 at sources (l >> 4) NK + s, s < NK (one
// contiguous run: NK / 2 ds_read_b128).
//
// Per column: x_t = (x_{t-1} @ a) * e_t (a^T for the textbook backward half of a split block,
// whose last step multiplies by a row of ones: row 625 of the padded table), exact 2^-k
// rescale every 8 columns (the row maximum by a 16-lane DPP reduction: a DPP row is one
// block), the exponent kept as an integer; outputs as the other forward sweeps: log P of
// whole blocks, the scaled vector and exponent of split halves (fwd_split_combine_kernel).
// Emission rows arrive HT columns at a time by direct-to-LDS loads from the padded table;
// observed symbols 64 columns at a time through the wave's LDS ring.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sweeps.h"
#include "trace.h"
#include "valu_sweep.h"

namespace itr {

// The lane index, opaque to loop-invariant code motion: a task's lane-dependent setup
// (slots, offsets, matrix slices) is rebuilt per task instead of hoisted out of the
// persistent task loop, where it would stay live across the other tasks' bodies
__device__ __forceinline__ int lane_id_fresh() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}

template <int IQ>
struct WaveVit {
  static_assert(IQ == 9, "8 A slots and one B slot per target group");
  static constexpr int XRW = 8 * IQ;                  // slots
  static constexpr int IQS = IQ + (IQ & 1);           // 16-byte aligned source chunks
  static constexpr int XN = 8 * IQS;                  // published vector slots
  static constexpr int HT = 8;   // columns per staged emission half-tile
  // a half-tile of emission rows [HT][XRW] arrives by NI direct-to-LDS loads of 16 bytes per
  // lane (1 KiB each); the buffer is rounded up to whole loads
  static constexpr int NI = (HT * XRW + 127) / 128, EB = 128 * NI;
  static_assert(XRW % 2 == 0, "16-byte pieces must not cross a row");
  // per-wave LDS (doubles): published vector + 64 sink slots, emission ring [2], symbol ring
  // [2][64] (uint16), the lanes' log a of target column IQ - 1 [IQ][64] (out of VGPRs: that
  // column, the B slots, is scanned least often)
  static constexpr int LX = XN + 64, LE = 2 * EB, LS = 2 * 64 / 4, LM = IQ * 64;
  static constexpr int WL = LX + LE + LS + LM;
};

// X row stride (doubles) with conflict-free ds_read_b128 A-operand reads: lane l reads row
// l & 3 at offset (l >> 4) NK; in each of the instruction's four 16-lane groups the distinct
// (row, offset) pairs must start on distinct 4-bank ranges of the 64 banks
constexpr bool xs_ok(int xs, int nk) {
  const int groups[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                             {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                             {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                             {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  for (int g = 0; g < 4; ++g)
    for (int a = 0; a < 16; ++a)
      for (int b = 0; b < 16; ++b) {
        const int la = groups[g][a], lb = groups[g][b];
        const int da = 2 * ((la & 3) * xs + (la >> 4) * nk), db = 2 * ((lb & 3) * xs + (lb >> 4) * nk);
        if (da == db) continue;  // same address: broadcast
        const int d = ((da - db) % 64 + 64) % 64;
        if (d < 4 || d > 60) return false;
      }
  return true;
}
constexpr int pick_xs(int minw, int nk) {
  for (int xs = minw + (minw & 1); xs < minw + 128; xs += 2)
    if (xs_ok(xs, nk)) return xs;
  return minw + (minw & 1);
}

template <int NT, int NK>
struct WF {
  static constexpr int ER = 16 * NT;   // padded targets = width of the padded emission table
  static constexpr int KP = 4 * NK;    // padded sources
  static constexpr int XS = pick_xs(ER > KP ? ER : KP, NK);
  static constexpr int HT = 2;         // columns per staged emission half-tile
  static constexpr int PIECES = HT * 4 * ER / 2;  // 16-byte pieces per half-tile
  static constexpr int NI = (PIECES + 63) / 64, EB = 128 * NI;
  // per-wave LDS (doubles): X [4][XS], emission ring [2][EB], symbols [2][4][64] (uint16),
  // the rows' final vectors [4][ER] (captured when a row completes)
  static constexpr int LX = 4 * XS, LE = 2 * EB, LS = 2 * 4 * 64 / 4, LF = 4 * ER;
  static constexpr int WL = LX + LE + LS + LF;
  static_assert(NK % 2 == 0, "A operands are read two at a time");
  static_assert(ER % 2 == 0, "16-byte pieces must not cross an emission row");
};

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ double row16_max_w(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  return fmax(v, dpp_f64<0x128>(v));
}
__device__ __forceinline__ double row16_sum_w(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  return v + dpp_f64<0x128>(v);
}

// The block's traceback by the wave that swept it (VitArgs.path non-null): its checkpoint
// rows and flag words were stored by this wave's buffer stores, so they are made visible to
// its own loads first (release: wait for the stores; acquire: drop the vector L1's lines),
// and the wave's LDS region is free for the traceback's tile rows once the last staging DMA
// has landed (the release waits for it too).
template <int XRW>
__device__ __forceinline__ void vit_wave_trace(const VitArgs& p, double* wl, int blk, int s) {
  static_assert(VIT_TILE * XRW <= 144 + 2 * 640, "the tile rows fit the wave's LDS region");
  if (p.path == nullptr) return;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  TraceArgs ta{};
  ta.n = p.n;
  ta.xr = p.xr;
  ta.off = p.off;
  ta.tile_off = p.tile_off;
  ta.obs = p.obs;
  ta.log_a = p.la;
  ta.log_e = p.log_e;
  ta.ckpt = p.ckpt;
  ta.stay = p.stay;
  ta.path = p.path;
  trace_block<(XRW + 63) / 64>(ta, wl, blk, s);
}

// maximum over the wave, uniform (every lane's value counts)
__device__ __forceinline__ double wave_max_u(double v) {
  v = fmax(v, dpp_f64<DPP_Q1>(v));
  v = fmax(v, dpp_f64<DPP_Q2>(v));
  v = fmax(v, dpp_f64<DPP_HM>(v));
  v = fmax(v, dpp_f64<DPP_R8>(v));
  return rows4_max(v);
}

template <int IQ>
__device__ __forceinline__ void vit_wave_task(const VitArgs& p, double* wl, int blk) {
  using C = WaveVit<IQ>;
  constexpr int IQS = C::IQS, XN = C::XN, HT = C::HT, NI = C::NI, EB = C::EB, XRW = C::XRW;
  const int l = lane_id_fresh(), g = l >> 3, q = l & 7;
  const int n = p.n;
  const int64_t xr = p.xr;
  double* X = wl;
  double* EST = X + C::LX;
  uint16_t* SYM = reinterpret_cast<uint16_t*>(EST + C::LE);
  double* M8 = EST + C::LE + C::LS;

  // owned target slots and their states (-1: padding)
  const int slA = IQ * g + q, slB = IQ * g + IQ - 1;
  const int stA = p.slot_state[slA];
  const int stB = q == 0 ? p.slot_state[slB] : -1;
  const bool inA = stA >= 0, inB = stB >= 0;
  // log a slice: source slots IQ q + k, target slots IQ g + r (r < IQ - 1 in VGPRs, r = IQ - 1
  // in M8); the diagonal stays out
  double m[IQ][IQ - 1];
#pragma unroll
  for (int k = 0; k < IQ; ++k) {
    const int si = p.slot_state[IQ * q + k];
#pragma unroll
    for (int r = 0; r < IQ; ++r) {
      const int sj = p.slot_state[IQ * g + r];
      const double v = (si >= 0 && sj >= 0 && si != sj) ? p.la[(int64_t)si * n + sj] : -INFINITY;
      if (r < IQ - 1)
        m[k][r] = v;
      else
        M8[k * 64 + l] = v;
    }
  }
  const double ldA = inA ? p.la[(int64_t)stA * n + stA] : -INFINITY;
  const double ldB = inB ? p.la[(int64_t)stB * n + stB] : -INFINITY;
  const double mA = inA ? p.slot_m[slA] : -INFINITY;
  const double mB = inB ? p.slot_m[slB] : -INFINITY;
  const int xiA = g * IQS + q;                          // X positions (B of q > 0: a sink)
  const int xiB = q == 0 ? g * IQS + IQ - 1 : XN + l;
  for (int i = l; i < C::LX; i += 64) X[i] = -INFINITY;

  const int64_t c0 = uni64(p.off[blk]);
  const int T = uni((int)(p.off[blk + 1] - c0));
  if (T > 0) {  // (no `continue` in this loop, same reason)
    const bool urgent = T >= p.prio_len;
    if (urgent) __builtin_amdgcn_s_setprio(3);
    const uint16_t* ob = p.obs + c0;
    // raw symbol loads; the clamp into the alphabet (memory safety only) is applied when a
    // chunk is committed to SYM, 64 columns after its load was issued (a clamp right at
    // the load would make the wave wait for it there)
    auto symg = [&](int s) -> int { return (int)ob[min(s, T - 1)]; };
    auto clamp_sym = [](int v) -> uint16_t { return (uint16_t)min(v, 624); };
    // symbols: chunks of 64 columns, two resident in SYM, the next one in flight
    SYM[l] = clamp_sym(symg(l));
    SYM[64 + l] = clamp_sym(symg(64 + l));
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
        const double* src = p.lew_p;
        if (e < HT * XRW) src += (int64_t)sym(h * HT + e / XRW) * XRW + e % XRW;
        __builtin_amdgcn_global_load_lds(
            src, (__attribute__((address_space(3))) void*)(d + 128 * i), 16, 0, 0);
      }
    };
    auto stage_wait = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
    const int o0 = sym(0);
    double xA = inA ? p.lpie[o0 * n + stA] : -INFINITY;
    double xB = inB ? p.lpie[o0 * n + stB] : -INFINITY;
    X[xiA] = xA;
    X[xiB] = xB;
    const int64_t tk0 = uni64(p.tile_off[blk]);
    // this block's checkpoint rows and flag words (tiles x xr records from tile tk0, by
    // state), stored through buffer resources: lane part = the state, uniform part = the
    // tile's record; a lane without a state stores out of bounds (nothing)
    const uint32_t nrec = (uint32_t)((T + VIT_TILE - 1) / VIT_TILE * xr);
    const __amdgpu_buffer_rsrc_t rck = buf_rsrc(p.ckpt + tk0 * xr, nrec * 8);
    const __amdgpu_buffer_rsrc_t rst = buf_rsrc(p.stay + tk0 * xr, nrec * 2);
    const uint32_t vA = inA ? (uint32_t)stA : kOffNone / 8, vB = inB ? (uint32_t)stB : kOffNone / 8;
    buf_store_f64(rck, vA * 8, 0, xA);
    buf_store_f64(rck, vB * 8, 0, xB);
    stage_issue(0);
    stage_wait();
    stage_issue(1);
    wave_lds_sync();
    // Stores are issued between a staging wait and the next staging issue: the checkpoint
    // row of a tile's first column at the following half-tile boundary, a tile's flag
    // words at the next tile's first boundary (or after the block).  A store issued just
    // before a vmcnt(0) would be waited for there.
    uint32_t pbA = 0, pbB = 0;
    int prec = -1;        // flag record of the previous tile (relative to tk0 * xr)
    int ckrec = -1;       // pending checkpoint row (record), its values
    double ckA = 0.0, ckB = 0.0;
    for (int t0 = 0; t0 < T; t0 += VIT_TILE) {
      const int rec = (t0 / VIT_TILE) * (int)xr;
      uint32_t bA = 0, bB = 0;
#ifdef ITR_VIT_UNROLL_TILE
#pragma unroll
#else
      // (not unrolled: sixteen copies of the step with its scan columns would fill the
      // instruction cache the CU shares with its neighbour)
#pragma unroll 1
#endif
      for (int sub = 0; sub < VIT_TILE; ++sub) {
        const int t = t0 + sub;
        if (t >= 1 && t < T) {
          if ((sub & (HT - 1)) == 0) {  // half-tile boundary (t >= 8)
            stage_wait();
            if (ckrec >= 0) {
              buf_store_f64(rck, vA * 8, (uint32_t)ckrec * 8, ckA);
              buf_store_f64(rck, vB * 8, (uint32_t)ckrec * 8, ckB);
              ckrec = -1;
            }
            if (sub == 0 && prec >= 0) {  // the previous tile's flag words
              buf_store_u16(rst, vA * 2, (uint32_t)prec * 2, (uint16_t)pbA);
              buf_store_u16(rst, vB * 2, (uint32_t)prec * 2, (uint16_t)pbB);
              prec = -1;
            }
            if ((t & 63) == 0) {  // next symbol chunk in, the one after requested
              SYM[(((t >> 6) + 1) & 1) * 64 + l] = clamp_sym(sin);
              sin = symg(t + 128 + l);
            }
            stage_issue(t / HT + 1);
          }
          const double* es = EST + ((t / HT) & 1) * EB + (t & (HT - 1)) * XRW;
          const double ecA = es[slA];
          const double ecB = es[slB];
          // omega_{t-1} of source chunk q (the scans' operands; over a group's 8 lanes, every
          // slot: Omega from them by a tree and three DPP steps, no cross-row traffic)
          double xs[IQ];
#pragma unroll
          for (int k = 0; k < IQ; ++k) xs[k] = X[q * IQS + k];
          double om = fmax(fmax(fmax(xs[0], xs[1]), fmax(xs[2], xs[3])),
                           fmax(fmax(xs[4], xs[5]), fmax(xs[6], xs[7])));
          if constexpr (IQ > 8) om = fmax(om, xs[8]);
          om = fmax(om, dpp_f64<DPP_Q1>(om));
          om = fmax(om, dpp_f64<DPP_Q2>(om));
          om = fmax(om, dpp_f64<DPP_HM>(om));
          const double ydA = (xA + ldA) + ecA;
          const double ydB = (xB + ldB) + ecB;
          // the bound test (exact: see the header)
          const bool failA = inA && !(ydA > (om + mA) + ecA);
          const bool failB = inB && !(ydB > (om + mB) + ecB);
          const uint64_t fA = __builtin_amdgcn_ballot_w64(failA);
          const uint64_t fB = __builtin_amdgcn_ballot_w64(failB);
          double zA = -INFINITY, zB = -INFINITY;
          // max over the group's lanes of the chunk maxima of target column r
          auto scan = [&](int r) {
            double y[IQ];
#pragma unroll
            for (int k = 0; k < IQ; ++k) y[k] = xs[k] + (r < IQ - 1 ? m[k][r] : M8[k * 64 + l]);
            double z = fmax(fmax(fmax(y[0], y[1]), fmax(y[2], y[3])),
                            fmax(fmax(y[4], y[5]), fmax(y[6], y[7])));
            if constexpr (IQ > 8) z = fmax(z, y[8]);
            return z;
          };
          auto group_max = [](double z) {
            z = fmax(z, dpp_f64<DPP_Q1>(z));
            z = fmax(z, dpp_f64<DPP_Q2>(z));
            return fmax(z, dpp_f64<DPP_HM>(z));
          };
          if ((fA | fB) != 0) {
            // target columns two at a time (two independent chains: the wave's step is
            // latency-bound), a pair when either of its columns has a failing target
#pragma unroll
            for (int r = 0; r < IQ - 1; r += 2) {
              if ((fA & (0x0303030303030303ull << r)) != 0) {
                double z0 = scan(r), z1 = scan(r + 1);
                z0 = group_max(z0);
                z1 = group_max(z1);
                zA = q == r ? z0 : (q == r + 1 ? z1 : zA);
              }
            }
            if (fB != 0) zB = group_max(scan(IQ - 1));
          }
          const double yoA = zA + ecA;
          const double yoB = zB + ecB;
          bA |= (uint32_t)(ydA > yoA) << sub;
          bB |= (uint32_t)(ydB > yoB) << sub;
          xA = fmax(ydA, yoA);
          xB = fmax(ydB, yoB);
          X[xiA] = xA;
          X[xiB] = xB;
          wave_lds_sync();  // omega_t visible to every lane for the next step
          if (sub == 0) {  // the tile's checkpoint row (t = t0 >= 16), stored later
            ckrec = rec;
            ckA = xA;
            ckB = xB;
          }
        }
      }
      pbA = bA;
      pbB = bB;
      prec = rec;
    }
    if (ckrec >= 0) {  // a checkpoint row whose half-tile boundary was past the block
      buf_store_f64(rck, vA * 8, (uint32_t)ckrec * 8, ckA);
      buf_store_f64(rck, vB * 8, (uint32_t)ckrec * 8, ckB);
    }
    buf_store_u16(rst, vA * 2, (uint32_t)prec * 2, (uint16_t)pbA);  // the last tile's flags
    buf_store_u16(rst, vB * 2, (uint32_t)prec * 2, (uint16_t)pbB);
    // last state = first argmax of omega_{T-1} by state index (optimizer.py:346)
    double bv = inA ? xA : -INFINITY;
    int bj = inA ? stA : 0x7fffffff;
    if (inB && (xB > bv || (xB == bv && stB < bj))) {
      bv = xB;
      bj = stB;
    }
    wave_first_max(bv, bj);
    if (l == 0) p.last_state[blk] = (uint8_t)bj;
    vit_wave_trace<XRW>(p, wl, blk, uni(bj));
    if (urgent) __builtin_amdgcn_s_setprio(0);
  }
}

// The full-scan per-wave step: lane l = 8 q + g, partial table in LDS, states in their own
// order (p.lew by state).
template <int IQ>
struct WaveVitFull {
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

template <int IQ>
__device__ __forceinline__ void vit_wave_task_full(const VitArgs& p, double* wl, int blk) {
  using C = WaveVitFull<IQ>;
  constexpr int XRW = C::XRW, NB = C::NB, IQS = C::IQS, XN = C::XN, PS = C::PS, HT = C::HT,
                NI = C::NI, EB = C::EB;
  // q high, g low: a 16-lane store group of the partial writes (ds_write_b64, banks mod 32)
  // then covers 8 target rows x 2 chunks at distinct banks (q low: 2 rows x 8 chunks, 2-way
  // on 4 banks; measured 41 of 141 LDS cycles per column as SQ_LDS_BANK_CONFLICT)
  const int l = lane_id_fresh(), q = l >> 3, g = l & 7;
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

    const int64_t c0 = uni64(p.off[blk]);
  const int T = uni((int)(p.off[blk + 1] - c0));
  if (T > 0) {  // (no `continue` in this loop, same reason)
    const bool urgent = T >= p.prio_len;
    if (urgent) __builtin_amdgcn_s_setprio(3);
    const uint16_t* ob = p.obs + c0;
    // raw symbol loads; the clamp into the alphabet (memory safety only) is applied when a
    // chunk is committed to SYM, 64 columns after its load was issued (a clamp right at
    // the load would make the wave wait for it there)
    auto symg = [&](int s) -> int { return (int)ob[min(s, T - 1)]; };
    auto clamp_sym = [](int v) -> uint16_t { return (uint16_t)min(v, 624); };
    // symbols: chunks of 64 columns, two resident in SYM, the next one in flight
    SYM[l] = clamp_sym(symg(l));
    SYM[64 + l] = clamp_sym(symg(64 + l));
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
    const int64_t tk0 = uni64(p.tile_off[blk]);
    // this block's checkpoint rows and flag words (tiles x xr records from tile tk0),
    // stored through buffer resources: lane part = the target's slot, uniform part = the
    // tile's record; a lane without a target stores out of bounds (nothing)
    const uint32_t nrec = (uint32_t)((T + VIT_TILE - 1) / VIT_TILE * xr);
    const __amdgpu_buffer_rsrc_t rck = buf_rsrc(p.ckpt + tk0 * xr, nrec * 8);
    const __amdgpu_buffer_rsrc_t rst = buf_rsrc(p.stay + tk0 * xr, nrec * 2);
    const uint32_t vA = inA ? (uint32_t)A : kOffNone / 8, vB = ownB ? (uint32_t)B : kOffNone / 8;
    buf_store_f64(rck, vA * 8, 0, xA);
    buf_store_f64(rck, vB * 8, 0, xB);
    stage_issue(0);
    stage_wait();
    stage_issue(1);
    // Stores are issued between a staging wait and the next staging issue: the checkpoint
    // row of a tile's first column at the following half-tile boundary, a tile's flag
    // words at the next tile's first boundary (or after the block).  A store issued just
    // before a vmcnt(0) would be waited for there.
    uint32_t pbA = 0, pbB = 0;
    int prec = -1;        // flag record of the previous tile (relative to tk0 * xr)
    int ckrec = -1;       // pending checkpoint row (record), its values
    double ckA = 0.0, ckB = 0.0;
    for (int t0 = 0; t0 < T; t0 += VIT_TILE) {
      const int rec = (t0 / VIT_TILE) * (int)xr;
      uint32_t bA = 0, bB = 0;
#pragma unroll
      for (int sub = 0; sub < VIT_TILE; ++sub) {
        const int t = t0 + sub;
        if (t >= 1 && t < T) {
          if ((sub & (HT - 1)) == 0) {  // half-tile boundary (t >= 8)
            stage_wait();
            if (ckrec >= 0) {
              buf_store_f64(rck, vA * 8, (uint32_t)ckrec * 8, ckA);
              buf_store_f64(rck, vB * 8, (uint32_t)ckrec * 8, ckB);
              ckrec = -1;
            }
            if (sub == 0 && prec >= 0) {  // the previous tile's flag words
              buf_store_u16(rst, vA * 2, (uint32_t)prec * 2, (uint16_t)pbA);
              buf_store_u16(rst, vB * 2, (uint32_t)prec * 2, (uint16_t)pbB);
              prec = -1;
            }
            if ((t & 63) == 0) {  // next symbol chunk in, the one after requested
              SYM[(((t >> 6) + 1) & 1) * 64 + l] = clamp_sym(sin);
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
          if (sub == 0) {  // the tile's checkpoint row (t = t0 >= 16), stored later
            ckrec = rec;
            ckA = xA;
            ckB = xB;
          }
        }
      }
      pbA = bA;
      pbB = bB;
      prec = rec;
    }
    if (ckrec >= 0) {  // a checkpoint row whose half-tile boundary was past the block
      buf_store_f64(rck, vA * 8, (uint32_t)ckrec * 8, ckA);
      buf_store_f64(rck, vB * 8, (uint32_t)ckrec * 8, ckB);
    }
    buf_store_u16(rst, vA * 2, (uint32_t)prec * 2, (uint16_t)pbA);  // the last tile's flags
    buf_store_u16(rst, vB * 2, (uint32_t)prec * 2, (uint16_t)pbB);
    // last state = first argmax of omega_{T-1}  (optimizer.py:346)
    double bv = inA ? xA : -INFINITY;
    int bj = inA ? A : 0x7fffffff;
    if (ownB && xB > bv) {  // B > A: a tie keeps A
      bv = xB;
      bj = B;
    }
    wave_first_max(bv, bj);
    if (l == 0) p.last_state[blk] = (uint8_t)bj;
    vit_wave_trace<XRW>(p, wl, blk, uni(bj));
    if (urgent) __builtin_amdgcn_s_setprio(0);
  }
}

// One Viterbi block on this wave: the bound-pruned step for blocks shorter than p.prune_len,
// the full scan for the others.  The two layouts carve the wave's LDS region differently, so
// a staging DMA still in flight from the wave's previous task (any kind) lands first.
template <int IQ>
struct WaveVitAny {
  static constexpr int WL =
      WaveVit<IQ>::WL > WaveVitFull<IQ>::WL ? WaveVit<IQ>::WL : WaveVitFull<IQ>::WL;
};
template <int IQ>
__device__ __forceinline__ void vit_wave_block(const VitArgs& p, double* wl, int blk) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int T = uni((int)(p.off[blk + 1] - p.off[blk]));
  if (T < p.prune_len)
    vit_wave_task<IQ>(p, wl, blk);
  else
    vit_wave_task_full<IQ>(p, wl, blk);
}

template <int NT, int NK>
__device__ __forceinline__ void fwd_wave_task(const WaveMfmaArgs& p, double* wl, int gi) {
  using C = WF<NT, NK>;
  constexpr int ER = C::ER, XS = C::XS, HT = C::HT, NI = C::NI, EB = C::EB, PIECES = C::PIECES;
  const int l = lane_id_fresh();
  const int n = p.n;
  const int rd = l >> 4;        // D row: the block this lane's results belong to
  const int ra = l & 3;         // A row: the block whose vector this lane feeds
  const int kk = l >> 4;        // A/B k-lane: sources kk NK + s
  const int jl = l & 15;        // D / B column within a tile: target 16 w + jl
  double* X = wl;
  double* EST = X + C::LX;
  uint16_t* SYM = reinterpret_cast<uint16_t*>(EST + C::LE);  // [2][4][64]
  double* FIN = EST + C::LE + C::LS;                         // [4][ER]

    // the four rows: task {block, split, slot}; T = steps of the row, Tb = block length
  int Tr[4], Tmax = 0;
  bool bwd = false;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int id = uni(p.groups[4 * gi + r]);
    int b = -1, sp = 0, Tb = 0;
    if (id >= 0) {
      b = uni(p.tasks[3 * id]);
      sp = uni(p.tasks[3 * id + 1]);
      Tb = uni((int)(p.off[b + 1] - p.off[b]));
    }
    Tr[r] = sp > 0 ? sp : (sp < 0 ? Tb + sp + 1 : Tb);
    Tmax = max(Tmax, Tr[r]);
    if (r == 0) bwd = sp < 0;
  }
  // this lane's D row
  const int idr = p.groups[4 * gi + rd];
  const int blk = idr >= 0 ? p.tasks[3 * idr] : -1;
  const int split = idr >= 0 ? p.tasks[3 * idr + 1] : 0;
  const int slot = idr >= 0 ? p.tasks[3 * idr + 2] : 0;
  const int64_t c0 = blk >= 0 ? p.off[blk] : 0;
  const int Tb = blk >= 0 ? (int)(p.off[blk + 1] - c0) : 0;
  const int T = split > 0 ? split : (split < 0 ? Tb + split + 1 : Tb);
  const int dir = split < 0 ? -1 : 1;
  if (Tmax == 0) {  // only empty blocks: log 1 = 0
    if (jl == 0 && blk >= 0 && split == 0) p.loglik[blk] = 0.0;
    return;
  }
  const bool urgent = Tmax >= p.prio_len;
  if (urgent) __builtin_amdgcn_s_setprio(2);

  // the matrix (a, or a^T for a group of backward halves) in the B layout
  double B[NT][NK];
  {
    const double* M = bwd ? p.aT : p.a;
#pragma unroll
    for (int w = 0; w < NT; ++w)
#pragma unroll
      for (int s = 0; s < NK; ++s) {
        const int i = kk * NK + s, j = 16 * w + jl;
        B[w][s] = (i < n && j < n) ? M[(int64_t)i * n + j] : 0.0;
      }
  }
  // symbols of the D row, step s: column s (forward) / Tb - 1 - s (backward), clamped into
  // the block; a backward half's last step reads row 625 (ones); loaded raw, fixed when a
  // 64-column chunk is committed to SYM (64 columns after its load was issued)
  auto sym_load = [&](int s) -> int {
    const int t = dir > 0 ? s : Tb - 1 - s;
    const int tc = min(max(t, 0), max(Tb - 1, 0));
    return (int)p.obs[Tb > 0 ? c0 + tc : 0];
  };
  auto sym_fix = [&](int s, int raw) -> uint16_t {
    if (split < 0 && s == T - 1) return (uint16_t)625;
    return (uint16_t)(Tb > 0 ? min(raw, 624) : 0);
  };
  // lane (rd, jl) stages positions 4 jl .. 4 jl + 3 of its row's chunks
  int sin[4];  // (raw 16-bit symbols)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int s0 = 4 * jl + i, s1 = 64 + 4 * jl + i;
    SYM[0 * 256 + rd * 64 + 4 * jl + i] = sym_fix(s0, sym_load(s0));
    SYM[1 * 256 + rd * 64 + 4 * jl + i] = sym_fix(s1, sym_load(s1));
    sin[i] = sym_load(128 + 4 * jl + i);
  }
  wave_lds_sync();
  auto sym_at = [&](int r, int s) -> int { return SYM[((s >> 6) & 1) * 256 + r * 64 + (s & 63)]; };
  // emission rows of half-tile h -> EST[h & 1]: element (u, r, j) at (u 4 + r) ER + j.
  // Piece 64 i + l of a half-tile is (column u, row r, targets 2c, 2c + 1): lane constants,
  // packed once per task as (r 64 + u) | 2c << 8 (the half-tile's symbols start at an even
  // column, so column u of it is SYM entry base + r 64 + u of one 64-column chunk)
  static_assert(HT == 2 && 2 * ER < (1 << 23), "piece packing");
  int pk[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int pc = 64 * i + l;
    const int u = pc / (2 * ER), rem = pc % (2 * ER), r = rem / (ER / 2), c = rem % (ER / 2);
    pk[i] = pc < PIECES ? ((r * 64 + u) | (2 * c) << 8) : -1;
  }
  auto stage_issue = [&](int h) {
    double* d = EST + (h & 1) * EB;
    const int s = h * HT;
    const int base = ((s >> 6) & 1) * 256 + (s & 63);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const double* src = p.ef;
      if (pk[i] >= 0) src += (int64_t)SYM[base + (pk[i] & 255)] * ER + (pk[i] >> 8);
      __builtin_amdgcn_global_load_lds(
          src, (__attribute__((address_space(3))) void*)(d + 128 * i), 16, 0, 0);
    }
  };
  auto stage_wait = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  // x_0 = pi e_0 (forward rows) / e_{Tb-1} (backward halves: x'_{Tb-1} = e_{Tb-1})
  double x[NT];
  int K = 0, Kfin = 0;
  {
    const int o0 = sym_at(rd, 0);
    const double* x0tab = dir < 0 ? p.emit : p.init;
#pragma unroll
    for (int w = 0; w < NT; ++w) {
      const int j = 16 * w + jl;
      x[w] = (T > 0 && j < n) ? x0tab[min(o0, 624) * n + j] : 0.0;
      X[rd * XS + j] = x[w];
      FIN[rd * ER + j] = x[w];
    }
  }
  stage_issue(0);
  stage_wait();
  stage_issue(1);
  wave_lds_sync();
  const int Tlast = T - 1;  // this lane's row is complete after step Tlast
  for (int t0 = 0; t0 < Tmax; t0 += HT) {
#pragma unroll
    for (int sub = 0; sub < HT; ++sub) {
      const int t = t0 + sub;
      if (t >= 1 && t < Tmax) {
        if (sub == 0) {
          stage_wait();
          if ((t & 63) == 0) {  // next symbol chunk in, the one after requested
            const int cb = (((t >> 6) + 1) & 1) * 256 + rd * 64 + 4 * jl;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int s = t + 64 + 4 * jl + i;
              SYM[cb + i] = sym_fix(s, sin[i]);
              sin[i] = sym_load(s + 64);
            }
            wave_lds_sync();
          }
          stage_issue(t / HT + 1);
        }
        // y = x_{t-1} @ a: NK k-steps x NT target tiles, NT independent chains
        double acc[NT];
#pragma unroll
        for (int w = 0; w < NT; ++w) acc[w] = 0.0;
        // A operands two at a time, the next pair's read issued before this pair's MFMAs;
        // the empty asm keeps the compiler from hoisting every read up front (their
        // registers would push the matrix slice into scratch)
        const double* xa = X + ra * XS + kk * NK;
        double a0 = xa[0], a1 = xa[1];
#pragma unroll
        for (int s = 0; s < NK; s += 2) {
          double n0 = a0, n1 = a1;
          if (s + 2 < NK) {
            n0 = xa[s + 2];
            n1 = xa[s + 3];
          }
#pragma unroll
          for (int w = 0; w < NT; ++w) acc[w] = mfma4(a0, B[w][s], acc[w]);
#pragma unroll
          for (int w = 0; w < NT; ++w) acc[w] = mfma4(a1, B[w][s + 1], acc[w]);
          a0 = n0;
          a1 = n1;
          asm volatile("" ::: "memory");
        }
        // x_t = y * e_t
        const double* es = EST + ((t / HT) & 1) * EB + ((t % HT) * 4 + rd) * ER + jl;
#pragma unroll
        for (int w = 0; w < NT; ++w) x[w] = acc[w] * es[16 * w];
        if ((t & 7) == 0) {  // exact 2^-k rescale by the row maximum
          double m = x[0];
#pragma unroll
          for (int w = 1; w < NT; ++w) m = fmax(m, x[w]);
          m = row16_max_w(m);
          const int e = (m > 0.0 && m < INFINITY) ? ilogb(m) : 0;
          const double sc = ldexp(1.0, -e);
          K += e;
#pragma unroll
          for (int w = 0; w < NT; ++w) x[w] *= sc;
        }
        wave_lds_sync();  // every lane's A reads of x_{t-1} precede the overwrite
#pragma unroll
        for (int w = 0; w < NT; ++w) X[rd * XS + 16 * w + jl] = x[w];
        wave_lds_sync();
        if (t == Tr[0] - 1 || t == Tr[1] - 1 || t == Tr[2] - 1 || t == Tr[3] - 1) {
          const bool cap = t == Tlast;  // a row completes (uniform test, lane-wise store)
          if (cap) {
#pragma unroll
            for (int w = 0; w < NT; ++w) FIN[rd * ER + 16 * w + jl] = x[w];
          }
          Kfin = cap ? K : Kfin;
        }
      }
    }
  }
  wave_lds_sync();  // final vectors
  // outputs of this lane's row
  if (blk >= 0 && T > 0) {
    if (split != 0) {  // half of a split block: the scaled vector and its exponent
      const int side = split < 0;
      double* sv = p.svec + ((int64_t)slot * 2 + side) * p.sstride;
#pragma unroll
      for (int w = 0; w < NT; ++w)
        if (16 * w + jl < n) sv[16 * w + jl] = FIN[rd * ER + 16 * w + jl];
      if (jl == 0) p.sK[slot * 2 + side] = Kfin;
    }
  }
  {  // log P = log(sum_j x_j) + K ln 2   (optimizer.py:160-162)
    double tot = 0.0;
#pragma unroll
    for (int w = 0; w < NT; ++w) tot += FIN[rd * ER + 16 * w + jl];  // padded targets hold 0
    tot = row16_sum_w(tot);
    if (jl == 0 && blk >= 0 && split == 0) p.loglik[blk] = T > 0 ? log(tot) + (double)Kfin * LN2 : 0.0;
  }
  if (urgent) __builtin_amdgcn_s_setprio(0);
}

}  // namespace itr
