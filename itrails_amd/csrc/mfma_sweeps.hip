// mfma_sweeps.hip — forward / backward+posterior sweeps of the iTRAILS HMM on the FP64
// matrix cores of MI355X (gfx950, CDNA4), four MAF blocks advanced in lock-step.
//
// Why lock-step: one block's column step is a vector x matrix product (1 x N . N x N), a
// 1/16-occupied MFMA tile.  v_mfma_f64_4x4x4_4b_f64 computes four independent 4x4x4
// products per instruction; with the four rows = four HMM blocks of similar length, every
// instruction advances 4 blocks x 16 target states x 4 source states, and a column step of
// the group is NK = ceil(N/4) instructions per 16-target tile (probed layout
// scripts/micro/mfma4_layout.hip):
//   sub-product g = (lane >> 2) & 3;  A: row lane & 3, k lane >> 4;  B: column lane & 3,
//   k lane >> 4;  D: row lane >> 4, column lane & 3.
// Here: A row = block of the group (x_{t-1} replicated over g), k-lane kk = lane >> 4 takes
// sources kk*NK + s at MFMA step s (one contiguous LDS run per lane), B column + 4g =
// target within the wave's 16-target tile, so lane l ends a step holding x_t of block
// r = l >> 4 at target j = 16 w + 4 g + (l & 3).  The lane's NK-slice of `a` lives in
// VGPRs for the whole kernel.  One wave per tile (NT waves); GB groups per workgroup share
// those registers (GB = 2: every wave runs two independent MFMA chains per step).
//
// Per step: MFMA chain (4 accumulators) -> x emission -> exact power-of-two rescale (every
// TE steps, maxima through LDS) -> publish to LDS -> one LDS-only barrier.  Emission values
// (and, backward, the stored forward rows) are gathered per lane from the L2-resident
// tables one tile of TE columns ahead, symbols two tiles ahead, so the step never waits on
// memory.  Blocks of a group end at different columns: each block's outputs stop at its own
// length (its lanes keep stepping on a clamped symbol, finite and unused).
//
// Numerics as the VALU sweeps (hmm_sweeps.hip): probability domain with exact 2^k
// rescaling — the reference's log-space recursion (optimizer.py:165-238) up to rounding
// (observed ~1e-15 relative; the bar is 1e-8).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {
namespace {

// reductions over the 16 lanes of a DPP row (= the 16 targets of one block in one wave):
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_ror:8
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  return v + dpp_f64<0x128>(v);
}
__device__ __forceinline__ double row16_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  return fmax(v, dpp_f64<0x128>(v));
}

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// Occupancy the register budget is sized for: GB = 1 kernels keep two workgroups per CU
// (N <= 96; the VALU tasks' matrix slice and staging set the budget), GB = 2 kernels one
// (their waves carry two groups each)
template <int NT, int NK, int GB, int MODE>
struct MOcc {
  static constexpr int wgs = GB == 1 ? (NK <= 24 ? 2 : 1) : 1;
  static constexpr int value = wgs * ((NT + 3) / 4);  // waves per SIMD (busiest SIMD)
};

// member rr of group gi (-1: none); with p.nmembers > 0 the groups are consecutive
// 4-chunks of a list of p.nmembers entries (the posterior's longest-first block order)
__device__ __forceinline__ int group_member(const MfmaArgs& p, int gi, int rr) {
  const int64_t k = 4 * (int64_t)gi + rr;
  if (gi >= p.ngroups || (p.nmembers > 0 && k >= p.nmembers)) return -1;
  return p.groups[k];
}

// LDS of one matrix-core task (carved from the kernel's dynamic LDS)
template <int NT, int NK, int GB, bool BWD = false>
struct MLds {
  static constexpr int KP = 4 * NK;
  static constexpr size_t x_off = 0;                                   // X[GB][2][4][KP]
  static constexpr size_t rs_off = x_off + (size_t)GB * 2 * 4 * KP * 8;  // RS[GB][2][4][NT]
  static constexpr size_t rm_off = rs_off + (size_t)GB * 2 * NT * 4 * 8; // RM[GB][NT][4]
  static constexpr size_t kf_off = rm_off + (size_t)GB * NT * 4 * 8;     // KF[GB][4]
  // MODE_BWD: alpha * beta rows Q[GB][2][4][16 NT] and their normalisers RN[GB][2][4]
  static constexpr size_t q_off = kf_off + (size_t)GB * 4 * 4 + 8;
  static constexpr size_t rn_off = q_off + (size_t)GB * 2 * 4 * 16 * NT * 8;
  static constexpr size_t bytes = BWD ? rn_off + (size_t)GB * 2 * 4 * 8 : q_off;
};

// y[gb] = x_gb(row ra, sources kk NK ..) @ B for the GB groups of a task.  The A operands
// (two per ds_read_b128) stream through a ring of D reads in flight per group, refilled
// behind the MFMAs that consume them: an LDS round trip (~100 cycles) then hides under 2 D GB
// MFMAs (16 cycles each).  With one read ahead (the round-4 form) every pair of MFMAs waited
// for its operands (lgkmcnt(1) before each pair in the ISA).  The empty asm keeps the
// compiler from hoisting every read to the top (their registers would spill the matrix
// slice) or from serialising them.  Same MFMAs, same accumulators, same order: bit-identical.
template <int NK, int GB>
__device__ __forceinline__ void mfma_chain(const double* const (&xs)[GB], const double (&B)[NK],
                                           double (&y)[GB]) {
  constexpr int W = 2;                 // A operands per group per read (one ds_read_b128)
  constexpr int NQ = (NK + W - 1) / W; // reads per group
  constexpr int D = NQ < 4 ? NQ : 4;   // reads in flight per group
  // four accumulator chains per group (source s into chain s % 4: the 52-cycle dependent
  // MFMA latency under 4 x 16 issue cycles), summed as (0 + 1) + (2 + 3)
  double acc[GB][4], ring[GB][D][W];
#pragma unroll
  for (int gb = 0; gb < GB; ++gb) {
    acc[gb][0] = acc[gb][1] = acc[gb][2] = acc[gb][3] = 0.0;
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int u = 0; u < W; ++u) ring[gb][d][u] = d * W + u < NK ? xs[gb][d * W + u] : 0.0;
  }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int qi = 0; qi < NQ; ++qi) {
    const int slot = qi % D;
#pragma unroll
    for (int u = 0; u < W; ++u)
#pragma unroll
      for (int gb = 0; gb < GB; ++gb) {
        const int k = qi * W + u;
        if (k < NK) acc[gb][k & 3] = mfma4(ring[gb][slot][u], B[k], acc[gb][k & 3]);
      }
    if (qi + D < NQ) {
#pragma unroll
      for (int gb = 0; gb < GB; ++gb)
#pragma unroll
        for (int u = 0; u < W; ++u) {
          const int k = (qi + D) * W + u;
          ring[gb][slot][u] = k < NK ? xs[gb][k] : 0.0;
        }
    }
    asm volatile("" ::: "memory");
  }
#pragma unroll
  for (int gb = 0; gb < GB; ++gb) y[gb] = (acc[gb][0] + acc[gb][1]) + (acc[gb][2] + acc[gb][3]);
}

// One task of the matrix-core sweep: the GB groups g0 .. g0+GB-1 of p.groups.
template <int NT, int NK, int GB, int MODE>
__device__ __forceinline__ void mfma_task(const MfmaArgs& p, unsigned char* smem, int g0) {
  constexpr int KP = 4 * NK;                  // padded source count
  constexpr int TE = GB == 1 ? 4 : 2;         // columns per prefetch tile
  static_assert(TE >= 2 && 8 % TE == 0, "rescale every 8 steps at tile starts");
  constexpr int TB = 64 * NT;
  using LD = MLds<NT, NK, GB, MODE == MODE_BWD>;
  auto X = reinterpret_cast<double (*)[2][4][KP]>(smem + LD::x_off);    // published vectors
  auto RS = reinterpret_cast<double (*)[2][4][NT]>(smem + LD::rs_off);  // row partial sums
  auto RM = reinterpret_cast<double (*)[NT][4]>(smem + LD::rm_off);     // row maxima
  auto KF = reinterpret_cast<int (*)[4]>(smem + LD::kf_off);
  auto Q = reinterpret_cast<double (*)[2][4][16 * NT]>(smem + LD::q_off);  // BWD: alpha*beta
  auto RN = reinterpret_cast<double (*)[2][4]>(smem + LD::rn_off);         // BWD: 1 / row sums

  const int n = p.n;
  const int tid = threadIdx.x;
  const int w = uni(tid >> 6);
  const int l = tid & 63;
  const int r = l >> 4;                            // block row of the group
  const int j = 16 * w + 4 * ((l >> 2) & 3) + (l & 3);  // target state
  const int ra = l & 3, kk = l >> 4;               // A operand: block row, k-lane
  const bool jv = j < n;
  const bool row_leader = (l & 15) == 0;
  // this lane's sink slot: one 64-double line set per workgroup (kSinkWgs of them), so the
  // discarded stores of different CUs never share a cache line
  double* const sink = p.sink + (int64_t)(blockIdx.x % kSinkWgs) * 64 + l;

  // Rows of the group(s).  MODE_FWD_LL: p.groups holds task ids of p.tasks {block, split,
  // slot} — whole blocks (split 0), first halves (split m > 0: columns [0, m)) or second
  // halves (split -m: the textbook backward from the end, contracting with a^T, see
  // valu_sweep.h); a group is all forward-shaped or all backward halves.  Other modes:
  // block ids.  T = steps of the row, Tb = block length, dir = column order.
  int T[GB], Tb[GB], dir[GB], Tmax = 0;
  int64_t c0[GB];
  int task_blk[GB], task_split[GB], task_slot[GB];
  bool backward_group = false;
#pragma unroll
  for (int gb = 0; gb < GB; ++gb) {
    const int gi = g0 + gb;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int id = group_member(p, gi, rr);
      int b2 = id, sp = 0, sl = 0;
      if (MODE == MODE_FWD_LL && id >= 0) {
        b2 = p.tasks[3 * id];
        sp = p.tasks[3 * id + 1];
        sl = p.tasks[3 * id + 2];
      }
      const int tb2 = b2 >= 0 ? (int)(p.off[b2 + 1] - p.off[b2]) : 0;
      const int t2 = sp > 0 ? sp : (sp < 0 ? tb2 + sp + 1 : tb2);
      Tmax = max(Tmax, t2);
      if (rr == 0 && sp < 0) backward_group = true;
      if (rr == r) {
        task_blk[gb] = b2;
        task_split[gb] = sp;
        task_slot[gb] = sl;
        Tb[gb] = tb2;
        T[gb] = t2;
        dir[gb] = sp < 0 ? -1 : 1;
        c0[gb] = b2 >= 0 ? p.off[b2] : 0;
      }
    }
  }
  Tmax = uni(Tmax);
  backward_group = uni(backward_group);
  (void)task_slot;
  (void)task_blk;

  double B[NK];  // this lane's slice of a (a^T for backward halves): rows kk*NK + s,
                 // column j (per task: a few L2 loads against thousands of steps)
  const double* mp = (MODE == MODE_FWD_LL && backward_group) ? p.matT : p.mat;
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    const int i = kk * NK + s;
    B[s] = (i < n && jv) ? mp[(int64_t)i * n + j] : 0.0;
  }
  for (int i = tid; i < GB * 2 * 4 * KP; i += TB) (&X[0][0][0][0])[i] = 0.0;
  lds_barrier();
  {
    if (MODE == MODE_FWD_LL && Tmax == 0 && tid < 4 * GB) {  // only empty blocks: log 1 = 0
      const int gi = g0 + (tid >> 2);
      const int id = group_member(p, gi, tid & 3);
      if (id >= 0) p.loglik[p.tasks[3 * id]] = 0.0;
    }
    if (Tmax > 0) {
      const bool urgent = Tmax >= p.prio_len;
      if (urgent) __builtin_amdgcn_s_setprio(2);
      // Prefetch with no load consumed inside its own tile: the symbol of step s of this
      // lane's row (column s forward, Tb - 1 - s backward, clamped into the block; an empty
      // row reads column 0 of the array) is loaded raw two tiles ahead, unconditionally;
      // one tile ahead its emission value is loaded from the address it gives (padded target
      // lanes read column 0: finite, and their products are 0); a backward half's last step
      // (a row of ones) is applied where the value is used.  A clamp or a select on a fresh
      // load makes hipcc wait for it on the spot (s_waitcnt vmcnt(0) every column).
      // (posterior modes: addresses as a per-row base plus one 32 x 32 -> 64-bit product with
      // the byte stride — v_mad_u64_u32 with the base as addend — instead of 64-bit index
      // arithmetic per load: (7,7) posterior 22.17-22.24 -> 22.11-22.16 ms; the forward
      // log-likelihood sweep keeps the index form, 4.00-4.04 against 4.02-4.11 ms with it,
      // profiles/r5abaddr_ab.txt)
      const uint16_t* obr[GB];
#pragma unroll
      for (int gb = 0; gb < GB; ++gb) obr[gb] = p.obs + (Tb[gb] > 0 ? c0[gb] : 0);
      auto sym = [&](int gb, int s) -> int {
        const int t = dir[gb] > 0 ? s : Tb[gb] - 1 - s;
        const int tc = min(max(t, 0), max(Tb[gb] - 1, 0));
        if constexpr (MODE == MODE_FWD_LL) return (int)p.obs[Tb[gb] > 0 ? c0[gb] + tc : 0];
        return (int)obr[gb][(uint32_t)tc];
      };
      const int jc = jv ? j : 0;
      const char* const ebase = reinterpret_cast<const char*>(p.emit + jc);
      const uint32_t rowb = (uint32_t)n * 8u;  // bytes per emission row
      auto emis = [&](int sy) -> double {
        if constexpr (MODE == MODE_FWD_LL) return p.emit[min(sy, 624) * n + jc];
        return *reinterpret_cast<const double*>(ebase + (uint64_t)(uint32_t)min(sy, 624) * rowb);
      };
      auto ones_at = [&](int gb, int s) -> bool {
        return MODE == MODE_FWD_LL && task_split[gb] < 0 && s == T[gb] - 1;
      };
      int snxt[GB][TE];
      double enxt[GB][TE];

      if constexpr (MODE == MODE_FWD_LL || MODE == MODE_FWD_STORE) {
        // ---------------- forward: x_t = (x_{t-1} @ a) * e_t  (optimizer.py:181-187)
        double x[GB], xfin[GB];
        int K[GB], Kfin[GB];
#pragma unroll
        for (int gb = 0; gb < GB; ++gb) {
          // x_0 = pi * e_0 (forward rows); a backward half starts from e_{Tb-1}
          const double* x0tab = dir[gb] < 0 ? p.emit : p.init;
          x[gb] = (T[gb] > 0 && jv) ? x0tab[min(sym(gb, 0), 624) * n + j] : 0.0;
          if (jv) X[gb][0][r][j] = x[gb];
          if (MODE == MODE_FWD_STORE && T[gb] > 0) p.alpha[c0[gb] * p.astride + j] = x[gb];
          xfin[gb] = x[gb];
          K[gb] = Kfin[gb] = 0;
#pragma unroll
          for (int u = 0; u < TE; ++u) {
            enxt[gb][u] = emis(sym(gb, u));
            snxt[gb][u] = sym(gb, TE + u);
          }
        }
        wait_vmem_all();
        lds_barrier();
        // The forward-store rows run whole tiles and store every step (past a row's end into
        // the sink): one path through the tile, so the wait for the next tile's loads at its
        // end does not also wait for the row stores issued after them (vmcnt counts both, in
        // order, and a skipped store would make the compiler assume the shorter count).
        for (int t0 = 0; t0 < Tmax; t0 += TE) {
          double ecur[GB][TE];
#pragma unroll
          for (int gb = 0; gb < GB; ++gb) {
#pragma unroll
            for (int u = 0; u < TE; ++u) ecur[gb][u] = enxt[gb][u];
#pragma unroll
            for (int u = 0; u < TE; ++u) {
              enxt[gb][u] = emis(snxt[gb][u]);
              snxt[gb][u] = sym(gb, t0 + 2 * TE + u);
            }
          }
#pragma unroll
          for (int sub = 0; sub < TE; ++sub) {
            const int t = t0 + sub;
            if (t >= 1 && (MODE == MODE_FWD_STORE || t < Tmax)) {
              const int buf = (t - 1) & 1;
              double y[GB];
              const double* xs[GB];
#pragma unroll
              for (int gb = 0; gb < GB; ++gb) xs[gb] = &X[gb][buf][ra][kk * NK];
              mfma_chain<NK, GB>(xs, B, y);
#pragma unroll
              for (int gb = 0; gb < GB; ++gb) {
                double sc = 1.0;
                if (sub == 1 && (t0 & 7) == 0 && t > 1) {  // maxima of x_{t-1} (t-1 = 0 mod 8)
                  double M = RM[gb][0][r];
#pragma unroll
                  for (int v = 1; v < NT; ++v) M = fmax(M, RM[gb][v][r]);
                  if (M > 0.0 && M < INFINITY) {
                    const int e = ilogb(M);
                    sc = ldexp(1.0, -e);
                    K[gb] += e;
                  }
                }
                x[gb] = (y[gb] * (ones_at(gb, t) ? 1.0 : ecur[gb][sub])) * sc;
                if constexpr (MODE == MODE_FWD_LL) {
                  if (t == T[gb] - 1) {
                    xfin[gb] = x[gb];
                    Kfin[gb] = K[gb];
                  }
                } else {
                  // past the row's end: the lane's sink slot (a select, not a branch)
                  double* dst = t < T[gb] ? reinterpret_cast<double*>(
                                                  reinterpret_cast<char*>(p.alpha + c0[gb] * p.astride + j) +
                                                  (uint64_t)(uint32_t)t * ((uint32_t)p.astride * 8u))
                                            : sink;
                  *dst = x[gb];
                }
                if (jv) X[gb][buf ^ 1][r][j] = x[gb];
                if (sub == 0 && (t0 & 7) == 0) {  // every 8th column: maxima for the rescale
                  const double m = row16_max(x[gb]);
                  if (row_leader) RM[gb][w][r] = m;
                }
              }
              lds_barrier();
            }
          }
        }
        if constexpr (MODE == MODE_FWD_LL) {
#pragma unroll
          for (int gb = 0; gb < GB; ++gb) {
            if (task_split[gb] != 0) {
              // half of a split block: the scaled vector and its exponent
              // (fwd_split_combine_kernel joins the halves)
              const int side = task_split[gb] < 0;
              if (jv) p.svec[((int64_t)task_slot[gb] * 2 + side) * p.astride + j] = xfin[gb];
              if (w == 0 && row_leader) p.sK[task_slot[gb] * 2 + side] = Kfin[gb];
            }
            // log P = log(sum_j x_j) + K ln 2   (optimizer.py:160-162)
            const double s = row16_sum(xfin[gb]);
            if (row_leader) RS[gb][0][r][w] = s;
            if (w == 0 && row_leader) KF[gb][r] = Kfin[gb];
          }
          lds_barrier();
          if (tid < 4 * GB) {
            const int gb = tid >> 2, rr = tid & 3;
            const int gi = g0 + gb;
            const int id = group_member(p, gi, rr);
            if (id >= 0 && p.tasks[3 * id + 1] == 0) {
              const int b2 = p.tasks[3 * id];
              double S = 0.0;
              for (int v = 0; v < NT; ++v) S += RS[gb][0][rr][v];
              const int T2 = (int)(p.off[b2 + 1] - p.off[b2]);
              p.loglik[b2] = T2 > 0 ? log(S) + (double)KF[gb][rr] * LN2 : 0.0;
            }
          }
        }
      } else {
        // ---------------- backward + posterior (optimizer.py:191-238)
        //   beta_{T-1} = 1;  beta_{t-1} = (beta_t * e_t) @ a   (vector @ a: the reference's form)
        //   post_t = alpha_t * beta_t / sum_j(alpha_t * beta_t)
        // Step s handles column t = T - 1 - s of every block of the group.  Only the product
        // and the vector it publishes sit on the step's critical path, and the normalisation
        // is taken off the three waves of SIMD 0 (VALU issue there, beside the matrix chain,
        // is what the step is short of): after barrier s every wave writes its
        // alpha_t * beta_t values to Q[s & 1]; at step s + 1 one wave (wave 1, on a SIMD with
        // two waves) sums each row of Q and publishes 1 / sum in RN; at step s + 2 every wave
        // stores its posterior row of column t (its product kept two steps).  Each array is
        // read one step after it is written and rewritten one step later: two buffers.  The
        // loop runs whole tiles, to two steps past the longest row, and every step stores
        // (lanes with no row into the sink): one path through the tile, so the wait for the
        // next tile's loads does not also wait for the stores issued after them.
        double bt[GB], q1[GB], q2[GB];  // alpha * beta of the last two steps
        double anxt[GB][TE];
        // Addresses as a per-row base plus one 32 x 32 -> 64-bit product (v_mad_u64_u32): the
        // tile's twelve loads and the step's store otherwise cost ~20 VALU instructions each
        // in 64-bit index arithmetic, and VALU issue — three waves on SIMD 0 — is what this
        // step is short of beside the matrix chain.  Rows clamp at the block's column 0 (an
        // empty row reads the arrays' first entries; padded target lanes read stored zeros).
        const uint16_t* ob[GB];
        const double* ab[GB];
        double* pb[GB];
#pragma unroll
        for (int gb = 0; gb < GB; ++gb) {
          const int64_t cb = T[gb] > 0 ? c0[gb] : 0;
          ob[gb] = p.obs + cb;
          ab[gb] = p.alpha + cb * p.astride + j;
          pb[gb] = p.post + cb * n + j;
        }
        const uint32_t ast8 = (uint32_t)p.astride * 8u, un8 = (uint32_t)n * 8u;  // byte strides
        auto bsym = [&](int gb, int s) -> int {  // symbol of column T-1-s
          return (int)ob[gb][(uint32_t)max(T[gb] - 1 - s, 0)];
        };
        auto bemis = [&](int sy) -> double { return emis(sy); };
        auto arow = [&](int gb, int s) -> double {  // stored forward row of column T-1-s
          return *reinterpret_cast<const double*>(reinterpret_cast<const char*>(ab[gb]) +
                                                  (uint64_t)(uint32_t)max(T[gb] - 1 - s, 0) * ast8);
        };
#pragma unroll
        for (int gb = 0; gb < GB; ++gb) {
          bt[gb] = (T[gb] > 0 && jv) ? 1.0 : 0.0;
          q1[gb] = q2[gb] = 0.0;
#pragma unroll
          for (int u = 0; u < TE; ++u) {
            enxt[gb][u] = bemis(bsym(gb, u));
            anxt[gb][u] = arow(gb, u);
            snxt[gb][u] = bsym(gb, TE + u);
          }
        }
        wait_vmem_all();
        const bool norm_wave = w == 1;
        const int nl = l & 15;  // the norm wave: lane nl of row r sums Q[..][r][nl NT ..]
        for (int s0 = 0; s0 < Tmax + 2; s0 += TE) {
          double ecur[GB][TE], acur[GB][TE];
#pragma unroll
          for (int gb = 0; gb < GB; ++gb) {
#pragma unroll
            for (int u = 0; u < TE; ++u) {
              ecur[gb][u] = enxt[gb][u];
              acur[gb][u] = anxt[gb][u];
            }
#pragma unroll
            for (int u = 0; u < TE; ++u) {
              enxt[gb][u] = bemis(snxt[gb][u]);
              anxt[gb][u] = arow(gb, s0 + TE + u);
              snxt[gb][u] = bsym(gb, s0 + 2 * TE + u);
            }
          }
#pragma unroll
          for (int sub = 0; sub < TE; ++sub) {
            const int s = s0 + sub;
            const int buf = sub & 1;  // s0 is a multiple of TE (even)
            const bool rescale = sub == 0 && (s0 & 7) == 0;
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) {
              const double v = bt[gb] * ecur[gb][sub];
              if (rescale) {
                const double m = row16_max(v);
                if (row_leader) RM[gb][w][r] = m;
              }
              if (jv) X[gb][buf][r][j] = v;
            }
            lds_barrier();
            // the normalisers of step s - 2 (published at step s - 1) and, on the norm wave,
            // the products of step s - 1
            double rn[GB], qs[GB][NT];
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) {
              rn[gb] = RN[gb][buf][r];
              if (norm_wave) {
#pragma unroll
                for (int v = 0; v < NT; ++v) qs[gb][v] = Q[gb][buf ^ 1][r][nl * NT + v];
              }
            }
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) {
              const double qv = acur[gb][sub] * bt[gb];  // padded states: 0 * 0
              Q[gb][buf][r][j] = qv;
              if (norm_wave) {
                double S = qs[gb][0];
#pragma unroll
                for (int v = 1; v < NT; ++v) S += qs[gb][v];
                S = row16_sum(S);
                if (row_leader) RN[gb][buf ^ 1][r] = recip_nr(S);
              }
              const int sp = s - 2;  // the column of step s - 2
              double* dst = (sp >= 0 && sp < T[gb] && jv)
                                ? reinterpret_cast<double*>(reinterpret_cast<char*>(pb[gb]) +
                                                            (uint64_t)(uint32_t)(T[gb] - 1 - sp) * un8)
                                : sink;
              *dst = q2[gb] * rn[gb];
              q2[gb] = q1[gb];
              q1[gb] = qv;
            }
            double y[GB];
            const double* xs[GB];
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) xs[gb] = &X[gb][buf][ra][kk * NK];
            mfma_chain<NK, GB>(xs, B, y);
#pragma unroll
            for (int gb = 0; gb < GB; ++gb) {
              double sc = 1.0;
              if (rescale) {  // (the maxima read here: before the chain their registers spill)
                double M = RM[gb][0][r];
#pragma unroll
                for (int v = 1; v < NT; ++v) M = fmax(M, RM[gb][v][r]);
                if (M > 0.0 && M < INFINITY) sc = ldexp(1.0, -ilogb(M));
              }
              bt[gb] = y[gb] * sc;
            }
          }
        }
      }
      if (urgent) __builtin_amdgcn_s_setprio(0);
    }
    lds_barrier();
  }
}

// The hybrid persistent sweep: the longest blocks (p.urgent: VALU tasks of `v`, one block —
// or half of a split block — per workgroup, lowest step latency) first, then the bulk as
// matrix-core groups.  One launch, one workgroup shape: no co-residency assumption between
// kernels is needed for the long blocks to start at once.
template <int NT, int NK, int GB, int MODE, int VRJ, int VIQ>
__global__ void __launch_bounds__(64 * NT, (MOcc<NT, NK, GB, MODE>::value))
    hybrid_sweep_kernel(MfmaArgs p, SweepArgs v) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int qslot[2];
  // VALU tasks.  The posterior splits its first v.nbeta (longest) blocks at column lo
  // (v.sub_lo): the forward-store launch runs, beside each one's forward sweep, its backward
  // sweep over [lo, T) storing beta rows (task 2k: block k backward, 2k + 1: forward); the
  // backward launch's VALU task then sweeps only [0, lo] from the stored beta_lo, and
  // post_combine forms the columns (lo, T).  The longest block then costs one sweep of its
  // length in the forward launch and lo columns in the backward one, instead of two whole
  // sweeps one after the other.
  // (the forward tasks are the first v.nblocks blocks of the order, the beta tasks the first
  // v.nbeta: the two sets interleaved longest first, then the longer set's rest)
  const int nb = MODE == MODE_FWD_STORE ? (int)v.nbeta : 0;
  const int np = min((int)v.nblocks, nb);
  const int64_t nvalu = v.nblocks + nb;
  for (;;) {
    if (threadIdx.x == 0) qslot[0] = atomicAdd(v.queue, 1);
    lds_barrier();
    const int bi = uni(qslot[0]);
    lds_barrier();
    if (bi >= nvalu) break;
    if (MODE == MODE_FWD_STORE && bi < 2 * np) {
      if (bi & 1)
        sweep_task<8, NT, VRJ, VIQ, MODE_FWD_STORE>(v, smem, bi >> 1);
      else
        sweep_task<8, NT, VRJ, VIQ, MODE_BETA>(v, smem, bi >> 1);
    } else if (MODE == MODE_FWD_STORE && nb > np) {
      sweep_task<8, NT, VRJ, VIQ, MODE_BETA>(v, smem, bi - np);
    } else {
      sweep_task<8, NT, VRJ, VIQ, MODE>(v, smem, bi - np);
    }
  }
  for (;;) {
    if (threadIdx.x == 0) qslot[1] = atomicAdd(p.queue, GB);
    lds_barrier();
    const int g0 = uni(qslot[1]);
    lds_barrier();
    if (g0 >= p.ngroups) break;
    mfma_task<NT, NK, GB, MODE>(p, smem, g0);
  }
  // the split blocks' combine (posterior rows of (lo, T) from the stored rows), taken by the
  // workgroups that run out of groups: it fills the launch's tail instead of a launch of its
  // own after it
  if constexpr (MODE == MODE_BWD) {
    for (;;) {
      if (threadIdx.x == 0) qslot[0] = v.ncomb > 0 ? atomicAdd(v.comb_queue, 1) : 0;
      lds_barrier();
      const int ci = uni(qslot[0]);
      lds_barrier();
      if (ci >= v.ncomb) break;
      const int blk = (int)v.comb[3 * ci];
      const int64_t c0 = v.off[blk], lo = v.sub_lo[blk];
      const int64_t t1 = v.comb[3 * ci + 2];
      const int xr = 16 * NT;
      for (int64_t t = v.comb[3 * ci + 1] + (threadIdx.x >> 6); t < t1; t += NT)
        post_combine_column(v.n, xr, v.alpha + (c0 + t) * xr,
                            v.beta_in + (v.beta_off[blk] + t - lo) * xr, v.post + (c0 + t) * v.n,
                            threadIdx.x & 63);
    }
  }
}

// ---------------------------------------------------------------------------------------
// configurations by state count: NT tiles of 16 targets, NK k-steps of 4 sources, GB groups
// ---------------------------------------------------------------------------------------
struct MCfg {
  int nmin, nmax, nt, nk, gb, viq;  // viq: sources per lane of the VALU tasks (8 lanes)
  double pfrac;  // posterior: blocks longer than pfrac x the longest run as VALU tasks
  bool post;     // the hybrid posterior beats the VALU-only one at this size
  double bfrac;  // posterior: VALU blocks at least bfrac x the longest are split ...
  double lofrac; // ... at column lofrac x T (itr_posterior)
};
// pfrac measured on the (7,7) model, 10 Mbp (round 2: 0.2 / 0.35 / 0.5 / 0.7 -> 203 / 264 /
// 281 / 259 M columns/s; round 5, with the long blocks' backward split (itr_posterior):
// 0.45 / 0.5 / 0.55 / 0.6 / 0.65 -> 23.9 / 22.8 / 22.4 / 23.1 / 25.1 ms, per-launch
// fractions no better, profiles/r5ab_posterior_variants.txt) and the (5,5) model
// (the (5,5) model, N = 70: hybrid posterior 465 M columns/s against 496 for the VALU-only
// three-wave sweeps in round 2; with round 5's backward step and split, 668-685 against
// 521-523 M (profiles/r5ab55*): the hybrid serves N = 65..72.  The introgression (5,5)
// model, N = 95: 421 against 461 M, so 81..96 stays VALU-only; other sizes unmeasured.)
// bfrac / lofrac: round 5 at N = 133 (0.5 / 0.4, profiles/r5ps_posterior_split.txt; 0.35 /
// 0.4 / 0.5 within 0.05 ms in round 6).  N = 70 re-swept in round 6 (profiles/r6e_*, r6f_
// posterior_params.txt): (pfrac, bfrac) = (0.35, 0.5) 14.6-14.8 ms, (0.35, 0.35) 13.2,
// (0.25, 0.35) 13.0-13.2, (0.2, 0.35) 14.2, (0.3, 0.3) 12.9-13.0, (0.25, 0.3) 12.5-12.7,
// (0.25, 0.25) 12.4-12.6; lofrac 0.3 / 0.35 / 0.45 / 0.5 no better than 0.4
constexpr MCfg kMCfgs[] = {
    {33, 48, 3, 12, 1, 6, 0.35, false, 0.5, 0.4},   {49, 64, 4, 16, 1, 8, 0.35, false, 0.5, 0.4},
    {65, 72, 5, 18, 1, 9, 0.25, true, 0.25, 0.4},    {73, 80, 5, 20, 1, 10, 0.35, false, 0.5, 0.4},
    {81, 96, 6, 24, 1, 12, 0.35, false, 0.5, 0.4},  {129, 136, 9, 34, 1, 17, 0.55, true, 0.5, 0.4},
    {137, 144, 9, 36, 1, 18, 0.55, true, 0.5, 0.4},
    // two groups per workgroup (experiment configuration, ITR_MCFG)
    {129, 136, 9, 34, 2, 17, 0.55, true, 0.5, 0.4}};
constexpr int kMCfgsAuto = 7;  // entries picked by state count

template <int NT, int NK, int GB, int MODE, int VIQ>
size_t lds_h() {
  using V = ValuSweep<8, NT, 2, VIQ, MODE>;
  // forward-store launches also run backward (beta) tasks
  using VB = ValuSweep<8, NT, 2, VIQ, MODE == MODE_FWD_STORE ? MODE_BETA : MODE>;
  return std::max(MLds<NT, NK, GB, MODE == MODE_BWD>::bytes, std::max(V::lds_bytes, VB::lds_bytes));
}
template <int NT, int NK, int GB, int MODE, int VIQ>
hipError_t launch_h(const MfmaArgs& a, const SweepArgs& v, int grid, size_t lds_min,
                    hipStream_t st) {
  const size_t lds = std::max(lds_h<NT, NK, GB, MODE, VIQ>(), lds_min);
  hipLaunchKernelGGL((hybrid_sweep_kernel<NT, NK, GB, MODE, 2, VIQ>), dim3(grid), dim3(64 * NT),
                     lds, st, a, v);
  return hipGetLastError();
}
template <int NT, int NK, int GB, int MODE, int VIQ>
int occ_h() {
  int nb = 0;
  const size_t lds = lds_h<NT, NK, GB, MODE, VIQ>();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &nb, hybrid_sweep_kernel<NT, NK, GB, MODE, 2, VIQ>, 64 * NT, lds) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}

template <int MODE>
hipError_t dispatch_m(int c, bool launch, const MfmaArgs* a, const SweepArgs* v, int grid,
                      size_t lds_min, hipStream_t st, int* occ) {
#define ITR_MCFG(C, NT, NK, GB, VIQ)                                        \
  case C:                                                                   \
    if (launch) return launch_h<NT, NK, GB, MODE, VIQ>(*a, *v, grid, lds_min, st); \
    *occ = occ_h<NT, NK, GB, MODE, VIQ>();                                  \
    return hipSuccess;
  switch (c) {
    ITR_MCFG(0, 3, 12, 1, 6)
    ITR_MCFG(1, 4, 16, 1, 8)
    ITR_MCFG(2, 5, 18, 1, 9)
    ITR_MCFG(3, 5, 20, 1, 10)
    ITR_MCFG(4, 6, 24, 1, 12)
    ITR_MCFG(5, 9, 34, 1, 17)
    ITR_MCFG(6, 9, 36, 1, 18)
    ITR_MCFG(7, 9, 34, 2, 17)
  }
#undef ITR_MCFG
  return hipErrorInvalidValue;
}

hipError_t dispatch_mode_m(int mode, int c, bool launch, const MfmaArgs* a, const SweepArgs* v,
                           int grid, size_t lds_min, hipStream_t st, int* occ) {
  switch (mode) {
    case MODE_FWD_LL: return dispatch_m<MODE_FWD_LL>(c, launch, a, v, grid, lds_min, st, occ);
    case MODE_FWD_STORE:
      return dispatch_m<MODE_FWD_STORE>(c, launch, a, v, grid, lds_min, st, occ);
    case MODE_BWD: return dispatch_m<MODE_BWD>(c, launch, a, v, grid, lds_min, st, occ);
  }
  return hipErrorInvalidValue;
}

}  // namespace

MfmaGeometry mfma_geometry(int n, int mode) {
  MfmaGeometry g{};
  g.cfg = -1;
  if (mode == MODE_VIT) return g;  // max-plus: no matrix-core form
  for (int c = 0; c < kMCfgsAuto; ++c)
    if (n >= kMCfgs[c].nmin && n <= kMCfgs[c].nmax) g.cfg = c;
  if (g.cfg >= 0 && mode != MODE_FWD_LL && !kMCfgs[g.cfg].post) g.cfg = -1;
#ifdef ITR_EXPERIMENT
  if (getenv("ITR_NO_MFMA")) g.cfg = -1;
  if (getenv("ITR_HYB_POST") && mode != MODE_FWD_LL) {  // force the hybrid posterior
    for (int c = 0; c < kMCfgsAuto; ++c)
      if (n >= kMCfgs[c].nmin && n <= kMCfgs[c].nmax) g.cfg = c;
  }
  if (getenv("ITR_MCFG")) {
    const int c = atoi(getenv("ITR_MCFG"));
    if (c >= 0 && c < (int)(sizeof kMCfgs / sizeof kMCfgs[0]) && n >= kMCfgs[c].nmin &&
        n <= kMCfgs[c].nmax)
      g.cfg = c;
  }
#endif
  if (g.cfg < 0) return g;
  g.block = 64 * kMCfgs[g.cfg].nt;
  g.xr = 16 * kMCfgs[g.cfg].nt;
  g.gb = kMCfgs[g.cfg].gb;
  g.pfrac = kMCfgs[g.cfg].pfrac;
  g.bfrac = kMCfgs[g.cfg].bfrac;
  g.lofrac = kMCfgs[g.cfg].lofrac;
#ifdef ITR_EXPERIMENT
  if (getenv("ITR_POST_URGENT_FRAC")) g.pfrac = atof(getenv("ITR_POST_URGENT_FRAC"));
#endif
  int occ = 1;
  (void)dispatch_mode_m(mode, g.cfg, false, nullptr, nullptr, 0, 0, nullptr, &occ);
  g.per_cu = occ;
  return g;
}

hipError_t launch_hybrid_sweep(int mode, const MfmaGeometry& g, int grid, const MfmaArgs& a,
                               const SweepArgs& v, hipStream_t st) {
  int occ = 0;
  return dispatch_mode_m(mode, g.cfg, true, &a, &v, grid, g.lds_min, st, &occ);
}

}  // namespace itr
