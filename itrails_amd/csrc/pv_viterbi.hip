// pv_viterbi.hip — the Viterbi sweep (optimizer.py:305-333) by PREDICTION AND VERIFICATION on
// MI355X (gfx950).  One wavefront decodes one block at a time; the waves of a workgroup share
// log a in LDS.  Device code written for this chip (no CUDA counterpart: the reference's
// sweep is a numba loop).
//
// The recursion omega_t[j] = max_i fl(fl(omega_{t-1}[i] + log a_ij) + log e_j(t)) is a
// chain of N x N max-plus steps whose latency bounds a block.  But the maximising source of
// almost every target is the same as one column earlier (the target itself for a stay, the
// same source for a refresh): on the (5,5) bench workload 97 % of the columns keep every
// target's maximising source (scripts/pv_stats.py).  So a window of up to 8 columns is
//
//   1. PREDICTED: v_t[j] = fl(fl(v_{t-1}[p_j] + log a_{p_j j}) + log e_j(t)), p_j the
//      target's last known maximising source: one add pair per target and column, the
//      value the reference computes for source p_j, bit for bit;
//   2. VERIFIED, all columns of the window at once (they are independent given the
//      predicted rows): a stay-predicted target passes when
//        v_t[j] > fl(fl(max_i v_{t-1}[i] + M_j) + log e_j(t)),   M_j = max_{i != j} log a_ij,
//      which bounds every other source (rounding is monotone): then j is the unique maximum,
//      omega_t[j] = v_t[j] and the stay flag is set.  ~85 % of the (column, target) pairs pass;
//      the others are compacted into a list and SCANNED exactly, one lane per pair
//      (yo = fl(max_{i != j} fl(v_{t-1}[i] + log a_ij) + log e_j), the form the other sweeps
//      use: omega = max(yd, yo), stay = yd > yo);
//   3. COMMITTED up to the first column whose scanned value differs from the prediction;
//      that column takes the exact values, the mispredicted targets take their new
//      maximising source, and the next window starts after it.
//
// Every committed value is the reference's value for that column (the verification proves
// it from exact inputs), so the outputs — omega at every 16-column tile's first column, the
// 16-bit stay-flag words, the last column's first argmax — are those of the other Viterbi
// sweeps bit for bit, and the traceback (hmm_sweeps.hip) is shared.
//
// Layout: lane l owns targets j = 64 s + l (s < NS slots).  Per wave in LDS: the value rows
// of the window [PV_K + 1][rss] (row k = column cb + k - 1 of the half-tile starting at cb),
// the half-tile's emission rows (direct-to-LDS loads from log E padded to xe columns), the
// per-target flag/misprediction bits, the pair list and the block's symbols.  Per workgroup:
// log a^T with a -inf diagonal (row stride rsa = 2 mod 4: 16 lanes reading 16 different
// target rows with ds_read_b128 hit distinct banks) and the diagonal.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {
namespace {

constexpr int PV_K = 8;  // columns per window at most = columns per staged emission half-tile
typedef double pv_d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int pv_lane() {  // opaque to hoisting out of the task loop
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ int mbcnt64(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Diagnostic build only (-DITR_DIAG): per block, lane 0 adds event counts and shader-clock
// cycles per phase into a.diag: [0] windows, [1] committed columns, [2] mispredicted
// windows, [3] scanned pairs, [4] windows with a gather, [8..12] cycles of prediction,
// tests + compaction, scans, commit, misprediction repair
#ifdef ITR_DIAG
#define PV_DIAG_DECL uint64_t dg[16] = {}; uint64_t dt = __builtin_amdgcn_s_memtime();
#define PV_CNT(i, v) (dg[i] += (uint64_t)(v))
#define PV_T(i)                                            \
  do {                                                     \
    __builtin_amdgcn_sched_barrier(0);                     \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();    \
    __builtin_amdgcn_sched_barrier(0);                     \
    dg[i] += now_ - dt;                                    \
    dt = now_;                                             \
  } while (0)
#define PV_FLUSH()                                                                   \
  do {                                                                               \
    if (l == 0 && a.diag)                                                            \
      for (int i_ = 0; i_ < 16; ++i_)                                                \
        if (dg[i_]) atomicAdd((unsigned long long*)&a.diag[i_], (unsigned long long)dg[i_]); \
  } while (0)
#else
#define PV_DIAG_DECL
#define PV_CNT(i, v)
#ifdef PV_MARKS
#define PV_T(i) asm volatile(";;PVMARK " #i ::: "memory")
#else
#define PV_T(i)
#endif
#define PV_FLUSH()
#endif

// Margin bookkeeping.  A target j is predicted from a PAIR of sources {q1, q2} (a stay is
// q = j): its value is fl(max(c_q1, c_q2) + log e_j), c_i = omega_{t-1}[i] + log a_ij, which is
// the reference's value whenever the maximising source is in the pair.  M = max(c_q1, c_q2) -
// max_{i not in pair} c_i > 0 proves it.  From one column to the next every candidate moves by
// its source's exact change d_i = omega_t[i] - omega_{t-1}[i], so
// M' >= M + min(d_q1, d_q2) - max_i d_i: a lower bound L on M carries over with a few adds per
// column and is reset from an exact scan (the three largest candidates).  L only ever
// decreases relative to M; a test passes when L exceeds a margin that covers the rounding of
// the additions involved (1e-6 + |omega| 2^-36).
// SAFE: some omega can be -inf (zero emissions, unreachable states): the infinities get
// their own cases; otherwise (every state reachable, every emission positive: the iTRAILS
// models) the plain differences are exact enough and carry no NaN
template <bool SAFE>
__device__ __forceinline__ double pv_delta(double now, double before) {
  if constexpr (SAFE) return now == -INFINITY ? -INFINITY : now - before;  // +inf: appears
  return now - before;
}
template <bool SAFE>
__device__ __forceinline__ double pv_adv(double L, double dp, double dm) {
  if constexpr (SAFE) {
    const double D = (dm == INFINITY || dp == -INFINITY) ? -INFINITY : dp - dm;
    return L + D;
  }
  return L + (dp - dm);
}
__device__ __forceinline__ double pv_margin(double top1, double top3) {
  return top3 == -INFINITY ? (top1 == -INFINITY ? -INFINITY : 1e300) : top1 - top3;
}
// top three of the union of two sorted triples (k-th largest = max_{i+j=k} min(a_i, b_j))
__device__ __forceinline__ void top3_merge(double& a1, double& a2, double& a3, double b1, double b2,
                                           double b3) {
  const double x1 = fmax(a1, b1);
  const double x2 = fmax(fmax(a2, b2), fmin(a1, b1));
  const double x3 = fmax(fmax(a3, b3), fmax(fmin(a1, b2), fmin(a2, b1)));
  a1 = x1;
  a2 = x2;
  a3 = x3;
}
template <int CTRL>
__device__ __forceinline__ void top3_dpp(double& a1, double& a2, double& a3) {
  top3_merge(a1, a2, a3, dpp_f64<CTRL>(a1), dpp_f64<CTRL>(a2), dpp_f64<CTRL>(a3));
}

template <int NS, bool SAFE>
__device__ __forceinline__ void pv_task(const PvArgs& a, double* wl, const double* LAT, int blk,
                                        const double (&ld)[NS]) {
  const int l = pv_lane();
  const int n = a.n, rss = a.rss, rs = a.rs, xe = a.xe, rsa = a.rsa;
  double* S = wl;                                           // [PV_K + 1][rss] value rows
  double* EC = S + (PV_K + 1) * rss;                        // [16][rs] log e ring (column & 15)
  double* SINK = EC + 16 * rs;                              // [64] stores of lanes without a slot
  double* PRV = SINK + 64;                                  // [lcap][2] pairs' omega, margin
  uint32_t* FB = reinterpret_cast<uint32_t*>(PRV + 2 * a.lcap);  // [rs + 64] flags | mis << 16
  int* PRI = reinterpret_cast<int*>(FB + rs + 64);          // [lcap] pairs' new sources i1 | i2 << 8
  uint16_t* LIST = reinterpret_cast<uint16_t*>(PRI + a.lcap);  // [lcap] pairs (r << 8 | j)
  uint16_t* SYM = LIST + a.lcap;                            // [2][64] observed symbols

  const int64_t c0 = uni64(a.off[blk]);
  const int T = uni((int)(a.off[blk + 1] - c0));
  if (T <= 0) return;
  const bool urgent = T >= a.prio_len;
  if (urgent) __builtin_amdgcn_s_setprio(3);
  const uint16_t* ob = a.obs + c0;
  // symbols: 64-column chunks, two resident in SYM, the next one in flight in `sin` (clamped
  // into the alphabet when committed: memory safety only, the host rejects such symbols)
  auto symg = [&](int c) -> int { return (int)ob[min(c, T - 1)]; };
  auto clamp_sym = [](int v) -> uint16_t { return (uint16_t)min(v, 624); };
  SYM[l] = clamp_sym(symg(l));
  SYM[64 + l] = clamp_sym(symg(64 + l));
  int sin = symg(128 + l);
  wave_lds_sync();
  auto sym = [&](int c) -> int { return SYM[((c >> 6) & 1) * 64 + (c & 63)]; };

  // slot s of lane l: target jt = 64 s + l; a lane whose target is outside the LDS rows
  // stores into SINK and reads a clamped column (its values are -inf and never counted)
  int jt[NS], jc[NS], je[NS];
  bool act[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    jt[s] = 64 * s + l;
    act[s] = jt[s] < n;
    jc[s] = min(jt[s], rs - 1);
    je[s] = min(jt[s], xe - 1);
  }
  auto slot = [&](double* base, int s) -> double* {  // this lane's entry of a row (or SINK)
    return jt[s] < rs ? base + jt[s] : SINK + l;
  };
  // log e rows: half-tile hp (8 columns) into registers by global loads issued a half-tile
  // ahead, then into the ring EC; hb = the last half-tile in the ring
  double en[PV_K][NS];
  auto e_issue = [&](int hp) {
    if ((hp & 7) == 0 && hp > 0) {  // a new 64-column chunk: the next one in, one requested
      SYM[((((hp >> 3)) + 1) & 1) * 64 + l] = clamp_sym(sin);
      sin = symg(64 * (hp >> 3) + 128 + l);
      wave_lds_sync();
    }
#pragma unroll
    for (int k = 0; k < PV_K; ++k) {
      const double* row = a.lep + (int64_t)sym(PV_K * hp + k) * xe;
#pragma unroll
      for (int s = 0; s < NS; ++s) en[k][s] = row[je[s]];
    }
  };
  auto e_commit = [&](int hp) {  // half-tile hp's rows (in en) into the ring
#pragma unroll
    for (int k = 0; k < PV_K; ++k)
#pragma unroll
      for (int s = 0; s < NS; ++s)
        *slot(EC + ((PV_K * hp + k) & 15) * rs, s) = act[s] ? en[k][s] : -INFINITY;
  };
  // checkpoint rows / flag words of this block (records from tile tk0), buffer stores: a
  // lane without a target stores out of bounds (nothing)
  const int64_t tk0 = uni64(a.tile_off[blk]);
  const int xr = a.xr;
  const uint32_t nrec = (uint32_t)((T + VIT_TILE - 1) / VIT_TILE * xr);
  const __amdgpu_buffer_rsrc_t rck = buf_rsrc(a.ckpt + tk0 * xr, nrec * 8);
  const __amdgpu_buffer_rsrc_t rst = buf_rsrc(a.stay + tk0 * xr, nrec * 2);
  uint32_t vo[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) vo[s] = act[s] ? (uint32_t)jt[s] : kOffNone / 8;

  // omega_0 = log(pi e_0)  (optimizer.py:317-318): tile 0's checkpoint
  double x[NS];
  {
    const int o0 = sym(0);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      x[s] = act[s] ? a.lpie[o0 * n + jt[s]] : -INFINITY;
      buf_store_f64(rck, vo[s] * 8, 0, x[s]);
    }
  }
  // the ring starts with half-tiles 0 and 1; half-tile 2 in flight
  e_issue(0);
  vm_wait_all();
  e_commit(0);
  int hb = 0;
  if (PV_K < T) {
    e_issue(1);
    vm_wait_all();
    e_commit(1);
    hb = 1;
    if (2 * PV_K < T) e_issue(2);
  }
  // predicted source pairs (first: the stay twice), their log a, the margin bound L at the
  // next column (-inf: unknown, so the first column of every block is scanned)
  int q1[NS], q2[NS];
  double la1[NS], la2[NS], L[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    q1[s] = q2[s] = jc[s];
    la1[s] = la2[s] = ld[s];
    L[s] = -INFINITY;
  }
  uint32_t flw[NS];  // stay flags of tiles ft and ft + 1 (bit c - 16 ft)
#pragma unroll
  for (int s = 0; s < NS; ++s) flw[s] = 0;
  int ft = 0;
  const int ch = rs >> 3;  // states per lane of the row-maximum pass and the refresh (8 lanes)
  const int gq = l & 7, gp = l >> 3;
  const int c4 = rs >> 2;  // sources per scanning lane (4 lanes per pair)
  const int hq = l & 3, hp = l >> 2;

  PV_DIAG_DECL
  int cw = 1;  // first column of the window (column cw - 1 is committed: x)
  while (cw < T) {
    PV_CNT(0, 1);
    PV_T(13);
    const int nk = min(PV_K, T - cw);  // window columns; row r = column cw + r - 1
    // the ring must hold the window's last column's half-tile
    if (((cw + nk - 1) >> 3) > hb) {
      vm_wait_all();
      ++hb;
      e_commit(hb);
      if (PV_K * (hb + 1) < T) e_issue(hb + 1);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      *slot(S, s) = x[s];  // row 0: the committed column
      FB[jt[s] < rs ? jt[s] : rs + l] = 0u;
    }
    wave_lds_sync();
    // ---- 1. prediction: v = max(c_q1, c_q2) + log e (c_q = omega[q] + log a_qj); pf: the
    // predicted stay flags (j the strict maximum of the pair); md: min(d_q1, d_q2) from row
    // r - 1 to r (d_q = the source's change)
    double e[PV_K][NS];
#pragma unroll
    for (int r = 1; r <= PV_K; ++r)
#pragma unroll
      for (int s = 0; s < NS; ++s) e[r - 1][s] = EC[((cw + r - 1) & 15) * rs + jc[s]];
    uint32_t pf[NS];
    double md[PV_K][NS], g1[NS], g2[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      pf[s] = 0;
      g1[s] = S[q1[s]];
      g2[s] = S[q2[s]];
    }
#pragma unroll
    for (int r = 1; r <= PV_K; ++r) {
      if (r > nk) break;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double c1 = g1[s] + la1[s], c2 = g2[s] + la2[s];
        const double v = fmax(c1, c2) + e[r - 1][s];
        const bool st = ((q1[s] == jt[s]) & ((q2[s] == jt[s]) | (c1 > c2))) |
                        ((q2[s] == jt[s]) & (c2 > c1));
        pf[s] |= (uint32_t)st << r;
        *slot(S + r * rss, s) = act[s] ? v : -INFINITY;
      }
      wave_lds_sync();
      double h1[NS], h2[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        h1[s] = S[r * rss + q1[s]];
        h2[s] = S[r * rss + q2[s]];
      }
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        md[r - 1][s] = fmin(pv_delta<SAFE>(h1[s], g1[s]), pv_delta<SAFE>(h2[s], g2[s]));
        g1[s] = h1[s];
        g2[s] = h2[s];
      }
    }
    PV_T(8);
    // ---- 2. verification ------------------------------------------------------------------
    // the largest change from row q = l >> 3 to row q + 1 over the chunk l & 7 of rs / 8
    // states, combined over the chunk lanes by DPP: lane 8 q holds it
    double dmx;
    {
      const double* row = S + gp * rss + gq * ch;
      double d0 = -INFINITY, d1 = -INFINITY;
#pragma unroll 4
      for (int q = 0; q < ch; q += 2) {
        const pv_d2 v = *reinterpret_cast<const pv_d2*>(row + q);
        const pv_d2 w = *reinterpret_cast<const pv_d2*>(row + rss + q);
        d0 = fmax(d0, pv_delta<true>(w.x, v.x));  // (the row padding is -inf)
        d1 = fmax(d1, pv_delta<true>(w.y, v.y));
      }
      dmx = fmax(d0, d1);
      dmx = fmax(dmx, dpp_f64<DPP_Q1>(dmx));
      dmx = fmax(dmx, dpp_f64<DPP_Q2>(dmx));
      dmx = fmax(dmx, dpp_f64<DPP_HM>(dmx));
    }
    // tests: the carried bound of every (column, target); fb: failing rows (bit r)
    uint32_t fb[NS];
    double L0[NS], thr[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      fb[s] = 0;
      L0[s] = L[s];
      thr[s] = 1e-6 + fabs(x[s]) * 0x1p-36;
    }
#pragma unroll
    for (int r = 1; r <= PV_K; ++r) {
      if (r > nk) break;
      const double dm = lane_f64(dmx, 8 * (r - 1));
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        fb[s] |= (uint32_t)(act[s] & !(L[s] > thr[s])) << r;
        L[s] = pv_adv<SAFE>(L[s], md[r - 1][s], dm);
      }
    }
    // pairs in (row, slot, lane) order; the list holds at most lcap pairs: the window ends
    // before the row that would overflow it (one row has at most 64 NS = lcap pairs)
    int ncut = nk, npairs = 0;
#pragma unroll
    for (int r = 1; r <= PV_K; ++r) {
      if (r > ncut) break;
      uint64_t m[NS];
      int cr = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        m[s] = __ballot((fb[s] >> r) & 1u);
        cr += __popcll(m[s]);
      }
      if (npairs + cr > a.lcap) {
        ncut = r - 1;
      } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          if ((fb[s] >> r) & 1u) LIST[npairs + mbcnt64(m[s])] = (uint16_t)((r << 8) | jt[s]);
          npairs += __popcll(m[s]);
        }
      }
    }
    wave_lds_sync();
    PV_T(9);
    PV_CNT(3, npairs);
    // exact scans, four lanes per pair (lane l & 3 takes sources [c4 (l & 3), +c4)): the
    // three largest candidates c_i = omega[i] + log a_ij over all i (the stay included), then
    // omega = fl(top1 + log e), the stay flag (c_j = top1 > top2), the misprediction, the
    // margin top1 - top3 of the top pair
    int rmis = PV_K + 1;  // first mispredicted row (none: PV_K + 1)
    for (int r0 = 0; r0 < npairs; r0 += 16) {
      const int idx = r0 + hp;
      const bool valid = idx < npairs;
      const int code = LIST[valid ? idx : 0];
      const int r = code >> 8, jj = code & 255;
      const double* sr = S + (r - 1) * rss + hq * c4;
      const double* lr = LAT + jj * rsa + hq * c4;
      double v1 = -INFINITY, v2 = -INFINITY, v3 = -INFINITY;
#pragma unroll 5
      for (int i = 0; i < c4; i += 2) {
        const pv_d2 sv2 = *reinterpret_cast<const pv_d2*>(sr + i);
        const pv_d2 lv2 = *reinterpret_cast<const pv_d2*>(lr + i);
        const double ca = sv2.x + lv2.x, cc = sv2.y + lv2.y;
        v3 = fmax(v3, fmin(v2, ca));
        v2 = fmax(v2, fmin(v1, ca));
        v1 = fmax(v1, ca);
        v3 = fmax(v3, fmin(v2, cc));
        v2 = fmax(v2, fmin(v1, cc));
        v1 = fmax(v1, cc);
      }
      top3_dpp<DPP_Q1>(v1, v2, v3);
      top3_dpp<DPP_Q2>(v1, v2, v3);
      const double* srow = S + (r - 1) * rss;
      const double ee = EC[((cw + r - 1) & 15) * rs + jj];
      const double cj = srow[jj] + LAT[jj * rsa + jj];
      const double ex = v1 + ee;
      const bool flg = (cj == v1) & (v1 > v2);
      const bool mis = valid & (ex != srow[rss + jj]);
      const bool lead = valid & (hq == 0);
      const uint32_t bits = (flg ? 1u << r : 0u) | (mis ? 1u << (16 + r) : 0u);
      if (lead & (bits != 0u)) atomicOr(&FB[jj], bits);
      if (lead) {
        PRV[2 * idx] = ex;
        PRV[2 * idx + 1] = pv_margin(v1, v3);
      }
      const uint64_t mb = __ballot(mis & (hq == 0));
      if (mb && rmis > PV_K) rmis = __builtin_amdgcn_readlane(r, __builtin_ctzll(mb));
    }
    PV_T(10);
    // ---- 3. commit rows 1 .. nc (up to the first mispredicted one) -------------------------
    const int nc = rmis <= PV_K ? rmis : ncut;
    // the pairs of row nc: [p0, p1) of the list (the list is in row order)
    int p0 = 0, p1 = 0;
#pragma unroll
    for (int r = 1; r <= PV_K; ++r) {
      if (r > ncut) break;
      int cr = 0;
#pragma unroll
      for (int s = 0; s < NS; ++s) cr += __popcll(__ballot((fb[s] >> r) & 1u));
      if (r < nc) p0 += cr;
      if (r <= nc) p1 += cr;
    }
    wave_lds_sync();
    double dml = lane_f64(dmx, 8 * (nc - 1));  // largest change from row nc - 1 to row nc
    if (rmis <= PV_K) {
      // corrected values of row nc (they only ever rise: the largest change grows by theirs)
      double dcor = -INFINITY;
      for (int i0 = p0; i0 < p1; i0 += 64) {
        const int idx = i0 + l;
        if (idx < p1) {
          const int jj = LIST[idx] & 255;
          const double ex = PRV[2 * idx];
          if ((FB[jj] >> (16 + nc)) & 1u) {
            dcor = fmax(dcor, pv_delta<SAFE>(ex, S[(nc - 1) * rss + jj]));
            S[nc * rss + jj] = ex;
          }
        }
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) dcor = fmax(dcor, __shfl_xor(dcor, d));
      dml = fmax(dml, dcor);
    }
    // new source pairs of the targets scanned at row nc: the first index reaching top1 and the
    // first other index reaching top2 (eight lanes per pair)
    for (int r0 = p0; r0 < p1; r0 += 8) {
      const int idx = r0 + gp;
      const bool valid = idx < p1;
      const int jj = LIST[valid ? idx : p0] & 255;
      const double* sr = S + (nc - 1) * rss + gq * ch;
      const double* lr = LAT + jj * rsa + gq * ch;
      double cv[16];
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        cv[i] = cv[i + 1] = -INFINITY;
        if (i < ch) {
          const pv_d2 sv2 = *reinterpret_cast<const pv_d2*>(sr + i);
          const pv_d2 lv2 = *reinterpret_cast<const pv_d2*>(lr + i);
          cv[i] = sv2.x + lv2.x;
          cv[i + 1] = sv2.y + lv2.y;
        }
      }
      double v1 = -INFINITY, v2 = -INFINITY, v3 = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v3 = fmax(v3, fmin(v2, cv[i]));
        v2 = fmax(v2, fmin(v1, cv[i]));
        v1 = fmax(v1, cv[i]);
      }
      top3_dpp<DPP_Q1>(v1, v2, v3);
      top3_dpp<DPP_Q2>(v1, v2, v3);
      top3_dpp<DPP_HM>(v1, v2, v3);
      int f1 = 0x7fff;
#pragma unroll
      for (int i = 15; i >= 0; --i) f1 = cv[i] == v1 ? gq * ch + i : f1;
      f1 = min(f1, dpp_i32<DPP_Q1>(f1));
      f1 = min(f1, dpp_i32<DPP_Q2>(f1));
      f1 = min(f1, dpp_i32<DPP_HM>(f1));
      int f2 = 0x7fff;
#pragma unroll
      for (int i = 15; i >= 0; --i) f2 = (cv[i] == v2 && gq * ch + i != f1) ? gq * ch + i : f2;
      f2 = min(f2, dpp_i32<DPP_Q1>(f2));
      f2 = min(f2, dpp_i32<DPP_Q2>(f2));
      f2 = min(f2, dpp_i32<DPP_HM>(f2));
      if (valid & (gq == 0)) PRI[idx] = min(f1, n - 1) | min(f2, n - 1) << 8;
    }
    wave_lds_sync();
    const int c1 = cw + nc;                           // first uncommitted column
    const uint32_t wm = ((2u << nc) - 1u) & ~1u;      // rows 1 .. nc
    const int sh = cw - 1 - 16 * ft;                  // row r -> flag bit r + sh
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint32_t fbw = FB[jt[s] < rs ? jt[s] : rs + l];
      const uint32_t fl = ((pf[s] & ~fb[s]) | fbw) & wm;
      flw[s] |= act[s] ? fl << sh : 0u;
      x[s] = act[s] ? S[nc * rss + jc[s]] : -INFINITY;
      // the bound at the next column: carried over the committed rows, or from the scan of
      // row nc with the new pair's changes from row nc - 1 to row nc
      double Lb = L0[s], mdl = 0.0;
      bool done = false;  // Lb is already the bound at the next column
      if (nc == nk && rmis > PV_K) {  // the whole window committed: the tests' bound
        Lb = L[s];
        done = true;
      } else {
#pragma unroll
        for (int r = 1; r <= PV_K; ++r) {
          if (r > nc) break;
          if (r < nc) Lb = pv_adv<SAFE>(Lb, md[r - 1][s], lane_f64(dmx, 8 * (r - 1)));
          else mdl = md[r - 1][s];
        }
      }
      const bool scl = act[s] & (((fb[s] >> nc) & 1u) != 0u);
      if (__ballot(scl)) {
        // this target's pair index: p0 + the pairs of row nc before it (slot order, lanes)
        int pos = p0 + mbcnt64(__ballot(scl));
#pragma unroll
        for (int s2 = 0; s2 < NS; ++s2)
          if (s2 < s) pos += __popcll(__ballot(act[s2] & (((fb[s2] >> nc) & 1u) != 0u)));
        pos = scl ? pos : p0;
        const int pr = PRI[pos];
        const int n1 = pr & 255, n2 = (pr >> 8) & 255;
        const double mg = PRV[2 * pos + 1];
        const double b1 = S[(nc - 1) * rss + n1], b2 = S[(nc - 1) * rss + n2];
        const double e1 = S[nc * rss + n1], e2 = S[nc * rss + n2];
        const double nl1 = LAT[jc[s] * rsa + n1], nl2 = LAT[jc[s] * rsa + n2];
        if (scl) {
          q1[s] = n1;
          q2[s] = n2;
          la1[s] = nl1;
          la2[s] = nl2;
          Lb = mg;
          mdl = fmin(pv_delta<SAFE>(e1, b1), pv_delta<SAFE>(e2, b2));
          done = false;
        }
      }
      L[s] = done ? Lb : pv_adv<SAFE>(Lb, mdl, dml);
    }
    // a tile's first column committed: its checkpoint row; a tile complete: its flag words
    {
      const int tc = 16 * ((cw + 15) >> 4);  // first tile column at or after cw
      if (tc < c1) {
        const int r = tc - cw + 1;
#pragma unroll
        for (int s = 0; s < NS; ++s)
          buf_store_f64(rck, vo[s] * 8, (uint32_t)((tc >> 4) * xr) * 8, S[r * rss + jc[s]]);
      }
      if (c1 >= 16 * (ft + 1)) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          buf_store_u16(rst, vo[s] * 2, (uint32_t)(ft * xr) * 2, (uint16_t)flw[s]);
          flw[s] >>= 16;
        }
        ++ft;
      }
    }
    PV_T(11);
    PV_CNT(1, nc);
    PV_CNT(2, rmis <= PV_K);
    cw = c1;
  }
  if (16 * ft < T) {  // the last tile's flag words
#pragma unroll
    for (int s = 0; s < NS; ++s) buf_store_u16(rst, vo[s] * 2, (uint32_t)(ft * xr) * 2, (uint16_t)flw[s]);
  }
  // last state = first argmax of omega_{T-1}  (optimizer.py:346)
  double bv = act[0] ? x[0] : -INFINITY;
  int bj = act[0] ? jt[0] : 0x7fffffff;
#pragma unroll
  for (int s = 1; s < NS; ++s) {
    const bool b = act[s] & (x[s] > bv);
    bv = b ? x[s] : bv;
    bj = b ? jt[s] : bj;
  }
  wave_first_max(bv, bj);
  if (l == 0) a.last_state[blk] = (uint8_t)bj;
  PV_FLUSH();
  if (urgent) __builtin_amdgcn_s_setprio(0);
}

// Every lane takes part in the queue atomic (lane 0 adds 1): see wave_sweeps.hip.  The
// first task of every wave is static — wave w of workgroup g takes order[w * grid + g] — so
// the longest blocks spread over the CUs one per workgroup before any CU gets a second.
__device__ __forceinline__ int pv_next(int* queue, int base) {
  return base + uni(atomicAdd(queue, (threadIdx.x & 63) == 0 ? 1 : 0));
}

template <int NS, bool SAFE>
__global__ void __launch_bounds__(NS == 1 ? 512 : 256) pv_vit_kernel(PvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* LAT = reinterpret_cast<double*>(smem);  // log a^T, rows padded to rsa with -inf
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < a.n * a.rsa; i += nt) LAT[i] = a.lat[i];
  __syncthreads();
  double* wl = LAT + (size_t)a.n * a.rsa + (size_t)(tid >> 6) * a.wl;
  const int l = tid & 63;
  double ld[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int j = 64 * s + l;
    ld[s] = j < a.n ? a.ldg[j] : -INFINITY;
  }
  const int waves = nt >> 6, grid = gridDim.x;
  int bi = (tid >> 6) * grid + blockIdx.x;  // static first task
  const int dyn = waves * grid;
  while (bi < a.nblocks) {
    pv_task<NS, SAFE>(a, wl, LAT, uni(a.order[bi]), ld);
    bi = pv_next(a.queue, dyn);
  }
}

}  // namespace

PvGeometry pv_geometry(int n) {
  PvGeometry g{};
  g.ns = -1;
  if (n < 1 || n > 128) return g;
  const int ns = (n + 63) / 64;
  const int rs = (n + 15) & ~15;          // value row width (multiple of 16: 8 chunks of even size)
  const int rss = rs + 2;                 // its stride (= 2 mod 4)
  const int rsa = rs + 2;                 // log a^T row stride
  const int xe = (n + 1) & ~1;            // padded log-emission row
  const int lcap = 64 * ns;               // pairs scanned per window at most
  // per wave: value rows, the log e ring (16 columns), sink, pair results (2 doubles + 1 int), flag
  // words (rs + 64), pair list, symbols
  const int wl = ((PV_K + 1) * rss + 16 * rs + 64 + 2 * lcap + (rs + 64) / 2 + lcap / 2 +
                  lcap / 4 + 32 + 1) & ~1;
  const int shared = n * rsa;
  const int budget = 160 * 1024 / 8 - shared;
  const int waves = std::min(ns == 1 ? 8 : 4, budget / wl);  // (the launch bounds)
  if (waves < 1) return g;
  g.ns = ns;
  g.waves = waves;
  g.block = 64 * waves;
  g.rsa = rsa;
  g.rs = rs;
  g.rss = rss;
  g.xe = xe;
  g.eb = 0;
  g.lcap = lcap;
  g.wl = wl;
  g.lds = (size_t)(shared + waves * wl) * sizeof(double);
  return g;
}

hipError_t launch_pv_vit(const PvGeometry& g, int grid, PvArgs a, hipStream_t st) {
  if (a.nblocks <= 0) return hipSuccess;
  a.rsa = g.rsa;
  a.rs = g.rs;
  a.rss = g.rss;
  a.xe = g.xe;
  a.eb = g.eb;
  a.lcap = g.lcap;
  a.wl = g.wl;
  switch (g.ns) {
    case 1:
      if (a.safe)
        hipLaunchKernelGGL((pv_vit_kernel<1, true>), dim3(grid), dim3(g.block), g.lds, st, a);
      else
        hipLaunchKernelGGL((pv_vit_kernel<1, false>), dim3(grid), dim3(g.block), g.lds, st, a);
      break;
    case 2:
      if (a.safe)
        hipLaunchKernelGGL((pv_vit_kernel<2, true>), dim3(grid), dim3(g.block), g.lds, st, a);
      else
        hipLaunchKernelGGL((pv_vit_kernel<2, false>), dim3(grid), dim3(g.block), g.lds, st, a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace itr
