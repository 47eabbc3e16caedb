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
#define PV_T(i)
#define PV_FLUSH()
#endif

// Margin bookkeeping.  For a target j with predicted source p, M = c_p - max_{i != p} c_i
// over the candidates c_i = omega_{t-1}[i] + log a_ij (c_j = the stay); M > 0 proves p the
// unique maximum.  From one column to the next every candidate moves by its source's exact
// change d_i = omega_t[i] - omega_{t-1}[i], so M' >= M + d_p - max_i d_i: a lower bound L
// on M carries over with two adds per column and is reset from a scan (top-2 of the
// candidates).  L only ever decreases relative to M; a test passes when L exceeds a margin
// that covers the rounding of the additions involved (thr below).
__device__ __forceinline__ double pv_delta(double now, double before) {
  return now == -INFINITY ? -INFINITY : now - before;  // +inf when a source appears
}
__device__ __forceinline__ double pv_adv(double L, double dp, double dm) {
  const double D = (dm == INFINITY || dp == -INFINITY) ? -INFINITY : dp - dm;
  return L + D;
}
__device__ __forceinline__ double pv_margin(double top1, double top2) {
  return top2 == -INFINITY ? (top1 == -INFINITY ? -INFINITY : 1e300) : top1 - top2;
}

template <int NS>
__device__ __forceinline__ void pv_task(const PvArgs& a, double* wl, const double* LAT,
                                        const double* LDG, int blk, const double (&ld)[NS],
                                        const double (&mj)[NS]) {
  const int l = pv_lane();
  const int n = a.n, rss = a.rss, rs = a.rs, xe = a.xe, rsa = a.rsa;
  double* S = wl;                                          // [PV_K + 1][rss] value rows
  double* EC = S + (PV_K + 1) * rss;                       // [PV_K][rs] the half-tile's log e
  double* MG = EC + PV_K * rs;                             // [rs] scanned margins
  double* SINK = MG + rs;                                  // [64] stores of lanes without a slot
  uint32_t* FB = reinterpret_cast<uint32_t*>(SINK + 64);   // [rs + 64] flags | mis << 16
  int* WIN = reinterpret_cast<int*>(FB + rs + 64);         // [rs] new maximising sources
  uint16_t* LIST = reinterpret_cast<uint16_t*>(WIN + rs);  // [lcap] pairs (k << 8 | j)
  uint16_t* SYM = LIST + a.lcap;                           // [2][64] observed symbols

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
  auto row_st = [&](int row, int s) -> double* {  // this lane's slot in a value row (or SINK)
    return jt[s] < rs ? S + row * rss + jt[s] : SINK + l;
  };
  // log e rows of half-tile h into registers (global loads, waited for a half-tile later)
  double en[PV_K][NS];
  auto e_issue = [&](int h) {
#pragma unroll
    for (int k = 0; k < PV_K; ++k) {
      const double* row = a.lep + (int64_t)sym(PV_K * h + k) * xe;
#pragma unroll
      for (int s = 0; s < NS; ++s) en[k][s] = row[je[s]];
    }
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
  e_issue(0);
  // predicted maximising sources: the target itself (stay) until a scan shows otherwise;
  // L: lower bound on the prediction's margin at the next column (-inf: unknown)
  int p[NS];
  double lap[NS], L[NS];
  bool stayp[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    p[s] = jc[s];
    lap[s] = ld[s];
    stayp[s] = act[s];
    L[s] = -INFINITY;
  }
  bool anysw = false;  // some target predicted from another source (gather through LDS)
  uint32_t flw[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) flw[s] = 0;
  double sv[PV_K + 1][NS];
#pragma unroll
  for (int k = 0; k <= PV_K; ++k)
#pragma unroll
    for (int s = 0; s < NS; ++s) sv[k][s] = -INFINITY;
  const int np = (n + 3) & ~3;  // scanned sources (padding -inf in both operands)

  PV_DIAG_DECL
  for (int h = 0; PV_K * h < T; ++h) {
    const int cb = PV_K * h;  // first column of the half-tile
    vm_wait_all();            // en holds half-tile h (and sin has arrived)
#pragma unroll
    for (int k = 0; k < PV_K; ++k)
#pragma unroll
      for (int s = 0; s < NS; ++s) *(jt[s] < rs ? EC + k * rs + jt[s] : SINK + l) = act[s] ? en[k][s] : -INFINITY;
    if ((cb & 63) == 0 && cb > 0) {  // next symbol chunk in, the one after requested
      SYM[(((cb >> 6) + 1) & 1) * 64 + l] = clamp_sym(sin);
      sin = symg(cb + 128 + l);
    }
    wave_lds_sync();
    // this lane's log e of a half-tile column (padding lanes: -inf)
    auto ecol = [&](int k, int s) -> double { return act[s] ? EC[k * rs + jc[s]] : -INFINITY; };
    if (cb + PV_K < T) e_issue(h + 1);
    int kstart = h == 0 ? 1 : 0;
    const int kend = min(PV_K, T - cb);
    while (kstart < kend) {
      PV_CNT(0, 1);
      PV_CNT(4, anysw);
      PV_T(13);
      // ---- 1. prediction of columns cb + kstart .. cb + kend - 1 -----------------------
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        *row_st(kstart, s) = x[s];  // the committed column: row kstart
        FB[jt[s] < rs ? jt[s] : rs + l] = 0u;
      }
#pragma unroll
      for (int k = 0; k < PV_K; ++k)
        if (k == kstart) {
#pragma unroll
          for (int s = 0; s < NS; ++s) sv[k][s] = x[s];
        }
#pragma unroll
      for (int k = 0; k < PV_K; ++k) {
        if (k >= kstart && k < kend) {
          double src[NS];
          if (anysw) {
            wave_lds_sync();
#pragma unroll
            for (int s = 0; s < NS; ++s) src[s] = S[k * rss + p[s]];
          } else {
#pragma unroll
            for (int s = 0; s < NS; ++s) src[s] = sv[k][s];
          }
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            const double v = (src[s] + lap[s]) + ecol(k, s);
            sv[k + 1][s] = v;
            *row_st(k + 1, s) = v;
          }
        }
      }
      wave_lds_sync();
      PV_T(8);
      // ---- 2. verification ------------------------------------------------------------------
      // row r = l >> 3 (the preceding column of window column r), chunk l & 7 of rs / 8
      // values: its maximum (om) and the largest change to row r + 1 (dmx), combined over
      // the chunk lanes by DPP
      double om, dmx;
      {
        const int ch = rs >> 3;
        const double* row = S + (l >> 3) * rss + (l & 7) * ch;
        double m0 = -INFINITY, m1 = -INFINITY, d0 = -INFINITY, d1 = -INFINITY;
#pragma unroll 4
        for (int q = 0; q < ch; q += 2) {
          const pv_d2 v = *reinterpret_cast<const pv_d2*>(row + q);
          const pv_d2 w = *reinterpret_cast<const pv_d2*>(row + rss + q);
          m0 = fmax(m0, v.x);
          m1 = fmax(m1, v.y);
          d0 = fmax(d0, pv_delta(w.x, v.x));
          d1 = fmax(d1, pv_delta(w.y, v.y));
        }
        om = fmax(m0, m1);
        dmx = fmax(d0, d1);
        om = fmax(om, dpp_f64<DPP_Q1>(om));
        dmx = fmax(dmx, dpp_f64<DPP_Q1>(dmx));
        om = fmax(om, dpp_f64<DPP_Q2>(om));
        dmx = fmax(dmx, dpp_f64<DPP_Q2>(dmx));
        om = fmax(om, dpp_f64<DPP_HM>(om));
        dmx = fmax(dmx, dpp_f64<DPP_HM>(dmx));
      }
      // the predicted source's change from row k to k + 1 (stays: the target's own)
      auto dps = [&](int k, int s) -> double {
        if (anysw) return pv_delta(S[(k + 1) * rss + p[s]], S[k * rss + p[s]]);
        return pv_delta(sv[k + 1][s], sv[k][s]);
      };
      // tests: a pair passes by its carried margin bound or by the plain bound of a stay
      // (yd > max_i omega_i + max_{i != j} log a_ij + log e_j); a target failing once is
      // scanned for the rest of the window
      uint32_t fb[NS];  // this lane's failing window columns (bit k)
      double L0[NS];    // the bound at the window's first column
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        fb[s] = 0;
        L0[s] = L[s];
      }
#pragma unroll
      for (int k = 0; k < PV_K; ++k) {
        if (k >= kstart && k < kend) {
          const double o1 = lane_f64(om, 8 * k);
          const double dm = lane_f64(dmx, 8 * k);
          const double thr = 1e-6 + fabs(o1) * 0x1p-40;
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            const double bnd = (o1 + mj[s]) + ecol(k, s);
            const bool c1 = L[s] > thr;
            const bool c2 = sv[k + 1][s] > bnd;
            const bool pass = (fb[s] == 0u) & (c1 | (stayp[s] & c2));
            fb[s] |= (uint32_t)(act[s] & !pass) << k;
            L[s] = pv_adv(L[s], dps(k, s), dm);
          }
        }
      }
      // pairs in (column, slot, lane) order; the list holds at most lcap pairs: the window
      // ends before the column that would overflow it (one column has at most 64 NS <= lcap)
      int kcut = kend, npairs = 0;
#pragma unroll
      for (int k = 0; k < PV_K; ++k) {
        if (k >= kstart && k < kcut) {
          uint64_t m[NS];
          int ck = 0;
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            m[s] = __ballot((fb[s] >> k) & 1u);
            ck += __popcll(m[s]);
          }
          if (npairs + ck > a.lcap) {
            kcut = k;
          } else {
#pragma unroll
            for (int s = 0; s < NS; ++s) {
              if ((fb[s] >> k) & 1u) LIST[npairs + mbcnt64(m[s])] = (uint16_t)((k << 8) | jt[s]);
              npairs += __popcll(m[s]);
            }
          }
        }
      }
      wave_lds_sync();
      PV_T(9);
      PV_CNT(3, npairs);
      // exact scans, one lane per pair, pairs in column order: the two largest candidates
      // over the sources i != j, the stay, omega = max(yd, yo), the flag, the margin; the
      // lane keeps the pairs of the window's last column and of the first mispredicted one
      int kmis = PV_K;  // first mispredicted window column (PV_K: none)
      double exr[NS], mgr[NS];  // per round: this lane's pair's omega and margin
      int kr[NS], jr[NS];       //   its column (-1: none) and target
      bool mr[NS];              //   mispredicted
#pragma unroll
      for (int rd = 0; rd < NS; ++rd) {
        kr[rd] = -1;
        jr[rd] = 0;
        exr[rd] = 0.0;
        mgr[rd] = 0.0;
        mr[rd] = false;
        if (64 * rd < npairs) {
          const int idx = 64 * rd + l;
          const bool valid = idx < npairs;
          const int code = LIST[valid ? idx : 0];
          const int k = code >> 8, jj = code & 255;
          const double* sr = S + k * rss;
          const double* lr = LAT + jj * rsa;
          double a1 = -INFINITY, a2 = -INFINITY, b1 = -INFINITY, b2 = -INFINITY;
#pragma unroll 4
          for (int i = 0; i < np; i += 2) {
            const pv_d2 sv2 = *reinterpret_cast<const pv_d2*>(sr + i);
            const pv_d2 lv2 = *reinterpret_cast<const pv_d2*>(lr + i);
            const double va = sv2.x + lv2.x, vb = sv2.y + lv2.y;
            a2 = fmax(a2, fmin(a1, va));
            a1 = fmax(a1, va);
            b2 = fmax(b2, fmin(b1, vb));
            b1 = fmax(b1, vb);
          }
          const double z1 = fmax(a1, b1), z2 = fmax(fmin(a1, b1), fmax(a2, b2));
          const double ee = EC[k * rs + jj];
          const double ydp = sr[jj] + LDG[jj];
          const double yd = ydp + ee;
          const double yo = z1 + ee;
          const double ex = fmax(yd, yo);
          const bool flg = yd > yo;
          const bool mis = valid & (ex != sr[rss + jj]);
          const uint32_t bits = (flg ? 1u << k : 0u) | (mis ? 1u << (16 + k) : 0u);
          if (valid & (bits != 0u)) atomicOr(&FB[jj], bits);
          const uint64_t mb = __ballot(mis);
          if (mb && kmis == PV_K) kmis = __builtin_amdgcn_readlane(k, __builtin_ctzll(mb));
          exr[rd] = ex;
          mgr[rd] = pv_margin(fmax(z1, ydp), fmax(fmin(z1, ydp), z2));
          kr[rd] = valid ? k : -1;
          jr[rd] = jj;
          mr[rd] = mis;
        }
      }
      PV_T(10);
      // ---- 3. commit up to the first mispredicted column ----------------------------------
      const int kfin = kmis < PV_K ? kmis + 1 : kcut;  // window columns [kstart, kfin)
      const int kl = kfin - 1;                         // the last committed window column
      // the pairs of column kl: margins (and, mispredicted, corrected values and the largest
      // change of a corrected entry from row kl to kl + 1)
      double dml = lane_f64(dmx, 8 * kl);
      {
        double dcor = -INFINITY;
#pragma unroll
        for (int rd = 0; rd < NS; ++rd) {
          if (kr[rd] == kl) {
            MG[jr[rd]] = mgr[rd];
            if (mr[rd]) {
              dcor = fmax(dcor, pv_delta(exr[rd], S[kl * rss + jr[rd]]));
              S[(kl + 1) * rss + jr[rd]] = exr[rd];
            }
          }
        }
        if (kmis < PV_K) {
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) dcor = fmax(dcor, __shfl_xor(dcor, d));
          dml = fmax(dml, dcor);
        }
      }
      if (kmis < PV_K) {
        // the mispredicted targets' new sources: the target itself when it stays, else the
        // first source whose candidate reaches omega (one more pass over the sources by the
        // lanes holding such a pair)
#pragma unroll
        for (int rd = 0; rd < NS; ++rd) {
          const bool misk = (kr[rd] == kl) & mr[rd];
          if (__ballot(misk)) {
            const int jj = jr[rd];
            const double exk = exr[rd];
            const double* sr = S + kl * rss;
            const double* lr = LAT + jj * rsa;
            const double ee = EC[kl * rs + jj];
            const double yd = (sr[jj] + LDG[jj]) + ee;
            const bool look = misk & !(yd >= exk);
            int f = jj;
            if (__ballot(look)) {
              f = 0x7fffffff;
#pragma unroll 4
              for (int i = 0; i < np; i += 2) {
                const pv_d2 sv2 = *reinterpret_cast<const pv_d2*>(sr + i);
                const pv_d2 lv2 = *reinterpret_cast<const pv_d2*>(lr + i);
                f = ((sv2.y + lv2.y) + ee == exk) ? min(f, i + 1) : f;
                f = ((sv2.x + lv2.x) + ee == exk) ? min(f, i) : f;
              }
              f = look ? f : jj;
            }
            if (misk) WIN[jj] = f;
          }
        }
      }
      wave_lds_sync();
      const uint32_t wm = ((1u << kfin) - 1u) & ~((1u << kstart) - 1u);
      uint32_t fbw[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        fbw[s] = FB[jc[s]];
        const uint32_t fl = ((stayp[s] ? ~fb[s] : 0u) | fbw[s]) & wm;
        flw[s] |= act[s] ? fl << (8 * (h & 1)) : 0u;
        x[s] = act[s] ? S[kfin * rss + jc[s]] : -INFINITY;
        // the margin bound at the next column: from the scan of column kl if the target was
        // scanned there, else carried over the committed columns; the last change with the
        // corrected row maximum
        double Lb = L0[s], dpl = 0.0;
#pragma unroll
        for (int k = 0; k < PV_K; ++k) {
          if (k >= kstart && k < kl) Lb = pv_adv(Lb, dps(k, s), lane_f64(dmx, 8 * k));
          if (k == kl) dpl = dps(k, s);  // (rows after the correction of a misprediction)
        }
        const double mgs = MG[jc[s]];
        Lb = (fb[s] & wm) ? mgs : Lb;
        L[s] = pv_adv(Lb, dpl, dml);
      }
      if ((h & 1) == 0 && h > 0 && kstart == 0) {  // column cb = tile (h / 2)'s first column
#pragma unroll
        for (int s = 0; s < NS; ++s)
          buf_store_f64(rck, vo[s] * 8, (uint32_t)((h >> 1) * xr) * 8, S[rss + jc[s]]);
      }
      PV_T(11);
      PV_CNT(1, kfin - kstart);
      PV_CNT(2, kmis < PV_K);
      if (kmis < PV_K) {  // the mispredicted targets of column cb + kmis take their new sources
        bool sw = false;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const bool m = act[s] & (((fbw[s] >> (16 + kmis)) & 1u) != 0u);
          const int w = WIN[jc[s]];
          p[s] = m ? w : p[s];
          const double lw = LAT[jc[s] * rsa + min(w, n - 1)];
          lap[s] = m ? (w == jt[s] ? ld[s] : lw) : lap[s];
          L[s] = m ? -INFINITY : L[s];
          stayp[s] = act[s] & (p[s] == jt[s]);
          sw = sw | (act[s] & (p[s] != jt[s]));
        }
        anysw = __ballot(sw) != 0;
      }
      PV_T(12);
      kstart = kfin;
    }
    if ((h & 1) || cb + PV_K >= T) {  // tile h / 2 complete: its flag words
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        buf_store_u16(rst, vo[s] * 2, (uint32_t)((h >> 1) * xr) * 2, (uint16_t)flw[s]);
        flw[s] = 0;
      }
    }
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

template <int NS>
__global__ void __launch_bounds__(NS == 1 ? 512 : 256) pv_vit_kernel(PvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* LAT = reinterpret_cast<double*>(smem);
  double* LDG = LAT + (size_t)a.n * a.rsa;
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int i = tid; i < a.n * a.rsa; i += nt) LAT[i] = a.lat[i];
  for (int i = tid; i < a.rs; i += nt) LDG[i] = i < a.n ? a.ldg[i] : -INFINITY;
  __syncthreads();
  double* wl = LDG + a.rs + (size_t)(tid >> 6) * a.wl;
  const int l = tid & 63;
  double ld[NS], mj[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int j = 64 * s + l;
    ld[s] = j < a.n ? a.ldg[j] : -INFINITY;
    mj[s] = j < a.n ? a.lmj[j] : -INFINITY;
  }
  const int waves = nt >> 6, grid = gridDim.x;
  int bi = (tid >> 6) * grid + blockIdx.x;  // static first task
  const int dyn = waves * grid;
  while (bi < a.nblocks) {
    pv_task<NS>(a, wl, LAT, LDG, uni(a.order[bi]), ld, mj);
    bi = pv_next(a.queue, dyn);
  }
}

}  // namespace

PvGeometry pv_geometry(int n) {
  PvGeometry g{};
  g.ns = -1;
  if (n < 1 || n > 128) return g;
  const int ns = (n + 63) / 64;
  const int rsa = ((n + 3) & ~3) + 2;     // = 2 mod 4, >= n rounded up to 4
  const int rs = (n + 15) & ~15;          // value row width (multiple of 16)
  const int rss = rs + 2;                 // its stride (= 2 mod 4)
  const int xe = (n + 1) & ~1;            // padded log-emission row
  const int eb = 0;
  const int lcap = 64 * ns;  // pairs scanned per window at most (one round per slot)
  // per wave: value rows, the half-tile's log e, margins, sink, FB (rs + 64 ints), WIN (rs
  // ints), pair list, symbols
  const int wl = ((PV_K + 1) * rss + PV_K * rs + rs + 64 + (rs + 64) / 2 + rs / 2 + lcap / 4 + 32 + 1) & ~1;
  const int shared = n * rsa + rs;
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
  g.eb = eb;
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
    case 1: hipLaunchKernelGGL(pv_vit_kernel<1>, dim3(grid), dim3(g.block), g.lds, st, a); break;
    case 2: hipLaunchKernelGGL(pv_vit_kernel<2>, dim3(grid), dim3(g.block), g.lds, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace itr
