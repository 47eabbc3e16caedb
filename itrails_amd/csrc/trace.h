// trace.h — the Viterbi traceback of one block by one wavefront (optimizer.py:336-354) over
// the checkpoint rows and stay flags the Viterbi sweeps write; device code only.  Used by
// vit_trace_kernel (hmm_sweeps.hip: blocks from a work counter) and by the per-wave Viterbi
// task (wave_tasks.h: a block traced by the wave that swept it, right after its sweep).
//
// Walking down from the last column with the current state s, the path stays in s as long
// as stay(t, s) holds: lane l reads s's flag word of tile k - l, so one load covers 1,024
// columns, and the highest clear bit of the highest tile with one is the next column u to
// resolve.  There bp(u, s) is the reference's first argmax over i of (omega_{u-1}[i] +
// log a_is) + log e_s(u) (lane i, +64, +128; first-max reduction).  omega_{u-1} is rebuilt
// from the checkpoint of its tile by at most 15 steps of the Viterbi recursion into the
// wave's LDS rows, each value max_i (omega[i] + log a_ij) + log e_j — bit-identical to the
// sweep's max(yd, yo) because IEEE rounding is monotone — and kept for further switches in
// the same tile.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sweeps.h"
#include "valu_sweep.h"

namespace itr {

// rows: VIT_TILE x n doubles of this wave's LDS; s: the block's last state
template <int G>  // state groups of 64 lanes: n <= 64 G
__device__ __forceinline__ void trace_block(const TraceArgs& p, double* rows, int blk, int s) {
  const int l = threadIdx.x & 63;
  const int n = p.n;
  const int64_t c0 = p.off[blk];
  const int T = uni((int)(p.off[blk + 1] - c0));
  if (T <= 0) return;
  const int64_t tk0 = p.tile_off[blk];
  uint8_t* path = p.path + c0;
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

}  // namespace itr
