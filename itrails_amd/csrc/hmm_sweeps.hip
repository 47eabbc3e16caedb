// hmm_sweeps.hip — forward / backward+posterior / Viterbi sweeps of the iTRAILS HMM on
// MI355X (gfx950, CDNA4).  Written for this chip; not a translation of any CUDA code (the
// reference has none: its sweeps are numba/NumPy loops, optimizer.py:145-354).
//
// Work decomposition
// ------------------
// A MAF block is a strictly sequential recurrence over its columns, so the only parallelism
// inside a block is the N x N state contraction of one column step.  One WORKGROUP owns one
// block at a time (blocks are pulled longest-first from a device work queue, so the long
// blocks that bound the makespan start first), and splits each step over W = ceil(N/16)
// wavefronts:
//
//   * wave w produces target states j in [16w, 16w+16): lane l = 8*jl + q holds
//     j = 16w + 8r + jl for r = 0,1 (RJ = 2 targets per lane, so every LDS broadcast of
//     x_i feeds two FMAs: the step is VALU-bound, not LDS-bound);
//   * the 8 lanes q = 0..7 sharing a j split the source-state sum over i into 8 ranges of
//     IQ states, i = q*IQ + k.  The lane's IQ x RJ slice of the transition matrix lives in
//     VGPRs for the whole kernel (no LDS or HBM traffic for `a` in the step loop);
//   * the 8 partial results are combined with three xor-butterfly shuffles, which gives the
//     identical (commutative) sum / first-max in all 8 lanes;
//   * x_{t-1} (the previous column's state vector, N doubles) is the only per-step
//     exchange: published to LDS, one workgroup barrier, then read back as broadcasts.
//
// Numerics
// --------
// forward / backward run in the probability domain with exact power-of-two rescaling
// (ldexp of the running maximum's exponent every 8 columns): mathematically identical to
// the reference's log-space max-shift recursion (optimizer.py:181-187, 205-212), no
// transcendental per state per column, and the rescaling itself is rounding-free.
// Viterbi is evaluated exactly as optimizer.py:325-330 rounds it — (omega_i + log a_ij)
// then + log e_j, IEEE adds only, first maximum wins — so paths are bit-identical for
// identical tables.  The kernel takes the argmax over y_ij = omega_i + log a_ij (one add
// fewer per pair) and proves, per state, that adding log e_j cannot create an earlier tie
// (pred(max y) + log e_j < max y + log e_j); if it can, that state is re-scanned with the
// reference's full expression.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "sweeps.h"

namespace itr {

static constexpr int Q = 8;       // lanes splitting the i-sum of one target state
static constexpr int J = 64 / Q;  // target states per slot per wave
static constexpr int RJ = 2;      // slots (target states) per lane
static constexpr int JW = J * RJ; // target states per wave
static constexpr int PD = 3;      // emission prefetch depth (columns)
static constexpr int PDA = 6;     // forward-row prefetch depth in the backward sweep
static constexpr double LN2 = 0.69314718055994530942;

// ---------------------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = fmax(v, __shfl_xor(v, d));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// first-maximum reduction key over the wave: larger value wins, equal values -> lower index
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

// Tile of observed symbols staged in LDS.  Tiles hold TB = blockDim.x consecutive STEPS of
// the sweep (forward: columns s; backward: columns T-1-s); two tiles are resident and the
// one after them is in flight in a register of every thread, so a global load is waited
// for one whole tile (TB steps) after it was issued.
struct ObsTiles {
  uint16_t* lds;     // [2][TB]
  const uint16_t* g; // block's first column
  int T, TB, dir;    // dir = +1 forward, -1 backward
  int inflight;      // this thread's element of the next tile to store

  __device__ __forceinline__ int col(int s) const { return dir > 0 ? s : T - 1 - s; }
  // symbols outside the 625-letter alphabet are clamped (memory safety; the host
  // wrappers reject them before they reach the device)
  __device__ __forceinline__ int fetch(int s) const {
    return (s >= 0 && s < T) ? min((int)g[col(s)], 624) : 0;
  }
  // block start: tiles 0 and 1 into LDS, tile 2 in flight
  __device__ __forceinline__ void start(int tid) {
    lds[tid] = (uint16_t)fetch(tid);
    lds[TB + tid] = (uint16_t)fetch(TB + tid);
    inflight = fetch(2 * TB + tid);
  }
  // call at step s (before the step's barrier); when s starts tile k >= 1, tile k+1 is
  // stored into the slot tile k-1 used, and tile k+2 is requested
  __device__ __forceinline__ void advance(int s, int tid) {
    if (s >= TB && (s % TB) == 0) {
      const int k = s / TB;
      lds[((k + 1) & 1) * TB + tid] = (uint16_t)inflight;
      inflight = fetch((k + 2) * TB + tid);
    }
  }
  __device__ __forceinline__ int get(int s) const {  // symbol at step s (LDS broadcast)
    return (s < T) ? (int)lds[((s / TB) & 1) * TB + (s % TB)] : 0;
  }
};

// ---------------------------------------------------------------------------------------
// the sweep kernel
// ---------------------------------------------------------------------------------------
// threads of the widest workgroup an IQ serves: N <= 8*IQ states -> ceil(N/16) waves
template <int IQ>
struct MaxBlock {
  static constexpr int value = 64 * ((Q * IQ + JW - 1) / JW);
};

template <int IQ, int MODE>
__global__ void __launch_bounds__(MaxBlock<IQ>::value) sweep_kernel(SweepArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = p.n;
  const int XP = p.xp;  // padded state count of the LDS vectors (multiple of 16)
  const int tid = threadIdx.x;
  const int TB = blockDim.x;
  const int W = TB >> 6;
  const int w = uni(tid >> 6);
  const int l = tid & 63;
  const int q = l & (Q - 1);
  const int jl = l >> 3;

  double* X = reinterpret_cast<double*>(smem);  // [2][XP]  published state vectors
  double* RED = X + 2 * XP;                     // [4][16]  per-wave partials (2 kinds x 2 bufs)
  int* SBLK = reinterpret_cast<int*>(RED + 64); // [4]      current block
  int* REDI = SBLK + 4;                         // [16]     per-wave argmax
  uint16_t* OBS = reinterpret_cast<uint16_t*>(REDI + 16);           // [2][TB]
  uint8_t* ORIG = reinterpret_cast<uint8_t*>(OBS + 2 * TB);          // [2][XP] (Viterbi)

  int jr[RJ];
  bool jv[RJ];
#pragma unroll
  for (int r = 0; r < RJ; ++r) {
    jr[r] = w * JW + r * J + jl;
    jv[r] = jr[r] < n;
  }

  // this lane's slice of a (or log a): rows i = q*IQ + k, columns jr[r]
  double m[IQ][RJ];
#pragma unroll
  for (int k = 0; k < IQ; ++k) {
    const int i = q * IQ + k;
#pragma unroll
    for (int r = 0; r < RJ; ++r)
      m[k][r] = (i < n && jv[r]) ? p.mat[(int64_t)i * n + jr[r]] : 0.0;
  }

  // padding of the published vectors (entries no lane ever writes): 0 for the
  // probability sweeps (contributes nothing), -inf for Viterbi (never a maximum)
  const double pad = (MODE == MODE_VIT) ? -INFINITY : 0.0;
  for (int i = tid; i < 2 * XP; i += TB) X[i] = pad;
  __syncthreads();

  for (;;) {
    if (tid == 0) SBLK[0] = atomicAdd(p.queue, 1);
    __syncthreads();
    const int bi = uni(SBLK[0]);
    __syncthreads();
    if (bi >= p.nblocks) break;
    const int blk = uni(p.order[bi]);
    const int64_t c0 = p.off[blk];
    const int T = uni((int)(p.off[blk + 1] - c0));
    if (T <= 0) {  // empty block: log-likelihood of nothing is 0, no other output
      if (MODE == MODE_FWD_LL && tid == 0) p.loglik[blk] = 0.0;
      continue;
    }

    ObsTiles ot{OBS, p.obs + c0, T, TB, (MODE == MODE_BWD) ? -1 : +1, 0};
    ot.start(tid);
    __syncthreads();

    if constexpr (MODE == MODE_FWD_LL || MODE == MODE_FWD_STORE) {
      // ---------------- forward: alpha_t = (alpha_{t-1} @ a) * e_t  (optimizer.py:181-187)
      const int o0 = ot.get(0);
      double x[RJ];
#pragma unroll
      for (int r = 0; r < RJ; ++r) x[r] = jv[r] ? p.init[o0 * n + jr[r]] : 0.0;
      if (MODE == MODE_FWD_STORE && q == 0) {
#pragma unroll
        for (int r = 0; r < RJ; ++r)
          if (jv[r]) p.alpha[c0 * n + jr[r]] = x[r];
      }
      double ering[PD][RJ];
#pragma unroll
      for (int d = 0; d < PD; ++d) {
        const int o = ot.get(1 + d);
#pragma unroll
        for (int r = 0; r < RJ; ++r)
          ering[d][r] = (1 + d < T && jv[r]) ? p.emit[o * n + jr[r]] : 0.0;
      }
      int K = 0;  // sum of the power-of-two exponents divided out so far
      int buf = 0;
      for (int t = 1; t < T; ++t) {
        double* Xb = X + buf * XP;
        if (q == 0) {
#pragma unroll
          for (int r = 0; r < RJ; ++r) Xb[jr[r]] = x[r];
        }
        const bool rescale = (t & 7) == 1;
        if (rescale) {
          double mx = x[0];
#pragma unroll
          for (int r = 1; r < RJ; ++r) mx = fmax(mx, x[r]);
          mx = wave_max(mx);
          if (l == 0) RED[buf * 16 + w] = mx;
        }
        ot.advance(t, tid);
        __syncthreads();
        double s = 1.0;
        if (rescale) {
          double M = RED[buf * 16];
          for (int v = 1; v < W; ++v) M = fmax(M, RED[buf * 16 + v]);
          if (M > 0.0 && M < INFINITY) {
            const int e = ilogb(M);
            s = ldexp(1.0, -e);
            K += e;
          }
        }
        double ec[RJ];
#pragma unroll
        for (int r = 0; r < RJ; ++r) ec[r] = ering[0][r];
#pragma unroll
        for (int d = 0; d + 1 < PD; ++d)
#pragma unroll
          for (int r = 0; r < RJ; ++r) ering[d][r] = ering[d + 1][r];
        {
          const int tn = t + PD;
          const int o = ot.get(tn);
#pragma unroll
          for (int r = 0; r < RJ; ++r)
            ering[PD - 1][r] = (tn < T && jv[r]) ? p.emit[o * n + jr[r]] : 0.0;
        }
        double acc[RJ];
#pragma unroll
        for (int r = 0; r < RJ; ++r) acc[r] = 0.0;
        const double* xs = Xb + q * IQ;
#pragma unroll
        for (int k = 0; k < IQ; ++k) {
          const double xi = xs[k];
#pragma unroll
          for (int r = 0; r < RJ; ++r) acc[r] = fma(xi, m[k][r], acc[r]);
        }
#pragma unroll
        for (int d = 1; d < Q; d <<= 1)
#pragma unroll
          for (int r = 0; r < RJ; ++r) acc[r] += __shfl_xor(acc[r], d);
#pragma unroll
        for (int r = 0; r < RJ; ++r) x[r] = (acc[r] * ec[r]) * s;
        if (MODE == MODE_FWD_STORE && q == 0) {
#pragma unroll
          for (int r = 0; r < RJ; ++r)
            if (jv[r]) p.alpha[(c0 + t) * n + jr[r]] = x[r];
        }
        buf ^= 1;
      }
      if constexpr (MODE == MODE_FWD_LL) {
        // log P = log(sum_j x_j) + K ln 2   (optimizer.py:160-162)
        double part = 0.0;
        if (q == 0) {
#pragma unroll
          for (int r = 0; r < RJ; ++r) part += jv[r] ? x[r] : 0.0;
        }
        part = wave_sum(part);
        if (l == 0) RED[buf * 16 + w] = part;
        __syncthreads();
        if (tid == 0) {
          double tot = 0.0;
          for (int v = 0; v < W; ++v) tot += RED[buf * 16 + v];
          p.loglik[blk] = log(tot) + (double)K * LN2;
        }
      }
    } else if constexpr (MODE == MODE_BWD) {
      // ---------------- backward + posterior (optimizer.py:191-238)
      //   beta_{T-1} = 1;  beta_{t-1} = (beta_t * e_t) @ a   (vector @ a: the reference's form)
      //   post_t = alpha_t * beta_t / sum_j(alpha_t * beta_t)
      double bt[RJ];
#pragma unroll
      for (int r = 0; r < RJ; ++r) bt[r] = jv[r] ? 1.0 : 0.0;
      // step s handles column t = T-1-s
      double ering[PD][RJ];
      double aring[PDA][RJ];
#pragma unroll
      for (int d = 0; d < PD; ++d) {
        const int o = ot.get(d);
#pragma unroll
        for (int r = 0; r < RJ; ++r) ering[d][r] = (d < T && jv[r]) ? p.emit[o * n + jr[r]] : 0.0;
      }
#pragma unroll
      for (int d = 0; d < PDA; ++d) {
        const int tcol = T - 1 - d;
#pragma unroll
        for (int r = 0; r < RJ; ++r)
          aring[d][r] = (tcol >= 0 && jv[r]) ? p.alpha[(c0 + tcol) * n + jr[r]] : 0.0;
      }
      int buf = 0;
      for (int s = 0; s < T; ++s) {
        const int t = T - 1 - s;
        double qv[RJ], part = 0.0;
#pragma unroll
        for (int r = 0; r < RJ; ++r) {
          qv[r] = aring[0][r] * bt[r];
          part += (q == 0) ? qv[r] : 0.0;
        }
        part = wave_sum(part);
        if (l == 0) RED[buf * 16 + w] = part;
        double* Xb = X + buf * XP;
        const bool more = t > 0;
        const bool rescale = (s & 7) == 0;
        double ec[RJ];
#pragma unroll
        for (int r = 0; r < RJ; ++r) ec[r] = ering[0][r];
        if (more) {
          double v[RJ];
#pragma unroll
          for (int r = 0; r < RJ; ++r) v[r] = bt[r] * ec[r];
          if (q == 0) {
#pragma unroll
            for (int r = 0; r < RJ; ++r) Xb[jr[r]] = v[r];
          }
          if (rescale) {
            double mx = fmax(v[0], v[1]);
            mx = wave_max(mx);
            if (l == 0) RED[32 + buf * 16 + w] = mx;
          }
        }
        if (s > 0) ot.advance(s, tid);
        __syncthreads();
        double S = 0.0;
        for (int u = 0; u < W; ++u) S += RED[buf * 16 + u];
        if (q == 0) {
#pragma unroll
          for (int r = 0; r < RJ; ++r)
            if (jv[r]) p.post[(c0 + t) * n + jr[r]] = qv[r] / S;
        }
        if (more) {
          double sc = 1.0;
          if (rescale) {
            double M = RED[32 + buf * 16];
            for (int u = 1; u < W; ++u) M = fmax(M, RED[32 + buf * 16 + u]);
            if (M > 0.0 && M < INFINITY) sc = ldexp(1.0, -ilogb(M));
          }
          // rotate prefetch rings
#pragma unroll
          for (int d = 0; d + 1 < PD; ++d)
#pragma unroll
            for (int r = 0; r < RJ; ++r) ering[d][r] = ering[d + 1][r];
          {
            const int sn = s + PD;
            const int o = ot.get(sn);
#pragma unroll
            for (int r = 0; r < RJ; ++r)
              ering[PD - 1][r] = (sn < T && jv[r]) ? p.emit[o * n + jr[r]] : 0.0;
          }
#pragma unroll
          for (int d = 0; d + 1 < PDA; ++d)
#pragma unroll
            for (int r = 0; r < RJ; ++r) aring[d][r] = aring[d + 1][r];
          {
            const int tcol = t - PDA;
#pragma unroll
            for (int r = 0; r < RJ; ++r)
              aring[PDA - 1][r] = (tcol >= 0 && jv[r]) ? p.alpha[(c0 + tcol) * n + jr[r]] : 0.0;
          }
          double acc[RJ];
#pragma unroll
          for (int r = 0; r < RJ; ++r) acc[r] = 0.0;
          const double* xs = Xb + q * IQ;
#pragma unroll
          for (int k = 0; k < IQ; ++k) {
            const double xi = xs[k];
#pragma unroll
            for (int r = 0; r < RJ; ++r) acc[r] = fma(xi, m[k][r], acc[r]);
          }
#pragma unroll
          for (int d = 1; d < Q; d <<= 1)
#pragma unroll
            for (int r = 0; r < RJ; ++r) acc[r] += __shfl_xor(acc[r], d);
#pragma unroll
          for (int r = 0; r < RJ; ++r) bt[r] = acc[r] * sc;
        }
        buf ^= 1;
      }
    } else {
      // ---------------- Viterbi (optimizer.py:305-333), back-pointers as uint8
      const int o0 = ot.get(0);
      double x[RJ];
#pragma unroll
      for (int r = 0; r < RJ; ++r) x[r] = jv[r] ? p.init[o0 * n + jr[r]] : -INFINITY;
      int org[RJ] = {0, 0};
      double ering[PD][RJ];
#pragma unroll
      for (int d = 0; d < PD; ++d) {
        const int o = ot.get(1 + d);
#pragma unroll
        for (int r = 0; r < RJ; ++r)
          ering[d][r] = (1 + d < T && jv[r]) ? p.emit[o * n + jr[r]] : 0.0;
      }
      const int64_t cbase = p.chunk_base[blk];
      int buf = 0;
      for (int t = 1; t < T; ++t) {
        double* Xb = X + buf * XP;
        uint8_t* Ob = ORIG + buf * XP;
        if (q == 0) {
#pragma unroll
          for (int r = 0; r < RJ; ++r) {
            Xb[jr[r]] = x[r];
            Ob[jr[r]] = (uint8_t)org[r];
          }
        }
        ot.advance(t, tid);
        __syncthreads();
        double ec[RJ];
#pragma unroll
        for (int r = 0; r < RJ; ++r) ec[r] = ering[0][r];
#pragma unroll
        for (int d = 0; d + 1 < PD; ++d)
#pragma unroll
          for (int r = 0; r < RJ; ++r) ering[d][r] = ering[d + 1][r];
        {
          const int tn = t + PD;
          const int o = ot.get(tn);
#pragma unroll
          for (int r = 0; r < RJ; ++r)
            ering[PD - 1][r] = (tn < T && jv[r]) ? p.emit[o * n + jr[r]] : 0.0;
        }
        const double* xs = Xb + q * IQ;
        double best[RJ];
        int arg[RJ];
        {
          const double x0 = xs[0];
#pragma unroll
          for (int r = 0; r < RJ; ++r) {
            best[r] = x0 + m[0][r];
            arg[r] = 0;
          }
        }
#pragma unroll
        for (int k = 1; k < IQ; ++k) {
          const double xi = xs[k];
#pragma unroll
          for (int r = 0; r < RJ; ++r) {
            const double y = xi + m[k][r];
            const bool gt = y > best[r];
            best[r] = gt ? y : best[r];
            arg[r] = gt ? k : arg[r];
          }
        }
#pragma unroll
        for (int r = 0; r < RJ; ++r) arg[r] += q * IQ;
        // combine the 8 i-ranges; on equal maxima the lower range (lower i) wins
#pragma unroll
        for (int d = 1; d < Q; d <<= 1) {
          const bool partner_hi = (q & d) == 0;
#pragma unroll
          for (int r = 0; r < RJ; ++r) {
            const double ob = __shfl_xor(best[r], d);
            const int oa = __shfl_xor(arg[r], d);
            const bool take = partner_hi ? (ob > best[r]) : !(best[r] > ob);
            best[r] = take ? ob : best[r];
            arg[r] = take ? oa : arg[r];
          }
        }
        double Mv[RJ];
        bool need[RJ];
        bool any_need = false;
#pragma unroll
        for (int r = 0; r < RJ; ++r) {
          Mv[r] = best[r] + ec[r];
          need[r] = jv[r] && (nextafter(best[r], -INFINITY) + ec[r] == Mv[r]);
          any_need |= need[r];
        }
        if (p.force_slow) {
#pragma unroll
          for (int r = 0; r < RJ; ++r) need[r] = jv[r];
          any_need = true;
        }
        if (__any(any_need)) {
          // rare: an earlier i might tie after adding log e_j -> reference expression
#pragma unroll
          for (int r = 0; r < RJ; ++r) {
            if (need[r]) {
              const double* la = p.mat + jr[r];
              double bb = (Xb[0] + la[0]) + ec[r];
              int aa = 0;
              for (int i = 1; i < n; ++i) {
                const double v = (Xb[i] + la[(int64_t)i * n]) + ec[r];
                if (v > bb) {
                  bb = v;
                  aa = i;
                }
              }
              arg[r] = aa;
            }
          }
        }
        // chunk origin tracking: org = state at column (chunk start - 1) on the best path
        const int tc = t % VIT_CHUNK;
#pragma unroll
        for (int r = 0; r < RJ; ++r) org[r] = (tc == 0) ? arg[r] : (int)Ob[arg[r]];
        if (q == 0) {
          const bool chunk_end = (tc == VIT_CHUNK - 1) || (t == T - 1);
#pragma unroll
          for (int r = 0; r < RJ; ++r) {
            if (jv[r]) {
              p.bp[(c0 + t) * n + jr[r]] = (uint8_t)arg[r];
              if (chunk_end && t >= VIT_CHUNK)
                p.chunk_map[(cbase + t / VIT_CHUNK) * n + jr[r]] = (uint8_t)org[r];
            }
          }
        }
#pragma unroll
        for (int r = 0; r < RJ; ++r) x[r] = jv[r] ? Mv[r] : -INFINITY;
        buf ^= 1;
      }
      // last state = first argmax of omega_{T-1}  (optimizer.py:346)
      double bv = jv[0] ? x[0] : -INFINITY;
      int bj = jv[0] ? jr[0] : 0x7fffffff;
#pragma unroll
      for (int r = 1; r < RJ; ++r) {
        if (jv[r] && (x[r] > bv || (x[r] == bv && jr[r] < bj))) {
          bv = x[r];
          bj = jr[r];
        }
      }
      wave_first_max(bv, bj);
      if (l == 0) {
        RED[buf * 16 + w] = bv;
        REDI[w] = bj;
      }
      __syncthreads();
      if (tid == 0) {
        double b = RED[buf * 16];
        int a = REDI[0];
        for (int v = 1; v < W; ++v) {
          const double c = RED[buf * 16 + v];
          if (c > b) {
            b = c;
            a = REDI[v];
          }
        }
        p.last_state[blk] = (uint8_t)a;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// Viterbi traceback (optimizer.py:336-354), chunked so that no thread chases more than
// VIT_CHUNK pointers:
//   chain: per block, walk the per-chunk maps from the last state to find every chunk's
//          end state (ceil(T/C) hops);
//   fill:  per chunk, chase the back-pointers from its end state (<= C hops).
// ---------------------------------------------------------------------------------------
__global__ void vit_chain_kernel(int n, int64_t nblocks, const int64_t* __restrict__ off,
                                 const int64_t* __restrict__ chunk_base,
                                 const uint8_t* __restrict__ chunk_map,
                                 const uint8_t* __restrict__ last_state,
                                 uint8_t* __restrict__ chunk_end) {
  const int64_t blk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= nblocks) return;
  const int64_t T = off[blk + 1] - off[blk];
  if (T <= 0) return;
  const int64_t cb = chunk_base[blk];
  const int64_t K = (T + VIT_CHUNK - 1) / VIT_CHUNK;
  int s = last_state[blk];
  chunk_end[cb + K - 1] = (uint8_t)s;
  for (int64_t k = K - 1; k >= 1; --k) {
    s = chunk_map[(cb + k) * n + s];
    chunk_end[cb + k - 1] = (uint8_t)s;
  }
}

__global__ void vit_fill_kernel(int n, int64_t nchunks, const int64_t* __restrict__ off,
                                const int64_t* __restrict__ chunk_base,
                                const int32_t* __restrict__ chunk_blk,
                                const uint8_t* __restrict__ chunk_end,
                                const uint8_t* __restrict__ bp, uint8_t* __restrict__ path) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const int blk = chunk_blk[c];
  const int64_t c0 = off[blk];
  const int64_t T = off[blk + 1] - c0;
  const int64_t k = c - chunk_base[blk];
  const int64_t lo = k * VIT_CHUNK;
  const int64_t hi = (lo + VIT_CHUNK < T) ? lo + VIT_CHUNK : T;
  int s = chunk_end[c];
  path[c0 + hi - 1] = (uint8_t)s;
  for (int64_t t = hi - 1; t > lo; --t) {
    s = bp[(c0 + t) * n + s];
    path[c0 + t - 1] = (uint8_t)s;
  }
}

// ---------------------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------------------
static int pick_iq(int n) {
  const int need = (n + Q - 1) / Q;
  const int menu[] = {4, 9, 12, 17, 24};
  for (int v : menu)
    if (v >= need) return v;
  return -1;
}

size_t sweep_lds_bytes(int xp, int tb) {
  return (size_t)2 * xp * sizeof(double) + 64 * sizeof(double) + 20 * sizeof(int) +
         (size_t)2 * tb * sizeof(uint16_t) + (size_t)2 * xp + 64;
}

template <int IQ, int MODE>
static hipError_t launch_iq(const SweepArgs& a, int grid, int block, size_t lds,
                            hipStream_t st) {
  hipLaunchKernelGGL((sweep_kernel<IQ, MODE>), dim3(grid), dim3(block), lds, st, a);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_mode(int iq, const SweepArgs& a, int grid, int block, size_t lds,
                              hipStream_t st) {
  switch (iq) {
    case 4: return launch_iq<4, MODE>(a, grid, block, lds, st);
    case 9: return launch_iq<9, MODE>(a, grid, block, lds, st);
    case 12: return launch_iq<12, MODE>(a, grid, block, lds, st);
    case 17: return launch_iq<17, MODE>(a, grid, block, lds, st);
    case 24: return launch_iq<24, MODE>(a, grid, block, lds, st);
  }
  return hipErrorInvalidValue;
}

template <int IQ, int MODE>
static int occ_iq(int block, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sweep_kernel<IQ, MODE>, block, lds) !=
      hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}
template <int MODE>
static int occ_mode(int iq, int block, size_t lds) {
  switch (iq) {
    case 4: return occ_iq<4, MODE>(block, lds);
    case 9: return occ_iq<9, MODE>(block, lds);
    case 12: return occ_iq<12, MODE>(block, lds);
    case 17: return occ_iq<17, MODE>(block, lds);
    case 24: return occ_iq<24, MODE>(block, lds);
  }
  return 1;
}

SweepGeometry sweep_geometry(int n, int mode) {
  SweepGeometry g{};
  g.iq = pick_iq(n);
  const int waves = (n + JW - 1) / JW;
  g.block = waves * 64;
  g.xp = waves * JW;
  if (Q * g.iq > g.xp) g.xp = Q * g.iq;
  g.xp = (g.xp + 15) & ~15;
  g.lds = sweep_lds_bytes(g.xp, g.block);
  int occ = 1;
  switch (mode) {
    case MODE_FWD_LL: occ = occ_mode<MODE_FWD_LL>(g.iq, g.block, g.lds); break;
    case MODE_FWD_STORE: occ = occ_mode<MODE_FWD_STORE>(g.iq, g.block, g.lds); break;
    case MODE_BWD: occ = occ_mode<MODE_BWD>(g.iq, g.block, g.lds); break;
    case MODE_VIT: occ = occ_mode<MODE_VIT>(g.iq, g.block, g.lds); break;
  }
  g.per_cu = occ;
  return g;
}

hipError_t launch_sweep(int mode, const SweepGeometry& g, int grid, const SweepArgs& a,
                        hipStream_t st) {
  switch (mode) {
    case MODE_FWD_LL: return launch_mode<MODE_FWD_LL>(g.iq, a, grid, g.block, g.lds, st);
    case MODE_FWD_STORE: return launch_mode<MODE_FWD_STORE>(g.iq, a, grid, g.block, g.lds, st);
    case MODE_BWD: return launch_mode<MODE_BWD>(g.iq, a, grid, g.block, g.lds, st);
    case MODE_VIT: return launch_mode<MODE_VIT>(g.iq, a, grid, g.block, g.lds, st);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_vit_traceback(int n, int64_t nblocks, int64_t nchunks, const int64_t* off,
                                const int64_t* chunk_base, const int32_t* chunk_blk,
                                const uint8_t* chunk_map, const uint8_t* last_state,
                                uint8_t* chunk_end, const uint8_t* bp, uint8_t* path,
                                hipStream_t st) {
  if (nblocks > 0) {
    const int tb = 256;
    hipLaunchKernelGGL(vit_chain_kernel, dim3((unsigned)((nblocks + tb - 1) / tb)), dim3(tb),
                       0, st, n, nblocks, off, chunk_base, chunk_map, last_state, chunk_end);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (nchunks > 0) {
    const int tb = 256;
    hipLaunchKernelGGL(vit_fill_kernel, dim3((unsigned)((nchunks + tb - 1) / tb)), dim3(tb), 0,
                       st, n, nchunks, off, chunk_base, chunk_blk, chunk_end, bp, path);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace itr
