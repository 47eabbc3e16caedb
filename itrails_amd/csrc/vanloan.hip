// vanloan.hip — every Van Loan integral of a model rebuild (vanloan.py:392-425) as one
// shared, batched evaluation on gfx950.
//
// The reference forms, per omega path p = (w_0 .. w_{L-1}) and interval length t, the block
// bidiagonal matrix C_p (diagonal blocks Q, super-diagonal blocks diag(m_{w_i}) Q
// diag(m_{w_{i+1}})), takes expm(C_p t) with its own Pade branch and scaling, and keeps the
// top-right block.  Every polynomial of a block upper triangular matrix, the Pade quotient and
// its squarings are block upper triangular again, and block (i, j) of any of them depends
// only on the sub-path w_i .. w_j.  So block (0, k-1) of every intermediate is a function of
// a distinct sub-path ("member"): the diagonal block Q t is one member per interval ("root"),
// each consecutive omega pair another, and so on.  One rebuild of the (5,5) model asks for
// ~1400 paths of length <= 5 over four intervals; they share ~500 distinct sub-paths per
// interval, so the evaluation here forms ~3.8x fewer block products than path-by-path expm,
// with no (L n)^2 matrices at all.
//
// Supports.  Block (0, k-1) of any product of C's blocks is a sum of chains
// Q^a D_{w0} Q D_{w1} Q^b ... Q^z (D_w = diag(m_w)): row r can be non-zero only if r reaches a
// state of class w_0 in Q's transition graph, column c only if c is reached from class
// w_{k-1}.  The coalescent CTMCs are nearly acyclic (reach density ~0.3) and the classes
// small, so a non-root member of the (5,5) rebuild lives on ~44 rows x ~5 columns of 203 x 203,
// and the inner index of a split X[s_0..l] Y[s_l..] runs only over the states both reached
// from and reaching class w_l.  Non-root members are stored compactly (their support rectangle,
// row-major); every other entry of the reference's dense evaluation is an exact zero (sums of
// products with a zero factor), so dropping them changes nothing but the order in which the
// non-zero terms are added.  Roots stay dense (n x n).
//
//   product  Z = alpha X Y + beta D + gamma I:  Z[s] = sum_l X[s_0..l] Y[s_l..k-1] over the
//            splits of member s.  Roots: pair_gemm_kernel (one 64x64 output tile per
//            workgroup, v_mfma_f64_16x16x4, the K loop running across split pairs).  Compact
//            members: compact_gemm_kernel (one workgroup per ~256 output entries, K lists of
//            the split's support intersection).  Members of zero blocks — e.g. sub-paths longer
//            than 3 of A^2 — are never read.
//   solve    (V - U) R = V + U by block back substitution: the one diagonal block of each
//            interval inverted by LU (dense.hip), then by sub-path length
//            R[s] = inv (N[s] - sum_{l>=1} M[s_0..l] R[s_l..k-1])
//   squaring s levels of R := R R, intervals with fewer squarings drop out level by level
//
// Pade branch and scaling: expm.py:16-143 choose them from ||C_p t||_1 per path; here one
// branch and one scaling serve all paths of an interval — those of the path with the largest
// norm (the 1-norms of an interval's paths differ by a few percent; the result is the same
// matrix function, evaluated with the most conservative of the reference's choices).
// Everything after the host-side plan is stream-ordered: no host synchronisation.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <deque>
#include <map>
#include <vector>

#include "dense.h"

namespace itr {
namespace {

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int TT = 64, TK = 16;

struct PairGemmArgs {
  int nb;        // block order
  int tn;        // tiles per block row (ceil(nb / 64))
  int64_t nout;  // output roots in this launch
  const double* X;
  const double* Y;
  double* Z;
  const double* D;  // may alias Z (read before written, same thread)
  double alpha, beta, gamma;
  const int* zoff;  // [nout] output offset (doubles) in Z and D
  const int* zid;   // [nout] 1: add gamma I
  const int* pofs;  // [nout + 1] split-pair range
  const int* px;    // X offset (doubles) of each pair
  const int* py;    // Y offset of each pair
};

// One 64x64 tile of one dense (root) output.  The grid is a multiple of 8 and workgroup b runs
// on XCD b % 8: logical tile ids are dealt so that the tiles of one output (which read the same
// X and Y blocks) land on the same XCD and share its L2.
__global__ void __launch_bounds__(256) pair_gemm_kernel(PairGemmArgs g) {
  // A tile kept row-major (m, k) with a pitch of 17 doubles and the B tile (k, n) with a
  // pitch of 80: the MFMA operand reads (16 lanes along m or n, the next 16 lanes one k
  // further) then hit 32 distinct bank pairs per half-wave — no LDS bank conflicts
  constexpr int PA = TK + 1, PB = TT + 16;
  __shared__ double As[TT * PA];
  __shared__ double Bs[TK * PB];
  const int tiles = g.tn * g.tn;
  const int64_t total = g.nout * tiles;
  const int64_t per = gridDim.x >> 3;
  const int64_t logical = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (logical >= total) return;
  const int64_t oi = logical / tiles;
  const int tile = (int)(logical - oi * tiles);
  const int tm = tile / g.tn, tnn = tile - tm * g.tn;
  const int nb = g.nb;
  const int p0 = g.pofs[oi], p1 = g.pofs[oi + 1];
  const int ksteps = (nb + TK - 1) / TK;
  const int nsteps = (p1 - p0) * ksteps;
  const int row0 = tm * TT, col0 = tnn * TT;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;

  bool row_live[2], col_live[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    row_live[i] = row0 + wr * 32 + i * 16 < nb;
    col_live[i] = col0 + wc * 32 + i * 16 < nb;
  }
  dbl4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};

  // A: lane -> row tid/4, four consecutive k (32 B per lane); B: lane -> column tid % 64,
  // k rows w, w+4, w+8, w+12 (a wave reads 512 contiguous bytes of one row and its 16-lane
  // store groups cover 32 distinct banks)
  constexpr int RA = TT * TK / 256 / 4, RB = TK * TT / 256;
  const int ar = tid >> 2, ak = (tid & 3) * 4;
  const int bcol = tid & 63;
  double ra[4 * RA], rb[RB];
  auto fetch = [&](int step) {
    const int pr = p0 + step / ksteps;
    const int k0 = (step % ksteps) * TK;
    const double* __restrict__ A = g.X + g.px[pr];
    const double* __restrict__ B = g.Y + g.py[pr];
    const int gr = row0 + ar;
#pragma unroll
    for (int h = 0; h < RA; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int gk = k0 + h * 16 + ak + e;
        ra[4 * h + e] = (gr < nb && gk < nb) ? A[(int64_t)gr * nb + gk] : 0.0;
      }
    const int gc = col0 + bcol;
#pragma unroll
    for (int e = 0; e < RB; ++e) {
      const int gk = k0 + w + 4 * e;
      rb[e] = (gk < nb && gc < nb) ? B[(int64_t)gk * nb + gc] : 0.0;
    }
  };
  if (nsteps > 0) fetch(0);
  for (int step = 0; step < nsteps; ++step) {
#pragma unroll
    for (int h = 0; h < RA; ++h)
#pragma unroll
      for (int e = 0; e < 4; ++e) As[ar * PA + h * 16 + ak + e] = ra[4 * h + e];
#pragma unroll
    for (int e = 0; e < RB; ++e) Bs[(w + 4 * e) * PB + bcol] = rb[e];
    __syncthreads();
    if (step + 1 < nsteps) fetch(step + 1);
#pragma unroll
    for (int kk = 0; kk < TK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[(wr * 32 + i * 16 + (l & 15)) * PA + kk + (l >> 4)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[(kk + (l >> 4)) * PB + wc * 32 + j * 16 + (l & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (row_live[i] && col_live[j])
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  const int zo = g.zoff[oi];
  double* __restrict__ C = g.Z + zo;
  const double* Dm = g.D ? g.D + zo : nullptr;
  const double gam = g.zid[oi] ? g.gamma : 0.0;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = row0 + wr * 32 + i * 16 + (l >> 4) + 4 * r;
        const int col = col0 + wc * 32 + j * 16 + (l & 15);
        if (row < nb && col < nb) {
          double v = g.alpha * acc[i][j][r];
          if (Dm) v += g.beta * Dm[(int64_t)row * nb + col];
          if (row == col) v += gam;
          C[(int64_t)row * nb + col] = v;
        }
      }
}

// Compact outputs: Z[s][i][j] = alpha sum_pairs sum_t X[xrow_i + kx_t] Y[ycol_j + ky_t ldy]
// + beta D[s][i][j] on the member's support rectangle (R x C, row-major).  X rows: a root
// (dense, the member's row states) or a compact member with the same row set; Y columns
// likewise.  Work item = a run of rows of one output (about 256 entries).
constexpr int kOH = 7;  // output header: zoff, R, C, rows_at, cols_at, pair begin, pair end
constexpr int kPH = 8;  // pair header: xoff, ldx, xroot, yoff, ldy, yroot, k_at, klen
struct CompactArgs {
  int nb;
  int nitems;
  const int* items;  // [nitems][3]: output, first row, rows
  const int* ohdr;
  const int* phdr;
  const int* tab;    // state lists and K lists (kx[klen] then ky[klen])
  const double* X;
  const double* Y;
  double* Z;
  const double* D;
  double alpha, beta;
};

__global__ void __launch_bounds__(256) compact_gemm_kernel(CompactArgs a) {
  const int it = blockIdx.x;
  if (it >= a.nitems) return;
  const int o = a.items[3 * it], row0 = a.items[3 * it + 1], nrows = a.items[3 * it + 2];
  const int* oh = a.ohdr + kOH * o;
  const int zoff = oh[0], C = oh[2];
  const int* rows = a.tab + oh[3];
  const int* cols = a.tab + oh[4];
  const int pb = oh[5], pe = oh[6];
  for (int e = threadIdx.x; e < nrows * C; e += 256) {
    const int ri = e / C;
    const int i = row0 + ri, jj = e - ri * C;
    double acc = 0.0;
    for (int q = pb; q < pe; ++q) {
      const int* ph = a.phdr + kPH * q;
      const double* xr = a.X + ph[0] + (ph[2] ? (int64_t)rows[i] * a.nb : (int64_t)i * ph[1]);
      const double* yc = a.Y + ph[3] + (ph[5] ? cols[jj] : jj);
      const int ldy = ph[4];
      const int klen = ph[7];
      const int* kx = a.tab + ph[6];
      const int* ky = kx + klen;
      for (int t = 0; t < klen; ++t) acc = fma(xr[kx[t]], yc[(int64_t)ky[t] * ldy], acc);
    }
    const int64_t zi = zoff + (int64_t)i * C + jj;
    double v = a.alpha * acc;
    if (a.D) v += a.beta * a.D[zi];
    a.Z[zi] = v;
  }
}

// out[e] = sum_t c[t] in[t][e] + (e in a root's diagonal ? cI : 0) over one member range
// (roots first: nident elements = the range's roots, n x n each)
struct LinArgs {
  int nb;
  int64_t count;   // elements
  int64_t nident;  // elements of the leading roots
  double* out;
  const double* in[4];
  double c[4];
  double cI;
};

__global__ void __launch_bounds__(256) member_lincomb_kernel(LinArgs a) {
  const int64_t nn = (int64_t)a.nb * a.nb;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < a.count;
       e += (int64_t)gridDim.x * 256) {
    double v = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (a.in[t]) v += a.c[t] * a.in[t][e];
    if (e < a.nident) {
      const int64_t w = e % nn;
      if (w / a.nb == w % a.nb) v += a.cI;
    }
    a.out[e] = v;
  }
}

// A of every member: roots Q t_j 2^-s_j (dense), consecutive pairs diag(m_a) Q diag(m_b) t_j
// 2^-s_j on their support rectangle (the reference's C t / 2^s: (q t) then the exact power of
// two), longer sub-paths 0
constexpr int kMD = 8;  // member descriptor: kind, mask a, mask b, offset, R, C, rows_at, cols_at
struct BuildArgs {
  int nb;
  const double* Q;      // nb x nb
  const double* masks;  // [nmasks][nb] 0/1
  const int* desc;      // [count][kMD]
  const int* tab;
  const double* tau;    // [count][2]: t_j, 2^-s_j
  double* A;
};

__global__ void __launch_bounds__(256) build_members_kernel(BuildArgs a) {
  const int64_t m = blockIdx.y;
  const int* d = a.desc + kMD * m;
  const int kind = d[0];
  const double* ma = a.masks + (int64_t)d[1] * a.nb;
  const double* mb = a.masks + (int64_t)d[2] * a.nb;
  const double t = a.tau[2 * m], sc = a.tau[2 * m + 1];
  const int64_t size = kind == 0 ? (int64_t)a.nb * a.nb : (int64_t)d[4] * d[5];
  const int C = d[5];
  const int* rows = a.tab + d[6];
  const int* cols = a.tab + d[7];
  double* out = a.A + d[3];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < size;
       e += (int64_t)gridDim.x * 256) {
    double v = 0.0;
    if (kind == 0) {
      v = (a.Q[e] * t) * sc;
    } else if (kind == 1) {
      const int i = (int)(e / C), j = (int)(e - (int64_t)i * C);
      const int r = rows[i], c = cols[j];
      v = ((ma[r] * a.Q[(int64_t)r * a.nb + c] * mb[c]) * t) * sc;
    }
    out[e] = v;
  }
}

// out[p] (dense n x n) = path p's member, scattered from its support rectangle
constexpr int kPD = 6;  // path descriptor: offset, C, root, rowpos_at, colpos_at, buffer
__global__ void __launch_bounds__(256) scatter_paths_kernel(int nb, const double* s0,
                                                            const double* s1, const int* pdesc,
                                                            const int* tab, double* out) {
  const int64_t p = blockIdx.y;
  const int64_t nn = (int64_t)nb * nb;
  const int* d = pdesc + kPD * p;
  const double* s = (d[5] ? s1 : s0) + d[0];
  const int C = d[1];
  const int* rp = tab + d[3];
  const int* cp = tab + d[4];
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn;
       e += (int64_t)gridDim.x * 256) {
    double v;
    if (d[2]) {
      v = s[e];
    } else {
      const int r = (int)(e / nb), c = (int)(e - (int64_t)r * nb);
      const int i = rp[r], j = cp[c];
      v = (i >= 0 && j >= 0) ? s[(int64_t)i * C + j] : 0.0;
    }
    out[p * nn + e] = v;
  }
}

// Pade coefficients (expm.py:29-140; same values as dense.hip)
const double kB3[] = {120, 60, 12, 1};
const double kB5[] = {30240, 15120, 3360, 420, 30, 1};
const double kB7[] = {17297280, 8648640, 1995840, 277200, 25200, 1512, 56, 1};
const double kB9[] = {17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0,
                      2162160.0,     110880.0,     3960.0,       90.0,        1.0};
const double kB13[] = {64764752532480000.0, 32382376266240000.0, 7771770303897600.0,
                       1187353796428800.0,  129060195264000.0,   10559470521600.0,
                       670442572800.0,      33522128640.0,       1323241920.0,
                       40840800.0,          960960.0,            16380.0,
                       182.0,               1.0};

void branch_of(double norm, int* m, int* s) {  // expm.py:26-143
  *s = 0;
  if (norm < 1.5e-2) *m = 3;
  else if (norm < 2.5e-1) *m = 5;
  else if (norm < 9.5e-1) *m = 7;
  else if (norm < 2.1) *m = 9;
  else {
    *m = 13;
    const double v = ceil(log(norm / 5.4) / log(2.0));
    *s = v > 0.0 ? (int)v : 0;
  }
}

struct Launch {
  int kind;  // 0 dense root product, 1 lincomb, 2 invert roots, 4 compact product
  int x, y, z, d;  // buffer ids (-1 none); NINV = the root inverses
  double alpha, beta, gamma;
  int64_t a0, a1, a2, a3, a4;  // descriptor offsets in H
  int64_t n0;                  // outputs / work items
};

struct VlPlan {
  // key: the request's structure
  int nb = 0, njobs = 0, nmasks = 0;
  std::vector<int32_t> job, mask;
  std::vector<int64_t> off;
  std::vector<uint8_t> masks;
  std::vector<uint64_t> qpat;  // Q != 0, bit rows
  std::vector<int> jm, js;
  // plan
  std::vector<int> H;  // device descriptor ints (support table first)
  std::vector<Launch> L;
  std::vector<std::vector<double>> coefs;  // per lincomb launch
  std::vector<int> mjob, moff;
  int NM = 0, maxroots = 0;
  int64_t tot = 0, maxsize = 0, pdesc_at = 0, desc_at = 0;
};

// grow-only device workspace and pinned staging, per device and calling thread (two threads
// evaluating on one device must not share the staging buffer or the workspace); a call
// waits for the previous call of its thread on that device (`done`) before reusing them
struct Ws {
  int dev = -1;
  char* d = nullptr;
  size_t dbytes = 0;
  int* h = nullptr;
  size_t hbytes = 0;
  hipEvent_t done = nullptr;
};
struct WsSet {
  Ws w[16];
  void release() {
    for (Ws& x : w) {
      if (x.done) (void)hipEventSynchronize(x.done);  // the last call's kernels are done
      if (x.d) (void)hipFree(x.d);
      if (x.h) (void)hipHostFree(x.h);
      if (x.done) (void)hipEventDestroy(x.done);
      x = Ws{};
    }
  }
  ~WsSet() { release(); }
};
thread_local WsSet g_ws;
thread_local std::deque<VlPlan> g_plans;  // recent launch plans of this thread

hipError_t ws_get(size_t dbytes, size_t hbytes, Ws** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e) return e;
  Ws& w = g_ws.w[dev & 15];
  if (!w.done) {
    if ((e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming))) return e;
  } else if ((e = hipEventSynchronize(w.done))) {  // the previous call has finished
    return e;
  }
  if (dbytes > w.dbytes) {
    if (w.d) (void)hipFree(w.d);
    w.d = nullptr;
    w.dbytes = 0;
    const size_t want = dbytes + dbytes / 4;
    if ((e = hipMalloc((void**)&w.d, want))) return e;
    w.dbytes = want;
  }
  if (hbytes > w.hbytes) {
    if (w.h) (void)hipHostFree(w.h);
    w.h = nullptr;
    w.hbytes = 0;
    const size_t want = hbytes + hbytes / 4;
    if ((e = hipHostMalloc((void**)&w.h, want, hipHostMallocDefault))) return e;
    w.hbytes = want;
  }
  *out = &w;
  return hipSuccess;
}

}  // namespace

void release_vanloan_workspace() {
  g_ws.release();
  g_plans.clear();
}

void vanloan_job_norms(int nb, const double* h_Q, int njobs, const double* h_t, int nmasks,
                       const uint8_t* h_masks, int64_t npaths, const int32_t* h_job,
                       const int64_t* h_off, const int32_t* h_mask, double* jnorm) {
  std::vector<double> cs(nb, 0.0);  // column sums of |Q|
  for (int r = 0; r < nb; ++r)
    for (int c = 0; c < nb; ++c) cs[c] += fabs(h_Q[(int64_t)r * nb + c]);
  // per mask a: (m_a^T |Q|)[c]; a pair's column sums are cs[c] + m_b[c] (m_a^T |Q|)[c]
  std::vector<std::vector<double>> mq(nmasks);
  std::vector<double> memo((size_t)nmasks * nmasks, -1.0);  // pair norms, computed once
  auto pnorm = [&](int a, int b) -> double {
    double& slot = memo[(size_t)a * nmasks + b];
    if (slot >= 0.0) return slot;
    if (mq[a].empty()) {
      mq[a].assign(nb, 0.0);
      const uint8_t* ma = h_masks + (int64_t)a * nb;
      for (int r = 0; r < nb; ++r)
        if (ma[r])
          for (int c = 0; c < nb; ++c) mq[a][c] += fabs(h_Q[(int64_t)r * nb + c]);
    }
    const uint8_t* mb = h_masks + (int64_t)b * nb;
    double best = 0.0;
    for (int c = 0; c < nb; ++c) best = std::max(best, cs[c] + (mb[c] ? mq[a][c] : 0.0));
    return slot = best;
  };
  const double cmax = *std::max_element(cs.begin(), cs.end());
  for (int j = 0; j < njobs; ++j) jnorm[j] = 0.0;
  for (int64_t p = 0; p < npaths; ++p) {
    const int j = h_job[p];
    const int L = (int)(h_off[p + 1] - h_off[p]);
    double nm = cmax;
    for (int i = 1; i < L; ++i)
      nm = std::max(nm, pnorm(h_mask[h_off[p] + i - 1], h_mask[h_off[p] + i]));
    jnorm[j] = std::max(jnorm[j], nm * fabs(h_t[j]));
  }
}

// The launch plan of one request: depends only on the path structure, the masks, Q's zero
// pattern and each interval's Pade branch and squaring count — not on Q's values or the
// interval lengths — so the optimizer's repeated rebuilds reuse it (plan cache below).
static hipError_t build_plan(VlPlan& P, int nb, const double* h_Q, int njobs, int nmasks,
                             const uint8_t* h_masks, int64_t npaths, const int32_t* h_job,
                             const int64_t* h_off, const int32_t* h_mask,
                             const std::vector<int>& jm, const std::vector<int>& js, int maxlen) {
  const int64_t nn = (int64_t)nb * nb;
  // ---- supports: transitive closure of Q's transition graph (bit rows, Warshall) ---------
  const int NW = (nb + 63) / 64;
  std::vector<uint64_t> reach((size_t)nb * NW, 0);
  auto bit = [&](int r, int c) { return (reach[(size_t)r * NW + (c >> 6)] >> (c & 63)) & 1; };
  for (int r = 0; r < nb; ++r) {
    reach[(size_t)r * NW + (r >> 6)] |= 1ull << (r & 63);
    for (int c = 0; c < nb; ++c)
      if (h_Q[(int64_t)r * nb + c] != 0.0) reach[(size_t)r * NW + (c >> 6)] |= 1ull << (c & 63);
  }
  for (int k = 0; k < nb; ++k)
    for (int i = 0; i < nb; ++i)
      if (bit(i, k))
        for (int w = 0; w < NW; ++w) reach[(size_t)i * NW + w] |= reach[(size_t)k * NW + w];
  // per class w: rows reaching it (to) and columns reached from it (from), as state lists,
  // position maps and the K lists of the splits (ints of one table, `T`)
  std::vector<int> T;
  T.reserve(1 << 16);
  const int iota_at = 0;
  for (int i = 0; i < nb; ++i) T.push_back(i);
  std::vector<int> to_n(nmasks), fr_n(nmasks), rl_at(nmasks), rr_at(nmasks), md_at(nmasks),
      md_n(nmasks), rp_at(nmasks), cp_at(nmasks);
  for (int w = 0; w < nmasks; ++w) {
    const uint8_t* mw = h_masks + (int64_t)w * nb;
    std::vector<uint64_t> fr(NW, 0);
    std::vector<int> tl, fl;
    for (int m = 0; m < nb; ++m)
      if (mw[m])
        for (int x = 0; x < NW; ++x) fr[x] |= reach[(size_t)m * NW + x];
    for (int r = 0; r < nb; ++r) {
      bool hit = false;
      for (int m = 0; m < nb && !hit; ++m) hit = mw[m] && bit(r, m);
      if (hit) tl.push_back(r);
      if ((fr[r >> 6] >> (r & 63)) & 1) fl.push_back(r);
    }
    to_n[w] = (int)tl.size();
    fr_n[w] = (int)fl.size();
    rl_at[w] = (int)T.size();  // to-states, then 0 .. R-1
    T.insert(T.end(), tl.begin(), tl.end());
    for (int i = 0; i < to_n[w]; ++i) T.push_back(i);
    rr_at[w] = (int)T.size();  // 0 .. C-1, then from-states
    for (int i = 0; i < fr_n[w]; ++i) T.push_back(i);
    T.insert(T.end(), fl.begin(), fl.end());
    std::vector<int> tp(nb, -1), fp(nb, -1);
    for (int i = 0; i < to_n[w]; ++i) tp[tl[i]] = i;
    for (int i = 0; i < fr_n[w]; ++i) fp[fl[i]] = i;
    std::vector<int> kx, ky;  // K = from(w) & to(w): X column / Y row positions
    for (int s = 0; s < nb; ++s)
      if (fp[s] >= 0 && tp[s] >= 0) {
        kx.push_back(fp[s]);
        ky.push_back(tp[s]);
      }
    md_at[w] = (int)T.size();
    md_n[w] = (int)kx.size();
    T.insert(T.end(), kx.begin(), kx.end());
    T.insert(T.end(), ky.begin(), ky.end());
    rp_at[w] = (int)T.size();
    T.insert(T.end(), tp.begin(), tp.end());
    cp_at[w] = (int)T.size();
    T.insert(T.end(), fp.begin(), fp.end());
  }

  // ---- members: distinct (interval, sub-path); roots carry an empty sequence -------------
  typedef std::pair<int, std::vector<int>> Key;
  std::map<Key, int> tmp_id;
  std::vector<Key> keys;
  auto add = [&](int j, const int32_t* s, int len) {
    Key k{j, len == 1 ? std::vector<int>() : std::vector<int>(s, s + len)};
    if (tmp_id.emplace(k, (int)keys.size()).second) keys.push_back(k);
  };
  for (int64_t p = 0; p < npaths; ++p) {
    const int L = (int)(h_off[p + 1] - h_off[p]);
    const int32_t* s = h_mask + h_off[p];
    for (int i = 0; i < L; ++i)
      for (int k = i; k < L; ++k) add(h_job[p], s + i, k - i + 1);
  }
  auto mlen = [&](const Key& k) { return k.second.empty() ? 1 : (int)k.second.size(); };
  // order: Pade branch, sub-path length, interval (roots of a branch group come first)
  std::vector<int> order(keys.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
  std::sort(order.begin(), order.end(), [&](int a, int b) {
    const Key &x = keys[a], &y = keys[b];
    if (jm[x.first] != jm[y.first]) return jm[x.first] < jm[y.first];
    if (mlen(x) != mlen(y)) return mlen(x) < mlen(y);
    return x < y;
  });
  const int NM = (int)keys.size();
  std::map<Key, int> id;
  std::vector<Key> mem(NM);
  for (int i = 0; i < NM; ++i) {
    mem[i] = keys[order[i]];
    id[mem[i]] = i;
  }
  auto root_of = [&](int j) { return id.at(Key{j, {}}); };
  auto sub = [&](const Key& k, int a, int b) -> int {  // member of k's positions a..b
    if (a == b) return root_of(k.first);
    return id.at(Key{k.first, std::vector<int>(k.second.begin() + a, k.second.begin() + b + 1)});
  };
  // support rectangle and offset (doubles) of every member, the same in every work buffer
  std::vector<int> mR(NM), mC(NM), moff(NM + 1);
  int64_t tot = 0;
  for (int i = 0; i < NM; ++i) {
    if (mlen(mem[i]) == 1) {
      mR[i] = mC[i] = nb;
    } else {
      mR[i] = to_n[mem[i].second.front()];
      mC[i] = fr_n[mem[i].second.back()];
    }
    moff[i] = (int)tot;
    tot += (int64_t)mR[i] * mC[i];
    if (tot >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  }
  moff[NM] = (int)tot;
  // splits l = 0 .. k-1 of each member: (X member s_0..l, Y member s_l..k-1)
  std::vector<std::vector<std::pair<int, int>>> splits(NM);
  for (int i = 0; i < NM; ++i) {
    const int L = mlen(mem[i]);
    if (L == 1) {
      splits[i].push_back({i, i});
      continue;
    }
    for (int l = 0; l < L; ++l) splits[i].push_back({sub(mem[i], 0, l), sub(mem[i], l, L - 1)});
  }

  // ---- launch plan -----------------------------------------------------------------------
  std::vector<int> groups_m;  // distinct branches in member order
  std::vector<int> gbeg, gend;
  for (int i = 0; i < NM; ++i) {
    const int m = jm[mem[i].first];
    if (groups_m.empty() || groups_m.back() != m) {
      groups_m.push_back(m);
      gbeg.push_back(i);
      gend.push_back(i);
    }
    gend.back() = i + 1;
  }
  // host descriptor stream (ints): the support table first, doubles after the ints
  std::vector<int> H(T);
  H.reserve(T.size() + (1 << 16));
  auto put = [&](int v) {
    H.push_back(v);
    return (int64_t)H.size() - 1;
  };
  std::vector<Launch> L;
  int nz[9];
  const int NINV = 8;
  // one split pair of compact output s: X = member a (or the inverse slot `inv`), Y = member b
  auto pair_hdr = [&](int s, int a, int b, int l, int inv) {
    const std::vector<int>& seq = mem[s].second;
    const bool xroot = inv >= 0 || mlen(mem[a]) == 1, yroot = mlen(mem[b]) == 1;
    int k_at, klen;
    if (xroot) {  // K = rows of s: root columns = states, Y rows = positions
      k_at = rl_at[seq.front()];
      klen = to_n[seq.front()];
    } else if (yroot) {  // K = columns of s: X columns = positions, root rows = states
      k_at = rr_at[seq.back()];
      klen = fr_n[seq.back()];
    } else {  // K = states both reached from and reaching class seq[l]
      k_at = md_at[seq[l]];
      klen = md_n[seq[l]];
    }
    put(inv >= 0 ? (int)(inv * nn) : moff[a]);
    put(xroot ? nb : mC[a]);
    put(xroot ? 1 : 0);
    put(moff[b]);
    put(yroot ? nb : mC[b]);
    put(yroot ? 1 : 0);
    put(k_at);
    put(klen);
  };
  // compact launch over outputs `outs` with pair lists `pl` (pair index l per entry)
  auto compact_launch = [&](int X, int Y, int Z, int D, double alpha, double beta,
                            const std::vector<int>& outs,
                            const std::vector<std::vector<std::pair<int, int>>>& pl,
                            const std::vector<std::vector<int>>& pls, int inv_g0) {
    if (outs.empty()) return;
    Launch ln{4, X, Y, Z, D, alpha, beta, 0.0, 0, 0, 0, 0, 0, 0};
    ln.a2 = (int64_t)H.size();  // pair headers
    std::vector<int> pbeg(outs.size()), pend(outs.size());
    int np = 0;
    for (size_t q = 0; q < outs.size(); ++q) {
      pbeg[q] = np;
      for (size_t t = 0; t < pl[q].size(); ++t) {
        const int a = pl[q][t].first, b = pl[q][t].second;
        pair_hdr(outs[q], a, b, pls[q][t], inv_g0 >= 0 ? root_of(mem[outs[q]].first) - inv_g0 : -1);
        ++np;
      }
      pend[q] = np;
    }
    ln.a1 = (int64_t)H.size();  // output headers
    for (size_t q = 0; q < outs.size(); ++q) {
      const int o = outs[q];
      put(moff[o]);
      put(mR[o]);
      put(mC[o]);
      put(rl_at[mem[o].second.front()]);
      put(rr_at[mem[o].second.back()] + mC[o]);
      put(pbeg[q]);
      put(pend[q]);
    }
    ln.a0 = (int64_t)H.size();  // work items, most work first
    std::vector<std::pair<int64_t, int>> ord(outs.size());
    for (size_t q = 0; q < outs.size(); ++q) {
      int64_t w = 0;
      for (size_t t = 0; t < pl[q].size(); ++t) w += 1;
      ord[q] = {-(w * mR[outs[q]] * mC[outs[q]]), (int)q};
    }
    std::stable_sort(ord.begin(), ord.end());
    int64_t items = 0;
    for (auto& oq : ord) {
      const int q = oq.second, o = outs[q];
      const int rpi = std::max(1, 256 / std::max(1, mC[o]));
      for (int r0 = 0; r0 < mR[o]; r0 += rpi) {
        put(q);
        put(r0);
        put(std::min(rpi, mR[o] - r0));
        ++items;
      }
    }
    ln.n0 = items;
    L.push_back(ln);
  };
  // dense launch over root outputs: pairs (X offset, Y offset)
  auto root_launch = [&](int X, int Y, int Z, int D, double alpha, double beta, double gamma,
                         const std::vector<int>& outs, const std::vector<std::vector<int>>& px,
                         const std::vector<std::vector<int>>& py) {
    if (outs.empty()) return;
    Launch ln{0, X, Y, Z, D, alpha, beta, gamma, 0, 0, 0, 0, 0, (int64_t)outs.size()};
    ln.a0 = (int64_t)H.size();
    for (int o : outs) put(moff[o]);
    ln.a1 = (int64_t)H.size();
    for (size_t q = 0; q < outs.size(); ++q) put(1);
    ln.a2 = (int64_t)H.size();
    int acc = 0;
    put(0);
    for (size_t q = 0; q < outs.size(); ++q) put(acc += (int)px[q].size());
    ln.a3 = (int64_t)H.size();
    for (auto& v : px)
      for (int x : v) put(x);
    ln.a4 = (int64_t)H.size();
    for (auto& v : py)
      for (int y : v) put(y);
    L.push_back(ln);
  };
  // product over members of [g0, g1) (or `only`): Z = alpha X Y + beta D + gamma I
  auto product = [&](int g0, int g1, int X, int Y, int Z, int D, double alpha, double beta,
                     double gamma, const std::vector<int>* only, bool skip_first_split) {
    std::vector<int> outs;
    if (only) outs = *only;
    else
      for (int i = g0; i < g1; ++i) outs.push_back(i);
    std::vector<int> routs, couts;
    std::vector<std::vector<int>> rpx, rpy, cls;
    std::vector<std::vector<std::pair<int, int>>> cpl;
    for (int o : outs) {
      std::vector<std::pair<int, int>> pl;
      std::vector<int> ls;
      const auto& sp = splits[o];
      for (size_t l = skip_first_split ? 1 : 0; l < sp.size(); ++l)
        if (mlen(mem[sp[l].first]) <= nz[X] && mlen(mem[sp[l].second]) <= nz[Y]) {
          pl.push_back(sp[l]);
          ls.push_back((int)l);
        }
      if (mlen(mem[o]) == 1) {
        routs.push_back(o);
        rpx.emplace_back();
        rpy.emplace_back();
        for (auto& pr : pl) {
          rpx.back().push_back(moff[pr.first]);
          rpy.back().push_back(moff[pr.second]);
        }
      } else {
        couts.push_back(o);
        cpl.push_back(pl);
        cls.push_back(ls);
      }
    }
    root_launch(X, Y, Z, D, alpha, beta, gamma, routs, rpx, rpy);
    compact_launch(X, Y, Z, D, alpha, beta, couts, cpl, cls, -1);
    int zz = std::min(maxlen, nz[X] + nz[Y] - 1);
    if (D >= 0) zz = std::max(zz, nz[D]);
    if (gamma != 0.0) zz = std::max(zz, 1);
    nz[Z] = zz;
  };
  auto lincomb = [&](int g0, int g1, int Z, std::vector<int> in, std::vector<double> c,
                     double cI) {
    Launch ln{1, -1, -1, Z, -1, cI, 0.0, 0.0, 0, 0, 0, 0, 0, 0};
    while (g0 + ln.n0 < g1 && mlen(mem[g0 + ln.n0]) == 1) ++ln.n0;  // leading roots
    ln.a0 = (int64_t)H.size();
    put(g0);
    put(g1);
    for (int t = 0; t < 4; ++t) put(t < (int)in.size() ? in[t] : -1);
    L.push_back(ln);
    int zz = cI != 0.0 ? 1 : 0;
    for (int b : in) zz = std::max(zz, nz[b]);
    nz[Z] = zz;
    return c;
  };
  std::vector<std::vector<double>> coefs;  // per lincomb launch
  std::vector<int> final_sel(njobs, 0);

  for (size_t gi = 0; gi < groups_m.size(); ++gi) {
    const int g0 = gbeg[gi], g1 = gend[gi], m = groups_m[gi];
    int nroots = 0;
    while (g0 + nroots < g1 && mlen(mem[g0 + nroots]) == 1) ++nroots;
    nz[0] = std::min(2, maxlen);
    // A2
    product(g0, g1, 0, 0, 1, -1, 1.0, 0.0, 0.0, nullptr, false);
    if (m == 13) {
      const double* b = kB13;
      product(g0, g1, 1, 1, 2, -1, 1.0, 0.0, 0.0, nullptr, false);  // A4
      product(g0, g1, 1, 2, 3, -1, 1.0, 0.0, 0.0, nullptr, false);  // A6 = A2 A4
      coefs.push_back(lincomb(g0, g1, 4, {3, 2, 1}, {b[13], b[11], b[9]}, 0.0));
      coefs.push_back(lincomb(g0, g1, 5, {3, 2, 1}, {b[7], b[5], b[3]}, b[1]));
      product(g0, g1, 3, 4, 6, 5, 1.0, 1.0, 0.0, nullptr, false);
      product(g0, g1, 0, 6, 7, -1, 1.0, 0.0, 0.0, nullptr, false);  // U
      coefs.push_back(lincomb(g0, g1, 4, {3, 2, 1}, {b[12], b[10], b[8]}, 0.0));
      coefs.push_back(lincomb(g0, g1, 5, {3, 2, 1}, {b[6], b[4], b[2]}, b[0]));
      product(g0, g1, 3, 4, 6, 5, 1.0, 1.0, 0.0, nullptr, false);  // V
    } else {
      const double* b = m == 3 ? kB3 : m == 5 ? kB5 : m == 7 ? kB7 : kB9;
      const int np = m / 2;
      for (int p = 2; p <= np; ++p)
        product(g0, g1, p - 1, 1, p, -1, 1.0, 0.0, 0.0, nullptr, false);
      std::vector<int> P{1};
      std::vector<double> cu{b[3]}, cv{b[2]};
      for (int p = 2; p <= np; ++p) {
        P.push_back(p);
        cu.push_back(b[2 * p + 1]);
        cv.push_back(b[2 * p]);
      }
      coefs.push_back(lincomb(g0, g1, 5, P, cu, b[1]));
      product(g0, g1, 0, 5, 7, -1, 1.0, 0.0, 0.0, nullptr, false);  // U
      coefs.push_back(lincomb(g0, g1, 6, P, cv, b[0]));              // V
    }
    // M = V - U (W1), N = V + U (W2)
    coefs.push_back(lincomb(g0, g1, 1, {6, 7}, {1.0, -1.0}, 0.0));
    coefs.push_back(lincomb(g0, g1, 2, {6, 7}, {1.0, 1.0}, 0.0));
    // inverse of each interval's diagonal block (the roots, members g0 .. g0+nroots)
    {
      Launch ln{2, 1, -1, NINV, -1, 0.0, 0.0, 0.0, 0, 0, 0, 0, 0, 0};
      ln.a0 = (int64_t)H.size();
      put(g0);
      put(nroots);
      L.push_back(ln);
    }
    // R (W3) by sub-path length: N[s] -= sum_{l>=1} M[s_0..l] R[s_l..]; R[s] = inv N[s]
    nz[3] = 0;
    for (int len = 1; len <= maxlen; ++len) {
      std::vector<int> outs;
      for (int i = g0; i < g1; ++i)
        if (mlen(mem[i]) == len) outs.push_back(i);
      if (outs.empty()) continue;
      if (len > 1) {
        nz[1] = maxlen;  // pairs l >= 1 only: X member length >= 2
        nz[3] = len - 1;
        product(g0, g1, 1, 3, 2, 2, -1.0, 1.0, 0.0, &outs, true);
      }
      // R[s] = inv[interval of s] N[s]: one pair per member
      if (len == 1) {
        std::vector<std::vector<int>> px(outs.size()), py(outs.size());
        for (size_t q = 0; q < outs.size(); ++q) {
          px[q].push_back((int)((root_of(mem[outs[q]].first) - g0) * nn));
          py[q].push_back(moff[outs[q]]);
        }
        root_launch(NINV, 2, 3, -1, 1.0, 0.0, 0.0, outs, px, py);
      } else {
        std::vector<std::vector<std::pair<int, int>>> pl(outs.size());
        std::vector<std::vector<int>> ls(outs.size());
        for (size_t q = 0; q < outs.size(); ++q) {
          pl[q].push_back({-1, outs[q]});
          ls[q].push_back(0);
        }
        compact_launch(NINV, 2, 3, -1, 1.0, 0.0, outs, pl, ls, g0);
      }
    }
    nz[3] = maxlen;
    // squarings, in lock-step over the intervals still squaring (W3 <-> W2)
    int smax = 0;
    for (int i = g0; i < g0 + nroots; ++i) smax = std::max(smax, js[mem[i].first]);
    for (int lev = 1; lev <= smax; ++lev) {
      std::vector<int> outs;
      for (int i = g0; i < g1; ++i)
        if (js[mem[i].first] >= lev) outs.push_back(i);
      const int X = (lev & 1) ? 3 : 2, Z = (lev & 1) ? 2 : 3;
      nz[X] = maxlen;
      product(g0, g1, X, X, Z, -1, 1.0, 0.0, 0.0, &outs, false);
    }
    for (int i = g0; i < g0 + nroots; ++i) final_sel[mem[i].first] = js[mem[i].first] & 1;
  }
  // output: path p = member (interval, whole path), W3 or W2 by its squaring parity
  const int64_t pdesc_at = (int64_t)H.size();
  for (int64_t p = 0; p < npaths; ++p) {
    const int L0 = (int)(h_off[p + 1] - h_off[p]);
    const int o = id.at(Key{h_job[p], L0 == 1 ? std::vector<int>()
                                              : std::vector<int>(h_mask + h_off[p],
                                                                 h_mask + h_off[p + 1])});
    put(moff[o]);
    put(mC[o]);
    put(L0 == 1 ? 1 : 0);
    put(L0 == 1 ? 0 : rp_at[h_mask[h_off[p]]]);
    put(L0 == 1 ? 0 : cp_at[h_mask[h_off[p + 1] - 1]]);
    put(final_sel[h_job[p]]);
  }
  // member descriptors for the A build
  const int64_t desc_at = (int64_t)H.size();
  int64_t maxsize = nn;
  for (int i = 0; i < NM; ++i) {
    const int len = mlen(mem[i]);
    put(len == 1 ? 0 : len == 2 ? 1 : 2);
    put(len == 2 ? mem[i].second[0] : 0);
    put(len == 2 ? mem[i].second[1] : 0);
    put(moff[i]);
    put(mR[i]);
    put(mC[i]);
    put(len == 1 ? iota_at : rl_at[mem[i].second.front()]);
    put(len == 1 ? iota_at : rr_at[mem[i].second.back()] + mC[i]);
    maxsize = std::max(maxsize, (int64_t)mR[i] * mC[i]);
  }
  while (H.size() & 1) put(0);
  P.maxroots = 0;
  for (size_t gi = 0; gi < groups_m.size(); ++gi) {
    int r = 0;
    while (gbeg[gi] + r < gend[gi] && mlen(mem[gbeg[gi] + r]) == 1) ++r;
    P.maxroots = std::max(P.maxroots, r);
  }
  P.NM = NM;
  P.tot = tot;
  P.maxsize = maxsize;
  P.pdesc_at = pdesc_at;
  P.desc_at = desc_at;
  P.mjob.resize(NM);
  for (int i = 0; i < NM; ++i) P.mjob[i] = mem[i].first;
  P.moff = std::move(moff);
  P.H = std::move(H);
  P.L = std::move(L);
  P.coefs = std::move(coefs);
  return hipSuccess;
}

hipError_t vanloan_paths(int nb, const double* h_Q, int njobs, const double* h_t, int nmasks,
                         const uint8_t* h_masks, int64_t npaths, const int32_t* h_job,
                         const int64_t* h_off, const int32_t* h_mask, const double* h_jnorm,
                         double* d_out, hipStream_t st) {
  if (npaths <= 0) return hipSuccess;
  const int64_t nn = (int64_t)nb * nb;

  // ---- norms -> Pade branch and scaling per interval (expm.py:16-143); a caller that
  // evaluates a subset of an interval's paths (the rank-split build) passes the norms of the
  // whole set so that every subset takes the same branch and scaling ----------------------
  std::vector<double> jnorm(njobs, 0.0);
  vanloan_job_norms(nb, h_Q, njobs, h_t, nmasks, h_masks, npaths, h_job, h_off, h_mask,
                    jnorm.data());
  if (h_jnorm)
    for (int j = 0; j < njobs; ++j) jnorm[j] = std::max(jnorm[j], h_jnorm[j]);
  int maxlen = 1;
  for (int64_t p = 0; p < npaths; ++p) maxlen = std::max(maxlen, (int)(h_off[p + 1] - h_off[p]));
  std::vector<int> jm(njobs, 13), js(njobs, 0);
  for (int j = 0; j < njobs; ++j) branch_of(jnorm[j], &jm[j], &js[j]);

  // ---- the plan: cached per thread by the request's structure ---------------------------
  const int NW = (nb + 63) / 64;
  std::vector<uint64_t> qpat((size_t)nb * NW, 0);
  for (int r = 0; r < nb; ++r)
    for (int c = 0; c < nb; ++c)
      if (h_Q[(int64_t)r * nb + c] != 0.0) qpat[(size_t)r * NW + (c >> 6)] |= 1ull << (c & 63);
  const int64_t nmask_ids = h_off[npaths];
  VlPlan* hit = nullptr;
  for (VlPlan& c : g_plans) {
    if (c.nb == nb && c.njobs == njobs && c.nmasks == nmasks &&
        (int64_t)c.job.size() == npaths && (int64_t)c.mask.size() == nmask_ids &&
        std::equal(c.job.begin(), c.job.end(), h_job) &&
        std::equal(c.off.begin(), c.off.end(), h_off) &&
        std::equal(c.mask.begin(), c.mask.end(), h_mask) &&
        std::equal(c.masks.begin(), c.masks.end(), h_masks) && c.qpat == qpat && c.jm == jm &&
        c.js == js) {
      hit = &c;
      break;
    }
  }
  if (!hit) {
    if (g_plans.size() >= 4) g_plans.pop_front();
    g_plans.emplace_back();
    VlPlan& c = g_plans.back();
    c.nb = nb;
    c.njobs = njobs;
    c.nmasks = nmasks;
    c.job.assign(h_job, h_job + npaths);
    c.off.assign(h_off, h_off + npaths + 1);
    c.mask.assign(h_mask, h_mask + nmask_ids);
    c.masks.assign(h_masks, h_masks + (int64_t)nmasks * nb);
    c.qpat = qpat;
    c.jm = jm;
    c.js = js;
    if (hipError_t e = build_plan(c, nb, h_Q, njobs, nmasks, h_masks, npaths, h_job, h_off,
                                  h_mask, jm, js, maxlen)) {
      g_plans.pop_back();
      return e;
    }
    hit = &c;
  }
  const VlPlan& P = *hit;

  // doubles: tau per member, Q, masks
  const int64_t nd_tau = 2 * (int64_t)P.NM, nd_q = nn, nd_m = (int64_t)nmasks * nb;
  const int64_t ints = (int64_t)P.H.size();
  const size_t hbytes = ints * sizeof(int) + (nd_tau + nd_q + nd_m) * sizeof(double);
  const int maxroots = P.maxroots;
  const int NINV = 8;
  const int64_t W = P.tot;
  const size_t dbytes = (size_t)(8 * W + (int64_t)maxroots * nn) * sizeof(double) +
                        (size_t)maxroots * nb * sizeof(int) + hbytes + 256;
  Ws* ws = nullptr;
  hipError_t e = ws_get(dbytes, hbytes, &ws);
  if (e) return e;
  int* hs = ws->h;
  std::copy(P.H.begin(), P.H.end(), hs);
  double* hd = reinterpret_cast<double*>(hs + ints);
  for (int i = 0; i < P.NM; ++i) {
    const int j = P.mjob[i];
    hd[2 * i] = h_t[j];
    hd[2 * i + 1] = ldexp(1.0, -js[j]);
  }
  std::copy(h_Q, h_Q + nn, hd + nd_tau);
  for (int64_t i = 0; i < nd_m; ++i) hd[nd_tau + nd_q + i] = h_masks[i] ? 1.0 : 0.0;

  double* Wb[9];
  double* base = reinterpret_cast<double*>(ws->d);
  for (int i = 0; i < 8; ++i) Wb[i] = base + (int64_t)i * W;
  Wb[NINV] = base + 8 * W;
  int* piv = reinterpret_cast<int*>(Wb[NINV] + (int64_t)maxroots * nn);
  char* dstage = reinterpret_cast<char*>(
      ((uintptr_t)(piv + (int64_t)maxroots * nb) + 255) & ~(uintptr_t)255);
  int* ds = reinterpret_cast<int*>(dstage);
  const double* dd = reinterpret_cast<const double*>(ds + ints);
  if ((e = hipMemcpyAsync(dstage, hs, hbytes, hipMemcpyHostToDevice, st))) return e;

  {
    const int bx = (int)std::min<int64_t>((P.maxsize + 255) / 256, 64);
    BuildArgs a{nb, dd + nd_tau, dd + nd_tau + nd_q, ds + P.desc_at, ds, dd, Wb[0]};
    for (int64_t m0 = 0; m0 < P.NM; m0 += 65535) {
      BuildArgs h = a;
      h.desc += kMD * m0;
      h.tau += 2 * m0;
      hipLaunchKernelGGL(build_members_kernel,
                         dim3(bx, (unsigned)std::min<int64_t>(65535, P.NM - m0)), dim3(256), 0, st,
                         h);
    }
    if ((e = hipGetLastError())) return e;
  }
  const int tn = (nb + TT - 1) / TT;
  size_t ci = 0;
  for (const Launch& ln : P.L) {
    if (ln.kind == 0) {
      if (ln.n0 == 0) continue;
      PairGemmArgs g{};
      g.nb = nb;
      g.tn = tn;
      g.X = Wb[ln.x];
      g.Y = Wb[ln.y];
      g.Z = Wb[ln.z];
      g.D = ln.d >= 0 ? Wb[ln.d] : nullptr;
      g.alpha = ln.alpha;
      g.beta = ln.beta;
      g.gamma = ln.gamma;
      g.nout = ln.n0;
      g.zoff = ds + ln.a0;
      g.zid = ds + ln.a1;
      g.pofs = ds + ln.a2;
      g.px = ds + ln.a3;
      g.py = ds + ln.a4;
      const int64_t total = g.nout * tn * tn;
      const unsigned grid = (unsigned)((total + 7) / 8 * 8);
      hipLaunchKernelGGL(pair_gemm_kernel, dim3(grid), dim3(256), 0, st, g);
    } else if (ln.kind == 4) {
      if (ln.n0 == 0) continue;
      CompactArgs a{};
      a.nb = nb;
      a.items = ds + ln.a0;
      a.ohdr = ds + ln.a1;
      a.phdr = ds + ln.a2;
      a.tab = ds;
      a.X = Wb[ln.x];
      a.Y = Wb[ln.y];
      a.Z = Wb[ln.z];
      a.D = ln.d >= 0 ? Wb[ln.d] : nullptr;
      a.alpha = ln.alpha;
      a.beta = ln.beta;
      for (int64_t i0 = 0; i0 < ln.n0; i0 += ((int64_t)1 << 30)) {
        CompactArgs h = a;
        h.nitems = (int)std::min<int64_t>((int64_t)1 << 30, ln.n0 - i0);
        h.items += 3 * i0;
        hipLaunchKernelGGL(compact_gemm_kernel, dim3(h.nitems), dim3(256), 0, st, h);
      }
    } else if (ln.kind == 1) {
      const int g0 = P.H[ln.a0], g1 = P.H[ln.a0 + 1];
      const std::vector<double>& c = P.coefs[ci++];
      LinArgs a{};
      a.nb = nb;
      a.count = (int64_t)P.moff[g1] - P.moff[g0];
      a.out = Wb[ln.z] + P.moff[g0];
      a.nident = ln.n0 * nn;
      for (int t = 0; t < 4; ++t) {
        const int b = P.H[ln.a0 + 2 + t];
        a.in[t] = b >= 0 ? Wb[b] + P.moff[g0] : nullptr;
        a.c[t] = t < (int)c.size() ? c[t] : 0.0;
      }
      a.cI = ln.alpha;
      const unsigned grid = (unsigned)std::min<int64_t>((a.count + 255) / 256, 256 * 64);
      hipLaunchKernelGGL(member_lincomb_kernel, dim3(grid), dim3(256), 0, st, a);
    } else if (ln.kind == 2) {
      const int g0 = P.H[ln.a0], nr = P.H[ln.a0 + 1];
      if (nb <= kInverseRegMax) {  // one workgroup per root in registers (dense.hip)
        if ((e = inverse_batched(nb, nr, Wb[1] + P.moff[g0], Wb[NINV], piv, nullptr, st)))
          return e;
        continue;
      }
      LinArgs a{};
      a.nb = nb;
      a.count = nr * nn;
      a.nident = nr * nn;
      a.out = Wb[NINV];
      a.cI = 1.0;
      hipLaunchKernelGGL(member_lincomb_kernel,
                         dim3((unsigned)std::min<int64_t>((nr * nn + 255) / 256, 4096)),
                         dim3(256), 0, st, a);
      if ((e = solve_batched(nb, nb, nr, Wb[1] + P.moff[g0], Wb[NINV], piv, st))) return e;
    }
    if ((e = hipGetLastError())) return e;
  }
  {
    const int bx = (int)std::min<int64_t>((nn + 255) / 256, 64);
    for (int64_t p0 = 0; p0 < npaths; p0 += 65535)
      hipLaunchKernelGGL(scatter_paths_kernel,
                         dim3(bx, (unsigned)std::min<int64_t>(65535, npaths - p0)), dim3(256), 0,
                         st, nb, Wb[3], Wb[2], ds + P.pdesc_at + kPD * p0, ds, d_out + p0 * nn);
    if ((e = hipGetLastError())) return e;
  }
  // the workspace and the staging buffer are free again once everything above has run: the
  // next call (ws_get) waits for this, whichever stream it is issued on (the model build
  // prefetches one evaluation on a side stream while others run on the main stream)
  return hipEventRecord(ws->done, st);
}

}  // namespace itr
