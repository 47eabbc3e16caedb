// vanloan.hip — every Van Loan integral of a model rebuild (vanloan.py:392-425) as one
// shared, batched evaluation on gfx950.
//
// The reference forms, per omega path p = (w_0 .. w_{L-1}) and interval length t, the block
// bidiagonal matrix C_p (diagonal blocks Q, super-diagonal blocks diag(m_{w_i}) Q
// diag(m_{w_{i+1}})), takes expm(C_p t) with its own Pade branch and scaling, and keeps the
// top-right block.  Every polynomial of a block upper triangular matrix, the Pade quotient and
// its squarings are block upper triangular again, and block (i, j) of any of them depends
// only on the sub-path w_i .. w_j.  So block (0, k-1) of every intermediate is a function of
// a distinct sub-path ("member"): the diagonal block Q t is one member per interval, each
// consecutive omega pair another, and so on.  One rebuild of the (5,5) model asks for ~1400
// paths of length <= 5 over four intervals; they share ~500 distinct sub-paths per interval,
// so the evaluation here forms ~3.8x fewer block products than path-by-path expm, with no
// (L n)^2 matrices at all.
//
//   product  Z = alpha X Y + beta D + gamma I:  Z[s] = sum_l X[s_0..l] Y[s_l..k-1] over the
//            splits of member s (pair_gemm_kernel: one 64x64 output tile per workgroup,
//            v_mfma_f64_16x16x4, the K loop running across the member's split pairs; members
//            of zero blocks — e.g. sub-paths longer than 3 of A^2 — are never read)
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
#include <map>
#include <vector>

#include "dense.h"

namespace itr {
namespace {

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int TT = 64, TK = 16;
constexpr int IDENT = 1 << 30;  // output member flag: add gamma I

struct PairGemmArgs {
  int nb;        // block order
  int tn;        // tiles per block row (ceil(nb / 64))
  int64_t nout;  // output members in this launch
  const double* X;
  const double* Y;
  double* Z;
  const double* D;  // may alias Z (read before written, same thread)
  double alpha, beta, gamma;
  const int* out;   // [nout] output member (| IDENT)
  const int* pofs;  // [nout + 1] split-pair range
  const int* px;    // X member of each pair
  const int* py;    // Y member of each pair
};

// One 64x64 tile of one output member.  The grid is a multiple of 8 and workgroup b runs on
// XCD b % 8: logical tile ids are dealt so that the tiles of one member (which read the same
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
  const int64_t nn = (int64_t)nb * nb;
  const int ow = g.out[oi];
  const int o = ow & (IDENT - 1);
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
    const double* __restrict__ A = g.X + (int64_t)g.px[pr] * nn;
    const double* __restrict__ B = g.Y + (int64_t)g.py[pr] * nn;
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

  double* __restrict__ C = g.Z + (int64_t)o * nn;
  const double* Dm = g.D ? g.D + (int64_t)o * nn : nullptr;
  const double gam = (ow & IDENT) ? g.gamma : 0.0;
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

// out[m] = sum_t c[t] in[t][m] + (m < nident ? cI I : 0) over members [0, count)
struct LinArgs {
  int nb;
  int64_t count;
  int64_t nident;
  double* out;
  const double* in[4];
  double c[4];
  double cI;
};

__global__ void __launch_bounds__(256) member_lincomb_kernel(LinArgs a) {
  const int64_t nn = (int64_t)a.nb * a.nb;
  const int64_t total = a.count * nn;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * 256) {
    double v = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
      if (a.in[t]) v += a.c[t] * a.in[t][e];
    const int64_t m = e / nn, r = (e - m * nn) / a.nb, c = e - m * nn - r * a.nb;
    if (m < a.nident && r == c) v += a.cI;
    a.out[e] = v;
  }
}

// A of every member: roots Q t_j 2^-s_j, consecutive pairs diag(m_a) Q diag(m_b) t_j 2^-s_j
// (the reference's C t / 2^s: (q t) then the exact power of two), longer sub-paths 0
struct BuildArgs {
  int nb;
  int64_t count;
  const double* Q;      // nb x nb
  const double* masks;  // [nmasks][nb] 0/1
  const int* desc;      // [count][3]: kind (0 root, 1 pair, 2 zero), mask a, mask b
  const double* tau;    // [count][2]: t_j, 2^-s_j
  double* A;
};

__global__ void __launch_bounds__(256) build_members_kernel(BuildArgs a) {
  const int64_t m = blockIdx.y;
  const int kind = a.desc[3 * m];
  const double* ma = a.masks + (int64_t)a.desc[3 * m + 1] * a.nb;
  const double* mb = a.masks + (int64_t)a.desc[3 * m + 2] * a.nb;
  const double t = a.tau[2 * m], sc = a.tau[2 * m + 1];
  const int64_t nn = (int64_t)a.nb * a.nb;
  double* out = a.A + m * nn;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn;
       e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / a.nb), c = (int)(e - (int64_t)r * a.nb);
    double v = 0.0;
    if (kind == 0) v = (a.Q[e] * t) * sc;
    else if (kind == 1) v = ((ma[r] * a.Q[e] * mb[c]) * t) * sc;
    out[e] = v;
  }
}

// out[i] = src[sel[i]][idx[i]]  (two candidate buffers)
__global__ void __launch_bounds__(256) gather_members_kernel(int nb, const double* s0,
                                                             const double* s1, const int* idx,
                                                             const int* sel, double* out) {
  const int64_t i = blockIdx.y;
  const int64_t nn = (int64_t)nb * nb;
  const double* s = (sel[i] ? s1 : s0) + (int64_t)idx[i] * nn;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nn;
       e += (int64_t)gridDim.x * 256)
    out[i * nn + e] = s[e];
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

void release_vanloan_workspace() { g_ws.release(); }

void vanloan_job_norms(int nb, const double* h_Q, int njobs, const double* h_t, int nmasks,
                       const uint8_t* h_masks, int64_t npaths, const int32_t* h_job,
                       const int64_t* h_off, const int32_t* h_mask, double* jnorm) {
  std::vector<double> cs(nb, 0.0);  // column sums of |Q|
  for (int r = 0; r < nb; ++r)
    for (int c = 0; c < nb; ++c) cs[c] += fabs(h_Q[(int64_t)r * nb + c]);
  // per mask a: (m_a^T |Q|)[c]; a pair's column sums are cs[c] + m_b[c] (m_a^T |Q|)[c]
  std::vector<std::vector<double>> mq(nmasks);
  auto pnorm = [&](int a, int b) -> double {
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
    return best;
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
  std::vector<char> jused(njobs, 0);
  int maxlen = 1;
  for (int64_t p = 0; p < npaths; ++p) {
    jused[h_job[p]] = 1;
    maxlen = std::max(maxlen, (int)(h_off[p + 1] - h_off[p]));
  }
  std::vector<int> jm(njobs, 13), js(njobs, 0);
  for (int j = 0; j < njobs; ++j) branch_of(jnorm[j], &jm[j], &js[j]);

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

  // ---- workspace: 8 member buffers, inverses, Q, masks, descriptors ----------------------
  const int64_t W = (int64_t)NM * nn;
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
  // host descriptor stream (ints), doubles after it
  std::vector<int> H;
  H.reserve(1 << 16);
  auto put = [&](int v) {
    H.push_back(v);
    return (int64_t)H.size() - 1;
  };
  struct Launch {
    int kind;  // 0 pair gemm, 1 lincomb, 2 solve roots, 3 gather out
    int x, y, z, d;  // buffer ids (-1 none); 8 = inverse buffer
    double alpha, beta, gamma;
    int64_t out_at, pofs_at, px_at, py_at;
    int64_t nout;
  };
  std::vector<Launch> L;
  int nz[9];
  const int NINV = 8;
  // product over members of [g0, g1): Z = alpha X Y + beta D + gamma I
  auto product = [&](int g0, int g1, int X, int Y, int Z, int D, double alpha, double beta,
                     double gamma, const std::vector<int>* only) {
    Launch ln{0, X, Y, Z, D, alpha, beta, gamma, 0, 0, 0, 0, 0};
    std::vector<int> outs;
    if (only) outs = *only;
    else
      for (int i = g0; i < g1; ++i) outs.push_back(i);
    // longest pair lists first (load balance)
    std::vector<std::vector<std::pair<int, int>>> pl(outs.size());
    for (size_t q = 0; q < outs.size(); ++q)
      for (auto& pr : splits[outs[q]])
        if (mlen(mem[pr.first]) <= nz[X] && mlen(mem[pr.second]) <= nz[Y]) pl[q].push_back(pr);
    std::vector<int> ord(outs.size());
    for (size_t q = 0; q < ord.size(); ++q) ord[q] = (int)q;
    std::stable_sort(ord.begin(), ord.end(),
                     [&](int a, int b) { return pl[a].size() > pl[b].size(); });
    ln.nout = (int64_t)outs.size();
    ln.out_at = (int64_t)H.size();
    for (int q : ord) put(outs[q] | (mlen(mem[outs[q]]) == 1 ? IDENT : 0));
    ln.pofs_at = (int64_t)H.size();
    int acc = 0;
    put(0);
    for (int q : ord) put(acc += (int)pl[q].size());
    ln.px_at = (int64_t)H.size();
    for (int q : ord)
      for (auto& pr : pl[q]) put(pr.first);
    ln.py_at = (int64_t)H.size();
    for (int q : ord)
      for (auto& pr : pl[q]) put(pr.second);
    L.push_back(ln);
    int zz = std::min(maxlen, nz[X] + nz[Y] - 1);
    if (D >= 0) zz = std::max(zz, nz[D]);
    if (gamma != 0.0) zz = std::max(zz, 1);
    nz[Z] = zz;
  };
  auto lincomb = [&](int g0, int g1, int Z, std::vector<int> in, std::vector<double> c,
                     double cI) {
    Launch ln{1, -1, -1, Z, -1, cI, 0.0, 0.0, 0, 0, 0, 0, 0};
    ln.out_at = (int64_t)H.size();
    put(g0);
    put(g1);
    for (int t = 0; t < 4; ++t) put(t < (int)in.size() ? in[t] : -1);
    ln.pofs_at = (int64_t)H.size();  // coefficients follow in the double table
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
    product(g0, g1, 0, 0, 1, -1, 1.0, 0.0, 0.0, nullptr);
    if (m == 13) {
      const double* b = kB13;
      product(g0, g1, 1, 1, 2, -1, 1.0, 0.0, 0.0, nullptr);  // A4
      product(g0, g1, 1, 2, 3, -1, 1.0, 0.0, 0.0, nullptr);  // A6 = A2 A4
      coefs.push_back(lincomb(g0, g1, 4, {3, 2, 1}, {b[13], b[11], b[9]}, 0.0));
      coefs.push_back(lincomb(g0, g1, 5, {3, 2, 1}, {b[7], b[5], b[3]}, b[1]));
      product(g0, g1, 3, 4, 6, 5, 1.0, 1.0, 0.0, nullptr);
      product(g0, g1, 0, 6, 7, -1, 1.0, 0.0, 0.0, nullptr);  // U
      coefs.push_back(lincomb(g0, g1, 4, {3, 2, 1}, {b[12], b[10], b[8]}, 0.0));
      coefs.push_back(lincomb(g0, g1, 5, {3, 2, 1}, {b[6], b[4], b[2]}, b[0]));
      product(g0, g1, 3, 4, 6, 5, 1.0, 1.0, 0.0, nullptr);  // V
    } else {
      const double* b = m == 3 ? kB3 : m == 5 ? kB5 : m == 7 ? kB7 : kB9;
      const int np = m / 2;
      for (int p = 2; p <= np; ++p) product(g0, g1, p - 1, 1, p, -1, 1.0, 0.0, 0.0, nullptr);
      std::vector<int> P{1};
      std::vector<double> cu{b[3]}, cv{b[2]};
      for (int p = 2; p <= np; ++p) {
        P.push_back(p);
        cu.push_back(b[2 * p + 1]);
        cv.push_back(b[2 * p]);
      }
      coefs.push_back(lincomb(g0, g1, 5, P, cu, b[1]));
      product(g0, g1, 0, 5, 7, -1, 1.0, 0.0, 0.0, nullptr);  // U
      coefs.push_back(lincomb(g0, g1, 6, P, cv, b[0]));      // V
    }
    // M = V - U (W1), N = V + U (W2)
    coefs.push_back(lincomb(g0, g1, 1, {6, 7}, {1.0, -1.0}, 0.0));
    coefs.push_back(lincomb(g0, g1, 2, {6, 7}, {1.0, 1.0}, 0.0));
    // inverse of each interval's diagonal block (the roots, members g0 .. g0+nroots)
    {
      Launch ln{2, 1, -1, NINV, -1, 0.0, 0.0, 0.0, 0, 0, 0, 0, 0};
      ln.out_at = (int64_t)H.size();
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
        // pairs l >= 1 only: X member length >= 2
        std::vector<std::vector<std::pair<int, int>>> save(outs.size());
        for (size_t q = 0; q < outs.size(); ++q) {
          save[q] = splits[outs[q]];
          splits[outs[q]].erase(splits[outs[q]].begin());
        }
        nz[1] = maxlen;
        nz[3] = len - 1;
        product(g0, g1, 1, 3, 2, 2, -1.0, 1.0, 0.0, &outs);
        for (size_t q = 0; q < outs.size(); ++q) splits[outs[q]] = save[q];
      }
      // R[s] = inv[interval of s] N[s]: one pair per member
      Launch ln{0, NINV, 2, 3, -1, 1.0, 0.0, 0.0, 0, 0, 0, 0, 0};
      ln.nout = (int64_t)outs.size();
      ln.out_at = (int64_t)H.size();
      for (int o : outs) put(o);
      ln.pofs_at = (int64_t)H.size();
      for (size_t q = 0; q <= outs.size(); ++q) put((int)q);
      ln.px_at = (int64_t)H.size();
      for (int o : outs) put(root_of(mem[o].first) - g0);  // inverse slot
      ln.py_at = (int64_t)H.size();
      for (int o : outs) put(o);
      L.push_back(ln);
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
      product(g0, g1, X, X, Z, -1, 1.0, 0.0, 0.0, &outs);
    }
    for (int i = g0; i < g0 + nroots; ++i) final_sel[mem[i].first] = js[mem[i].first] & 1;
  }
  // output: path p = member (interval, whole path); W3 or W2 by its squaring parity
  const int64_t out_idx_at = (int64_t)H.size();
  for (int64_t p = 0; p < npaths; ++p) {
    const int L0 = (int)(h_off[p + 1] - h_off[p]);
    put(id.at(Key{h_job[p], L0 == 1 ? std::vector<int>()
                                    : std::vector<int>(h_mask + h_off[p], h_mask + h_off[p + 1])}));
  }
  const int64_t out_sel_at = (int64_t)H.size();
  for (int64_t p = 0; p < npaths; ++p) put(final_sel[h_job[p]]);
  // member descriptors for the A build
  const int64_t desc_at = (int64_t)H.size();
  for (int i = 0; i < NM; ++i) {
    const int len = mlen(mem[i]);
    put(len == 1 ? 0 : len == 2 ? 1 : 2);
    put(len == 2 ? mem[i].second[0] : 0);
    put(len == 2 ? mem[i].second[1] : 0);
  }
  while (H.size() & 1) put(0);
  // doubles: tau per member, Q, masks
  const int64_t nd_tau = 2 * (int64_t)NM, nd_q = nn, nd_m = (int64_t)nmasks * nb;
  const int64_t ints = (int64_t)H.size();
  const size_t hbytes = ints * sizeof(int) + (nd_tau + nd_q + nd_m) * sizeof(double);
  int maxroots = 0;
  for (size_t gi = 0; gi < groups_m.size(); ++gi) {
    int r = 0;
    while (gbeg[gi] + r < gend[gi] && mlen(mem[gbeg[gi] + r]) == 1) ++r;
    maxroots = std::max(maxroots, r);
  }
  const size_t dbytes = (size_t)(8 * W + (int64_t)maxroots * nn) * sizeof(double) +
                        (size_t)maxroots * nb * sizeof(int) + hbytes + 256;
  Ws* ws = nullptr;
  hipError_t e = ws_get(dbytes, hbytes, &ws);
  if (e) return e;
  int* hs = ws->h;
  std::copy(H.begin(), H.end(), hs);
  double* hd = reinterpret_cast<double*>(hs + ints);
  for (int i = 0; i < NM; ++i) {
    const int j = mem[i].first;
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

  const int bx = (int)std::min<int64_t>((nn + 255) / 256, 64);
  {
    BuildArgs a{nb, NM, dd + nd_tau, dd + nd_tau + nd_q, ds + desc_at, dd, Wb[0]};
    for (int64_t m0 = 0; m0 < NM; m0 += 65535) {
      BuildArgs h = a;
      h.desc += 3 * m0;
      h.tau += 2 * m0;
      h.A += m0 * nn;
      hipLaunchKernelGGL(build_members_kernel,
                         dim3(bx, (unsigned)std::min<int64_t>(65535, NM - m0)), dim3(256), 0, st,
                         h);
    }
    if ((e = hipGetLastError())) return e;
  }
  const int tn = (nb + TT - 1) / TT;
  size_t ci = 0;
  for (const Launch& ln : L) {
    if (ln.kind == 0) {
      if (ln.nout == 0) continue;
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
      const int64_t chunk = ((int64_t)1 << 30) / (tn * tn);  // grid.x limit
      for (int64_t o0 = 0; o0 < ln.nout; o0 += chunk) {
        PairGemmArgs h = g;
        h.nout = std::min<int64_t>(chunk, ln.nout - o0);
        h.out = ds + ln.out_at + o0;
        h.pofs = ds + ln.pofs_at + o0;
        h.px = ds + ln.px_at;
        h.py = ds + ln.py_at;
        const int64_t total = h.nout * tn * tn;
        const unsigned grid = (unsigned)((total + 7) / 8 * 8);
        hipLaunchKernelGGL(pair_gemm_kernel, dim3(grid), dim3(256), 0, st, h);
      }
    } else if (ln.kind == 1) {
      const int g0 = H[ln.out_at], g1 = H[ln.out_at + 1];
      const std::vector<double>& c = coefs[ci++];
      LinArgs a{};
      a.nb = nb;
      a.count = g1 - g0;
      a.out = Wb[ln.z] + (int64_t)g0 * nn;
      int nr = 0;
      while (g0 + nr < g1 && mlen(mem[g0 + nr]) == 1) ++nr;
      a.nident = nr;
      for (int t = 0; t < 4; ++t) {
        const int b = H[ln.out_at + 2 + t];
        a.in[t] = b >= 0 ? Wb[b] + (int64_t)g0 * nn : nullptr;
        a.c[t] = t < (int)c.size() ? c[t] : 0.0;
      }
      a.cI = ln.alpha;
      const int64_t total = a.count * nn;
      const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 256 * 64);
      hipLaunchKernelGGL(member_lincomb_kernel, dim3(grid), dim3(256), 0, st, a);
    } else if (ln.kind == 2) {
      const int g0 = H[ln.out_at], nr = H[ln.out_at + 1];
      LinArgs a{};
      a.nb = nb;
      a.count = nr;
      a.nident = nr;
      a.out = Wb[NINV];
      a.cI = 1.0;
      hipLaunchKernelGGL(member_lincomb_kernel,
                         dim3((unsigned)std::min<int64_t>((nr * nn + 255) / 256, 4096)),
                         dim3(256), 0, st, a);
      if ((e = solve_batched(nb, nb, nr, Wb[1] + (int64_t)g0 * nn, Wb[NINV], piv, st)))
        return e;
    }
    if ((e = hipGetLastError())) return e;
  }
  for (int64_t p0 = 0; p0 < npaths; p0 += 65535)
    hipLaunchKernelGGL(gather_members_kernel,
                       dim3(bx, (unsigned)std::min<int64_t>(65535, npaths - p0)), dim3(256), 0,
                       st, nb, Wb[3], Wb[2], ds + out_idx_at + p0, ds + out_sel_at + p0,
                       d_out + p0 * nn);
  if ((e = hipGetLastError())) return e;
  // the workspace and the staging buffer are free again once everything above has run: the
  // next call (ws_get) waits for this, whichever stream it is issued on (the model build
  // prefetches one evaluation on a side stream while others run on the main stream)
  return hipEventRecord(ws->done, st);
}

}  // namespace itr
