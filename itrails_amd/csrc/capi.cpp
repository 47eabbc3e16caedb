// capi.cpp — the C ABI declared in include/itrails_hip.h: object lifetimes, argument
// checking, workspace management and kernel launches.  No compute happens on the host.
#include "capi_internal.h"

namespace itr_host {

namespace {
thread_local std::string g_err;
}  // namespace

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace itr_host

using namespace itr_host;

namespace {

// ---- per-thread kernel timing (HIP events on the launch stream) -----------------------
struct Timer {
  std::string name;
  int device = -1;
  hipEvent_t a = nullptr, b = nullptr;
  bool armed = false;
};
thread_local std::deque<Timer> g_timers;  // stable addresses: nested Scopes hold Timer*

Timer* timer(const char* name) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  for (auto& t : g_timers)
    if (t.name == name) {
      if (t.device != dev) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
        t.a = t.b = nullptr;
      }
      if (!t.a) {
        (void)hipEventCreate(&t.a);
        (void)hipEventCreate(&t.b);
        t.device = dev;
      }
      return &t;
    }
  g_timers.push_back(Timer{name, dev});
  Timer* t = &g_timers.back();
  (void)hipEventCreate(&t->a);
  (void)hipEventCreate(&t->b);
  return t;
}
struct Scope {
  Timer* t;
  hipStream_t s;
  Scope(const char* name, hipStream_t st) : t(timer(name)), s(st) {
    (void)hipEventRecord(t->a, s);
  }
  ~Scope() {
    (void)hipEventRecord(t->b, s);
    t->armed = true;
  }
};


// Two CU-masked streams per device and host thread: `lng` on `reserve` CUs spread over the
// device, `blk` on the others, plus fork / join events.  itr_viterbi decodes the longest
// blocks on `lng` with the 9-wave VALU layout (one workgroup per CU, lowest step latency)
// while everything else runs on `blk`; the masks keep the two launches off each other's CUs
// whatever order the dispatcher takes them in.  Three streams: with the caller's that is the
// 4 hardware queues a process gets by default (GPU_MAX_HW_QUEUES); a fifth stream shares a
// queue with another and serialises against it (measured: 10 -> 12.5 ms per forward+Viterbi).
struct Partition {
  int device = -1, reserve = 0, reserve2 = 0;
  bool masked = true;
  hipStream_t lng = nullptr, lng2 = nullptr;  // the reserved CUs
  hipStream_t blk = nullptr;                   // the other CUs
  hipEvent_t fork = nullptr, jl = nullptr, jl2 = nullptr, jb = nullptr;
  std::vector<uint32_t> mb;    // the other CUs' mask
};
// The calling thread's partitions, at most one per device; destroyed with the thread (each
// thread that decodes owns its streams, so a worker thread's exit returns its hardware-queue
// streams)
struct Partitions {
  std::deque<Partition> v;
  static void destroy(Partition& x) {  // waits for the streams' work
    int dev = 0;
    const bool have_dev = hipGetDevice(&dev) == hipSuccess;
    (void)hipSetDevice(x.device);
    for (hipStream_t* q : {&x.lng, &x.lng2, &x.blk})
      if (*q) {
        (void)hipStreamSynchronize(*q);
        (void)hipStreamDestroy(*q);
        *q = nullptr;
      }
    for (hipEvent_t* e : {&x.fork, &x.jl, &x.jl2, &x.jb})
      if (*e) {
        (void)hipEventDestroy(*e);
        *e = nullptr;
      }
    x.device = -1;  // (matches no device: a slot whose re-creation failed stays unused)
    if (have_dev) (void)hipSetDevice(dev);
  }
  void release() {
    for (auto& x : v) destroy(x);
    v.clear();
  }
  ~Partitions() { release(); }
};
thread_local Partitions g_parts;

// the calling thread's partition of the current device (nullptr: none yet)
Partition* current_partition() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  for (auto& x : g_parts.v)
    if (x.device == dev) return &x;
  return nullptr;
}

// lng on `reserve` CUs, lng2 on `reserve2` others (0: lng2 on lng's CUs), blk on the rest
int partition(int reserve, int reserve2, Partition** out, bool masked = true) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  for (auto& x : g_parts.v)
    if (x.device == dev && x.reserve == reserve && x.reserve2 == reserve2 && x.masked == masked) {
      *out = &x;
      return 0;
    }
  // one partition per thread and device: its three streams plus the caller's are the 4
  // hardware queues the process gets on that device (GPU_MAX_HW_QUEUES); a second partition's
  // streams would share queues with the first's and serialise behind them.  Only this
  // device's partition is replaced (its work drained first); other devices' stay, so one
  // thread can drive several GPUs in turn without re-creating streams.
  Partition* slot = nullptr;
  for (auto& x : g_parts.v)
    if (x.device == dev) slot = &x;
  if (slot) Partitions::destroy(*slot);
  const int cus = cu_count();
  const int nw = (cus + 31) / 32;
  std::vector<uint32_t> ml(nw, 0u), ml2(nw, 0u), mb(nw, 0u);
  // Logical CU-mask bit b addresses XCC b % X, CU b / X of that XCC, and an XCC left with no
  // bit set is not masked at all (measured on MI355X, X = 8: scripts/micro/cumask2.hip,
  // profiles/r3r_cumask.txt).  So the reserved CUs are chosen per XCC — reserve / X of each
  // XCC's cus / X, spread over its CU indices — and each XCC keeps at least one CU on every
  // side of the partition.
  const int X = (cus % 8 == 0) ? 8 : 1, L = cus / X;
  std::vector<char> in(cus, 0);  // 1: lng, 2: lng2
  {
    // within an XCC, CU index k belongs to shader engine k % 4 (cumask2.hip: local k ->
    // se k % 4); the dispatcher deals a launch's workgroups to the shader engines in turn, so
    // each set takes the same number of CUs from every engine (a one-workgroup-per-CU launch
    // then finds a CU in whichever engine its workgroup is dealt to)
    const int S = (L % 4 == 0) ? 4 : 1, E = L / S;  // engines per XCC, CUs per engine
    for (int x = 0; x < X; ++x) {
      const int r1 = reserve / X + (x < reserve % X ? 1 : 0);
      const int r2 = reserve2 / X + (x < reserve2 % X ? 1 : 0);
      for (int set = 1; set <= 2; ++set) {
        const int r = set == 1 ? r1 : r2;
        for (int k = 0; k < r; ++k) {
          const int se = k % S;
          // the j-th CU of this set in engine se, after the CUs of the sets before it
          const int j = k / S + (set == 2 ? r1 / S + (se < r1 % S ? 1 : 0) : 0);
          if (j >= E - 1) continue;  // every engine keeps a CU for the bulk
          in[(int)((int64_t)(j * S + se) * X + x)] = (char)set;
        }
      }
    }
  }
  for (int c = 0; c < cus; ++c)
    (in[c] == 1 ? ml : in[c] == 2 ? ml2 : mb)[c / 32] |= 1u << (c % 32);
  if (reserve <= 0) std::fill(ml.begin(), ml.end(), 0xFFFFFFFFu);  // (lng unused)
  if (reserve2 <= 0) ml2 = ml;
  if (!masked) {  // no masks
    std::fill(ml.begin(), ml.end(), 0xFFFFFFFFu);
    std::fill(ml2.begin(), ml2.end(), 0xFFFFFFFFu);
    std::fill(mb.begin(), mb.end(), 0xFFFFFFFFu);
  }
  Partition x;
  x.device = dev;
  x.reserve = reserve;
  x.reserve2 = reserve2;
  x.masked = masked;
  hipError_t err = hipExtStreamCreateWithCUMask(&x.lng, (uint32_t)ml.size() * 32, ml.data());
  if (err == hipSuccess)
    err = hipExtStreamCreateWithCUMask(&x.lng2, (uint32_t)ml2.size() * 32, ml2.data());
  if (err == hipSuccess)
    err = hipExtStreamCreateWithCUMask(&x.blk, (uint32_t)mb.size() * 32, mb.data());
  for (hipEvent_t* e : {&x.fork, &x.jl, &x.jl2, &x.jb})
    if (err == hipSuccess) err = hipEventCreateWithFlags(e, hipEventDisableTiming);
  if (err != hipSuccess) {  // nothing half-built stays behind (the old slot is already dead)
    Partitions::destroy(x);
    return fail(ITR_EHIP, "partition: stream/event creation failed: %s", hipGetErrorString(err));
  }
  x.device = dev;
  x.mb = mb;
  if (slot) {
    *slot = x;  // (in place: the other devices' entries keep their addresses)
  } else {
    g_parts.v.push_back(x);
    slot = &g_parts.v.back();
  }
  *out = slot;
  return 0;
}

}  // namespace

namespace {

// Workspace: Viterbi = one checkpoint row (f64) and one flag word (u16) per state per
// 16-column tile record; posterior = the forward rows of every column.
int vit_stride(int n) {
  const itr::WaveVitGeometry wv = itr::wave_vit_geometry(n);
  return wv.iq > 0 ? wv.xr : itr::sweep_row_stride(n, itr::MODE_VIT);
}

// matrix-core posterior exists: 100 blocks of 100 kbp at N = 70, 51.3 against 61.4 ms)
// Small models (N <= 48) are latency-bound at any block count: the whole posterior's work is
// a fraction of the longest block's two sweeps (the reference's example (3,3) model, N = 27,
// 10 Mbp: ~1 ms of VALU work against 18,377 x (~0.2 + ~0.4) us), so they take the split too.
bool post_split_path(int n, itr_plan_t p) {
  return p->npsplit > 0 && n <= 128 && (p->nblocks <= 2 * (int64_t)cu_count() || n <= 48);
}

// The matrix-core posterior's split set: the first nbeta blocks of the order (VALU tasks of
// the backward launch, at least MfmaGeometry.bfrac of the longest block and >= 512 columns) and
// their beta rows (brows = their columns).  itr_posterior splits them, reserve() sizes their
// rows with it.
std::pair<int64_t, int64_t> hybrid_beta_set(itr_plan_t p, int n) {
  if (p->nblocks == 0) return {0, 0};
  const itr::MfmaGeometry gb = itr::mfma_geometry(n, itr::MODE_BWD);
  int64_t nurg = 0, nbeta = 0, brows = 0;
  const double lim = std::max(512.0, gb.pfrac * (double)p->sorted_len[0]);
  while (nurg < p->nblocks && (double)p->sorted_len[nurg] > lim) ++nurg;
  double bfrac = gb.bfrac;
#ifdef ITR_EXPERIMENT
  if (getenv("ITR_POST_BFRAC")) bfrac = atof(getenv("ITR_POST_BFRAC"));
#endif
  const double blim = std::max(512.0, bfrac * (double)p->sorted_len[0]);
  while (nbeta < std::min(p->npsplit, nurg) && (double)p->sorted_len[nbeta] >= blim)
    brows += p->sorted_len[nbeta++];
  return {nbeta, brows};
}

int reserve(itr_plan_t p, int n, bool vit, bool post) {
  const int xr = vit_stride(n);
  const int xa = itr::sweep_row_stride(n, itr::MODE_BWD);
  if (xr < 0 || xa < 0) return fail(ITR_EINVAL, "n_states=%d unsupported", n);
  size_t need_rows = 0;
  if (vit) {
    need_rows = (size_t)std::max<int64_t>(p->ntiles, 1) * xr;
    const size_t need = need_rows;
    if (need > p->stay_cap) {
      dev_free(p->d_stay);
      if (int e = dev_alloc(&p->d_stay, need)) return e;
      p->stay_cap = need;
    }
  }
  if (post) {
    const itr::MfmaGeometry g = itr::mfma_geometry(n, itr::MODE_BWD);
    const int stride = g.cfg >= 0 ? std::max(xa, g.xr) : xa;
    need_rows = std::max(need_rows, (size_t)p->total * stride);
  }
  // beta rows: the VALU-only concurrent split's (stride xa) or the matrix-core posterior's
  // split set (stride of its forward-store rows), whichever itr_posterior will take
  size_t beta_need = 0;
  if (post && post_split_path(n, p)) {
    beta_need = (size_t)p->beta_rows * xa;
  } else if (post) {
    const itr::MfmaGeometry gf = itr::mfma_geometry(n, itr::MODE_FWD_STORE);
    if (gf.cfg >= 0) beta_need = (size_t)hybrid_beta_set(p, n).second * gf.xr;
  }
  if (beta_need > p->beta_cap) {
    dev_free(p->d_beta);
    p->beta_cap = 0;
    if (int e = dev_alloc(&p->d_beta, beta_need)) return e;
    p->beta_cap = beta_need;
  }
  if (need_rows > p->alpha_cap) {
    dev_free(p->d_alpha);
    if (int e = dev_alloc(&p->d_alpha, need_rows)) return e;
    p->alpha_cap = need_rows;
  }
  return 0;
}

itr::SweepArgs base_args(itr_model_t m, itr_plan_t p, const uint16_t* obs) {
  itr::SweepArgs a{};
  a.n = m->n;
  a.nblocks = p->nblocks;
  a.off = p->d_off;
  a.order = p->d_order;
  a.queue = p->d_queue;
  a.sink = p->d_sink;
  a.obs = obs;
  a.prio_len = p->prio_len;
  a.tile_off = p->d_tile_off;
  return a;
}

#ifdef ITR_DIAG
uint64_t* g_diag = nullptr;  // diagnostic build: per-segment cycle sums of the last sweep
#endif

// tname: kernel timer (nullptr: none); max_grid > 0 caps the persistent grid
// cus: the CUs the launch's stream may use (default: all)
int run_sweep(int mode, itr::SweepArgs a, hipStream_t st, const char* tname,
              int64_t max_grid = -1, int cus = 0, bool zero_queue = true, bool share_cu = false) {
  itr::SweepGeometry g = itr::sweep_geometry(a.n, mode);
  if (g.iq < 0) return fail(ITR_EINVAL, "n_states=%d unsupported", a.n);
  a.xp = g.xp;
  if (cus <= 0) cus = cu_count();
  int64_t grid = (int64_t)g.per_cu * cus;
  if (grid > a.nblocks) grid = a.nblocks;
  if (max_grid > 0 && grid > max_grid) grid = max_grid;
  if (grid <= 0) return 0;
  // one per CU (unless the caller packs several long blocks per CU: share_cu)
  if (grid <= cus && !share_cu) g.lds = std::max(g.lds, itr::kExclusiveLds);
  if (zero_queue) HIP_TRY(hipMemsetAsync(a.queue, 0, sizeof(int), st));
#ifdef ITR_DIAG
  if (getenv("ITR_VERBOSE"))
    fprintf(stderr, "[itr] %s: n=%d cfg=%d block=%d lds=%zu per_cu=%d grid=%lld\n", tname, a.n,
            g.iq, g.block, g.lds, g.per_cu, (long long)grid);
  if (!g_diag) HIP_TRY(hipMalloc(&g_diag, 16 * sizeof(uint64_t)));
  HIP_TRY(hipMemsetAsync(g_diag, 0, 16 * sizeof(uint64_t), st));
  a.diag = g_diag;
  a.diag_wave = getenv("ITR_DIAG_WAVE") ? atoi(getenv("ITR_DIAG_WAVE")) : 0;
#endif
  if (tname) {
    Scope sc(tname, st);
    HIP_TRY(itr::launch_sweep(mode, g, (int)grid, a, st));
  } else {
    HIP_TRY(itr::launch_sweep(mode, g, (int)grid, a, st));
  }
  return 0;
}

// Hybrid sweep (mfma_sweeps.hip): the plan's urgent VALU tasks (v.tasks / v.order, v.nblocks)
// then its matrix-core groups, in one persistent launch.  g from itr::mfma_geometry.
// valu / mfma: launch the VALU tasks / the matrix-core groups (both: one launch; one of them:
// that part only, so the two can run on different CU sets); zero_queues: reset the two work
// counters on `st` first (a split launch resets them once, before both parts).
constexpr int64_t kCombCols = 256;  // columns per combine task of the posterior's backward launch

// nbeta (posterior, forward-store launch): the first nbeta blocks of the order also get a
// backward task storing beta rows into v.beta (over [v.sub_lo[block], T)).
int run_hybrid(int mode, itr_model_t m, itr_plan_t p, itr::SweepArgs v, const itr::MfmaGeometry& g,
               hipStream_t st, const char* tname, bool valu = true, bool mfma = true,
               int64_t max_grid = -1, bool zero_queues = true, int cus = 0,
               bool share_cu = false, int64_t nbeta = 0, int qbase = 3) {
  if (cus <= 0) cus = cu_count();
  itr::MfmaArgs a{};
  a.n = m->n;
  const bool ll = mode == itr::MODE_FWD_LL;
  int64_t nurg = 0;  // posterior: blocks longer than pfrac x the longest are VALU tasks
  if (!ll) {
    const double lim = std::max(512.0, g.pfrac * (double)(p->nblocks ? p->sorted_len[0] : 0));
    while (nurg < p->nblocks && (double)p->sorted_len[nurg] > lim) ++nurg;
    v.order = p->d_order;
    v.nblocks = nurg;
    v.nbeta = mode == itr::MODE_FWD_STORE ? nbeta : 0;
  }
  a.ngroups = ll ? p->ngroups_ll : (p->nblocks - nurg + 3) / 4;
  a.groups = ll ? p->d_groups_ll : p->d_order + nurg;
  a.nmembers = ll ? 0 : p->nblocks - nurg;
  a.tasks = p->d_mtasks;
  a.matT = m->aT;
  a.svec = p->d_svec;
  a.sK = p->d_sK;
  a.queue = p->d_queue + qbase + 1;
  a.off = p->d_off;
  a.obs = v.obs;
  a.mat = m->a;
  a.emit = m->E;
  a.init = m->PIE;
  a.loglik = v.loglik;
  a.alpha = v.alpha;
  a.astride = g.xr;
  a.post = v.post;
  a.sink = v.sink;
  a.prio_len = INT32_MAX;
  v.queue = p->d_queue + qbase;
  v.prio_len = 0;  // every VALU task of the hybrid is a long block: raised wave priority
  // a part launched alone takes the other part's loop through a counter of its own (the
  // real counter belongs to the concurrent launch of that part)
  if (!valu) {
    v.nblocks = 0;
    v.nbeta = 0;
    v.queue = p->d_queue + 8;
  }
  if (!mfma) {
    a.ngroups = 0;
    a.queue = p->d_queue + 9;
  }
  const int64_t work = v.nblocks + v.nbeta + (a.ngroups + g.gb - 1) / g.gb;
  int per_cu = g.per_cu;
  int64_t grid = std::min<int64_t>((int64_t)per_cu * cus, work);
  if (max_grid > 0) grid = std::min(grid, max_grid);
  if (grid <= 0) return 0;
  itr::MfmaGeometry gx = g;
  // one workgroup per CU (unless the caller packs several VALU tasks per CU: share_cu)
  if (grid <= cus && !share_cu) gx.lds_min = itr::kExclusiveLds;
  if (zero_queues) HIP_TRY(hipMemsetAsync(p->d_queue + qbase, 0, 2 * sizeof(int), st));
#ifdef ITR_DIAG
  if (getenv("ITR_VERBOSE"))
    fprintf(stderr, "[itr] %s hybrid: n=%d cfg=%d block=%d per_cu=%d grid=%lld valu=%lld groups=%lld\n",
            tname, a.n, g.cfg, g.block, g.per_cu, (long long)grid, (long long)v.nblocks,
            (long long)a.ngroups);
#endif
  std::optional<Scope> sc;
  if (tname) sc.emplace(tname, st);
  HIP_TRY(itr::launch_hybrid_sweep(mode, gx, (int)grid, a, v, st));
  return 0;
}

// The forward's VALU tasks alone (the plan's urgent tasks: the longest blocks and the split
// ones' halves, v.tasks / v.nblocks) on `st`, at most max_grid at a time: on lane groups
// (lane_groups.h, ~35 VALU instructions per column on one wave per SIMD) where that layout
// exists for the state count, else the hybrid launch's VALU part.  The work counter
// (d_queue[3]) must be zero.
int run_valu_forward(itr_model_t m, itr_plan_t p, itr::SweepArgs v, const itr::MfmaGeometry& g,
                     hipStream_t st, int64_t max_grid, bool share_cu) {
  const itr::FwdGroupGeometry fg = itr::fwd_group_geometry(m->n);
  bool groups = fg.block > 0 && fg.xr == g.xr;
#ifdef ITR_EXPERIMENT
  if (getenv("ITR_NO_FWD_GROUPS")) groups = false;
#endif
  if (groups) {
    v.queue = p->d_queue + 3;
    v.prio_len = 0;
    itr::FwdGroupGeometry gx = fg;
    const int64_t grid = std::min<int64_t>(max_grid, v.nblocks);
    if (grid <= 0) return 0;
    if (!share_cu) gx.lds = std::max(gx.lds, itr::kExclusiveLds);  // one per CU
    HIP_TRY(itr::launch_fwd_group(gx, (int)grid, v, st));
    return 0;
  }
  return run_hybrid(itr::MODE_FWD_LL, m, p, v, g, st, nullptr, true, false, max_grid, false, 0,
                    share_cu);
}

int forward_impl(itr_model_t m, itr_plan_t p, const uint16_t* obs, double* loglik,
                 hipStream_t st, int cus);

}  // namespace

extern "C" {

int itr_version(void) { return 1; }

const char* itr_last_error(void) { return g_err.c_str(); }

int itr_device_count(int* n) {
  if (!n) return fail(ITR_EINVAL, "null pointer");
  HIP_TRY(hipGetDeviceCount(n));
  return 0;
}

int itr_model_create(int n, const double* a, const double* la, const double* E,
                     const double* LE, const double* PIE, const double* LPIE,
                     itr_model_t* out) {
  if (!out) return fail(ITR_EINVAL, "null output pointer");
  *out = nullptr;
  if (n < 1 || n > ITR_MAX_STATES)
    return fail(ITR_EINVAL, "n_states=%d outside [1, %d]", n, ITR_MAX_STATES);
  if (!a || !la || !E || !LE || !PIE || !LPIE) return fail(ITR_EINVAL, "null table pointer");
  auto* m = new itr_model();
  m->n = n;
  if (hipGetDevice(&m->device) != hipSuccess) {
    delete m;
    return fail(ITR_EHIP, "hipGetDevice failed");
  }
  const size_t nn = (size_t)n * n, on = (size_t)ITR_NOBS * n;
  double** dst[6] = {&m->a, &m->la, &m->E, &m->LE, &m->PIE, &m->LPIE};
  const double* src[6] = {a, la, E, LE, PIE, LPIE};
  const size_t cnt[6] = {nn, nn, on, on, on, on};
  for (int i = 0; i < 6; ++i) {
    int e = dev_alloc(dst[i], cnt[i]);
    if (!e && hipMemcpy(*dst[i], src[i], cnt[i] * sizeof(double), hipMemcpyHostToDevice) !=
                  hipSuccess)
      e = fail(ITR_EHIP, "table upload failed");
    if (e) {
      itr_model_destroy(m);
      return e;
    }
  }
  // a^T for the backward halves of split forward sweeps (a layout copy)
  std::vector<double> at((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) at[(size_t)j * n + i] = a[(size_t)i * n + j];
  int e = dev_alloc(&m->aT, nn);
  if (!e && hipMemcpy(m->aT, at.data(), nn * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    e = fail(ITR_EHIP, "table upload failed");
  if (e) {
    itr_model_destroy(m);
    return e;
  }
  if (itr::prune_vit_geometry(n).waves > 0) {  // the bound of the pruned Viterbi step
    std::vector<double> mj(n, -INFINITY);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j)
        if (i != j) mj[j] = std::max(mj[j], la[(size_t)i * n + j]);
    e = dev_alloc(&m->MJ, (size_t)n);
    if (!e && hipMemcpy(m->MJ, mj.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
      e = fail(ITR_EHIP, "table upload failed");
    if (e) {
      itr_model_destroy(m);
      return e;
    }
  }
  const itr::WaveVitGeometry wv = itr::wave_vit_geometry(n);
  if (wv.iq > 0) {  // (the per-wave Viterbi's tables: on the first Viterbi call)
    m->xrw = wv.xr;
    m->h_a.assign(a, a + nn);
    m->h_la.assign(la, la + nn);
    m->h_LE.assign(LE, LE + on);
    m->h_E.assign(E, E + (size_t)256 * n);
    m->h_PIE.assign(PIE, PIE + (size_t)256 * n);
  }
  const itr::WaveMfmaGeometry wf = itr::wave_mfma_geometry(n);
  const bool need_ef = wf.mixed;  // the mixed launch's forward groups
  if (need_ef) {
    const int w = wf.er;
    std::vector<double> ef((size_t)(ITR_NOBS + 1) * w, 0.0);
    for (int o = 0; o < ITR_NOBS; ++o)
      for (int j = 0; j < n; ++j) ef[(size_t)o * w + j] = E[(size_t)o * n + j];
    for (int j = 0; j < w; ++j) ef[(size_t)ITR_NOBS * w + j] = 1.0;
    e = dev_alloc(&m->EF, ef.size());
    if (!e && hipMemcpy(m->EF, ef.data(), ef.size() * sizeof(double), hipMemcpyHostToDevice) !=
                  hipSuccess)
      e = fail(ITR_EHIP, "table upload failed");
    if (e) {
      itr_model_destroy(m);
      return e;
    }
    m->erf = w;
  }
  *out = m;
  return 0;
}

int itr_model_destroy(itr_model_t m) {
  if (!m) return 0;
  dev_free(m->a);
  dev_free(m->la);
  dev_free(m->E);
  dev_free(m->LE);
  dev_free(m->PIE);
  dev_free(m->LPIE);
  dev_free(m->aT);
  dev_free(m->LEW);
  dev_free(m->LEWP);
  dev_free(m->VSLOT);
  dev_free(m->VMB);
  dev_free(m->MJ);
  dev_free(m->EF);
  delete m;
  return 0;
}

int itr_model_n_states(itr_model_t m, int* n) {
  if (!m || !n) return fail(ITR_EINVAL, "null pointer");
  *n = m->n;
  return 0;
}

int itr_plan_reserve(itr_plan_t p, int n, int for_posterior) {
  if (int e = check_plan(p)) return e;
  if (n < 1 || n > ITR_MAX_STATES) return fail(ITR_EINVAL, "bad n_states");
  return reserve(p, n, !for_posterior, for_posterior != 0);
}

int itr_forward_loglik(itr_model_t m, itr_plan_t p, const uint16_t* obs, double* loglik,
                       void* stream) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->nblocks == 0) return 0;
  if ((!obs && p->total > 0) || !loglik) return fail(ITR_EINVAL, "null device pointer");
  return forward_impl(m, p, obs, loglik, (hipStream_t)stream, 0);
}

}  // extern "C"

namespace {

// the forward log-likelihood sweep on a stream that may use `cus` CUs (0: all)
int forward_impl(itr_model_t m, itr_plan_t p, const uint16_t* obs, double* loglik,
                 hipStream_t st, int cus) {
  itr::SweepArgs a = base_args(m, p, obs);
  a.mat = m->a;
  a.matT = m->aT;
  a.emit = m->E;
  a.init = m->PIE;
  a.loglik = loglik;
  a.tasks = p->d_tasks;
  a.nblocks = p->ntasks;
  a.svec = p->d_svec;
  a.sK = p->d_sK;
  if (!a.tasks || (p->nsplit > 0 && (!a.svec || !a.sK || !p->d_split_blk)))
    return fail(ITR_ESTATE, "forward task tables missing");
  const itr::MfmaGeometry g = itr::mfma_geometry(m->n, itr::MODE_FWD_LL);
  int xr = itr::sweep_row_stride(m->n, itr::MODE_FWD_LL);
  if (g.cfg >= 0 && p->ngroups_ll > 0) {
    a.tasks = p->d_utasks;
    a.nblocks = p->nutasks;
    const itr::FwdGroupGeometry fgeo = itr::fwd_group_geometry(m->n);
    bool part = cus == 0 && p->nutasks > 0 && fgeo.block > 0 && fgeo.xr == g.xr;
#ifdef ITR_EXPERIMENT
    if (getenv("ITR_NO_FWD_GROUPS")) part = false;
#endif
    if (part) {
      // The VALU tasks (the longest blocks' halves) one per reserved CU on the lane-group
      // layout, the matrix-core groups on the other CUs; the reserved CUs join the groups when
      // their task is done.  The set: one CU per task, in whole XCC sets, at most a quarter of
      // the chip (masked streams: a group workgroup beside a running half slows it down)
      const int ncu = cu_count();
      const int X = (ncu % 8 == 0) ? 8 : 1;
      int rfr = (int)std::min<int64_t>((p->nutasks + X - 1) / X * X, ncu / 4);
      Partition* pt = nullptr;
      int rv = 0;  // a Viterbi set left by a forward + Viterbi call: matrix-core groups there too
      bool reused = false;
      // The thread keeps one partition per device; re-creating its CU-masked streams for each
      // call of an alternating loglik / viterbi sequence (the host-block wrappers) cost ~40 ms
      // a call, so the forward takes the forward + Viterbi call's partition when there is one.
      // (a partition without a second set has lng2 on lng's CUs: the halves go there)
      if (Partition* cur = current_partition())
        if (cur->masked && cur->reserve > 0) {
          pt = cur;
          reused = true;
          rv = cur->reserve2 > 0 ? cur->reserve : 0;
          rfr = cur->reserve2 > 0 ? cur->reserve2 : cur->reserve;
        }
      if (!pt)
        if (int e = partition(0, rfr, &pt)) return e;
      Scope sc("forward", st);
      HIP_TRY(hipMemsetAsync(p->d_queue + 3, 0, 2 * sizeof(int), st));
      HIP_TRY(hipEventRecord(pt->fork, st));
      HIP_TRY(hipStreamWaitEvent(pt->lng2, pt->fork, 0));
      HIP_TRY(hipStreamWaitEvent(pt->blk, pt->fork, 0));
      if (rv > 0) HIP_TRY(hipStreamWaitEvent(pt->lng, pt->fork, 0));
      if (int e = run_hybrid(itr::MODE_FWD_LL, m, p, a, g, pt->blk, nullptr, false, true,
                             (int64_t)g.per_cu * (ncu - rfr - rv), false, ncu - rfr - rv))
        return e;
      if (rv > 0)
        if (int e = run_hybrid(itr::MODE_FWD_LL, m, p, a, g, pt->lng, nullptr, false, true,
                               (int64_t)g.per_cu * rv, false, rv))
          return e;
      // (on a forward + Viterbi partition the set was sized for fwd_per_cu halves per CU)
      const int64_t fg = reused ? std::max<int64_t>(rfr, std::min<int64_t>(
                                      p->nutasks, (int64_t)std::max(1, p->fwd_per_cu) * rfr))
                                : rfr;
      if (int e = run_valu_forward(m, p, a, g, pt->lng2, fg, fg > rfr)) return e;
      if (int e = run_hybrid(itr::MODE_FWD_LL, m, p, a, g, pt->lng2, nullptr, false, true,
                             (int64_t)g.per_cu * rfr, false, rfr))
        return e;
      HIP_TRY(hipEventRecord(pt->jl2, pt->lng2));
      HIP_TRY(hipEventRecord(pt->jb, pt->blk));
      HIP_TRY(hipStreamWaitEvent(st, pt->jl2, 0));
      HIP_TRY(hipStreamWaitEvent(st, pt->jb, 0));
      if (rv > 0) {
        HIP_TRY(hipEventRecord(pt->jl, pt->lng));
        HIP_TRY(hipStreamWaitEvent(st, pt->jl, 0));
      }
    } else if (int e = run_hybrid(itr::MODE_FWD_LL, m, p, a, g, st, "forward", true, true, -1,
                                  true, cus)) {
      return e;
    }
    HIP_TRY(itr::launch_fwd_split_combine(m->n, g.xr, (int)p->nhsplit, p->d_hsplit_blk,
                                          p->d_svec, p->d_sK, loglik, st));
    return 0;
  }
  if (int e = run_sweep(itr::MODE_FWD_LL, a, st, "forward", -1, cus)) return e;
  HIP_TRY(itr::launch_fwd_split_combine(m->n, xr, (int)p->nsplit, p->d_split_blk, p->d_svec,
                                        p->d_sK, loglik, st));
  return 0;
}

// The per-wave Viterbi's slot order (wave_tasks.h): a target column r of the layout is
// scanned when any of its 8 target slots fails the bound test, so the states that fail
// most often share the first columns.  How often a state fails is measured once per model
// on the host: the bound test along 2,048 columns drawn from the model itself (8 blocks of
// 256, hidden path from pi and a, N-free symbols from E), a few ms at N = 70.  The order only
// moves work between scan columns; the decoded path does not depend on it.
int vit_slot_tables(itr_model_t m) {
  std::lock_guard<std::mutex> lock(m->vit_mu);
  if (m->LEW) return 0;
  const int n = m->n, w = m->xrw;
  const std::vector<double>& la = m->h_la;
  std::vector<double> mj(n, -INFINITY);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      if (i != j) mj[j] = std::max(mj[j], la[(size_t)i * n + j]);
  std::vector<int> rank(n);
  std::iota(rank.begin(), rank.end(), 0);
  // how often each state fails the pruned step's bound on 8 sequences of 256 columns
  // sampled from the model (one host thread per sequence, each with its own generator)
  constexpr int kSeq = 8;
  std::vector<std::vector<int64_t>> fails_b(kSeq, std::vector<int64_t>(n, 0));
  std::vector<double> pi_w(n, 0.0);
  for (int j = 0; j < n; ++j)
    for (int o = 0; o < 256; ++o) pi_w[j] += m->h_PIE[(size_t)o * n + j];
  auto sequence = [&](int b) {
    uint64_t rs = 0x2545F4914F6CDD1Dull + 0x632BE59BD9B4E019ull * (uint64_t)b;
    auto rnd = [&]() {  // splitmix64 -> [0, 1)
      uint64_t z = (rs += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      return (double)((z ^ (z >> 31)) >> 11) * 0x1.0p-53;
    };
    auto draw = [&](auto&& prob, int cnt) {  // index by cumulative weight
      double tot = 0.0;
      for (int k = 0; k < cnt; ++k) tot += prob(k);
      double u = rnd() * tot;
      for (int k = 0; k < cnt; ++k) {
        u -= prob(k);
        if (u < 0.0) return k;
      }
      return cnt - 1;
    };
    std::vector<int64_t>& fails = fails_b[b];
    std::vector<double> om(n), nx(n);
    int s = draw([&](int j) { return pi_w[j]; }, n);
    int o = draw([&](int k) { return m->h_E[(size_t)k * n + s]; }, 256);
    for (int j = 0; j < n; ++j) om[j] = std::log(m->h_PIE[(size_t)o * n + j]);
    for (int t = 1; t < 256; ++t) {
      s = draw([&](int j) { return m->h_a[(size_t)s * n + j]; }, n);
      o = draw([&](int k) { return m->h_E[(size_t)k * n + s]; }, 256);
      const double* le = m->h_LE.data() + (size_t)o * n;
      const double top = *std::max_element(om.begin(), om.end());
      for (int j = 0; j < n; ++j) {
        const double yd = (om[j] + la[(size_t)j * n + j]) + le[j];
        if (!(yd > (top + mj[j]) + le[j])) ++fails[j];
        double yo = -INFINITY;
        for (int i = 0; i < n; ++i)
          if (i != j) yo = std::max(yo, om[i] + la[(size_t)i * n + j]);
        nx[j] = std::max(yd, yo + le[j]);
      }
      om.swap(nx);
    }
  };
  parallel_for(std::min(kSeq, host_threads()) == kSeq ? kSeq : 1, [&](int w) {
    if (std::min(kSeq, host_threads()) == kSeq) {
      sequence(w);
    } else {
      for (int b = 0; b < kSeq; ++b) sequence(b);
    }
  });
  std::vector<int64_t> fails(n, 0);
  for (int b = 0; b < kSeq; ++b)
    for (int j = 0; j < n; ++j) fails[j] += fails_b[b][j];
  std::stable_sort(rank.begin(), rank.end(), [&](int x, int y) { return fails[x] > fails[y]; });
  // rank k < 64: column k / 8 of group k % 8 (A slots); then the groups' B slots (column 8)
  const int iq = w / 8;
  std::vector<int32_t> slot(w, -1);
  for (int k = 0; k < n; ++k)
    slot[k < 8 * (iq - 1) ? iq * (k % 8) + k / 8 : iq * (k - 8 * (iq - 1)) + iq - 1] = rank[k];
  // log E padded to w columns: by state (full scan) and by slot (pruned step)
  std::vector<double> lew((size_t)ITR_NOBS * w, -INFINITY), lewp(lew.size(), -INFINITY),
      vmb(w, -INFINITY);
  for (int o = 0; o < ITR_NOBS; ++o)
    for (int j = 0; j < n; ++j) lew[(size_t)o * w + j] = m->h_LE[(size_t)o * n + j];
  for (int sl = 0; sl < w; ++sl) {
    if (slot[sl] < 0) continue;
    vmb[sl] = mj[slot[sl]];
    for (int o = 0; o < ITR_NOBS; ++o) lewp[(size_t)o * w + sl] = m->h_LE[(size_t)o * n + slot[sl]];
  }
  int e = dev_alloc(&m->VSLOT, (size_t)w);
  if (!e) e = dev_alloc(&m->VMB, (size_t)w);
  if (!e) e = dev_alloc(&m->LEW, lew.size());
  if (!e) e = dev_alloc(&m->LEWP, lewp.size());
  if (!e && (hipMemcpy(m->VSLOT, slot.data(), w * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(m->VMB, vmb.data(), w * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(m->LEW, lew.data(), lew.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(m->LEWP, lewp.data(), lewp.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess))
    e = fail(ITR_EHIP, "table upload failed");
  if (e) {
    dev_free(m->VSLOT);
    dev_free(m->VMB);
    dev_free(m->LEW);
    dev_free(m->LEWP);
    return e;
  }
  for (auto* v : {&m->h_a, &m->h_la, &m->h_LE, &m->h_E, &m->h_PIE}) std::vector<double>().swap(*v);
  return 0;
}

// The Viterbi sweep and traceback of every block into `path`; with fwd_loglik, the forward
// log-likelihood sweep too, overlapped with the Viterbi sweep's longest blocks.
//
// Work placement.  A block's sweep is a strictly sequential chain, so the
// longest blocks need the lowest step latency and the bulk the highest throughput:
//   * the longest blocks' Viterbi (longer than 0.55 x the longest, >= 2,048 columns): the
//     9-wave VALU layout, one workgroup per CU, on `reserve` CUs (CU-masked stream lng);
//   * with the forward: its latency-bound VALU tasks (halves of the longest blocks) on rf of
//     those reserved CUs (lng2), and on the other CUs (blk) ONE persistent launch of
//     per-wavefront tasks from a single queue ordered by expected duration: forward groups
//     of four tasks on the matrix cores and one Viterbi block per wave (wave_sweeps.hip);
//   * without the mixed launch (other state counts): the forward's matrix-core groups, then
//     the per-wave Viterbi on blk.
// When the long blocks would keep the reserved CUs busy longer than the rest keeps the
// others (few, equally long blocks), every block goes to the 9-wave layout: with the
// forward and at most 3/4 as many blocks as CUs, one CU per block and the forward on the
// remaining CUs at the same time; otherwise on all CUs after the forward.
int viterbi_impl(itr_model_t m, itr_plan_t p, const uint16_t* obs, uint8_t* path,
                 hipStream_t st, double* fwd_loglik) {
  if (int e = reserve(p, m->n, true, false)) return e;
  std::optional<Scope> both;  // the combined call's timer: fork to join, traceback excluded
  if (fwd_loglik) both.emplace("forward_viterbi", st);
  itr::SweepArgs a = base_args(m, p, obs);
  a.mat = m->la;
  a.emit = m->LE;
  a.init = m->LPIE;
  a.queue = p->d_queue + 2;  // own counter: may run concurrently with a forward sweep
  a.xrec = vit_stride(m->n);  // (the record stride every Viterbi layout of this call writes)
  a.alpha = p->d_alpha;
  a.stay = p->d_stay;
  a.last_state = p->d_last;
  // traceback of blocks order[from, from + count) (vit_trace_kernel); the long blocks'
  // tracebacks run on their reserved CUs right after their Viterbi sweep (`traced` of them),
  // the rest after the join
  auto trace_args = [&]() {
    itr::TraceArgs ta{};
    ta.n = m->n;
    ta.xr = vit_stride(m->n);
    ta.off = p->d_off;
    ta.tile_off = p->d_tile_off;
    ta.queue = p->d_queue + 1;
    ta.obs = obs;
    ta.log_a = m->la;
    ta.log_e = m->LE;
    ta.ckpt = p->d_alpha;
    ta.stay = p->d_stay;
    ta.last_state = p->d_last;
    ta.path = path;
    return ta;
  };
  int64_t traced = 0;
  int64_t trace_end = p->nblocks;  // the final traceback walks order[traced, trace_end)
  const itr::WaveVitGeometry wv = itr::wave_vit_geometry(m->n);
  bool wave = wv.iq > 0 && m->xrw == wv.xr;
  const int cus = cu_count();
  if (wave && !p->wave_ok) wave = false;  // the long work would need more than half the CUs
  if (wave)
    if (int e = vit_slot_tables(m)) return e;
  // the reserved CU sets (plan_partition: sized for the forward+Viterbi call; the
  // Viterbi-only call runs on the same CU-masked streams, with its own long set swept by
  // both sets)
  const int64_t nlong_c = wave ? p->vit_nlong : 0;
  const int64_t rf0 = p->fwd_reserve;
  const int64_t rv0 = nlong_c > 0 ? std::max(1, p->vit_reserve) : 0;
  // whole XCC sets: a mask that leaves an XCC without a reserved CU does not mask it at all
  const int X = (cus % 8 == 0) ? 8 : 1;
  const int Xr = X;  // rounding unit of the reserved sets
  const int rvr = (int)std::min<int64_t>((rv0 + Xr - 1) / Xr * Xr, cus / 2);
  const int rfr = (int)std::min<int64_t>((rf0 + Xr - 1) / Xr * Xr, cus / 4);
  const int reserve_cus = rvr + rfr;
  const bool vonly = fwd_loglik == nullptr;
  const int64_t nlong = vonly ? (wave && reserve_cus > 0 ? p->vit_nlong_v : 0) : nlong_c;
  // Few blocks, all long (e.g. 100 blocks of 100 kbp): one CU per block for the 9-wave
  // Viterbi sweep and the forward sweep beside it on the remaining CUs (at least a quarter
  // of the chip), instead of one after the other
  // Small models (N <= 48, e.g. the reference's example (3,3) model, N = 27): both sweeps
  // are bound by the longest block's step latency, not by throughput (10 Mbp at N = 27:
  // Viterbi 3.6 ms = 18,377 x 195 ns, forward 2.0 ms), so they run side by side on two halves
  // of the chip instead of one after the other
  const bool small = !wave && fwd_loglik && m->n <= 48;
  const bool few = !wave && fwd_loglik && (p->nblocks <= cus - cus / 4 || small);
  if (few) {
    // the Viterbi blocks alone on their CUs (masked), the forward on the others with as
    // many workgroups per CU as it needs to run every task at once (100 x 100 kbp: 200
    // halves on 156 CUs; one per CU queued a second round: 62 ms, unmasked 36.5 ms,
    // profiles/r3t_partition.txt)
    Partition* pt = nullptr;
    // one CU per block in whole shader-engine sets (32 CUs: one per engine of every XCC):
    // the dispatcher deals the blocks' workgroups to the engines in turn
    const int X = (cus % 32 == 0) ? 32 : 1;
    const int rv = small ? (cus / 2 + X - 1) / X * X
                         : (int)std::min<int64_t>((p->nblocks + X - 1) / X * X, cus - cus / 4);
    if (int e = partition(rv, 0, &pt)) return e;
    HIP_TRY(hipEventRecord(pt->fork, st));
    HIP_TRY(hipStreamWaitEvent(pt->lng, pt->fork, 0));
    HIP_TRY(hipStreamWaitEvent(pt->blk, pt->fork, 0));
    if (int e = run_sweep(itr::MODE_VIT, a, pt->lng, nullptr, p->nblocks, rv)) return e;
    if (int e = forward_impl(m, p, obs, fwd_loglik, pt->blk, cus - rv)) return e;
    HIP_TRY(hipEventRecord(pt->jl, pt->lng));
    HIP_TRY(hipEventRecord(pt->jb, pt->blk));
    HIP_TRY(hipStreamWaitEvent(st, pt->jl, 0));
    HIP_TRY(hipStreamWaitEvent(st, pt->jb, 0));
  } else if (!wave && fwd_loglik) {  // no overlap: the forward sweep first, on st
    if (int e = forward_impl(m, p, obs, fwd_loglik, st, 0)) return e;
  }
  if (wave) {
    itr::VitArgs w{};
    w.n = m->n;
    w.xr = wv.xr;
    w.nblocks = p->nblocks - nlong;
    w.order = p->d_order + nlong;
    w.queue = p->d_queue + 7;
    w.off = p->d_off;
    w.tile_off = p->d_tile_off;
    w.obs = obs;
    w.la = m->la;
    w.lew = m->LEW;
    w.lpie = m->LPIE;
    w.slot_state = m->VSLOT;
    w.slot_m = m->VMB;
    w.lew_p = m->LEWP;
    w.prune_len = p->prune_override >= 0
                      ? (int)std::min<int64_t>(p->prune_override, INT32_MAX)
                      : (vonly ? p->vit_prune_len_v : p->vit_prune_len);
    w.log_e = m->LE;  // each bulk block traced by its wave right after its sweep
    w.path = path;
    trace_end = nlong;
    w.ckpt = p->d_alpha;
    w.stay = p->d_stay;
    w.last_state = p->d_last;
    // the bulk's longest blocks (about one per SIMD pair) at raised wave priority
    w.prio_len = (int)std::max<int64_t>(1, p->sorted_len[std::min<int64_t>(p->nblocks - 1,
                                                                          nlong + cus / 2)]);
    std::optional<Scope> sc;
    if (!fwd_loglik) sc.emplace("viterbi", st);
    Partition* pt = nullptr;
    const itr::MfmaGeometry gf = itr::mfma_geometry(m->n, itr::MODE_FWD_LL);
    const itr::WaveMfmaGeometry wf = itr::wave_mfma_geometry(m->n);
    // the forward's VALU tasks (halves of the longest blocks) on rf reserved CUs, the long
    // blocks' Viterbi on rv others (plan_partition)
    const bool hyb_fwd = fwd_loglik && gf.cfg >= 0 && p->ngroups_ll > 0;
    const bool split_fwd = hyb_fwd && p->nutasks > 0 && p->fwd_reserve > 0;
    // (the mixed launch also serves a forward without VALU tasks: every half in the groups)
    bool mixed = hyb_fwd && (split_fwd || p->nutasks == 0) && wf.mixed && m->EF && p->nmix > 0;
    itr::SweepArgs af = base_args(m, p, obs);
    af.mat = m->a;
    af.matT = m->aT;
    af.emit = m->E;
    af.init = m->PIE;
    af.loglik = fwd_loglik;
    af.tasks = p->d_utasks;
    af.nblocks = p->nutasks;
    af.svec = p->d_svec;
    af.sK = p->d_sK;
    // (the forward's reserved set exists without the forward too — one partition, one set
    // of streams per plan; the Viterbi-only call sweeps its long set on it too)
    // every work counter of this call, [2] .. [13], in one memset before the fork (the bulk
    // queue is shared with the reserved CUs' late launches)
    HIP_TRY(hipMemsetAsync(p->d_queue + 2, 0, 12 * sizeof(int), st));
    hipStream_t sb = st;
    const int ocus = cus - reserve_cus;  // CUs of the sb launches
    // the mixed launch: forward groups (the hybrid plan's matrix-core tasks) and the per-wave
    // Viterbi blocks from one queue ordered by expected duration (plan: mix list)
    itr::WaveMfmaArgs f{};
    if (mixed) {
      f.n = m->n;
      f.ngroups = p->ngroups_ll;
      f.groups = p->d_groups_ll;
      f.tasks = p->d_mtasks;
      f.off = p->d_off;
      f.obs = obs;
      f.a = m->a;
      f.aT = m->aT;
      f.ef = m->EF;
      f.emit = m->E;
      f.init = m->PIE;
      f.loglik = fwd_loglik;
      f.svec = p->d_svec;
      f.sstride = gf.xr;
      f.sK = p->d_sK;
      f.prio_len = p->mix_prio_fwd;
      w.prio_len = p->mix_prio_vit;
    }
    auto launch_bulk = [&]() -> int {  // (the makespan's critical path: enqueued first)
      const int64_t grid = std::min<int64_t>((int64_t)wf.mixed_per_cu * ocus, (p->nmix + 3) / 4);
      HIP_TRY(itr::launch_wave_mixed(wf, (int)grid, w, f, p->d_mix, (int)p->nmix,
                                     p->d_queue + 12, sb));
      return 0;
    };
    if (reserve_cus > 0) {
      // the long blocks' Viterbi on lng (rvr CUs), the forward's VALU halves on lng2 (rfr
      // others): separate masks, so each set joins the bulk queue as soon as its own long
      // work is done without a bulk workgroup landing beside a running long task
      if (int e = partition(rvr, rfr, &pt)) return e;
      HIP_TRY(hipEventRecord(pt->fork, st));
      HIP_TRY(hipStreamWaitEvent(pt->blk, pt->fork, 0));
      HIP_TRY(hipStreamWaitEvent(pt->lng, pt->fork, 0));
      HIP_TRY(hipStreamWaitEvent(pt->lng2, pt->fork, 0));
      sb = pt->blk;
      if (mixed)
        if (int e = launch_bulk()) return e;
      if (nlong > 0 && !vonly) {
        a.nblocks = nlong;
        const int lpc = p->long_per_cu;
        if (int e = run_sweep(itr::MODE_VIT, a, pt->lng, nullptr, (int64_t)lpc * rvr, 0, false,
                              lpc > 1))
          return e;
        itr::TraceArgs tl = trace_args();
        tl.nblocks = nlong;
        tl.order = p->d_order;
        tl.queue = p->d_queue + 13;
        HIP_TRY(itr::launch_vit_traceback(tl, (int)std::min<int64_t>((nlong + 3) / 4, 4 * rvr),
                                          pt->lng));
        traced = nlong;
      } else if (nlong > 0) {  // Viterbi alone: both reserved sets sweep the long set
        a.nblocks = nlong;
        const int lpc = p->long_per_cu;
        if (rvr > 0)
          if (int e = run_sweep(itr::MODE_VIT, a, pt->lng, nullptr, (int64_t)lpc * rvr, 0, false,
                                lpc > 1))
            return e;
        if (rfr > 0)
          if (int e = run_sweep(itr::MODE_VIT, a, pt->lng2, nullptr, (int64_t)lpc * rfr, 0, false,
                                lpc > 1))
            return e;
      }
      if (split_fwd) {
        const int64_t fg = (int64_t)p->fwd_per_cu * rfr;  // forward halves at a time on the set
        if (int e = run_valu_forward(m, p, af, gf, pt->lng2, fg, fg > rfr)) return e;
      }
    } else if (mixed) {
      if (int e = launch_bulk()) return e;
    }
    if (mixed) {
      if (pt) {  // the reserved CUs join the bulk queue when their long work is done
        if (rvr > 0)
          HIP_TRY(itr::launch_wave_mixed(wf, wf.mixed_per_cu * rvr, w, f, p->d_mix,
                                         (int)p->nmix, p->d_queue + 12, pt->lng, 1));
        if (rfr > 0)
          HIP_TRY(itr::launch_wave_mixed(wf, wf.mixed_per_cu * rfr, w, f, p->d_mix,
                                         (int)p->nmix, p->d_queue + 12, pt->lng2, 2));
      }
    } else {
      if (split_fwd) {
        if (int e = run_hybrid(itr::MODE_FWD_LL, m, p, af, gf, sb, nullptr, false, true,
                               (int64_t)gf.per_cu * ocus, false))
          return e;
      } else if (fwd_loglik) {
        if (int e = forward_impl(m, p, obs, fwd_loglik, sb, ocus)) return e;
      }
      if (w.nblocks > 0) {  // the per-wave sweep: after the forward's matrix-core groups
        const int64_t grid = std::min<int64_t>((int64_t)wv.per_cu * ocus, (w.nblocks + 3) / 4);
        HIP_TRY(itr::launch_wave_vit(wv, (int)grid, w, sb));
        if (pt && rvr > 0)  // the reserved CUs join when their long work is done
          HIP_TRY(itr::launch_wave_vit(wv, wv.per_cu * rvr, w, pt->lng, 1));
        if (pt && rfr > 0)
          HIP_TRY(itr::launch_wave_vit(wv, wv.per_cu * rfr, w, pt->lng2, 2));
      }
    }
    if (pt) {
      HIP_TRY(hipEventRecord(pt->jl, pt->lng));
      HIP_TRY(hipEventRecord(pt->jb, pt->blk));
      HIP_TRY(hipStreamWaitEvent(st, pt->jl, 0));
      HIP_TRY(hipStreamWaitEvent(st, pt->jb, 0));
      HIP_TRY(hipEventRecord(pt->jl2, pt->lng2));
      HIP_TRY(hipStreamWaitEvent(st, pt->jl2, 0));
    }
    if (split_fwd || mixed)  // log P of the split blocks from their two halves
      HIP_TRY(itr::launch_fwd_split_combine(m->n, gf.xr, (int)p->nhsplit, p->d_hsplit_blk,
                                            p->d_svec, p->d_sK, fwd_loglik, st));
  } else if (!few) {
    const itr::PruneVitGeometry pg = itr::prune_vit_geometry(m->n);
    // Only where it measured faster (profiles/r5h_pv_lab.txt): N = 133 on short blocks
    // (mean 300: 5.4 vs 8.2 ms per 3 Mbp).  Its scans read log a from LDS, so a column costs
    // LDS bandwidth in proportion to its failing targets: 6 % of them fail on short blocks,
    // 15 % on the config-2 layout (71 vs 25 ms) and 46 % deep inside long blocks (3.2 us per
    // lone column vs 0.64 on the 9-wave layout); at N = 95 the 9-wave layout wins throughout.
    const int64_t mean_len = p->total / std::max<int64_t>(1, p->nblocks);
    // (at least four blocks per CU: N = 137..140 fit one or two beside the matrix, far below
    // the measured regime; N = 141..144 do not fit at all, pg.waves = 0)
    bool prune = pg.waves >= 4 && m->MJ && m->n > 128 && mean_len <= 400 &&
                 p->nblocks > 2 * cus;
    if (prune) {
      // one block per wavefront, log a in LDS, the bound-pruned step (prune_vit.hip)
      itr::PruneVitArgs v{};
      v.n = m->n;
      v.xr = vit_stride(m->n);
      v.nblocks = p->nblocks;
      v.order = p->d_order;
      v.queue = p->d_queue + 2;
      v.off = p->d_off;
      v.tile_off = p->d_tile_off;
      v.obs = obs;
      v.la = m->la;
      v.mj = m->MJ;
      v.log_e = m->LE;
      v.lpie = m->LPIE;
      v.ckpt = p->d_alpha;
      v.stay = p->d_stay;
      v.last_state = p->d_last;
      // the blocks long enough to be the makespan (about one per SIMD) at raised priority
      v.prio_len = (int)std::max<int64_t>(
          1, p->sorted_len[std::min<int64_t>(p->nblocks - 1, (int64_t)cus * 4)]);
      HIP_TRY(hipMemsetAsync(v.queue, 0, sizeof(int), st));
      const int64_t grid = std::min<int64_t>(cus, (p->nblocks + pg.waves - 1) / pg.waves);
      std::optional<Scope> sc;
      if (!fwd_loglik) sc.emplace("viterbi", st);
      HIP_TRY(itr::launch_prune_vit(pg, (int)grid, v, st));
    } else {
      if (int e = run_sweep(itr::MODE_VIT, a, st, "viterbi")) return e;
    }
  }
  both.reset();
  itr::TraceArgs ta = trace_args();
  ta.nblocks = std::max<int64_t>(0, trace_end - traced);
  ta.order = p->d_order + traced;
  // one wave per block, 4 waves per workgroup (LDS: 4 x 16 recomputed rows)
  const int64_t grid = std::min<int64_t>((ta.nblocks + 3) / 4, (int64_t)cu_count() * 4);
  if (ta.nblocks > 0) HIP_TRY(hipMemsetAsync(ta.queue, 0, sizeof(int), st));
  Scope sc("traceback", st);
  if (ta.nblocks > 0) HIP_TRY(itr::launch_vit_traceback(ta, (int)grid, st));
  return 0;
}

}  // namespace

extern "C" {

int itr_viterbi(itr_model_t m, itr_plan_t p, const uint16_t* obs, uint8_t* path,
                void* stream) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->nblocks == 0 || p->total == 0) return 0;
  if (!obs || !path) return fail(ITR_EINVAL, "null device pointer");
  return viterbi_impl(m, p, obs, path, (hipStream_t)stream, nullptr);
}

int itr_forward_viterbi(itr_model_t m, itr_plan_t p, const uint16_t* obs, double* loglik,
                        uint8_t* path, void* stream) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->nblocks == 0) return 0;
  if (!obs || !path || !loglik) return fail(ITR_EINVAL, "null device pointer");
  if (p->total == 0) return itr_forward_loglik(m, p, obs, loglik, stream);
  return viterbi_impl(m, p, obs, path, (hipStream_t)stream, loglik);
}

int itr_block_rows(itr_model_t m, int kind, const uint16_t* obs, int64_t T, double* rows,
                   double* prev, void* stream) {
  if (int e = check_model(m)) return e;
  if (kind < 0 || kind > 2) return fail(ITR_EINVAL, "kind %d is not 0, 1 or 2", kind);
  if (T < 1) return fail(ITR_EINVAL, "a block of %lld columns (the reference indexes V[0])",
                         (long long)T);
  if (!obs || !rows) return fail(ITR_EINVAL, "null device pointer");
  itr::RowArgs a{};
  a.kind = kind;
  a.n = m->n;
  a.T = T;
  a.obs = obs;
  a.a = m->a;
  a.log_a = m->la;
  a.emit = m->E;
  a.log_emit = m->LE;
  a.lpie = m->LPIE;
  a.rows = rows;
  a.prev = kind == 2 ? prev : nullptr;
  HIP_TRY(itr::launch_rows(a, (hipStream_t)stream));
  return 0;
}

int itr_model_prepare_viterbi(itr_model_t m) {
  if (int e = check_model(m)) return e;
  if (m->xrw == 0) return 0;  // (no per-wave layout for this state count)
  return vit_slot_tables(m);
}

int itr_backtrack_rows(const double* omega, const double* prev, int64_t T, int n, double* path,
                       void* stream) {
  if (T < 1 || n < 1 || n > ITR_MAX_STATES) return fail(ITR_EINVAL, "bad T / n");
  if (!omega || !path || (T > 1 && !prev)) return fail(ITR_EINVAL, "null device pointer");
  HIP_TRY(itr::launch_backtrack_rows(omega, prev, T, n, path, (hipStream_t)stream));
  return 0;
}

int itr_posterior(itr_model_t m, itr_plan_t p, const uint16_t* obs, double* post,
                  void* stream) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->nblocks == 0 || p->total == 0) return 0;
  if (!obs || !post) return fail(ITR_EINVAL, "null device pointer");
  if (int e = reserve(p, m->n, false, true)) return e;
  hipStream_t st = (hipStream_t)stream;
  itr::SweepArgs a = base_args(m, p, obs);
  a.mat = m->a;
  a.emit = m->E;
  a.init = m->PIE;
  a.alpha = p->d_alpha;
  const itr::MfmaGeometry g = itr::mfma_geometry(m->n, itr::MODE_FWD_STORE);
  if (g.cfg >= 0 && !post_split_path(m->n, p)) {
    // forward rows at the hybrid's stride g.xr for every block (reserve() sized for it)
    const itr::MfmaGeometry gb = itr::mfma_geometry(m->n, itr::MODE_BWD);
    // The longest blocks (at least g.bfrac of the longest) are split at column
    // lo = g.lofrac x T: their backward sweep over [lo, T) (beta rows) runs beside their
    // forward sweep in the forward launch, the backward launch's VALU task sweeps [0, lo]
    // from the stored beta_lo, and post_combine forms the posteriors of (lo, T).  A whole
    // VALU backward + posterior sweep (~0.95 us per column at N = 133) outlasts the
    // matrix-core bulk of the backward launch.  (Splitting the forward sweep as well — a
    // forward + posterior sweep over [hi, T) in the backward launch — measured slower: 24.1
    // against 23.0 ms per (7,7) posterior, profiles/r5ps3_*.)
    double lofrac = g.lofrac;
#ifdef ITR_EXPERIMENT
    if (getenv("ITR_POST_LO")) lofrac = atof(getenv("ITR_POST_LO"));
#endif
    // (split blocks are VALU tasks of the backward launch: a prefix of its VALU set, whose
    // limit mirrors run_hybrid's; their forward sweep is a VALU task or a matrix-core group)
    const auto [nbeta, brows] = hybrid_beta_set(p, m->n);
    if (nbeta > 0 && p->sublo_key != std::make_pair(nbeta, lofrac)) {
      if (!p->d_sublo)
        if (int e = dev_alloc(&p->d_sublo, p->nblocks)) return e;
      std::vector<int64_t> lo(p->nblocks, 0), comb;
      for (int64_t k = 0; k < nbeta; ++k) {  // (blocks >= 512 columns)
        const int64_t T = p->sorted_len[k];
        const int64_t l = std::clamp<int64_t>((int64_t)(lofrac * (double)T), 1, T - 2);
        lo[p->h_order[k]] = l;
        for (int64_t t0 = l + 1; t0 < T; t0 += kCombCols)  // combine tasks of (lo, T)
          comb.insert(comb.end(), {p->h_order[k], t0, std::min(T, t0 + kCombCols)});
      }
      HIP_TRY(hipMemcpy(p->d_sublo, lo.data(), lo.size() * sizeof(int64_t),
                        hipMemcpyHostToDevice));
      dev_free(p->d_comb);
      p->d_comb = nullptr;
      if (int e = dev_alloc(&p->d_comb, comb.size())) return e;
      HIP_TRY(hipMemcpy(p->d_comb, comb.data(), comb.size() * sizeof(int64_t),
                        hipMemcpyHostToDevice));
      p->ncomb = (int64_t)comb.size() / 3;
      p->sublo_key = {nbeta, lofrac};
    }
    if (nbeta > 0 && (size_t)brows * g.xr > p->beta_cap) {
      dev_free(p->d_beta);
      p->beta_cap = 0;
      if (int e = dev_alloc(&p->d_beta, (size_t)brows * g.xr)) return e;
      p->beta_cap = (size_t)brows * g.xr;
    }
    if (nbeta > 0) {
      a.beta = p->d_beta;
      a.beta_off = p->d_boff;
      a.sub_lo = p->d_sublo;
    }
    // the two launches' work counters ([3, 4] forward, [5, 6] backward) and the combine
    // tasks' ([7]) zeroed by one memset up front
    HIP_TRY(hipMemsetAsync(p->d_queue + 3, 0, 5 * sizeof(int), st));
    // (the longest blocks' forward sweeps on lane groups, one per reserved CU beside the
    // matrix-core groups on the others, measured slower: 18.2 against 15.2 ms per (5,5)
    // posterior — the groups lost 80 CUs for most of the launch, profiles/r6d_posterior_ab.txt;
    // in one launch a VALU task and a group workgroup share each CU)
    if (int e = run_hybrid(itr::MODE_FWD_STORE, m, p, a, g, st, "posterior_fwd", true, true, -1,
                           false, 0, false, nbeta))
      return e;
    a.post = post;
    a.beta = nullptr;
    a.beta_in = nbeta > 0 ? p->d_beta : nullptr;
    // the combine of (lo, T) as tasks at the end of the backward launch's queue (a launch of
    // its own after it: 0.2-0.27 ms; beside it on a side stream it delayed that launch's
    // workgroups by as much as it saved, profiles/r5ptl3_*)
    if (nbeta > 0) {
      a.comb = p->d_comb;
      a.ncomb = p->ncomb;
      a.comb_queue = p->d_queue + 7;
    }
    return run_hybrid(itr::MODE_BWD, m, p, a, gb, st, "posterior_bwd", true, true, -1, false, 0,
                      false, 0, 5);
  }
  const int nl = (int)p->npsplit;
  if (post_split_path(m->n, p)) {
    // the longest blocks: backward sweep (beta rows) concurrently with every block's forward
    // sweep; then the short blocks' backward+posterior sweep and the long blocks' combine
    itr::SweepGeometry g = itr::sweep_geometry(m->n, itr::MODE_BWD);
    if (g.iq < 0) return fail(ITR_EINVAL, "n_states=%d unsupported", m->n);
    a.xp = g.xp;
    itr::SweepArgs b = a;
    b.beta = p->d_beta;
    b.beta_off = p->d_boff;
    const int64_t grid = std::min<int64_t>((int64_t)g.per_cu * cu_count(), p->nblocks + nl);
    if (grid <= cu_count()) g.lds = std::max(g.lds, itr::kExclusiveLds);
    HIP_TRY(hipMemsetAsync(a.queue, 0, sizeof(int), st));
    {
      Scope sc("posterior_fwd", st);
      HIP_TRY(itr::launch_post_split(g, (int)grid, a, b, nl, st));
    }
    itr::SweepArgs c = a;
    c.post = post;
    Scope sc("posterior_bwd", st);  // the short blocks' sweep + the long blocks' combine
    if (p->nblocks > nl) {
      c.order = p->d_order + nl;
      c.nblocks = p->nblocks - nl;
      if (int e = run_sweep(itr::MODE_BWD, c, st, "posterior_bwd_short")) return e;
    }
    HIP_TRY(itr::launch_post_combine(m->n, itr::sweep_row_stride(m->n, itr::MODE_BWD), nl,
                                     p->sorted_len[0], p->d_order, p->d_off, p->d_alpha,
                                     p->d_beta, p->d_boff, post, st));
    return 0;
  }
  if (int e = run_sweep(itr::MODE_FWD_STORE, a, st, "posterior_fwd")) return e;
  a.post = post;
  return run_sweep(itr::MODE_BWD, a, st, "posterior_bwd");
}

// ---- host conveniences -----------------------------------------------------------------
int itr_release_streams(void) {
  g_parts.release();
  return 0;
}

int itr_last_kernel_ms(const char* which, double* ms) {
  if (!which || !ms) return fail(ITR_EINVAL, "null pointer");
  for (auto& t : g_timers)
    if (t.name == which && t.armed) {
      HIP_TRY(hipEventSynchronize(t.b));
      float f = 0.f;
      HIP_TRY(hipEventElapsedTime(&f, t.a, t.b));
      *ms = f;
      return 0;
    }
  return fail(ITR_ESTATE, "no timing recorded for '%s'", which);
}

#ifdef ITR_DIAG
// diagnostic build only (not part of the ABI): cycle sums of the last sweep
ITR_API int itr_diag_read(uint64_t* out) {
  if (!g_diag) return fail(ITR_ESTATE, "no diagnostic data");
  HIP_TRY(hipMemcpy(out, g_diag, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return 0;
}
#endif

int itr_expm_batched(int n, int64_t batch, const double* A, double* out, void* stream) {
  if (n < 1 || batch < 0) return fail(ITR_EINVAL, "bad expm shape n=%d batch=%lld", n,
                                      (long long)batch);
  if (batch == 0) return 0;
  if (!A || !out) return fail(ITR_EINVAL, "null device pointer");
  hipStream_t st = (hipStream_t)stream;
  Scope sc("expm", st);
  const hipError_t e = itr::expm_batched(n, batch, A, out, st);
  if (e != hipSuccess) return fail(ITR_EHIP, "expm failed: %s", hipGetErrorString(e));
  return 0;
}

int itr_expm_blocktri_batched(int n_block, int n_blocks, int64_t batch, const double* A,
                              double* out, void* stream) {
  if (n_block < 1 || n_blocks < 1 || batch < 0)
    return fail(ITR_EINVAL, "bad block expm shape n_block=%d n_blocks=%d batch=%lld", n_block,
                n_blocks, (long long)batch);
  if (batch == 0) return 0;
  if (!A || !out) return fail(ITR_EINVAL, "null device pointer");
  hipStream_t st = (hipStream_t)stream;
  Scope sc("expm", st);
  const hipError_t e = itr::expm_blocktri_batched(n_block, n_blocks, batch, A, out, st);
  if (e != hipSuccess) return fail(ITR_EHIP, "block expm failed: %s", hipGetErrorString(e));
  return 0;
}

namespace {
int check_vanloan_paths(int n, const double* h_Q, int n_jobs, const double* h_t, int n_masks,
                        const uint8_t* h_masks, int64_t n_paths, const int32_t* h_path_job,
                        const int64_t* h_path_off, const int32_t* h_path_mask) {
  if (n < 1 || n_jobs < 0 || n_masks < 0 || n_paths < 0)
    return fail(ITR_EINVAL, "bad Van Loan shape n=%d jobs=%d masks=%d paths=%lld", n, n_jobs,
                n_masks, (long long)n_paths);
  if (n_paths == 0) return 0;
  if (!h_Q || !h_t || !h_path_job || !h_path_off || !h_path_mask)
    return fail(ITR_EINVAL, "null pointer");
  if (h_path_off[0] != 0) return fail(ITR_EINVAL, "path offsets must start at 0");
  for (int64_t p = 0; p < n_paths; ++p) {
    const int64_t L = h_path_off[p + 1] - h_path_off[p];
    if (L < 1) return fail(ITR_EINVAL, "path %lld is empty", (long long)p);
    if (h_path_job[p] < 0 || h_path_job[p] >= n_jobs)
      return fail(ITR_EINVAL, "path %lld: interval %d out of range", (long long)p,
                  h_path_job[p]);
    if (L > 1)
      for (int64_t i = h_path_off[p]; i < h_path_off[p + 1]; ++i)
        if (h_path_mask[i] < 0 || h_path_mask[i] >= n_masks)
          return fail(ITR_EINVAL, "path %lld: mask id %d out of range", (long long)p,
                      h_path_mask[i]);
  }
  if (n_masks > 0 && !h_masks) return fail(ITR_EINVAL, "null masks");
  return 0;
}
}  // namespace

int itr_vanloan_paths_ex(int n, const double* h_Q, int n_jobs, const double* h_t, int n_masks,
                         const uint8_t* h_masks, int64_t n_paths, const int32_t* h_path_job,
                         const int64_t* h_path_off, const int32_t* h_path_mask,
                         const double* h_job_norm, double* d_out, void* stream) {
  if (int rc = check_vanloan_paths(n, h_Q, n_jobs, h_t, n_masks, h_masks, n_paths, h_path_job,
                                   h_path_off, h_path_mask))
    return rc;
  if (n_paths == 0) return 0;
  if (!d_out) return fail(ITR_EINVAL, "null pointer");
  hipStream_t st = (hipStream_t)stream;
  Scope sc("vanloan", st);
  const hipError_t e = itr::vanloan_paths(n, h_Q, n_jobs, h_t, n_masks, h_masks, n_paths,
                                          h_path_job, h_path_off, h_path_mask, h_job_norm,
                                          d_out, st);
  if (e != hipSuccess) return fail(ITR_EHIP, "Van Loan evaluation failed: %s",
                                   hipGetErrorString(e));
  return 0;
}

int itr_vanloan_paths(int n, const double* h_Q, int n_jobs, const double* h_t, int n_masks,
                      const uint8_t* h_masks, int64_t n_paths, const int32_t* h_path_job,
                      const int64_t* h_path_off, const int32_t* h_path_mask, double* d_out,
                      void* stream) {
  return itr_vanloan_paths_ex(n, h_Q, n_jobs, h_t, n_masks, h_masks, n_paths, h_path_job,
                              h_path_off, h_path_mask, nullptr, d_out, stream);
}

int itr_vanloan_job_norms(int n, const double* h_Q, int n_jobs, const double* h_t, int n_masks,
                          const uint8_t* h_masks, int64_t n_paths, const int32_t* h_path_job,
                          const int64_t* h_path_off, const int32_t* h_path_mask,
                          double* h_job_norm) {
  if (int rc = check_vanloan_paths(n, h_Q, n_jobs, h_t, n_masks, h_masks, n_paths, h_path_job,
                                   h_path_off, h_path_mask))
    return rc;
  if (n_jobs > 0 && !h_job_norm) return fail(ITR_EINVAL, "null pointer");
  if (n_paths == 0) {
    for (int j = 0; j < n_jobs; ++j) h_job_norm[j] = 0.0;
    return 0;
  }
  itr::vanloan_job_norms(n, h_Q, n_jobs, h_t, n_masks, h_masks, n_paths, h_path_job,
                         h_path_off, h_path_mask, h_job_norm);
  return 0;
}

int itr_expm_batched_host(int n, int64_t batch, const double* h_A, double* h_out) {
  if (n < 1 || batch < 0) return fail(ITR_EINVAL, "bad expm shape");
  if (batch == 0) return 0;
  if (!h_A || !h_out) return fail(ITR_EINVAL, "null host pointer");
  const size_t bytes = (size_t)batch * n * n * sizeof(double);
  DevBuf a, o;
  HIP_TRY(hipMalloc(&a.p, bytes));
  HIP_TRY(hipMalloc(&o.p, bytes));
  HIP_TRY(hipMemcpy(a.p, h_A, bytes, hipMemcpyHostToDevice));
  if (int e = itr_expm_batched(n, batch, (const double*)a.p, (double*)o.p, nullptr)) return e;
  HIP_TRY(hipMemcpy(h_out, o.p, bytes, hipMemcpyDeviceToHost));
  return 0;
}

int itr_inverse_batched(int n, int64_t batch, const double* M, double* out, void* stream) {
  if (n < 1 || batch < 0)
    return fail(ITR_EINVAL, "bad inverse shape n=%d batch=%lld", n, (long long)batch);
  if (batch == 0) return 0;
  if (!M || !out) return fail(ITR_EINVAL, "null device pointer");
  if (M == out) return fail(ITR_EINVAL, "the inverse is not computed in place");
  hipStream_t st = (hipStream_t)stream;
  int* piv = nullptr;
  double* work = nullptr;
  HIP_TRY(hipMallocAsync((void**)&piv, (size_t)batch * n * sizeof(int), st));
  if (n > itr::kInverseRegMax &&
      hipMallocAsync((void**)&work, (size_t)batch * n * n * sizeof(double), st) != hipSuccess) {
    (void)hipFreeAsync(piv, st);
    return fail(ITR_EHIP, "inverse workspace allocation failed");
  }
  Scope sc("inverse", st);
  const hipError_t e = itr::inverse_batched(n, batch, M, out, piv, work, st);
  (void)hipFreeAsync(piv, st);
  if (work) (void)hipFreeAsync(work, st);
  if (e != hipSuccess) return fail(ITR_EHIP, "inverse failed: %s", hipGetErrorString(e));
  return 0;
}

int itr_solve_batched(int n, int nrhs, int64_t batch, double* M, double* R, void* stream) {
  if (n < 1 || nrhs < 1 || batch < 0)
    return fail(ITR_EINVAL, "bad solve shape n=%d nrhs=%d batch=%lld", n, nrhs,
                (long long)batch);
  if (batch == 0) return 0;
  if (!M || !R) return fail(ITR_EINVAL, "null device pointer");
  hipStream_t st = (hipStream_t)stream;
  int* piv = nullptr;
  HIP_TRY(hipMallocAsync((void**)&piv, (size_t)batch * n * sizeof(int), st));
  Scope sc("solve", st);
  const hipError_t e = itr::solve_batched(n, nrhs, batch, M, R, piv, st);
  (void)hipFreeAsync(piv, st);
  if (e != hipSuccess) return fail(ITR_EHIP, "solve failed: %s", hipGetErrorString(e));
  return 0;
}

int itr_chain_rows(int k, int ng, int rmax, const int32_t* src, const int32_t* oms,
                   const int32_t* ome, const int32_t* dst, const int32_t* cols, const double* P,
                   int64_t ldp, const double* F, int64_t ldf, const double* M, double* out,
                   int64_t ldo, void* stream) {
  if (k < 1 || ng < 0 || rmax < 0 || ng > 65535)
    return fail(ITR_EINVAL, "bad chain-rows shape k=%d groups=%d rmax=%d", k, ng, rmax);
  if (ng == 0 || rmax == 0) return 0;
  if (!src || !dst || !P || !M || !out || ((oms || ome) && !F))
    return fail(ITR_EINVAL, "null device pointer");
  itr::ChainRowsArgs a{k, rmax, src, oms, ome, dst, cols, P, ldp, F, ldf, M, out, ldo};
  const hipError_t e = itr::chain_rows(a, ng, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ITR_EHIP, "chain rows failed: %s", hipGetErrorString(e));
  return 0;
}

int itr_group_sum(int64_t nn, int ng, const int32_t* off, const int32_t* paths, const double* S,
                  double* M, void* stream) {
  if (nn < 1 || ng < 0 || ng > 65535)
    return fail(ITR_EINVAL, "bad group-sum shape nn=%lld groups=%d", (long long)nn, ng);
  if (ng == 0) return 0;
  if (!off || !M) return fail(ITR_EINVAL, "null device pointer");
  const hipError_t e = itr::group_sum(nn, ng, off, paths, S, M, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ITR_EHIP, "group sum failed: %s", hipGetErrorString(e));
  return 0;
}

int itr_gemm_batched(int m, int n, int k, int64_t batch, double alpha, const double* A,
                     const double* B, double beta, double* C, void* stream) {
  if (m < 1 || n < 1 || k < 1 || batch < 0)
    return fail(ITR_EINVAL, "bad gemm shape %dx%dx%d batch=%lld", m, n, k, (long long)batch);
  if (batch == 0) return 0;
  if (!A || !B || !C) return fail(ITR_EINVAL, "null device pointer");
  itr::GemmArgs g{};
  g.m = m;
  g.n = n;
  g.k = k;
  g.A = itr::Mat{(double*)A, (int64_t)m * k, k};
  g.B = itr::Mat{(double*)B, (int64_t)k * n, n};
  g.C = itr::Mat{C, (int64_t)m * n, n};
  g.D = beta != 0.0 ? g.C : itr::Mat{nullptr, 0, 0};
  g.alpha = alpha;
  g.beta = beta;
  g.gamma = 0.0;
  g.idx = nullptr;
  const hipError_t e = itr::gemm_batched(g, batch, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ITR_EHIP, "gemm failed: %s", hipGetErrorString(e));
  return 0;
}

int itr_emission_rows(int n_states, const double* tables, double* out, void* stream) {
  if (n_states < 0) return fail(ITR_EINVAL, "bad state count %d", n_states);
  if (n_states == 0) return 0;
  if (!tables || !out) return fail(ITR_EINVAL, "null device pointer");
  const hipError_t e = itr::launch_emission(n_states, tables, out, (hipStream_t)stream);
  if (e != hipSuccess) return fail(ITR_EHIP, "emission launch failed: %s", hipGetErrorString(e));
  return 0;
}

}  // extern "C"
