// host_io.cpp — the C ABI's host-buffer entry points: the drop-in calls on the reference's
// own V_lst blocks (packed by host threads into pinned memory), the synchronous host-buffer
// conveniences with the chunked copy-out of large results, MAF ingest and the result
// writers.  Host code only; the sweeps themselves are capi.cpp's entry points.
#include "capi_internal.h"

using namespace itr_host;

namespace {

// Device -> pageable host copy of a large result (the posterior rows: 10.6 GB per 10 Mbp at
// N = 133).  A plain hipMemcpy stages through the runtime's pinned buffers and writes (and
// page-faults) the destination from one thread; here chunks go to two pinned staging buffers
// on their own stream while host threads copy the previous chunk out, so the PCIe transfer
// overlaps the faulting copies and those run on several cores.
constexpr size_t kStageBytes = size_t(128) << 20;
// The calling thread's staging buffers, stream and events; they belong to one device and
// are recreated when the thread's current device changes.  itr_release_staging() frees them.
struct Staging {
  int device = -1;
  void* stage[2] = {nullptr, nullptr};
  hipStream_t cs = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  void release() {
    for (int i = 0; i < 2; ++i) {
      if (stage[i]) (void)hipHostFree(stage[i]);
      if (ev[i]) (void)hipEventDestroy(ev[i]);
      stage[i] = nullptr;
      ev[i] = nullptr;
    }
    if (cs) (void)hipStreamDestroy(cs);
    cs = nullptr;
    device = -1;
  }
};
// (freed with the thread, or by itr_release_staging)
struct StagingSlot : Staging {
  ~StagingSlot() { release(); }
};
thread_local StagingSlot g_stage;

// The calling thread's pinned host buffer and device buffer of the host-block entry points
// (grow-only, per device): no allocation, no pageable copy per call.
struct HostIO {
  int device = -1;
  void* pin = nullptr;
  size_t pin_cap = 0;
  void* dbuf = nullptr;
  size_t dcap = 0;
  hipStream_t st = nullptr;  // the calls' own non-blocking stream (no legacy-stream syncs)
  hipEvent_t legacy = nullptr;  // recorded on the null stream: st waits for its earlier work
  ~HostIO() { release(); }      // (a thread's buffers and stream go with the thread)
  void release() {
    if (st) (void)hipStreamSynchronize(st);
    if (pin) (void)hipHostFree(pin);
    if (dbuf) (void)hipFree(dbuf);
    if (st) (void)hipStreamDestroy(st);
    if (legacy) (void)hipEventDestroy(legacy);
    pin = dbuf = nullptr;
    st = nullptr;
    legacy = nullptr;
    pin_cap = dcap = 0;
    device = -1;
  }
  int reserve(size_t pin_bytes, size_t dev_bytes) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    if (dev != device) {
      release();
      device = dev;
    }
    if (!st) HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    if (!legacy) HIP_TRY(hipEventCreateWithFlags(&legacy, hipEventDisableTiming));
    if (pin_bytes > pin_cap) {
      if (pin) (void)hipHostFree(pin);
      pin = nullptr;
      pin_cap = 0;
      HIP_TRY(hipHostMalloc(&pin, pin_bytes, hipHostMallocDefault));
      pin_cap = pin_bytes;
    }
    if (dev_bytes > dcap) {
      if (dbuf) (void)hipFree(dbuf);
      dbuf = nullptr;
      dcap = 0;
      HIP_TRY(hipMalloc(&dbuf, dev_bytes));
      dcap = dev_bytes;
    }
    return 0;
  }
};
thread_local HostIO g_hio;

int copy_out_large(void* dst, const void* src, size_t bytes) {
  if (bytes < 2 * kStageBytes) {
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
  }
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  Staging& sg = g_stage;
  if (sg.device != dev) {
    sg.release();
    HIP_TRY(hipStreamCreateWithFlags(&sg.cs, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
      HIP_TRY(hipHostMalloc(&sg.stage[i], kStageBytes, hipHostMallocDefault));
      HIP_TRY(hipEventCreateWithFlags(&sg.ev[i], hipEventDisableTiming));
    }
    sg.device = dev;
  }
  void* const* stage = sg.stage;
  hipStream_t cs = sg.cs;
  hipEvent_t* ev = sg.ev;
  HIP_TRY(hipStreamSynchronize(nullptr));  // the sweep ran on the null stream
  const size_t nch = (bytes + kStageBytes - 1) / kStageBytes;
  auto issue = [&](size_t c) -> int {
    const size_t off = c * kStageBytes, len = std::min(kStageBytes, bytes - off);
    HIP_TRY(hipMemcpyAsync(stage[c & 1], (const char*)src + off, len, hipMemcpyDeviceToHost,
                           cs));
    HIP_TRY(hipEventRecord(ev[c & 1], cs));
    return 0;
  };
  if (int e = issue(0)) return e;
  const int nt = 8;
  for (size_t c = 0; c < nch; ++c) {
    HIP_TRY(hipEventSynchronize(ev[c & 1]));
    if (c + 1 < nch)
      if (int e = issue(c + 1)) return e;
    const size_t off = c * kStageBytes, len = std::min(kStageBytes, bytes - off);
    const char* s = (const char*)stage[c & 1];
    char* d = (char*)dst + off;
    std::vector<std::thread> th;
    for (int w = 1; w < nt; ++w)
      th.emplace_back([=] { memcpy(d + len * w / nt, s + len * w / nt,
                                   len * (w + 1) / nt - len * w / nt); });
    memcpy(d, s, len / nt);
    for (auto& t : th) t.join();
  }
  return 0;
}
}  // namespace

extern "C" {

int itr_forward_loglik_host(itr_model_t m, itr_plan_t p, const uint16_t* h_obs,
                            double* h_ll) {
  if (int e = check_plan(p)) return e;
  if (p->nblocks == 0) return 0;
  if ((!h_obs && p->total) || !h_ll) return fail(ITR_EINVAL, "null host pointer");
  DevBuf o, l;
  HIP_TRY(hipMalloc(&o.p, std::max<int64_t>(p->total, 1) * sizeof(uint16_t)));
  HIP_TRY(hipMalloc(&l.p, p->nblocks * sizeof(double)));
  if (p->total)
    HIP_TRY(hipMemcpy(o.p, h_obs, p->total * sizeof(uint16_t), hipMemcpyHostToDevice));
  if (int e = itr_forward_loglik(m, p, (const uint16_t*)o.p, (double*)l.p, nullptr)) return e;
  HIP_TRY(hipMemcpy(h_ll, l.p, p->nblocks * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int itr_viterbi_host(itr_model_t m, itr_plan_t p, const uint16_t* h_obs, uint8_t* h_path) {
  if (int e = check_plan(p)) return e;
  if (p->total == 0) return 0;
  if (!h_obs || !h_path) return fail(ITR_EINVAL, "null host pointer");
  DevBuf o, y;
  HIP_TRY(hipMalloc(&o.p, p->total * sizeof(uint16_t)));
  HIP_TRY(hipMalloc(&y.p, p->total));
  HIP_TRY(hipMemcpy(o.p, h_obs, p->total * sizeof(uint16_t), hipMemcpyHostToDevice));
  if (int e = itr_viterbi(m, p, (const uint16_t*)o.p, (uint8_t*)y.p, nullptr)) return e;
  HIP_TRY(hipMemcpy(h_path, y.p, p->total, hipMemcpyDeviceToHost));
  return 0;
}

int itr_posterior_host(itr_model_t m, itr_plan_t p, const uint16_t* h_obs, double* h_post) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->total == 0) return 0;
  if (!h_obs || !h_post) return fail(ITR_EINVAL, "null host pointer");
  DevBuf o, y;
  const size_t bytes = (size_t)p->total * m->n * sizeof(double);
  HIP_TRY(hipMalloc(&o.p, p->total * sizeof(uint16_t)));
  HIP_TRY(hipMalloc(&y.p, bytes));
  HIP_TRY(hipMemcpy(o.p, h_obs, p->total * sizeof(uint16_t), hipMemcpyHostToDevice));
  if (int e = itr_posterior(m, p, (const uint16_t*)o.p, (double*)y.p, nullptr)) return e;
  return copy_out_large(h_post, y.p, bytes);
}

int itr_release_staging(void) {
  g_stage.release();
  g_hio.release();
  itr::release_vanloan_workspace();
  return 0;
}

struct itr_maf {
  itr::MafResult r;
};

int itr_maf_open(const char* path, const char* const* species, const char* ref,
                 itr_maf_t* out) {
  if (!out) return fail(ITR_EINVAL, "null output pointer");
  *out = nullptr;
  if (!path || !species) return fail(ITR_EINVAL, "null path or species list");
  for (int k = 0; k < 4; ++k)
    if (!species[k]) return fail(ITR_EINVAL, "species list needs 4 names");
  auto* h = new itr_maf();
  std::string err;
  const int rc = itr::maf_read(path, species, ref, &h->r, &err);
  if (rc) {
    delete h;
    return fail(rc == 2 ? ITR_EDATA : ITR_EINVAL, "%s", err.c_str());
  }
  *out = h;
  return 0;
}

int itr_maf_sizes(itr_maf_t h, int64_t* n_blocks, int64_t* n_columns, int64_t* n_coord_blocks,
                  int64_t* n_coords) {
  if (!h) return fail(ITR_EINVAL, "null MAF handle");
  if (n_blocks) *n_blocks = (int64_t)h->r.off.size() - 1;
  if (n_columns) *n_columns = (int64_t)h->r.obs.size();
  if (n_coord_blocks) *n_coord_blocks = (int64_t)h->r.coord_off.size() - 1;
  if (n_coords) *n_coords = (int64_t)h->r.coords.size();
  return 0;
}

int itr_maf_copy(itr_maf_t h, uint16_t* obs, int64_t* block_off, int64_t* coords,
                 int64_t* coord_off) {
  if (!h) return fail(ITR_EINVAL, "null MAF handle");
  const auto& r = h->r;
  if (obs && !r.obs.empty()) memcpy(obs, r.obs.data(), r.obs.size() * sizeof(uint16_t));
  if (block_off) memcpy(block_off, r.off.data(), r.off.size() * sizeof(int64_t));
  if (coords && !r.coords.empty()) memcpy(coords, r.coords.data(), r.coords.size() * sizeof(int64_t));
  if (coord_off) memcpy(coord_off, r.coord_off.data(), r.coord_off.size() * sizeof(int64_t));
  return 0;
}

int itr_maf_close(itr_maf_t h) {
  delete h;
  return 0;
}

// V_lst -> (uint16 columns, int64 offsets): the blocks are split into contiguous ranges of
// about equal column count, one per thread; each thread converts and range-checks its own
// blocks, and the first bad symbol (lowest block) is reported.
namespace {
// V_lst -> uint16 columns at the given offsets: the blocks are split into contiguous ranges
// of about equal column count, one per thread; each thread converts and range-checks its
// own blocks, and the first bad symbol (lowest block) is reported.
// Blocks [0, n_blocks) of the given arrays (block_off absolute: obs + block_off[k] is block
// k's first column; k_base = the first block's index in messages).
int pack_blocks(const int64_t* const* blocks, const int64_t* lens, const int64_t* block_off,
                int64_t n_blocks, uint16_t* obs, int64_t k_base = 0) {
  const int64_t c_begin = block_off[0], total = block_off[n_blocks] - c_begin;
  if (total == 0) return 0;
  const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, total >> 18));
  std::vector<int64_t> bad(nt, -1), bad_col(nt, -1);
  parallel_for(nt, [&](int w) {
    const int64_t lo_col = c_begin + total * w / nt, hi_col = c_begin + total * (w + 1) / nt;
    // blocks whose first column falls in [lo_col, hi_col)
    int64_t k = std::lower_bound(block_off, block_off + n_blocks, lo_col) - block_off;
    for (; k < n_blocks && block_off[k] < hi_col; ++k) {
      const int64_t* src = blocks[k];
      uint16_t* dst = obs + block_off[k];
      const int64_t len = lens[k];
      int64_t ok = 1;
      for (int64_t t = 0; t < len; ++t) {
        const int64_t v = src[t];
        ok &= (uint64_t)v < (uint64_t)ITR_NOBS;
        dst[t] = (uint16_t)v;
      }
      if (!ok) {
        int64_t t = 0;
        while ((uint64_t)src[t] < (uint64_t)ITR_NOBS) ++t;
        bad[w] = k;
        bad_col[w] = t;
        return;
      }
    }
  });
  for (int w = 0; w < nt; ++w)
    if (bad[w] >= 0)
      return fail(ITR_EDATA, "observed symbol %lld (block %lld, column %lld) outside the "
                  "625-letter alphabet", (long long)blocks[bad[w]][bad_col[w]],
                  (long long)(k_base + bad[w]), (long long)bad_col[w]);
  return 0;
}


// the blocks of a host-block call against the plan's layout; packed into pinned memory and
// copied to the device buffer on the thread's own stream g_hio.st, which first waits for the
// work the caller queued on the null stream (a sweep of the same plan on stream 0 finishes
// before this call's sweep touches the plan's workspace)
int upload_blocks(itr_plan_t p, const int64_t* const* blocks, const int64_t* lens,
                  int64_t n_blocks, size_t extra_dev, uint16_t** d_obs) {
  if (n_blocks != p->nblocks)
    return fail(ITR_EINVAL, "%lld blocks for a plan of %lld", (long long)n_blocks,
                (long long)p->nblocks);
  if (n_blocks > 0 && !lens) return fail(ITR_EINVAL, "null lengths");
  for (int64_t k = 0; k < n_blocks; ++k) {
    if (lens[k] != p->h_off[k + 1] - p->h_off[k])
      return fail(ITR_EINVAL, "block %lld has %lld columns, the plan %lld", (long long)k,
                  (long long)lens[k], (long long)(p->h_off[k + 1] - p->h_off[k]));
    if (lens[k] > 0 && !blocks[k]) return fail(ITR_EINVAL, "block %lld is null", (long long)k);
  }
  const size_t ob = (size_t)std::max<int64_t>(p->total, 1) * sizeof(uint16_t);
  const size_t ob16 = (ob + 255) & ~(size_t)255;
  if (int e = g_hio.reserve(std::max(ob, (size_t)p->total), ob16 + extra_dev)) return e;
  uint16_t* h = (uint16_t*)g_hio.pin;
  *d_obs = (uint16_t*)g_hio.dbuf;
  HIP_TRY(hipEventRecord(g_hio.legacy, nullptr));
  HIP_TRY(hipStreamWaitEvent(g_hio.st, g_hio.legacy, 0));
  // two halves (by blocks): the first half's copy runs while the second is packed
  const int64_t kh = std::lower_bound(p->h_off.begin(), p->h_off.end() - 1, p->total / 2) -
                     p->h_off.begin();
  const int64_t cuts[3] = {0, std::min<int64_t>(kh, n_blocks), n_blocks};
  for (int part = 0; part < 2; ++part) {
    const int64_t k0 = cuts[part], k1 = cuts[part + 1];
    if (k1 <= k0) continue;
    if (int e = pack_blocks(blocks + k0, lens + k0, p->h_off.data() + k0, k1 - k0, h, k0)) {
      (void)hipStreamSynchronize(g_hio.st);  // (the first half's copy still reads the buffer)
      return e;
    }
    const int64_t c0 = p->h_off[k0], c1 = p->h_off[k1];
    if (c1 > c0)
      HIP_TRY(hipMemcpyAsync(*d_obs + c0, h + c0, (c1 - c0) * sizeof(uint16_t),
                             hipMemcpyHostToDevice, g_hio.st));
  }
  return 0;
}
size_t dev_tail(itr_plan_t p) {  // first byte after the observations in g_hio.dbuf
  const size_t ob = (size_t)std::max<int64_t>(p->total, 1) * sizeof(uint16_t);
  return (ob + 255) & ~(size_t)255;
}
}  // namespace

int itr_pack_symbols(const int64_t* const* blocks, const int64_t* lens, int64_t n_blocks,
                     uint16_t* obs, int64_t* block_off) {
  if (n_blocks < 0 || !block_off || (n_blocks > 0 && !lens))
    return fail(ITR_EINVAL, "bad pack arguments");
  block_off[0] = 0;
  for (int64_t k = 0; k < n_blocks; ++k) {
    if (lens[k] < 0) return fail(ITR_EINVAL, "block %lld has negative length", (long long)k);
    if (lens[k] > 0 && !blocks[k]) return fail(ITR_EINVAL, "block %lld is null", (long long)k);
    block_off[k + 1] = block_off[k] + lens[k];
  }
  if (block_off[n_blocks] == 0) return 0;
  if (!obs) return fail(ITR_EINVAL, "null output");
  return pack_blocks(blocks, lens, block_off, n_blocks, obs);
}

namespace {
// ITR_HOST_TIMING=1: stage times of the host-block entry points on stderr (diagnostics)
struct HostClock {
  bool on = getenv("ITR_HOST_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(const char* what) {
    if (!on) return;
    (void)hipDeviceSynchronize();
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "%s %.3f ms  ", what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
  void end() {
    if (on) fprintf(stderr, "\n");
  }
};
}  // namespace

int itr_forward_loglik_blocks(itr_model_t m, itr_plan_t p, const int64_t* const* blocks,
                              const int64_t* lens, int64_t n_blocks, double* h_ll) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->nblocks > 0 && !h_ll) return fail(ITR_EINVAL, "null output");
  uint16_t* d_obs = nullptr;
  const size_t tail = dev_tail(p);
  HostClock clk;
  if (int e = upload_blocks(p, blocks, lens, n_blocks, (size_t)p->nblocks * 8 + 8, &d_obs))
    return e;
  clk.lap("loglik: pack+h2d");
  if (p->nblocks == 0) return 0;
  double* d_ll = (double*)((char*)g_hio.dbuf + tail);
  if (int e = itr_forward_loglik(m, p, d_obs, d_ll, g_hio.st)) return e;
  clk.lap("sweep");
  HIP_TRY(hipMemcpyAsync(h_ll, d_ll, p->nblocks * sizeof(double), hipMemcpyDeviceToHost,
                         g_hio.st));
  HIP_TRY(hipStreamSynchronize(g_hio.st));
  clk.lap("d2h");
  clk.end();
  return 0;
}

int itr_viterbi_blocks(itr_model_t m, itr_plan_t p, const int64_t* const* blocks,
                       const int64_t* lens, int64_t n_blocks, double* h_path) {
  if (int e = check_model(m)) return e;
  if (int e = check_plan(p)) return e;
  if (p->total > 0 && !h_path) return fail(ITR_EINVAL, "null output");
  uint16_t* d_obs = nullptr;
  const size_t tail = dev_tail(p);
  HostClock clk;
  if (int e = upload_blocks(p, blocks, lens, n_blocks, (size_t)p->total + 8, &d_obs)) return e;
  clk.lap("viterbi: pack+h2d");
  if (p->total == 0) return 0;
  uint8_t* d_path = (uint8_t*)g_hio.dbuf + tail;
  if (int e = itr_viterbi(m, p, d_obs, d_path, g_hio.st)) return e;
  const int64_t total = p->total;
  const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, total >> 18));
  // while the device sweeps: host threads map the output's pages (one write per 4 KiB), so
  // the widening below does not page-fault its way through a fresh 8-bytes-per-column array
  if (!clk.on)
    parallel_for(nt, [&](int w) {
      const int64_t lo = total * w / nt, hi = total * (w + 1) / nt;
      for (int64_t c = lo; c < hi; c += 512) h_path[c] = 0.0;
    });
  clk.lap("sweep");
  // the states back through the pinned buffer (the observations' upload finished before the
  // sweep on this stream), widened to float64 (the reference's path dtype) by host threads
  uint8_t* h = (uint8_t*)g_hio.pin;
  HIP_TRY(hipMemcpyAsync(h, d_path, p->total, hipMemcpyDeviceToHost, g_hio.st));
  HIP_TRY(hipStreamSynchronize(g_hio.st));
  clk.lap("d2h");
  parallel_for(nt, [&](int w) {
    const int64_t lo = total * w / nt, hi = total * (w + 1) / nt;
    for (int64_t c = lo; c < hi; ++c) h_path[c] = (double)h[c];
  });
  clk.lap("to_f64");
  clk.end();
  return 0;
}

int itr_format_float(double x, char* out, int cap) {
  char b[40];
  const int n = itr::format_pyfloat(x, b);
  if (!out || cap < n + 1) return fail(ITR_EINVAL, "buffer too small");
  memcpy(out, b, n);
  out[n] = 0;
  return 0;
}

namespace {
// per-column reference coordinates must cover exactly the decoded columns: the writers read
// coords[c] for every column c
int check_coords(const int64_t* block_off, int64_t n_blocks, const int64_t* coords,
                 int64_t n_coords) {
  if (!coords) return 0;
  const int64_t total = n_blocks > 0 ? block_off[n_blocks] : 0;
  if (n_coords != total)
    return fail(ITR_EINVAL, "%lld reference coordinates for %lld decoded columns",
                (long long)n_coords, (long long)total);
  return 0;
}
}  // namespace

int itr_write_viterbi_csv(const char* path, const uint8_t* states, const int64_t* block_off,
                          int64_t n_blocks, const int64_t* coords, int64_t n_coords) {
  if (!path || (n_blocks > 0 && (!states || !block_off)) || n_blocks < 0)
    return fail(ITR_EINVAL, "bad arguments");
  if (int e = check_coords(block_off, n_blocks, coords, n_coords)) return e;
  std::string err;
  if (itr::write_viterbi_csv(path, states, block_off, n_blocks, coords, &err))
    return fail(ITR_EINVAL, "%s", err.c_str());
  return 0;
}

int itr_write_posterior_csv(const char* path, const double* post, int n_states,
                            const int64_t* block_off, int64_t n_blocks, const int64_t* coords,
                            int64_t n_coords, int threads) {
  if (!path || n_states < 0 || n_blocks < 0 || (n_blocks > 0 && (!post || !block_off)))
    return fail(ITR_EINVAL, "bad arguments");
  if (int e = check_coords(block_off, n_blocks, coords, n_coords)) return e;
  std::string err;
  if (itr::write_posterior_csv(path, post, n_states, block_off, n_blocks, coords, threads, &err))
    return fail(ITR_EINVAL, "%s", err.c_str());
  return 0;
}

}  // extern "C"
