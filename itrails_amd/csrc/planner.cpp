// planner.cpp — plan creation (itr_plan_create*): the processing order, the forward
// log-likelihood task lists (split blocks, VALU tasks, matrix-core groups), the mixed
// forward + Viterbi queue and the CU partition of the decoding calls, with the per-column
// cost constants they are derived from.  Host code only; the plan's device tables are
// uploaded once here.
#include "capi_internal.h"

using namespace itr_host;

namespace {

// Per-column costs of the sweep layouts of the (5,5) model (N = 65..72, the only state counts
// with the per-wave layouts), measured on MI355X (profiles/r3l_*, r3u_*):
//   kVitLone    a Viterbi block alone on its CU, 9-wave VALU layout           325 ns / column
//   kVitWaveLat a per-wave Viterbi block's step under full load (latency)      800 ns / column
//   kBulkCu     forward + Viterbi of a column in the mixed per-wave launch     180 CU-ns / column
//               (calibrated on chr10: 0.15 / 0.165 / 0.18 / 0.195 us -> forward+Viterbi call
//               8.52 / 8.49 / 8.29-8.69 / 8.41-8.56 ms, profiles/r3ab5_partition.txt)
//   kFwdValu    a forward VALU half alone on its CU                            370 ns / column
//   kBulkVit    Viterbi alone of a column in the per-wave launch               115 CU-ns / column
//               (10 M columns of short blocks in 4.43 ms on 256 CUs)
//   kVitWaveLatV  a per-wave Viterbi block's step in that launch under full    700 ns / column
//               load (two waves per SIMD: ~640 ns alone), calibrated on the chr10 Viterbi-only
//               call with 0 / 30 / 59 / 80 / 100 / 124 long blocks: 12.1 / 6.42 / 5.76 / 5.80 /
//               6.02 / 7.97 ms (profiles/r4m_vit_long_set.txt; this rule picks 69)
//   kMixFwd / kMixVit  the mixed queue's ordering weights: per-column step times under full
//               load at N = 70 of a matrix-core forward group (~0.92 us) and a per-wave Viterbi
//               block (~0.64 us), measured on chr10 (profiles/r3l_*)
//   kMixPrio    mixed-queue entries that run at raised wave priority: about one per SIMD pair
//   kVitPairEff the effective step of a 9-wave Viterbi block that shares its reserved CU with a
//               second long block for part of its sweep (alone 318 ns, with a partner for the
//               whole sweep 407 ns, three per CU 613 ns; profiles/r4pp_pair_long_blocks.txt);
//   kPairShare  two long blocks per reserved CU only when the one-per-CU long set would hold
//               more than this share of the chip: chr10 (35 CUs) 7.62-7.70 -> 7.44-7.48 ms
//               per step with the long set on 24 CUs (same box, interleaved); the chr100
//               shards (12-16 CUs) keep one per CU: paired with bins sized by 360 ns, one
//               shard went 8.5 -> 9.5 ms (profiles/r4pab_pair_ab.txt)
//   kPruneCol   a per-wave Viterbi block takes the bound-pruned step (fewer instructions per
//               column, a longer dependent chain: wave_tasks.h) when its length x kPruneCol
//               fits within the expected makespan, the full scan otherwise; chr10
//               forward+Viterbi with 1.0 / 1.4 / 2.0 / 2.9 / 4.0 / 6.0 us and all blocks on the
//               full scan: 7.95-7.99 / 7.64-7.65 / 7.67-7.73 / 7.82 / 7.85 / 7.94 / 8.12 ms per
//               step; chr100 (every block pruned) 59.4 -> 51.6 ms, its world-8 shards 8.96 ->
//               8.61 ms; the Viterbi-only call stays at its long set's floor (6.1 ms)
//               (profiles/r4pc_prune_col.txt)
//   kMixGroupCol  the per-column step a forward half may take in a matrix-core group and
//               still finish within the expected makespan (sets the floor of the VALU-task
//               threshold): chr100 world-8 shards with 0.7 / 1.0 / 1.4 us -> slowest shard
//               14.05 / 12.17 / 10.31 ms vs 10.75 ms with the fraction rule alone
//               (profiles/r4w_shard_threshold.txt)
// Calibrated at N = 70 only; tests/test_partition.py pins the decisions they produce for the
// benchmark layouts, so that a recalibration cannot move a layout onto another branch unseen.
constexpr double kVitLone = 325e-9, kVitWaveLat = 800e-9, kBulkCu = 180e-9, kFwdValu = 370e-9,
                 kBulkVit = 115e-9, kVitWaveLatV = 700e-9, kMixFwd = 0.92, kMixVit = 0.64,
                 kMixGroupCol = 1.4e-6, kPruneCol = 1.4e-6, kVitPairEff = 360e-9,
                 kPairShare = 1.0 / 8, kFwdPairStep = 480e-9;
constexpr int kFwdPairMin = 16;
constexpr int64_t kMixPrio = 512;

// Bins of capacity `cap` (first fit, items longest first): the CUs a set of sequential tasks
// needs to finish within cap
int ffd_bins(const std::vector<int64_t>& items, double cap) {
  std::vector<double> bins;
  for (int64_t t : items) {
    bool placed = false;
    for (double& b : bins)
      if (b + (double)t <= cap) {
        b += (double)t;
        placed = true;
        break;
      }
    if (!placed) bins.push_back((double)t);
  }
  return (int)bins.size();
}

// The forward+Viterbi CU partition of a plan (viterbi_impl).  Expected makespan T: the whole
// workload at the bulk layouts' throughput over every CU, or the longest block alone on the
// 9-wave layout, whichever is longer.  A block whose per-wave Viterbi step latency would
// exceed T joins the long set; the long set gets the CUs it needs to finish within T at the
// lone-block step time, the forward's VALU halves (`ulen`) the CUs they need at theirs,
// rounded up to whole XCC sets (8 CUs: one per XCC).  The reserved CUs join the bulk queue
// when their long work is done, so a generous reservation costs little.
void plan_partition(itr_plan_t p, const std::vector<int64_t>& ulen, int cus) {
  const int64_t nblocks = p->nblocks;
  const double tmax = nblocks ? (double)p->sorted_len[0] : 0.0;
  const double wlat = kVitWaveLat, bulk = kBulkCu;
  const double T = std::max((double)p->total * bulk / cus, tmax * kVitLone);
  int64_t k = 0, cols = 0;
  std::vector<int64_t> lng;
  while (k < nblocks && p->sorted_len[k] >= 2048 && (double)p->sorted_len[k] * wlat > T) {
    lng.push_back(p->sorted_len[k]);
    cols += p->sorted_len[k++];
  }
  p->vit_nlong = k;
  p->vit_long_cols = cols;
  // Long blocks a reserved CU sweeps at a time: two (bins sized by the shared step
  // kVitPairEff) when the one-per-CU long set would hold more than kPairShare of the chip
  // and its longest block still fits the makespan at the shared step — the freed CUs go to
  // the bulk; otherwise one.
  double step = kVitLone;
  const double pstep = kVitPairEff;
  int lpc = 1;
  if (ffd_bins(lng, T / kVitLone) > kPairShare * cus && tmax * pstep <= T) {
    lpc = 2;
    step = pstep;
  }
  p->long_per_cu = lpc;
  const int rv = (ffd_bins(lng, T / step) + lpc - 1) / lpc;
  std::vector<int64_t> halves(ulen);
  std::sort(halves.begin(), halves.end(), std::greater<int64_t>());
  int rf = ffd_bins(halves, T / kFwdValu);
  // two forward halves per reserved CU at a time when the one-per-CU set is large (more
  // than kFwdPairMin CUs), bins sized by the shared step kFwdPairStep
  int fpc = 1;
  const double fstep = kFwdPairStep;
  const int fmin = kFwdPairMin;
  if (rf > fmin) {
    const int rf2 = (ffd_bins(halves, T / fstep) + 1) / 2;
    if (rf2 < rf) {
      rf = rf2;
      fpc = 2;
    }
  }
  p->fwd_per_cu = fpc;
  p->fwd_reserve = rf;  // (viterbi_impl rounds both up to whole XCC sets)
  p->vit_reserve = rv;
  p->wave_ok = rv + rf <= cus / 2;
  // the Viterbi-only call (itr_viterbi) on the same two reserved sets: its own makespan (the
  // per-wave Viterbi's bulk cost, no forward) decides its long set, which both reserved sets
  // sweep before they join the bulk
  const double Tv = std::max((double)p->total * kBulkVit / cus, tmax * kVitLone);
  int64_t kv = 0;
  while (kv < nblocks && p->sorted_len[kv] >= 2048 && (double)p->sorted_len[kv] * kVitWaveLatV > Tv)
    ++kv;
  p->vit_nlong_v = kv;
  // the per-wave Viterbi's step per block: bound-pruned below these lengths (kPruneCol)
  const double pcol = kPruneCol;
  p->vit_prune_len = (int)std::min(T / pcol, (double)INT32_MAX);
  p->vit_prune_len_v = (int)std::min(Tv / pcol, (double)INT32_MAX);
  if (getenv("ITR_VERBOSE"))
    fprintf(stderr, "[itr] partition: T %.3f ms, long %lld blocks (%lld cols), rv %d rf %d (%zu halves)%s, "
            "pruned below %d / %d columns\n",
            T * 1e3, (long long)k, (long long)cols, p->vit_reserve, rf, halves.size(),
            p->wave_ok ? "" : ", no wave layout", p->vit_prune_len, p->vit_prune_len_v);
}

// The posterior's concurrent split (launch_post_split): only on the VALU-only posterior
// (no matrix-core form at this state count) and only where the blocks are few
// (latency-bound: 10 Mbp in 100 blocks of 100 kbp, 96.9 -> 60 ms); with thousands of blocks
// the sweeps are throughput-bound and the extra beta rows cost more than the shorter tail
// (chr10: 20.7 vs 23.4 ms).  reserve() sizes the beta rows by the same test.
// (the VALU-only concurrent split takes few-block workloads at N <= 128 even where the

}  // namespace

namespace itr_host {

// cus > 0: plan for that many CUs instead of the device's; host_only: the host-side plan
// (task lists, CU partition) without device allocations or uploads (itr_plan_partition_info)
int plan_create_impl(const int64_t* off, int64_t nblocks, double split_frac,
                     double post_split_frac, int cus, bool host_only, itr_plan_t* out) {
  if (!out) return fail(ITR_EINVAL, "null output pointer");
  *out = nullptr;
  if (nblocks < 0 || (nblocks > 0 && !off)) return fail(ITR_EINVAL, "bad block offsets");
  if (nblocks > INT32_MAX) return fail(ITR_EINVAL, "too many blocks");
  std::vector<int64_t> h_off(off, off + nblocks + 1);
  if (h_off[0] != 0) return fail(ITR_EINVAL, "block_off[0] must be 0");
  for (int64_t k = 0; k < nblocks; ++k) {
    if (h_off[k + 1] < h_off[k]) return fail(ITR_EINVAL, "block offsets decrease at %lld",
                                            (long long)k);
    if (h_off[k + 1] - h_off[k] > INT32_MAX) return fail(ITR_EINVAL, "block too long");
  }
  auto* p = new itr_plan();
  (void)hipGetDevice(&p->device);
  p->nblocks = nblocks;
  p->total = h_off[nblocks];
  p->h_off = h_off;
  std::vector<int64_t> tile_off(nblocks + 1, 0);
  for (int64_t k = 0; k < nblocks; ++k)
    tile_off[k + 1] = tile_off[k] + itr::vit_tiles(h_off[k + 1] - h_off[k]);
  p->ntiles = tile_off[nblocks];
  // longest-first processing order (stable: equal lengths keep block order)
  std::vector<int32_t> order(nblocks);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) {
    return h_off[x + 1] - h_off[x] > h_off[y + 1] - h_off[y];
  });
  p->sorted_len.resize(nblocks);
  for (int64_t k = 0; k < nblocks; ++k) p->sorted_len[k] = h_off[order[k] + 1] - h_off[order[k]];
  p->h_order.assign(order.begin(), order.end());
  if (nblocks > 0) {
    const int64_t k = std::min<int64_t>(nblocks - 1, 255);
    const int64_t T = h_off[order[k] + 1] - h_off[order[k]];
    p->prio_len = (int)std::max<int64_t>(T, 1);
  }
  // Forward log-likelihood tasks.  The longest block bounds the sweep's makespan (one
  // workgroup steps it column by column), so blocks at least half as long as the longest
  // (and >= 512 columns) become two half-length tasks — forward over the first half,
  // textbook backward over the second — whose vectors fwd_split_combine_kernel joins.
  // Tasks run longest first.  Two task lists over the same split blocks (slots):
  //   tasks   every block (the VALU-only sweep, state counts without a matrix-core form);
  //   the hybrid sweeps' own lists below.
  const int64_t tmax = nblocks ? h_off[order[0] + 1] - h_off[order[0]] : 0;
  std::vector<int32_t> split_blk;
  // split_frac (itr_plan_create_ex; negative = the default 0.5): 0 disables the split (tests
  // compare the split forward with the unsplit one)
  const double frac = split_frac < 0 ? 0.5 : split_frac;
  auto is_split = [&](int64_t T) {
    return frac > 0 && T >= 512 && (double)T >= frac * (double)tmax;
  };
  std::vector<int32_t> slot_of(nblocks, -1);
  for (int64_t k = 0; k < nblocks; ++k) {
    const int32_t b = order[k];
    if (is_split(h_off[b + 1] - h_off[b])) {
      slot_of[b] = (int32_t)split_blk.size();
      split_blk.push_back(b);
    }
  }
  // posterior split set (blocks at least post_split_frac of the longest, default a quarter,
  // >= 512 columns; 0 disables): a prefix of the order
  std::vector<int64_t> boff(nblocks, -1);
  {
    const double pfrac = post_split_frac < 0 ? 0.25 : post_split_frac;
    int64_t rows = 0, k = 0;
    for (; k < nblocks; ++k) {
      const int64_t T = h_off[order[k] + 1] - h_off[order[k]];
      if (!(pfrac > 0 && T >= 512 && (double)T >= pfrac * (double)tmax)) break;
      boff[order[k]] = rows;
      rows += T;
    }
    p->npsplit = k;
    p->beta_rows = rows;
  }
  auto make_tasks = [&](int64_t count) {
    std::vector<int32_t> tasks;
    std::vector<int64_t> tlen;
    for (int64_t k = 0; k < count; ++k) {
      const int32_t b = order[k];
      const int64_t T = h_off[b + 1] - h_off[b];
      if (slot_of[b] >= 0) {
        const int32_t m = (int32_t)(T / 2), slot = slot_of[b];
        tasks.insert(tasks.end(), {b, m, slot, b, -m, slot});
        tlen.push_back(m);
        tlen.push_back(T - m + 1);
      } else {
        tasks.insert(tasks.end(), {b, 0, 0});
        tlen.push_back(T);
      }
    }
    std::vector<int64_t> idx(tlen.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return tlen[x] > tlen[y]; });
    std::vector<int32_t> sorted(tasks.size());
    for (size_t k = 0; k < idx.size(); ++k)
      for (int c = 0; c < 3; ++c) sorted[3 * k + c] = tasks[3 * idx[k] + c];
    return sorted;
  };
  std::vector<int32_t> tasks = make_tasks(nblocks);
  // Hybrid sweeps (mfma_sweeps.hip).  A matrix-core group steps four blocks in about twice
  // the VALU step time, so the longest work stays on the lower-latency VALU path and the
  // bulk goes through the matrix cores.  Forward log-likelihood, with
  // L = ufrac * longest:  T > 2L -> VALU tasks (split halves as above);  L < T <= 2L -> two
  // matrix-core halves (first half forward, second half the textbook backward);  T <= L ->
  // whole block in a matrix-core group.  (The posterior's split is chosen per call, run_hybrid.)
  // Split slots of the hybrid forward are numbered separately (hsplit_blk).
  // ufrac measured on the (5,5) model, 10 Mbp (scripts/gpu_r2b.sh: 0.12 / 0.18 / 0.22 / 0.25
  // / 0.28 / 0.33 -> forward 4.93 / 4.24 / 3.97 / 3.85 / 3.80 / 3.97 ms)
  double ufrac = 0.28;
  // ... and never below what a matrix-core group finishes within the plan's expected makespan
  // (kMixGroupCol per column of its longest member): a smaller alignment with a short longest
  // block (a chr100 shard) would otherwise send many blocks to the VALU tasks and reserve CUs
  // for them that the bulk needs
  double colns = kMixGroupCol;
  double L = std::max(256.0, ufrac * (double)tmax);
  if (colns > 0) {
    const int ncu = cus > 0 ? cus : cu_count();
    const double Tm = std::max((double)h_off[nblocks] * kBulkCu / ncu, (double)tmax * kVitLone);
    L = std::max(L, Tm / colns);
  }
  std::vector<int32_t> hsplit_blk, utasks, mtasks;
  std::vector<int64_t> ulen;
  struct MT { int32_t id; int64_t steps; bool bwd; };
  std::vector<MT> fwd_t, bwd_t;
  for (int64_t k = 0; k < nblocks; ++k) {
    const int32_t b = order[k];
    const int64_t T = h_off[b + 1] - h_off[b];
    if ((double)T > 2 * L) {
      if (is_split(T)) {
        const int32_t m = (int32_t)(T / 2), slot = (int32_t)hsplit_blk.size();
        hsplit_blk.push_back(b);
        utasks.insert(utasks.end(), {b, m, slot, b, -m, slot});
        ulen.push_back(m);
        ulen.push_back(T - m + 1);
      } else {
        utasks.insert(utasks.end(), {b, 0, 0});
        ulen.push_back(T);
      }
    } else if ((double)T > L && T >= 512) {
      const int32_t m = (int32_t)(T / 2), slot = (int32_t)hsplit_blk.size();
      hsplit_blk.push_back(b);
      fwd_t.push_back({(int32_t)(mtasks.size() / 3), m, false});
      mtasks.insert(mtasks.end(), {b, m, slot});
      bwd_t.push_back({(int32_t)(mtasks.size() / 3), T - m + 1, true});
      mtasks.insert(mtasks.end(), {b, -m, slot});
    } else {
      fwd_t.push_back({(int32_t)(mtasks.size() / 3), T, false});
      mtasks.insert(mtasks.end(), {b, 0, 0});
    }
  }
  {  // VALU tasks longest first
    std::vector<int64_t> idx(ulen.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) { return ulen[x] > ulen[y]; });
    std::vector<int32_t> sorted(utasks.size());
    for (size_t k = 0; k < idx.size(); ++k)
      for (int c = 0; c < 3; ++c) sorted[3 * k + c] = utasks[3 * idx[k] + c];
    utasks.swap(sorted);
  }
  // matrix-core groups: forward-shaped tasks and second halves grouped separately (a group
  // shares its matrix operand), longest first, merged two groups at a time so that a
  // workgroup running two groups (GB = 2) always gets two of one kind
  auto by_steps = [](const MT& x, const MT& y) { return x.steps > y.steps; };
  std::stable_sort(fwd_t.begin(), fwd_t.end(), by_steps);
  std::stable_sort(bwd_t.begin(), bwd_t.end(), by_steps);
  std::vector<int32_t> groups_ll;
  {
    size_t fi = 0, bi2 = 0;
    auto take_group = [&](std::vector<MT>& v, size_t& i) {
      for (int r = 0; r < 4; ++r) groups_ll.push_back(i < v.size() ? v[i++].id : -1);
    };
    while (fi < fwd_t.size() || bi2 < bwd_t.size()) {
      const bool pick_f = bi2 >= bwd_t.size() ||
                          (fi < fwd_t.size() && fwd_t[fi].steps >= bwd_t[bi2].steps);
      for (int g = 0; g < 2; ++g) {
        if (pick_f) take_group(fwd_t, fi);
        else take_group(bwd_t, bi2);
      }
    }
  }
  // Viterbi long set and the CU partition of the forward+Viterbi call
  plan_partition(p, ulen, cus > 0 ? cus : cu_count());
  // The mixed queue: forward groups (steps = their longest member) and the remaining Viterbi
  // blocks merged by expected duration (kMixFwd, kMixVit), longest first.
  std::vector<int32_t> mix;
  {
    const int64_t ng = (int64_t)groups_ll.size() / 4;
    std::vector<int64_t> gsteps(ng, 0);
    for (int64_t g = 0; g < ng; ++g)
      for (int r = 0; r < 4; ++r) {
        const int32_t id = groups_ll[4 * g + r];
        if (id < 0) continue;
        const int32_t b = mtasks[3 * id], sp = mtasks[3 * id + 1];
        const int64_t Tb = h_off[b + 1] - h_off[b];
        gsteps[g] = std::max(gsteps[g], sp > 0 ? (int64_t)sp : (sp < 0 ? Tb + sp + 1 : Tb));
      }
    std::vector<int64_t> gidx(ng);
    std::iota(gidx.begin(), gidx.end(), 0);
    std::stable_sort(gidx.begin(), gidx.end(), [&](int64_t x, int64_t y) { return gsteps[x] > gsteps[y]; });
    const double cf = kMixFwd, cv = kMixVit;
    int64_t gi = 0, vi = p->vit_nlong;
    const int64_t nprio = kMixPrio;
    while (gi < ng || vi < nblocks) {
      const bool take_f = vi >= nblocks ||
                          (gi < ng && cf * (double)gsteps[gidx[gi]] >= cv * (double)p->sorted_len[vi]);
      if ((int64_t)mix.size() == nprio) {
        p->mix_prio_fwd = (int)std::max<int64_t>(1, gi < ng ? gsteps[gidx[gi]] : 1);
        p->mix_prio_vit = (int)std::max<int64_t>(1, vi < nblocks ? p->sorted_len[vi] : 1);
      }
      if (take_f) mix.push_back(-(int32_t)gidx[gi++] - 1);
      else mix.push_back(order[vi++]);
    }
    p->nmix = (int64_t)mix.size();
  }
  p->nutasks = (int64_t)utasks.size() / 3;
  p->ngroups_ll = (int64_t)groups_ll.size() / 4;
  p->nhsplit = (int64_t)hsplit_blk.size();
  p->ntasks = (int64_t)tasks.size() / 3;
  p->nsplit = (int64_t)split_blk.size();
  if (host_only) {
    *out = p;
    return 0;
  }
  int e = 0;
  if (!e) e = dev_alloc(&p->d_tasks, tasks.size());
  if (!e) e = dev_alloc(&p->d_mix, mix.size());
  if (!e) e = dev_alloc(&p->d_utasks, utasks.size());
  if (!e) e = dev_alloc(&p->d_mtasks, mtasks.size());
  if (!e) e = dev_alloc(&p->d_groups_ll, groups_ll.size());
  if (!e) e = dev_alloc(&p->d_hsplit_blk, hsplit_blk.size());
  if (!e) e = dev_alloc(&p->d_split_blk, split_blk.size());
  const size_t nslots = (size_t)std::max(p->nsplit, p->nhsplit);
  if (!e) e = dev_alloc(&p->d_svec, nslots * 2 * 256);
  if (!e) e = dev_alloc(&p->d_sK, nslots * 2);
  if (!e) e = dev_alloc(&p->d_off, nblocks + 1);
  if (!e) e = dev_alloc(&p->d_tile_off, nblocks + 1);
  if (!e) e = dev_alloc(&p->d_boff, nblocks);
  if (!e) e = dev_alloc(&p->d_order, nblocks);
  if (!e) e = dev_alloc(&p->d_queue, 16);
  if (!e && hipMemset(p->d_queue, 0, 16 * sizeof(int)) != hipSuccess)
    e = fail(ITR_EHIP, "plan workspace init failed");
  if (!e) e = dev_alloc(&p->d_sink, 64 * (size_t)itr::kSinkWgs);
  if (!e) e = dev_alloc(&p->d_last, nblocks);
  auto up = [&](void* d, const void* h, size_t bytes) {
    if (e || bytes == 0) return;
    if (hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) != hipSuccess)
      e = fail(ITR_EHIP, "plan upload failed");
  };
  up(p->d_off, h_off.data(), (nblocks + 1) * sizeof(int64_t));
  up(p->d_tile_off, tile_off.data(), (nblocks + 1) * sizeof(int64_t));
  up(p->d_boff, boff.data(), nblocks * sizeof(int64_t));
  up(p->d_order, order.data(), nblocks * sizeof(int32_t));
  up(p->d_tasks, tasks.data(), tasks.size() * sizeof(int32_t));
  up(p->d_mix, mix.data(), mix.size() * sizeof(int32_t));
  up(p->d_utasks, utasks.data(), utasks.size() * sizeof(int32_t));
  up(p->d_mtasks, mtasks.data(), mtasks.size() * sizeof(int32_t));
  up(p->d_groups_ll, groups_ll.data(), groups_ll.size() * sizeof(int32_t));
  up(p->d_hsplit_blk, hsplit_blk.data(), hsplit_blk.size() * sizeof(int32_t));
  up(p->d_split_blk, split_blk.data(), split_blk.size() * sizeof(int32_t));
  if (e) {
    itr_plan_destroy(p);
    return e;
  }
  *out = p;
  return 0;
}

}  // namespace itr_host

extern "C" {

int itr_plan_create(const int64_t* off, int64_t nblocks, itr_plan_t* out) {
  return itr_plan_create_ex(off, nblocks, -1.0, -1.0, out);
}

int itr_plan_create_ex(const int64_t* off, int64_t nblocks, double split_frac,
                       double post_split_frac, itr_plan_t* out) {
  return plan_create_impl(off, nblocks, split_frac, post_split_frac, 0, false, out);
}

int itr_plan_partition_info(const int64_t* off, int64_t nblocks, int cus, int64_t* out) {
  if (!out || cus < 1) return fail(ITR_EINVAL, "bad arguments");
  itr_plan_t p = nullptr;
  if (int e = plan_create_impl(off, nblocks, -1.0, -1.0, cus, true, &p)) return e;
  out[0] = p->vit_nlong;
  out[1] = p->vit_long_cols;
  out[2] = p->vit_reserve;
  out[3] = p->fwd_reserve;
  out[4] = p->wave_ok ? 1 : 0;
  out[5] = p->vit_nlong_v;
  out[6] = p->nutasks;
  out[7] = p->nmix;
  out[8] = p->vit_prune_len;
  out[9] = p->vit_prune_len_v;
  delete p;  // (host-only: nothing on the device)
  return 0;
}

int itr_plan_set_prune_len(itr_plan_t p, int64_t len) {
  if (int e = check_plan(p)) return e;
  p->prune_override = len < 0 ? -1 : len;
  return 0;
}

int itr_plan_destroy(itr_plan_t p) {
  if (!p) return 0;
  dev_free(p->d_off);
  dev_free(p->d_tile_off);
  dev_free(p->d_boff);
  dev_free(p->d_sublo);
  dev_free(p->d_comb);
  dev_free(p->d_beta);
  dev_free(p->d_order);
  dev_free(p->d_queue);
  dev_free(p->d_sink);
  dev_free(p->d_stay);
  dev_free(p->d_tasks);
  dev_free(p->d_mix);
  dev_free(p->d_utasks);
  dev_free(p->d_mtasks);
  dev_free(p->d_groups_ll);
  dev_free(p->d_hsplit_blk);
  dev_free(p->d_split_blk);
  dev_free(p->d_svec);
  dev_free(p->d_sK);
  dev_free(p->d_last);
  dev_free(p->d_alpha);
  delete p;
  return 0;
}

int itr_plan_total_columns(itr_plan_t p, int64_t* total) {
  if (!p || !total) return fail(ITR_EINVAL, "null pointer");
  *total = p->total;
  return 0;
}

}  // extern "C"
