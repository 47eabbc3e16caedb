// sweeps.h — internal interface between the C ABI (capi.cpp) and the HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace itr {

enum SweepMode {
  MODE_FWD_LL = 0,
  MODE_FWD_STORE = 1,
  MODE_BWD = 2,
  MODE_VIT = 3,
  // the backward sweep storing beta rows only (the hybrid posterior's split blocks, inside
  // the forward-store launch): MODE_BWD's arithmetic without its posterior code
  MODE_BETA = 4
};

// Viterbi columns per tile: one omega checkpoint row and one 16-bit stay-flag word per
// state per tile of every block (tiles start at each block's first column)
constexpr int VIT_TILE = 16;
inline int64_t vit_tiles(int64_t T) { return (T + VIT_TILE - 1) / VIT_TILE; }

struct SweepArgs {
  int n;                        // hidden states
  int xp;                       // padded length of the LDS state vectors
  int64_t nblocks;
  const int64_t* off;           // [nblocks+1] column offsets of the blocks
  const int32_t* order;         // [nblocks] processing order (longest first)
  int* queue;                   // work counter, zero at launch
  const uint16_t* obs;          // [total] observed symbols
  const double* mat;            // a (forward/backward) or log a (Viterbi), n x n
  const double* matT;           // a^T (MODE_FWD_LL: backward halves of split blocks)
  const double* emit;           // E or log E, 625 x n
  const double* init;           // pi*E or log(pi*E), 625 x n
  double* loglik;               // [nblocks]                       (MODE_FWD_LL)
  double* alpha;                // [total x XR] rescaled forward rows (FWD_STORE out, BWD in);
                                //   Viterbi: [tiles x XR] checkpoint rows (MODE_VIT out)
  double* post;                 // [total x n] posteriors          (MODE_BWD)
  double* sink;                 // [64] write target of padded states (MODE_BWD)
  uint16_t* stay;               // [tiles x XR] bit u of (tile, j): bp(16 tile + u, j) == j
                                //   is certain (MODE_VIT)
  const int64_t* tile_off;      // [nblocks+1] first tile record of every block (MODE_VIT)
  uint8_t* last_state;          // [nblocks] argmax of the last column (MODE_VIT)
  int prio_len;                 // blocks at least this long run at raised wave priority
  double* beta;                 // MODE_BWD, optional: store the backward rows beta_t here
                                //   (row beta_off[block] + t, stride XR) instead of posteriors
  const int64_t* beta_off;      //   [nblocks] first beta row of every split block
  int64_t nbeta;                // hybrid MODE_FWD_STORE: the first nbeta blocks of `order`
                                //   also get a backward task storing beta rows (see
                                //   mfma_sweeps.hip); 0 elsewhere
  const int64_t* sub_lo;        // MODE_BWD, optional, [nblocks]: lo > 0 splits the block at
                                //   column lo: a beta task (beta set) sweeps columns [lo, T)
                                //   only, storing beta_lo .. beta_{T-1}; a posterior task
                                //   sweeps columns [0, lo] only, from beta_lo (beta_in)
  const double* beta_in;        //   the stored beta rows the posterior tasks start from
  const int64_t* comb;          // hybrid MODE_BWD: ncomb combine tasks {block, t0, t1}: the
  int64_t ncomb;                //   posterior rows of columns [t0, t1) from the stored alpha
  int* comb_queue;              //   and beta rows (the split blocks' (lo, T)), after the
                                //   matrix-core groups; their work counter
  const int32_t* tasks;         // MODE_FWD_LL: [nblocks x 3] {block, split, slot}, see capi.cpp
  double* svec;                 // MODE_FWD_LL: [nsplit x 2 x XR] vectors of split blocks
  int* sK;                      // MODE_FWD_LL: [nsplit x 2] their power-of-two exponents
  int xrec;                     // MODE_VIT on the lane-group layout (lane_groups.h): record
                                //   stride of the checkpoint rows / flag words
  uint64_t* diag;               // diagnostic build only: per-segment cycle sums
  int diag_wave;                // diagnostic build only: the wave that reports
};

struct SweepGeometry {
  int iq;       // kernel configuration index (negative: unsupported)
  int block;    // threads per workgroup (64 * waves)
  int xp;       // padded vector length
  size_t lds;   // dynamic LDS bytes
  int per_cu;   // resident workgroups per CU (occupancy API)
};

SweepGeometry sweep_geometry(int n, int mode);
// row stride (padded states) of the back-pointer rows (MODE_VIT) / forward rows (FWD_STORE,
// BWD: both use the same configuration)
int sweep_row_stride(int n, int mode);

// Posterior of long blocks with concurrent forward and backward sweeps (hmm_sweeps.hip):
// one persistent launch running f (MODE_FWD_STORE over f.nblocks blocks of f.order) and, for
// the first nlong blocks of b.order, the backward sweep storing its rows into b.beta; then
// post_combine forms alpha_t beta_t / sum_j alpha_t beta_t for those blocks' columns.
hipError_t launch_post_split(const SweepGeometry& g, int grid, const SweepArgs& f,
                             const SweepArgs& b, int nlong, hipStream_t st);
// sub_lo (optional): the blocks' beta rows start at column sub_lo[block] (row beta_off +
// t - lo) and only columns (lo, T) are formed (the posterior task did [0, lo])
hipError_t launch_post_combine(int n, int xr, int nlong, int64_t tmax, const int32_t* order,
                               const int64_t* off, const double* alpha, const double* beta,
                               const int64_t* beta_off, double* post, hipStream_t st,
                               const int64_t* sub_lo = nullptr);
hipError_t launch_sweep(int mode, const SweepGeometry& g, int grid, const SweepArgs& a,
                        hipStream_t st);

// Matrix-core sweeps (mfma_sweeps.hip): groups of four blocks advanced in lock-step
constexpr int kSinkWgs = 1024;  // workgroups with a sink line set of their own (MfmaArgs.sink)
struct MfmaArgs {
  int n;                        // hidden states
  int64_t ngroups;
  const int32_t* groups;        // [ngroups x 4] longest group first (-1: none): task ids of
                                //   `tasks` (MODE_FWD_LL) or block ids (other modes)
  int64_t nmembers;             // > 0: groups = consecutive 4-chunks of this many entries
  const int32_t* tasks;         // MODE_FWD_LL: {block, split, slot} (see SweepArgs.tasks)
  int* queue;                   // work counter, zero at launch
  const int64_t* off;           // [nblocks+1]
  const uint16_t* obs;          // [total]
  const double* mat;            // a, n x n
  const double* matT;           // a^T (MODE_FWD_LL: groups of second halves)
  const double* emit;           // E, 625 x n
  const double* init;           // pi*E, 625 x n
  double* loglik;               // [nblocks]                  (MODE_FWD_LL)
  double* alpha;                // forward rows, row stride astride (FWD_STORE out, BWD in)
  int64_t astride;
  double* post;                 // [total x n]                (MODE_BWD)
  double* sink;                 // [kSinkWgs x 64] store target of lanes with no row to write
                                //   (FWD_STORE, BWD): every step stores unconditionally
  double* svec;                 // MODE_FWD_LL: split halves' vectors [slots x 2 x astride]
  int* sK;                      // MODE_FWD_LL: their power-of-two exponents [slots x 2]
  int prio_len;                 // groups at least this long run at raised wave priority
};
struct MfmaGeometry {
  int cfg;      // configuration index (negative: no matrix-core form for this n / mode)
  int block;    // threads per workgroup
  int xr;       // padded targets (row stride of stored forward rows >= xr)
  int gb;       // groups per workgroup
  int per_cu;   // resident workgroups per CU (occupancy API)
  double pfrac; // posterior sweeps: blocks longer than pfrac x the longest are VALU tasks
  double bfrac; // posterior: VALU-task blocks at least bfrac x the longest are split at ...
  double lofrac;//   ... column lofrac x T (backward over [lo, T) beside the forward sweep)
  size_t lds_min;  // launch with at least this much LDS (kExclusiveLds: one workgroup per CU)
};

// Dynamic LDS that leaves room for one workgroup per CU (160 KiB LDS per CU): requested when
// a launch has no more tasks than CUs, so the dispatcher cannot stack two of them on one CU
// (two co-resident sweeps step at ~1.6x the lone step time).
constexpr size_t kExclusiveLds = 81 * 1024;
MfmaGeometry mfma_geometry(int n, int mode);
// one launch: the VALU tasks of `v` (v.tasks / v.order, v.nblocks of them: the longest
// blocks, on the VALU configuration {8 lanes, g.block / 64 waves, 2 targets per lane}, whose
// rows have the same stride g.xr) first, then the matrix-core groups of `a`
hipError_t launch_hybrid_sweep(int mode, const MfmaGeometry& g, int grid, const MfmaArgs& a,
                               const SweepArgs& v, hipStream_t st);

// Viterbi with one block per wavefront (wave_tasks.h, wave_sweeps.hip)
struct VitArgs {
  int n;                        // hidden states
  int xr;                       // record stride of the checkpoint rows / flag words
  int64_t nblocks;              // blocks of `order`
  const int32_t* order;         // [nblocks] longest first
  int* queue;                   // work counter, zero at launch
  const int64_t* off;           // [plan blocks + 1]
  const int64_t* tile_off;      // [plan blocks + 1]
  const uint16_t* obs;          // [total]
  const double* la;             // log a, n x n
  const double* lew;            // log E, 625 x xr, by state (padding: -inf): full-scan step
  const double* lpie;           // log(pi E), 625 x n
  // the bound-pruned step (wave_tasks.h): its slot order and log E in that order
  const int32_t* slot_state;    // [xr] state of each slot (-1: padding)
  const double* slot_m;         // [xr] max_{i != j} log a_ij of the slot's state j
  const double* lew_p;          // log E, 625 x xr, columns in slot order (padding: -inf)
  int prune_len;                // blocks shorter than this take the bound-pruned step
  // non-null: the wave traces each block right after its sweep (trace.h) into `path`
  const double* log_e;          // 625 x n (state order)
  uint8_t* path;                // [total]
  double* ckpt;                 // [tiles x xr]
  uint16_t* stay;               // [tiles x xr]
  uint8_t* last_state;          // [plan blocks]
  int prio_len;                 // blocks at least this long run at raised wave priority
};
struct WaveVitGeometry {
  int iq;       // sources (= targets) per lane chunk; negative: no wave layout for this n
  int block;    // threads per workgroup
  int xr;       // padded targets (8 iq): record stride and log-emission table width
  size_t lds;   // dynamic LDS bytes
  int per_cu;   // resident workgroups per CU
};
WaveVitGeometry wave_vit_geometry(int n);
// role: 0 = bulk launch, 1 / 2 = a reserved set's late launch (only the kernel name differs)
hipError_t launch_wave_vit(const WaveVitGeometry& g, int grid, const VitArgs& p,
                           hipStream_t st, int role = 0);

// Viterbi for 72 < N <= 144 (prune_vit.hip): one block per wavefront, log a in the
// workgroup's LDS, the bound-pruned step; outputs as VitArgs' (ckpt / stay / last_state)
struct PruneVitArgs {
  int n;                        // hidden states
  int xr;                       // record stride of the checkpoint rows / flag words
  int64_t nblocks;              // blocks of `order`
  const int32_t* order;         // [nblocks] longest first
  int* queue;                   // work counter, zero at launch
  const int64_t* off;           // [plan blocks + 1]
  const int64_t* tile_off;      // [plan blocks + 1]
  const uint16_t* obs;          // [total]
  const double* la;             // log a, n x n
  const double* mj;             // [n] max_{i != j} log a_ij
  const double* log_e;          // 625 x n
  const double* lpie;           // log(pi E), 625 x n
  double* ckpt;                 // [tiles x xr]
  uint16_t* stay;               // [tiles x xr]
  uint8_t* last_state;          // [plan blocks]
  int prio_len;                 // blocks at least this long run at raised wave priority
  unsigned long long* diag;     // experiment build only: {columns, failing targets, passes}
};
struct PruneVitGeometry {
  int waves;    // wavefronts (blocks at a time) per workgroup; 0: no layout for this n
  int block;    // threads per workgroup
  int sources;  // sources per scanning lane
  size_t lds;   // dynamic LDS bytes
};
PruneVitGeometry prune_vit_geometry(int n);
hipError_t launch_prune_vit(const PruneVitGeometry& g, int grid, const PruneVitArgs& p,
                            hipStream_t st);

// The reference's per-column matrices of one block (rows.hip): kind 0 = log alpha, 1 = log
// beta, 2 = omega (+ prev when non-null); rows / prev are [T][n] / [T-1][n] float64
struct RowArgs {
  int kind, n;
  int64_t T;
  const uint16_t* obs;
  const double *a, *log_a, *emit, *log_emit, *lpie;
  double* rows;
  double* prev;
};
hipError_t launch_rows(const RowArgs& p, hipStream_t st);
hipError_t launch_backtrack_rows(const double* omega, const double* prev, int64_t T, int n,
                                 double* path, hipStream_t st);

// The forward log-likelihood sweep with one group of four tasks per wavefront on the matrix
// cores (wave_fwd.hip): the throughput form for short tasks
struct WaveMfmaArgs {
  int n;                        // hidden states
  int64_t ngroups;
  const int32_t* groups;        // [ngroups x 4] task ids (-1: none), longest first; a group is
                                //   all forward-shaped tasks or all backward halves
  const int32_t* tasks;         // {block, split, slot} (SweepArgs.tasks)
  int* queue;                   // work counter, zero at launch
  const int64_t* off;           // [plan blocks + 1]
  const uint16_t* obs;          // [total]
  const double* a;              // a, n x n
  const double* aT;             // a^T (groups of backward halves)
  const double* ef;             // E padded to er columns (zeros), row 625 = ones: 626 x er
  const double* emit;           // E, 625 x n (a backward half's first vector)
  const double* init;           // pi E, 625 x n
  double* loglik;               // [plan blocks]
  double* svec;                 // split halves' vectors, row stride sstride
  int64_t sstride;
  int* sK;                      // their power-of-two exponents [slots x 2]
  int prio_len;                 // groups at least this long run at raised wave priority
};
struct WaveMfmaGeometry {
  int cfg;      // configuration (negative: none for this n)
  int block;    // threads per workgroup
  int er;       // padded targets: width of the padded emission table
  size_t lds;   // dynamic LDS bytes
  int per_cu;   // resident workgroups per CU
  bool mixed;   // the mixed launch (Viterbi blocks + forward groups, one queue) exists
  size_t mixed_lds;
  int mixed_per_cu;
};
WaveMfmaGeometry wave_mfma_geometry(int n);
hipError_t launch_wave_mfma(const WaveMfmaGeometry& g, int grid, const WaveMfmaArgs& p,
                            hipStream_t st);
// forward groups and Viterbi blocks from one queue (wave_sweeps.hip): list entry e >= 0 = the
// Viterbi block e (v), e < 0 = forward group -e - 1 (f); queue zero at launch
hipError_t launch_wave_mixed(const WaveMfmaGeometry& g, int grid, const VitArgs& v,
                             const WaveMfmaArgs& f, const int32_t* list, int nlist, int* queue,
                             hipStream_t st, int role = 0);

// The forward log-likelihood's VALU tasks (SweepArgs.tasks: the longest blocks and the
// halves of the split ones) on lane groups per target (lane_groups.h, hmm_sweeps.hip): their
// lowest step latency, on the reserved CUs of a partitioned call; xr = the row stride of the
// split halves' vectors (the hybrid configuration's)
struct FwdGroupGeometry {
  int block;    // threads per workgroup (0: no lane-group forward for this state count)
  int xr;       // target slots = split-vector stride
  size_t lds;   // dynamic LDS bytes
  int per_cu;   // resident workgroups per CU
};
FwdGroupGeometry fwd_group_geometry(int n);
hipError_t launch_fwd_group(const FwdGroupGeometry& g, int grid, const SweepArgs& a,
                            hipStream_t st);

// log-likelihoods of the split blocks of a forward sweep
hipError_t launch_fwd_split_combine(int n, int xr, int nsplit, const int32_t* split_blk,
                                    const double* svec, const int* sK, double* loglik,
                                    hipStream_t st);

// Viterbi traceback over the checkpoint rows and stay flags written by MODE_VIT
struct TraceArgs {
  int n;                      // hidden states
  int xr;                     // row stride of the tile records
  int64_t nblocks;
  const int64_t* off;         // [nblocks+1]
  const int64_t* tile_off;    // [nblocks+1]
  const int32_t* order;       // [nblocks] longest first
  int* queue;                 // work counter, zero at launch
  const uint16_t* obs;        // [total]
  const double* log_a;        // n x n
  const double* log_e;        // 625 x n
  const double* ckpt;         // [tiles x xr] omega at each tile's first column
  const uint16_t* stay;       // [tiles x xr] stay-flag words
  const uint8_t* last_state;  // [nblocks]
  uint8_t* path;              // [total]
};
hipError_t launch_vit_traceback(const TraceArgs& a, int grid, hipStream_t st);

}  // namespace itr
