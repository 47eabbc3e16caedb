// wave_sweeps.hip — persistent launches of the per-wavefront sweep tasks (wave_tasks.h) for
// MI355X (gfx950): Viterbi blocks, forward groups, or both from one mixed queue.  Every
// workgroup is four independent wavefronts (no barrier); a wave pulls its next task from a
// device counter, longest first, until the queue is drained.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "wave_tasks.h"

namespace itr {
namespace {

template <int IQ>
using VitLayout = WaveVitAny<IQ>;

constexpr int kWaves = 4;  // independent wavefronts per workgroup

// every lane takes part in the queue atomic (lane 0 adds 1): with a lane-divergent
// `if (l == 0)` at the loop head hipcc (ROCm 7.2) built a lane-divergent inner loop in which
// lanes 1..63 re-read a stale index and the wave never finished
__device__ __forceinline__ int next_task(int* queue) {
  return uni(atomicAdd(queue, (threadIdx.x & 63) == 0 ? 1 : 0));
}

// ROLE only names the launch in kernel traces: 0 = the bulk launch, 1 / 2 = the late launches
// of the reserved CU sets joining the same queue (same code)
template <int IQ, int ROLE>
__global__ void __launch_bounds__(64 * kWaves, 2) wave_vit_kernel(VitArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* wl = reinterpret_cast<double*>(smem) + (size_t)(threadIdx.x >> 6) * VitLayout<IQ>::WL;
  for (;;) {
    const int bi = next_task(p.queue);
    if (bi >= p.nblocks) break;
    vit_wave_block<IQ>(p, wl, uni(p.order[bi]));
  }
}

#ifdef ITR_EXPERIMENT  // the forward alone on the per-wave layout: experiment library only
template <int NT, int NK>
__global__ void __launch_bounds__(64 * kWaves, 2) wave_fwd_kernel(WaveMfmaArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* wl = reinterpret_cast<double*>(smem) + (size_t)(threadIdx.x >> 6) * WF<NT, NK>::WL;
  for (;;) {
    const int gi = next_task(p.queue);
    if (gi >= p.ngroups) break;
    fwd_wave_task<NT, NK>(p, wl, gi);
  }
}
#endif

// One queue of both kinds: entry e >= 0 = the Viterbi block e, e < 0 = forward group -e - 1.
template <int IQ, int NT, int NK>
struct Mixed {
  static constexpr int WL = VitLayout<IQ>::WL > WF<NT, NK>::WL ? VitLayout<IQ>::WL : WF<NT, NK>::WL;
};
template <int IQ, int NT, int NK, int ROLE>
__global__ void __launch_bounds__(64 * kWaves, 2)
    wave_mixed_kernel(VitArgs v, WaveMfmaArgs f, const int32_t* list, int nlist, int* queue) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* wl =
      reinterpret_cast<double*>(smem) + (size_t)(threadIdx.x >> 6) * Mixed<IQ, NT, NK>::WL;
  for (;;) {
    const int k = next_task(queue);
    if (k >= nlist) break;
    const int e = uni(list[k]);
    if (e < 0) {
      fwd_wave_task<NT, NK>(f, wl, -e - 1);
    } else {
      vit_wave_block<IQ>(v, wl, e);
    }
  }
}

template <class K>
int occupancy(K kernel, size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, 64 * kWaves, lds) != hipSuccess ||
      nb < 1)
    nb = 1;
  return nb;
}

struct WCfg {
  int nmin, nmax, nt, nk;
};
constexpr WCfg kWCfgs[] = {{33, 48, 3, 12}, {49, 64, 4, 16}, {65, 72, 5, 18}};

template <int NT, int NK>
[[maybe_unused]] size_t wf_lds() {
  return (size_t)kWaves * WF<NT, NK>::WL * sizeof(double);
}

}  // namespace

WaveVitGeometry wave_vit_geometry(int n) {
  WaveVitGeometry g{};
  g.iq = -1;
  if (n > 64 && n <= 72) g.iq = 9;  // the (5,5) model, N = 70
  if (g.iq < 0) return g;
  g.block = 64 * kWaves;
  g.xr = 8 * g.iq;
  g.lds = (size_t)kWaves * VitLayout<9>::WL * sizeof(double);
  g.per_cu = occupancy(wave_vit_kernel<9, 0>, g.lds);
  return g;
}

hipError_t launch_wave_vit(const WaveVitGeometry& g, int grid, const VitArgs& p,
                           hipStream_t st, int role) {
  if (g.iq != 9) return hipErrorInvalidValue;
  switch (role) {
    case 0: hipLaunchKernelGGL((wave_vit_kernel<9, 0>), dim3(grid), dim3(g.block), g.lds, st, p); break;
    case 1: hipLaunchKernelGGL((wave_vit_kernel<9, 1>), dim3(grid), dim3(g.block), g.lds, st, p); break;
    default: hipLaunchKernelGGL((wave_vit_kernel<9, 2>), dim3(grid), dim3(g.block), g.lds, st, p); break;
  }
  return hipGetLastError();
}

WaveMfmaGeometry wave_mfma_geometry(int n) {
  WaveMfmaGeometry g{};
  g.cfg = -1;
  for (int c = 0; c < (int)(sizeof kWCfgs / sizeof kWCfgs[0]); ++c)
    if (n >= kWCfgs[c].nmin && n <= kWCfgs[c].nmax) g.cfg = c;
  if (g.cfg < 0) return g;
  g.block = 64 * kWaves;
  g.er = 16 * kWCfgs[g.cfg].nt;
#ifdef ITR_EXPERIMENT
  switch (g.cfg) {
    case 0: g.lds = wf_lds<3, 12>(); g.per_cu = occupancy(wave_fwd_kernel<3, 12>, g.lds); break;
    case 1: g.lds = wf_lds<4, 16>(); g.per_cu = occupancy(wave_fwd_kernel<4, 16>, g.lds); break;
    case 2: g.lds = wf_lds<5, 18>(); g.per_cu = occupancy(wave_fwd_kernel<5, 18>, g.lds); break;
  }
#endif
  // the mixed launch (Viterbi blocks + forward groups) exists for the (5,5) model's sizes
  g.mixed = (n > 64 && n <= 72) && g.cfg == 2;
  if (g.mixed) {
    g.mixed_lds = (size_t)kWaves * Mixed<9, 5, 18>::WL * sizeof(double);
    g.mixed_per_cu = occupancy(wave_mixed_kernel<9, 5, 18, 0>, g.mixed_lds);
  }
  return g;
}

hipError_t launch_wave_mfma(const WaveMfmaGeometry& g, int grid, const WaveMfmaArgs& p,
                            hipStream_t st) {
#ifndef ITR_EXPERIMENT
  (void)g, (void)grid, (void)p, (void)st;
  return hipErrorInvalidValue;
#else
  switch (g.cfg) {
    case 0: hipLaunchKernelGGL((wave_fwd_kernel<3, 12>), dim3(grid), dim3(g.block), g.lds, st, p); break;
    case 1: hipLaunchKernelGGL((wave_fwd_kernel<4, 16>), dim3(grid), dim3(g.block), g.lds, st, p); break;
    case 2: hipLaunchKernelGGL((wave_fwd_kernel<5, 18>), dim3(grid), dim3(g.block), g.lds, st, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
#endif
}

hipError_t launch_wave_mixed(const WaveMfmaGeometry& g, int grid, const VitArgs& v,
                             const WaveMfmaArgs& f, const int32_t* list, int nlist, int* queue,
                             hipStream_t st, int role) {
  if (!g.mixed) return hipErrorInvalidValue;
  switch (role) {
    case 0:
      hipLaunchKernelGGL((wave_mixed_kernel<9, 5, 18, 0>), dim3(grid), dim3(g.block), g.mixed_lds,
                         st, v, f, list, nlist, queue);
      break;
    case 1:
      hipLaunchKernelGGL((wave_mixed_kernel<9, 5, 18, 1>), dim3(grid), dim3(g.block), g.mixed_lds,
                         st, v, f, list, nlist, queue);
      break;
    default:
      hipLaunchKernelGGL((wave_mixed_kernel<9, 5, 18, 2>), dim3(grid), dim3(g.block), g.mixed_lds,
                         st, v, f, list, nlist, queue);
      break;
  }
  return hipGetLastError();
}

}  // namespace itr
