// hk_kernels.hip -- gfx950 kernels of the batched hockey simulator (one lane = one arena, 64-lane blocks).
// Per-arena logic: hk_step.h (state layout), hk_arena.h (physics), hk_solver.h (contact solver).
#include "hk_core.h"

__constant__ hk::Scene g_scene;

#include "hk_step.h"

namespace hk {

// wave-aggregated counter add (one atomic per wave)
HK_DEV void wave_count(unsigned long long *ctr, int idx, int pred) {
  const unsigned long long m = __ballot(pred);
  if (m && (threadIdx.x & 63) == (__ffsll((long long)m) - 1)) atomicAdd(&ctr[idx], (unsigned long long)__popcll(m));
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) reset_kernel(DevState s, KCfg cfg, const uint8_t *mask, const float *params,
                                                   const int32_t *max_t_in, const uint8_t *one_in) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  if (mask && !mask[a]) return;
  reset_lane(s, cfg, a, params, max_t_in, one_in);
}

__global__ void __launch_bounds__(64) step_kernel(DevState s, KCfg cfg, StepIO io) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = a < s.n;
  int done_edge = 0, win1 = 0, win2 = 0, ntoi = 0, ovf = 0, nbig = 0;
  PhaseT T;
#ifdef HK_PHASE_TIMERS
  for (int k = 0; k < 8; ++k) T.acc[k] = 0;
  T.last = __builtin_amdgcn_s_memtime();
#endif
  __shared__ float lds[kLdsPerLane * 64];
  if (live) {
    LaneOut out;
    step_lane(s, cfg, io, a, lds, threadIdx.x & 63, T, out);
    done_edge = out.done_edge;
    win1 = out.win1;
    win2 = out.win2;
    ntoi = out.ntoi;
    ovf = out.ovf;
    nbig = out.nbig;
  }
  wave_count(s.counters, 0, live);
  wave_count(s.counters, 1, done_edge);
  wave_count(s.counters, 2, win1);
  wave_count(s.counters, 3, win2);
  // few lanes carry TOI events / large islands; one atomic per lane that has any
  if (ntoi > 0) atomicAdd(&s.counters[4], (unsigned long long)ntoi);
  wave_count(s.counters, 5, ovf);
  if (nbig > 0) atomicAdd(&s.counters[6], (unsigned long long)nbig);
#ifdef HK_PHASE_TIMERS
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&s.counters[8 + k], T.acc[k]);
  if (io.debug && live) {  // wave cycles (whole step) for the tail analysis
    unsigned long long tot = 0;
    for (int k = 0; k < 8; ++k) tot += T.acc[k];
    io.debug[a * 8] = (float)tot;
  }
#endif
}

__global__ void __launch_bounds__(64) observe_kernel(DevState s, KCfg cfg, float *obs, float *obs2) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  observe_lane(s, cfg, a, obs, obs2);
}

__global__ void __launch_bounds__(64) get_state_kernel(DevState s, KCfg cfg, float *st, int32_t *aux) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  get_state_lane(s, a, st, aux);
}

__global__ void __launch_bounds__(64) set_state_kernel(DevState s, KCfg cfg, const uint8_t *mask, const float *st,
                                                       const int32_t *aux) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  if (mask && !mask[a]) return;
  set_state_lane(s, cfg, a, st, aux);
}

__global__ void init_kernel(DevState s, KCfg cfg) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  init_lane(s, cfg, a);
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
static inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + 63) / 64)); }

hipError_t launch_init(const DevState &s, const KCfg &cfg, hipStream_t st) {
  hipLaunchKernelGGL(init_kernel, grid_for(s.n), dim3(64), 0, st, s, cfg);
  return hipGetLastError();
}
hipError_t launch_reset(const DevState &s, const KCfg &cfg, const uint8_t *mask, const float *params,
                        const int32_t *max_t, const uint8_t *one, hipStream_t st) {
  hipLaunchKernelGGL(reset_kernel, grid_for(s.n), dim3(64), 0, st, s, cfg, mask, params, max_t, one);
  return hipGetLastError();
}
hipError_t launch_step(const DevState &s, const KCfg &cfg, const StepIO &io, hipStream_t st) {
  hipLaunchKernelGGL(step_kernel, grid_for(s.n), dim3(64), 0, st, s, cfg, io);
  return hipGetLastError();
}
hipError_t launch_observe(const DevState &s, const KCfg &cfg, float *obs, float *obs2, hipStream_t st) {
  hipLaunchKernelGGL(observe_kernel, grid_for(s.n), dim3(64), 0, st, s, cfg, obs, obs2);
  return hipGetLastError();
}
hipError_t launch_get_state(const DevState &s, const KCfg &cfg, float *state, int32_t *aux, hipStream_t st) {
  hipLaunchKernelGGL(get_state_kernel, grid_for(s.n), dim3(64), 0, st, s, cfg, state, aux);
  return hipGetLastError();
}
hipError_t launch_set_state(const DevState &s, const KCfg &cfg, const uint8_t *mask, const float *state,
                            const int32_t *aux, hipStream_t st) {
  hipLaunchKernelGGL(set_state_kernel, grid_for(s.n), dim3(64), 0, st, s, cfg, mask, state, aux);
  return hipGetLastError();
}
int64_t workspace_words_per_arena() { return (int64_t)kBigC * kSlotWords; }
hipError_t upload_scene(const Scene &sc) { return hipMemcpyToSymbol(HIP_SYMBOL(g_scene), &sc, sizeof(Scene)); }

}  // namespace hk
