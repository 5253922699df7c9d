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

// io pointers of step k of a rollout: every array carries a leading [nsteps] dimension
HK_DEV StepIO step_io(const StepIO &io, int k, int nsteps, int64_t n) {
  StepIO r = io;
  const int64_t o = (int64_t)k * n;
  r.actions = io.actions ? io.actions + o * 8 : nullptr;
  r.opp_inc = io.opp_inc ? io.opp_inc + o * 2 : nullptr;
  r.obs = io.obs ? io.obs + o * 18 : nullptr;
  r.obs2 = io.obs2 ? io.obs2 + o * 18 : nullptr;
  r.reward = io.reward ? io.reward + o : nullptr;
  r.reward2 = io.reward2 ? io.reward2 + o : nullptr;
  r.done = io.done ? io.done + o : nullptr;
  r.info = io.info ? io.info + o * 4 : nullptr;
  r.info2 = io.info2 ? io.info2 + o * 4 : nullptr;
  r.actions_out = io.actions_out ? io.actions_out + o * 8 : nullptr;
  r.debug = (k == nsteps - 1) ? io.debug : nullptr;  // diagnostics describe the last step
  return r;
}

// nsteps consecutive HockeyEnv.step calls of every arena (nsteps == 1: hk_step; > 1: hk_rollout).  The
// arenas of a wave advance independently of every other wave, so a rollout launch is not paced by the
// slowest wave of each step.
template <bool kRollout>
__global__ void __launch_bounds__(64) step_kernel(DevState s, KCfg cfg, StepIO io, int nsteps) {
  if (!kRollout) nsteps = 1;
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
    for (int k = 0; k < nsteps; ++k) {
      LaneOut out;
      step_lane(s, cfg, step_io(io, k, nsteps, s.n), a, lds, threadIdx.x & 63, T, out);
      done_edge += out.done_edge;
      win1 += out.win1;
      win2 += out.win2;
      ntoi += out.ntoi;
      ovf |= out.ovf;
      nbig += out.nbig;
    }
  }
  const unsigned long long lanes = __ballot(live);
  if ((threadIdx.x & 63) == 0 && lanes) atomicAdd(&s.counters[0], (unsigned long long)__popcll(lanes) * nsteps);
  // per-lane sums (episode ends, goals, TOI events, large islands are sparse): one atomic per lane that has any
  if (done_edge > 0) atomicAdd(&s.counters[1], (unsigned long long)done_edge);
  if (win1 > 0) atomicAdd(&s.counters[2], (unsigned long long)win1);
  if (win2 > 0) atomicAdd(&s.counters[3], (unsigned long long)win2);
  if (ntoi > 0) atomicAdd(&s.counters[4], (unsigned long long)ntoi);
  wave_count(s.counters, 5, ovf);
  if (nbig > 0) atomicAdd(&s.counters[6], (unsigned long long)nbig);
#ifdef HK_PHASE_TIMERS
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&s.counters[8 + k], T.acc[k]);
  if (io.debug && live) {  // wave cycles (whole launch) for the tail analysis
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
hipError_t launch_step(const DevState &s, const KCfg &cfg, const StepIO &io, int nsteps, hipStream_t st) {
  if (nsteps == 1)
    hipLaunchKernelGGL(step_kernel<false>, grid_for(s.n), dim3(64), 0, st, s, cfg, io, 1);
  else
    hipLaunchKernelGGL(step_kernel<true>, grid_for(s.n), dim3(64), 0, st, s, cfg, io, nsteps);
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
