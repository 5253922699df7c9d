// hk_hostcheck.cpp -- the per-arena device code (hk_step.h / hk_arena.h / hk_solver.h / hk_geom.h)
// compiled for the host CPU, as a DEBUG AND TEST HARNESS ONLY.
//
// It lets the CPU test suite run the kernel's own per-lane logic against the oracle without a GPU, and
// gives gdb a build of the physics (GPU debuggers are unavailable on the pool).  It is never loaded by
// the product package (hockey_amd refuses to run without libhockey_hip.so and has no CPU path); only
// tests/ and scripts/ use libhockey_hostcheck.so.  The code is the same source as the kernel: g++ with
// -ffp-contract=off on x86-64 SSE gives the same IEEE float/double results as gfx950 (correctly rounded
// +,-,*,/,sqrt; no contraction), which the parity tests check.
#include <hip/hip_runtime.h>  // host-only under g++: __device__ / __forceinline__ expand to host code

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

static inline int __float_as_int(float x) { int r; std::memcpy(&r, &x, 4); return r; }
static inline unsigned __float_as_uint(float x) { unsigned r; std::memcpy(&r, &x, 4); return r; }
static inline float __int_as_float(int x) { float r; std::memcpy(&r, &x, 4); return r; }
static inline float __uint_as_float(unsigned x) { float r; std::memcpy(&r, &x, 4); return r; }
static inline int __ffs(unsigned x) { return __builtin_ffs((int)x); }
static inline int __popc(unsigned x) { return __builtin_popcount(x); }
static inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
static inline int __double2hiint(double d) { uint64_t u; std::memcpy(&u, &d, 8); return (int)(u >> 32); }
static inline double __hiloint2double(int hi, int lo) {
  const uint64_t u = ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}

#define HK_HOST_DIAG
#include "../hk_core.h"

constexpr hk::Scene g_scene =  // the kernels' compile-time scene (hk_scene_gen.cpp)
#include "../hk_scene_data.inc"
    ;

#define SLDS g_scene  // the host build reads the one scene copy
#include "../hk_step.h"

unsigned long long hk::g_hk_host_diag[4];
unsigned long long hk::g_hk_flop_ev[hk::EV_N];

using namespace hk;

struct HostCtx {
  int64_t n;
  std::vector<float> f, man, ws;
  std::vector<int32_t> i;
  std::vector<double> phase;
  std::vector<unsigned long long> counters;
  std::vector<float> lds;
  DevState s;
  KCfg cfg;
};

extern "C" {

// cfg = {keep_mode, mode, auto_reset, vel_ref, policy0, policy1, diag_flags}; seed; arena_offset
void *hkh_create(int64_t n, const int *cfg6, uint64_t seed, int64_t arena_offset) {
  HostCtx *c = new HostCtx();
  c->n = n;
  c->f.assign((size_t)NFF * n, 0.0f);
  c->i.assign((size_t)NPW * n, 0);
  c->man.assign((size_t)NSOLID * NMF * n, 0.0f);
  c->phase.assign((size_t)3 * n, 0.0);
  c->counters.assign(16, 0ull);
  c->lds.assign((size_t)kLdsWords, 0.0f);
  c->s.f = c->f.data();
  c->s.i = c->i.data();
  c->s.man = c->man.data();
  c->ws.assign((size_t)kBigC * kSlotWords * n, 0.0f);
  c->s.ws = c->ws.data();
  c->s.phase = c->phase.data();
  c->s.counters = c->counters.data();
  c->s.n = n;
  std::memset(&c->cfg, 0, sizeof(c->cfg));
  c->cfg.keep_mode = cfg6[0];
  c->cfg.mode = cfg6[1];
  c->cfg.auto_reset = cfg6[2];
  c->cfg.vel_ref = cfg6[3];
  c->cfg.policy[0] = cfg6[4];
  c->cfg.policy[1] = cfg6[5];
  c->cfg.seed = seed;
  c->cfg.arena_offset = arena_offset;
  c->cfg.diag = cfg6[6];
  for (int64_t a = 0; a < n; ++a) init_lane(c->s, c->cfg, a);
  return c;
}

void hkh_destroy(void *h) { delete (HostCtx *)h; }

void hkh_reset(void *h, const uint8_t *mask, const float *params, const int32_t *max_t, const uint8_t *one) {
  HostCtx *c = (HostCtx *)h;
  for (int64_t a = 0; a < c->n; ++a)
    if (!mask || mask[a]) reset_lane(c->s, c->cfg, a, params, max_t, one);
}

// io layout == StepIO (same field order as include/hockey.h's hk_step_io)
void hkh_step(void *h, const StepIO *io) {
  HostCtx *c = (HostCtx *)h;
  for (int64_t a = 0; a < c->n; ++a) {
    PhaseT T;
    LaneOut out;
    StepWords m;
    fetch_words(m, c->s, c->cfg, *io, a);
    step_lane(c->s, c->cfg, *io, a, c->lds.data(), (int)(a & 63), T, out, m);
    c->counters[0] += 1;
    c->counters[1] += out.done_edge;
    c->counters[2] += out.win1;
    c->counters[3] += out.win2;
    c->counters[4] += out.ntoi;
    c->counters[5] += out.ovf;
    c->counters[6] += out.nbig;
    c->counters[7] += out.bad_policy;
  }
}

void hkh_get_state(void *h, float *st, int32_t *aux) {
  HostCtx *c = (HostCtx *)h;
  for (int64_t a = 0; a < c->n; ++a) get_state_lane(c->s, a, st, aux);
}

void hkh_set_state(void *h, const uint8_t *mask, const float *st, const int32_t *aux) {
  HostCtx *c = (HostCtx *)h;
  for (int64_t a = 0; a < c->n; ++a)
    if (!mask || mask[a]) set_state_lane(c->s, c->cfg, a, st, aux);
}

void hkh_observe(void *h, float *obs, float *obs2) {
  HostCtx *c = (HostCtx *)h;
  for (int64_t a = 0; a < c->n; ++a) observe_lane(c->s, c->cfg, a, obs, obs2);
}

// raw SoA state (diagnostics): f [NFF][N] floats, i [NPW][N] packed int words
void hkh_raw(void *h, float **f, int32_t **i) {
  HostCtx *c = (HostCtx *)h;
  *f = c->f.data();
  *i = c->i.data();
}

// event counts of the algorithmic FLOP count (hk_core.h HK_EV), process-wide; read and cleared
void hkh_flop_events(unsigned long long *out) {
  std::memcpy(out, hk::g_hk_flop_ev, sizeof(hk::g_hk_flop_ev));
  std::memset(hk::g_hk_flop_ev, 0, sizeof(hk::g_hk_flop_ev));
}
int hkh_flop_event_count(void) { return hk::EV_N; }

// velocity-loop coverage counters (hk_solver.h HK_HOST_DIAG_INC), process-wide; read and cleared
void hkh_diag(unsigned long long *out4) {
  std::memcpy(out4, hk::g_hk_host_diag, sizeof(hk::g_hk_host_diag));
  std::memset(hk::g_hk_host_diag, 0, sizeof(hk::g_hk_host_diag));
}

void hkh_counters(void *h, unsigned long long *out16) {
  HostCtx *c = (HostCtx *)h;
  std::memcpy(out16, c->counters.data(), 16 * sizeof(unsigned long long));
}

}  // extern "C"
