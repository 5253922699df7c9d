// hk_step.h -- per-arena entry points of the hot path: HBM state <-> register arena, HockeyEnv.reset,
// HockeyEnv.step (one lane = one arena).  The __global__ wrappers live in hk_kernels.hip.
//
// HBM layout (struct of arrays, arena index innermost so a wave's 64 lanes touch 64 consecutive dwords
// of every field):
//   f[NFF][N]            float  body state: per dynamic body {origin x,y, COM x,y, angle, vx, vy, w,
//                               sleep time} + the puck's pending force (TRAIN_DEFENSE reset)
//   i[NPW][N]            int32  the packed int words (hk_kernels.h PW_*): touching mask | awake | done |
//                               one_starts, enabled mask | winner, has_puck1 | has_puck2 | max_t, time,
//                               episode and step counters (the 12 logical words I_* live in registers)
//   man[NSOLID][N][NMF]  float  Box2D manifold record (64 B) of every solid pair (read/written in place,
//                               touching only; hk_arena.h man_rec)
//   phase[3][N]          double BasicOpponent phases: player 1, player 2, player 2's weak bot under a per-arena
//                               override (global np.random stream -> per-arena Philox)
#pragma once
#include "hk_arena.h"

namespace hk {

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 (counter-based RNG): key = seed, counter = (arena lo, arena hi, step/episode, purpose)
// ------------------------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };
HK_DEV U4 philox(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  U4 c = {c0, c1, c2, c3};
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    U4 n = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
HK_DEV float u01f(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
HK_DEV double u01d(uint32_t a, uint32_t b) {  // numpy random_double construction (53 bits)
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}
enum { RNG_ACTION = 1, RNG_PHASE = 2, RNG_RESET = 3, RNG_PHASE0 = 4 };

// ------------------------------------------------------------------------------------------------
// world <-> HBM
// ------------------------------------------------------------------------------------------------
HK_DEV float &F(const DevState &s, int field, int64_t a) { return s.f[(int64_t)field * s.n + a]; }
// packed int word k (PW_*) of arena a
HK_DEV uint32_t &PW(const DevState &s, int k, int64_t a) {
  return reinterpret_cast<uint32_t *>(s.i)[(int64_t)k * s.n + a];
}
HK_DEV void load_ints(const DevState &s, int64_t a, uint32_t (&pw)[NPW], int32_t (&iw)[NIF]) {
#pragma unroll
  for (int k = 0; k < NPW; ++k) pw[k] = PW(s, k, a);
  unpack_ints(pw, iw);
}

// The HBM words one arena's step reads before it computes anything: its state, the acting BasicOpponents'
// phases, the per-arena policy override, phase increments and external actions.  step_kernel issues these
// loads before its scene copy, so the whole fetch costs one memory latency instead of one per dependent use.
struct StepWords {
  float f[NFF];
  uint32_t pw[NPW];  // the packed int words as fetched
  int32_t i[NIF];    // ... unpacked
  double ph[3];
  double inc[2];
  float act[8];
  int32_t pol2;
};
HK_DEV void fetch_words(StepWords &m, const DevState &s, const KCfg &cfg, const StepIO &io, int64_t a) {
#pragma unroll
  for (int k = 0; k < NFF; ++k) m.f[k] = F(s, k, a);
#pragma unroll
  for (int k = 0; k < NPW; ++k) m.pw[k] = PW(s, k, a);
  unpack_ints(m.pw, m.i);
  // phase rows a bot may use (wave-uniform conditions; row 2 only under an override)
  m.ph[0] = cfg.policy[0] >= 2 ? s.phase[a] : 0.0;
  m.ph[1] = (cfg.policy[1] >= 2 || io.policy2) ? s.phase[s.n + a] : 0.0;
  m.ph[2] = io.policy2 ? s.phase[2 * s.n + a] : 0.0;
  m.pol2 = io.policy2 ? (int32_t)io.policy2[a] : 0;
#pragma unroll
  for (int p = 0; p < 2; ++p) m.inc[p] = io.opp_inc ? io.opp_inc[a * 2 + p] : 0.0;
#pragma unroll
  for (int k = 0; k < 8; ++k) m.act[k] = io.actions ? io.actions[a * 8 + k] : 0.0f;
}

// the register arena from its HBM words (f: NFF floats, iw: NIF ints)
HK_DEV void unpack_arena(Arena &w, const float *fw, const int32_t *iw, int64_t a, const DevState &s, int keep_mode,
                         int vel_ref, float *lds, int lane) {
  const int awake = iw[I_AWAKE];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int o = b * FB;
    w.d.px[b] = fw[o + FB_PX];
    w.d.py[b] = fw[o + FB_PY];
    w.d.cx[b] = fw[o + FB_CX];
    w.d.cy[b] = fw[o + FB_CY];
    w.d.a[b] = fw[o + FB_A];
    const rot q = rot_set(w.d.a[b]);
    w.d.qs[b] = q.s;
    w.d.qc[b] = q.c;
    w.d.c0x[b] = w.d.cx[b];
    w.d.c0y[b] = w.d.cy[b];
    w.d.a0[b] = w.d.a[b];
    w.d.al0[b] = 0.0f;
    w.d.vx[b] = fw[o + FB_VX];
    w.d.vy[b] = fw[o + FB_VY];
    w.d.w[b] = fw[o + FB_W];
    w.d.sleep[b] = fw[o + FB_SLEEP];
    w.d.awake[b] = (awake >> b) & 1;
    w.d.fx[b] = 0.0f;
    w.d.fy[b] = 0.0f;
    w.d.tq[b] = 0.0f;
    w.d.ld[b] = 0.0f;
    w.d.ad[b] = 0.0f;
  }
  w.d.fx[B_PK] = fw[F_PFX];
  w.d.fy[B_PK] = fw[F_PFY];
  w.keep_mode = keep_mode;
  w.vel_ref = vel_ref;
  w.has1 = iw[I_HAS1];
  w.has2 = iw[I_HAS2];
  w.time = iw[I_TIME];
  w.done = iw[I_DONE];
  w.winner = iw[I_WINNER];
  w.max_t = iw[I_MAXT];
  w.n_toi = 0;
  w.overflow = 0;
  w.n_big = 0;
  w.force_big = 0;
#ifdef HK_PHASE_TIMERS
  w.dg_vit_isl = w.dg_vit_toi = w.dg_pit = w.dg_toi_calls = w.dg_nc_max = 0;
#endif
  w.touch = (uint32_t)iw[I_TOUCH];
  w.enabled = (uint32_t)iw[I_ENABLED];
  w.toiflag = w.cisl = w.bisl = 0u;
  w.man = s.man;
  w.ws = s.ws;
  w.n = s.n;
  w.a = a;
  w.lds = lds;
  w.lane = lane;
#ifdef HK_TRACE
  w.trace = nullptr;
#endif
}
HK_DEV void load_arena(Arena &w, const DevState &s, int64_t a, int keep_mode, int vel_ref, float *lds, int lane) {
  float fw[NFF];
  uint32_t pw[NPW];
  int32_t iw[NIF];
#pragma unroll
  for (int k = 0; k < NFF; ++k) fw[k] = F(s, k, a);
  load_ints(s, a, pw, iw);
  unpack_arena(w, fw, iw, a, s, keep_mode, vel_ref, lds, lane);
}

// the logical int words of an arena after a step / reset (one_starts, episode and step passed in)
HK_DEV void arena_ints(const Arena &w, int awake, int one, int ep, int step, int32_t (&iw)[NIF]) {
  iw[I_AWAKE] = awake;
  iw[I_HAS1] = w.has1;
  iw[I_HAS2] = w.has2;
  iw[I_TIME] = w.time;
  iw[I_DONE] = w.done;
  iw[I_WINNER] = w.winner;
  iw[I_MAXT] = w.max_t;
  iw[I_TOUCH] = (int)w.touch;
  iw[I_ENABLED] = (int)w.enabled;
  iw[I_ONE] = one;
  iw[I_EPISODE] = ep;
  iw[I_STEP] = step;
}
// one < 0: keep the stored one_starts bit
HK_DEV void store_arena(const Arena &w, const DevState &s, int64_t a, int one = -1) {
  int awake = 0;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int o = b * FB;
    F(s, o + FB_PX, a) = w.d.px[b];
    F(s, o + FB_PY, a) = w.d.py[b];
    F(s, o + FB_CX, a) = w.d.cx[b];
    F(s, o + FB_CY, a) = w.d.cy[b];
    F(s, o + FB_A, a) = w.d.a[b];
    F(s, o + FB_VX, a) = w.d.vx[b];
    F(s, o + FB_VY, a) = w.d.vy[b];
    F(s, o + FB_W, a) = w.d.w[b];
    F(s, o + FB_SLEEP, a) = w.d.sleep[b];
    awake |= (w.d.awake[b] & 1) << b;
  }
  F(s, F_PFX, a) = w.d.fx[B_PK];
  F(s, F_PFY, a) = w.d.fy[B_PK];
  if (one < 0) one = (int)(PW(s, PW_TAW, a) >> 31);
  int32_t iw[NIF];
  uint32_t pw[NPW];
  arena_ints(w, awake, one, 0, 0, iw);
  pack_ints(iw, pw);
  PW(s, PW_TAW, a) = pw[PW_TAW];
  PW(s, PW_ENW, a) = pw[PW_ENW];
  PW(s, PW_HM, a) = pw[PW_HM];
  PW(s, PW_TIME, a) = pw[PW_TIME];
}

// store_arena after a step: the same words, but the fields that rarely change in play (sleep times, the puck's
// pending force, awake bits, has_puck, done, winner, time limit, touching / enabled masks) are written only by
// lanes whose value changed against the step's fetched words (fw, iw).  A wave whose 16 lanes of a 64-B segment
// all keep their value issues no write for it, which takes those fields off the HBM write traffic.
// one / ep / step: the arena's one_starts, episode and step words after this step
HK_DEV void store_arena_changed(const Arena &w, const DevState &s, int64_t a, const float *fw, const uint32_t *pw0,
                                int one, int ep, int step) {
  int awake = 0;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const int o = b * FB;
    F(s, o + FB_PX, a) = w.d.px[b];
    F(s, o + FB_PY, a) = w.d.py[b];
    F(s, o + FB_CX, a) = w.d.cx[b];
    F(s, o + FB_CY, a) = w.d.cy[b];
    F(s, o + FB_A, a) = w.d.a[b];
    F(s, o + FB_VX, a) = w.d.vx[b];
    F(s, o + FB_VY, a) = w.d.vy[b];
    F(s, o + FB_W, a) = w.d.w[b];
    if (__float_as_uint(w.d.sleep[b]) != __float_as_uint(fw[o + FB_SLEEP])) F(s, o + FB_SLEEP, a) = w.d.sleep[b];
    awake |= (w.d.awake[b] & 1) << b;
  }
  if (__float_as_uint(w.d.fx[B_PK]) != __float_as_uint(fw[F_PFX])) F(s, F_PFX, a) = w.d.fx[B_PK];
  if (__float_as_uint(w.d.fy[B_PK]) != __float_as_uint(fw[F_PFY])) F(s, F_PFY, a) = w.d.fy[B_PK];
  int32_t iw[NIF];
  uint32_t pw[NPW];
  arena_ints(w, awake, one, ep, step, iw);
  pack_ints(iw, pw);
  PW(s, PW_TIME, a) = pw[PW_TIME];
  PW(s, PW_STEP, a) = pw[PW_STEP];
#pragma unroll
  for (int k = 0; k < NPW; ++k)
    if (k != PW_TIME && k != PW_STEP && pw[k] != pw0[k]) PW(s, k, a) = pw[k];
}

// HockeyEnv.reset body re-creation (hockey_env.py:345-418) from placement params.
// player*_has_puck is NOT cleared (the reference's reset never assigns it).
HK_DEV void reset_arena(Arena &w, const float *p6, int max_t) {
  const float ix[3] = {2.0f, p6[0], p6[2]}, iy[3] = {4.0f, p6[1], p6[3]};
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const rot q = rot_set(0.0f);
    xform x;
    x.p = V(ix[b], iy[b]);
    x.q = q;
    const v2 c = mul_xv(x, V(g_scene.lcx[b], g_scene.lcy[b]));
    w.d.px[b] = ix[b];
    w.d.py[b] = iy[b];
    w.d.qs[b] = q.s;
    w.d.qc[b] = q.c;
    w.d.a[b] = w.d.a0[b] = 0.0f;
    w.d.al0[b] = 0.0f;
    w.d.cx[b] = w.d.c0x[b] = c.x;
    w.d.cy[b] = w.d.c0y[b] = c.y;
    w.d.vx[b] = w.d.vy[b] = w.d.w[b] = 0.0f;
    w.d.fx[b] = w.d.fy[b] = w.d.tq[b] = 0.0f;
    w.d.ld[b] = w.d.ad[b] = 0.0f;
    w.d.sleep[b] = 0.0f;
    w.d.awake[b] = 1;
  }
  w.d.ld[B_PK] = 0.05f;
  if (p6[4] != 0.0f || p6[5] != 0.0f) apply_force<B_PK>(w, V(p6[4], p6[5]));
  w.touch = 0u;
  w.enabled = (1u << NP) - 1u;
  w.max_t = max_t;
  w.time = 0;
  w.done = 0;
  w.winner = 0;
}

// device placement (same formulas as hockey_amd/placement.py with Philox uniforms instead of PCG64)
HK_DEV void device_placement(uint64_t seed, int64_t a, uint32_t episode, int mode, int one_starts, float *p6,
                             int &max_t) {
  const double W = 10.0, H = 8.0;
  U4 r0 = philox(seed, (uint32_t)a, (uint32_t)(a >> 32), episode, RNG_RESET);
  U4 r1 = philox(seed, (uint32_t)a, (uint32_t)(a >> 32), episode, RNG_RESET + 0x100);
  const double u0 = u01d(r0.x, r0.y), u1 = u01d(r0.z, r0.w), u2 = u01d(r1.x, r1.y), u3 = u01d(r1.z, r1.w);
  U4 r2 = philox(seed, (uint32_t)a, (uint32_t)(a >> 32), episode, RNG_RESET + 0x200);
  const double u4 = u01d(r2.x, r2.y);
  int k = 0;  // k-th uniform of this reset (a select chain: no indexed private array)
  auto unif = [&](double lo, double hi) {
    const double x = k == 0 ? u0 : (k == 1 ? u1 : (k == 2 ? u2 : (k == 3 ? u3 : u4)));
    ++k;
    return lo + (hi - lo) * x;
  };
  max_t = mode == 0 ? 250 : 80;
  double p2x = 4 * W / 5, p2y = H / 2;
  if (mode != 0) {
    p2x = 4 * W / 5 + unif(-W / 3, W / 6);
    p2y = H / 2 + unif(-H / 4, H / 4);
  }
  double px, py;
  float fx = 0.0f, fy = 0.0f;
  if (mode == 0 || mode == 1) {
    if (one_starts || mode == 1) {
      px = W / 2 - unif(H / 8, H / 4);
      py = H / 2 + unif(-H / 8, H / 8);
    } else {
      px = W / 2 + unif(H / 8, H / 4);
      py = H / 2 + unif(-H / 8, H / 8);
    }
  } else {
    px = W / 2 + unif(0, W / 3);
    py = H / 2 + 0.8 * unif(-H / 2, H / 2);
    float aim = (float)(H / 2 + .6 * unif(-75.0 / 60.0, 75.0 / 60.0));
    float dx = (float)px - 0.0f, dy = (float)py - aim;
    float ln = sqrtf(dx * dx + dy * dy);
    dx = dx / ln;
    dy = dy / ln;
    const float m = g_scene.mass[B_PK];
    fx = ((-dx * 60.0f) * m) / 0.02f;
    fy = ((-dy * 60.0f) * m) / 0.02f;
  }
  p6[0] = (float)p2x; p6[1] = (float)p2y; p6[2] = (float)px; p6[3] = (float)py; p6[4] = fx; p6[5] = fy;
}

HK_DEV void write_info(float *dst, int64_t a, const double *info) {
  float *p = dst + a * 4;
  if (((uintptr_t)p & 15) == 0) {  // one 16-B store: the lane's row is written whole, no partial-line write
    *reinterpret_cast<float4 *>(p) = float4{(float)info[0], (float)info[1], (float)info[2], (float)info[3]};
  } else {
    for (int k = 0; k < 4; ++k) p[k] = (float)info[k];
  }
}

// This lane's K-float output row (arena a, row-major [N][K]).  Device build, full wave with a 16-B-aligned wave
// block: the 64 rows are staged in the wave's free LDS work-list area and written as 16-B stores of consecutive
// memory, so each store instruction writes whole 64-B segments (a per-lane dword store covers every row of the
// wave at one word, and the L2 then writes each line piecewise).  Otherwise per-lane stores.
template <int K>
HK_DEV void store_row(float *dst, int64_t a, const float *v, float *stage, int lane) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(64 * K <= kToiQ * kToiItemWords, "the staged rows fit the TOI work-list area");
  float *base = dst + (a - lane) * K;
  if (__ballot(1) == ~0ull && ((uintptr_t)base & 15) == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) stage[lane * K + j] = v[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const float4 *src = reinterpret_cast<const float4 *>(stage);
    float4 *d4 = reinterpret_cast<float4 *>(base);
#pragma unroll
    for (int q = 0; q < (16 * K + 63) / 64; ++q)
      if (q * 64 + lane < 16 * K) d4[q * 64 + lane] = src[q * 64 + lane];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the stage is free again for the next row
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return;
  }
#endif
  for (int j = 0; j < K; ++j) dst[a * K + j] = v[j];
}

// HockeyEnv.reset of arena a: explicit placement params or device placement (Philox), one_starting toggle.
HK_DEV void reset_lane(const DevState &s, const KCfg &cfg, int64_t a, const float *params, const int32_t *max_t_in,
                       const uint8_t *one_in) {
  Arena w;
  load_arena(w, s, a, cfg.keep_mode, cfg.vel_ref, nullptr, 0);
  float p6[6];
  int mt;
  uint32_t pw[NPW];
  int32_t iw[NIF];
  load_ints(s, a, pw, iw);
  int one = iw[I_ONE];
  if (params) {
    for (int k = 0; k < 6; ++k) p6[k] = params[a * 6 + k];
    mt = cfg.mode == 0 ? 250 : 80;
    if (cfg.mode == 0) one = one_in ? (int)one_in[a] : !one;
  } else {
    if (cfg.mode == 0) one = one_in ? (int)one_in[a] : !one;
    const uint32_t ep = (uint32_t)iw[I_EPISODE];
    device_placement(cfg.seed, cfg.arena_offset + a, ep, cfg.mode, one, p6, mt);
  }
  if (max_t_in) mt = max_t_in[a];
  reset_arena(w, p6, mt);
  store_arena(w, s, a, one);
  PW(s, PW_EPISODE, a) = (uint32_t)iw[I_EPISODE] + 1u;
}

// One HockeyEnv.step of arena a (policy actions, pre-solve laws, world.Step, outputs, then auto-reset).
struct LaneOut { int done_edge, win1, win2, ntoi, ovf, nbig, bad_policy; };

// m: the step's HBM words (fetch_words), fetched by the caller so that it can issue them early
HK_DEV void step_lane(const DevState &s, const KCfg &cfg, const StepIO &io, int64_t a, float *lds, int lane,
                      PhaseT &T, LaneOut &out, const StepWords &m) {
  HK_EV(EV_STEP, 1);
  Arena w;
  unpack_arena(w, m.f, m.i, a, s, cfg.keep_mode, cfg.vel_ref, lds, lane);
  w.force_big = cfg.diag & 1;
#ifdef HK_TRACE
  w.trace = io.debug ? io.debug + a * kTraceStride : nullptr;
#endif
  const uint32_t stepc = (uint32_t)m.i[I_STEP];
  HK_TIC_SPLIT(T, 14);
  // ---- actions: external / Philox random / fused BasicOpponent ----
  float a8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a8[k] = m.act[k];  // external actions (zeros without io.actions)
  int bad_policy = 0;
  for (int p = 0; p < 2; ++p) {
    int pol = cfg.policy[p], row = p;  // row: the acting BasicOpponent's phase (DevState::phase)
    if (p == 1 && io.policy2) {
      pol = m.pol2;
      row = pol == 2 ? 2 : 1;
      if (pol > 3) {  // not an HK_POLICY_*: counted (HK_CNT_BAD_POLICY), the player acts with zeros
        bad_policy = 1;
        pol = -1;
      }
    }
    if (pol <= 0) {
      if (pol < 0)
        for (int k = 0; k < 4; ++k) a8[4 * p + k] = 0.0f;
    } else if (pol == 1) {
      const int64_t ga = cfg.arena_offset + a;
      U4 r = philox(cfg.seed, (uint32_t)ga, (uint32_t)(ga >> 32), stepc, RNG_ACTION + 0x10 * p);
      a8[4 * p + 0] = 2.0f * u01f(r.x) - 1.0f;
      a8[4 * p + 1] = 2.0f * u01f(r.y) - 1.0f;
      a8[4 * p + 2] = 2.0f * u01f(r.z) - 1.0f;
      a8[4 * p + 3] = 2.0f * u01f(r.w) - 1.0f;
    } else {
      float o[18];
      if (p == 0) observe(w, o); else observe_two(w, o);
      double inc;
      if (io.opp_inc) inc = p == 0 ? m.inc[0] : m.inc[1];
      else {
        const int64_t ga = cfg.arena_offset + a;
        U4 r = philox(cfg.seed, (uint32_t)ga, (uint32_t)(ga >> 32), stepc, RNG_PHASE + 0x10 * p);
        inc = 0.0 + (0.2 - 0.0) * u01d(r.x, r.y);
      }
      double ph = row == 0 ? m.ph[0] : (row == 1 ? m.ph[1] : m.ph[2]);
      basic_opponent(pol == 2, w.keep_mode, ph, inc, o, &a8[4 * p]);
      s.phase[row * s.n + a] = ph;
    }
  }
  if (io.actions_out)
    for (int k = 0; k < 8; ++k) io.actions_out[a * 8 + k] = a8[k];
  // ---- HockeyEnv.step ----
  const int was_done = w.done;
  HK_TIC_SPLIT(T, 15);
  HK_TIC(T, 0);
  presolve(w, a8);
  HK_TIC(T, 0);
#ifndef HK_PHASE_TIMERS
  if (io.debug) {
#ifdef HK_TRACE
    float *d = io.debug + a * kTraceStride;
#else
    float *d = io.debug + a * 13;
#endif
    d[0] = w.d.fx[B_P1]; d[1] = w.d.fy[B_P1]; d[2] = w.d.fx[B_P2]; d[3] = w.d.fy[B_P2];
    d[4] = w.d.fx[B_PK]; d[5] = w.d.fy[B_PK]; d[6] = w.d.tq[B_P1]; d[7] = w.d.tq[B_P2];
    d[8] = w.d.ld[B_P1]; d[9] = w.d.ld[B_P2]; d[10] = w.d.ld[B_PK]; d[11] = w.d.ad[B_P1]; d[12] = w.d.ad[B_P2];
  }
#endif

  if (!(io.flags & 1)) {
    world_step(w, T);
  } else {
#pragma unroll
    for (int b = 0; b < 3; ++b) { w.d.fx[b] = 0.0f; w.d.fy[b] = 0.0f; w.d.tq[b] = 0.0f; }
  }
  float o[18];
  observe(w, o);
  if (io.final_obs)
    for (int k = 0; k < 18; ++k) io.final_obs[a * 18 + k] = o[k];
  if (w.time >= w.max_t) w.done = 1;
  double info[4];
  info_side<0>(w, info);
  if (io.info) write_info(io.info, a, info);
  if (io.reward) io.reward[a] = (float)(compute_reward(w) + info[1]);
  if (io.info2 || io.reward2) {
    double info2[4];
    info_side<1>(w, info2);
    if (io.info2) write_info(io.info2, a, info2);
    if (io.reward2) io.reward2[a] = (float)(-compute_reward(w) + info2[1]);
  }
  if (io.done) io.done[a] = (uint8_t)w.done;
  w.time += 1;
  if (io.record) {  // the step's float64 values for single-env callers (hk_step_io.record)
    double i2[4];
    info_side<1>(w, i2);
    double *rec = io.record + a * 16;
    for (int k = 0; k < 4; ++k) {
      rec[k] = info[k];
      rec[4 + k] = i2[k];
    }
    rec[8] = compute_reward(w) + info[1];
    rec[9] = -compute_reward(w) + i2[1];
    rec[10] = w.has1;
    rec[11] = w.has2;
    rec[12] = w.time;
    rec[13] = w.done;
    rec[14] = w.winner;
    rec[15] = 0.0;
  }
  const int done_edge = !was_done && w.done, winner = w.winner;
  int one_new = m.i[I_ONE], ep_new = m.i[I_EPISODE];
  if (cfg.auto_reset && w.done) {  // the next episode starts now; obs / obs2 describe its first state
    int one = m.i[I_ONE];
    if (cfg.mode == 0) one = !one;
    const uint32_t ep = (uint32_t)m.i[I_EPISODE];
    float p6[6];
    int mt;
    device_placement(cfg.seed, cfg.arena_offset + a, ep, cfg.mode, one, p6, mt);
    reset_arena(w, p6, mt);
    one_new = one;
    ep_new = (int)(ep + 1);
    observe(w, o);
  }
  float *stage = lds + kLdsPerLane * 64;  // the TOI / narrow-phase work-list area, free after world_step
  if (io.obs) store_row<18>(io.obs, a, o, stage, lane);
  if (io.obs2) {
    observe_two(w, o);
    store_row<18>(io.obs2, a, o, stage, lane);
  }
  store_arena_changed(w, s, a, m.f, m.pw, one_new, ep_new, (int)(stepc + 1));
  HK_TIC(T, 12);  // diagnostics: outputs and state store
  out.done_edge = done_edge;
  out.win1 = done_edge && winner == 1;
  out.win2 = done_edge && winner == -1;
  out.ntoi = w.n_toi;
  out.ovf = w.overflow;
  out.nbig = w.n_big;
  out.bad_policy = bad_policy;
#ifdef HK_PHASE_TIMERS
  if (io.debug) {  // diagnostics build: per-lane work counters
    float *d = io.debug + a * 24;
    d[1] = (float)w.n_toi; d[2] = (float)w.dg_vit_isl; d[3] = (float)w.dg_vit_toi; d[4] = (float)w.dg_pit;
    d[5] = (float)w.dg_toi_calls; d[6] = (float)w.dg_nc_max; d[7] = (float)w.n_big;
    d[21] = (float)T.fam[0]; d[22] = (float)T.fam[1]; d[23] = (float)T.fam[2];
  }
#endif
}


HK_DEV void observe_lane(const DevState &s, const KCfg &cfg, int64_t a, float *obs, float *obs2) {
  Arena w;
  load_arena(w, s, a, cfg.keep_mode, cfg.vel_ref, nullptr, 0);
  float o[18];
  if (obs) {
    observe(w, o);
    for (int k = 0; k < 18; ++k) obs[a * 18 + k] = o[k];
  }
  if (obs2) {
    observe_two(w, o);
    for (int k = 0; k < 18; ++k) obs2[a * 18 + k] = o[k];
  }
}

// _get_info / get_info_agent_two / get_reward(_get_info()) / get_reward_agent_two(...) of the current state,
// float64 like the reference (hockey_env.py:518-591)
HK_DEV void info_lane(const DevState &s, const KCfg &cfg, int64_t a, double *info, double *info2, double *reward,
                      double *reward2) {
  Arena w;
  load_arena(w, s, a, cfg.keep_mode, cfg.vel_ref, nullptr, 0);
  double i1[4], i2[4];
  info_side<0>(w, i1);
  info_side<1>(w, i2);
  for (int k = 0; k < 4; ++k) {
    if (info) info[a * 4 + k] = i1[k];
    if (info2) info2[a * 4 + k] = i2[k];
  }
  if (reward) reward[a] = compute_reward(w) + i1[1];
  if (reward2) reward2[a] = -compute_reward(w) + i2[1];
}

HK_DEV void get_state_lane(const DevState &s, int64_t a, float *st, int32_t *aux) {
  for (int b = 0; b < 3; ++b) {
    const int o = b * FB;
    if (st) {
      st[a * 18 + 6 * b + 0] = F(s, o + FB_PX, a);
      st[a * 18 + 6 * b + 1] = F(s, o + FB_PY, a);
      st[a * 18 + 6 * b + 2] = F(s, o + FB_A, a);
      st[a * 18 + 6 * b + 3] = F(s, o + FB_VX, a);
      st[a * 18 + 6 * b + 4] = F(s, o + FB_VY, a);
      st[a * 18 + 6 * b + 5] = F(s, o + FB_W, a);
    }
  }
  if (aux) {
    uint32_t pw[NPW];
    int32_t iw[NIF];
    load_ints(s, a, pw, iw);
    aux[a * 5 + 0] = iw[I_HAS1];
    aux[a * 5 + 1] = iw[I_HAS2];
    aux[a * 5 + 2] = iw[I_TIME];
    aux[a * 5 + 3] = iw[I_DONE];
    aux[a * 5 + 4] = iw[I_WINNER];
  }
}

// One body's pybox2d setters in set_state's order: position, angle, linearVelocity, angularVelocity
// (hockey_env.py:595-606).  A NaN entry means "setter not called" (set_state never assigns the puck's angle
// or angular velocity, :604-605), so a NaN position pair / angle / velocity pair / omega is skipped.
HK_DEV bool nan_f(float x) { return x != x; }  // IEEE: only a NaN compares unequal to itself (no fast-math)
template <int B>
HK_DEV void set_body_state(Arena &w, const float *x) {
  if (!(nan_f(x[0]) && nan_f(x[1]))) set_transform<B>(w, V(x[0], x[1]), w.d.a[B]);
  if (!nan_f(x[2])) set_transform<B>(w, V(w.d.px[B], w.d.py[B]), x[2]);
  if (!(nan_f(x[3]) && nan_f(x[4]))) set_linear_velocity<B>(w, V(x[3], x[4]));
  if (!nan_f(x[5])) set_angular_velocity<B>(w, x[5]);
}

// HockeyEnv.set_state (hockey_env.py:594-608) raw form: pybox2d setters, contacts untouched
HK_DEV void set_state_lane(const DevState &s, const KCfg &cfg, int64_t a, const float *st, const int32_t *aux) {
  Arena w;
  load_arena(w, s, a, cfg.keep_mode, cfg.vel_ref, nullptr, 0);
  if (st) {
    const float *x = st + a * 18;
    set_body_state<B_P1>(w, x);
    set_body_state<B_P2>(w, x + 6);
    set_body_state<B_PK>(w, x + 12);
  }
  if (aux) {
    w.has1 = aux[a * 5 + 0];
    w.has2 = aux[a * 5 + 1];
    w.time = aux[a * 5 + 2];
    w.done = aux[a * 5 + 3];
    w.winner = aux[a * 5 + 4];
  }
  store_arena(w, s, a);
}

HK_DEV void init_lane(const DevState &s, const KCfg &cfg, int64_t a) {
  // all zero: winner 0 is stored as 1 (PW_ENW), one_starts 0 -- HockeyEnv.__init__ sets one_starts = True and resets
  // with one_starting=True (hockey_env.py:117,155); hk_create's first reset toggles this 0 -> 1
  int32_t iw[NIF] = {};
  uint32_t pw[NPW];
  pack_ints(iw, pw);
  for (int k = 0; k < NPW; ++k) PW(s, k, a) = pw[k];
  for (int k = 0; k < NFF; ++k) F(s, k, a) = 0.0f;
  for (int p = 0; p < 3; ++p) {  // row 2: player 2's weak bot under a per-arena override
    const int64_t ga = cfg.arena_offset + a;
    U4 r = philox(cfg.seed, (uint32_t)ga, (uint32_t)(ga >> 32), 0, RNG_PHASE0 + 0x10 * p);
    s.phase[p * s.n + a] = 0.0 + (kPiD - 0.0) * u01d(r.x, r.y);  // BasicOpponent.__init__ U(0, pi)
  }
}

}  // namespace hk
