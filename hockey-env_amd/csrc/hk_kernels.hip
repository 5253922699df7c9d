// hk_kernels.hip -- gfx950 kernels of the batched hockey simulator.
//
// HBM layout (struct of arrays, arena index innermost so a wave's 64 lanes touch 64 consecutive
// dwords of every field):
//   f[NFF][N]            float  body state: per dynamic body {origin x,y, COM x,y, angle, vx, vy, w,
//                               sleep time} + the puck's pending force (TRAIN_DEFENSE reset)
//   i[NIF][N]            int32  awake bits, has_puck1/2, time, done, winner, max_t, touching mask,
//                               enabled mask, one_starts, episode and step counters
//   man[NSOLID][NMF][N]  float  Box2D manifold of every solid pair (read only where touching)
//   phase[2][N]          double BasicOpponent phases (global np.random stream -> per-arena Philox)
// One lane = one arena; a block is one or more waves of independent arenas.
#include "hk_core.h"

__constant__ hk::Scene g_scene;

#include "hk_fast.h"
#include "hk_kernels.h"

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
HK_DEV int32_t &I(const DevState &s, int field, int64_t a) { return s.i[(int64_t)field * s.n + a]; }
HK_DEV float &M(const DevState &s, int slot, int field, int64_t a) {
  return s.man[((int64_t)slot * NMF + field) * s.n + a];
}

HK_DEV void load_world(World &w, const DevState &s, int64_t a, int keep_mode, int vel_ref) {
  init_static_bodies(w);
  const int awake = I(s, I_AWAKE, a);
  for (int b = 0; b < 3; ++b) {
    Body &B = w.b[b];
    const int o = b * FB;
    B.xf.p = V(F(s, o + FB_PX, a), F(s, o + FB_PY, a));
    B.c = V(F(s, o + FB_CX, a), F(s, o + FB_CY, a));
    B.a = F(s, o + FB_A, a);
    B.xf.q = rot_set(B.a);
    B.c0 = B.c;
    B.a0 = B.a;
    B.v = V(F(s, o + FB_VX, a), F(s, o + FB_VY, a));
    B.w = F(s, o + FB_W, a);
    B.sleep = F(s, o + FB_SLEEP, a);
    B.awake = (awake >> b) & 1;
    B.force = V(0.0f, 0.0f);
    B.torque = 0.0f;
    B.ld = 0.0f;
    B.ad = 0.0f;
  }
  w.b[B_PK].force = V(F(s, F_PFX, a), F(s, F_PFY, a));
  w.keep_mode = keep_mode;
  w.vel_ref = vel_ref;
  w.has1 = I(s, I_HAS1, a);
  w.has2 = I(s, I_HAS2, a);
  w.time = I(s, I_TIME, a);
  w.done = I(s, I_DONE, a);
  w.winner = I(s, I_WINNER, a);
  w.max_t = I(s, I_MAXT, a);
  w.n_toi = 0;
  w.overflow = 0;
  const uint32_t touch = (uint32_t)I(s, I_TOUCH, a), en = (uint32_t)I(s, I_ENABLED, a);
  for (int p = 0; p < NP; ++p) {
    Contact &c = w.c[p];
    c.touching = (touch >> p) & 1;
    c.enabled = (en >> p) & 1;
    c.toi_flag = 0;
    c.toi_count = 0;
    c.island_flag = 0;
    c.toi = 1.0f;
    c.m.count = 0;
    const int slot = g_scene.manslot[p];
    if (c.touching && slot >= 0) {
      const int meta = __float_as_int(M(s, slot, M_META, a));
      c.m.count = meta & 0xff;
      c.m.type = meta >> 8;
      c.m.ln = V(M(s, slot, M_LNX, a), M(s, slot, M_LNY, a));
      c.m.lp = V(M(s, slot, M_LPX, a), M(s, slot, M_LPY, a));
      for (int j = 0; j < 2; ++j) {
        const int o = M_P0X + j * 5;
        c.m.pt_lp[j] = V(M(s, slot, o + 0, a), M(s, slot, o + 1, a));
        c.m.id[j] = (uint32_t)__float_as_int(M(s, slot, o + 2, a));
        c.m.ni[j] = M(s, slot, o + 3, a);
        c.m.ti[j] = M(s, slot, o + 4, a);
      }
    }
  }
}

HK_DEV void store_world(const World &w, const DevState &s, int64_t a) {
  int awake = 0;
  for (int b = 0; b < 3; ++b) {
    const Body &B = w.b[b];
    const int o = b * FB;
    F(s, o + FB_PX, a) = B.xf.p.x;
    F(s, o + FB_PY, a) = B.xf.p.y;
    F(s, o + FB_CX, a) = B.c.x;
    F(s, o + FB_CY, a) = B.c.y;
    F(s, o + FB_A, a) = B.a;
    F(s, o + FB_VX, a) = B.v.x;
    F(s, o + FB_VY, a) = B.v.y;
    F(s, o + FB_W, a) = B.w;
    F(s, o + FB_SLEEP, a) = B.sleep;
    awake |= (B.awake & 1) << b;
  }
  F(s, F_PFX, a) = w.b[B_PK].force.x;
  F(s, F_PFY, a) = w.b[B_PK].force.y;
  I(s, I_AWAKE, a) = awake;
  I(s, I_HAS1, a) = w.has1;
  I(s, I_HAS2, a) = w.has2;
  I(s, I_TIME, a) = w.time;
  I(s, I_DONE, a) = w.done;
  I(s, I_WINNER, a) = w.winner;
  I(s, I_MAXT, a) = w.max_t;
  uint32_t touch = 0, en = 0;
  for (int p = 0; p < NP; ++p) {
    const Contact &c = w.c[p];
    touch |= (uint32_t)(c.touching & 1) << p;
    en |= (uint32_t)(c.enabled & 1) << p;
    const int slot = g_scene.manslot[p];
    if (c.touching && slot >= 0) {
      M(s, slot, M_META, a) = __int_as_float(c.m.count | (c.m.type << 8));
      M(s, slot, M_LNX, a) = c.m.ln.x;
      M(s, slot, M_LNY, a) = c.m.ln.y;
      M(s, slot, M_LPX, a) = c.m.lp.x;
      M(s, slot, M_LPY, a) = c.m.lp.y;
      for (int j = 0; j < c.m.count; ++j) {
        const int o = M_P0X + j * 5;
        M(s, slot, o + 0, a) = c.m.pt_lp[j].x;
        M(s, slot, o + 1, a) = c.m.pt_lp[j].y;
        M(s, slot, o + 2, a) = __int_as_float((int)c.m.id[j]);
        M(s, slot, o + 3, a) = c.m.ni[j];
        M(s, slot, o + 4, a) = c.m.ti[j];
      }
    }
  }
  I(s, I_TOUCH, a) = (int)touch;
  I(s, I_ENABLED, a) = (int)en;
}

// HockeyEnv.reset body re-creation (hockey_env.py:345-418) from placement params.
// player*_has_puck is NOT cleared (the reference's reset never assigns it).
HK_DEV void reset_world(World &w, const float *p6, int max_t) {
  const v2 pos[3] = {V(2.0f, 4.0f), V(p6[0], p6[1]), V(p6[2], p6[3])};
  for (int i = 0; i < 3; ++i) {
    Body &b = w.b[i];
    b.xf.p = pos[i];
    b.xf.q = rot_set(0.0f);
    b.a = b.a0 = 0.0f;
    b.alpha0 = 0.0f;
    b.c = b.c0 = mul_xv(b.xf, b.lc);
    b.v = V(0.0f, 0.0f);
    b.w = 0.0f;
    b.force = V(0.0f, 0.0f);
    b.torque = 0.0f;
    b.ld = 0.0f;
    b.ad = 0.0f;
    b.sleep = 0.0f;
    b.awake = 1;
  }
  w.b[B_PK].ld = 0.05f;
  if (p6[4] != 0.0f || p6[5] != 0.0f) apply_force(w.b[B_PK], V(p6[4], p6[5]));
  for (int p = 0; p < NP; ++p) {
    Contact &c = w.c[p];
    c.touching = 0;
    c.enabled = 1;
    c.m.count = 0;
  }
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
  double u[4] = {u01d(r0.x, r0.y), u01d(r0.z, r0.w), u01d(r1.x, r1.y), u01d(r1.z, r1.w)};
  U4 r2 = philox(seed, (uint32_t)a, (uint32_t)(a >> 32), episode, RNG_RESET + 0x200);
  double u4 = u01d(r2.x, r2.y);
  int k = 0;
  auto unif = [&](double lo, double hi) { double x = (k < 4) ? u[k] : u4; ++k; return lo + (hi - lo) * x; };
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

// wave-aggregated counter add (one atomic per wave)
HK_DEV void wave_count(unsigned long long *ctr, int idx, int pred) {
  const unsigned long long m = __ballot(pred);
  if (m && (threadIdx.x & 63) == (__ffsll((long long)m) - 1)) atomicAdd(&ctr[idx], (unsigned long long)__popcll(m));
}

HK_DEV void write_info(float *dst, int64_t a, const double *info) {
  for (int k = 0; k < 4; ++k) dst[a * 4 + k] = (float)info[k];
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) reset_kernel(DevState s, KCfg cfg, const uint8_t *mask, const float *params,
                                                   const int32_t *max_t_in, const uint8_t *one_in) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  if (mask && !mask[a]) return;
  World w;
  load_world(w, s, a, cfg.keep_mode, cfg.vel_ref);
  float p6[6];
  int mt;
  int one = I(s, I_ONE, a);
  if (params) {
    for (int k = 0; k < 6; ++k) p6[k] = params[a * 6 + k];
    mt = cfg.mode == 0 ? 250 : 80;
    if (cfg.mode == 0) one = one_in ? (int)one_in[a] : !one;
  } else {
    if (cfg.mode == 0) one = one_in ? (int)one_in[a] : !one;
    const uint32_t ep = (uint32_t)I(s, I_EPISODE, a);
    device_placement(cfg.seed, cfg.arena_offset + a, ep, cfg.mode, one, p6, mt);
  }
  if (max_t_in) mt = max_t_in[a];
  reset_world(w, p6, mt);
  store_world(w, s, a);
  I(s, I_ONE, a) = one;
  I(s, I_EPISODE, a) = I(s, I_EPISODE, a) + 1;
}

__global__ void __launch_bounds__(64) step_kernel(DevState s, KCfg cfg, StepIO io) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = a < s.n;
  int done_edge = 0, win1 = 0, win2 = 0, ntoi = 0, ovf = 0;
  PhaseT T;
#ifdef HK_PHASE_TIMERS
  for (int k = 0; k < 8; ++k) T.acc[k] = 0;
  T.last = __builtin_amdgcn_s_memtime();
#endif
  if (live) {
    World w;
    Solver S;
    load_world(w, s, a, cfg.keep_mode, cfg.vel_ref);
    const uint32_t stepc = (uint32_t)I(s, I_STEP, a);
    if (cfg.auto_reset && w.done) {
      int one = I(s, I_ONE, a);
      if (cfg.mode == 0) one = !one;
      const uint32_t ep = (uint32_t)I(s, I_EPISODE, a);
      float p6[6];
      int mt;
      device_placement(cfg.seed, cfg.arena_offset + a, ep, cfg.mode, one, p6, mt);
      reset_world(w, p6, mt);
      I(s, I_ONE, a) = one;
      I(s, I_EPISODE, a) = (int)(ep + 1);
    }
    // ---- actions: external / Philox random / fused BasicOpponent ----
    float a8[8];
    for (int p = 0; p < 2; ++p) {
      const int pol = cfg.policy[p];
      if (pol == 0) {
        for (int k = 0; k < 4; ++k) a8[4 * p + k] = io.actions ? io.actions[a * 8 + 4 * p + k] : 0.0f;
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
        if (io.opp_inc) inc = io.opp_inc[a * 2 + p];
        else {
          const int64_t ga = cfg.arena_offset + a;
          U4 r = philox(cfg.seed, (uint32_t)ga, (uint32_t)(ga >> 32), stepc, RNG_PHASE + 0x10 * p);
          inc = 0.0 + (0.2 - 0.0) * u01d(r.x, r.y);
        }
        double ph = s.phase[p * s.n + a];
        basic_opponent(pol == 2, w.keep_mode, ph, inc, o, &a8[4 * p]);
        s.phase[p * s.n + a] = ph;
      }
    }
    if (io.actions_out)
      for (int k = 0; k < 8; ++k) io.actions_out[a * 8 + k] = a8[k];
    // ---- HockeyEnv.step ----
    const int was_done = w.done;
    HK_TIC(T, 0);
    presolve(w, a8);
    HK_TIC(T, 1);
    if (io.debug) {
      float *d = io.debug + a * 13;
      d[0] = w.b[B_P1].force.x; d[1] = w.b[B_P1].force.y; d[2] = w.b[B_P2].force.x; d[3] = w.b[B_P2].force.y;
      d[4] = w.b[B_PK].force.x; d[5] = w.b[B_PK].force.y; d[6] = w.b[B_P1].torque; d[7] = w.b[B_P2].torque;
      d[8] = w.b[B_P1].ld; d[9] = w.b[B_P2].ld; d[10] = w.b[B_PK].ld; d[11] = w.b[B_P1].ad; d[12] = w.b[B_P2].ad;
    }
    if (!(io.flags & 1)) {
      world_step(w, S, cfg.ablate, T);
    } else {
      for (int i = 0; i < 3; ++i) { w.b[i].force = V(0.0f, 0.0f); w.b[i].torque = 0.0f; }
    }
    float o[18];
    if (io.obs) {
      observe(w, o);
      for (int k = 0; k < 18; ++k) io.obs[a * 18 + k] = o[k];
    }
    if (w.time >= w.max_t) w.done = 1;
    double info[4];
    info_side(w, 0, info);
    if (io.info) write_info(io.info, a, info);
    if (io.reward) io.reward[a] = (float)(compute_reward(w) + info[1]);
    if (io.obs2 || io.info2 || io.reward2) {
      if (io.obs2) {
        observe_two(w, o);
        for (int k = 0; k < 18; ++k) io.obs2[a * 18 + k] = o[k];
      }
      double info2[4];
      info_side(w, 1, info2);
      if (io.info2) write_info(io.info2, a, info2);
      if (io.reward2) io.reward2[a] = (float)(-compute_reward(w) + info2[1]);
    }
    if (io.done) io.done[a] = (uint8_t)w.done;
    w.time += 1;
    store_world(w, s, a);
    I(s, I_STEP, a) = (int)(stepc + 1);
    HK_TIC(T, 5);
    done_edge = (!was_done && w.done);
    win1 = done_edge && w.winner == 1;
    win2 = done_edge && w.winner == -1;
    ntoi = w.n_toi;
    ovf = w.overflow;
  }
  wave_count(s.counters, 0, live);
  wave_count(s.counters, 1, done_edge);
  wave_count(s.counters, 2, win1);
  wave_count(s.counters, 3, win2);
  if (__ballot(ntoi > 0)) {
    // few lanes carry TOI events; sum them with one atomic per lane that has any
    if (ntoi > 0) atomicAdd(&s.counters[4], (unsigned long long)ntoi);
  }
  wave_count(s.counters, 5, ovf);
#ifdef HK_PHASE_TIMERS
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&s.counters[8 + k], T.acc[k]);
#endif
}

__global__ void __launch_bounds__(64) observe_kernel(DevState s, KCfg cfg, float *obs, float *obs2) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  World w;
  load_world(w, s, a, cfg.keep_mode, cfg.vel_ref);
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

__global__ void __launch_bounds__(64) get_state_kernel(DevState s, KCfg cfg, float *st, int32_t *aux) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
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
    aux[a * 5 + 0] = I(s, I_HAS1, a);
    aux[a * 5 + 1] = I(s, I_HAS2, a);
    aux[a * 5 + 2] = I(s, I_TIME, a);
    aux[a * 5 + 3] = I(s, I_DONE, a);
    aux[a * 5 + 4] = I(s, I_WINNER, a);
  }
}

// HockeyEnv.set_state (hockey_env.py:594-608) raw form: pybox2d setters, contacts untouched
__global__ void __launch_bounds__(64) set_state_kernel(DevState s, KCfg cfg, const uint8_t *mask, const float *st,
                                                       const int32_t *aux) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  if (mask && !mask[a]) return;
  World w;
  load_world(w, s, a, cfg.keep_mode, cfg.vel_ref);
  if (st) {
    for (int i = 0; i < 3; ++i) {
      Body &b = w.b[i];
      const float *x = st + a * 18 + 6 * i;
      set_transform(b, V(x[0], x[1]), b.a);
      set_transform(b, b.xf.p, x[2]);
      set_linear_velocity(b, V(x[3], x[4]));
      set_angular_velocity(b, x[5]);
    }
  }
  if (aux) {
    w.has1 = aux[a * 5 + 0];
    w.has2 = aux[a * 5 + 1];
    w.time = aux[a * 5 + 2];
    w.done = aux[a * 5 + 3];
    w.winner = aux[a * 5 + 4];
  }
  store_world(w, s, a);
}

__global__ void init_kernel(DevState s, KCfg cfg) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= s.n) return;
  for (int k = 0; k < NIF; ++k) I(s, k, a) = 0;
  for (int k = 0; k < NFF; ++k) F(s, k, a) = 0.0f;
  // HockeyEnv.__init__ sets one_starts = True and resets with one_starting=True (hockey_env.py:117,155);
  // hk_create's first reset toggles this 0 -> 1.
  I(s, I_ONE, a) = 0;
  for (int p = 0; p < 2; ++p) {
    const int64_t ga = cfg.arena_offset + a;
    U4 r = philox(cfg.seed, (uint32_t)ga, (uint32_t)(ga >> 32), 0, RNG_PHASE0 + 0x10 * p);
    s.phase[p * s.n + a] = 0.0 + (kPiD - 0.0) * u01d(r.x, r.y);  // BasicOpponent.__init__ U(0, pi)
  }
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
hipError_t upload_scene(const Scene &sc) { return hipMemcpyToSymbol(HIP_SYMBOL(g_scene), &sc, sizeof(Scene)); }

}  // namespace hk
