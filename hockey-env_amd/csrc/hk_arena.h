// hk_arena.h -- one arena per lane, register-resident (v3 of the step kernel).
//
// Reference mapping (hockey/hockey_env.py; Box2D 2.3 for world.Step, restated by the CPU test oracle):
//   presolve()        HockeyEnv.step pre-solve half :659-680 (translation :436-470, boundaries :420-434,
//                     rotation :472-483, puck damping :610-616, hold :618-620, shoot :622-633)
//   world_step()      world.Step(0.02, 180, 60) :682 = Collide -> Solve -> SolveTOI -> ClearForces
//   begin_contact()   ContactDetector.BeginContact :44-76
//   observe*/info*    _get_obs :485-498, obs_agent_two :500-516, _get_info :542-566,
//                     get_info_agent_two :568-591, rewards :518-540
//   basic_opponent()  BasicOpponent.act :787-833
//
// State layout per lane:
//   * the 3 dynamic bodies live in register arrays (Dyn), indexed with compile-time indices or through
//     3-way selects for a runtime body id; static bodies are compile-time scene data (constexpr Scene,
//     and its LDS copy for per-lane ids);
//   * contact state is bitmasks over the 27-pair table (touching / enabled / TOI / island flags);
//   * Box2D manifolds stay in HBM (DevState::man, 64-B records [slot][arena], see man_rec) and are read
//     or written in place where Box2D reads or writes them;
//   * per-pair TOI alphas / sub-step counts and the static bodies' sweep alpha0 live in LDS
//     ([k][64 lanes], conflict-free for any k);
//   * pair loops are uniform across the wave, so scene data arrives through scalar loads.
// Nothing in the step touches private (scratch) memory.  Float operation order is the oracle's.
#pragma once
#include "hk_geom.h"
#include "hk_kernels.h"

namespace hk {

#define SC g_scene
// The scene again, as the step kernel's LDS copy (hk_kernels.hip: g_scene_lds, filled at kernel start).
// Scene data indexed by a per-lane (divergent) pair / fixture / body id is read from here: a ds_read instead
// of a gather through the vector L1 from the code object's constant table.  Compile-time and wave-uniform
// indices keep using SC (instruction literals / scalar loads).
#ifndef SLDS
#define SLDS g_scene_lds
#endif

// register-resident solver slots.  Strong-vs-strong statistics (host build, 2.4M arena-steps): island
// solves with 0/1/2/3/4+ contacts 70.3/29.7/1.5/0.02/3e-4 %, TOI mini-islands with 1/2 contacts
// 99.7/0.3 %.  Larger solves take the HBM slot file (HbmSlots), bit-identically.
constexpr int kIslandC = 4;
constexpr int kToiC = 2;
constexpr int kBigC = kMaxIsland;  // generic solver bound (geometric max is 9)
constexpr uint32_t kEdgeMask[3] = {(1u << 8) | (1u << 10) | (0xFFu << 11),   // player1: 8, 10, 11..18
                                   (1u << 9) | (1u << 10) | (0xFFu << 19),   // player2: 9, 10, 19..26
                                   0x3FFu};                                  // puck: 0..9
constexpr uint32_t kSensorMask = (1u << 6) | (1u << 7);
// pairs that take part in continuous collision: static A, not a sensor (Box2D: a non-bullet dynamic pair
// and sensors never get a TOI)
constexpr uint32_t kToiPairs = 0x7FFFFFFu & ~kSensorMask & ~((1u << 8) | (1u << 9) | (1u << 10));
constexpr uint32_t pair_mask_of_scene(bool toi) {
  uint32_t m = 0u;
  for (int p = 0; p < NP; ++p)
    if (toi ? (!g_scene.sensor[p] && g_scene.pbodyA[p] >= 3) : g_scene.sensor[p] != 0) m |= 1u << p;
  return m;
}
static_assert(pair_mask_of_scene(true) == kToiPairs && pair_mask_of_scene(false) == kSensorMask,
              "pair masks follow the compiled scene's pair table");

// LDS per lane: [0,27) TOI alpha per pair, [27,35) static sweep alpha0, [35,62) TOI sub-step count; then,
// per wave, the work list of the cooperative b2TimeOfImpact drain (toi_drain_wave): kToiQ items of
// kToiItemWords words
constexpr int kLdsToi = 0, kLdsSal0 = 27, kLdsCnt = 35, kLdsPerLane = 62;
constexpr int kToiQ = 128, kToiItemWords = 9;
constexpr int kLdsWords = kLdsPerLane * 64 + kToiQ * kToiItemWords;

struct Dyn {
  float px[3], py[3], qs[3], qc[3];      // transform (origin, rotation)
  float cx[3], cy[3], a[3];              // sweep c, a (COM, angle)
  float c0x[3], c0y[3], a0[3], al0[3];   // sweep c0, a0, alpha0
  float vx[3], vy[3], w[3];
  float fx[3], fy[3], tq[3];
  float ld[3], ad[3], sleep[3];
  int awake[3];
};

struct Arena {
  Dyn d;
  uint32_t touch, enabled, toiflag, cisl, bisl;
  int keep_mode, max_t, time, done, winner, has1, has2, vel_ref;
  int force_big;  // diagnostics: always take the generic (large-island) solver
  int n_toi, overflow, n_big;  // TOI events, island overflow flag, large-island (generic) solves
#ifdef HK_PHASE_TIMERS
  int dg_vit_isl, dg_vit_toi, dg_pit, dg_toi_calls, dg_nc_max;  // diagnostics build: per-lane work
#endif
  float *man;   // HBM manifolds
  float *ws;    // HBM slot workspace of large islands (HbmSlots)
  int64_t n, a;
  float *lds;   // this wave's LDS block
  int lane;
#ifdef HK_TRACE
  float *trace;  // diagnostic build: per-phase snapshots (HK_TRACE_POINT)
#endif
};

// Diagnostic build only (make TRACE=1): snapshot the arena after phase k into io.debug[a][13 + 24k ...].
#ifdef HK_TRACE
constexpr int kTraceStride = 13 + 24 * 4 + 128;
HK_DEV void trace_point(const Arena &w, int k) {
  if (!w.trace) return;
  float *t = w.trace + 13 + 24 * k;
  for (int b = 0; b < 3; ++b) {
    t[6 * b + 0] = w.d.px[b]; t[6 * b + 1] = w.d.py[b]; t[6 * b + 2] = w.d.a[b];
    t[6 * b + 3] = w.d.vx[b]; t[6 * b + 4] = w.d.vy[b]; t[6 * b + 5] = w.d.w[b];
  }
  t[18] = __int_as_float((int)w.touch);
  t[19] = __int_as_float((int)w.enabled);
  t[20] = __int_as_float(w.d.awake[0] | (w.d.awake[1] << 1) | (w.d.awake[2] << 2));
  t[21] = (float)w.n_toi;
  t[22] = (float)w.n_big;
  t[23] = __int_as_float((int)w.cisl);
}
#define HK_TRACE_POINT(w, k) trace_point(w, k)
#define HK_TRACE_SLOT(w, k, s)                                              \
  do {                                                                      \
    if ((w).trace) {                                                        \
      const float *_src = reinterpret_cast<const float *>(&(s));            \
      for (int _q = 0; _q < 64 && _q < (int)(sizeof(s) / 4); ++_q)          \
        (w).trace[13 + 96 + 64 * (k) + _q] = _src[_q];                      \
    }                                                                       \
  } while (0)
#else
#define HK_TRACE_SLOT(w, k, s) ((void)0)
#define HK_TRACE_POINT(w, k) ((void)0)
#endif

// ------------------------------------------------------------------------------------------------
// runtime-id access to the register body file (3-way selects, static -> default)
// ------------------------------------------------------------------------------------------------
// Operands are read into locals first so clang emits straight-line selects (v_cndmask) instead of the
// branch trees it generates for conditional operators over memory operands.
template <typename T>
HK_DEV T pick(const T (&x)[3], int b, T dflt) {
  const T x0 = x[0], x1 = x[1], x2 = x[2];
  T r = dflt;
  r = (b == 2) ? x2 : r;
  r = (b == 1) ? x1 : r;
  r = (b == 0) ? x0 : r;
  return r;
}
template <typename T>
HK_DEV void place(T (&x)[3], int b, T v) {
  const T x0 = x[0], x1 = x[1], x2 = x[2];
  x[0] = (b == 0) ? v : x0;
  x[1] = (b == 1) ? v : x1;
  x[2] = (b == 2) ? v : x2;
}
// Pair sides (build_scene): body A is player 1, player 2 or a static body, never the puck; body B is a
// dynamic body.  The side-specific selects drop the comparisons that can never hold (velocity-loop VALU).
constexpr bool pair_sides_ok() {
  for (int p = 0; p < NP; ++p)
    if (g_scene.pbodyA[p] == B_PK || g_scene.pbodyB[p] > B_PK) return false;
  return true;
}
static_assert(pair_sides_ok(), "pair body A is never the puck, pair body B is always dynamic");
template <typename T>
HK_DEV T pick_a(const T (&x)[3], int b, T dflt) {
  const T x0 = x[0], x1 = x[1];
  T r = (b == 1) ? x1 : dflt;
  r = (b == 0) ? x0 : r;
  return r;
}
template <typename T>
HK_DEV T pick_b(const T (&x)[3], int b) {
  const T x0 = x[0], x1 = x[1], x2 = x[2];
  T r = (b == 1) ? x1 : x2;
  r = (b == 0) ? x0 : r;
  return r;
}
template <typename T>
HK_DEV void place_a(T (&x)[3], int b, T v) {
  const T x0 = x[0], x1 = x[1];
  x[0] = (b == 0) ? v : x0;
  x[1] = (b == 1) ? v : x1;
}
HK_DEV float &LDS(Arena &w, int k) { return w.lds[k * 64 + w.lane]; }
// Box2D manifold record of solid-pair slot `slot` for this arena: [slot][arena][16 words].  A lane's
// record is one 64-B block, so the per-lane (divergent) slot accesses of the near-pair / island / TOI
// queues touch one cache line per record instead of one per field; lanes on the same slot read 4 KiB
// contiguous per wave.  Accesses are whole 16-B quads (global_load/store_dwordx4).
struct alignas(16) Quad { float x, y, z, w; };
HK_DEV Quad *man_rec(const Arena &w, int slot) {
  return reinterpret_cast<Quad *>(w.man + ((int64_t)slot * w.n + w.a) * NMF);
}

// per-lane body id -> dynamic-body constants by select (a static body reads 0)
HK_DEV float inv_mass(int b) { return pick(SC.invMass, b, 0.0f); }
HK_DEV float inv_inertia(int b) { return pick(SC.invI, b, 0.0f); }
HK_DEV v2 local_center(int b) { return V(pick(SC.lcx, b, 0.0f), pick(SC.lcy, b, 0.0f)); }

HK_DEV xform body_xf(const Arena &w, int b) {
  xform x;
  if (b < 3) {
    x.p = V(pick(w.d.px, b, 0.0f), pick(w.d.py, b, 0.0f));
    x.q.s = pick(w.d.qs, b, 0.0f);
    x.q.c = pick(w.d.qc, b, 1.0f);
  } else {
    x.p = V(SLDS.spx[b], SLDS.spy[b]);
    x.q.s = 0.0f;  // rot_set(0) == (+0, 1)
    x.q.c = 1.0f;
  }
  return x;
}
HK_DEV v2 body_c(const Arena &w, int b) {
  return b < 3 ? V(pick(w.d.cx, b, 0.0f), pick(w.d.cy, b, 0.0f)) : V(SLDS.spx[b], SLDS.spy[b]);
}
HK_DEV Sweep body_sweep(Arena &w, int b) {
  Sweep s;
  if (b < 3) {
    s.lc = local_center(b);
    s.c0 = V(pick(w.d.c0x, b, 0.0f), pick(w.d.c0y, b, 0.0f));
    s.c = V(pick(w.d.cx, b, 0.0f), pick(w.d.cy, b, 0.0f));
    s.a0 = pick(w.d.a0, b, 0.0f);
    s.a = pick(w.d.a, b, 0.0f);
    s.alpha0 = pick(w.d.al0, b, 0.0f);
  } else {  // static: c0 == c == origin and a0 == a == 0 forever; only alpha0 moves (b2Sweep::Advance)
    s.lc = V(0.0f, 0.0f);
    s.c0 = s.c = V(SLDS.spx[b], SLDS.spy[b]);
    s.a0 = s.a = 0.0f;
    s.alpha0 = LDS(w, kLdsSal0 + b - 3);
  }
  return s;
}
HK_DEV void body_set_sweep(Arena &w, int b, const Sweep &s) {
  if (b < 3) {
    place(w.d.c0x, b, s.c0.x);
    place(w.d.c0y, b, s.c0.y);
    place(w.d.cx, b, s.c.x);
    place(w.d.cy, b, s.c.y);
    place(w.d.a0, b, s.a0);
    place(w.d.a, b, s.a);
    place(w.d.al0, b, s.alpha0);
  } else {
    LDS(w, kLdsSal0 + b - 3) = s.alpha0;
  }
}
// b2Body::SynchronizeTransform
HK_DEV void sync_xf(Arena &w, int b) {
  if (b >= 3) return;  // a static transform is its origin (c - R(0) * 0 == c exactly)
  const float a = pick(w.d.a, b, 0.0f);
  const rot q = rot_set(a);
  const v2 p = vsub(V(pick(w.d.cx, b, 0.0f), pick(w.d.cy, b, 0.0f)), mul_rv(q, local_center(b)));
  place(w.d.qs, b, q.s);
  place(w.d.qc, b, q.c);
  place(w.d.px, b, p.x);
  place(w.d.py, b, p.y);
}
// b2Body::SetAwake (dynamic bodies only; a static body has no awake state that matters here)
HK_DEV void set_awake(Arena &w, int b, int flag) {
  if (b >= 3) return;
  if (flag) {
    if (!pick(w.d.awake, b, 1)) {
      place(w.d.awake, b, 1);
      place(w.d.sleep, b, 0.0f);
    }
  } else {
    place(w.d.awake, b, 0);
    place(w.d.sleep, b, 0.0f);
    place(w.d.vx, b, 0.0f);
    place(w.d.vy, b, 0.0f);
    place(w.d.w, b, 0.0f);
    place(w.d.fx, b, 0.0f);
    place(w.d.fy, b, 0.0f);
    place(w.d.tq, b, 0.0f);
  }
}
// b2Body::Advance
HK_DEV void body_advance(Arena &w, int b, float alpha) {
  Sweep s = body_sweep(w, b);
  sweep_advance(s, alpha);
  s.c = s.c0;
  s.a = s.a0;
  body_set_sweep(w, b, s);
  sync_xf(w, b);
}

// compile-time body helpers (b2Body setters used by the env laws)
template <int B>
HK_DEV void set_transform(Arena &w, v2 p, float angle) {
  const rot q = rot_set(angle);
  w.d.qs[B] = q.s;
  w.d.qc[B] = q.c;
  w.d.px[B] = p.x;
  w.d.py[B] = p.y;
  xform x;
  x.p = p;
  x.q = q;
  const v2 c = mul_xv(x, V(SC.lcx[B], SC.lcy[B]));
  w.d.cx[B] = c.x;
  w.d.cy[B] = c.y;
  w.d.a[B] = angle;
  w.d.c0x[B] = c.x;
  w.d.c0y[B] = c.y;
  w.d.a0[B] = angle;
}
template <int B>
HK_DEV void wake(Arena &w) {
  if (!w.d.awake[B]) { w.d.awake[B] = 1; w.d.sleep[B] = 0.0f; }
}
template <int B>
HK_DEV void set_linear_velocity(Arena &w, v2 v) {
  if (dot(v, v) > 0.0f) wake<B>(w);
  w.d.vx[B] = v.x;
  w.d.vy[B] = v.y;
}
template <int B>
HK_DEV void set_angular_velocity(Arena &w, float om) {
  if (om * om > 0.0f) wake<B>(w);
  w.d.w[B] = om;
}
template <int B>
HK_DEV void apply_force(Arena &w, v2 f) {
  wake<B>(w);
  w.d.fx[B] = w.d.fx[B] + f.x;
  w.d.fy[B] = w.d.fy[B] + f.y;
}
template <int B>
HK_DEV void apply_torque(Arena &w, float t) {
  wake<B>(w);
  w.d.tq[B] += t;
}

// ------------------------------------------------------------------------------------------------
// lane-local broad phase (exact outcome-preserving rejection)
//   Box2D clipping emits points up to sqrt(2) * totalRadius from the reference polygon: reach = 2 * (rA + rB)
//   for polygon pairs; b2CollidePolygonAndCircle and b2TestOverlap need the core distance within rA + rB;
//   every TOI "touching" exit needs the core distance below target + tol < rA + rB at some t.
// ------------------------------------------------------------------------------------------------
HK_DEV float box_gap(float ax0, float ay0, float ax1, float ay1, const float *b) {
  return fmaxf(fmaxf(b[0] - ax1, ax0 - b[2]), fmaxf(b[1] - ay1, ay0 - b[3]));
}
// Axis-aligned box around a player's core (radius-free polygon) relative to its COM at the rotation q:
// {min x, min y, max x, max y} of R(q) (v_i - lc).  Second stage of the far tests below: the bounding disc
// (rcore) is loose for the elongated racket, and a player parked in front of its own goal otherwise sends
// its goal and goal-side wall pairs to the narrow phase / b2TimeOfImpact every step, where they come out
// separated (oracle statistics: ~90 % of b2TimeOfImpact calls).
HK_DEV void player_core_box(const Arena &w, int f, int b, float q_s, float q_c, float (&e)[4],
                            const Scene &S = SC) {
  e[0] = e[1] = kFltMax;
  e[2] = e[3] = -kFltMax;
#pragma unroll
  for (int k = 0; k < kMaxPolyVerts; ++k) {
    if (k < S.fx[f].count) {
      const float ux = S.fx[f].vx[k] - S.lcx[b], uy = S.fx[f].vy[k] - S.lcy[b];
      const float rx = q_c * ux - q_s * uy, ry = q_s * ux + q_c * uy;
      e[0] = fminf(e[0], rx); e[1] = fminf(e[1], ry);
      e[2] = fmaxf(e[2], rx); e[3] = fmaxf(e[3], ry);
    }
  }
}
// both players' core boxes at their current rotations, computed once per pass over the pair table
struct CoreBoxes {
  float e[2][4];
};
HK_DEV void core_boxes(const Arena &w, CoreBoxes &cb) {
  player_core_box(w, F_P1, B_P1, w.d.qs[B_P1], w.d.qc[B_P1], cb.e[0]);
  player_core_box(w, F_P2, B_P2, w.d.qs[B_P2], w.d.qc[B_P2], cb.e[1]);
}
HK_DEV bool static_far_collide(const Scene &S, int fA, int bB, v2 cB, const float (&e)[4], float reach) {
  return box_gap(cB.x + e[0], cB.y + e[1], cB.x + e[2], cB.y + e[3], S.fx_aabb[fA]) > reach;
}
// cb: the players' core boxes when the caller has them (pair-table passes), else computed here
// S: SC for a wave-uniform p (pair-table loops), SLDS for a per-lane p
HK_DEV bool pair_far_collide(const Arena &w, int p, const CoreBoxes *cb = nullptr, const Scene &S = SC) {
  const int fA = S.pairA[p], fB = S.pairB[p], bA = S.pbodyA[p], bB = S.pbodyB[p];
  // A polygon-circle manifold (and a sensor overlap) needs the circle centre within the total radius of
  // the polygon core, so a circle pair is far beyond total + rounding margin; polygon pairs keep the
  // clipping bound 2 * total (+ kFarMargin).
  const float total = S.fx[fA].radius + S.fx[fB].radius;
  const float reach = S.fx[fB].circle ? total + kToiMargin : 2.0f * total + kFarMargin;
  const v2 cB = body_c(w, bB);
  const float rB = S.rcore[bB];
  if (bA >= 3) {
    if (box_gap(cB.x - rB, cB.y - rB, cB.x + rB, cB.y + rB, S.fx_aabb[fA]) > reach) return true;
    if (bB == B_PK) return false;  // a circle's core is its centre: the disc test is already exact
    if (cb) return static_far_collide(S, fA, bB, cB, cb->e[bB == B_P2 ? 1 : 0], reach);
    float e[4];
    player_core_box(w, fB, bB, pick(w.d.qs, bB, 0.0f), pick(w.d.qc, bB, 1.0f), e, S);
    return static_far_collide(S, fA, bB, cB, e, reach);
  }
  const v2 cA = body_c(w, bA);
  const float lim = S.rcore[bA] + rB + reach;
  const float dx = cA.x - cB.x, dy = cA.y - cB.y;
  return dx * dx + dy * dy > lim * lim;
}
// b2TimeOfImpact can only report TOUCHING when the GJK core distance falls below target + tolerance at
// some t.  B's core stays within rcore of its COM, which moves on the segment c0 -> c, so the box gap between
// that swept disc's AABB and A's core AABB bounds the core distance from below: a gap above target +
// tolerance (+ kToiMargin) means alpha = 1 exactly, without running the iteration.
// For a player the second stage bounds its core by the exact box at the end-of-sweep rotation q = rot(a)
// (the transform is synchronised with the sweep whenever the scan runs), widened by rcore * |a - a0|:
// a core point moves at most that far as the angle runs over [a0, a].
// S: SC for a wave-uniform p (first scan pass), SLDS for a per-lane p (later passes)
HK_DEV bool pair_far_toi(const Arena &w, int p, const CoreBoxes &cb, const Scene &S = SC) {  // static A, dynamic B
  const int fA = S.pairA[p], fB = S.pairB[p], bB = S.pbodyB[p];
  // b2TimeOfImpact returns TOUCHING only at a t where the core distance (GJK, or a separation function
  // bounded below by it) is under target + tolerance, target = max(linearSlop, rA + rB - 3 linearSlop),
  // tolerance = linearSlop / 4; every other outcome maps to alpha 1.  A lower bound on the distance above
  // that threshold (+ kToiMargin for rounding) therefore gives alpha 1 exactly.
  const float total = S.fx[fA].radius + S.fx[fB].radius;
  const float reach = fmaxf(kLinearSlop, total - 3.0f * kLinearSlop) + 0.25f * kLinearSlop + kToiMargin;
  const float r = S.rcore[bB];
  const float c0x = pick(w.d.c0x, bB, 0.0f), c0y = pick(w.d.c0y, bB, 0.0f);
  const float cx = pick(w.d.cx, bB, 0.0f), cy = pick(w.d.cy, bB, 0.0f);
  const float lx = fminf(c0x, cx), ly = fminf(c0y, cy), hx = fmaxf(c0x, cx), hy = fmaxf(c0y, cy);
  if (box_gap(lx - r, ly - r, hx + r, hy + r, S.fx_aabb[fA]) > reach) return true;
  if (bB == B_PK) return false;  // circle: exact already
  const float(&e)[4] = cb.e[bB == B_P2 ? 1 : 0];
  const float rot = r * fabsf(pick(w.d.a, bB, 0.0f) - pick(w.d.a0, bB, 0.0f));
  return box_gap(lx + e[0] - rot, ly + e[1] - rot, hx + e[2] + rot, hy + e[3] + rot, S.fx_aabb[fA]) > reach;
}

// First-pass bulk settlement of the TOI scan (solve_toi).  A dynamic body whose swept core box lies inside its
// interior rectangle is farther than the TOI reach from each of its static fixtures (walls bound the
// rectangle in y, posts and goals in x), so pair_far_toi holds for all of its TOI pairs.  The rectangles are
// compile-time (1 mm inside the exact bound); the static_asserts re-check every fixture against them.
struct Rect { float x0, y0, x1, y1; };
constexpr float cmax(float a, float b) { return a > b ? a : b; }
constexpr float cmin(float a, float b) { return a < b ? a : b; }
constexpr float toi_reach(int fB) {
  const float total = g_scene.fx[F_WT].radius + g_scene.fx[fB].radius;
  return cmax(kLinearSlop, total - 3.0f * kLinearSlop) + 0.25f * kLinearSlop + kToiMargin;
}
constexpr Rect interior_rect(int fB, bool goals) {
  const float e = toi_reach(fB) + 1e-3f;
  float xl = cmax(g_scene.fx_aabb[F_PLT][2], g_scene.fx_aabb[F_PLB][2]);
  float xr = cmin(g_scene.fx_aabb[F_PRT][0], g_scene.fx_aabb[F_PRB][0]);
  if (goals) {
    xl = cmax(xl, g_scene.fx_aabb[F_G1][2]);
    xr = cmin(xr, g_scene.fx_aabb[F_G2][0]);
  }
  return Rect{xl + e, g_scene.fx_aabb[F_WB][3] + e, xr - e, g_scene.fx_aabb[F_WT][1] - e};
}
constexpr Rect kInteriorPuck = interior_rect(F_PK, false), kInteriorPlayer = interior_rect(F_P1, true);
constexpr bool rect_clear(const Rect &r, int f, float reach) {
  const float *b = g_scene.fx_aabb[f];
  return cmax(cmax(b[0] - r.x1, r.x0 - b[2]), cmax(b[1] - r.y1, r.y0 - b[3])) > reach;
}
constexpr bool interior_ok() {
  const int fs[8] = {F_WT, F_WB, F_PLT, F_PLB, F_PRT, F_PRB, F_G1, F_G2};
  bool ok = g_scene.fx[F_P1].radius == g_scene.fx[F_P2].radius;
  for (int k = 0; k < 8; ++k) ok = ok && rect_clear(kInteriorPlayer, fs[k], toi_reach(F_P1));
  for (int k = 0; k < 6; ++k) ok = ok && rect_clear(kInteriorPuck, fs[k], toi_reach(F_PK));
  for (int p = 0; p < NP; ++p)  // the puck's TOI pairs are 0..5, the players' their static pairs (kEdgeMask)
    if ((kToiPairs >> p) & 1u) {
      const int f = g_scene.pairA[p];
      const bool known = f == F_WT || f == F_WB || f == F_PLT || f == F_PLB || f == F_PRT || f == F_PRB ||
                         (g_scene.pbodyB[p] != B_PK && (f == F_G1 || f == F_G2));
      ok = ok && known;
    }
  return ok;
}
static_assert(interior_ok(), "interior rectangles clear every static fixture of a TOI pair by the TOI reach");
HK_DEV bool inside(const Rect &r, float lx, float ly, float hx, float hy) {
  return lx > r.x0 && ly > r.y0 && hx < r.x1 && hy < r.y1;
}

// ------------------------------------------------------------------------------------------------
// ContactDetector.BeginContact (hockey_env.py:44-76) and b2Contact::Update
// ------------------------------------------------------------------------------------------------
HK_DEV void begin_contact(Arena &w, int p) {  // per-lane p
  const int bA = SLDS.pbodyA[p], bB = SLDS.pbodyB[p];
  const int hasPK = (bA == B_PK || bB == B_PK);
  if ((bA == B_G2 || bB == B_G2) && hasPK) { w.done = 1; w.winner = 1; }
  if ((bA == B_G1 || bB == B_G1) && hasPK) { w.done = 1; w.winner = -1; }
  if ((bA == B_P1 || bB == B_P1) && hasPK) {
    if (w.keep_mode && (double)w.d.vx[B_PK] < 0.1)
      if (w.has1 == 0) w.has1 = 15;
  }
  if ((bA == B_P2 || bB == B_P2) && hasPK) {
    if (w.keep_mode && (double)w.d.vx[B_PK] > -0.1)
      if (w.has2 == 0) w.has2 = 15;
  }
}

// Narrow phase of pair p for the arena whose manifold records start at `man` (arena index a of n): the
// manifold from the two fixtures' transforms, the impulse carry-over from the stored manifold (ids matched,
// meaningful only if the pair was touching), and the whole-record write when touching.  Returns touching.
// Reads only its arguments, the scene and the pair's own record, so any lane may run it for any arena.
HK_DEV int narrow_phase(float *man, int64_t n, int64_t a, int p, int was, const xform &xA, const xform &xB) {
  const int fA = SLDS.pairA[p], fB = SLDS.pairB[p], bA = SLDS.pbodyA[p];
  // the stored manifold (ids / impulses) of a touching pair is requested before the narrow phase so its
  // HBM / L2 latency overlaps the clipping arithmetic
  const int slot = SLDS.manslot[p];
  Quad *rec = reinterpret_cast<Quad *>(man + ((int64_t)(slot < 0 ? 0 : slot) * n + a) * NMF);
  Quad o0 = Quad{0.0f, 0.0f, 0.0f, 0.0f}, o2 = o0, o3 = o0;
  if (slot >= 0 && was) {
    o0 = rec[0];
    o2 = rec[2];
    o3 = rec[3];
  }
  if (SLDS.sensor[p]) return test_overlap(SLDS.fx[fA], xA, SLDS.fx[fB], xB);
  Manifold m;
  if (SLDS.fx[fB].circle) {  // puck: A is a static quad or a player
    const RFix<1> cB = load_fix<1>(SLDS.fx[fB]);
    if (bA >= 3) collide_poly_circle(m, load_fix<kStaticVerts>(SLDS.fx[fA]), xA, cB, xB);
    else collide_poly_circle(m, load_fix<kMaxPolyVerts>(SLDS.fx[fA]), xA, cB, xB);
  } else {  // player B: A is a static quad or the other player
    const RFix<kMaxPolyVerts> pB = load_fix<kMaxPolyVerts>(SLDS.fx[fB]);
    if (bA >= 3) collide_polygons(m, load_fix<kStaticVerts>(SLDS.fx[fA]), xA, pB, xB);
    else collide_polygons(m, load_fix<kMaxPolyVerts>(SLDS.fx[fA]), xA, pB, xB);
  }
  const int touching = m.count > 0;
  if (touching) {
    // match old contact ids to carry impulses (the stored manifold is meaningful only if touching)
    int oc = 0;
    uint32_t oid0 = 0u, oid1 = 0u;
    float oni0 = 0.0f, oni1 = 0.0f, oti0 = 0.0f, oti1 = 0.0f;
    if (was) {
      oc = __float_as_int(o0.x) & 0xff;
      oid0 = (uint32_t)__float_as_int(o2.y);
      oid1 = (uint32_t)__float_as_int(o2.z);
      oni0 = o3.x;
      oti0 = o3.y;
      oni1 = o3.z;
      oti1 = o3.w;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i < m.count) {
        m.ni[i] = 0.0f;
        m.ti[i] = 0.0f;
        if (oc > 0 && oid0 == m.id[i]) { m.ni[i] = oni0; m.ti[i] = oti0; }
        else if (oc > 1 && oid1 == m.id[i]) { m.ni[i] = oni1; m.ti[i] = oti1; }
      }
    }
    // whole-record write; a one-point manifold's point-1 words are zeroed (every reader is bounded by
    // the point count, as in Box2D)
    const bool two = m.count > 1;
    rec[0] = Quad{__int_as_float(m.count | (m.type << 8)), m.ln.x, m.ln.y, m.lp.x};
    rec[1] = Quad{m.lp.y, m.pt_lp[0].x, m.pt_lp[0].y, two ? m.pt_lp[1].x : 0.0f};
    rec[2] = Quad{two ? m.pt_lp[1].y : 0.0f, __int_as_float((int)m.id[0]), two ? __int_as_float((int)m.id[1]) : 0,
                  0.0f};
    rec[3] = Quad{m.ni[0], m.ti[0], two ? m.ni[1] : 0.0f, two ? m.ti[1] : 0.0f};
  }
  return touching;
}

// b2Contact::Update bookkeeping of pair p once its narrow phase has run: enable, wake-ups on a touching
// change (solid pairs), the touching bit and BeginContact -- the order-dependent side effects, applied by the
// owner lane in pair order.
HK_DEV void pair_update_apply(Arena &w, int p, int touching) {
  const uint32_t bit = 1u << p;
  const int was = (w.touch & bit) != 0u;
  w.enabled |= bit;
  if (!SLDS.sensor[p] && touching != was) { set_awake(w, SLDS.pbodyA[p], 1); set_awake(w, SLDS.pbodyB[p], 1); }
  w.touch = touching ? (w.touch | bit) : (w.touch & ~bit);
  if (!was && touching) begin_contact(w, p);
}

// b2Contact::Update for a pair the broad phase could not reject: narrow phase, impulse carry-over,
// wake-ups and BeginContact.
HK_DEV void pair_update_near(Arena &w, int p) {
  const int was = (w.touch & (1u << p)) != 0u;
  const int touching = narrow_phase(w.man, w.n, w.a, p, was, body_xf(w, SLDS.pbodyA[p]), body_xf(w, SLDS.pbodyB[p]));
  pair_update_apply(w, p, touching);
}

// b2Contact::Update for a pair the broad phase rejects: not touching (no manifold, no BeginContact)
HK_DEV void pair_update_far(Arena &w, int p, const Scene &S = SC) {
  const uint32_t bit = 1u << p;
  const int was = (w.touch & bit) != 0u;
  w.enabled |= bit;
  if (!S.sensor[p] && was) { set_awake(w, S.pbodyA[p], 1); set_awake(w, S.pbodyB[p], 1); }
  w.touch &= ~bit;
}

HK_DEV void pair_update(Arena &w, int p) {  // per-lane p (TOI events)
  if (pair_far_collide(w, p, nullptr, SLDS)) pair_update_far(w, p, SLDS);
  else pair_update_near(w, p);
}

// The near pairs' narrow phases of the whole wave, dealt out over all its lanes (device build; every lane of
// the wave that runs the step calls it).  Per lane, `near` holds the pairs whose narrow phase must run.  With
// every dynamic body awake the narrow phases of one lane are independent of each other (transforms do not
// change during Collide, wake-ups of awake bodies are no-ops, BeginContact touches no narrow-phase input), so
// they may run anywhere and in any order: each (lane, pair) goes to an LDS work list with the pair's two body
// transforms, a worker lane runs narrow_phase for the owner's arena (reading and writing the owner's manifold
// record in HBM) and leaves `touching` in the owner's LDS row; the owner then applies the order-dependent
// bookkeeping in pair order.  A lane with k near pairs no longer holds the wave for k narrow phases.
HK_DEV void collide_near_wave(Arena &w, uint32_t near) {
#if defined(__HIP_DEVICE_COMPILE__)
  float *q = w.lds + kLdsPerLane * 64;
  const uint64_t lt = (1ull << w.lane) - 1ull;
  const int64_t a0 = w.a - w.lane;  // arena of lane 0 of this wave
  while (wave_any(near != 0u)) {
    const int cnt = __popc(near);
    int off = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const uint64_t m = __ballot((cnt >> b) & 1);
      off += __popcll(m & lt) << b;
      total += __popcll(m) << b;
    }
    uint32_t listed = 0u;
    for (uint32_t m = near; m && off < kToiQ; m &= m - 1u, ++off) {
      const int p = __ffs(m) - 1;
      const xform xA = body_xf(w, SLDS.pbodyA[p]), xB = body_xf(w, SLDS.pbodyB[p]);
      const int was = (w.touch >> p) & 1u;
      float *it = q + off * kToiItemWords;
      it[0] = __int_as_float(p | (w.lane << 8) | (was << 16));
      it[1] = xA.p.x;
      it[2] = xA.p.y;
      it[3] = xA.q.s;
      it[4] = xA.q.c;
      it[5] = xB.p.x;
      it[6] = xB.p.y;
      it[7] = xB.q.s;
      it[8] = xB.q.c;
      listed |= m & (0u - m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n = total < kToiQ ? total : kToiQ;
    const uint64_t act = __ballot(1);  // workers: the wave's active lanes (see toi_drain_wave)
    const int rank = __popcll(act & lt), nact = __popcll(act);
    for (int k = rank; k < n; k += nact) {
      const float *it = q + k * kToiItemWords;
      const int tag = __float_as_int(it[0]), p = tag & 255, owner = (tag >> 8) & 255, was = (tag >> 16) & 1;
      xform xA, xB;
      xA.p = V(it[1], it[2]);
      xA.q.s = it[3];
      xA.q.c = it[4];
      xB.p = V(it[5], it[6]);
      xB.q.s = it[7];
      xB.q.c = it[8];
      const int touching = narrow_phase(w.man, w.n, a0 + owner, p, was, xA, xB);
      w.lds[(kLdsToi + p) * 64 + owner] = touching ? 1.0f : 0.0f;  // the TOI cache row is free until SolveTOI
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    near &= ~listed;
    for (uint32_t m = listed; m; m &= m - 1u) {  // pair order
      const int p = __ffs(m) - 1;
      pair_update_apply(w, p, LDS(w, kLdsToi + p) != 0.0f);
    }
  }
#else  // host build (one lane at a time): the lane's own queue in pair order
  while (near) {
    const int p = __ffs(near) - 1;
    near &= near - 1u;
    pair_update_near(w, p);
  }
#endif
}

// b2ContactManager::Collide.  With every dynamic body awake (the normal state of play: no arena-step of a
// strong-vs-strong run has a sleeping body) the pair order only matters among pairs that can touch
// (wake-ups are no-ops, far pairs fire no BeginContact), so the far pairs are settled first and the near
// pairs' narrow phases are dealt out over the wave (collide_near_wave).  A lane with a sleeping body takes
// Box2D's sequential loop afterwards.
HK_DEV void collide(Arena &w) {
  const bool fast = w.d.awake[0] && w.d.awake[1] && w.d.awake[2];
  uint32_t near = 0u;
  if (fast) {
    CoreBoxes cb;
    core_boxes(w, cb);
#pragma unroll
    for (int p = 0; p < NP; ++p) {  // uniform loop, unrolled: the scene data are literals
      if (pair_far_collide(w, p, &cb)) pair_update_far(w, p);
      else near |= 1u << p;
    }
  }
  collide_near_wave(w, near);  // every lane (a lane on the sequential path contributes worker capacity)
  if (fast) return;
  for (int p = 0; p < NP; ++p) {
    const int bA = SC.pbodyA[p], bB = SC.pbodyB[p];
    const int activeA = bA < 3 && pick(w.d.awake, bA, 0);
    const int activeB = pick(w.d.awake, bB, 0);
    if (!activeA && !activeB) continue;
    pair_update(w, p);
  }
}

}  // namespace hk

#include "hk_solver.h"

namespace hk {

// ------------------------------------------------------------------------------------------------
// b2World::Solve: islands by DFS (Box2D's seed order and edge order), solved together (they share no
// dynamic body), position early exit and sleep per island.
// ------------------------------------------------------------------------------------------------
template <typename SL>
HK_DEV bool solve_islands(Arena &w, SL &S, float dt, PhaseT &T) {
  constexpr int MAXS = SlotCap<SL>::value;
  const float h = dt;
  int island_of[3] = {-1, -1, -1};
  int nc = 0, nisl = 0;
  uint32_t inis = 0u;
  const uint32_t live = w.enabled & w.touch & ~kSensorMask;
  const int seed_order[3] = {B_PK, B_P2, B_P1};
#pragma unroll
  for (int si = 0; si < 3; ++si) {
    const int seed = seed_order[si];
    if (island_of[seed] >= 0 || !w.d.awake[seed]) continue;
    const int isl = nisl++;
    int st0 = seed, st1 = 0, st2 = 0, sc = 1;  // DFS stack of dynamic bodies (statics never propagate)
    island_of[seed] = isl;
    while (sc > 0) {
      const int bi = sc == 3 ? st2 : (sc == 2 ? st1 : st0);
      --sc;
      set_awake(w, bi, 1);
      uint32_t m = pick(kEdgeMask, bi, 0u) & live & ~inis;
      while (m) {
        const int e = __ffs(m) - 1;
        m &= m - 1u;
        inis |= 1u << e;
        S.set_pair(nc, e, isl);
        ++nc;
        const int pa = SLDS.pbodyA[e], pb = SLDS.pbodyB[e];
        const int other = pa == bi ? pb : pa;
        if (other >= 3) continue;
        if (pick(island_of, other, 0) >= 0) continue;
        place(island_of, other, isl);
        if (sc == 0) st0 = other; else if (sc == 1) st1 = other; else st2 = other;
        ++sc;
      }
    }
  }
  if (nc > MAXS) return false;
  // integrate velocities (b2Island::Solve), in place in the register body file
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    if (island_of[b] >= 0) {
      w.d.c0x[b] = w.d.cx[b];
      w.d.c0y[b] = w.d.cy[b];
      w.d.a0[b] = w.d.a[b];
      v2 v = V(w.d.vx[b], w.d.vy[b]);
      float wv = w.d.w[b];
      v = vadd(v, vs(h, vadd(vs(1.0f, V(0.0f, 0.0f)), vs(SC.invMass[b], V(w.d.fx[b], w.d.fy[b])))));
      wv += h * SC.invI[b] * w.d.tq[b];
      v = vs(1.0f / (1.0f + h * w.d.ld[b]), v);
      wv *= 1.0f / (1.0f + h * w.d.ad[b]);
      w.d.vx[b] = v.x;
      w.d.vy[b] = v.y;
      w.d.w[b] = wv;
    }
  }
  HK_TRACE_POINT(w, 3);
  S.each(nc, [&](FSlot &s, int) {
    fslot_load(s, w, fs_pair(s), 1, fs_isl(s));
    fslot_init_velocity(s, w);
  });
  S.each(nc, [&](FSlot &s, int) { fslot_warm_start(s, w.d); });
  HK_TIC(T, 2);  // diagnostics: island setup (DFS, integrate, constraint init, warm start)
  const int vit = velocity_iterations(S, w.d, nc, island_of, T);
  HK_TIC(T, 3);  // diagnostics: velocity iterations
#ifdef HK_PHASE_TIMERS
  w.dg_vit_isl += vit;
  w.dg_nc_max = nc > w.dg_nc_max ? nc : w.dg_nc_max;
#endif
  (void)vit;
  S.each(nc, [&](FSlot &s, int) { fslot_store(s, w); });
#pragma unroll
  for (int b = 0; b < 3; ++b)
    if (island_of[b] >= 0) integrate_one(h, w.d, b);
  int solved = 0;
  const int all = (1 << nisl) - 1;
  S.load_geo(nc, w);
  for (int it = 0; it < kPosIters && (solved & all) != all; ++it) {
    HK_MARK(pos_begin);
    float ms0 = 0.0f, ms1 = 0.0f, ms2 = 0.0f;
    S.each(nc, [&](FSlot &s, int i) {
      const int isl = fs_isl(s);
      if (!((solved >> isl) & 1)) {
        const float m = fslot_solve_position(s, w, kBaumgarte, 0.0f, S.geo(i, s, w));
        ms0 = isl == 0 ? fmin2(ms0, m) : ms0;
        ms1 = isl == 1 ? fmin2(ms1, m) : ms1;
        ms2 = isl == 2 ? fmin2(ms2, m) : ms2;
      }
    });
#ifdef HK_PHASE_TIMERS
    w.dg_pit++;
#endif
    if (ms0 >= -3.0f * kLinearSlop) solved |= 1;
    if (ms1 >= -3.0f * kLinearSlop) solved |= 2;
    if (ms2 >= -3.0f * kLinearSlop) solved |= 4;
    HK_MARK(pos_end);
  }
#pragma unroll
  for (int b = 0; b < 3; ++b)
    if (island_of[b] >= 0) sync_xf(w, b);
  const float linTolSqr = kLinearSleepTol * kLinearSleepTol;
  const float angTolSqr = kAngularSleepTol * kAngularSleepTol;
  for (int isl = 0; isl < nisl; ++isl) {
    float minSleep = kFltMax;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      if (island_of[b] == isl) {
        if (w.d.w[b] * w.d.w[b] > angTolSqr || w.d.vx[b] * w.d.vx[b] + w.d.vy[b] * w.d.vy[b] > linTolSqr) {
          w.d.sleep[b] = 0.0f;
          minSleep = 0.0f;
        } else {
          w.d.sleep[b] += h;
          minSleep = fmin2(minSleep, w.d.sleep[b]);
        }
      }
    }
    if (minSleep >= kTimeToSleep && ((solved >> isl) & 1)) {
#pragma unroll
      for (int b = 0; b < 3; ++b)
        if (island_of[b] == isl) set_awake(w, b, 0);
    }
  }
  return true;
}

// ------------------------------------------------------------------------------------------------
// b2World::SolveTOI.  In this scene a TOI pair is always (static A, dynamic B), so the mini-island
// holds exactly one dynamic body: B plus its touching static contacts (minContact first, then B's
// contact edges in order).  Mass gating of SolveTOIPositionConstraints is therefore the identity.
// ------------------------------------------------------------------------------------------------
template <typename SL>
HK_DEV void toi_island_solve(Arena &w, SL &S, int minc, uint32_t extra, int nc, int db, float sub_dt, PhaseT &T) {
  uint32_t m = extra;
  S.each(nc, [&](FSlot &s, int i) {
    int p = minc;
    if (i > 0) { p = __ffs(m) - 1; m &= m - 1u; }
    fslot_load(s, w, p, 0, 0);
  });
  for (int it = 0; it < 20; ++it) {
    float minSep = 0.0f;
    S.each(nc, [&](FSlot &s, int i) {
      // geometry re-read per pass here: caching it in the slot file miscompiles on gfx950 in this loop
      // (ROCm 7.2; caught by the GPU lockstep tests), and TOI position passes are few
      minSep = fslot_solve_position(s, w, kToiBaumgarte, minSep, man_geo(w, fs_pair(s)));
    });
    if (minSep >= -1.5f * kLinearSlop) break;
  }
  HK_TIC(T, 10);  // diagnostics: TOI position passes
  // leap of faith (the static body's c0 already equals its c)
  place(w.d.c0x, db, pick(w.d.cx, db, 0.0f));
  place(w.d.c0y, db, pick(w.d.cy, db, 0.0f));
  place(w.d.a0, db, pick(w.d.a, db, 0.0f));
  S.each(nc, [&](FSlot &s, int) { fslot_init_velocity(s, w); });
  const int isl_of[3] = {db == 0 ? 0 : -1, db == 1 ? 0 : -1, db == 2 ? 0 : -1};  // one island: B
  const int vit = velocity_iterations(S, w.d, nc, isl_of, T);
  HK_TIC(T, 11);  // diagnostics: TOI velocity iterations
#ifdef HK_PHASE_TIMERS
  w.dg_vit_toi += vit;
#endif
  (void)vit;
#pragma unroll
  for (int b = 0; b < 3; ++b)
    if (b == db) integrate_one(sub_dt, w.d, b);
  sync_xf(w, db);
}

// b2TimeOfImpact of static-vs-dynamic pair p from the two sweeps -> alpha in the step's [alpha0, 1] frame
// (sB.alpha0 == max(alpha0 A, alpha0 B) after alignment)
HK_DEV float toi_pair_sweeps(int p, const Sweep &sA, const Sweep &sB) {
  const Proxy<kStaticVerts, true> pA = make_proxy<kStaticVerts, true>(SLDS.fx[SLDS.pairA[p]]);
  const Proxy<kMaxPolyVerts> pB = make_proxy<kMaxPolyVerts>(SLDS.fx[SLDS.pairB[p]]);
  float beta;
  const int st = time_of_impact(pA, pB, sA, sB, 1.0f, beta);
  return st == TOI_TOUCHING ? fmin2(sB.alpha0 + (1.0f - sB.alpha0) * beta, 1.0f) : 1.0f;
}
// per-lane pair p of this lane's arena
HK_DEV float toi_pair(Arena &w, int p) {
#ifdef HK_PHASE_TIMERS
  w.dg_toi_calls++;
#endif
  return toi_pair_sweeps(p, body_sweep(w, SLDS.pbodyA[p]), body_sweep(w, SLDS.pbodyB[p]));
}
// runs the lane's queued b2TimeOfImpact calls in pair order; `below` tracks the pairs whose cached alpha is
// below 1 (the only ones the minimum selection can pick: it starts at 1 and compares strictly)
HK_DEV void toi_drain(Arena &w, uint32_t &pending, uint32_t &below) {
  while (pending) {
    const int p = __ffs(pending) - 1;
    pending &= pending - 1u;
    float alpha = toi_pair(w, p);
    LDS(w, kLdsToi + p) = alpha;
    below = alpha < 1.0f ? (below | (1u << p)) : (below & ~(1u << p));
  }
}

// Cooperative drain (device build; every lane of the wave that runs the step calls it, with or without queued
// pairs).  A per-lane queue holds the wave for as many rounds as its longest queue; here the wave's queued
// (lane, pair) calls are listed in LDS -- pair id, owner lane and the two sweeps' inputs, copied at this point
// -- and dealt out to all lanes, so a lane with k queued pairs no longer costs k rounds.  A worker writes alpha
// into the owner's TOI cache slot; the owner then updates `below`.  The calls are independent (each reads only
// its own pair's sweeps, which nothing changes until the drain is over), and a worker runs the same arithmetic
// on the same inputs as the owner would: bit-identical alphas.  The host build (one lane at a time) drains per
// lane.
HK_DEV void toi_drain_wave(Arena &w, uint32_t &pending, uint32_t &below) {
#if defined(__HIP_DEVICE_COMPILE__)
  float *q = w.lds + kLdsPerLane * 64;
  const uint64_t lt = (1ull << w.lane) - 1ull;  // lanes below this one
  while (wave_any(pending != 0u)) {
    // exclusive prefix sum of the lanes' queue lengths (<= 27: five bit-planes of ballots)
    const int cnt = __popc(pending);
    int off = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 5; ++b) {
      const uint64_t m = __ballot((cnt >> b) & 1);
      off += __popcll(m & lt) << b;
      total += __popcll(m) << b;
    }
    uint32_t listed = 0u;
    for (uint32_t m = pending; m && off < kToiQ; m &= m - 1u, ++off) {
      const int p = __ffs(m) - 1;
      const Sweep sB = body_sweep(w, SLDS.pbodyB[p]);
      float *it = q + off * kToiItemWords;
      it[0] = __int_as_float(p | (w.lane << 8));
      it[1] = sB.c0.x;
      it[2] = sB.c0.y;
      it[3] = sB.c.x;
      it[4] = sB.c.y;
      it[5] = sB.a0;
      it[6] = sB.a;
      it[7] = sB.alpha0;
      it[8] = LDS(w, kLdsSal0 + SLDS.pbodyA[p] - 3);  // the static body's alpha0
      listed |= m & (0u - m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int n = total < kToiQ ? total : kToiQ;
    // the workers are the wave's ACTIVE lanes (a partial last wave, or a single-arena context, has fewer
    // than 64): active lane r takes items r, r + nact, ...
    const uint64_t act = __ballot(1);
    const int rank = __popcll(act & lt), nact = __popcll(act);
    for (int k = rank; k < n; k += nact) {
      const float *it = q + k * kToiItemWords;
      const int tag = __float_as_int(it[0]), p = tag & 255, owner = tag >> 8;
      const int bA = SLDS.pbodyA[p], bB = SLDS.pbodyB[p];
      Sweep sA, sB;
      sA.lc = V(0.0f, 0.0f);
      sA.c0 = sA.c = V(SLDS.spx[bA], SLDS.spy[bA]);
      sA.a0 = sA.a = 0.0f;
      sA.alpha0 = it[8];
      sB.lc = local_center(bB);
      sB.c0 = V(it[1], it[2]);
      sB.c = V(it[3], it[4]);
      sB.a0 = it[5];
      sB.a = it[6];
      sB.alpha0 = it[7];
      w.lds[(kLdsToi + p) * 64 + owner] = toi_pair_sweeps(p, sA, sB);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifdef HK_PHASE_TIMERS
    w.dg_toi_calls += __popc(listed);
#endif
    pending &= ~listed;
    for (uint32_t m = listed; m; m &= m - 1u) {
      const int p = __ffs(m) - 1;
      const float alpha = LDS(w, kLdsToi + p);
      below = alpha < 1.0f ? (below | (1u << p)) : (below & ~(1u << p));
    }
  }
#else
  toi_drain(w, pending, below);
#endif
}

HK_DEV void solve_toi(Arena &w, float dt, PhaseT &T) {
#pragma unroll
  for (int b = 0; b < 3; ++b) w.d.al0[b] = 0.0f;
  for (int k = 0; k < 8; ++k) LDS(w, kLdsSal0 + k) = 0.0f;
  for (int p = 0; p < NP; ++p) LDS(w, kLdsCnt + p) = 0.0f;  // TOI alphas: only read below 1 (`below`)
  w.toiflag = 0u;
  w.cisl = 0u;
  w.bisl = 0u;
  uint32_t below = 0u;      // pairs whose cached TOI alpha (LDS) is < 1
  uint32_t exhausted = 0u;  // pairs past b2_maxSubSteps TOI events this step (toi_count > 8, kept in LDS)
  uint32_t redo = 0u;       // pairs a later scan pass must visit: the last event's body's contacts
  bool first = true;
  // The lanes stay together in this loop until every lane is done (`act`), so that the b2TimeOfImpact calls
  // of step (2) can be dealt out over the whole wave (toi_drain_wave).  A lane that is done only contributes
  // worker capacity.
  bool act = true;
  while (wave_any(act)) {
    HK_TIC(T, 5);  // diagnostics: events / min selection -> "toi-events"
    uint32_t elig = 0u, pending = 0u;
    if (act) {
      // (1) In pair order: eligibility, sweep alignment (the only order-dependent side effect) and the cheap
      //     far rejection.  Pairs that need a real b2TimeOfImpact are queued.  During a step the alignment
      //     only ever advances a STATIC body's alpha0 (TOI events come in non-decreasing alpha, and only the
      //     moved body's pairs are re-evaluated, so a0(static) <= a0(dynamic) for them); the queued TOIs
      //     therefore see exactly the sweeps the sequential scan would.  Should a dynamic body ever be
      //     advanced here, its lane first drains its queue so the sequential order is kept regardless.
      CoreBoxes cb;  // the players' poses are fixed during the pass (only sweep starts move)
      core_boxes(w, cb);
      uint32_t todo;
      if (first) {
        uint32_t settled = 0u;
        // The first pass has no order-dependent side effect (every alpha0 is still 0, so the alignment is a
        // no-op): the TOI pairs of a body inside its interior rectangle are settled in bulk as eligible with
        // alpha 1, exactly what the per-pair pass below would record for them.
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const float lx = fminf(w.d.c0x[b], w.d.cx[b]), ly = fminf(w.d.c0y[b], w.d.cy[b]);
          const float hx = fmaxf(w.d.c0x[b], w.d.cx[b]), hy = fmaxf(w.d.c0y[b], w.d.cy[b]);
          bool in;
          if (b == B_PK) {
            in = inside(kInteriorPuck, lx, ly, hx, hy);  // a circle's core is its centre
          } else {
            const float(&e)[4] = cb.e[b];
            const float rot = SC.rcore[b] * fabsf(w.d.a[b] - w.d.a0[b]);
            in = inside(kInteriorPlayer, lx + e[0] - rot, ly + e[1] - rot, hx + e[2] + rot, hy + e[3] + rot);
          }
          if (in && w.d.awake[b]) settled |= kEdgeMask[b];
        }
        settled &= kToiPairs & w.enabled;
        elig |= settled;
        w.toiflag |= settled;
        below &= ~settled;
        // The rest of the first pass has no order-dependent side effect either, so it runs as a uniform loop
        // over the compile-time TOI pair table (scene data as literals, per-lane predicates) instead of each
        // lane walking its own pairs through LDS lookups: the same flags and far tests, so the same queue.
        const uint32_t open = kToiPairs & w.enabled & ~settled;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          if (!((kToiPairs >> p) & 1u)) continue;
          const uint32_t bit = 1u << p;
          const bool live = (open & bit) && w.d.awake[SC.pbodyB[p]];
          elig |= live ? bit : 0u;
          const bool far = live && pair_far_toi(w, p, cb, SC);
          below &= far ? ~bit : ~0u;
          pending |= (live && !far) ? bit : 0u;
        }
        w.toiflag |= elig;
        todo = 0u;
      } else {
        // Later passes: an event re-enables TOI only on the moved dynamic body's contacts (their flags were
        // cleared).  Every other pair keeps its eligibility and cached alpha (cached pairs are eligible;
        // the rest were skipped for reasons no event changes), so only `redo` is visited.
        elig = w.toiflag & w.enabled & ~exhausted;
        todo = redo & kToiPairs & w.enabled & ~exhausted & ~w.toiflag;
      }
      // in pair order, per lane: eligibility, sweep alignment and the far test of the pairs still open
      while (todo) {
        const int p = __ffs(todo) - 1;
        todo &= todo - 1u;
        const uint32_t bit = 1u << p;
        const int bA = SLDS.pbodyA[p], bB = SLDS.pbodyB[p];
        if (!pick(w.d.awake, bB, 0)) continue;
        elig |= bit;
        w.toiflag |= bit;
        const float a0A = LDS(w, kLdsSal0 + bA - 3), a0B = pick(w.d.al0, bB, 0.0f);
        if (a0A < a0B) {
          LDS(w, kLdsSal0 + bA - 3) = a0B;  // static b2Sweep::Advance: only alpha0 moves
        } else if (a0B < a0A) {
          toi_drain(w, pending, below);  // keep the sequential order for this lane (see above)
          Sweep sw = body_sweep(w, bB);
          sweep_advance(sw, a0A);
          body_set_sweep(w, bB, sw);
        }
        if (pair_far_toi(w, p, cb, SLDS)) {
          below &= ~bit;
        } else {
          pending |= bit;
        }
      }
      first = false;
    }
    HK_TIC(T, 6);  // diagnostics: scan pass -> "toi-scan"
    // (2) the queued b2TimeOfImpact calls of the whole wave, dealt out over all its lanes
    toi_drain_wave(w, pending, below);
    HK_TIC(T, 7);  // diagnostics: b2TimeOfImpact -> "toi-solve" slot
    if (!act) continue;
    // (3) Box2D's minimum: first pair (in order) with the smallest alpha.  Pairs at alpha 1 never win the
    //     strict comparison, so only the lane's eligible pairs below 1 are visited (usually none or one).
    int minc = -1;
    float minAlpha = 1.0f;
    for (uint32_t m = elig & below; m; m &= m - 1u) {
      const int p = __ffs(m) - 1;
      const float alpha = LDS(w, kLdsToi + p);
      if (alpha < minAlpha) { minc = p; minAlpha = alpha; }
    }
    if (minc < 0 || 1.0f - 10.0f * kFltEps < minAlpha) {
      act = false;
      continue;
    }
    // ---- one TOI event (per-lane pair) ----
    const int bA = SLDS.pbodyA[minc], bB = SLDS.pbodyB[minc];  // static A, dynamic B
    const uint32_t mbit = 1u << minc;
    const Sweep backA = body_sweep(w, bA), backB = body_sweep(w, bB);
    body_advance(w, bA, minAlpha);
    body_advance(w, bB, minAlpha);
    pair_update_near(w, minc);  // the broad-phase shortcut only ever skips narrow phases that find no contact
    HK_TIC(T, 8);  // diagnostics: TOI event advance + contact update
    w.toiflag &= ~mbit;
    const float cnt = LDS(w, kLdsCnt + minc) + 1.0f;
    LDS(w, kLdsCnt + minc) = cnt;
    if (cnt > (float)kMaxSubSteps) exhausted |= mbit;
    if (!(w.enabled & mbit) || !(w.touch & mbit)) {
      w.enabled &= ~mbit;
      body_set_sweep(w, bA, backA);
      body_set_sweep(w, bB, backB);
      sync_xf(w, bA);
      sync_xf(w, bB);
      redo = 0u;  // sweeps restored: every other pair's flag and alpha stand
      continue;
    }
    w.n_toi++;
    set_awake(w, bA, 1);
    set_awake(w, bB, 1);
    w.bisl = (1u << bA) | (1u << bB);
    w.cisl |= mbit;
    uint32_t extra = 0u;  // other island contacts, added in B's (ascending) edge order
    int nc = 1;
    // B's contacts with static bodies (its TOI pairs) not yet in the island.  Their broad-phase tests read only
    // B's advanced pose and the scene, so they run first as a uniform loop over the compile-time pair table; a
    // rejected pair's b2Contact::Update (not touching: enabled, touching bit, wake-ups of awake bodies) changes
    // only its own bits, so it commutes with the other updates, and its tentative advance of the static body is
    // undone in the per-lane walk anyway.  The remaining (near) pairs keep the walk in edge order.
    const uint32_t cand = pick(kEdgeMask, bB, 0u) & kToiPairs & ~w.cisl;
    uint32_t m = 0u;
    {
      CoreBoxes cbe;
      core_boxes(w, cbe);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        if (!((kToiPairs >> p) & 1u)) continue;
        const uint32_t bit = 1u << p;
        if (!(cand & bit)) continue;
        if (pair_far_collide(w, p, &cbe, SC)) pair_update_far(w, p, SC);
        else m |= bit;
      }
    }
    while (m) {
      const int e = __ffs(m) - 1;
      m &= m - 1u;
      const uint32_t ebit = 1u << e;
      const int other = SLDS.pbodyA[e];  // the static body of a TOI pair
      const Sweep backup = body_sweep(w, other);
      if (!((w.bisl >> other) & 1u)) body_advance(w, other, minAlpha);
      pair_update_near(w, e);
      if (!(w.enabled & ebit) || !(w.touch & ebit)) {
        body_set_sweep(w, other, backup);
        continue;
      }
      w.cisl |= ebit;
      extra |= ebit;
      ++nc;
      w.bisl |= 1u << other;
    }
    HK_TIC(T, 9);  // diagnostics: TOI island build
    const float sub_dt = (1.0f - minAlpha) * dt;
    if (nc > kBigC) { w.overflow = 1; nc = kBigC; }
    if (nc <= kToiC && !w.force_big) {
      RegSlots<kToiC> S;
      toi_island_solve(w, S, minc, extra, nc, bB, sub_dt, T);
    } else {
      w.n_big++;
      HbmSlots S{w.ws, w.n, w.a};
      toi_island_solve(w, S, minc, extra, nc, bB, sub_dt, T);
    }
    // reset island flags; invalidate the TOIs of the displaced dynamic body
    w.bisl = 0u;
    const uint32_t em = pick(kEdgeMask, bB, 0u);
    w.toiflag &= ~em;
    w.cisl &= ~em;
    redo = em;
  }
}

// b2World::Step (hockey_env.py:682)
HK_DEV void world_step(Arena &w, PhaseT &T) {
  const float dt = 0.02f;
  collide(w);
  HK_TIC(T, 1);
  HK_TRACE_POINT(w, 0);
  bool done = false;
  if (!w.force_big) {
    RegSlots<kIslandC> S;
    done = solve_islands(w, S, dt, T);
  }
  if (!done) {  // more island contacts than register slots: identical solve on the HBM slot file
    w.n_big++;
    HbmSlots S{w.ws, w.n, w.a};
    solve_islands(w, S, dt, T);
  }
  HK_TIC(T, 4);  // diagnostics: position iterations + sleep
  HK_TRACE_POINT(w, 1);
  solve_toi(w, dt, T);
  HK_TIC(T, 5);
  HK_TRACE_POINT(w, 2);
#pragma unroll
  for (int b = 0; b < 3; ++b) { w.d.fx[b] = 0.0f; w.d.fy[b] = 0.0f; w.d.tq[b] = 0.0f; }
}

// ------------------------------------------------------------------------------------------------
// HockeyEnv.step laws (hockey_env.py:420-483, 610-633), numpy NEP-50 + pybox2d float32 semantics
// ------------------------------------------------------------------------------------------------
constexpr double kDtPy = 0.02;  // self.timeStep = 1.0 / FPS  (hockey_env.py:119)
constexpr double kPiD = 3.141592653589793;

template <int B>
HK_DEV void check_boundaries(Arena &w, float &f0, float &f1, int one) {
  const double px = w.d.px[B], py = w.d.py[B];
  if ((one && px < 1.5 && f0 < 0) || (!one && px > 8.5 && f0 > 0) || (one && px > 5.0 && f0 > 0) ||
      (!one && px < 5.0 && f0 < 0)) {
    float vel0 = w.d.vx[B];
    if (w.vel_ref) { w.d.vx[B] = 0.0f; vel0 = 0.0f; }
    f0 = -vel0;
  }
  if ((py > 8.0 - 1.2 && f1 > 0) || (py < 1.2 && f1 < 0)) {
    float vel1 = w.d.vy[B];
    if (w.vel_ref) { w.d.vy[B] = 0.0f; vel1 = 0.0f; }
    f1 = -vel1;
  }
}

template <int B>
HK_DEV void translation_law(Arena &w, float a0, float a1) {
  constexpr int one = (B == B_P1);
  const double vx = w.d.vx[B], vy = w.d.vy[B];
  const double speed = sqrt(vx * vx + vy * vy);
  float f0, f1;
  if (one) { f0 = a0 * 6000.0f; f1 = a1 * 6000.0f; }
  else { f0 = (-a0) * 6000.0f; f1 = (-a1) * 6000.0f; }
  const double px = w.d.px[B], m = SC.mass[B];
  if ((one && px > 5.0 - 0.5) || (!one && px < 5.0 + 0.5)) {
    f0 = 0.0f;
    if (one) {
      if (vx > 0) f0 = (float)((((-2.0) * vx) * m) / kDtPy);
      f0 = f0 + (float)(((((-1.0) * (px - 5.0)) * vx) * m) / kDtPy);
    } else {
      if (vx < 0) f0 = (float)((((-2.0) * vx) * m) / kDtPy);
      f0 = f0 + (float)((((1.0 * (px - 5.0)) * vx) * m) / kDtPy);
    }
    w.d.ld[B] = 20.0f;
    check_boundaries<B>(w, f0, f1, one);
    apply_force<B>(w, V(f0, f1));
    return;
  }
  if (speed < 10.0) {
    w.d.ld[B] = 5.0f;
    check_boundaries<B>(w, f0, f1, one);
    apply_force<B>(w, V(f0, f1));
  } else {
    w.d.ld[B] = 20.0f;
    const float mf = (float)m;
    const float d0 = (0.02f * f0) / mf, d1 = (0.02f * f1) / mf;
    const double nx = vx + (double)d0, ny = vy + (double)d1;
    if (sqrt(nx * nx + ny * ny) < speed) {
      check_boundaries<B>(w, f0, f1, one);
      apply_force<B>(w, V(f0, f1));
    }
  }
}

template <int B>
HK_DEV void rotation_law(Arena &w, float a) {
  const double ang = w.d.a[B], wv = w.d.w[B], m = SC.mass[B];
  if (fabs(ang) > kPiD / 3) {
    double t = 0.0;
    if (ang * wv > 0) t = (((-0.1) * wv) * m) / kDtPy;
    t = t + (((-0.1) * ang) * m) / kDtPy;
    w.d.ad[B] = 10.0f;
    apply_torque<B>(w, (float)t);
  } else {
    w.d.ad[B] = 2.0f;
    apply_torque<B>(w, a * 400.0f);
  }
}

template <int B>
HK_DEV void shoot(Arena &w) {
  const double ca = hk_cos((double)w.d.a[B]), sa = hk_sin((double)w.d.a[B]);
  const double sgn = B == B_P1 ? 1.0 : -1.0;
  v2 f = V((float)(ca * sgn), (float)(sa * sgn));
  const float m = SC.mass[B_PK];
  f = V(f.x * m, f.y * m);
  f = V(f.x / 0.02f, f.y / 0.02f);
  f = V(f.x * 60.0f, f.y * 60.0f);
  apply_force<B_PK>(w, f);
}

template <int B>
HK_DEV void keep_puck(Arena &w) {
  set_transform<B_PK>(w, V(w.d.px[B], w.d.py[B]), w.d.a[B_PK]);
  set_linear_velocity<B_PK>(w, V(w.d.vx[B], w.d.vy[B]));
}

HK_DEV float clip1(float x) { return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x); }

HK_DEV void presolve(Arena &w, const float *a8) {
  float a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = clip1(a8[i]);
  translation_law<B_P1>(w, a[0], a[1]);
  rotation_law<B_P1>(w, a[2]);
  translation_law<B_P2>(w, a[4], a[5]);
  rotation_law<B_P2>(w, a[6]);
  {
    const double vx = w.d.vx[B_PK], vy = w.d.vy[B_PK];
    const double s = sqrt(vx * vx + vy * vy);
    w.d.ld[B_PK] = s > 25.0 ? 10.0f : 0.05f;
  }
  if (w.keep_mode) {
    if (w.has1 > 1) {
      keep_puck<B_P1>(w);
      w.has1 -= 1;
      if (w.has1 == 1 || a[3] > 0.5f) { shoot<B_P1>(w); w.has1 = 0; }
    }
    if (w.has2 > 1) {
      keep_puck<B_P2>(w);
      w.has2 -= 1;
      if (w.has2 == 1 || a[7] > 0.5f) { shoot<B_P2>(w); w.has2 = 0; }
    }
  }
}

HK_DEV void observe(const Arena &w, float *o) {
  const Dyn &d = w.d;
  o[0] = d.px[0] - 5.0f; o[1] = d.py[0] - 4.0f; o[2] = d.a[0];
  o[3] = d.vx[0]; o[4] = d.vy[0]; o[5] = d.w[0];
  o[6] = d.px[1] - 5.0f; o[7] = d.py[1] - 4.0f; o[8] = d.a[1];
  o[9] = d.vx[1]; o[10] = d.vy[1]; o[11] = d.w[1];
  o[12] = d.px[2] - 5.0f; o[13] = d.py[2] - 4.0f;
  o[14] = d.vx[2]; o[15] = d.vy[2];
  o[16] = w.keep_mode ? (float)w.has1 : 0.0f;
  o[17] = w.keep_mode ? (float)w.has2 : 0.0f;
}

HK_DEV void observe_two(const Arena &w, float *o) {
  const Dyn &d = w.d;
  o[0] = -(d.px[1] - 5.0f); o[1] = -(d.py[1] - 4.0f); o[2] = d.a[1];
  o[3] = -d.vx[1]; o[4] = -d.vy[1]; o[5] = d.w[1];
  o[6] = -(d.px[0] - 5.0f); o[7] = -(d.py[0] - 4.0f); o[8] = d.a[0];
  o[9] = -d.vx[0]; o[10] = -d.vy[0]; o[11] = d.w[0];
  o[12] = -(d.px[2] - 5.0f); o[13] = -(d.py[2] - 4.0f);
  o[14] = -d.vx[2]; o[15] = -d.vy[2];
  o[16] = w.keep_mode ? (float)w.has2 : 0.0f;
  o[17] = w.keep_mode ? (float)w.has1 : 0.0f;
}

// _get_info / get_info_agent_two (hockey_env.py:542-591), double like the reference
template <int TWO>
HK_DEV void info_side(const Arena &w, double *info4) {
  constexpr int me = TWO ? B_P2 : B_P1;
  const Dyn &d = w.d;
  const double T = (double)w.max_t;
  double close = 0.0;
  const int cond = TWO ? ((double)d.px[2] > 5.0 && (double)d.vx[2] >= 0) : ((double)d.px[2] < 5.0 && (double)d.vx[2] <= 0);
  if (cond) {
    const float dx = d.px[me] - d.px[2], dy = d.py[me] - d.py[2];
    const double dd = sqrt((double)dx * (double)dx + (double)dy * (double)dy);
    const double max_dist = 250.0 / 60.0;
    const double factor = -30.0 / ((max_dist * T) / 2);
    close = close + dd * factor;
  }
  const double touch = ((TWO ? w.has2 : w.has1) == 15) ? 1.0 : 0.0;
  const double f2 = TWO ? (-1.0) / (T * 25) : 1.0 / (T * 25);
  info4[0] = TWO ? -w.winner : w.winner;
  info4[1] = close;
  info4[2] = touch;
  info4[3] = (double)d.vx[2] * f2;
}

HK_DEV double compute_reward(const Arena &w) {
  double r = 0;
  if (w.done) {
    if (w.winner == 1) r += 10;
    else if (w.winner != 0) r -= 10;
  }
  return r;
}

// BasicOpponent.act (hockey_env.py:787-833) on an own-frame float32 obs, double arithmetic
HK_DEV void basic_opponent(int weak, int keep_mode, double &phase, double inc, const float *of, float *act) {
  const double p1x = of[0], p1y = of[1], p1a = of[2];
  const double v1[3] = {of[3], of[4], of[5]};
  const double pkx = of[12], pky = of[13], pvx = of[14], pvy = of[15];
  double tx, ty;
  phase += inc;
  const double kp = weak ? 0.5 : 10.0, kd = 0.5;
  if (pvx < 30.0 / 60.0) {
    const double dx = p1x - pkx, dy = p1y - pky;
    const double dist = sqrt(dx * dx + dy * dy);
    double ady = p1y - pky;
    if (ady < 0) ady = -ady;
    if (p1x < pkx && ady < 30.0 / 60.0) {
      tx = pkx + 0.2;
      ty = pky + (pvy * dist) * 0.1;
    } else {
      tx = -210.0 / 60.0;
      ty = pky;
    }
  } else {
    tx = -210.0 / 60.0;
    ty = 0.0;
  }
  const double ta = (kPiD / 3) * hk_sin(phase);
  const double o16 = of[16];
  const double shoot_ = (keep_mode && o16 > 0 && o16 < 7) ? 1.0 : 0.0;
  const double err[3] = {tx - p1x, ty - p1y, ta - p1a};
  const double gains[3] = {kp, kp / 5, kp / 2};
  const double tb[3] = {0.1, 0.1, 0.1 * 10};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    double q = err[i] / (v1[i] + 0.01);
    if (q < 0) q = -q;
    const double nb = (q < tb[i]) ? 1.0 : 0.0;
    const double x = err[i] * gains[i] - (v1[i] * nb) * kd;
    act[i] = (float)(x < -1.0 ? -1.0 : (x > 1.0 ? 1.0 : x));
  }
  act[3] = (float)shoot_;
}

#undef SC
}  // namespace hk
