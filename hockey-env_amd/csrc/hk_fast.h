// hk_fast.h -- register-resident contact solver (the hot loop of b2Island::Solve / SolveTOI).
//
// Why: one lane runs one arena's Gauss-Seidel loop (180 velocity iterations x island contacts, up to
// 60 / 20 position iterations).  Addressing constraints and body velocities through private arrays
// (v1) put every iteration behind scratch-memory round trips (~7k cycles per contact-iteration at one
// wave per SIMD).  Here the island's contacts live in kFastC fixed register slots (loops fully unrolled,
// slot indices compile-time), and the <=3 dynamic bodies' positions / velocities in registers addressed
// by body id through select chains (a static body reads as zero velocity / fixed origin, exactly what
// Box2D's island arrays hold for it).  Islands with more contacts (~2e-4 of arena-steps) take the
// generic path in hk_world.h.  Float operation order is identical to the generic path / the oracle.
#pragma once
#include "hk_world.h"

namespace hk {

#define SC g_scene

constexpr int kFastC = 3;

struct FSlot {
  int p, bA, bB, vcount, pcount, type, isl;
  float mA, mB, iA, iB, fr, re;
  float sAx, sAy;  // origin of a static body A (bA == 3)
  float nx, ny;
  float rAx[2], rAy[2], rBx[2], rBy[2], ni[2], ti[2], nm[2], tm[2], bias[2];
  float Kxx, Kxy, Kyx, Kyy, Nxx, Nxy, Nyx, Nyy;
  float lpsx[2], lpsy[2], lnx, lny, lpx, lpy, lcAx, lcAy, lcBx, lcBy, rA, rB;
};

struct FBodies {  // dynamic bodies 0..2 (player1, player2, puck)
  float cx[3], cy[3], a[3], vx[3], vy[3], w[3];
};

HK_DEV float sel3(int b, float x0, float x1, float x2, float dflt) {
  return b == 0 ? x0 : (b == 1 ? x1 : (b == 2 ? x2 : dflt));
}
HK_DEV void put3(int b, float v, float &x0, float &x1, float &x2) {
  x0 = b == 0 ? v : x0;
  x1 = b == 1 ? v : x1;
  x2 = b == 2 ? v : x2;
}
HK_DEV void get_vel(const FBodies &B, int b, v2 &v, float &w) {
  v = V(sel3(b, B.vx[0], B.vx[1], B.vx[2], 0.0f), sel3(b, B.vy[0], B.vy[1], B.vy[2], 0.0f));
  w = sel3(b, B.w[0], B.w[1], B.w[2], 0.0f);
}
HK_DEV void set_vel(FBodies &B, int b, v2 v, float w) {
  put3(b, v.x, B.vx[0], B.vx[1], B.vx[2]);
  put3(b, v.y, B.vy[0], B.vy[1], B.vy[2]);
  put3(b, w, B.w[0], B.w[1], B.w[2]);
}
HK_DEV void get_pos(const FBodies &B, int b, float sx, float sy, v2 &c, float &a) {
  c = V(sel3(b, B.cx[0], B.cx[1], B.cx[2], sx), sel3(b, B.cy[0], B.cy[1], B.cy[2], sy));
  a = sel3(b, B.a[0], B.a[1], B.a[2], 0.0f);
}
HK_DEV void set_pos(FBodies &B, int b, v2 c, float a) {
  put3(b, c.x, B.cx[0], B.cx[1], B.cx[2]);
  put3(b, c.y, B.cy[0], B.cy[1], B.cy[2]);
  put3(b, a, B.a[0], B.a[1], B.a[2]);
}

// b2ContactSolver constructor for one contact (solver_init in hk_world.h)
HK_DEV void fslot_load(FSlot &s, const World &w, int p, int warm, int isl) {
  const Contact &c = w.c[p];
  const int pa = SC.pbodyA[p], pb = SC.pbodyB[p];
  s.p = p;
  s.isl = isl;
  s.bA = pa < 3 ? pa : 3;
  s.bB = pb;  // always dynamic
  const Body &bA = w.b[pa];
  const Body &bB = w.b[pb];
  s.fr = SC.friction[p];
  s.re = SC.restitution[p];
  s.mA = bA.invMass; s.mB = bB.invMass; s.iA = bA.invI; s.iB = bB.invI;
  s.sAx = SC.spx[pa];
  s.sAy = SC.spy[pa];
  s.vcount = c.m.count;
  s.pcount = c.m.count;
  s.type = c.m.type;
  s.Kxx = s.Kxy = s.Kyx = s.Kyy = 0.0f;
  s.Nxx = s.Nxy = s.Nyx = s.Nyy = 0.0f;
  s.lnx = c.m.ln.x; s.lny = c.m.ln.y; s.lpx = c.m.lp.x; s.lpy = c.m.lp.y;
  s.lcAx = bA.lc.x; s.lcAy = bA.lc.y; s.lcBx = bB.lc.x; s.lcBy = bB.lc.y;
  s.rA = SC.fx[SC.pairA[p]].radius;
  s.rB = SC.fx[SC.pairB[p]].radius;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool on = j < c.m.count;
    s.ni[j] = on && warm ? 1.0f * c.m.ni[j] : 0.0f;
    s.ti[j] = on && warm ? 1.0f * c.m.ti[j] : 0.0f;
    s.rAx[j] = s.rAy[j] = s.rBx[j] = s.rBy[j] = 0.0f;
    s.nm[j] = s.tm[j] = s.bias[j] = 0.0f;
    s.lpsx[j] = on ? c.m.pt_lp[j].x : 0.0f;
    s.lpsy[j] = on ? c.m.pt_lp[j].y : 0.0f;
  }
}

// InitializeVelocityConstraints for one contact
HK_DEV void fslot_init_velocity(FSlot &s, const FBodies &B) {
  const float mA = s.mA, mB = s.mB, iA = s.iA, iB = s.iB;
  v2 cA, cB, vA, vB;
  float aA, aB, wA, wB;
  get_pos(B, s.bA, s.sAx, s.sAy, cA, aA);
  get_pos(B, s.bB, 0.0f, 0.0f, cB, aB);
  get_vel(B, s.bA, vA, wA);
  get_vel(B, s.bB, vB, wB);
  xform xA, xB;
  xA.q = rot_set(aA);
  xB.q = rot_set(aB);
  xA.p = vsub(cA, mul_rv(xA.q, V(s.lcAx, s.lcAy)));
  xB.p = vsub(cB, mul_rv(xB.q, V(s.lcBx, s.lcBy)));
  // b2WorldManifold::Initialize
  v2 normal, pts[2];
  {
    Manifold m;
    m.type = s.type;
    m.count = s.pcount;
    m.ln = V(s.lnx, s.lny);
    m.lp = V(s.lpx, s.lpy);
    m.pt_lp[0] = V(s.lpsx[0], s.lpsy[0]);
    m.pt_lp[1] = V(s.lpsx[1], s.lpsy[1]);
    if (m.type == 1) {
      normal = mul_rv(xA.q, m.ln);
      v2 plane = mul_xv(xA, m.lp);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        v2 clip = mul_xv(xB, m.pt_lp[i]);
        v2 ca = vadd(clip, vs(s.rA - dot(vsub(clip, plane), normal), normal));
        v2 cb = vsub(clip, vs(s.rB, normal));
        pts[i] = vs(0.5f, vadd(ca, cb));
      }
    } else {
      normal = mul_rv(xB.q, m.ln);
      v2 plane = mul_xv(xB, m.lp);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        v2 clip = mul_xv(xA, m.pt_lp[i]);
        v2 cb = vadd(clip, vs(s.rB - dot(vsub(clip, plane), normal), normal));
        v2 ca = vsub(clip, vs(s.rA, normal));
        pts[i] = vs(0.5f, vadd(ca, cb));
      }
      normal = vneg(normal);
    }
  }
  s.nx = normal.x;
  s.ny = normal.y;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < s.vcount) {
      v2 rA = vsub(pts[j], cA), rB = vsub(pts[j], cB);
      s.rAx[j] = rA.x; s.rAy[j] = rA.y; s.rBx[j] = rB.x; s.rBy[j] = rB.y;
      float rnA = crs(rA, normal), rnB = crs(rB, normal);
      float kN = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      s.nm[j] = kN > 0.0f ? 1.0f / kN : 0.0f;
      v2 tangent = crs_vs(normal, 1.0f);
      float rtA = crs(rA, tangent), rtB = crs(rB, tangent);
      float kT = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
      s.tm[j] = kT > 0.0f ? 1.0f / kT : 0.0f;
      s.bias[j] = 0.0f;
      float vRel = dot(normal, vsub(vsub(vadd(vB, crs_sv(wB, rB)), vA), crs_sv(wA, rA)));
      if (vRel < -kVelocityThreshold) s.bias[j] = -s.re * vRel;
    }
  }
  if (s.vcount == 2) {
    v2 r1A = V(s.rAx[0], s.rAy[0]), r1B = V(s.rBx[0], s.rBy[0]);
    v2 r2A = V(s.rAx[1], s.rAy[1]), r2B = V(s.rBx[1], s.rBy[1]);
    float rn1A = crs(r1A, normal), rn1B = crs(r1B, normal);
    float rn2A = crs(r2A, normal), rn2B = crs(r2B, normal);
    float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
    float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
    float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
    if (k11 * k11 < 1000.0f * (k11 * k22 - k12 * k12)) {
      s.Kxx = k11; s.Kxy = k12; s.Kyx = k12; s.Kyy = k22;
      float a = s.Kxx, b = s.Kyx, c = s.Kxy, d = s.Kyy;
      float det = a * d - b * c;
      if (det != 0.0f) det = 1.0f / det;
      s.Nxx = det * d; s.Nyx = -det * b;
      s.Nxy = -det * c; s.Nyy = det * a;
    } else {
      s.vcount = 1;
    }
  }
}

HK_DEV void fslot_warm_start(const FSlot &s, FBodies &B) {
  v2 vA, vB;
  float wA, wB;
  get_vel(B, s.bA, vA, wA);
  get_vel(B, s.bB, vB, wB);
  const v2 normal = V(s.nx, s.ny), tangent = crs_vs(normal, 1.0f);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < s.vcount) {
      v2 P = vadd(vs(s.ni[j], normal), vs(s.ti[j], tangent));
      wA -= s.iA * crs(V(s.rAx[j], s.rAy[j]), P);
      vA = vsub(vA, vs(s.mA, P));
      wB += s.iB * crs(V(s.rBx[j], s.rBy[j]), P);
      vB = vadd(vB, vs(s.mB, P));
    }
  }
  set_vel(B, s.bA, vA, wA);
  set_vel(B, s.bB, vB, wB);
}

// one b2ContactSolver::SolveVelocityConstraints pass over one contact
HK_DEV void fslot_solve_velocity(FSlot &s, FBodies &B) {
  const float mA = s.mA, iA = s.iA, mB = s.mB, iB = s.iB;
  v2 vA, vB;
  float wA, wB;
  get_vel(B, s.bA, vA, wA);
  get_vel(B, s.bB, vB, wB);
  const v2 normal = V(s.nx, s.ny), tangent = crs_vs(normal, 1.0f);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < s.vcount) {
      const v2 rA = V(s.rAx[j], s.rAy[j]), rB = V(s.rBx[j], s.rBy[j]);
      v2 dv = vsub(vsub(vadd(vB, crs_sv(wB, rB)), vA), crs_sv(wA, rA));
      float vt = dot(dv, tangent) - 0.0f;
      float lambda = s.tm[j] * (-vt);
      float maxF = s.fr * s.ni[j];
      float newI = fclamp(s.ti[j] + lambda, -maxF, maxF);
      lambda = newI - s.ti[j];
      s.ti[j] = newI;
      v2 P = vs(lambda, tangent);
      vA = vsub(vA, vs(mA, P));
      wA -= iA * crs(rA, P);
      vB = vadd(vB, vs(mB, P));
      wB += iB * crs(rB, P);
    }
  }
  if (s.vcount == 1) {
    const v2 rA = V(s.rAx[0], s.rAy[0]), rB = V(s.rBx[0], s.rBy[0]);
    v2 dv = vsub(vsub(vadd(vB, crs_sv(wB, rB)), vA), crs_sv(wA, rA));
    float vn = dot(dv, normal);
    float lambda = -s.nm[0] * (vn - s.bias[0]);
    float newI = fmax2(s.ni[0] + lambda, 0.0f);
    lambda = newI - s.ni[0];
    s.ni[0] = newI;
    v2 P = vs(lambda, normal);
    vA = vsub(vA, vs(mA, P));
    wA -= iA * crs(rA, P);
    vB = vadd(vB, vs(mB, P));
    wB += iB * crs(rB, P);
  } else {
    const v2 r1A = V(s.rAx[0], s.rAy[0]), r1B = V(s.rBx[0], s.rBy[0]);
    const v2 r2A = V(s.rAx[1], s.rAy[1]), r2B = V(s.rBx[1], s.rBy[1]);
    v2 a = V(s.ni[0], s.ni[1]);
    v2 dv1 = vsub(vsub(vadd(vB, crs_sv(wB, r1B)), vA), crs_sv(wA, r1A));
    v2 dv2 = vsub(vsub(vadd(vB, crs_sv(wB, r2B)), vA), crs_sv(wA, r2A));
    float vn1 = dot(dv1, normal), vn2 = dot(dv2, normal);
    v2 b;
    b.x = vn1 - s.bias[0];
    b.y = vn2 - s.bias[1];
    b = vsub(b, V(s.Kxx * a.x + s.Kyx * a.y, s.Kxy * a.x + s.Kyy * a.y));
    v2 x = vneg(V(s.Nxx * b.x + s.Nyx * b.y, s.Nxy * b.x + s.Nyy * b.y));
    int ok = 0;
    if (x.x >= 0.0f && x.y >= 0.0f) ok = 1;
    if (!ok) {
      x.x = -s.nm[0] * b.x;
      x.y = 0.0f;
      vn2 = s.Kxy * x.x + b.y;
      if (x.x >= 0.0f && vn2 >= 0.0f) ok = 1;
    }
    if (!ok) {
      x.x = 0.0f;
      x.y = -s.nm[1] * b.y;
      vn1 = s.Kyx * x.y + b.x;
      if (x.y >= 0.0f && vn1 >= 0.0f) ok = 1;
    }
    if (!ok) {
      x.x = 0.0f;
      x.y = 0.0f;
      vn1 = b.x;
      vn2 = b.y;
      if (vn1 >= 0.0f && vn2 >= 0.0f) ok = 1;
    }
    if (ok) {
      v2 d = vsub(x, a);
      v2 P1 = vs(d.x, normal), P2 = vs(d.y, normal);
      vA = vsub(vA, vs(mA, vadd(P1, P2)));
      wA -= iA * (crs(r1A, P1) + crs(r2A, P2));
      vB = vadd(vB, vs(mB, vadd(P1, P2)));
      wB += iB * (crs(r1B, P1) + crs(r2B, P2));
      s.ni[0] = x.x;
      s.ni[1] = x.y;
    }
  }
  set_vel(B, s.bA, vA, wA);
  set_vel(B, s.bB, vB, wB);
}

// one NGS position pass over one contact; mass scales select SolveTOIPositionConstraints
HK_DEV float fslot_solve_position(const FSlot &s, FBodies &B, float baum, float mA, float iA, float mB, float iB,
                                  float minSep) {
  v2 cA, cB;
  float aA, aB;
  get_pos(B, s.bA, s.sAx, s.sAy, cA, aA);
  get_pos(B, s.bB, 0.0f, 0.0f, cB, aB);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < s.pcount) {
      xform xA, xB;
      xA.q = rot_set(aA);
      xB.q = rot_set(aB);
      xA.p = vsub(cA, mul_rv(xA.q, V(s.lcAx, s.lcAy)));
      xB.p = vsub(cB, mul_rv(xB.q, V(s.lcBx, s.lcBy)));
      v2 normal, point;
      float sep;
      if (s.type == 1) {
        normal = mul_rv(xA.q, V(s.lnx, s.lny));
        v2 plane = mul_xv(xA, V(s.lpx, s.lpy));
        v2 clip = mul_xv(xB, V(s.lpsx[j], s.lpsy[j]));
        sep = dot(vsub(clip, plane), normal) - s.rA - s.rB;
        point = clip;
      } else {
        normal = mul_rv(xB.q, V(s.lnx, s.lny));
        v2 plane = mul_xv(xB, V(s.lpx, s.lpy));
        v2 clip = mul_xv(xA, V(s.lpsx[j], s.lpsy[j]));
        sep = dot(vsub(clip, plane), normal) - s.rA - s.rB;
        point = clip;
        normal = vneg(normal);
      }
      v2 rA = vsub(point, cA), rB = vsub(point, cB);
      minSep = fmin2(minSep, sep);
      float C = fclamp(baum * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
      float rnA = crs(rA, normal), rnB = crs(rB, normal);
      float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      float impulse = K > 0.0f ? -C / K : 0.0f;
      v2 Pv = vs(impulse, normal);
      cA = vsub(cA, vs(mA, Pv));
      aA -= iA * crs(rA, Pv);
      cB = vadd(cB, vs(mB, Pv));
      aB += iB * crs(rB, Pv);
    }
  }
  if (s.bA < 3) set_pos(B, s.bA, cA, aA);
  set_pos(B, s.bB, cB, aB);
  return minSep;
}

// ------------------------------------------------------------------------------------------------
// Exact early exit of the 180 velocity iterations.  One iteration is a deterministic map F of the
// solver state X = (dynamic body velocities, accumulated normal / tangent impulses).  We snapshot X at
// every iteration it = 3 (mod 4) and compare it bitwise with the snapshot from it - 4: equality means
// F^4 has a fixed point there, so X_k is 4-periodic from it - 4 on and, because 179 - it = 0 (mod 4),
// X_179 == X_it.  Stopping at `it` therefore returns exactly what 180 iterations return (periods 1, 2
// and 4 are caught).  On the oracle's strong-vs-strong workload ~99% of island solves and ~96% of TOI
// solves become periodic, most within 4-12 iterations.
// ------------------------------------------------------------------------------------------------
constexpr int kSnapN = 9 + 4 * kFastC;

HK_DEV void solver_snapshot(const FSlot *S, const FBodies &B, uint32_t *x) {
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    x[3 * b + 0] = __float_as_uint(B.vx[b]);
    x[3 * b + 1] = __float_as_uint(B.vy[b]);
    x[3 * b + 2] = __float_as_uint(B.w[b]);
  }
#pragma unroll
  for (int i = 0; i < kFastC; ++i) {
    x[9 + 4 * i + 0] = __float_as_uint(S[i].ni[0]);
    x[9 + 4 * i + 1] = __float_as_uint(S[i].ni[1]);
    x[9 + 4 * i + 2] = __float_as_uint(S[i].ti[0]);
    x[9 + 4 * i + 3] = __float_as_uint(S[i].ti[1]);
  }
}

// 180 velocity iterations over nc slots, with the exact periodic early exit
HK_DEV void fast_velocity_iterations(FSlot *S, FBodies &B, int nc) {
  uint32_t snap[kSnapN];
#pragma unroll
  for (int k = 0; k < kSnapN; ++k) snap[k] = 0u;
  bool active = nc > 0;
  for (int it = 0; it < kVelIters && active; ++it) {
#pragma unroll
    for (int i = 0; i < kFastC; ++i)
      if (i < nc) fslot_solve_velocity(S[i], B);
    if ((it & 3) == 3) {
      uint32_t cur[kSnapN];
      solver_snapshot(S, B, cur);
      uint32_t diff = 0u;
#pragma unroll
      for (int k = 0; k < kSnapN; ++k) {
        diff |= cur[k] ^ snap[k];
        snap[k] = cur[k];
      }
      if (it >= 7 && diff == 0u) active = false;
    }
  }
}

HK_DEV void fslot_store(const FSlot &s, World &w) {
  Manifold &m = w.c[s.p].m;
#pragma unroll
  for (int j = 0; j < 2; ++j)
    if (j < s.vcount) { m.ni[j] = s.ni[j]; m.ti[j] = s.ti[j]; }
}

HK_DEV void integrate_one(float h, FBodies &B, int b) {
  v2 c = V(B.cx[b], B.cy[b]), v = V(B.vx[b], B.vy[b]);
  float a = B.a[b], wv = B.w[b];
  v2 tr = vs(h, v);
  if (dot(tr, tr) > kMaxTranslation * kMaxTranslation) {
    float ratio = kMaxTranslation / vlen(tr);
    v = vs(ratio, v);
  }
  float rotn = h * wv;
  if (rotn * rotn > kMaxRotation * kMaxRotation) {
    float ratio = kMaxRotation / fabs2(rotn);
    wv *= ratio;
  }
  c = vadd(c, vs(h, v));
  a += h * wv;
  B.cx[b] = c.x; B.cy[b] = c.y; B.a[b] = a; B.vx[b] = v.x; B.vy[b] = v.y; B.w[b] = wv;
}

// ------------------------------------------------------------------------------------------------
// b2World::Solve for the whole arena: islands are found exactly like the generic path (same DFS and
// contact order); their contacts are solved in one interleaved pass (islands share no dynamic body, so
// this is bit-identical), with per-island position early exit and per-island sleep.
// Returns false (state untouched except the DFS wake-ups) when the arena needs the generic path.
// ------------------------------------------------------------------------------------------------
HK_DEV bool fast_islands(World &w, float dt) {
  const float h = dt;
  const int seed_order[3] = {B_PK, B_P2, B_P1};
  int island_of[3] = {-1, -1, -1};
  int slot_p[kFastC] = {0, 0, 0}, slot_isl[kFastC] = {0, 0, 0};
  int nc = 0, nisl = 0;
  uint32_t in_island = 0;  // contacts already added
  for (int si = 0; si < 3; ++si) {
    const int seed = seed_order[si];
    if (island_of[seed] >= 0 || !w.b[seed].awake) continue;
    const int isl = nisl++;
    // DFS over dynamic bodies (static bodies never propagate and hold no state)
    int stack[3], sc = 0;
    stack[sc++] = seed;
    island_of[seed] = isl;
    while (sc > 0) {
      const int bi = stack[--sc];
      set_awake(w.b[bi], 1);
      for (int k = 0; k < 10; ++k) {
        const int e = SC.edges[bi][k];
        const Contact &c = w.c[e];
        if ((in_island >> e) & 1u) continue;
        if (!c.enabled || !c.touching) continue;
        if (SC.sensor[e]) continue;
        in_island |= 1u << e;
        if (nc < kFastC) {
#pragma unroll
          for (int q = 0; q < kFastC; ++q) {
            slot_p[q] = (q == nc) ? e : slot_p[q];
            slot_isl[q] = (q == nc) ? isl : slot_isl[q];
          }
        }
        ++nc;
        const int other = (SC.pbodyA[e] == bi) ? SC.pbodyB[e] : SC.pbodyA[e];
        if (other >= 3) continue;
        if (island_of[other] >= 0) continue;
        island_of[other] = isl;
        stack[sc++] = other;
      }
    }
  }
  if (nc > kFastC) return false;
  // integrate velocities (b2Island::Solve) into registers
  FBodies B;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    Body &bd = w.b[b];
    v2 v = bd.v;
    float wv = bd.w;
    if (island_of[b] >= 0) {
      bd.c0 = bd.c;
      bd.a0 = bd.a;
      v = vadd(v, vs(h, vadd(vs(1.0f, V(0.0f, 0.0f)), vs(bd.invMass, bd.force))));
      wv += h * bd.invI * bd.torque;
      v = vs(1.0f / (1.0f + h * bd.ld), v);
      wv *= 1.0f / (1.0f + h * bd.ad);
    }
    B.cx[b] = bd.c.x; B.cy[b] = bd.c.y; B.a[b] = bd.a; B.vx[b] = v.x; B.vy[b] = v.y; B.w[b] = wv;
  }
  FSlot S[kFastC];
#pragma unroll
  for (int i = 0; i < kFastC; ++i)
    if (i < nc) fslot_load(S[i], w, slot_p[i], 1, slot_isl[i]);
#pragma unroll
  for (int i = 0; i < kFastC; ++i)
    if (i < nc) fslot_init_velocity(S[i], B);
#pragma unroll
  for (int i = 0; i < kFastC; ++i)
    if (i < nc) fslot_warm_start(S[i], B);
  fast_velocity_iterations(S, B, nc);
#pragma unroll
  for (int i = 0; i < kFastC; ++i)
    if (i < nc) fslot_store(S[i], w);
#pragma unroll
  for (int b = 0; b < 3; ++b)
    if (island_of[b] >= 0) integrate_one(h, B, b);
  // position iterations, early exit per island (b2Island::Solve positionSolved)
  int solved = 0;  // bit per island
  for (int it = 0; it < kPosIters; ++it) {
    float ms0 = 0.0f, ms1 = 0.0f, ms2 = 0.0f;
#pragma unroll
    for (int i = 0; i < kFastC; ++i) {
      if (i < nc && !((solved >> S[i].isl) & 1)) {
        float m = fslot_solve_position(S[i], B, kBaumgarte, S[i].mA, S[i].iA, S[i].mB, S[i].iB, 0.0f);
        ms0 = S[i].isl == 0 ? fmin2(ms0, m) : ms0;
        ms1 = S[i].isl == 1 ? fmin2(ms1, m) : ms1;
        ms2 = S[i].isl == 2 ? fmin2(ms2, m) : ms2;
      }
    }
    if (ms0 >= -3.0f * kLinearSlop) solved |= 1;
    if (ms1 >= -3.0f * kLinearSlop) solved |= 2;
    if (ms2 >= -3.0f * kLinearSlop) solved |= 4;
    if ((solved & ((1 << nisl) - 1)) == (1 << nisl) - 1) break;
  }
  // copy back + sleep (per island)
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    if (island_of[b] >= 0) {
      Body &bd = w.b[b];
      bd.c = V(B.cx[b], B.cy[b]);
      bd.a = B.a[b];
      bd.v = V(B.vx[b], B.vy[b]);
      bd.w = B.w[b];
      synchronize_transform(bd);
    }
  }
  const float linTolSqr = kLinearSleepTol * kLinearSleepTol;
  const float angTolSqr = kAngularSleepTol * kAngularSleepTol;
  for (int isl = 0; isl < nisl; ++isl) {
    float minSleep = kFltMax;
    // body order inside the island does not affect min / per-body updates
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      if (island_of[b] == isl) {
        Body &bd = w.b[b];
        if (bd.w * bd.w > angTolSqr || dot(bd.v, bd.v) > linTolSqr) {
          bd.sleep = 0.0f;
          minSleep = 0.0f;
        } else {
          bd.sleep += h;
          minSleep = fmin2(minSleep, bd.sleep);
        }
      }
    }
    if (minSleep >= kTimeToSleep && ((solved >> isl) & 1)) {
#pragma unroll
      for (int b = 0; b < 3; ++b)
        if (island_of[b] == isl) set_awake(w.b[b], 0);
    }
  }
  return true;
}

// b2Island::SolveTOI for a mini-island of <= kFastC contacts (minContact first).  toiA/toiB are the
// body ids of the TOI pair (toiA may be static).
HK_DEV void fast_toi_island(World &w, const int *icont, int nc, int toiA, int toiB, float sub_dt, const int *ibodies,
                            int nb) {
  FBodies B;
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    const Body &bd = w.b[b];
    B.cx[b] = bd.c.x; B.cy[b] = bd.c.y; B.a[b] = bd.a; B.vx[b] = bd.v.x; B.vy[b] = bd.v.y; B.w[b] = bd.w;
  }
  FSlot S[kFastC];
  int cid[kFastC] = {icont[0], nc > 1 ? icont[1] : 0, nc > 2 ? icont[2] : 0};
#pragma unroll
  for (int i = 0; i < kFastC; ++i)
    if (i < nc) fslot_load(S[i], w, cid[i], 0, 0);
  for (int it = 0; it < 20; ++it) {
    float minSep = 0.0f;
#pragma unroll
    for (int i = 0; i < kFastC; ++i) {
      if (i < nc) {
        const int pa = SC.pbodyA[S[i].p], pb = SC.pbodyB[S[i].p];
        const bool toa = (pa == toiA || pa == toiB), tob = (pb == toiA || pb == toiB);
        minSep = fslot_solve_position(S[i], B, kToiBaumgarte, toa ? S[i].mA : 0.0f, toa ? S[i].iA : 0.0f,
                                      tob ? S[i].mB : 0.0f, tob ? S[i].iB : 0.0f, minSep);
      }
    }
    if (minSep >= -1.5f * kLinearSlop) break;
  }
  // leap of faith: new safe state
  if (toiA < 3) {
    w.b[toiA].c0 = V(sel3(toiA, B.cx[0], B.cx[1], B.cx[2], 0.0f), sel3(toiA, B.cy[0], B.cy[1], B.cy[2], 0.0f));
    w.b[toiA].a0 = sel3(toiA, B.a[0], B.a[1], B.a[2], 0.0f);
  } else {
    w.b[toiA].c0 = w.b[toiA].c;
    w.b[toiA].a0 = w.b[toiA].a;
  }
  w.b[toiB].c0 = V(sel3(toiB, B.cx[0], B.cx[1], B.cx[2], 0.0f), sel3(toiB, B.cy[0], B.cy[1], B.cy[2], 0.0f));
  w.b[toiB].a0 = sel3(toiB, B.a[0], B.a[1], B.a[2], 0.0f);
#pragma unroll
  for (int i = 0; i < kFastC; ++i)
    if (i < nc) fslot_init_velocity(S[i], B);
  fast_velocity_iterations(S, B, nc);
  // integrate + sync the island's dynamic bodies
  for (int k = 0; k < nb; ++k) {
    const int b = ibodies[k];
    if (b >= 3) continue;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q == b) integrate_one(sub_dt, B, q);
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    bool inisl = false;
    for (int k = 0; k < nb; ++k) inisl |= (ibodies[k] == q);
    if (inisl) {
      Body &bd = w.b[q];
      bd.c = V(B.cx[q], B.cy[q]);
      bd.a = B.a[q];
      bd.v = V(B.vx[q], B.vy[q]);
      bd.w = B.w[q];
      synchronize_transform(bd);
    }
  }
}

// b2World::Step for one arena (hockey_env.py:682): Collide -> Solve -> SolveTOI -> ClearForces
HK_DEV void world_step(World &w, Solver &S, int ablate, PhaseT &T) {
  const float dt = 0.02f;
  if (!(ablate & 8)) collide(w);
  HK_TIC(T, 2);
  if ((ablate & 16) || !fast_islands(w, dt)) solve_islands(w, S, dt, ablate);
  HK_TIC(T, 3);
  if (!(ablate & 4)) solve_toi(w, S, dt, ablate, T);
  HK_TIC(T, 4);
  for (int i = 0; i < 3; ++i) { w.b[i].force = V(0.0f, 0.0f); w.b[i].torque = 0.0f; }
}

#undef SC
}  // namespace hk
