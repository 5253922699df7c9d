// hk_solver.h -- register-resident contact solver (the hot loop of b2Island::Solve / SolveTOI).
//
// One lane runs one arena's Gauss-Seidel loop (180 velocity iterations x island contacts, up to 60 / 20
// position iterations; Box2D 2.3 b2ContactSolver, restated by the CPU test oracle).  The island's contacts
// live in MAXS fixed register slots (loops fully unrolled, slot indices compile-time); body positions and
// velocities are the arena's register body file (Dyn), addressed by body id through select chains -- a
// static body reads as zero velocity at its fixed origin, exactly what Box2D's island arrays hold for it.
// Float operation order is the oracle's.
#pragma once
// (included from hk_arena.h, which provides Arena / Dyn / pick / place / MF and the SC alias)

namespace hk {



struct FSlot {
  int p, bA, bB, vcount, pcount, type, isl;
  float mA, mB, iA, iB, fr, re;
  float sAx, sAy;  // origin of a static body A (bA == 3)
  float nx, ny;
  float rAx[2], rAy[2], rBx[2], rBy[2], ni[2], ti[2], nm[2], tm[2], bias[2];
  float Kxx, Kxy, Kyx, Kyy, Nxx, Nxy, Nyx, Nyy;
  float lpsx[2], lpsy[2], lnx, lny, lpx, lpy, lcAx, lcAy, lcBx, lcBy, rA, rB;
  uint32_t sn[4];  // impulse snapshot for the periodic early exit (velocity_iterations)
};
constexpr int kSlotWords = (int)(sizeof(FSlot) / 4);

HK_DEV void get_vel(const Dyn &B, int b, v2 &v, float &w) {
  v = V(pick(B.vx, b, 0.0f), pick(B.vy, b, 0.0f));
  w = pick(B.w, b, 0.0f);
}
HK_DEV void set_vel(Dyn &B, int b, v2 v, float w) {
  place(B.vx, b, v.x);
  place(B.vy, b, v.y);
  place(B.w, b, w);
}
HK_DEV void get_pos(const Dyn &B, int b, float sx, float sy, v2 &c, float &a) {
  c = V(pick(B.cx, b, sx), pick(B.cy, b, sy));
  a = pick(B.a, b, 0.0f);
}
HK_DEV void set_pos(Dyn &B, int b, v2 c, float a) {
  place(B.cx, b, c.x);
  place(B.cy, b, c.y);
  place(B.a, b, a);
}

// b2ContactSolver constructor for one contact
HK_DEV void fslot_load(FSlot &s, const Arena &w, int p, int warm, int isl) {
  const int pa = SC.pbodyA[p], pb = SC.pbodyB[p];
  const int slot = SC.manslot[p];
  s.p = p;
  s.isl = isl;
  s.bA = pa < 3 ? pa : 3;
  s.bB = pb;  // always dynamic
  s.fr = SC.friction[p];
  s.re = SC.restitution[p];
  s.mA = inv_mass(pa); s.mB = inv_mass(pb); s.iA = inv_inertia(pa); s.iB = inv_inertia(pb);
  s.sAx = SC.spx[pa];
  s.sAy = SC.spy[pa];
  const int meta = __float_as_int(MF(w, slot, M_META));
  s.vcount = meta & 0xff;
  s.pcount = s.vcount;
  s.type = meta >> 8;
  s.Kxx = s.Kxy = s.Kyx = s.Kyy = 0.0f;
  s.Nxx = s.Nxy = s.Nyx = s.Nyy = 0.0f;
  s.lnx = MF(w, slot, M_LNX); s.lny = MF(w, slot, M_LNY); s.lpx = MF(w, slot, M_LPX); s.lpy = MF(w, slot, M_LPY);
  const v2 lcA = local_center(pa), lcB = local_center(pb);
  s.lcAx = lcA.x; s.lcAy = lcA.y; s.lcBx = lcB.x; s.lcBy = lcB.y;
  s.rA = SC.fx[SC.pairA[p]].radius;
  s.rB = SC.fx[SC.pairB[p]].radius;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool on = j < s.pcount;
    const int o = M_P0X + j * 5;
    s.ni[j] = on && warm ? 1.0f * MF(w, slot, o + 3) : 0.0f;
    s.ti[j] = on && warm ? 1.0f * MF(w, slot, o + 4) : 0.0f;
    s.rAx[j] = s.rAy[j] = s.rBx[j] = s.rBy[j] = 0.0f;
    s.nm[j] = s.tm[j] = s.bias[j] = 0.0f;
    s.lpsx[j] = on ? MF(w, slot, o + 0) : 0.0f;
    s.lpsy[j] = on ? MF(w, slot, o + 1) : 0.0f;
  }
}

// InitializeVelocityConstraints for one contact
HK_DEV void fslot_init_velocity(FSlot &s, const Dyn &B) {
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

HK_DEV void fslot_warm_start(const FSlot &s, Dyn &B) {
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
HK_DEV void fslot_solve_velocity(FSlot &s, Dyn &B) {
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
HK_DEV float fslot_solve_position(const FSlot &s, Dyn &B, float baum, float mA, float iA, float mB, float iB,
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
// Slot files.  Both run fn(slot, i) over the first nc slots in order (Gauss-Seidel order matters).
//   RegSlots: kFastC slots in registers, loops fully unrolled (compile-time slot indices) -- the hot path.
//   HbmSlots: up to kBigC slots in the HBM workspace DevState::ws ([slot][word][arena], lane-contiguous);
//             each visit loads one slot into registers, runs fn and writes it back.  Used by the rare
//             large islands (~1e-5 of arena-steps) so they neither inflate the hot path's register
//             budget nor use private (scratch) memory.
struct RegSlots {
  FSlot s[kFastC];
  template <typename Fn>
  HK_DEV void each(int nc, Fn &&fn) {
#pragma unroll
    for (int i = 0; i < kFastC; ++i)
      if (i < nc) fn(s[i], i);
  }
  HK_DEV void set_pair(int nc, int p, int isl) {
#pragma unroll
    for (int q = 0; q < kFastC; ++q) {
      s[q].p = (q == nc) ? p : s[q].p;
      s[q].isl = (q == nc) ? isl : s[q].isl;
    }
  }
};

struct HbmSlots {
  float *ws;
  int64_t n, a;
  HK_DEV float &word(int i, int k) const { return ws[((int64_t)i * kSlotWords + k) * n + a]; }
  template <typename Fn>
  HK_DEV void each(int nc, Fn &&fn) {
#pragma unroll 1
    for (int i = 0; i < nc; ++i) {
      FSlot t;
      uint32_t *tw = reinterpret_cast<uint32_t *>(&t);
#pragma unroll
      for (int k = 0; k < kSlotWords; ++k) tw[k] = __float_as_uint(word(i, k));
      fn(t, i);
#pragma unroll
      for (int k = 0; k < kSlotWords; ++k) word(i, k) = __uint_as_float(tw[k]);
    }
  }
  HK_DEV void set_pair(int nc, int p, int isl) {
    if (nc < kBigC) {
      word(nc, (int)(offsetof(FSlot, p) / 4)) = __int_as_float(p);
      word(nc, (int)(offsetof(FSlot, isl) / 4)) = __int_as_float(isl);
    }
  }
};
template <typename SL> struct SlotCap;
template <> struct SlotCap<RegSlots> { static constexpr int value = kFastC; };
template <> struct SlotCap<HbmSlots> { static constexpr int value = kBigC; };

// 180 velocity iterations over nc slots, with the exact periodic early exit
template <typename SL>
HK_DEV void velocity_iterations(SL &S, Dyn &B, int nc) {
  uint32_t sb[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) sb[k] = 0u;
  S.each(nc, [&](FSlot &s, int) { s.sn[0] = s.sn[1] = s.sn[2] = s.sn[3] = 0u; });
  bool active = nc > 0;
  for (int it = 0; it < kVelIters && active; ++it) {
    S.each(nc, [&](FSlot &s, int) { fslot_solve_velocity(s, B); });
    if ((it & 3) == 3) {
      uint32_t diff = 0u;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const uint32_t x = __float_as_uint(B.vx[b]), y = __float_as_uint(B.vy[b]), z = __float_as_uint(B.w[b]);
        diff |= (x ^ sb[3 * b]) | (y ^ sb[3 * b + 1]) | (z ^ sb[3 * b + 2]);
        sb[3 * b] = x;
        sb[3 * b + 1] = y;
        sb[3 * b + 2] = z;
      }
      S.each(nc, [&](FSlot &s, int) {
        const uint32_t x0 = __float_as_uint(s.ni[0]), x1 = __float_as_uint(s.ni[1]);
        const uint32_t x2 = __float_as_uint(s.ti[0]), x3 = __float_as_uint(s.ti[1]);
        diff |= (x0 ^ s.sn[0]) | (x1 ^ s.sn[1]) | (x2 ^ s.sn[2]) | (x3 ^ s.sn[3]);
        s.sn[0] = x0;
        s.sn[1] = x1;
        s.sn[2] = x2;
        s.sn[3] = x3;
      });
      if (it >= 7 && diff == 0u) active = false;
    }
  }
}

HK_DEV void fslot_store(const FSlot &s, Arena &w) {
  const int slot = SC.manslot[s.p];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    if (j < s.vcount) {
      MF(w, slot, M_P0X + j * 5 + 3) = s.ni[j];
      MF(w, slot, M_P0X + j * 5 + 4) = s.ti[j];
    }
}

HK_DEV void integrate_one(float h, Dyn &B, int b) {
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


}  // namespace hk
