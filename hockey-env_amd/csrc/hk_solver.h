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

// Host harness only (hostcheck, HK_HOST_DIAG): how often the velocity loop's island retirement and slot swaps
// ran, so a CPU test can show that its lockstep runs exercised them.  [0] an island retired while another
// of its lane's islands kept iterating, [1] a lane's live contacts were swapped into slots 0/1, [2] an S3 lane
// entered the three-contact shape family, [3] an S2 lane ran a two-contact shape chunk.
#ifdef HK_HOST_DIAG
extern unsigned long long g_hk_host_diag[4];
#define HK_HOST_DIAG_INC(k) (++g_hk_host_diag[k])
#else
#define HK_HOST_DIAG_INC(k) ((void)0)
#endif


// One contact of the solver.  Only what the velocity iterations touch lives here (36 words); the
// position-phase geometry (manifold points / normal, local centres, radii, static origins) is re-read from
// the in-place HBM manifold and the scene when a position pass or InitializeVelocityConstraints needs it,
// so it is not live in registers across the 180-iteration velocity loop.
struct FSlot {
  int bits;  // pair | island << 5 | bodyA << 7 | bodyB << 11 | vcount << 15 | pcount << 17 | type << 19
  float mA, mB, iA, iB, fr;
  float nx, ny;
  float rAx[2], rAy[2], rBx[2], rBy[2], ni[2], ti[2], nm[2], tm[2], bias[2];
  float Kxx, Kxy, Kyy, Nxx, Nxy, Nyy;  // K and its inverse are symmetric (Box2D stores ex.y == ey.x)
  uint32_t sn[4];                       // impulse snapshot for the periodic early exit (velocity_iterations)
};
constexpr int kSlotWords = (int)(sizeof(FSlot) / 4);

HK_DEV int fs_pair(const FSlot &s) { return s.bits & 31; }
HK_DEV int fs_isl(const FSlot &s) { return (s.bits >> 5) & 3; }
HK_DEV int fs_bA(const FSlot &s) { return (s.bits >> 7) & 15; }
HK_DEV int fs_bB(const FSlot &s) { return (s.bits >> 11) & 15; }
HK_DEV int fs_vcount(const FSlot &s) { return (s.bits >> 15) & 3; }
HK_DEV int fs_pcount(const FSlot &s) { return (s.bits >> 17) & 3; }
HK_DEV int fs_type(const FSlot &s) { return (s.bits >> 19) & 3; }

// body access by pair side (pick_a / pick_b / place_a: body A is never the puck, body B is dynamic)
HK_DEV void get_vel_a(const Dyn &B, int b, v2 &v, float &w) {
  v = V(pick_a(B.vx, b, 0.0f), pick_a(B.vy, b, 0.0f));
  w = pick_a(B.w, b, 0.0f);
}
HK_DEV void get_vel_b(const Dyn &B, int b, v2 &v, float &w) {
  v = V(pick_b(B.vx, b), pick_b(B.vy, b));
  w = pick_b(B.w, b);
}
HK_DEV void set_vel_a(Dyn &B, int b, v2 v, float w) {
  place_a(B.vx, b, v.x);
  place_a(B.vy, b, v.y);
  place_a(B.w, b, w);
}
HK_DEV void set_vel_b(Dyn &B, int b, v2 v, float w) {
  place(B.vx, b, v.x);
  place(B.vy, b, v.y);
  place(B.w, b, w);
}
// position of body b (a static body sits at its origin with angle 0)
HK_DEV void get_pos_a(const Dyn &B, int b, v2 &c, float &a) {
  if (b < 3) {
    c = V(pick_a(B.cx, b, 0.0f), pick_a(B.cy, b, 0.0f));
    a = pick_a(B.a, b, 0.0f);
  } else {
    c = V(SLDS.spx[b], SLDS.spy[b]);
    a = 0.0f;
  }
}
HK_DEV void get_pos_b(const Dyn &B, int b, v2 &c, float &a) {
  c = V(pick_b(B.cx, b), pick_b(B.cy, b));
  a = pick_b(B.a, b);
}
HK_DEV void set_pos_a(Dyn &B, int b, v2 c, float a) {
  place_a(B.cx, b, c.x);
  place_a(B.cy, b, c.y);
  place_a(B.a, b, a);
}
HK_DEV void set_pos_b(Dyn &B, int b, v2 c, float a) {
  place(B.cx, b, c.x);
  place(B.cy, b, c.y);
  place(B.a, b, a);
}

// fixture radii of a pair: fixture A is always a polygon (walls, goals, players); B is a player polygon or
// the puck circle (build_scene checks this layout)
HK_DEV float pair_rA() { return kPolyRadius; }
HK_DEV float pair_rB(int bB) { return bB == B_PK ? SC.fx[F_PK].radius : kPolyRadius; }

// position-phase view of a contact's manifold (read in place from HBM)
struct ManGeo {
  int type, count;
  v2 ln, lp, pt[2];
};
HK_DEV ManGeo man_geo(const Arena &w, int p) {
  const Quad *rec = man_rec(w, SLDS.manslot[p]);
  const Quad q0 = rec[0], q1 = rec[1], q2 = rec[2];
  ManGeo g;
  const int meta = __float_as_int(q0.x);
  g.count = meta & 0xff;
  g.type = meta >> 8;
  g.ln = V(q0.y, q0.z);
  g.lp = V(q0.w, q1.x);
  g.pt[0] = V(q1.y, q1.z);
  g.pt[1] = g.count > 1 ? V(q1.w, q2.x) : V(0.0f, 0.0f);
  return g;
}

// b2ContactSolver constructor for one contact
HK_DEV void fslot_load(FSlot &s, const Arena &w, int p, int warm, int isl) {
  const int pa = SLDS.pbodyA[p], pb = SLDS.pbodyB[p];
  const Quad *rec = man_rec(w, SLDS.manslot[p]);
  const int meta = __float_as_int(rec[0].x);
  const int count = meta & 0xff, type = meta >> 8;
  s.bits = p | (isl << 5) | (pa << 7) | (pb << 11) | (count << 15) | (count << 17) | (type << 19);
  s.fr = SLDS.friction[p];
  s.mA = inv_mass(pa); s.mB = inv_mass(pb); s.iA = inv_inertia(pa); s.iB = inv_inertia(pb);
  s.Kxx = s.Kxy = s.Kyy = 0.0f;
  s.Nxx = s.Nxy = s.Nyy = 0.0f;
  s.nx = s.ny = 0.0f;
  Quad q3 = Quad{0.0f, 0.0f, 0.0f, 0.0f};
  if (warm) q3 = rec[3];
  const float mni[2] = {q3.x, q3.z}, mti[2] = {q3.y, q3.w};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const bool on = j < count;
    s.ni[j] = on && warm ? 1.0f * mni[j] : 0.0f;
    s.ti[j] = on && warm ? 1.0f * mti[j] : 0.0f;
    s.rAx[j] = s.rAy[j] = s.rBx[j] = s.rBy[j] = 0.0f;
    s.nm[j] = s.tm[j] = s.bias[j] = 0.0f;
  }
  s.sn[0] = s.sn[1] = s.sn[2] = s.sn[3] = 0u;
}

// InitializeVelocityConstraints for one contact
HK_DEV void fslot_init_velocity(FSlot &s, const Arena &w) {
  const Dyn &B = w.d;
  const float mA = s.mA, mB = s.mB, iA = s.iA, iB = s.iB;
  const int bA = fs_bA(s), bB = fs_bB(s), p = fs_pair(s);
  const float rAr = pair_rA(), rBr = pair_rB(bB);
  v2 cA, cB, vA, vB;
  float aA, aB, wA, wB;
  get_pos_a(B, bA, cA, aA);
  get_pos_b(B, bB, cB, aB);
  get_vel_a(B, bA, vA, wA);
  get_vel_b(B, bB, vB, wB);
  xform xA, xB;
  if (bA >= 3) {  // static body: angle +0, rot_set(+0) == (+0, 1)
    xA.q.s = 0.0f;
    xA.q.c = 1.0f;
  } else {
    xA.q = rot_set(aA);
  }
  xB.q = rot_set(aB);
  xA.p = vsub(cA, mul_rv(xA.q, local_center(bA)));
  xB.p = vsub(cB, mul_rv(xB.q, local_center(bB)));
  // b2WorldManifold::Initialize
  const ManGeo m = man_geo(w, p);
  v2 normal, pts[2];
  if (m.type == 1) {
    normal = mul_rv(xA.q, m.ln);
    v2 plane = mul_xv(xA, m.lp);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      v2 clip = mul_xv(xB, m.pt[i]);
      v2 ca = vadd(clip, vs(rAr - dot(vsub(clip, plane), normal), normal));
      v2 cb = vsub(clip, vs(rBr, normal));
      pts[i] = vs(0.5f, vadd(ca, cb));
    }
  } else {
    normal = mul_rv(xB.q, m.ln);
    v2 plane = mul_xv(xB, m.lp);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      v2 clip = mul_xv(xA, m.pt[i]);
      v2 cb = vadd(clip, vs(rBr - dot(vsub(clip, plane), normal), normal));
      v2 ca = vsub(clip, vs(rAr, normal));
      pts[i] = vs(0.5f, vadd(ca, cb));
    }
    normal = vneg(normal);
  }
  s.nx = normal.x;
  s.ny = normal.y;
  const float re = SLDS.restitution[p];
  const int vcount = fs_vcount(s);
  HK_EV(EV_INIT, 1);
  HK_EV(EV_INIT_PT, vcount);
  HK_EV(EV_INIT_BLOCK, vcount == 2);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < vcount) {
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
      if (vRel < -kVelocityThreshold) s.bias[j] = -re * vRel;
    }
  }
  if (vcount == 2) {
    v2 r1A = V(s.rAx[0], s.rAy[0]), r1B = V(s.rBx[0], s.rBy[0]);
    v2 r2A = V(s.rAx[1], s.rAy[1]), r2B = V(s.rBx[1], s.rBy[1]);
    float rn1A = crs(r1A, normal), rn1B = crs(r1B, normal);
    float rn2A = crs(r2A, normal), rn2B = crs(r2B, normal);
    float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
    float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
    float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
    if (k11 * k11 < 1000.0f * (k11 * k22 - k12 * k12)) {
      s.Kxx = k11; s.Kxy = k12; s.Kyy = k22;
      float a = s.Kxx, b = s.Kxy, c = s.Kxy, d = s.Kyy;
      float det = a * d - b * c;
      if (det != 0.0f) det = 1.0f / det;
      s.Nxx = det * d;
      s.Nxy = -det * c;
      s.Nyy = det * a;
    } else {
      s.bits = (s.bits & ~(3 << 15)) | (1 << 15);  // vcount = 1
    }
  }
}

HK_DEV void fslot_warm_start(const FSlot &s, Dyn &B) {
  const int bA = fs_bA(s), bB = fs_bB(s), vcount = fs_vcount(s);
  HK_EV(EV_WARM_PT, vcount);
  v2 vA, vB;
  float wA, wB;
  get_vel_a(B, bA, vA, wA);
  get_vel_b(B, bB, vB, wB);
  const v2 normal = V(s.nx, s.ny), tangent = crs_vs(normal, 1.0f);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < vcount) {
      v2 P = vadd(vs(s.ni[j], normal), vs(s.ti[j], tangent));
      wA -= s.iA * crs(V(s.rAx[j], s.rAy[j]), P);
      vA = vsub(vA, vs(s.mA, P));
      wB += s.iB * crs(V(s.rBx[j], s.rBy[j]), P);
      vB = vadd(vB, vs(s.mB, P));
    }
  }
  set_vel_a(B, bA, vA, wA);
  set_vel_b(B, bB, vB, wB);
}

// one b2ContactSolver::SolveVelocityConstraints pass over one contact (tangent rows, then the normal row or the
// 2-point block solver), on the two bodies' velocities held in locals; the 2-vector arithmetic is packed fp32
// relative velocity at a contact point, dv = vB + wB x rB - vA - wA x rA (Box2D's operation order)
template <bool kSA>
HK_DEV f2 rel_vel(f2 vA, float wA, f2 vB, float wB, f2 rA, f2 rB) {
  if constexpr (kSA) return (vB + bc(wB) * perp(rB)) - bc(0.0f) * perp(rA);
  else return ((vB + bc(wB) * perp(rB)) - vA) - bc(wA) * perp(rA);
}

// (f2) with Box2D's float operations in Box2D's order.
// kSA: body A is static, so vA = wA = +0 at every solve (the callers reset them) and A's updates are dead.
// The relative velocity then keeps only the operations that can change a bit: u - (+0) == u for every u,
// but u - (+0)*perp(rA) can turn a -0 of u into +0, so that product stays (loop-invariant, hoisted).
// kP: the manifold's point count when the caller knows it for every lane running the call (1 or 2), else 0
// (read per lane): a wave whose lanes all solve one-point contacts skips the block solver's code entirely.
template <bool kSA = false, int kP = 0>
HK_DEV void fslot_solve_velocity_p(FSlot &s, f2 &vA, float &wA, f2 &vB, float &wB) {
  const float mA = s.mA, iA = s.iA, mB = s.mB, iB = s.iB;
  const int vcount = kP ? kP : fs_vcount(s);
  HK_EV(vcount == 1 ? EV_VEL1 : EV_VEL2, 1);
  const f2 normal = f2{s.nx, s.ny}, tangent = f2{1.0f * s.ny, -1.0f * s.nx};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < vcount) {
      const f2 rA = f2{s.rAx[j], s.rAy[j]}, rB = f2{s.rBx[j], s.rBy[j]};
      const f2 dv = rel_vel<kSA>(vA, wA, vB, wB, rA, rB);
      float vt = pdot(dv, tangent) - 0.0f;
      float lambda = s.tm[j] * (-vt);
      float maxF = s.fr * s.ni[j];
      float newI = fclamp(s.ti[j] + lambda, -maxF, maxF);
      lambda = newI - s.ti[j];
      s.ti[j] = newI;
      const f2 P = bc(lambda) * tangent;
      if constexpr (!kSA) {
        vA = vA - bc(mA) * P;
        wA -= iA * pcrs(rA, P);
      }
      vB = vB + bc(mB) * P;
      wB += iB * pcrs(rB, P);
    }
  }
  if (vcount == 1) {
    const f2 rA = f2{s.rAx[0], s.rAy[0]}, rB = f2{s.rBx[0], s.rBy[0]};
    const f2 dv = rel_vel<kSA>(vA, wA, vB, wB, rA, rB);
    float vn = pdot(dv, normal);
    float lambda = -s.nm[0] * (vn - s.bias[0]);
    float newI = fmax2(s.ni[0] + lambda, 0.0f);
    lambda = newI - s.ni[0];
    s.ni[0] = newI;
    const f2 P = bc(lambda) * normal;
    if constexpr (!kSA) {
      vA = vA - bc(mA) * P;
      wA -= iA * pcrs(rA, P);
    }
    vB = vB + bc(mB) * P;
    wB += iB * pcrs(rB, P);
  } else {
    const f2 r1A = f2{s.rAx[0], s.rAy[0]}, r1B = f2{s.rBx[0], s.rBy[0]};
    const f2 r2A = f2{s.rAx[1], s.rAy[1]}, r2B = f2{s.rBx[1], s.rBy[1]};
    v2 a = V(s.ni[0], s.ni[1]);
    const f2 dv1 = rel_vel<kSA>(vA, wA, vB, wB, r1A, r1B);
    const f2 dv2 = rel_vel<kSA>(vA, wA, vB, wB, r2A, r2B);
    float vn1 = pdot(dv1, normal), vn2 = pdot(dv2, normal);
    v2 b;
    b.x = vn1 - s.bias[0];
    b.y = vn2 - s.bias[1];
    b = vsub(b, V(s.Kxx * a.x + s.Kxy * a.y, s.Kxy * a.x + s.Kyy * a.y));
    // Box2D's four cases (both points / point 1 only / point 2 only / none), first one that holds wins.  All four
    // candidates are computed and the winner picked by selects: the same float operations as the if-cascade, without
    // its exec-mask juggling -- the cascade's short blocks were issued predicated anyway (r06, -DHK_ASM_MARKS dump).
    const v2 x1 = vneg(V(s.Nxx * b.x + s.Nxy * b.y, s.Nxy * b.x + s.Nyy * b.y));
    const float x2x = -s.nm[0] * b.x, vn2c = s.Kxy * x2x + b.y;  // case 2: x = (x2x, 0)
    const float x3y = -s.nm[1] * b.y, vn1c = s.Kxy * x3y + b.x;  // case 3: x = (0, x3y)
    const bool ok1 = (x1.x >= 0.0f) & (x1.y >= 0.0f);
    const bool ok2 = (x2x >= 0.0f) & (vn2c >= 0.0f);
    const bool ok3 = (x3y >= 0.0f) & (vn1c >= 0.0f);
    const bool ok4 = (b.x >= 0.0f) & (b.y >= 0.0f);  // case 4: x = (0, 0)
    v2 x;
    x.x = ok1 ? x1.x : (ok2 ? x2x : 0.0f);
    x.y = ok1 ? x1.y : ((!ok2 & ok3) ? x3y : 0.0f);
    const bool ok = ok1 | ok2 | ok3 | ok4;
    (void)vn1;
    (void)vn2;
    if (ok) {
      const v2 d = vsub(x, a);
      const f2 P1 = bc(d.x) * normal, P2 = bc(d.y) * normal;
      if constexpr (!kSA) {
        vA = vA - bc(mA) * (P1 + P2);
        wA -= iA * (pcrs(r1A, P1) + pcrs(r2A, P2));
      }
      vB = vB + bc(mB) * (P1 + P2);
      wB += iB * (pcrs(r1B, P1) + pcrs(r2B, P2));
      s.ni[0] = x.x;
      s.ni[1] = x.y;
    }
  }
}

template <int kP = 0>
HK_DEV void fslot_solve_velocity(FSlot &s, Dyn &B) {
  const int bA = fs_bA(s), bB = fs_bB(s);
  v2 vA, vB;
  float wA, wB;
  get_vel_a(B, bA, vA, wA);
  get_vel_b(B, bB, vB, wB);
  f2 pA = F2(vA), pB = F2(vB);
  fslot_solve_velocity_p<false, kP>(s, pA, wA, pB, wB);
  set_vel_a(B, bA, V2(pA), wA);
  set_vel_b(B, bB, V2(pB), wB);
}

// one NGS position pass over one contact (b2ContactSolver::SolvePositionConstraints body).  In this scene
// SolveTOIPositionConstraints' mass gating is the identity (see solve_toi), so one routine serves both.
// The 2-vector arithmetic is packed (f2): the same float operations in the same order as the scalar form.
HK_DEV float fslot_solve_position(const FSlot &s, Arena &w, float baum, float minSep, const ManGeo &m) {
  HK_MARK(posrow_begin);
  Dyn &B = w.d;
  const float mA = s.mA, mB = s.mB, iA = s.iA, iB = s.iB;
  const int bA = fs_bA(s), bB = fs_bB(s), pcount = fs_pcount(s);
  HK_EV(EV_POS_PT, pcount);
  const f2 lcA = F2(local_center(bA)), lcB = F2(local_center(bB));
  const float rAr = pair_rA(), rBr = pair_rB(bB);
  v2 cA0, cB0;
  float aA, aB;
  get_pos_a(B, bA, cA0, aA);
  get_pos_b(B, bB, cB0, aB);
  f2 cA = F2(cA0), cB = F2(cB0);
  const f2 ln = F2(m.ln), lp = F2(m.lp);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    if (j < pcount) {
      rot qA, qB;
      // a static body stays at angle +0 (iA == 0 keeps aA bit-exact), and rot_set(+0) == (+0, 1)
      if (bA >= 3) {
        qA.s = 0.0f;
        qA.c = 1.0f;
      } else {
        qA = rot_set(aA);
      }
      qB = rot_set(aB);
      const f2 pA = cA - prv(qA, lcA), pB = cB - prv(qB, lcB);
      f2 normal, point;
      float sep;
      if (m.type == 1) {
        normal = prv(qA, ln);
        const f2 plane = prv(qA, lp) + pA;
        const f2 clip = prv(qB, F2(m.pt[j])) + pB;
        sep = pdot(clip - plane, normal) - rAr - rBr;
        point = clip;
      } else {
        normal = prv(qB, ln);
        const f2 plane = prv(qB, lp) + pB;
        const f2 clip = prv(qA, F2(m.pt[j])) + pA;
        sep = pdot(clip - plane, normal) - rAr - rBr;
        point = clip;
        normal = -normal;
      }
      const f2 rA = point - cA, rB = point - cB;
      minSep = fmin2(minSep, sep);
      float C = fclamp(baum * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
      float rnA = pcrs(rA, normal), rnB = pcrs(rB, normal);
      float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      float impulse = K > 0.0f ? -C / K : 0.0f;
      const f2 P = bc(impulse) * normal;
      cA = cA - bc(mA) * P;
      aA -= iA * pcrs(rA, P);
      cB = cB + bc(mB) * P;
      aB += iB * pcrs(rB, P);
    }
  }
  if (bA < 3) set_pos_a(B, bA, V2(cA), aA);
  set_pos_b(B, bB, V2(cB), aB);
  HK_MARK(posrow_end);
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
//   RegSlots<C>: C slots in registers, loops fully unrolled (compile-time slot indices) -- the hot path
//             (islands: C = kIslandC, TOI mini-islands: C = kToiC).
//   HbmSlots: up to kBigC slots in the HBM workspace DevState::ws ([slot][word][arena], lane-contiguous);
//             each visit loads one slot into registers, runs fn and writes it back.  Used by the rare
//             large islands (~1e-5 of arena-steps) so they neither inflate the hot path's register
//             budget nor use private (scratch) memory.
template <int C>
struct RegSlots {
  static constexpr bool kRegister = true;
  static_assert(C >= 2, "the one- and two-contact loops use slots 0 and 1");
  FSlot s[C];
  ManGeo g[C];  // position-phase geometry, loaded once per position loop (load_geo)
  HK_DEV void load_geo(int nc, const Arena &w) {
#pragma unroll
    for (int i = 0; i < C; ++i)
      if (i < nc) g[i] = man_geo(w, fs_pair(s[i]));
  }
  HK_DEV const ManGeo &geo(int i, const FSlot &, const Arena &) const { return g[i]; }
  template <typename Fn>
  HK_DEV void each(int nc, Fn &&fn) {
#pragma unroll
    for (int i = 0; i < C; ++i)
      if (i < nc) fn(s[i], i);
  }
  HK_DEV void set_pair(int nc, int p, int isl) {
#pragma unroll
    for (int q = 0; q < C; ++q) s[q].bits = (q == nc) ? (p | (isl << 5)) : s[q].bits;
  }
};

struct HbmSlots {
  static constexpr bool kRegister = false;
  float *ws;
  int64_t n, a;
  HK_DEV float &word(int i, int k) const { return ws[((int64_t)i * kSlotWords + k) * n + a]; }
  template <typename Fn>
  HK_DEV void each(int nc, Fn &&fn) {
#pragma unroll 1
    for (int i = 0; i < nc; ++i) {
      FSlot t;
      float tw[kSlotWords];
#pragma unroll
      for (int k = 0; k < kSlotWords; ++k) tw[k] = word(i, k);
      __builtin_memcpy(&t, tw, sizeof(FSlot));
      fn(t, i);
      __builtin_memcpy(tw, &t, sizeof(FSlot));
#pragma unroll
      for (int k = 0; k < kSlotWords; ++k) word(i, k) = tw[k];
    }
  }
  HK_DEV void set_pair(int nc, int p, int isl) {
    if (nc < kBigC) word(nc, (int)(offsetof(FSlot, bits) / 4)) = __int_as_float(p | (isl << 5));
  }
  HK_DEV void load_geo(int, const Arena &) {}
  HK_DEV ManGeo geo(int, const FSlot &s, const Arena &w) const { return man_geo(w, fs_pair(s)); }
};
template <typename SL> struct SlotCap;
template <int C> struct SlotCap<RegSlots<C>> { static constexpr int value = C; };
template <> struct SlotCap<HbmSlots> { static constexpr int value = kBigC; };

// ------------------------------------------------------------------------------------------------
// Velocity-loop families and the wave's re-dispatch.  A wave runs the cheapest loop that covers the lanes
// still iterating, and re-picks it every few iterations: most solves exit periodic within 8-16 iterations,
// and the wave's 180-iteration tail then runs only the code its remaining lanes need (one-contact before
// two-contact before the general slot loop; one-point rows without the block solver; the static-body-A
// row).  Every variant computes the same float operations in the same order for the lanes it runs, and a
// lane's snapshot chain is carried across variants of a family, so the result is bit-identical to 180
// iterations of the body-file loop.  A family switch restarts the snapshot (the next comparison is skipped).
// ------------------------------------------------------------------------------------------------
HK_DEV int chunk_end(int it) {
  const int e = it + (it < 24 ? 8 : 32);
  return e < kVelIters ? e : kVelIters;
}
static_assert(kVelIters % 4 == 0, "the snapshot period divides the iteration count");

// One-contact family (the common case, and the usual owner of a wave's 180-iteration tail): the two bodies'
// velocities stay in locals for the whole loop instead of round-tripping through the body file's selects
// every iteration.  A static body's velocity is re-read as +0 at every iteration, exactly what get_vel
// returns in the general loop; the snapshot compares the same values the general loop compares.
// kSA: no running lane has a dynamic body A, so A's velocity row is dropped (fslot_solve_velocity_p).
template <bool kSA, int kP>
HK_DEV void vone_chunk(FSlot &s, bool dynA, uint32_t mA, f2 &vA, float &wA, f2 &vB, float &wB, uint32_t (&sn)[10],
                       int &it, int stop, int first, bool &active) {
  if constexpr (kSA && kP == 1) HK_MARK(vone_begin_s1);
  else if constexpr (kSA && kP == 2) HK_MARK(vone_begin_s2);
  else if constexpr (kSA) HK_MARK(vone_begin_s0);
  else if constexpr (kP == 1) HK_MARK(vone_begin_d1);
  else if constexpr (kP == 2) HK_MARK(vone_begin_d2);
  else HK_MARK(vone_begin_d0);
  for (; it < stop && active; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // a static body A is +0 at every solve (mA = 0 clears it to +0 bit for bit; lane_mask: no exec branch).
      // kSA: no running lane has a dynamic body A, and the static-A row neither reads nor writes A's velocity
      // (nor is it written back for a static body), so the reset is dead there and skipped (r06).
      if constexpr (!kSA) {
        vA = f2{mask_f(vA[0], mA), mask_f(vA[1], mA)};
        wA = mask_f(wA, mA);
      }
      fslot_solve_velocity_p<kSA, kP>(s, vA, wA, vB, wB);
    }
    // kSA: every running lane's body-A words are 0; kP == 1: every running lane solves one point, so the second
    // point's impulses never change in this chunk or a later one of this family (the running set only shrinks and
    // keeps kP == 1) and are left out of the comparison (r06)
    const uint32_t x[10] = {__float_as_uint(vB[0]), __float_as_uint(vB[1]), __float_as_uint(wB),
                            kSA ? 0u : (dynA ? __float_as_uint(vA[0]) : 0u),
                            kSA ? 0u : (dynA ? __float_as_uint(vA[1]) : 0u),
                            kSA ? 0u : (dynA ? __float_as_uint(wA) : 0u), __float_as_uint(s.ni[0]),
                            kP == 1 ? sn[7] : __float_as_uint(s.ni[1]), __float_as_uint(s.ti[0]),
                            kP == 1 ? sn[9] : __float_as_uint(s.ti[1])};
    uint32_t diff = 0u;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      diff |= x[k] ^ sn[k];
      sn[k] = x[k];
    }
    if (it + 3 >= first && diff == 0u) active = false;
  }
  HK_MARK(vone_end);
  if (it >= kVelIters) active = false;  // 180 iterations done
}
HK_DEV void vone_family(FSlot &s, Dyn &B, int &it, bool &active, int first) {
  const bool entered = active;
  const int bA = fs_bA(s), bB = fs_bB(s), vc = fs_vcount(s);
  const bool dynA = bA < 3;
  const uint32_t mA = lane_mask(dynA);
  v2 vA2, vB2;
  float wA, wB;
  get_vel_a(B, bA, vA2, wA);
  get_vel_b(B, bB, vB2, wB);
  f2 vA = F2(vA2), vB = F2(vB2);
  uint32_t sn[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) sn[k] = 0u;
  while (wave_any(active)) {
    const int stop = chunk_end(it);
    const bool sa = !wave_any(active && dynA);
    const bool p1 = !wave_any(active && vc != 1), p2 = !wave_any(active && vc != 2);
    if (sa) {
      if (p1) vone_chunk<true, 1>(s, dynA, mA, vA, wA, vB, wB, sn, it, stop, first, active);
      else if (p2) vone_chunk<true, 2>(s, dynA, mA, vA, wA, vB, wB, sn, it, stop, first, active);
      else vone_chunk<true, 0>(s, dynA, mA, vA, wA, vB, wB, sn, it, stop, first, active);
    } else {
      if (p1) vone_chunk<false, 1>(s, dynA, mA, vA, wA, vB, wB, sn, it, stop, first, active);
      else if (p2) vone_chunk<false, 2>(s, dynA, mA, vA, wA, vB, wB, sn, it, stop, first, active);
      else vone_chunk<false, 0>(s, dynA, mA, vA, wA, vB, wB, sn, it, stop, first, active);
    }
  }
  if (entered) {
    if (dynA) set_vel_a(B, bA, V2(vA), wA);
    set_vel_b(B, bB, V2(vB), wB);
  }
}

// Two-contact family (at most two live contacts; a one-contact lane runs it with contact 1 masked off).
// Each contact keeps its two bodies' velocities in locals; after a contact is solved, the other contact's
// copy of any body it shares (equal body index) is refreshed from it, so every solve reads exactly the
// velocities the body-file loop reads, at 2 selects per shared-body component instead of the body file's
// gather and scatter.  A static body A is +0 at every solve, as get_vel_a returns it.  The snapshot covers
// every island body (each appears in some contact) and both contacts' impulses: the set the general loop
// compares, some bodies twice.  When the two contacts belong to different islands (`sep`: no shared
// dynamic body), each contact's half of the snapshot is its island's whole state, so a contact whose half
// is periodic retires on its own (on0 / on1 false) while the other keeps iterating (see velocity_iterations).
HK_DEV f2 sel2(bool c, f2 a, f2 b) { return f2{c ? a[0] : b[0], c ? a[1] : b[1]}; }
struct TwoState {
  f2 vA0, vB0, vA1, vB1;
  float wA0, wB0, wA1, wB1;
  uint32_t sn[20];
};
// kG: some lane has retired contact 0 (it is then skipped by a per-lane branch; otherwise solved unguarded)
template <int kP0, int kP1, bool kG>
HK_DEV void vtwo_chunk(FSlot &s0, FSlot &s1, TwoState &t, bool two, bool sep, bool dA0, bool dA1, uint32_t mA0,
                       uint32_t mA1, bool a1a0, bool a1b0, bool b1a0, bool b1b0, int &it, int stop, int first,
                       bool &active, bool &on0, bool &on1) {
  // the state lives in this function's own locals for the loop (selects between fields of a by-reference
  // struct turn into pointer selects, which keep the struct in scratch memory)
  f2 vA0 = t.vA0, vB0 = t.vB0, vA1 = t.vA1, vB1 = t.vB1;
  float wA0 = t.wA0, wB0 = t.wB0, wA1 = t.wA1, wB1 = t.wB1;
  uint32_t sn[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) sn[k] = t.sn[k];
  HK_MARK(vtwo_begin);
  for (; it < stop && active; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!kG || on0) {
        vA0 = f2{mask_f(vA0[0], mA0), mask_f(vA0[1], mA0)};  // static A: +0 (lane_mask)
        wA0 = mask_f(wA0, mA0);
        fslot_solve_velocity_p<false, kP0>(s0, vA0, wA0, vB0, wB0);
        vA1 = sel2(a1a0, vA0, sel2(a1b0, vB0, vA1));
        wA1 = a1a0 ? wA0 : (a1b0 ? wB0 : wA1);
        vB1 = sel2(b1a0, vA0, sel2(b1b0, vB0, vB1));
        wB1 = b1a0 ? wA0 : (b1b0 ? wB0 : wB1);
      }
      if (on1) {
        vA1 = f2{mask_f(vA1[0], mA1), mask_f(vA1[1], mA1)};
        wA1 = mask_f(wA1, mA1);
        fslot_solve_velocity_p<false, kP1>(s1, vA1, wA1, vB1, wB1);
        vA0 = sel2(a1a0, vA1, sel2(b1a0, vB1, vA0));
        wA0 = a1a0 ? wA1 : (b1a0 ? wB1 : wA0);
        vB0 = sel2(a1b0, vA1, sel2(b1b0, vB1, vB0));
        wB0 = a1b0 ? wA1 : (b1b0 ? wB1 : wB0);
      }
    }
    const uint32_t x[20] = {__float_as_uint(vB0[0]), __float_as_uint(vB0[1]), __float_as_uint(wB0),
                            dA0 ? __float_as_uint(vA0[0]) : 0u, dA0 ? __float_as_uint(vA0[1]) : 0u,
                            dA0 ? __float_as_uint(wA0) : 0u, __float_as_uint(s0.ni[0]), __float_as_uint(s0.ni[1]),
                            __float_as_uint(s0.ti[0]), __float_as_uint(s0.ti[1]),
                            two ? __float_as_uint(vB1[0]) : 0u, two ? __float_as_uint(vB1[1]) : 0u,
                            two ? __float_as_uint(wB1) : 0u, dA1 ? __float_as_uint(vA1[0]) : 0u,
                            dA1 ? __float_as_uint(vA1[1]) : 0u, dA1 ? __float_as_uint(wA1) : 0u,
                            two ? __float_as_uint(s1.ni[0]) : 0u, two ? __float_as_uint(s1.ni[1]) : 0u,
                            two ? __float_as_uint(s1.ti[0]) : 0u, two ? __float_as_uint(s1.ti[1]) : 0u};
    uint32_t d0 = 0u, d1 = 0u;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      d0 |= x[k] ^ sn[k];
      sn[k] = x[k];
    }
#pragma unroll
    for (int k = 10; k < 20; ++k) {
      d1 |= x[k] ^ sn[k];
      sn[k] = x[k];
    }
    if (it + 3 >= first) {
      if (sep) {
        on0 = on0 && d0 != 0u;
        on1 = on1 && d1 != 0u;
        if (on0 != on1) HK_HOST_DIAG_INC(0);
      } else if ((d0 | d1) == 0u) {
        on0 = false;
        on1 = false;
      }
      if (!on0 && !on1) active = false;
    }
  }
  HK_MARK(vtwo_end);
  if (it >= kVelIters) active = false;
  t.vA0 = vA0; t.vB0 = vB0; t.vA1 = vA1; t.vB1 = vB1;
  t.wA0 = wA0; t.wB0 = wB0; t.wA1 = wA1; t.wB1 = wB1;
#pragma unroll
  for (int k = 0; k < 20; ++k) t.sn[k] = sn[k];
}
// The tail's two-contact shape (r06, scripts/tail_shape_study.c: ~90 % of the two-contact family's iterations from
// iteration 56 on): one island whose contact 1 has a static body A and contact 0's body A as its body B (b1 == a0:
// player-puck, then wall-player), optionally with one-contact lanes riding along.  The shared body has ONE home
// (contact 0's A locals): contact 1 reads it directly and its update is committed back with one select per component
// (riders discard theirs), instead of the generic chunk's per-lane refresh selects after both contacts and its
// exec-mask guard on contact 1; contact 1 runs the static-body-A row.  Riders (two == false) compute a dummy contact
// 1 on their own slot 1, whose impulses are restored at the chunk's end (that slot may hold another island's retired
// contact); their snapshot words of contact 1 are 0, as in the generic chunk.  Every S2 lane's float operations are
// the generic chunk's, in its order, so the result is bit-identical; the snapshot words keep their meaning (contact
// 1's body B words are the shared body's, contact 1's static body A words are 0), so the chain carries across.
template <int kP0, int kP1>
HK_DEV void vtwo_s2_chunk(FSlot &s0, FSlot &s1, TwoState &t, bool two, bool s2, bool dA0, uint32_t mA0, int &it,
                          int stop, int first, bool &active, bool &on0, bool &on1) {
  f2 vA0 = t.vA0, vB0 = t.vB0;
  float wA0 = t.wA0, wB0 = t.wB0;
  uint32_t sn[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) sn[k] = t.sn[k];
  if (active && two) HK_HOST_DIAG_INC(3);
  const float ni0 = s1.ni[0], ni1 = s1.ni[1], ti0 = s1.ti[0], ti1 = s1.ti[1];
  HK_MARK(vtwo_s2_begin);
  for (; it < stop && active; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vA0 = f2{mask_f(vA0[0], mA0), mask_f(vA0[1], mA0)};  // a rider's static A: +0 (lane_mask)
      wA0 = mask_f(wA0, mA0);
      fslot_solve_velocity_p<false, kP0>(s0, vA0, wA0, vB0, wB0);
      f2 vA1 = f2{0.0f, 0.0f}, vB1 = vA0;
      float wA1 = 0.0f, wB1 = wA0;
      fslot_solve_velocity_p<true, kP1>(s1, vA1, wA1, vB1, wB1);
      vA0 = sel2(two, vB1, vA0);
      wA0 = two ? wB1 : wA0;
    }
    const uint32_t x[20] = {__float_as_uint(vB0[0]), __float_as_uint(vB0[1]), __float_as_uint(wB0),
                            dA0 ? __float_as_uint(vA0[0]) : 0u, dA0 ? __float_as_uint(vA0[1]) : 0u,
                            dA0 ? __float_as_uint(wA0) : 0u, __float_as_uint(s0.ni[0]), __float_as_uint(s0.ni[1]),
                            __float_as_uint(s0.ti[0]), __float_as_uint(s0.ti[1]),
                            two ? __float_as_uint(vA0[0]) : 0u, two ? __float_as_uint(vA0[1]) : 0u,
                            two ? __float_as_uint(wA0) : 0u, 0u, 0u, 0u,
                            two ? __float_as_uint(s1.ni[0]) : 0u, two ? __float_as_uint(s1.ni[1]) : 0u,
                            two ? __float_as_uint(s1.ti[0]) : 0u, two ? __float_as_uint(s1.ti[1]) : 0u};
    uint32_t d = 0u;
#pragma unroll
    for (int k = 0; k < 20; ++k) {
      d |= x[k] ^ sn[k];
      sn[k] = x[k];
    }
    if (it + 3 >= first && d == 0u) {  // no lane here is split over two islands (see the dispatch)
      on0 = false;
      on1 = false;
      active = false;
    }
  }
  HK_MARK(vtwo_s2_end);
  if (it >= kVelIters) active = false;
  t.vA0 = vA0; t.vB0 = vB0; t.wA0 = wA0; t.wB0 = wB0;
  // the generic chunks' copy of the shared body, for S2 lanes only: a lane of another shape that finished in an
  // earlier chunk runs this code too (exec is not masked here) and its copies must stay as they are
  t.vB1 = sel2(s2, vA0, t.vB1);
  t.wB1 = s2 ? wA0 : t.wB1;
  s1.ni[0] = two ? s1.ni[0] : ni0;
  s1.ni[1] = two ? s1.ni[1] : ni1;
  s1.ti[0] = two ? s1.ti[0] : ti0;
  s1.ti[1] = two ? s1.ti[1] : ti1;
#pragma unroll
  for (int k = 0; k < 20; ++k) t.sn[k] = sn[k];
}

// The aliased two-contact chunk for mixed waves (r06): every running lane is an S2 lane (b1 == a0, contact 1 static
// A), a "TB" lane (b1 == b0: contact 1's body B is contact 0's body B, e.g. wall-puck then player-puck, or a TOI
// mini-island's two static contacts on one body), or a one-contact rider -- with any point counts (scripts/
// tail_shape_study.c: the slowest waves mostly mix S2 lanes whose contact 1 has one and two points, or run TB
// lanes).  The shared body has one home per lane (contact 0's A for S2, its B for TB): contact 1 reads it through one
// select per component and commits its update with one per component and shape, instead of the generic chunk's
// refresh selects after both contacts and its exec-mask guard; contact 1's own body A lives in locals (static for
// S2, +0 by its lane mask).  Riders as in vtwo_s2_chunk.  Bit-identical to the generic chunk for every lane.
template <int kP0, int kP1>
HK_DEV void vtwo_alias_chunk(FSlot &s0, FSlot &s1, TwoState &t, bool two, bool s2, bool tb, bool dA0, bool dA1,
                             uint32_t mA0, uint32_t mA1, int &it, int stop, int first, bool &active, bool &on0,
                             bool &on1) {
  f2 vA0 = t.vA0, vB0 = t.vB0, vA1 = t.vA1;
  float wA0 = t.wA0, wB0 = t.wB0, wA1 = t.wA1;
  uint32_t sn[20];
#pragma unroll
  for (int k = 0; k < 20; ++k) sn[k] = t.sn[k];
  if (active && two) HK_HOST_DIAG_INC(3);
  const float ni0 = s1.ni[0], ni1 = s1.ni[1], ti0 = s1.ti[0], ti1 = s1.ti[1];
  HK_MARK(vtwo_alias_begin);
  for (; it < stop && active; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vA0 = f2{mask_f(vA0[0], mA0), mask_f(vA0[1], mA0)};
      wA0 = mask_f(wA0, mA0);
      fslot_solve_velocity_p<false, kP0>(s0, vA0, wA0, vB0, wB0);
      f2 vB1 = sel2(s2, vA0, vB0);  // the shared body (a rider: a dummy copy)
      float wB1 = s2 ? wA0 : wB0;
      vA1 = f2{mask_f(vA1[0], mA1), mask_f(vA1[1], mA1)};
      wA1 = mask_f(wA1, mA1);
      fslot_solve_velocity_p<false, kP1>(s1, vA1, wA1, vB1, wB1);
      vA0 = sel2(s2, vB1, vA0);
      wA0 = s2 ? wB1 : wA0;
      vB0 = sel2(tb, vB1, vB0);
      wB0 = tb ? wB1 : wB0;
    }
    const f2 sh = sel2(s2, vA0, vB0);
    const float wsh = s2 ? wA0 : wB0;
    const uint32_t x[20] = {__float_as_uint(vB0[0]), __float_as_uint(vB0[1]), __float_as_uint(wB0),
                            dA0 ? __float_as_uint(vA0[0]) : 0u, dA0 ? __float_as_uint(vA0[1]) : 0u,
                            dA0 ? __float_as_uint(wA0) : 0u, __float_as_uint(s0.ni[0]), __float_as_uint(s0.ni[1]),
                            __float_as_uint(s0.ti[0]), __float_as_uint(s0.ti[1]),
                            two ? __float_as_uint(sh[0]) : 0u, two ? __float_as_uint(sh[1]) : 0u,
                            two ? __float_as_uint(wsh) : 0u, dA1 ? __float_as_uint(vA1[0]) : 0u,
                            dA1 ? __float_as_uint(vA1[1]) : 0u, dA1 ? __float_as_uint(wA1) : 0u,
                            two ? __float_as_uint(s1.ni[0]) : 0u, two ? __float_as_uint(s1.ni[1]) : 0u,
                            two ? __float_as_uint(s1.ti[0]) : 0u, two ? __float_as_uint(s1.ti[1]) : 0u};
    uint32_t d = 0u;
#pragma unroll
    for (int k = 0; k < 20; ++k) {
      d |= x[k] ^ sn[k];
      sn[k] = x[k];
    }
    if (it + 3 >= first && d == 0u) {  // no lane here is split over two islands (see the dispatch)
      on0 = false;
      on1 = false;
      active = false;
    }
  }
  HK_MARK(vtwo_alias_end);
  if (it >= kVelIters) active = false;
  const bool shaped = s2 || tb;  // only these lanes' contact-1 copies changed (others ran no iteration here or are riders)
  t.vA0 = vA0; t.vB0 = vB0; t.wA0 = wA0; t.wB0 = wB0;
  t.vB1 = sel2(shaped, sel2(s2, vA0, vB0), t.vB1);
  t.wB1 = shaped ? (s2 ? wA0 : wB0) : t.wB1;
  t.vA1 = sel2(tb, vA1, t.vA1);
  t.wA1 = tb ? wA1 : t.wA1;
  s1.ni[0] = two ? s1.ni[0] : ni0;
  s1.ni[1] = two ? s1.ni[1] : ni1;
  s1.ti[0] = two ? s1.ti[0] : ti0;
  s1.ti[1] = two ? s1.ti[1] : ti1;
#pragma unroll
  for (int k = 0; k < 20; ++k) t.sn[k] = sn[k];
}

// runs until every lane is done or no running lane has both contacts live (then the one-contact family takes
// over).  on0 / on1 in: the lane's contacts that iterate (on1 == two); out: the ones still unfinished.
HK_DEV void vtwo_family(FSlot &s0, FSlot &s1, Dyn &B, bool two, int &it, bool &active, int first, bool &on0,
                        bool &on1) {
  const bool entered = active;
  const int a0 = fs_bA(s0), b0 = fs_bB(s0);
  const int a1 = two ? fs_bA(s1) : 15, b1 = two ? fs_bB(s1) : 15;  // 15: matches no body
  const bool dA0 = a0 < 3, dA1 = a1 < 3;
  const uint32_t mA0 = lane_mask(dA0), mA1 = lane_mask(dA1);
  const bool a1a0 = a1 == a0, a1b0 = a1 == b0, b1a0 = b1 == a0, b1b0 = b1 == b0;
  const bool sep = two && fs_isl(s0) != fs_isl(s1);
  const int vc0 = fs_vcount(s0), vc1 = two ? fs_vcount(s1) : 1;
  TwoState t;
  v2 q;
  get_vel_a(B, a0, q, t.wA0);
  t.vA0 = F2(q);
  get_vel_b(B, b0, q, t.wB0);
  t.vB0 = F2(q);
  get_vel_a(B, a1, q, t.wA1);
  t.vA1 = F2(q);
  get_vel_b(B, b1, q, t.wB1);
  t.vB1 = F2(q);
#pragma unroll
  for (int k = 0; k < 20; ++k) t.sn[k] = 0u;
  // the S2 shape (see vtwo_s2_chunk): one island, contact 1's body A static and its body B contact 0's body A
  const bool s2 = two && !sep && !dA1 && b1a0;
  const bool tb = two && !sep && b1b0;  // TB lanes (see vtwo_alias_chunk)
  while (wave_any(active) && wave_any(active && on0 && on1)) {
    const int stop = chunk_end(it);
    // S2 chunk: every running lane is an S2 lane with both contacts live, or a one-contact rider (two == false)
    const bool s2ok = !wave_any(active && (!on0 || (two && !(s2 && on1))));
    if (s2ok && !wave_any(active && two && vc1 != 1)) {
      if (!wave_any(active && vc0 != 1))
        vtwo_s2_chunk<1, 1>(s0, s1, t, two, s2, dA0, mA0, it, stop, first, active, on0, on1);
      else
        vtwo_s2_chunk<0, 1>(s0, s1, t, two, s2, dA0, mA0, it, stop, first, active, on0, on1);
    } else if (s2ok && !wave_any(active && two && vc1 != 2)) {
      if (!wave_any(active && vc0 != 1))
        vtwo_s2_chunk<1, 2>(s0, s1, t, two, s2, dA0, mA0, it, stop, first, active, on0, on1);
      else
        vtwo_s2_chunk<0, 2>(s0, s1, t, two, s2, dA0, mA0, it, stop, first, active, on0, on1);
    } else if (!wave_any(active && (!on0 || (two && !((s2 || tb) && on1))))) {
      // aliased chunk: S2 and TB lanes with both contacts live, and one-contact riders
      const bool p0 = !wave_any(active && vc0 != 1), p1 = !wave_any(active && two && vc1 != 1);
      if (p0 && p1)
        vtwo_alias_chunk<1, 1>(s0, s1, t, two, s2, tb, dA0, dA1, mA0, mA1, it, stop, first, active, on0, on1);
      else if (p0)
        vtwo_alias_chunk<1, 0>(s0, s1, t, two, s2, tb, dA0, dA1, mA0, mA1, it, stop, first, active, on0, on1);
      else if (p1)
        vtwo_alias_chunk<0, 1>(s0, s1, t, two, s2, tb, dA0, dA1, mA0, mA1, it, stop, first, active, on0, on1);
      else
        vtwo_alias_chunk<0, 0>(s0, s1, t, two, s2, tb, dA0, dA1, mA0, mA1, it, stop, first, active, on0, on1);
    } else if (wave_any(active && !on0))
      vtwo_chunk<0, 0, true>(s0, s1, t, two, sep, dA0, dA1, mA0, mA1, a1a0, a1b0, b1a0, b1b0, it, stop, first, active, on0,
                             on1);
    else if (!wave_any(active && (vc0 != 1 || vc1 != 1)))
      vtwo_chunk<1, 1, false>(s0, s1, t, two, sep, dA0, dA1, mA0, mA1, a1a0, a1b0, b1a0, b1b0, it, stop, first, active, on0,
                              on1);
    // a wave whose running lanes agree on both point counts runs the rows without the other count's code (a
    // lane of a one-contact island rides along with contact 1 masked off, whatever kP1 says)
    else if (!wave_any(active && (vc0 != 1 || (two && vc1 != 2))))
      vtwo_chunk<1, 2, false>(s0, s1, t, two, sep, dA0, dA1, mA0, mA1, a1a0, a1b0, b1a0, b1b0, it, stop, first, active, on0,
                              on1);
    else if (!wave_any(active && (vc0 != 2 || (two && vc1 != 1))))
      vtwo_chunk<2, 1, false>(s0, s1, t, two, sep, dA0, dA1, mA0, mA1, a1a0, a1b0, b1a0, b1b0, it, stop, first, active, on0,
                              on1);
    else if (!wave_any(active && (vc0 != 2 || (two && vc1 != 2))))
      vtwo_chunk<2, 2, false>(s0, s1, t, two, sep, dA0, dA1, mA0, mA1, a1a0, a1b0, b1a0, b1b0, it, stop, first, active, on0,
                              on1);
    else
      vtwo_chunk<0, 0, false>(s0, s1, t, two, sep, dA0, dA1, mA0, mA1, a1a0, a1b0, b1a0, b1b0, it, stop, first, active, on0,
                              on1);
  }
  if (entered) {
    if (dA0) set_vel_a(B, a0, V2(t.vA0), t.wA0);
    set_vel_b(B, b0, V2(t.vB0), t.wB0);
    if (two) {
      if (dA1) set_vel_a(B, a1, V2(t.vA1), t.wA1);
      set_vel_b(B, b1, V2(t.vB1), t.wB1);
    }
  }
}

// The tail's three-contact shape (r06, scripts/tail_shape_study.c): one island of three one-point contacts, slot 0
// = (static, X), slot 1 = (Y, X), slot 2 = (static, Y) -- wall-puck, player-puck, wall-player -- optionally with
// riders: one-contact lanes (their contact swapped into slot 0) and S2 two-contact lanes (player-puck, wall-player:
// their live contacts swapped into slots 0 and 1, as the two-contact family holds them; the slowest waves of the
// bench workload mostly hold S3 and S2 lanes together).  X and Y live in locals, aliased at compile time, instead of
// the general family's body-file gathers and scatters (~30 selects per contact): slot 0 runs the generic row on
// (A0, X) (a rider's own bodies; an S3 lane's A0 is static, +0), slot 1 the dynamic row on (Y, X) -- an S2 lane's
// on (+0, A0), its static body A and its body B, contact 0's body A, by one select per component in and out (the
// row with a +0 body A is bit-identical to the static-body-A row: see fslot_solve_velocity_p) -- whose update of X a
// non-S3 lane discards, slot 2 the static-body-A row on Y, S3 lanes only in effect.  Non-S3 lanes' slot 2
// impulses, and one-contact riders' slot 1 impulses, are restored at the end (another island's retired contacts may
// sit there).  The snapshot covers X, Y, A0 and the impulses of the slots the lane solves: the island's whole
// state, so the periodic exit stays exact; this family starts its own chain.  Each lane's float operations are the
// general / two-contact families', in their order.  Runs while some S3 lane iterates.
template <int kP0, int kP1>
HK_DEV void vthree_s3_chunk(FSlot &s0, FSlot &s1, FSlot &s2, bool s3, bool s2l, uint32_t mA0, uint32_t mY, bool dA0,
                            f2 &vA0, float &wA0, f2 &vX, float &wX, f2 &vY, float &wY, uint32_t (&sn)[19], int &it,
                            int stop, int first, bool &active) {
  HK_MARK(vthree_begin);
  for (; it < stop && active; it += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vA0 = f2{mask_f(vA0[0], mA0), mask_f(vA0[1], mA0)};  // static A (every S3 lane, static riders): +0
      wA0 = mask_f(wA0, mA0);
      fslot_solve_velocity_p<false, kP0>(s0, vA0, wA0, vX, wX);
      f2 vB1 = sel2(s2l, vA0, vX);  // an S2 lane's contact 1 acts on its body A0
      float wB1 = s2l ? wA0 : wX;
      vY = f2{mask_f(vY[0], mY), mask_f(vY[1], mY)};  // an S2 lane's contact 1 has a static body A: +0
      wY = mask_f(wY, mY);
      fslot_solve_velocity_p<false, kP1>(s1, vY, wY, vB1, wB1);
      vX = sel2(s3, vB1, vX);
      wX = s3 ? wB1 : wX;
      vA0 = sel2(s2l, vB1, vA0);
      wA0 = s2l ? wB1 : wA0;
      f2 vA2 = f2{0.0f, 0.0f};
      float wA2 = 0.0f;
      fslot_solve_velocity_p<true, 1>(s2, vA2, wA2, vY, wY);
    }
    const bool sl1 = s3 || s2l;  // lanes that solve slot 1
    const uint32_t x[19] = {__float_as_uint(vX[0]), __float_as_uint(vX[1]), __float_as_uint(wX),
                            dA0 ? __float_as_uint(vA0[0]) : 0u, dA0 ? __float_as_uint(vA0[1]) : 0u,
                            dA0 ? __float_as_uint(wA0) : 0u, __float_as_uint(s0.ni[0]), __float_as_uint(s0.ni[1]),
                            __float_as_uint(s0.ti[0]), __float_as_uint(s0.ti[1]),
                            s3 ? __float_as_uint(vY[0]) : 0u, s3 ? __float_as_uint(vY[1]) : 0u,
                            s3 ? __float_as_uint(wY) : 0u, sl1 ? __float_as_uint(s1.ni[0]) : 0u,
                            sl1 ? __float_as_uint(s1.ti[0]) : 0u, sl1 ? __float_as_uint(s1.ni[1]) : 0u,
                            sl1 ? __float_as_uint(s1.ti[1]) : 0u, s3 ? __float_as_uint(s2.ni[0]) : 0u,
                            s3 ? __float_as_uint(s2.ti[0]) : 0u};
    uint32_t d = 0u;
#pragma unroll
    for (int k = 0; k < 19; ++k) {
      d |= x[k] ^ sn[k];
      sn[k] = x[k];
    }
    if (it + 3 >= first && d == 0u) active = false;
  }
  HK_MARK(vthree_end);
  if (it >= kVelIters) active = false;
}
HK_DEV bool s3_shape(const FSlot &s0, const FSlot &s1, const FSlot &s2) {
  return fs_bA(s0) >= 3 && fs_bA(s2) >= 3 && fs_bA(s1) < 3 && fs_bB(s0) == fs_bB(s1) && fs_bA(s1) == fs_bB(s2) &&
         fs_vcount(s0) == 1 && fs_vcount(s1) == 1 && fs_vcount(s2) == 1;
}
// S2 pair from slot bits: contact 1 (bits1) static A, its body B contact 0's body A, one island
HK_DEV bool s2_bits(int bits0, int bits1) {
  const int a0 = (bits0 >> 7) & 15, a1 = (bits1 >> 7) & 15, b1 = (bits1 >> 11) & 15;
  return a1 >= 3 && b1 == a0 && ((bits0 >> 5) & 3) == ((bits1 >> 5) & 3);
}
// s3: an S3 lane; s2l: an S2 lane (its contacts in slots 0 and 1); else a one-contact rider (slot 0)
HK_DEV void vthree_s3_family(FSlot &s0, FSlot &s1, FSlot &s2, Dyn &B, bool s3, bool s2l, int &it, bool &active,
                             int first) {
  const bool entered = active;
  const int a0 = fs_bA(s0), x = fs_bB(s0), y = s3 ? fs_bA(s1) : x;
  const bool dA0 = a0 < 3;
  const uint32_t mA0 = lane_mask(dA0), mY = lane_mask(s3);
  v2 q;
  float wA0, wX, wY;
  get_vel_a(B, a0, q, wA0);
  f2 vA0 = F2(q);
  get_vel_b(B, x, q, wX);
  f2 vX = F2(q);
  get_vel_b(B, y, q, wY);
  f2 vY = F2(q);
  const float ni1[2] = {s1.ni[0], s1.ni[1]}, ti1[2] = {s1.ti[0], s1.ti[1]};
  const float ni2[2] = {s2.ni[0], s2.ni[1]}, ti2[2] = {s2.ti[0], s2.ti[1]};
  uint32_t sn[19];
#pragma unroll
  for (int k = 0; k < 19; ++k) sn[k] = 0u;
  // the point-count variant is picked once per family entry (the running set only shrinks, so one-point stays
  // one-point), each in its own loop: picking it per chunk inside one loop made the kernel spill (both variants'
  // invariants hoisted together; 16 -> 152 B of scratch per lane, make resource-usage)
  if (!wave_any(active && (fs_vcount(s0) != 1 || (s2l && fs_vcount(s1) != 1)))) {
    while (wave_any(active && s3)) {
      const int stop = chunk_end(it);
      vthree_s3_chunk<1, 1>(s0, s1, s2, s3, s2l, mA0, mY, dA0, vA0, wA0, vX, wX, vY, wY, sn, it, stop, first, active);
    }
  } else {
    while (wave_any(active && s3)) {
      const int stop = chunk_end(it);
      vthree_s3_chunk<0, 0>(s0, s1, s2, s3, s2l, mA0, mY, dA0, vA0, wA0, vX, wX, vY, wY, sn, it, stop, first, active);
    }
  }
  if (entered) {
    if (dA0) set_vel_a(B, a0, V2(vA0), wA0);
    set_vel_b(B, x, V2(vX), wX);
    if (s3) set_vel_b(B, y, V2(vY), wY);
  }
  const bool sl1 = s3 || s2l;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    s1.ni[j] = sl1 ? s1.ni[j] : ni1[j];
    s1.ti[j] = sl1 ? s1.ti[j] : ti1[j];
    s2.ni[j] = s3 ? s2.ni[j] : ni2[j];
    s2.ti[j] = s3 ? s2.ti[j] : ti2[j];
  }
}

// General family: the slot loop over the body file (any island size, register or HBM slots).  Islands
// share no dynamic body, so each island's state (its bodies' velocities, its contacts' impulses) evolves
// on its own: an island whose state is periodic retires on its own (its slots leave `live` and are no
// longer solved; its state at iteration 179 is the current one), while the lane's other islands keep
// iterating.  With `leave`, it returns after a chunk once no running lane has more than two live contacts.
// kP == 1: every live contact of every running lane has one point (the caller checks at entry; the running set and
// the live contacts only shrink), so the rows skip the block solver and the per-slot point-count branch (r06).
template <typename SL, int kP = 0>
HK_DEV void vgen_family(SL &S, Dyn &B, int nc, uint32_t &live, const int (&isl_of)[3], int &it, bool &active,
                        int first, bool leave) {
  uint32_t sb[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) sb[k] = 0u;
  uint32_t im0 = 0u, im1 = 0u, im2 = 0u;  // slots of islands 0, 1, 2
  S.each(nc, [&](FSlot &s, int i) {
    s.sn[0] = s.sn[1] = s.sn[2] = s.sn[3] = 0u;
    const int k = fs_isl(s);
    im0 |= k == 0 ? 1u << i : 0u;
    im1 |= k == 1 ? 1u << i : 0u;
    im2 |= k == 2 ? 1u << i : 0u;
  });
  while (wave_any(active)) {
    if (leave && !wave_any(active && __popc(live) > 2)) return;
    const int stop = chunk_end(it);
    HK_MARK(vit_begin);
    for (; it < stop && active; it += 4) {  // 4 iterations per trip: the snapshot period
#pragma unroll
      for (int u = 0; u < 4; ++u)
        S.each(nc, [&](FSlot &s, int i) {
          if ((live >> i) & 1u) fslot_solve_velocity<kP>(s, B);
        });
      uint32_t d0 = 0u, d1 = 0u, d2 = 0u;  // per-island snapshot differences
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const uint32_t x = __float_as_uint(B.vx[b]), y = __float_as_uint(B.vy[b]), z = __float_as_uint(B.w[b]);
        const uint32_t d = (x ^ sb[3 * b]) | (y ^ sb[3 * b + 1]) | (z ^ sb[3 * b + 2]);
        d0 |= isl_of[b] == 0 ? d : 0u;
        d1 |= isl_of[b] == 1 ? d : 0u;
        d2 |= isl_of[b] == 2 ? d : 0u;
        sb[3 * b] = x;
        sb[3 * b + 1] = y;
        sb[3 * b + 2] = z;
      }
      S.each(nc, [&](FSlot &s, int) {
        const uint32_t x0 = __float_as_uint(s.ni[0]), x1 = __float_as_uint(s.ni[1]);
        const uint32_t x2 = __float_as_uint(s.ti[0]), x3 = __float_as_uint(s.ti[1]);
        const uint32_t d = (x0 ^ s.sn[0]) | (x1 ^ s.sn[1]) | (x2 ^ s.sn[2]) | (x3 ^ s.sn[3]);
        const int k = fs_isl(s);
        d0 |= k == 0 ? d : 0u;
        d1 |= k == 1 ? d : 0u;
        d2 |= k == 2 ? d : 0u;
        s.sn[0] = x0;
        s.sn[1] = x1;
        s.sn[2] = x2;
        s.sn[3] = x3;
      });
      if (it + 3 >= first) {
        const uint32_t before = live;
        live &= (d0 == 0u ? ~im0 : ~0u) & (d1 == 0u ? ~im1 : ~0u) & (d2 == 0u ? ~im2 : ~0u);
        if (live == 0u) active = false;
        else if (live != before) HK_HOST_DIAG_INC(0);
      }
    }
    HK_MARK(vit_end);
    if (it >= kVelIters) active = false;
  }
}

// per-lane exchange of register slots i (compile-time) and j (runtime, j >= i), word by word through selects.
// The words are copied out and back with memcpy (no type-punned pointer: strict-aliasing clean on the host and
// sanitizer builds; SROA keeps every word in a register on the device).
template <int C>
HK_DEV void slot_swap(RegSlots<C> &S, int i, int j) {
  static_assert(sizeof(FSlot) == kSlotWords * 4, "FSlot is kSlotWords words");
  uint32_t a[kSlotWords];
  __builtin_memcpy(a, &S.s[i], sizeof(FSlot));
#pragma unroll
  for (int q = 0; q < C; ++q) {
    if (q <= i) continue;
    uint32_t b[kSlotWords];
    __builtin_memcpy(b, &S.s[q], sizeof(FSlot));
    const bool sw = j == q;
#pragma unroll
    for (int k = 0; k < kSlotWords; ++k) {
      const uint32_t x = a[k], y = b[k];
      a[k] = sw ? y : x;
      b[k] = sw ? x : y;
    }
    __builtin_memcpy(&S.s[q], b, sizeof(FSlot));
  }
  __builtin_memcpy(&S.s[i], a, sizeof(FSlot));
}

// 180 velocity iterations over nc slots, with the exact periodic early exit.  Register slots: the wave walks
// the families general -> two -> one as the lanes' LIVE contacts allow (contacts of islands that have not
// yet become periodic; islands retire one by one, see vgen_family / vtwo_family).  The one- and two-contact
// families run on slots 0 and 1: a lane whose live contacts sit elsewhere has them swapped there (in slot
// order, so an island's Gauss-Seidel order is kept) and back afterwards.  HBM slots: the general loop.
// isl_of[b]: island of dynamic body b (-1: none).
template <typename SL>
HK_DEV int velocity_iterations(SL &S, Dyn &B, int nc, const int (&isl_of)[3], PhaseT &T) {
  int it = 0;
  uint32_t live = nc > 0 ? (1u << nc) - 1u : 0u;
  bool active = nc > 0;
  int first = 7;  // the first comparison against a snapshot taken by this loop (it + 3 == 7)
  if constexpr (SL::kRegister) {
    static_assert(SlotCap<SL>::value >= 2, "the one- and two-contact families use slots 0 and 1");
    while (wave_any(active)) {
      const int nl = __popc(live);
      HK_FAM_T0();
      // S3 family (vthree_s3_family): every running lane is an S3 lane (its three live contacts in slots 0-2), an
      // S2 lane (two live contacts) or a one-contact rider
      bool s3 = false, s2l = false, s3ok = false;
      int j0 = 0, j1 = 1;
      if constexpr (SlotCap<SL>::value >= 3) {
        s3 = active && nl == 3 && live == 7u && s3_shape(S.s[0], S.s[1], S.s[2]);
        j0 = nl >= 1 ? __ffs(live) - 1 : 0;
        j1 = nl >= 2 ? __ffs(live & (live - 1u)) - 1 : 1;
        if (wave_any(s3)) {
          int b0 = 0, b1 = 0;  // the live slots' bits, by select (slot indices are runtime per lane)
#pragma unroll
          for (int q = 0; q < SlotCap<SL>::value; ++q) {
            b0 = q == j0 ? S.s[q].bits : b0;
            b1 = q == j1 ? S.s[q].bits : b1;
          }
          s2l = active && nl == 2 && s2_bits(b0, b1);
        }
        s3ok = wave_any(s3) && !wave_any(active && !s3 && !s2l && nl != 1);
      }
      if (s3ok) {
        if constexpr (SlotCap<SL>::value >= 3) {
          // riders' and S2 lanes' live contacts to slots 0 (and 1), in slot order, as the two-contact family has them
          const bool mv0 = !s3 && j0 != 0, mv1 = s2l && j1 != 1;
          const bool any0 = wave_any(active && mv0), any1 = wave_any(mv1);
          if (any0) slot_swap(S, 0, mv0 ? j0 : 0);
          if (any1) slot_swap(S, 1, mv1 ? j1 : 1);
          const bool entered = active;
          if (s3) HK_HOST_DIAG_INC(2);
          vthree_s3_family(S.s[0], S.s[1], S.s[2], B, s3, s2l, it, active, first);
          live = entered && !active ? 0u : live;
          if (any1) slot_swap(S, 1, mv1 ? j1 : 1);
          if (any0) slot_swap(S, 0, mv0 ? j0 : 0);
          HK_FAM_ADD(T, 0);
        }
      } else if (wave_any(active && nl > 2)) {
        bool p1 = true;  // every live contact one-point
        S.each(nc, [&](FSlot &s, int i) { p1 = p1 && (((live >> i) & 1u) == 0u || fs_vcount(s) == 1); });
        if (!wave_any(active && !p1)) vgen_family<SL, 1>(S, B, nc, live, isl_of, it, active, first, true);
        else vgen_family<SL, 0>(S, B, nc, live, isl_of, it, active, first, true);
        HK_FAM_ADD(T, 0);
      } else {
        const bool fam2 = wave_any(active && nl > 1);
        const int j0 = nl > 0 ? __ffs(live) - 1 : 0;
        const int j1 = nl > 1 ? __ffs(live & (live - 1u)) - 1 : 1;
        const bool perm = wave_any(active && (j0 != 0 || (fam2 && j1 != 1)));
        if (perm) {
          if (active && (j0 != 0 || (fam2 && j1 != 1))) HK_HOST_DIAG_INC(1);
          slot_swap(S, 0, j0);
          if (fam2) slot_swap(S, 1, j1);
        }
        if (fam2) {
          bool on0 = active, on1 = active && nl > 1;
          vtwo_family(S.s[0], S.s[1], B, nl > 1, it, active, first, on0, on1);
          live &= (on0 ? ~0u : ~(1u << j0)) & (nl > 1 && !on1 ? ~(1u << j1) : ~0u);
          HK_FAM_ADD(T, 1);
        } else {
          const bool entered = active;
          vone_family(S.s[0], B, it, active, first);
          live = entered ? 0u : live;
          HK_FAM_ADD(T, 2);
        }
        if (perm) {
          if (fam2) slot_swap(S, 1, j1);
          slot_swap(S, 0, j0);
        }
      }
      active = live != 0u && it < kVelIters;
      first = it + 7;  // the next family starts a fresh snapshot
    }
  } else {
    vgen_family(S, B, nc, live, isl_of, it, active, first, false);
  }
  return it;
}

HK_DEV void fslot_store(const FSlot &s, Arena &w) {  // b2ContactSolver::StoreImpulses (j < pointCount)
  float *q3 = reinterpret_cast<float *>(man_rec(w, SLDS.manslot[fs_pair(s)]) + 3);
  const int vcount = fs_vcount(s);
  if (vcount == 2) {
    *reinterpret_cast<Quad *>(q3) = Quad{s.ni[0], s.ti[0], s.ni[1], s.ti[1]};
  } else if (vcount == 1) {
    q3[0] = s.ni[0];
    q3[1] = s.ti[0];
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
