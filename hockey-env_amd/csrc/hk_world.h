// hk_world.h -- per-lane world: narrow phase, GJK/TOI, sequential-impulse solver, islands, env laws.
// Included by hk_kernels.hip after the definition of the __constant__ scene `g_scene`.
// Reference mapping (hockey/hockey_env.py) is given per function; Box2D 2.3 function names are the
// third-party algorithm restated for this scene.
#pragma once
#include "hk_core.h"

namespace hk {

#define SC g_scene

struct Body {
  v2 lc, c0, c;
  float a0, a, alpha0;
  xform xf;
  v2 v;
  float w;
  v2 force;
  float torque;
  float mass, invMass, I, invI;
  float ld, ad, sleep;
  int awake, dynamic, island_flag, island_index;
};

struct Manifold {
  v2 pt_lp[2];
  float ni[2], ti[2];
  uint32_t id[2];
  v2 ln, lp;
  int type, count;  // type 1 = faceA, 2 = faceB
};

struct Contact {
  int touching, enabled, toi_flag, toi_count, island_flag;
  float toi;
  Manifold m;
};

struct World {
  Body b[NB];
  Contact c[NP];
  int keep_mode, max_t, time, done, winner, has1, has2, vel_ref;
  int n_toi, overflow;
};

// ------------------------------------------------------------------------------------------------
// body helpers (b2Body.h / b2Body.cpp)
// ------------------------------------------------------------------------------------------------
HK_DEV void set_transform(Body &b, v2 p, float angle) {
  b.xf.q = rot_set(angle);
  b.xf.p = p;
  b.c = mul_xv(b.xf, b.lc);
  b.a = angle;
  b.c0 = b.c;
  b.a0 = angle;
}
HK_DEV void set_awake(Body &b, int flag) {
  if (flag) {
    if (!b.awake) { b.awake = 1; b.sleep = 0.0f; }
  } else {
    b.awake = 0;
    b.sleep = 0.0f;
    b.v = V(0.0f, 0.0f);
    b.w = 0.0f;
    b.force = V(0.0f, 0.0f);
    b.torque = 0.0f;
  }
}
HK_DEV void set_linear_velocity(Body &b, v2 v) {
  if (!b.dynamic) return;
  if (dot(v, v) > 0.0f) set_awake(b, 1);
  b.v = v;
}
HK_DEV void set_angular_velocity(Body &b, float w) {
  if (!b.dynamic) return;
  if (w * w > 0.0f) set_awake(b, 1);
  b.w = w;
}
HK_DEV void apply_force(Body &b, v2 f) {
  if (!b.awake) set_awake(b, 1);
  if (b.awake) b.force = vadd(b.force, f);
}
HK_DEV void apply_torque(Body &b, float t) {
  if (!b.awake) set_awake(b, 1);
  if (b.awake) b.torque += t;
}
HK_DEV void synchronize_transform(Body &b) {
  b.xf.q = rot_set(b.a);
  b.xf.p = vsub(b.c, mul_rv(b.xf.q, b.lc));
}

// static bodies (origin, angle 0, zero mass) and dynamic-body mass properties from the scene
HK_DEV void init_static_bodies(World &w) {
  for (int i = B_WT; i < NB; ++i) {
    Body &b = w.b[i];
    b.lc = V(0.0f, 0.0f);
    b.xf.p = V(SC.spx[i], SC.spy[i]);
    b.xf.q = rot_set(0.0f);
    b.c = b.c0 = b.xf.p;
    b.a = b.a0 = b.alpha0 = 0.0f;
    b.v = V(0.0f, 0.0f);
    b.w = 0.0f;
    b.force = V(0.0f, 0.0f);
    b.torque = 0.0f;
    b.mass = b.invMass = b.I = b.invI = 0.0f;
    b.ld = b.ad = b.sleep = 0.0f;
    b.awake = 1;
    b.dynamic = 0;
    b.island_flag = 0;
    b.island_index = 0;
  }
  for (int i = 0; i < 3; ++i) {
    Body &b = w.b[i];
    b.mass = SC.mass[i];
    b.invMass = SC.invMass[i];
    b.I = SC.I[i];
    b.invI = SC.invI[i];
    b.lc = V(SC.lcx[i], SC.lcy[i]);
    b.dynamic = 1;
    b.island_flag = 0;
    b.island_index = 0;
    b.alpha0 = 0.0f;
  }
}

// ------------------------------------------------------------------------------------------------
// narrow phase (b2CollidePolygonAndCircle, b2CollidePolygons)
// ------------------------------------------------------------------------------------------------
#define FXV(f, i) V((f).vx[i], (f).vy[i])
#define FXN(f, i) V((f).nx[i], (f).ny[i])

HK_DEV void collide_poly_circle(Manifold &m, const Fixture &pa, xform xfA, const Fixture &cb, xform xfB) {
  m.count = 0;
  v2 c = mul_xv(xfB, FXV(cb, 0));
  v2 cl = mulT_xv(xfA, c);
  int ni = 0;
  float sep = -kFltMax;
  float radius = pa.radius + cb.radius;
  for (int i = 0; i < pa.count; ++i) {
    float s = dot(FXN(pa, i), vsub(cl, FXV(pa, i)));
    if (s > radius) return;
    if (s > sep) { sep = s; ni = i; }
  }
  int i1 = ni, i2 = i1 + 1 < pa.count ? i1 + 1 : 0;
  v2 v1 = FXV(pa, i1), v2_ = FXV(pa, i2);
  if (sep < kFltEps) {
    m.count = 1; m.type = 1; m.ln = FXN(pa, ni); m.lp = vs(0.5f, vadd(v1, v2_));
    m.pt_lp[0] = FXV(cb, 0); m.id[0] = 0;
    return;
  }
  float u1 = dot(vsub(cl, v1), vsub(v2_, v1));
  float u2 = dot(vsub(cl, v2_), vsub(v1, v2_));
  if (u1 <= 0.0f) {
    if (vdist2(cl, v1) > radius * radius) return;
    m.count = 1; m.type = 1; m.ln = vsub(cl, v1); vnormalize(m.ln); m.lp = v1;
    m.pt_lp[0] = FXV(cb, 0); m.id[0] = 0;
  } else if (u2 <= 0.0f) {
    if (vdist2(cl, v2_) > radius * radius) return;
    m.count = 1; m.type = 1; m.ln = vsub(cl, v2_); vnormalize(m.ln); m.lp = v2_;
    m.pt_lp[0] = FXV(cb, 0); m.id[0] = 0;
  } else {
    v2 fc = vs(0.5f, vadd(v1, v2_));
    float s = dot(vsub(cl, fc), FXN(pa, i1));
    if (s > radius) return;
    m.count = 1; m.type = 1; m.ln = FXN(pa, i1); m.lp = fc;
    m.pt_lp[0] = FXV(cb, 0); m.id[0] = 0;
  }
}

HK_DEV float find_max_separation(int &edge, const Fixture &p1, xform xf1, const Fixture &p2, xform xf2) {
  xform xf = mulT_xx(xf2, xf1);
  int best = 0;
  float maxs = -kFltMax;
  for (int i = 0; i < p1.count; ++i) {
    v2 n = mul_rv(xf.q, FXN(p1, i));
    v2 v1 = mul_xv(xf, FXV(p1, i));
    float si = kFltMax;
    for (int j = 0; j < p2.count; ++j) {
      float sij = dot(n, vsub(FXV(p2, j), v1));
      if (sij < si) si = sij;
    }
    if (si > maxs) { maxs = si; best = i; }
  }
  edge = best;
  return maxs;
}

struct ClipV { v2 v; uint32_t id; };
HK_DEV uint32_t cf_id(uint32_t ia, uint32_t ib, uint32_t ta, uint32_t tb) { return ia | (ib << 8) | (ta << 16) | (tb << 24); }

HK_DEV void find_incident_edge(ClipV c[2], const Fixture &p1, xform xf1, int edge1, const Fixture &p2, xform xf2) {
  v2 n1 = mulT_rv(xf2.q, mul_rv(xf1.q, FXN(p1, edge1)));
  int index = 0;
  float mind = kFltMax;
  for (int i = 0; i < p2.count; ++i) {
    float d = dot(n1, FXN(p2, i));
    if (d < mind) { mind = d; index = i; }
  }
  int i1 = index, i2 = i1 + 1 < p2.count ? i1 + 1 : 0;
  c[0].v = mul_xv(xf2, FXV(p2, i1));
  c[0].id = cf_id(edge1, i1, 1, 0);
  c[1].v = mul_xv(xf2, FXV(p2, i2));
  c[1].id = cf_id(edge1, i2, 1, 0);
}

HK_DEV int clip_segment(ClipV out[2], const ClipV in[2], v2 normal, float offset, int vA) {
  int n = 0;
  float d0 = dot(normal, in[0].v) - offset;
  float d1 = dot(normal, in[1].v) - offset;
  if (d0 <= 0.0f) out[n++] = in[0];
  if (d1 <= 0.0f) out[n++] = in[1];
  if (d0 * d1 < 0.0f) {
    float interp = d0 / (d0 - d1);
    out[n].v = vadd(in[0].v, vs(interp, vsub(in[1].v, in[0].v)));
    out[n].id = cf_id(vA, (in[0].id >> 8) & 0xffu, 0, 1);
    ++n;
  }
  return n;
}

HK_DEV void collide_polygons(Manifold &m, const Fixture &pA, xform xfA, const Fixture &pB, xform xfB) {
  m.count = 0;
  float total = pA.radius + pB.radius;
  int eA = 0, eB = 0;
  float sA = find_max_separation(eA, pA, xfA, pB, xfB);
  if (sA > total) return;
  float sB = find_max_separation(eB, pB, xfB, pA, xfA);
  if (sB > total) return;
  const float k_tol = 0.1f * kLinearSlop;
  const bool flip = sB > sA + k_tol;
  const Fixture &p1 = flip ? pB : pA;
  const Fixture &p2 = flip ? pA : pB;
  xform xf1 = flip ? xfB : xfA, xf2 = flip ? xfA : xfB;
  int edge1 = flip ? eB : eA;
  m.type = flip ? 2 : 1;
  ClipV inc[2];
  find_incident_edge(inc, p1, xf1, edge1, p2, xf2);
  int iv1 = edge1, iv2 = edge1 + 1 < p1.count ? edge1 + 1 : 0;
  v2 v11 = FXV(p1, iv1), v12 = FXV(p1, iv2);
  v2 lt = vsub(v12, v11);
  vnormalize(lt);
  v2 ln = crs_vs(lt, 1.0f);
  v2 pp = vs(0.5f, vadd(v11, v12));
  v2 tangent = mul_rv(xf1.q, lt);
  v2 normal = crs_vs(tangent, 1.0f);
  v11 = mul_xv(xf1, v11);
  v12 = mul_xv(xf1, v12);
  float front = dot(normal, v11);
  float side1 = -dot(tangent, v11) + total;
  float side2 = dot(tangent, v12) + total;
  ClipV cp1[2], cp2[2];
  int np = clip_segment(cp1, inc, vneg(tangent), side1, iv1);
  if (np < 2) return;
  np = clip_segment(cp2, cp1, tangent, side2, iv2);
  if (np < 2) return;
  m.ln = ln;
  m.lp = pp;
  int pc = 0;
  for (int i = 0; i < 2; ++i) {
    float sep = dot(normal, cp2[i].v) - front;
    if (sep <= total) {
      m.pt_lp[pc] = mulT_xv(xf2, cp2[i].v);
      uint32_t id = cp2[i].id;
      if (flip) id = cf_id((id >> 8) & 0xffu, id & 0xffu, (id >> 24) & 0xffu, (id >> 16) & 0xffu);
      m.id[pc] = id;
      ++pc;
    }
  }
  m.count = pc;
}

// ------------------------------------------------------------------------------------------------
// GJK distance + TOI (b2Distance.cpp, b2TimeOfImpact.cpp)
// ------------------------------------------------------------------------------------------------
struct Proxy { const float *vx, *vy; int count; float radius; };
HK_DEV Proxy make_proxy(const Fixture &f) { Proxy p; p.vx = f.vx; p.vy = f.vy; p.count = f.count; p.radius = f.radius; return p; }
HK_DEV v2 pv(const Proxy &p, int i) { return V(p.vx[i], p.vy[i]); }
HK_DEV int proxy_support(const Proxy &p, v2 d) {
  int best = 0;
  float bv = dot(pv(p, 0), d);
  for (int i = 1; i < p.count; ++i) {
    float v = dot(pv(p, i), d);
    if (v > bv) { best = i; bv = v; }
  }
  return best;
}

struct SimplexCache { float metric; int count; int iA[3], iB[3]; };
struct SVert { v2 wA, wB, w; float a; int iA, iB; };
struct Simplex { SVert v[3]; int count; };

HK_DEV float simplex_metric(const Simplex &s) {
  if (s.count == 2) return vdist(s.v[0].w, s.v[1].w);
  if (s.count == 3) return crs(vsub(s.v[1].w, s.v[0].w), vsub(s.v[2].w, s.v[0].w));
  return 0.0f;
}
HK_DEV void simplex_read(Simplex &s, const SimplexCache &cache, const Proxy &pA, xform xA, const Proxy &pB, xform xB) {
  s.count = cache.count;
  for (int i = 0; i < s.count; ++i) {
    SVert &v = s.v[i];
    v.iA = cache.iA[i];
    v.iB = cache.iB[i];
    v.wA = mul_xv(xA, pv(pA, v.iA));
    v.wB = mul_xv(xB, pv(pB, v.iB));
    v.w = vsub(v.wB, v.wA);
    v.a = 0.0f;
  }
  if (s.count > 1) {
    float m1 = cache.metric, m2 = simplex_metric(s);
    if (m2 < 0.5f * m1 || 2.0f * m1 < m2 || m2 < kFltEps) s.count = 0;
  }
  if (s.count == 0) {
    SVert &v = s.v[0];
    v.iA = 0; v.iB = 0;
    v.wA = mul_xv(xA, pv(pA, 0));
    v.wB = mul_xv(xB, pv(pB, 0));
    v.w = vsub(v.wB, v.wA);
    v.a = 1.0f;
    s.count = 1;
  }
}
HK_DEV void simplex_write(const Simplex &s, SimplexCache &cache) {
  cache.metric = simplex_metric(s);
  cache.count = s.count;
  for (int i = 0; i < s.count; ++i) { cache.iA[i] = s.v[i].iA; cache.iB[i] = s.v[i].iB; }
}
HK_DEV v2 simplex_search_dir(const Simplex &s) {
  if (s.count == 1) return vneg(s.v[0].w);
  v2 e12 = vsub(s.v[1].w, s.v[0].w);
  float sgn = crs(e12, vneg(s.v[0].w));
  if (sgn > 0.0f) return crs_sv(1.0f, e12);
  return crs_vs(e12, 1.0f);
}
HK_DEV void simplex_witness(const Simplex &s, v2 &pA, v2 &pB) {
  if (s.count == 1) { pA = s.v[0].wA; pB = s.v[0].wB; }
  else if (s.count == 2) {
    pA = vadd(vs(s.v[0].a, s.v[0].wA), vs(s.v[1].a, s.v[1].wA));
    pB = vadd(vs(s.v[0].a, s.v[0].wB), vs(s.v[1].a, s.v[1].wB));
  } else {
    pA = vadd(vadd(vs(s.v[0].a, s.v[0].wA), vs(s.v[1].a, s.v[1].wA)), vs(s.v[2].a, s.v[2].wA));
    pB = pA;
  }
}
HK_DEV void solve2(Simplex &s) {
  v2 w1 = s.v[0].w, w2 = s.v[1].w;
  v2 e12 = vsub(w2, w1);
  float d12_2 = -dot(w1, e12);
  if (d12_2 <= 0.0f) { s.v[0].a = 1.0f; s.count = 1; return; }
  float d12_1 = dot(w2, e12);
  if (d12_1 <= 0.0f) { s.v[1].a = 1.0f; s.count = 1; s.v[0] = s.v[1]; return; }
  float inv = 1.0f / (d12_1 + d12_2);
  s.v[0].a = d12_1 * inv;
  s.v[1].a = d12_2 * inv;
  s.count = 2;
}
HK_DEV void solve3(Simplex &s) {
  v2 w1 = s.v[0].w, w2 = s.v[1].w, w3 = s.v[2].w;
  v2 e12 = vsub(w2, w1);
  float w1e12 = dot(w1, e12), w2e12 = dot(w2, e12);
  float d12_1 = w2e12, d12_2 = -w1e12;
  v2 e13 = vsub(w3, w1);
  float w1e13 = dot(w1, e13), w3e13 = dot(w3, e13);
  float d13_1 = w3e13, d13_2 = -w1e13;
  v2 e23 = vsub(w3, w2);
  float w2e23 = dot(w2, e23), w3e23 = dot(w3, e23);
  float d23_1 = w3e23, d23_2 = -w2e23;
  float n123 = crs(e12, e13);
  float d123_1 = n123 * crs(w2, w3);
  float d123_2 = n123 * crs(w3, w1);
  float d123_3 = n123 * crs(w1, w2);
  if (d12_2 <= 0.0f && d13_2 <= 0.0f) { s.v[0].a = 1.0f; s.count = 1; return; }
  if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) {
    float inv = 1.0f / (d12_1 + d12_2);
    s.v[0].a = d12_1 * inv; s.v[1].a = d12_2 * inv; s.count = 2; return;
  }
  if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) {
    float inv = 1.0f / (d13_1 + d13_2);
    s.v[0].a = d13_1 * inv; s.v[2].a = d13_2 * inv; s.count = 2; s.v[1] = s.v[2]; return;
  }
  if (d12_1 <= 0.0f && d23_2 <= 0.0f) { s.v[1].a = 1.0f; s.count = 1; s.v[0] = s.v[1]; return; }
  if (d13_1 <= 0.0f && d23_1 <= 0.0f) { s.v[2].a = 1.0f; s.count = 1; s.v[0] = s.v[2]; return; }
  if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) {
    float inv = 1.0f / (d23_1 + d23_2);
    s.v[1].a = d23_1 * inv; s.v[2].a = d23_2 * inv; s.count = 2; s.v[0] = s.v[2]; return;
  }
  float inv = 1.0f / (d123_1 + d123_2 + d123_3);
  s.v[0].a = d123_1 * inv; s.v[1].a = d123_2 * inv; s.v[2].a = d123_3 * inv; s.count = 3;
}

HK_DEV float gjk_distance(SimplexCache &cache, const Proxy &pA, xform xA, const Proxy &pB, xform xB, int use_radii) {
  Simplex s;
  simplex_read(s, cache, pA, xA, pB, xB);
  int saveA[3], saveB[3], saveCount;
  int iter = 0;
  while (iter < 20) {
    saveCount = s.count;
    for (int i = 0; i < saveCount; ++i) { saveA[i] = s.v[i].iA; saveB[i] = s.v[i].iB; }
    if (s.count == 2) solve2(s);
    else if (s.count == 3) solve3(s);
    if (s.count == 3) break;
    v2 d = simplex_search_dir(s);
    if (vlen2(d) < kFltEps * kFltEps) break;
    SVert &v = s.v[s.count];
    v.iA = proxy_support(pA, mulT_rv(xA.q, vneg(d)));
    v.wA = mul_xv(xA, pv(pA, v.iA));
    v.iB = proxy_support(pB, mulT_rv(xB.q, d));
    v.wB = mul_xv(xB, pv(pB, v.iB));
    v.w = vsub(v.wB, v.wA);
    ++iter;
    int dup = 0;
    for (int i = 0; i < saveCount; ++i)
      if (v.iA == saveA[i] && v.iB == saveB[i]) { dup = 1; break; }
    if (dup) break;
    ++s.count;
  }
  v2 pa, pb;
  simplex_witness(s, pa, pb);
  float dist = vdist(pa, pb);
  simplex_write(s, cache);
  if (use_radii) {
    float rA = pA.radius, rB = pB.radius;
    if (dist > rA + rB && dist > kFltEps) dist -= rA + rB;
    else dist = 0.0f;
  }
  return dist;
}

HK_DEV int test_overlap(const Fixture &fA, xform xA, const Fixture &fB, xform xB) {
  Proxy pA = make_proxy(fA), pB = make_proxy(fB);
  SimplexCache cache;
  cache.count = 0;
  cache.metric = 0.0f;
  float d = gjk_distance(cache, pA, xA, pB, xB, 1);
  return d < 10.0f * kFltEps;
}

struct Sweep { v2 lc, c0, c; float a0, a, alpha0; };
HK_DEV void sweep_xf(const Sweep &s, xform &xf, float beta) {
  xf.p = vadd(vs(1.0f - beta, s.c0), vs(beta, s.c));
  float angle = (1.0f - beta) * s.a0 + beta * s.a;
  xf.q = rot_set(angle);
  xf.p = vsub(xf.p, mul_rv(xf.q, s.lc));
}
HK_DEV void sweep_advance(Sweep &s, float alpha) {
  float beta = (alpha - s.alpha0) / (1.0f - s.alpha0);
  s.c0 = vadd(s.c0, vs(beta, vsub(s.c, s.c0)));
  s.a0 += beta * (s.a - s.a0);
  s.alpha0 = alpha;
}
HK_DEV void sweep_normalize(Sweep &s) {
  float twoPi = 2.0f * kPi;
  float d = twoPi * floorf(s.a0 / twoPi);
  s.a0 -= d;
  s.a -= d;
}
HK_DEV Sweep body_sweep(const Body &b) {
  Sweep s;
  s.lc = b.lc; s.c0 = b.c0; s.c = b.c; s.a0 = b.a0; s.a = b.a; s.alpha0 = b.alpha0;
  return s;
}
HK_DEV void body_set_sweep(Body &b, const Sweep &s) {
  b.lc = s.lc; b.c0 = s.c0; b.c = s.c; b.a0 = s.a0; b.a = s.a; b.alpha0 = s.alpha0;
}

enum { SF_POINTS = 0, SF_FACEA, SF_FACEB };
struct SepFn { Proxy pA, pB; Sweep sA, sB; int type; v2 lp, axis; };

HK_DEV void sep_init(SepFn &f, const SimplexCache &cache, const Proxy &pA, const Sweep &sA, const Proxy &pB,
                     const Sweep &sB, float t1) {
  f.pA = pA; f.pB = pB; f.sA = sA; f.sB = sB;
  xform xA, xB;
  sweep_xf(f.sA, xA, t1);
  sweep_xf(f.sB, xB, t1);
  if (cache.count == 1) {
    f.type = SF_POINTS;
    v2 a = mul_xv(xA, pv(pA, cache.iA[0]));
    v2 b = mul_xv(xB, pv(pB, cache.iB[0]));
    f.axis = vsub(b, a);
    vnormalize(f.axis);
  } else if (cache.iA[0] == cache.iA[1]) {
    f.type = SF_FACEB;
    v2 b1 = pv(pB, cache.iB[0]), b2 = pv(pB, cache.iB[1]);
    f.axis = crs_vs(vsub(b2, b1), 1.0f);
    vnormalize(f.axis);
    v2 normal = mul_rv(xB.q, f.axis);
    f.lp = vs(0.5f, vadd(b1, b2));
    v2 pb = mul_xv(xB, f.lp);
    v2 pa = mul_xv(xA, pv(pA, cache.iA[0]));
    float s = dot(vsub(pa, pb), normal);
    if (s < 0.0f) f.axis = vneg(f.axis);
  } else {
    f.type = SF_FACEA;
    v2 a1 = pv(pA, cache.iA[0]), a2 = pv(pA, cache.iA[1]);
    f.axis = crs_vs(vsub(a2, a1), 1.0f);
    vnormalize(f.axis);
    v2 normal = mul_rv(xA.q, f.axis);
    f.lp = vs(0.5f, vadd(a1, a2));
    v2 pa = mul_xv(xA, f.lp);
    v2 pb = mul_xv(xB, pv(pB, cache.iB[0]));
    float s = dot(vsub(pb, pa), normal);
    if (s < 0.0f) f.axis = vneg(f.axis);
  }
}
HK_DEV float sep_find_min(const SepFn &f, int &iA, int &iB, float t) {
  xform xA, xB;
  sweep_xf(f.sA, xA, t);
  sweep_xf(f.sB, xB, t);
  if (f.type == SF_POINTS) {
    v2 axA = mulT_rv(xA.q, f.axis), axB = mulT_rv(xB.q, vneg(f.axis));
    iA = proxy_support(f.pA, axA);
    iB = proxy_support(f.pB, axB);
    v2 a = mul_xv(xA, pv(f.pA, iA)), b = mul_xv(xB, pv(f.pB, iB));
    return dot(vsub(b, a), f.axis);
  } else if (f.type == SF_FACEA) {
    v2 normal = mul_rv(xA.q, f.axis);
    v2 a = mul_xv(xA, f.lp);
    v2 axB = mulT_rv(xB.q, vneg(normal));
    iA = -1;
    iB = proxy_support(f.pB, axB);
    v2 b = mul_xv(xB, pv(f.pB, iB));
    return dot(vsub(b, a), normal);
  } else {
    v2 normal = mul_rv(xB.q, f.axis);
    v2 b = mul_xv(xB, f.lp);
    v2 axA = mulT_rv(xA.q, vneg(normal));
    iB = -1;
    iA = proxy_support(f.pA, axA);
    v2 a = mul_xv(xA, pv(f.pA, iA));
    return dot(vsub(a, b), normal);
  }
}
HK_DEV float sep_eval(const SepFn &f, int iA, int iB, float t) {
  xform xA, xB;
  sweep_xf(f.sA, xA, t);
  sweep_xf(f.sB, xB, t);
  if (f.type == SF_POINTS) {
    v2 a = mul_xv(xA, pv(f.pA, iA)), b = mul_xv(xB, pv(f.pB, iB));
    return dot(vsub(b, a), f.axis);
  } else if (f.type == SF_FACEA) {
    v2 normal = mul_rv(xA.q, f.axis);
    v2 a = mul_xv(xA, f.lp);
    v2 b = mul_xv(xB, pv(f.pB, iB));
    return dot(vsub(b, a), normal);
  } else {
    v2 normal = mul_rv(xB.q, f.axis);
    v2 b = mul_xv(xB, f.lp);
    v2 a = mul_xv(xA, pv(f.pA, iA));
    return dot(vsub(a, b), normal);
  }
}

enum { TOI_UNKNOWN = 0, TOI_FAILED, TOI_OVERLAPPED, TOI_TOUCHING, TOI_SEPARATED };

HK_DEV int time_of_impact(const Proxy &pA, const Proxy &pB, Sweep sA, Sweep sB, float tMax, float &t_out) {
  int state = TOI_UNKNOWN;
  t_out = tMax;
  sweep_normalize(sA);
  sweep_normalize(sB);
  float total = pA.radius + pB.radius;
  float target = fmax2(kLinearSlop, total - 3.0f * kLinearSlop);
  float tol = 0.25f * kLinearSlop;
  float t1 = 0.0f;
  int iter = 0;
  SimplexCache cache;
  cache.count = 0;
  cache.metric = 0.0f;
  for (;;) {
    xform xA, xB;
    sweep_xf(sA, xA, t1);
    sweep_xf(sB, xB, t1);
    float dist = gjk_distance(cache, pA, xA, pB, xB, 0);
    if (dist <= 0.0f) { state = TOI_OVERLAPPED; t_out = 0.0f; break; }
    if (dist < target + tol) { state = TOI_TOUCHING; t_out = t1; break; }
    SepFn fcn;
    sep_init(fcn, cache, pA, sA, pB, sB, t1);
    int done = 0;
    float t2 = tMax;
    int push = 0;
    for (;;) {
      int iA, iB;
      float s2 = sep_find_min(fcn, iA, iB, t2);
      if (s2 > target + tol) { state = TOI_SEPARATED; t_out = tMax; done = 1; break; }
      if (s2 > target - tol) { t1 = t2; break; }
      float s1 = sep_eval(fcn, iA, iB, t1);
      if (s1 < target - tol) { state = TOI_FAILED; t_out = t1; done = 1; break; }
      if (s1 <= target + tol) { state = TOI_TOUCHING; t_out = t1; done = 1; break; }
      int rit = 0;
      float a1 = t1, a2 = t2;
      for (;;) {
        float t;
        if (rit & 1) t = a1 + (target - s1) * (a2 - a1) / (s2 - s1);
        else t = 0.5f * (a1 + a2);
        ++rit;
        float s = sep_eval(fcn, iA, iB, t);
        if (fabs2(s - target) < tol) { t2 = t; break; }
        if (s > target) { a1 = t; s1 = s; } else { a2 = t; s2 = s; }
        if (rit == 50) break;
      }
      ++push;
      if (push == kMaxPolyVerts) break;
    }
    ++iter;
    if (done) break;
    if (iter == 20) { state = TOI_FAILED; t_out = t1; break; }
  }
  return state;
}

// ------------------------------------------------------------------------------------------------
// contact update + ContactDetector (hockey_env.py:44-76)
// ------------------------------------------------------------------------------------------------
HK_DEV void begin_contact(World &w, int p) {
  int bA = SC.pbodyA[p], bB = SC.pbodyB[p];
  int hasPK = (bA == B_PK || bB == B_PK);
  if ((bA == B_G2 || bB == B_G2) && hasPK) { w.done = 1; w.winner = 1; }
  if ((bA == B_G1 || bB == B_G1) && hasPK) { w.done = 1; w.winner = -1; }
  if ((bA == B_P1 || bB == B_P1) && hasPK) {
    if (w.keep_mode && (double)w.b[B_PK].v.x < 0.1)
      if (w.has1 == 0) w.has1 = 15;
  }
  if ((bA == B_P2 || bB == B_P2) && hasPK) {
    if (w.keep_mode && (double)w.b[B_PK].v.x > -0.1)
      if (w.has2 == 0) w.has2 = 15;
  }
}

HK_DEV void contact_update(World &w, int p) {
  Contact &c = w.c[p];
  const int oc = c.m.count;
  const uint32_t oid0 = c.m.id[0], oid1 = c.m.id[1];
  const float oni0 = c.m.ni[0], oni1 = c.m.ni[1], oti0 = c.m.ti[0], oti1 = c.m.ti[1];
  c.enabled = 1;
  int was = c.touching, touching;
  const Fixture &fA = SC.fx[SC.pairA[p]];
  const Fixture &fB = SC.fx[SC.pairB[p]];
  Body &bA = w.b[SC.pbodyA[p]];
  Body &bB = w.b[SC.pbodyB[p]];
  if (SC.sensor[p]) {
    touching = test_overlap(fA, bA.xf, fB, bB.xf);
    c.m.count = 0;
  } else {
    if (fB.circle) collide_poly_circle(c.m, fA, bA.xf, fB, bB.xf);
    else collide_polygons(c.m, fA, bA.xf, fB, bB.xf);
    touching = c.m.count > 0;
    for (int i = 0; i < c.m.count; ++i) {
      c.m.ni[i] = 0.0f;
      c.m.ti[i] = 0.0f;
      if (oc > 0 && oid0 == c.m.id[i]) { c.m.ni[i] = oni0; c.m.ti[i] = oti0; }
      else if (oc > 1 && oid1 == c.m.id[i]) { c.m.ni[i] = oni1; c.m.ti[i] = oti1; }
    }
    if (touching != was) { set_awake(bA, 1); set_awake(bB, 1); }
  }
  c.touching = touching;
  if (!was && touching) begin_contact(w, p);
}

// ------------------------------------------------------------------------------------------------
// Lane-local broad phase.  Box2D only evaluates a pair once its fat AABBs overlap; here every pair
// of the fixed table is live, so a conservative bounding test decides when the exact narrow phase /
// time of impact cannot produce a contact point, a sensor overlap or a TOI "touching" event.  In that
// case the pair takes exactly the outcome the full computation would have produced (touching = 0,
// manifold count 0, alpha = 1), so results are bit-identical to the exhaustive oracle
// (tests/test_gpu_parity.py runs the oracle WITHOUT this filter).
//   * Box2D polygon clipping can emit points up to sqrt(2) * totalRadius from the reference polygon
//     and the circle manifold up to totalRadius: reach = 2 * (rA + rB).
//   * every TOI "touching" exit needs the core distance below target + tol < rA + rB at some t
//     (GJK distance, or an axis separation that upper-bounds it, b2TimeOfImpact).
// ------------------------------------------------------------------------------------------------
HK_DEV float box_gap(float ax0, float ay0, float ax1, float ay1, const float *b) {
  return fmaxf(fmaxf(b[0] - ax1, ax0 - b[2]), fmaxf(b[1] - ay1, ay0 - b[3]));
}

HK_DEV bool pair_far_collide(const World &w, int p) {
  const int fA = SC.pairA[p], fB = SC.pairB[p];
  const int bA = SC.pbodyA[p], bB = SC.pbodyB[p];
  const float reach = 2.0f * (SC.fx[fA].radius + SC.fx[fB].radius) + kFarMargin;
  const Body &B = w.b[bB];
  const float rB = SC.rcore[bB];
  if (bA >= B_WT) {
    return box_gap(B.c.x - rB, B.c.y - rB, B.c.x + rB, B.c.y + rB, SC.fx_aabb[fA]) > reach;
  }
  const Body &A = w.b[bA];
  const float lim = SC.rcore[bA] + rB + reach;
  const float dx = A.c.x - B.c.x, dy = A.c.y - B.c.y;
  return dx * dx + dy * dy > lim * lim;
}

HK_DEV bool pair_far_toi(const World &w, int p) {  // static A, dynamic B, sweeps already aligned
  const int fA = SC.pairA[p], fB = SC.pairB[p];
  const Body &B = w.b[SC.pbodyB[p]];
  const float reach = 2.0f * (SC.fx[fA].radius + SC.fx[fB].radius) + kFarMargin;
  const float r = SC.rcore[SC.pbodyB[p]];
  return box_gap(fminf(B.c0.x, B.c.x) - r, fminf(B.c0.y, B.c.y) - r, fmaxf(B.c0.x, B.c.x) + r,
                 fmaxf(B.c0.y, B.c.y) + r, SC.fx_aabb[fA]) > reach;
}

// contact_update for a pair the broad phase rejected: the exact result of contact_update with no
// manifold point / no overlap
HK_DEV void contact_update_far(World &w, int p) {
  Contact &c = w.c[p];
  c.enabled = 1;
  const int was = c.touching;
  c.m.count = 0;
  if (!SC.sensor[p] && was) { set_awake(w.b[SC.pbodyA[p]], 1); set_awake(w.b[SC.pbodyB[p]], 1); }
  c.touching = 0;
}

HK_DEV void contact_update_any(World &w, int p) {
  if (pair_far_collide(w, p)) contact_update_far(w, p);
  else contact_update(w, p);
}

HK_DEV void collide(World &w) {
  for (int p = 0; p < NP; ++p) {
    Body &bA = w.b[SC.pbodyA[p]];
    Body &bB = w.b[SC.pbodyB[p]];
    int activeA = bA.awake && bA.dynamic;
    int activeB = bB.awake && bB.dynamic;
    if (!activeA && !activeB) continue;
    contact_update_any(w, p);
  }
}

// ------------------------------------------------------------------------------------------------
// contact solver (b2ContactSolver.cpp)
// ------------------------------------------------------------------------------------------------
struct VCPoint { v2 rA, rB; float ni, ti, nm, tm, bias; };
struct VC {
  VCPoint p[2];
  v2 normal;
  float Kexx, Kexy, Keyx, Keyy, Nexx, Nexy, Neyx, Neyy;
  int iA, iB, count, ci;
  float mA, mB, iIA, iIB, friction, restitution;
};
struct PC {
  v2 lps[2], ln, lp, lcA, lcB;
  int iA, iB, type, count;
  float mA, mB, iIA, iIB, rA, rB;
};
struct Solver {
  int n;
  VC vc[kMaxIsland];
  PC pc[kMaxIsland];
};

HK_DEV void solver_init(World &w, Solver &S, const int *clist, int n, int warm) {
  S.n = n;
  for (int i = 0; i < n; ++i) {
    const int p = clist[i];
    Contact &c = w.c[p];
    const Body &bA = w.b[SC.pbodyA[p]];
    const Body &bB = w.b[SC.pbodyB[p]];
    VC &vc = S.vc[i];
    PC &pc = S.pc[i];
    vc.friction = SC.friction[p];
    vc.restitution = SC.restitution[p];
    vc.iA = bA.island_index; vc.iB = bB.island_index;
    vc.mA = bA.invMass; vc.mB = bB.invMass; vc.iIA = bA.invI; vc.iIB = bB.invI;
    vc.ci = p;
    vc.count = c.m.count;
    vc.Kexx = vc.Kexy = vc.Keyx = vc.Keyy = 0.0f;
    vc.Nexx = vc.Nexy = vc.Neyx = vc.Neyy = 0.0f;
    pc.iA = bA.island_index; pc.iB = bB.island_index;
    pc.mA = bA.invMass; pc.mB = bB.invMass;
    pc.lcA = bA.lc; pc.lcB = bB.lc;
    pc.iIA = bA.invI; pc.iIB = bB.invI;
    pc.ln = c.m.ln; pc.lp = c.m.lp;
    pc.count = c.m.count;
    pc.rA = SC.fx[SC.pairA[p]].radius;
    pc.rB = SC.fx[SC.pairB[p]].radius;
    pc.type = c.m.type;
    for (int j = 0; j < c.m.count; ++j) {
      VCPoint &vp = vc.p[j];
      if (warm) { vp.ni = 1.0f * c.m.ni[j]; vp.ti = 1.0f * c.m.ti[j]; }
      else { vp.ni = 0.0f; vp.ti = 0.0f; }
      vp.rA = V(0.0f, 0.0f); vp.rB = V(0.0f, 0.0f);
      vp.nm = 0.0f; vp.tm = 0.0f; vp.bias = 0.0f;
      pc.lps[j] = c.m.pt_lp[j];
    }
  }
}

struct PosV { v2 c; float a; };
struct VelV { v2 v; float w; };

HK_DEV void world_manifold(const Manifold &m, xform xA, float rA, xform xB, float rB, v2 &normal, v2 pts[2]) {
  if (m.type == 1) {
    normal = mul_rv(xA.q, m.ln);
    v2 plane = mul_xv(xA, m.lp);
    for (int i = 0; i < m.count; ++i) {
      v2 clip = mul_xv(xB, m.pt_lp[i]);
      v2 cA = vadd(clip, vs(rA - dot(vsub(clip, plane), normal), normal));
      v2 cB = vsub(clip, vs(rB, normal));
      pts[i] = vs(0.5f, vadd(cA, cB));
    }
  } else {
    normal = mul_rv(xB.q, m.ln);
    v2 plane = mul_xv(xB, m.lp);
    for (int i = 0; i < m.count; ++i) {
      v2 clip = mul_xv(xA, m.pt_lp[i]);
      v2 cB = vadd(clip, vs(rB - dot(vsub(clip, plane), normal), normal));
      v2 cA = vsub(clip, vs(rA, normal));
      pts[i] = vs(0.5f, vadd(cA, cB));
    }
    normal = vneg(normal);
  }
}

HK_DEV void solver_init_velocity(World &w, Solver &S, const PosV *P, const VelV *Vl) {
  for (int i = 0; i < S.n; ++i) {
    VC &vc = S.vc[i];
    PC &pc = S.pc[i];
    const Manifold &m = w.c[vc.ci].m;
    float mA = vc.mA, mB = vc.mB, iA = vc.iIA, iB = vc.iIB;
    v2 cA = P[vc.iA].c, cB = P[vc.iB].c;
    float aA = P[vc.iA].a, aB = P[vc.iB].a;
    v2 vA = Vl[vc.iA].v, vB = Vl[vc.iB].v;
    float wA = Vl[vc.iA].w, wB = Vl[vc.iB].w;
    xform xA, xB;
    xA.q = rot_set(aA);
    xB.q = rot_set(aB);
    xA.p = vsub(cA, mul_rv(xA.q, pc.lcA));
    xB.p = vsub(cB, mul_rv(xB.q, pc.lcB));
    v2 normal, pts[2];
    world_manifold(m, xA, pc.rA, xB, pc.rB, normal, pts);
    vc.normal = normal;
    for (int j = 0; j < vc.count; ++j) {
      VCPoint &vp = vc.p[j];
      vp.rA = vsub(pts[j], cA);
      vp.rB = vsub(pts[j], cB);
      float rnA = crs(vp.rA, vc.normal), rnB = crs(vp.rB, vc.normal);
      float kN = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      vp.nm = kN > 0.0f ? 1.0f / kN : 0.0f;
      v2 tangent = crs_vs(vc.normal, 1.0f);
      float rtA = crs(vp.rA, tangent), rtB = crs(vp.rB, tangent);
      float kT = mA + mB + iA * rtA * rtA + iB * rtB * rtB;
      vp.tm = kT > 0.0f ? 1.0f / kT : 0.0f;
      vp.bias = 0.0f;
      float vRel = dot(vc.normal, vsub(vsub(vadd(vB, crs_sv(wB, vp.rB)), vA), crs_sv(wA, vp.rA)));
      if (vRel < -kVelocityThreshold) vp.bias = -vc.restitution * vRel;
    }
    if (vc.count == 2) {
      VCPoint &p1 = vc.p[0], &p2 = vc.p[1];
      float rn1A = crs(p1.rA, vc.normal), rn1B = crs(p1.rB, vc.normal);
      float rn2A = crs(p2.rA, vc.normal), rn2B = crs(p2.rB, vc.normal);
      float k11 = mA + mB + iA * rn1A * rn1A + iB * rn1B * rn1B;
      float k22 = mA + mB + iA * rn2A * rn2A + iB * rn2B * rn2B;
      float k12 = mA + mB + iA * rn1A * rn2A + iB * rn1B * rn2B;
      if (k11 * k11 < 1000.0f * (k11 * k22 - k12 * k12)) {
        vc.Kexx = k11; vc.Kexy = k12; vc.Keyx = k12; vc.Keyy = k22;
        float a = vc.Kexx, b = vc.Keyx, c = vc.Kexy, d = vc.Keyy;
        float det = a * d - b * c;
        if (det != 0.0f) det = 1.0f / det;
        vc.Nexx = det * d; vc.Neyx = -det * b;
        vc.Nexy = -det * c; vc.Neyy = det * a;
      } else {
        vc.count = 1;
      }
    }
  }
}

HK_DEV void solver_warm_start(Solver &S, VelV *Vl) {
  for (int i = 0; i < S.n; ++i) {
    VC &vc = S.vc[i];
    float mA = vc.mA, iA = vc.iIA, mB = vc.mB, iB = vc.iIB;
    v2 vA = Vl[vc.iA].v, vB = Vl[vc.iB].v;
    float wA = Vl[vc.iA].w, wB = Vl[vc.iB].w;
    v2 normal = vc.normal, tangent = crs_vs(normal, 1.0f);
    for (int j = 0; j < vc.count; ++j) {
      VCPoint &vp = vc.p[j];
      v2 P = vadd(vs(vp.ni, normal), vs(vp.ti, tangent));
      wA -= iA * crs(vp.rA, P);
      vA = vsub(vA, vs(mA, P));
      wB += iB * crs(vp.rB, P);
      vB = vadd(vB, vs(mB, P));
    }
    Vl[vc.iA].v = vA; Vl[vc.iA].w = wA;
    Vl[vc.iB].v = vB; Vl[vc.iB].w = wB;
  }
}

HK_DEV void solver_solve_velocity(Solver &S, VelV *Vl) {
  for (int i = 0; i < S.n; ++i) {
    VC &vc = S.vc[i];
    float mA = vc.mA, iA = vc.iIA, mB = vc.mB, iB = vc.iIB;
    v2 vA = Vl[vc.iA].v, vB = Vl[vc.iB].v;
    float wA = Vl[vc.iA].w, wB = Vl[vc.iB].w;
    v2 normal = vc.normal, tangent = crs_vs(normal, 1.0f);
    float friction = vc.friction;
    for (int j = 0; j < vc.count; ++j) {
      VCPoint &vp = vc.p[j];
      v2 dv = vsub(vsub(vadd(vB, crs_sv(wB, vp.rB)), vA), crs_sv(wA, vp.rA));
      float vt = dot(dv, tangent) - 0.0f;
      float lambda = vp.tm * (-vt);
      float maxF = friction * vp.ni;
      float newI = fclamp(vp.ti + lambda, -maxF, maxF);
      lambda = newI - vp.ti;
      vp.ti = newI;
      v2 P = vs(lambda, tangent);
      vA = vsub(vA, vs(mA, P));
      wA -= iA * crs(vp.rA, P);
      vB = vadd(vB, vs(mB, P));
      wB += iB * crs(vp.rB, P);
    }
    if (vc.count == 1) {
      VCPoint &vp = vc.p[0];
      v2 dv = vsub(vsub(vadd(vB, crs_sv(wB, vp.rB)), vA), crs_sv(wA, vp.rA));
      float vn = dot(dv, normal);
      float lambda = -vp.nm * (vn - vp.bias);
      float newI = fmax2(vp.ni + lambda, 0.0f);
      lambda = newI - vp.ni;
      vp.ni = newI;
      v2 P = vs(lambda, normal);
      vA = vsub(vA, vs(mA, P));
      wA -= iA * crs(vp.rA, P);
      vB = vadd(vB, vs(mB, P));
      wB += iB * crs(vp.rB, P);
    } else {
      VCPoint &c1 = vc.p[0], &c2 = vc.p[1];
      v2 a = V(c1.ni, c2.ni);
      v2 dv1 = vsub(vsub(vadd(vB, crs_sv(wB, c1.rB)), vA), crs_sv(wA, c1.rA));
      v2 dv2 = vsub(vsub(vadd(vB, crs_sv(wB, c2.rB)), vA), crs_sv(wA, c2.rA));
      float vn1 = dot(dv1, normal), vn2 = dot(dv2, normal);
      v2 b;
      b.x = vn1 - c1.bias;
      b.y = vn2 - c2.bias;
      b = vsub(b, V(vc.Kexx * a.x + vc.Keyx * a.y, vc.Kexy * a.x + vc.Keyy * a.y));
      v2 x = vneg(V(vc.Nexx * b.x + vc.Neyx * b.y, vc.Nexy * b.x + vc.Neyy * b.y));
      int ok = 0;
      if (x.x >= 0.0f && x.y >= 0.0f) ok = 1;
      if (!ok) {
        x.x = -c1.nm * b.x;
        x.y = 0.0f;
        vn2 = vc.Kexy * x.x + b.y;
        if (x.x >= 0.0f && vn2 >= 0.0f) ok = 1;
      }
      if (!ok) {
        x.x = 0.0f;
        x.y = -c2.nm * b.y;
        vn1 = vc.Keyx * x.y + b.x;
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
        wA -= iA * (crs(c1.rA, P1) + crs(c2.rA, P2));
        vB = vadd(vB, vs(mB, vadd(P1, P2)));
        wB += iB * (crs(c1.rB, P1) + crs(c2.rB, P2));
        c1.ni = x.x;
        c2.ni = x.y;
      }
    }
    Vl[vc.iA].v = vA; Vl[vc.iA].w = wA;
    Vl[vc.iB].v = vB; Vl[vc.iB].w = wB;
  }
}

HK_DEV void solver_store(World &w, const Solver &S) {
  for (int i = 0; i < S.n; ++i) {
    const VC &vc = S.vc[i];
    Manifold &m = w.c[vc.ci].m;
    for (int j = 0; j < vc.count; ++j) { m.ni[j] = vc.p[j].ni; m.ti[j] = vc.p[j].ti; }
  }
}

HK_DEV void psm(const PC &pc, xform xA, xform xB, int idx, v2 &normal, v2 &point, float &sep) {
  if (pc.type == 1) {
    normal = mul_rv(xA.q, pc.ln);
    v2 plane = mul_xv(xA, pc.lp);
    v2 clip = mul_xv(xB, pc.lps[idx]);
    sep = dot(vsub(clip, plane), normal) - pc.rA - pc.rB;
    point = clip;
  } else {
    normal = mul_rv(xB.q, pc.ln);
    v2 plane = mul_xv(xB, pc.lp);
    v2 clip = mul_xv(xA, pc.lps[idx]);
    sep = dot(vsub(clip, plane), normal) - pc.rA - pc.rB;
    point = clip;
    normal = vneg(normal);
  }
}

HK_DEV float solver_position_pass(const Solver &S, PosV *P, int toi, int toiA, int toiB) {
  float minSep = 0.0f;
  for (int i = 0; i < S.n; ++i) {
    const PC &pc = S.pc[i];
    float mA, iA, mB, iB;
    if (toi) {
      mA = 0.0f; iA = 0.0f; mB = 0.0f; iB = 0.0f;
      if (pc.iA == toiA || pc.iA == toiB) { mA = pc.mA; iA = pc.iIA; }
      if (pc.iB == toiA || pc.iB == toiB) { mB = pc.mB; iB = pc.iIB; }
    } else {
      mA = pc.mA; iA = pc.iIA; mB = pc.mB; iB = pc.iIB;
    }
    v2 cA = P[pc.iA].c, cB = P[pc.iB].c;
    float aA = P[pc.iA].a, aB = P[pc.iB].a;
    for (int j = 0; j < pc.count; ++j) {
      xform xA, xB;
      xA.q = rot_set(aA);
      xB.q = rot_set(aB);
      xA.p = vsub(cA, mul_rv(xA.q, pc.lcA));
      xB.p = vsub(cB, mul_rv(xB.q, pc.lcB));
      v2 normal, point;
      float sep;
      psm(pc, xA, xB, j, normal, point, sep);
      v2 rA = vsub(point, cA), rB = vsub(point, cB);
      minSep = fmin2(minSep, sep);
      float C = fclamp((toi ? kToiBaumgarte : kBaumgarte) * (sep + kLinearSlop), -kMaxLinearCorrection, 0.0f);
      float rnA = crs(rA, normal), rnB = crs(rB, normal);
      float K = mA + mB + iA * rnA * rnA + iB * rnB * rnB;
      float impulse = K > 0.0f ? -C / K : 0.0f;
      v2 Pv = vs(impulse, normal);
      cA = vsub(cA, vs(mA, Pv));
      aA -= iA * crs(rA, Pv);
      cB = vadd(cB, vs(mB, Pv));
      aB += iB * crs(rB, Pv);
    }
    P[pc.iA].c = cA; P[pc.iA].a = aA;
    P[pc.iB].c = cB; P[pc.iB].a = aB;
  }
  return minSep;
}

// ------------------------------------------------------------------------------------------------
// islands (b2World::Solve / b2Island::Solve) and continuous collision (b2World::SolveTOI)
// ------------------------------------------------------------------------------------------------
HK_DEV void integrate_positions(float h, PosV *P, VelV *Vl, int n) {
  for (int i = 0; i < n; ++i) {
    v2 c = P[i].c, v = Vl[i].v;
    float a = P[i].a, wv = Vl[i].w;
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
    P[i].c = c; P[i].a = a; Vl[i].v = v; Vl[i].w = wv;
  }
}

HK_DEV void solve_islands(World &w, Solver &S, float dt, int ablate) {
  const float h = dt;
  const int seed_order[3] = {B_PK, B_P2, B_P1};
  for (int i = 0; i < NB; ++i) w.b[i].island_flag = 0;
  for (int p = 0; p < NP; ++p) w.c[p].island_flag = 0;
  for (int si = 0; si < 3; ++si) {
    const int seed = seed_order[si];
    Body &sb = w.b[seed];
    if (sb.island_flag || !sb.awake) continue;
    int ibodies[NB], nb = 0, icont[NP], nc = 0;
    int stack[NB], sc = 0;
    stack[sc++] = seed;
    sb.island_flag = 1;
    while (sc > 0) {
      int bi = stack[--sc];
      Body &b = w.b[bi];
      b.island_index = nb;
      ibodies[nb++] = bi;
      set_awake(b, 1);
      if (!b.dynamic) continue;
      for (int k = 0; k < 10; ++k) {
        const int e = SC.edges[bi][k];
        Contact &c = w.c[e];
        if (c.island_flag) continue;
        if (!c.enabled || !c.touching) continue;
        if (SC.sensor[e]) continue;
        icont[nc++] = e;
        c.island_flag = 1;
        int other = (SC.pbodyA[e] == bi) ? SC.pbodyB[e] : SC.pbodyA[e];
        if (w.b[other].island_flag) continue;
        stack[sc++] = other;
        w.b[other].island_flag = 1;
      }
    }
    if (nc > kMaxIsland) { w.overflow = 1; nc = kMaxIsland; }
    PosV P[NB];
    VelV Vl[NB];
    for (int i = 0; i < nb; ++i) {
      Body &b = w.b[ibodies[i]];
      v2 c = b.c, v = b.v;
      float a = b.a, wv = b.w;
      b.c0 = b.c;
      b.a0 = b.a;
      if (b.dynamic) {
        v = vadd(v, vs(h, vadd(vs(1.0f, V(0.0f, 0.0f)), vs(b.invMass, b.force))));
        wv += h * b.invI * b.torque;
        v = vs(1.0f / (1.0f + h * b.ld), v);
        wv *= 1.0f / (1.0f + h * b.ad);
      }
      P[i].c = c; P[i].a = a; Vl[i].v = v; Vl[i].w = wv;
    }
    solver_init(w, S, icont, nc, 1);
    solver_init_velocity(w, S, P, Vl);
    solver_warm_start(S, Vl);
    for (int it = 0; it < ((ablate & 1) ? 0 : kVelIters); ++it) solver_solve_velocity(S, Vl);
    solver_store(w, S);
    integrate_positions(h, P, Vl, nb);
    int solved = 0;
    for (int it = 0; it < ((ablate & 2) ? 1 : kPosIters); ++it) {
      float minSep = solver_position_pass(S, P, 0, 0, 0);
      if (minSep >= -3.0f * kLinearSlop) { solved = 1; break; }
    }
    for (int i = 0; i < nb; ++i) {
      Body &b = w.b[ibodies[i]];
      b.c = P[i].c; b.a = P[i].a; b.v = Vl[i].v; b.w = Vl[i].w;
      synchronize_transform(b);
    }
    float minSleep = kFltMax;
    const float linTolSqr = kLinearSleepTol * kLinearSleepTol;
    const float angTolSqr = kAngularSleepTol * kAngularSleepTol;
    for (int i = 0; i < nb; ++i) {
      Body &b = w.b[ibodies[i]];
      if (!b.dynamic) continue;
      if (b.w * b.w > angTolSqr || dot(b.v, b.v) > linTolSqr) {
        b.sleep = 0.0f;
        minSleep = 0.0f;
      } else {
        b.sleep += h;
        minSleep = fmin2(minSleep, b.sleep);
      }
    }
    if (minSleep >= kTimeToSleep && solved)
      for (int i = 0; i < nb; ++i) set_awake(w.b[ibodies[i]], 0);
    for (int i = 0; i < nb; ++i)
      if (!w.b[ibodies[i]].dynamic) w.b[ibodies[i]].island_flag = 0;
  }
}

HK_DEV void body_advance(Body &b, float alpha) {
  Sweep s = body_sweep(b);
  sweep_advance(s, alpha);
  s.c = s.c0;
  s.a = s.a0;
  body_set_sweep(b, s);
  b.xf.q = rot_set(b.a);
  b.xf.p = vsub(b.c, mul_rv(b.xf.q, b.lc));
}

// register-resident mini-island solver (hk_fast.h)
HK_DEV void fast_toi_island(World &w, const int *icont, int nc, int toiA, int toiB, float sub_dt, const int *ibodies,
                            int nb);

HK_DEV void solve_toi(World &w, Solver &S, float dt, int ablate, PhaseT &T) {
  for (int i = 0; i < NB; ++i) { w.b[i].island_flag = 0; w.b[i].alpha0 = 0.0f; }
  for (int p = 0; p < NP; ++p) {
    w.c[p].toi_flag = 0; w.c[p].island_flag = 0; w.c[p].toi_count = 0; w.c[p].toi = 1.0f;
  }
  for (;;) {
    int minc = -1;
    float minAlpha = 1.0f;
    for (int p = 0; p < NP; ++p) {
      Contact &c = w.c[p];
      if (!c.enabled) continue;
      if (c.toi_count > kMaxSubSteps) continue;
      float alpha = 1.0f;
      if (c.toi_flag) {
        alpha = c.toi;
      } else {
        if (SC.sensor[p]) continue;
        Body &bA = w.b[SC.pbodyA[p]];
        Body &bB = w.b[SC.pbodyB[p]];
        int activeA = bA.awake && bA.dynamic, activeB = bB.awake && bB.dynamic;
        if (!activeA && !activeB) continue;
        int collideA = !bA.dynamic, collideB = !bB.dynamic;
        if (!collideA && !collideB) continue;
        float alpha0 = bA.alpha0;
        if (bA.alpha0 < bB.alpha0) {
          alpha0 = bB.alpha0;
          Sweep s = body_sweep(bA); sweep_advance(s, alpha0); body_set_sweep(bA, s);
        } else if (bB.alpha0 < bA.alpha0) {
          alpha0 = bA.alpha0;
          Sweep s = body_sweep(bB); sweep_advance(s, alpha0); body_set_sweep(bB, s);
        }
        if (pair_far_toi(w, p)) {
          alpha = 1.0f;
        } else {
          Proxy pA = make_proxy(SC.fx[SC.pairA[p]]), pB = make_proxy(SC.fx[SC.pairB[p]]);
          float beta;
          int st = time_of_impact(pA, pB, body_sweep(bA), body_sweep(bB), 1.0f, beta);
          if (st == TOI_TOUCHING) alpha = fmin2(alpha0 + (1.0f - alpha0) * beta, 1.0f);
          else alpha = 1.0f;
        }
        c.toi = alpha;
        c.toi_flag = 1;
      }
      if (alpha < minAlpha) { minc = p; minAlpha = alpha; }
    }
    HK_TIC(T, 6);
    if (minc < 0 || 1.0f - 10.0f * kFltEps < minAlpha) break;
    Contact &mc = w.c[minc];
    const int iA_ = SC.pbodyA[minc], iB_ = SC.pbodyB[minc];
    Body &bA = w.b[iA_];
    Body &bB = w.b[iB_];
    Sweep backA = body_sweep(bA), backB = body_sweep(bB);
    body_advance(bA, minAlpha);
    body_advance(bB, minAlpha);
    contact_update(w, minc);
    mc.toi_flag = 0;
    ++mc.toi_count;
    if (!mc.enabled || !mc.touching) {
      mc.enabled = 0;
      body_set_sweep(bA, backA);
      body_set_sweep(bB, backB);
      synchronize_transform(bA);
      synchronize_transform(bB);
      continue;
    }
    w.n_toi++;
    set_awake(bA, 1);
    set_awake(bB, 1);
    int ibodies[NB], nb = 0, icont[NP], nc = 0;
    bA.island_index = nb; ibodies[nb++] = iA_;
    bB.island_index = nb; ibodies[nb++] = iB_;
    icont[nc++] = minc;
    bA.island_flag = 1;
    bB.island_flag = 1;
    mc.island_flag = 1;
    const int two[2] = {iA_, iB_};
    for (int k = 0; k < 2; ++k) {
      const int bi = two[k];
      if (!w.b[bi].dynamic) continue;
      for (int q = 0; q < 10; ++q) {
        const int e = SC.edges[bi][q];
        Contact &c = w.c[e];
        if (c.island_flag) continue;
        int other = (SC.pbodyA[e] == bi) ? SC.pbodyB[e] : SC.pbodyA[e];
        Body &ob = w.b[other];
        if (ob.dynamic) continue;
        if (SC.sensor[e]) continue;
        Sweep backup = body_sweep(ob);
        if (!ob.island_flag) body_advance(ob, minAlpha);
        contact_update_any(w, e);
        if (!c.enabled || !c.touching) {
          body_set_sweep(ob, backup);
          synchronize_transform(ob);
          continue;
        }
        c.island_flag = 1;
        icont[nc++] = e;
        if (ob.island_flag) continue;
        ob.island_flag = 1;
        ob.island_index = nb;
        ibodies[nb++] = other;
      }
    }
    if (nc > kMaxIsland) { w.overflow = 1; nc = kMaxIsland; }
    const float sub_dt = (1.0f - minAlpha) * dt;
    HK_TIC(T, 4);
    if (nc <= 3) {
      fast_toi_island(w, icont, nc, iA_, iB_, sub_dt, ibodies, nb);
      HK_TIC(T, 7);
    } else {
    PosV P[NB];
    VelV Vl[NB];
    for (int i = 0; i < nb; ++i) {
      Body &b = w.b[ibodies[i]];
      P[i].c = b.c; P[i].a = b.a; Vl[i].v = b.v; Vl[i].w = b.w;
    }
    solver_init(w, S, icont, nc, 0);
    for (int it = 0; it < 20; ++it) {
      float minSep = solver_position_pass(S, P, 1, bA.island_index, bB.island_index);
      if (minSep >= -1.5f * kLinearSlop) break;
    }
    bA.c0 = P[bA.island_index].c;
    bA.a0 = P[bA.island_index].a;
    bB.c0 = P[bB.island_index].c;
    bB.a0 = P[bB.island_index].a;
    solver_init_velocity(w, S, P, Vl);
    for (int it = 0; it < ((ablate & 1) ? 0 : kVelIters); ++it) solver_solve_velocity(S, Vl);
    integrate_positions(sub_dt, P, Vl, nb);
    for (int i = 0; i < nb; ++i) {
      Body &b = w.b[ibodies[i]];
      b.c = P[i].c; b.a = P[i].a; b.v = Vl[i].v; b.w = Vl[i].w;
      synchronize_transform(b);
    }
    }  // generic path
    for (int i = 0; i < nb; ++i) {
      Body &b = w.b[ibodies[i]];
      b.island_flag = 0;
      if (!b.dynamic) continue;
      for (int q = 0; q < 10; ++q) {
        const int e = SC.edges[ibodies[i]][q];
        w.c[e].toi_flag = 0;
        w.c[e].island_flag = 0;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// HockeyEnv.step laws (hockey_env.py:420-483, 610-633), numpy NEP-50 + pybox2d float32 semantics
// ------------------------------------------------------------------------------------------------
constexpr double kDtPy = 0.02;  // self.timeStep = 1.0 / FPS  (hockey_env.py:119)
constexpr double kPiD = 3.141592653589793;

HK_DEV void check_boundaries(World &w, Body &b, float &f0, float &f1, int one) {
  double px = b.xf.p.x, py = b.xf.p.y;
  if ((one && px < 1.5 && f0 < 0) || (!one && px > 8.5 && f0 > 0) || (one && px > 5.0 && f0 > 0) ||
      (!one && px < 5.0 && f0 < 0)) {
    float vel0 = b.v.x;
    if (w.vel_ref) { b.v.x = 0.0f; vel0 = 0.0f; }
    f0 = -vel0;
  }
  if ((py > 8.0 - 1.2 && f1 > 0) || (py < 1.2 && f1 < 0)) {
    float vel1 = b.v.y;
    if (w.vel_ref) { b.v.y = 0.0f; vel1 = 0.0f; }
    f1 = -vel1;
  }
}

HK_DEV void translation_law(World &w, Body &b, float a0, float a1, int one) {
  double vx = b.v.x, vy = b.v.y;
  double speed = sqrt(vx * vx + vy * vy);
  float f0, f1;
  if (one) { f0 = a0 * 6000.0f; f1 = a1 * 6000.0f; }
  else { f0 = (-a0) * 6000.0f; f1 = (-a1) * 6000.0f; }
  double px = b.xf.p.x, m = b.mass;
  if ((one && px > 5.0 - 0.5) || (!one && px < 5.0 + 0.5)) {
    f0 = 0.0f;
    if (one) {
      if (vx > 0) f0 = (float)((((-2.0) * vx) * m) / kDtPy);
      f0 = f0 + (float)(((((-1.0) * (px - 5.0)) * vx) * m) / kDtPy);
    } else {
      if (vx < 0) f0 = (float)((((-2.0) * vx) * m) / kDtPy);
      f0 = f0 + (float)((((1.0 * (px - 5.0)) * vx) * m) / kDtPy);
    }
    b.ld = 20.0f;
    check_boundaries(w, b, f0, f1, one);
    apply_force(b, V(f0, f1));
    return;
  }
  if (speed < 10.0) {
    b.ld = 5.0f;
    check_boundaries(w, b, f0, f1, one);
    apply_force(b, V(f0, f1));
  } else {
    b.ld = 20.0f;
    float mf = (float)m;
    float d0 = (0.02f * f0) / mf, d1 = (0.02f * f1) / mf;
    double nx = vx + (double)d0, ny = vy + (double)d1;
    if (sqrt(nx * nx + ny * ny) < speed) {
      check_boundaries(w, b, f0, f1, one);
      apply_force(b, V(f0, f1));
    }
  }
}

HK_DEV void rotation_law(Body &b, float a) {
  double ang = b.a, wv = b.w, m = b.mass;
  if (fabs(ang) > kPiD / 3) {
    double t = 0.0;
    if (ang * wv > 0) t = (((-0.1) * wv) * m) / kDtPy;
    t = t + (((-0.1) * ang) * m) / kDtPy;
    b.ad = 10.0f;
    apply_torque(b, (float)t);
  } else {
    b.ad = 2.0f;
    apply_torque(b, a * 400.0f);
  }
}

HK_DEV void shoot(World &w, const Body &p, int one) {
  double ca = hk_cos((double)p.a), sa = hk_sin((double)p.a);
  double sgn = one ? 1.0 : -1.0;
  v2 f = V((float)(ca * sgn), (float)(sa * sgn));
  float m = w.b[B_PK].mass;
  f = V(f.x * m, f.y * m);
  f = V(f.x / 0.02f, f.y / 0.02f);
  f = V(f.x * 60.0f, f.y * 60.0f);
  apply_force(w.b[B_PK], f);
}

HK_DEV void keep_puck(World &w, const Body &p) {
  Body &pk = w.b[B_PK];
  set_transform(pk, p.xf.p, pk.a);
  set_linear_velocity(pk, p.v);
}

HK_DEV float clip1(float x) { return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x); }

HK_DEV void observe(const World &w, float *o) {
  const Body &p1 = w.b[B_P1], &p2 = w.b[B_P2], &pk = w.b[B_PK];
  o[0] = p1.xf.p.x - 5.0f; o[1] = p1.xf.p.y - 4.0f; o[2] = p1.a;
  o[3] = p1.v.x; o[4] = p1.v.y; o[5] = p1.w;
  o[6] = p2.xf.p.x - 5.0f; o[7] = p2.xf.p.y - 4.0f; o[8] = p2.a;
  o[9] = p2.v.x; o[10] = p2.v.y; o[11] = p2.w;
  o[12] = pk.xf.p.x - 5.0f; o[13] = pk.xf.p.y - 4.0f;
  o[14] = pk.v.x; o[15] = pk.v.y;
  o[16] = w.keep_mode ? (float)w.has1 : 0.0f;
  o[17] = w.keep_mode ? (float)w.has2 : 0.0f;
}

HK_DEV void observe_two(const World &w, float *o) {
  const Body &p1 = w.b[B_P1], &p2 = w.b[B_P2], &pk = w.b[B_PK];
  o[0] = -(p2.xf.p.x - 5.0f); o[1] = -(p2.xf.p.y - 4.0f); o[2] = p2.a;
  o[3] = -p2.v.x; o[4] = -p2.v.y; o[5] = p2.w;
  o[6] = -(p1.xf.p.x - 5.0f); o[7] = -(p1.xf.p.y - 4.0f); o[8] = p1.a;
  o[9] = -p1.v.x; o[10] = -p1.v.y; o[11] = p1.w;
  o[12] = -(pk.xf.p.x - 5.0f); o[13] = -(pk.xf.p.y - 4.0f);
  o[14] = -pk.v.x; o[15] = -pk.v.y;
  o[16] = w.keep_mode ? (float)w.has2 : 0.0f;
  o[17] = w.keep_mode ? (float)w.has1 : 0.0f;
}

// _get_info / get_info_agent_two (hockey_env.py:542-591), double like the reference
HK_DEV void info_side(const World &w, int two, double *info4) {
  const Body &me = w.b[two ? B_P2 : B_P1], &pk = w.b[B_PK];
  double T = (double)w.max_t;
  double close = 0.0;
  int cond = two ? ((double)pk.xf.p.x > 5.0 && (double)pk.v.x >= 0) : ((double)pk.xf.p.x < 5.0 && (double)pk.v.x <= 0);
  if (cond) {
    float dx = me.xf.p.x - pk.xf.p.x, dy = me.xf.p.y - pk.xf.p.y;
    double d = sqrt((double)dx * (double)dx + (double)dy * (double)dy);
    double max_dist = 250.0 / 60.0;
    double factor = -30.0 / ((max_dist * T) / 2);
    close = close + d * factor;
  }
  double touch = ((two ? w.has2 : w.has1) == 15) ? 1.0 : 0.0;
  double f2 = two ? (-1.0) / (T * 25) : 1.0 / (T * 25);
  info4[0] = two ? -w.winner : w.winner;
  info4[1] = close;
  info4[2] = touch;
  info4[3] = (double)pk.v.x * f2;
}

HK_DEV double compute_reward(const World &w) {
  double r = 0;
  if (w.done) {
    if (w.winner == 1) r += 10;
    else if (w.winner != 0) r -= 10;
  }
  return r;
}

// the pre-solve half of HockeyEnv.step (hockey_env.py:659-680)
HK_DEV void presolve(World &w, const float *a8) {
  float a[8];
  for (int i = 0; i < 8; ++i) a[i] = clip1(a8[i]);
  Body &p1 = w.b[B_P1], &p2 = w.b[B_P2], &pk = w.b[B_PK];
  translation_law(w, p1, a[0], a[1], 1);
  rotation_law(p1, a[2]);
  translation_law(w, p2, a[4], a[5], 0);
  rotation_law(p2, a[6]);
  {
    double vx = pk.v.x, vy = pk.v.y;
    double s = sqrt(vx * vx + vy * vy);
    pk.ld = s > 25.0 ? 10.0f : 0.05f;
  }
  if (w.keep_mode) {
    if (w.has1 > 1) {
      keep_puck(w, p1);
      w.has1 -= 1;
      if (w.has1 == 1 || a[3] > 0.5f) { shoot(w, p1, 1); w.has1 = 0; }
    }
    if (w.has2 > 1) {
      keep_puck(w, p2);
      w.has2 -= 1;
      if (w.has2 == 1 || a[7] > 0.5f) { shoot(w, p2, 0); w.has2 = 0; }
    }
  }
}

// BasicOpponent.act (hockey_env.py:787-833) on an own-frame float32 obs, double arithmetic
HK_DEV void basic_opponent(int weak, int keep_mode, double &phase, double inc, const float *of, float *act) {
  double p1x = of[0], p1y = of[1], p1a = of[2];
  double v1[3] = {of[3], of[4], of[5]};
  double pkx = of[12], pky = of[13], pvx = of[14], pvy = of[15];
  double tx, ty;
  phase += inc;
  double kp = weak ? 0.5 : 10.0, kd = 0.5;
  if (pvx < 30.0 / 60.0) {
    double dx = p1x - pkx, dy = p1y - pky;
    double dist = sqrt(dx * dx + dy * dy);
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
  double ta = (kPiD / 3) * hk_sin(phase);
  double o16 = of[16];
  double shoot_ = (keep_mode && o16 > 0 && o16 < 7) ? 1.0 : 0.0;
  double err[3] = {tx - p1x, ty - p1y, ta - p1a};
  double gains[3] = {kp, kp / 5, kp / 2};
  double tb[3] = {0.1, 0.1, 0.1 * 10};
  for (int i = 0; i < 3; ++i) {
    double q = err[i] / (v1[i] + 0.01);
    if (q < 0) q = -q;
    double nb = (q < tb[i]) ? 1.0 : 0.0;
    double x = err[i] * gains[i] - (v1[i] * nb) * kd;
    act[i] = (float)(x < -1.0 ? -1.0 : (x > 1.0 ? 1.0 : x));
  }
  act[3] = (float)shoot_;
}

#undef SC
}  // namespace hk
