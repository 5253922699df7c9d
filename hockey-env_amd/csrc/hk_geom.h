// hk_geom.h -- Box2D 2.3 geometry for the hockey scene: narrow phase (b2CollidePolygonAndCircle,
// b2CollidePolygons, b2ClipSegmentToLine), GJK distance (b2Distance / b2TestOverlap), sweeps and
// conservative-advancement time of impact (b2TimeOfImpact, b2SeparationFunction).
// All functions are register-resident: fixtures come from the compile-time scene (or its LDS copy),
// simplex vertices are named (no runtime-indexed private arrays), so nothing here touches scratch memory.
// Float operation order matches the CPU test oracle bit for bit.
#pragma once
#include "hk_core.h"

namespace hk {

struct Manifold {
  v2 pt_lp[2];
  float ni[2], ti[2];
  uint32_t id[2];
  v2 ln, lp;
  int type, count;  // type 1 = faceA, 2 = faceB
};

// ------------------------------------------------------------------------------------------------
// Register fixtures.  A query copies the fixture's vertices / normals into registers once; loops run over
// the compile-time bound N with `i < count` guards (statics have 4 vertices, players 7, the puck circle 1),
// and a runtime index selects through a chain.  Whether the fixture address is wave-uniform (scalar loads)
// or per lane (a lane's own pair), nothing is re-loaded inside the loops.
// ------------------------------------------------------------------------------------------------
template <int N>
struct RFix {
  float vx[N], vy[N], nx[N], ny[N];
  int count;
  float radius;
};
template <int N>
HK_DEV RFix<N> load_fix(const Fixture &f) {
  RFix<N> r;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    r.vx[k] = f.vx[k];
    r.vy[k] = f.vy[k];
    r.nx[k] = f.nx[k];
    r.ny[k] = f.ny[k];
  }
  r.count = f.count;
  r.radius = f.radius;
  return r;
}
template <int N>
HK_DEV v2 fxv(const RFix<N> &f, int i) {
  float x = f.vx[0], y = f.vy[0];
#pragma unroll
  for (int k = 1; k < N; ++k) {
    const float xk = f.vx[k], yk = f.vy[k];
    x = (i == k) ? xk : x;
    y = (i == k) ? yk : y;
  }
  return V(x, y);
}
template <int N>
HK_DEV v2 fxn(const RFix<N> &f, int i) {
  float x = f.nx[0], y = f.ny[0];
#pragma unroll
  for (int k = 1; k < N; ++k) {
    const float xk = f.nx[k], yk = f.ny[k];
    x = (i == k) ? xk : x;
    y = (i == k) ? yk : y;
  }
  return V(x, y);
}

// b2CollidePolygonAndCircle (the circle's centre is its local position cb.vx[0], cb.vy[0])
template <int NA>
HK_DEV void collide_poly_circle(Manifold &m, const RFix<NA> &pa, xform xfA, const RFix<1> &cb, xform xfB) {
  HK_EV(EV_POLY_CIRCLE, 1);
  m.count = 0;
  const v2 cpos = V(cb.vx[0], cb.vy[0]);
  v2 c = mul_xv(xfB, cpos);
  v2 cl = mulT_xv(xfA, c);
  int ni = 0;
  float sep = -kFltMax;
  float radius = pa.radius + cb.radius;
  bool out = false;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    if (i < pa.count && !out) {
      const float s = dot(V(pa.nx[i], pa.ny[i]), vsub(cl, V(pa.vx[i], pa.vy[i])));
      if (s > radius) out = true;
      else if (s > sep) { sep = s; ni = i; }
    }
  }
  if (out) return;
  int i1 = ni, i2 = i1 + 1 < pa.count ? i1 + 1 : 0;
  v2 v1 = fxv(pa, i1), v2_ = fxv(pa, i2);
  if (sep < kFltEps) {
    m.count = 1; m.type = 1; m.ln = fxn(pa, ni); m.lp = vs(0.5f, vadd(v1, v2_));
    m.pt_lp[0] = cpos; m.id[0] = 0;
    return;
  }
  float u1 = dot(vsub(cl, v1), vsub(v2_, v1));
  float u2 = dot(vsub(cl, v2_), vsub(v1, v2_));
  if (u1 <= 0.0f) {
    if (vdist2(cl, v1) > radius * radius) return;
    m.count = 1; m.type = 1; m.ln = vsub(cl, v1); vnormalize(m.ln); m.lp = v1;
    m.pt_lp[0] = cpos; m.id[0] = 0;
  } else if (u2 <= 0.0f) {
    if (vdist2(cl, v2_) > radius * radius) return;
    m.count = 1; m.type = 1; m.ln = vsub(cl, v2_); vnormalize(m.ln); m.lp = v2_;
    m.pt_lp[0] = cpos; m.id[0] = 0;
  } else {
    v2 fc = vs(0.5f, vadd(v1, v2_));
    v2 n1 = fxn(pa, i1);
    float s = dot(vsub(cl, fc), n1);
    if (s > radius) return;
    m.count = 1; m.type = 1; m.ln = n1; m.lp = fc;
    m.pt_lp[0] = cpos; m.id[0] = 0;
  }
}

// b2FindMaxSeparation (first edge with the strictly largest separation)
template <int N1, int N2>
HK_DEV float find_max_separation(int &edge, const RFix<N1> &p1, xform xf1, const RFix<N2> &p2, xform xf2) {
  xform xf = mulT_xx(xf2, xf1);
  int best = 0;
  float maxs = -kFltMax;
#pragma unroll
  for (int i = 0; i < N1; ++i) {
    if (i < p1.count) {
      v2 n = mul_rv(xf.q, V(p1.nx[i], p1.ny[i]));
      v2 v1 = mul_xv(xf, V(p1.vx[i], p1.vy[i]));
      float si = kFltMax;
#pragma unroll
      for (int j = 0; j < N2; ++j) {
        if (j < p2.count) {
          const float sij = dot(n, vsub(V(p2.vx[j], p2.vy[j]), v1));
          si = sij < si ? sij : si;
        }
      }
      const bool take = si > maxs;
      maxs = take ? si : maxs;
      best = take ? i : best;
    }
  }
  edge = best;
  return maxs;
}

struct ClipV { v2 v; uint32_t id; };
HK_DEV uint32_t cf_id(uint32_t ia, uint32_t ib, uint32_t ta, uint32_t tb) { return ia | (ib << 8) | (ta << 16) | (tb << 24); }

template <int N1, int N2>
HK_DEV void find_incident_edge(ClipV c[2], const RFix<N1> &p1, xform xf1, int edge1, const RFix<N2> &p2, xform xf2) {
  v2 n1 = mulT_rv(xf2.q, mul_rv(xf1.q, fxn(p1, edge1)));
  int index = 0;
  float mind = kFltMax;
#pragma unroll
  for (int i = 0; i < N2; ++i) {
    if (i < p2.count) {
      const float d = dot(n1, V(p2.nx[i], p2.ny[i]));
      const bool take = d < mind;
      mind = take ? d : mind;
      index = take ? i : index;
    }
  }
  int i1 = index, i2 = i1 + 1 < p2.count ? i1 + 1 : 0;
  c[0].v = mul_xv(xf2, fxv(p2, i1));
  c[0].id = cf_id(edge1, i1, 1, 0);
  c[1].v = mul_xv(xf2, fxv(p2, i2));
  c[1].id = cf_id(edge1, i2, 1, 0);
}

// b2ClipSegmentToLine, written with selects (no dynamically indexed private arrays)
HK_DEV int clip_segment(ClipV out[2], const ClipV in[2], v2 normal, float offset, int vA) {
  const float d0 = dot(normal, in[0].v) - offset;
  const float d1 = dot(normal, in[1].v) - offset;
  const bool k0 = d0 <= 0.0f, k1 = d1 <= 0.0f, cross = d0 * d1 < 0.0f;
  const float interp = d0 / (d0 - d1);  // used only when the segment crosses the line
  ClipV ix;
  ix.v = vadd(in[0].v, vs(interp, vsub(in[1].v, in[0].v)));
  ix.id = cf_id(vA, (in[0].id >> 8) & 0xffu, 0, 1);
  out[0] = k0 ? in[0] : (k1 ? in[1] : ix);
  out[1] = (k0 && k1) ? in[1] : ix;
  return (int)k0 + (int)k1 + (int)cross;
}

// the reference-face part of b2CollidePolygons (p1 = reference polygon, p2 = incident polygon)
template <int N1, int N2>
HK_DEV void clip_polygons(Manifold &m, const RFix<N1> &p1, xform xf1, int edge1, const RFix<N2> &p2, xform xf2,
                          bool flip, float total) {
  m.type = flip ? 2 : 1;
  ClipV inc[2];
  find_incident_edge(inc, p1, xf1, edge1, p2, xf2);
  int iv1 = edge1, iv2 = edge1 + 1 < p1.count ? edge1 + 1 : 0;
  v2 v11 = fxv(p1, iv1), v12 = fxv(p1, iv2);
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
  v2 q[2];
  uint32_t qid[2];
  bool keep[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float sep = dot(normal, cp2[i].v) - front;
    keep[i] = sep <= total;
    q[i] = mulT_xv(xf2, cp2[i].v);
    uint32_t id = cp2[i].id;
    if (flip) id = cf_id((id >> 8) & 0xffu, id & 0xffu, (id >> 24) & 0xffu, (id >> 16) & 0xffu);
    qid[i] = id;
  }
  // kept points, in order
  m.pt_lp[0] = keep[0] ? q[0] : q[1];
  m.id[0] = keep[0] ? qid[0] : qid[1];
  m.pt_lp[1] = q[1];
  m.id[1] = qid[1];
  m.count = (int)keep[0] + (int)keep[1];
}

// b2CollidePolygons
template <int NA, int NB>
HK_DEV void collide_polygons(Manifold &m, const RFix<NA> &pA, xform xfA, const RFix<NB> &pB, xform xfB) {
  HK_EV(EV_POLYGONS, 1);
  m.count = 0;
  float total = pA.radius + pB.radius;
  int eA = 0, eB = 0;
  float sA = find_max_separation(eA, pA, xfA, pB, xfB);
  if (sA > total) return;
  float sB = find_max_separation(eB, pB, xfB, pA, xfA);
  if (sB > total) return;
  const float k_tol = 0.1f * kLinearSlop;
  if (sB > sA + k_tol) clip_polygons(m, pB, xfB, eB, pA, xfA, true, total);
  else clip_polygons(m, pA, xfA, eA, pB, xfB, false, total);
}

// ------------------------------------------------------------------------------------------------
// GJK distance + TOI (b2Distance.cpp, b2TimeOfImpact.cpp)
// ------------------------------------------------------------------------------------------------
// Register proxies: the fixture's vertices are copied into registers once per query (statics have <= 4
// vertices, players 7, the puck 1), so GJK / TOI iterations run on registers instead of re-loading
// vertices from memory with per-lane addresses.  Vertex fetch by index is a select chain.
template <int N, bool kStaticBody = false>
struct Proxy {
  static constexpr bool kStatic = kStaticBody;  // the fixture's body never moves (sweep c0 == c, angle 0)
  float vx[N], vy[N];
  int count;
  float radius;
};
template <int N, bool kStaticBody = false>
HK_DEV Proxy<N, kStaticBody> make_proxy(const Fixture &f) {
  Proxy<N, kStaticBody> p;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    p.vx[k] = f.vx[k];
    p.vy[k] = f.vy[k];
  }
  p.count = f.count;
  p.radius = f.radius;
  return p;
}
template <int N, bool S>
HK_DEV v2 pv(const Proxy<N, S> &p, int i) {
  float x = p.vx[0], y = p.vy[0];
#pragma unroll
  for (int k = 1; k < N; ++k) {
    const float xk = p.vx[k], yk = p.vy[k];
    x = (i == k) ? xk : x;
    y = (i == k) ? yk : y;
  }
  return V(x, y);
}
// b2DistanceProxy::GetSupport: first vertex with the strictly largest projection
template <int N, bool S>
HK_DEV int proxy_support(const Proxy<N, S> &p, v2 d) {
  int best = 0;
  float bv = dot(V(p.vx[0], p.vy[0]), d);
#pragma unroll
  for (int i = 1; i < N; ++i) {
    const float v = dot(V(p.vx[i], p.vy[i]), d);
    const bool take = (i < p.count) && (v > bv);
    best = take ? i : best;
    bv = take ? v : bv;
  }
  return best;
}

// ---- GJK with a register-resident simplex (b2Simplex m_v1/m_v2/m_v3) ----
struct SimplexCache { float metric; int count; int iA[3], iB[3]; };
struct SVert { v2 wA, wB, w; float a; int iA, iB; };
struct Simplex { SVert v1, v2, v3; int count; };

HK_DEV float simplex_metric(const Simplex &s) {
  if (s.count == 2) return vdist(s.v1.w, s.v2.w);
  if (s.count == 3) return crs(vsub(s.v2.w, s.v1.w), vsub(s.v3.w, s.v1.w));
  return 0.0f;
}
template <typename PA, typename PB>
HK_DEV SVert make_svert(const PA &pA, xform xA, const PB &pB, xform xB, int iA, int iB) {
  SVert v;
  v.iA = iA;
  v.iB = iB;
  v.wA = mul_xv(xA, pv(pA, iA));
  v.wB = mul_xv(xB, pv(pB, iB));
  v.w = vsub(v.wB, v.wA);
  v.a = 0.0f;
  return v;
}
template <typename PA, typename PB>
HK_DEV void simplex_read(Simplex &s, const SimplexCache &cache, const PA &pA, xform xA, const PB &pB, xform xB) {
  s.count = cache.count;
  s.v1.wA = s.v1.wB = s.v1.w = V(0.0f, 0.0f);
  s.v1.a = 0.0f;
  s.v1.iA = s.v1.iB = 0;
  s.v2 = s.v1;
  s.v3 = s.v1;
  if (s.count > 0) s.v1 = make_svert(pA, xA, pB, xB, cache.iA[0], cache.iB[0]);
  if (s.count > 1) s.v2 = make_svert(pA, xA, pB, xB, cache.iA[1], cache.iB[1]);
  if (s.count > 2) s.v3 = make_svert(pA, xA, pB, xB, cache.iA[2], cache.iB[2]);
  if (s.count > 1) {
    float m1 = cache.metric, m2 = simplex_metric(s);
    if (m2 < 0.5f * m1 || 2.0f * m1 < m2 || m2 < kFltEps) s.count = 0;
  }
  if (s.count == 0) {
    s.v1 = make_svert(pA, xA, pB, xB, 0, 0);
    s.v1.a = 1.0f;
    s.count = 1;
  }
}
HK_DEV void simplex_write(const Simplex &s, SimplexCache &cache) {
  cache.metric = simplex_metric(s);
  cache.count = s.count;
  cache.iA[0] = s.v1.iA; cache.iB[0] = s.v1.iB;
  cache.iA[1] = s.v2.iA; cache.iB[1] = s.v2.iB;
  cache.iA[2] = s.v3.iA; cache.iB[2] = s.v3.iB;
}
HK_DEV v2 simplex_search_dir(const Simplex &s) {
  if (s.count == 1) return vneg(s.v1.w);
  v2 e12 = vsub(s.v2.w, s.v1.w);
  float sgn = crs(e12, vneg(s.v1.w));
  if (sgn > 0.0f) return crs_sv(1.0f, e12);
  return crs_vs(e12, 1.0f);
}
HK_DEV void simplex_witness(const Simplex &s, v2 &pA, v2 &pB) {
  if (s.count == 1) { pA = s.v1.wA; pB = s.v1.wB; }
  else if (s.count == 2) {
    pA = vadd(vs(s.v1.a, s.v1.wA), vs(s.v2.a, s.v2.wA));
    pB = vadd(vs(s.v1.a, s.v1.wB), vs(s.v2.a, s.v2.wB));
  } else {
    pA = vadd(vadd(vs(s.v1.a, s.v1.wA), vs(s.v2.a, s.v2.wA)), vs(s.v3.a, s.v3.wA));
    pB = pA;
  }
}
HK_DEV void solve2(Simplex &s) {
  v2 w1 = s.v1.w, w2 = s.v2.w;
  v2 e12 = vsub(w2, w1);
  float d12_2 = -dot(w1, e12);
  if (d12_2 <= 0.0f) { s.v1.a = 1.0f; s.count = 1; return; }
  float d12_1 = dot(w2, e12);
  if (d12_1 <= 0.0f) { s.v2.a = 1.0f; s.count = 1; s.v1 = s.v2; return; }
  float inv = 1.0f / (d12_1 + d12_2);
  s.v1.a = d12_1 * inv;
  s.v2.a = d12_2 * inv;
  s.count = 2;
}
HK_DEV void solve3(Simplex &s) {
  v2 w1 = s.v1.w, w2 = s.v2.w, w3 = s.v3.w;
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
  if (d12_2 <= 0.0f && d13_2 <= 0.0f) { s.v1.a = 1.0f; s.count = 1; return; }
  if (d12_1 > 0.0f && d12_2 > 0.0f && d123_3 <= 0.0f) {
    float inv = 1.0f / (d12_1 + d12_2);
    s.v1.a = d12_1 * inv; s.v2.a = d12_2 * inv; s.count = 2; return;
  }
  if (d13_1 > 0.0f && d13_2 > 0.0f && d123_2 <= 0.0f) {
    float inv = 1.0f / (d13_1 + d13_2);
    s.v1.a = d13_1 * inv; s.v3.a = d13_2 * inv; s.count = 2; s.v2 = s.v3; return;
  }
  if (d12_1 <= 0.0f && d23_2 <= 0.0f) { s.v2.a = 1.0f; s.count = 1; s.v1 = s.v2; return; }
  if (d13_1 <= 0.0f && d23_1 <= 0.0f) { s.v3.a = 1.0f; s.count = 1; s.v1 = s.v3; return; }
  if (d23_1 > 0.0f && d23_2 > 0.0f && d123_1 <= 0.0f) {
    float inv = 1.0f / (d23_1 + d23_2);
    s.v2.a = d23_1 * inv; s.v3.a = d23_2 * inv; s.count = 2; s.v1 = s.v3; return;
  }
  float inv = 1.0f / (d123_1 + d123_2 + d123_3);
  s.v1.a = d123_1 * inv; s.v2.a = d123_2 * inv; s.v3.a = d123_3 * inv; s.count = 3;
}

// b2Distance (returns the distance; witness points are not needed by the callers)
template <typename PA, typename PB>
HK_DEV float gjk_distance(SimplexCache &cache, const PA &pA, xform xA, const PB &pB, xform xB, int use_radii) {
  Simplex s;
  HK_EV(EV_GJK, 1);
  simplex_read(s, cache, pA, xA, pB, xB);
  int sA0 = 0, sA1 = 0, sA2 = 0, sB0 = 0, sB1 = 0, sB2 = 0, saveCount;
  int iter = 0;
  while (iter < 20) {
    HK_EV(EV_GJK_IT, 1);
    saveCount = s.count;
    sA0 = s.v1.iA; sB0 = s.v1.iB;
    sA1 = s.v2.iA; sB1 = s.v2.iB;
    sA2 = s.v3.iA; sB2 = s.v3.iB;
    if (s.count == 2) solve2(s);
    else if (s.count == 3) solve3(s);
    if (s.count == 3) break;
    v2 d = simplex_search_dir(s);
    if (vlen2(d) < kFltEps * kFltEps) break;
    const int iA = proxy_support(pA, mulT_rv(xA.q, vneg(d)));
    const int iB = proxy_support(pB, mulT_rv(xB.q, d));
    SVert nv;
    nv.iA = iA;
    nv.wA = mul_xv(xA, pv(pA, iA));
    nv.iB = iB;
    nv.wB = mul_xv(xB, pv(pB, iB));
    nv.w = vsub(nv.wB, nv.wA);
    nv.a = 0.0f;
    if (s.count == 1) s.v2 = nv; else s.v3 = nv;
    ++iter;
    bool dup = (saveCount > 0 && iA == sA0 && iB == sB0) || (saveCount > 1 && iA == sA1 && iB == sB1) ||
               (saveCount > 2 && iA == sA2 && iB == sB2);
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
  const Proxy<kStaticVerts> pA = make_proxy<kStaticVerts>(fA);  // A: a static goal sensor
  const Proxy<kMaxPolyVerts> pB = make_proxy<kMaxPolyVerts>(fB);
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
// b2Sweep::GetTransform of the proxy's body: a static body has a0 == a == +0 and local centre 0, so the
// angle interpolates to +0 exactly, rot_set(+0) == (+0, 1) and the centre offset subtracts +0 -- only the
// position interpolation remains (it is kept: (1-b)*c0 + b*c need not round to c).
template <typename P>
HK_DEV void sweep_xf_of(const Sweep &s, xform &xf, float beta) {
  if constexpr (P::kStatic) {
    xf.p = vadd(vs(1.0f - beta, s.c0), vs(beta, s.c));
    xf.q.s = 0.0f;
    xf.q.c = 1.0f;
  } else {
    sweep_xf(s, xf, beta);
  }
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

enum { SF_POINTS = 0, SF_FACEA, SF_FACEB };
template <typename PA, typename PB>
struct SepFn {
  PA pA;
  PB pB;
  Sweep sA, sB;
  int type;
  v2 lp, axis;
};

template <typename PA, typename PB>
HK_DEV void sep_init(SepFn<PA, PB> &f, const SimplexCache &cache, const PA &pA, const Sweep &sA, const PB &pB,
                     const Sweep &sB, float t1) {
  f.pA = pA; f.pB = pB; f.sA = sA; f.sB = sB;
  xform xA, xB;
  sweep_xf_of<PA>(f.sA, xA, t1);
  sweep_xf_of<PB>(f.sB, xB, t1);
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
// The three separation-function types evaluate the same shape of expression with the roles of A / B, the local
// point and the axis rotation swapped; here the roles are picked by selects and one expression is evaluated, with
// each type's float operations in its own order.  The cooperative TOI drain runs different pairs (so different
// types) on the lanes of a wave, and the if-chain ran all three bodies behind exec masks (r06).
template <typename PA, typename PB>
HK_DEV float sep_find_min(const SepFn<PA, PB> &f, int &iA, int &iB, float t) {
  HK_EV(EV_SEP_MIN, 1);
  xform xA, xB;
  sweep_xf_of<PA>(f.sA, xA, t);
  sweep_xf_of<PB>(f.sB, xB, t);
  const bool pts = f.type == SF_POINTS, fa = f.type == SF_FACEA, fb = f.type == SF_FACEB;
  const rot q = fa ? xA.q : xB.q;
  const v2 nr = mul_rv(q, f.axis);
  const v2 n = pts ? f.axis : nr;  // points: the axis; face A / B: the axis rotated by A / B
  const v2 axA = mulT_rv(xA.q, pts ? f.axis : vneg(n)), axB = mulT_rv(xB.q, vneg(n));
  const int sA = proxy_support(f.pA, axA), sB = proxy_support(f.pB, axB);
  iA = fa ? -1 : sA;
  iB = fb ? -1 : sB;
  const v2 a = mul_xv(xA, fa ? f.lp : pv(f.pA, sA)), b = mul_xv(xB, fb ? f.lp : pv(f.pB, sB));
  return dot(fb ? vsub(a, b) : vsub(b, a), n);
}
template <typename PA, typename PB>
HK_DEV float sep_eval(const SepFn<PA, PB> &f, int iA, int iB, float t) {
  HK_EV(EV_SEP_EVAL, 1);
  xform xA, xB;
  sweep_xf_of<PA>(f.sA, xA, t);
  sweep_xf_of<PB>(f.sB, xB, t);
  const bool pts = f.type == SF_POINTS, fa = f.type == SF_FACEA, fb = f.type == SF_FACEB;
  const rot q = fa ? xA.q : xB.q;
  const v2 nr = mul_rv(q, f.axis);
  const v2 n = pts ? f.axis : nr;
  const v2 a = mul_xv(xA, fa ? f.lp : pv(f.pA, iA)), b = mul_xv(xB, fb ? f.lp : pv(f.pB, iB));
  return dot(fb ? vsub(a, b) : vsub(b, a), n);
}

enum { TOI_UNKNOWN = 0, TOI_FAILED, TOI_OVERLAPPED, TOI_TOUCHING, TOI_SEPARATED };

template <typename PA, typename PB>
HK_DEV int time_of_impact(const PA &pA, const PB &pB, Sweep sA, Sweep sB, float tMax, float &t_out) {
  HK_EV(EV_TOI, 1);
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
    sweep_xf_of<PA>(sA, xA, t1);
    sweep_xf_of<PB>(sB, xB, t1);
    float dist = gjk_distance(cache, pA, xA, pB, xB, 0);
    if (dist <= 0.0f) { state = TOI_OVERLAPPED; t_out = 0.0f; break; }
    if (dist < target + tol) { state = TOI_TOUCHING; t_out = t1; break; }
    SepFn<PA, PB> fcn;
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

}  // namespace hk
