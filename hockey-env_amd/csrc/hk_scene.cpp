// hk_scene.cpp -- host construction of the static scene (run at build time by hk_scene_gen.cpp).
//
// Geometry of hockey/hockey_env.py:183-343 (players :183-202, puck :204-220, walls/posts :222-319,
// goals :321-343) turned into Box2D 2.3 shapes exactly as box2d-py would: vertices are computed in
// double by the reference and rounded to float32, b2PolygonShape::Set welds + gift-wraps them into a
// CCW hull with unit normals, and b2PolygonShape/b2CircleShape::ComputeMass + b2Body::ResetMassData
// give the float32 mass, centre and inertia.  The contact pair table is the category/mask filter of
// SURVEY.md A.3 in a fixed canonical order.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "hk_kernels.h"

namespace hk {
namespace {

struct hv2 { float x, y; };
inline hv2 H(float x, float y) { return {x, y}; }
inline hv2 hsub(hv2 a, hv2 b) { return H(a.x - b.x, a.y - b.y); }
inline hv2 hadd(hv2 a, hv2 b) { return H(a.x + b.x, a.y + b.y); }
inline hv2 hs(float s, hv2 a) { return H(s * a.x, s * a.y); }
inline float hdot(hv2 a, hv2 b) { return a.x * b.x + a.y * b.y; }
inline float hcrs(hv2 a, hv2 b) { return a.x * b.y - a.y * b.x; }

void poly_set(Fixture &f, const hv2 *in, int count) {
  hv2 ps[kMaxPolyVerts];
  int n = 0;
  for (int i = 0; i < count; ++i) {
    bool uniq = true;
    for (int j = 0; j < n; ++j) {
      hv2 d = hsub(in[i], ps[j]);
      if (hdot(d, d) < 0.5f * kLinearSlop) { uniq = false; break; }
    }
    if (uniq) ps[n++] = in[i];
  }
  int i0 = 0;
  float x0 = ps[0].x;
  for (int i = 1; i < n; ++i) {
    float x = ps[i].x;
    if (x > x0 || (x == x0 && ps[i].y < ps[i0].y)) { i0 = i; x0 = x; }
  }
  int hull[kMaxPolyVerts], m = 0, ih = i0;
  for (;;) {
    hull[m] = ih;
    int ie = 0;
    for (int j = 1; j < n; ++j) {
      if (ie == ih) { ie = j; continue; }
      hv2 r = hsub(ps[ie], ps[hull[m]]);
      hv2 v = hsub(ps[j], ps[hull[m]]);
      float c = hcrs(r, v);
      if (c < 0.0f) ie = j;
      if (c == 0.0f && hdot(v, v) > hdot(r, r)) ie = j;
    }
    ++m;
    ih = ie;
    if (ie == i0) break;
  }
  f.count = m;
  for (int i = 0; i < m; ++i) { f.vx[i] = ps[hull[i]].x; f.vy[i] = ps[hull[i]].y; }
  for (int i = 0; i < m; ++i) {
    int i2 = i + 1 < m ? i + 1 : 0;
    hv2 e = H(f.vx[i2] - f.vx[i], f.vy[i2] - f.vy[i]);
    hv2 nrm = H(1.0f * e.y, -1.0f * e.x);  // b2Cross(edge, 1)
    float l = std::sqrt(nrm.x * nrm.x + nrm.y * nrm.y);
    if (l >= kFltEps) {
      float inv = 1.0f / l;
      nrm.x *= inv;
      nrm.y *= inv;
    }
    f.nx[i] = nrm.x;
    f.ny[i] = nrm.y;
  }
  f.circle = 0;
  f.radius = kPolyRadius;
}

void body_mass_from(float mass, hv2 center, float I, float &m_out, float &im, hv2 &lc, float &Ib, float &iI) {
  m_out = 0.0f + mass;
  hv2 l = hadd(H(0.0f, 0.0f), hs(mass, center));
  Ib = 0.0f + I;
  im = 1.0f / m_out;
  l = hs(im, l);
  Ib -= m_out * hdot(l, l);
  iI = 1.0f / Ib;
  lc = l;
}

void poly_mass(const Fixture &f, float density, float &m, float &im, hv2 &lc, float &Ib, float &iI) {
  hv2 center = H(0.0f, 0.0f), s = H(0.0f, 0.0f);
  float area = 0.0f, I = 0.0f;
  for (int i = 0; i < f.count; ++i) s = hadd(s, H(f.vx[i], f.vy[i]));
  s = hs(1.0f / (float)f.count, s);
  const float k_inv3 = 1.0f / 3.0f;
  for (int i = 0; i < f.count; ++i) {
    hv2 e1 = hsub(H(f.vx[i], f.vy[i]), s);
    int j = i + 1 < f.count ? i + 1 : 0;
    hv2 e2 = hsub(H(f.vx[j], f.vy[j]), s);
    float D = hcrs(e1, e2);
    float tri = 0.5f * D;
    area += tri;
    center = hadd(center, hs(tri * k_inv3, hadd(e1, e2)));
    float ex1 = e1.x, ey1 = e1.y, ex2 = e2.x, ey2 = e2.y;
    float intx2 = ex1 * ex1 + ex2 * ex1 + ex2 * ex2;
    float inty2 = ey1 * ey1 + ey2 * ey1 + ey2 * ey2;
    I += (0.25f * k_inv3 * D) * (intx2 + inty2);
  }
  float mass = density * area;
  center = hs(1.0f / area, center);
  hv2 mc = hadd(center, s);
  float Im = density * I;
  Im += mass * (hdot(mc, mc) - hdot(center, center));
  body_mass_from(mass, mc, Im, m, im, lc, Ib, iI);
}

void poly_fixture(Scene &sc, int fi, int bi, const double (*px)[2], int sensor) {
  const double SCALE = 60.0;
  hv2 in[4];
  for (int k = 0; k < 4; ++k) in[k] = H((float)(px[k][0] / SCALE), (float)(px[k][1] / SCALE));
  Fixture &f = sc.fx[fi];
  poly_set(f, in, 4);
  f.body = bi;
  f.sensor = sensor;
  f.friction = 0.1f;
  f.restitution = 0.0f;
}

}  // namespace

void build_scene(Scene &sc) {
  std::memset(&sc, 0, sizeof(sc));
  const double SCALE = 60.0, W = 600.0 / SCALE, Hh = 480.0 / SCALE;
  const double wall[4][2] = {{-250, 10}, {-250, -10}, {250, -10}, {250, 10}};
  const double a135 = (Hh - 1) / 2 * SCALE - 75, a128 = (Hh - 1) / 2 * SCALE - 75 - 7;
  const double post[4][2] = {{-10, a135}, {10, a128}, {10, -5}, {-10, -5}};
  double plt[4][2], prt[4][2], prb[4][2];
  for (int i = 0; i < 4; ++i) {
    plt[i][0] = post[i][0]; plt[i][1] = -post[i][1];
    prt[i][0] = -post[i][0]; prt[i][1] = -post[i][1];
    prb[i][0] = -post[i][0]; prb[i][1] = post[i][1];
  }
  const double goal[4][2] = {{-10, 75}, {10, 75}, {10, -75}, {-10, -75}};
  poly_fixture(sc, F_WT, B_WT, wall, 0);
  poly_fixture(sc, F_WB, B_WB, wall, 0);
  poly_fixture(sc, F_PLT, B_PLT, plt, 0);
  poly_fixture(sc, F_PLB, B_PLB, post, 0);
  poly_fixture(sc, F_PRT, B_PRT, prt, 0);
  poly_fixture(sc, F_PRB, B_PRB, prb, 0);
  poly_fixture(sc, F_G1S, B_G1, goal, 1);
  poly_fixture(sc, F_G1, B_G1, goal, 0);
  poly_fixture(sc, F_G2S, B_G2, goal, 1);
  poly_fixture(sc, F_G2, B_G2, goal, 0);
  const double spos[8][2] = {{W / 2, Hh - .5}, {W / 2, .5}, {W / 2 - 245 / SCALE, Hh - .5}, {W / 2 - 245 / SCALE, .5},
                             {W / 2 + 245 / SCALE, Hh - .5}, {W / 2 + 245 / SCALE, 0.5},
                             {W / 2 - 245 / SCALE - 10 / SCALE, Hh / 2}, {W / 2 + 245 / SCALE + 10 / SCALE, Hh / 2}};
  for (int i = 0; i < 8; ++i) {
    sc.spx[B_WT + i] = (float)spos[i][0];
    sc.spy[B_WT + i] = (float)spos[i][1];
  }
  const double rack[7][2] = {{-10, 20}, {5, 20}, {5, -20}, {-10, -20}, {-18, -10}, {-21, 0}, {-18, 10}};
  for (int p = 0; p < 2; ++p) {
    hv2 in[7];
    for (int i = 0; i < 7; ++i) {
      double x = p ? (-rack[i][0]) / SCALE * 1.2 : rack[i][0] / SCALE * 1.2;
      in[i] = H((float)x, (float)(rack[i][1] / SCALE * 1.2));
    }
    Fixture &f = sc.fx[p ? F_P2 : F_P1];
    poly_set(f, in, 7);
    f.body = p ? B_P2 : B_P1;
    f.sensor = 0;
    f.friction = 1.0f;
    f.restitution = 0.0f;
    hv2 lc;
    poly_mass(f, (float)(200.0 / 1.2), sc.mass[p], sc.invMass[p], lc, sc.I[p], sc.invI[p]);
    sc.lcx[p] = lc.x;
    sc.lcy[p] = lc.y;
  }
  Fixture &pk = sc.fx[F_PK];
  pk.circle = 1;
  pk.count = 1;
  pk.vx[0] = 0.0f;
  pk.vy[0] = 0.0f;
  pk.radius = (float)(13 / SCALE);
  pk.body = B_PK;
  pk.friction = 0.1f;
  pk.restitution = 0.95f;
  {
    const float r = pk.radius, density = 7.0f;
    float mass = density * kPi * r * r;
    float I = mass * (0.5f * r * r + hdot(H(0.0f, 0.0f), H(0.0f, 0.0f)));
    hv2 lc;
    body_mass_from(mass, H(0.0f, 0.0f), I, sc.mass[B_PK], sc.invMass[B_PK], lc, sc.I[B_PK], sc.invI[B_PK]);
    sc.lcx[B_PK] = lc.x;
    sc.lcy[B_PK] = lc.y;
  }
  // canonical pair table {fixture A, fixture B}: A = polygon / static side, B = circle / dynamic side
  const int pairs[NP][2] = {
      {F_WT, F_PK}, {F_WB, F_PK}, {F_PLT, F_PK}, {F_PLB, F_PK}, {F_PRT, F_PK}, {F_PRB, F_PK},
      {F_G1S, F_PK}, {F_G2S, F_PK}, {F_P1, F_PK}, {F_P2, F_PK}, {F_P1, F_P2},
      {F_WT, F_P1}, {F_WB, F_P1}, {F_PLT, F_P1}, {F_PLB, F_P1}, {F_PRT, F_P1}, {F_PRB, F_P1},
      {F_G1, F_P1}, {F_G2, F_P1},
      {F_WT, F_P2}, {F_WB, F_P2}, {F_PLT, F_P2}, {F_PLB, F_P2}, {F_PRT, F_P2}, {F_PRB, F_P2},
      {F_G1, F_P2}, {F_G2, F_P2}};
  int slot = 0;
  for (int p = 0; p < NP; ++p) {
    const Fixture &fA = sc.fx[pairs[p][0]], &fB = sc.fx[pairs[p][1]];
    sc.pairA[p] = pairs[p][0];
    sc.pairB[p] = pairs[p][1];
    sc.pbodyA[p] = fA.body;
    sc.pbodyB[p] = fB.body;
    sc.sensor[p] = fA.sensor || fB.sensor;
    sc.friction[p] = std::sqrt(fA.friction * fB.friction);                      // b2MixFriction
    sc.restitution[p] = fA.restitution > fB.restitution ? fA.restitution : fB.restitution;  // b2MixRestitution
    sc.manslot[p] = sc.sensor[p] ? -1 : slot++;
    // the solver derives radii from this layout (hk_solver.h pair_rA / pair_rB)
    if (fA.radius != kPolyRadius || (fB.body != B_PK && fB.radius != kPolyRadius) || fA.body == B_PK) std::abort();
    // TOI and sensor queries hold a static fixture A in a 4-vertex register proxy (hk_geom.h)
    if (fA.body >= B_WT && fA.count > kStaticVerts) std::abort();
  }
  for (int f = 0; f < NF; ++f) {
    const Fixture &fx = sc.fx[f];
    if (fx.body < B_WT) continue;
    float mnx = 1e30f, mny = 1e30f, mxx = -1e30f, mxy = -1e30f;
    for (int k = 0; k < fx.count; ++k) {
      float x = fx.vx[k] + sc.spx[fx.body], y = fx.vy[k] + sc.spy[fx.body];
      mnx = x < mnx ? x : mnx; mny = y < mny ? y : mny; mxx = x > mxx ? x : mxx; mxy = y > mxy ? y : mxy;
    }
    sc.fx_aabb[f][0] = mnx; sc.fx_aabb[f][1] = mny; sc.fx_aabb[f][2] = mxx; sc.fx_aabb[f][3] = mxy;
  }
  for (int b = 0; b < 3; ++b) {
    const Fixture &fx = sc.fx[b == B_PK ? F_PK : (b == B_P1 ? F_P1 : F_P2)];
    float r = 0.0f;
    for (int k = 0; k < fx.count; ++k) {
      float dx = fx.vx[k] - sc.lcx[b], dy = fx.vy[k] - sc.lcy[b];
      float d = std::sqrt(dx * dx + dy * dy);
      r = d > r ? d : r;
    }
    sc.rcore[b] = r;
  }
  const int e1[10] = {8, 10, 11, 12, 13, 14, 15, 16, 17, 18};
  const int e2[10] = {9, 10, 19, 20, 21, 22, 23, 24, 25, 26};
  for (int k = 0; k < 10; ++k) {
    sc.edges[B_P1][k] = e1[k];
    sc.edges[B_P2][k] = e2[k];
    sc.edges[B_PK][k] = k;
  }
}

}  // namespace hk
