/* Test harness (tests/test_broadphase_bound.py): hill-climbs the ratio of the radius-free (core) distance to the
   total radius over player-vs-polygon configurations where the oracle's b2CollidePolygons restatement emits
   contact points.  The kernel's collide broad phase (hk_arena.h pair_far_collide) rejects polygon pairs beyond
   2 x total radius + kFarMargin; this measures how much of that bound contacts actually use. */
#ifndef RESTARTS
#define RESTARTS 300
#endif
#include "../../oracle/hk_oracle.c"
/* Hill-climb the core-distance / total-radius ratio over touching player-vs-fixture configurations. */
static unsigned long long st = 0x9E3779B97F4A7C15ull;
static double rnd(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return (st >> 11) * (1.0 / 9007199254740992.0); }
static const int statics[9] = {F_WT, F_WB, F_PLT, F_PLB, F_PRT, F_PRB, F_G1, F_G2, F_P2};
static double ratio(int k, double px, double py, double pa, double qa, int *touch) {
  const fixture *fa = FX(statics[k]), *fb = FX(F_P1);
  xform xa, xb;
  if (k < 8) xa = SCENE.proto[fa->body].xf; else { xa.p = V(5.0f, 4.0f); xa.q = rot_set((float)qa); }
  xb.p = V((float)px, (float)py); xb.q = rot_set((float)pa);
  manifold m; collide_polygons(&m, fa, xa, fb, xb);
  *touch = m.count > 0;
  proxy A = make_proxy(fa), B = make_proxy(fb); simplex_cache c; c.count = 0; c.metric = 0; v2 oa, ob;
  return gjk_distance(&c, &A, xa, &B, xb, 0, &oa, &ob) / (fa->radius + fb->radius);
}
int main(void) {
  init_scene();
  double overall = 0;
  for (int k = 0; k < 9; ++k) {
    double best = 0;
    for (int restart = 0; restart < RESTARTS; ++restart) {
      const fixture *fa = FX(statics[k]);
      v2 base = k < 8 ? vadd(SCENE.proto[fa->body].xf.p, fa->v[(int)(rnd() * fa->count)]) : V(5.0f, 4.0f);
      double px = base.x + (rnd() - 0.5) * 1.0, py = base.y + (rnd() - 0.5) * 1.0, pa = (rnd() - 0.5) * 6.3, qa = (rnd() - 0.5) * 6.3;
      int t; double r = ratio(k, px, py, pa, qa, &t);
      int tries = 0;
      while (!t && tries++ < 2000) { px = base.x + (rnd() - 0.5) * 1.0; py = base.y + (rnd() - 0.5) * 1.0; pa = (rnd() - 0.5) * 6.3; r = ratio(k, px, py, pa, qa, &t); }
      if (!t) continue;
      double step = 0.02;
      for (int it = 0; it < 20000; ++it) {
        double nx = px + (rnd() - 0.5) * step, ny = py + (rnd() - 0.5) * step, na = pa + (rnd() - 0.5) * step * 3, nq = qa + (rnd() - 0.5) * step * 3;
        int tt; double rr = ratio(k, nx, ny, na, nq, &tt);
        if (tt && rr >= r) { px = nx; py = ny; pa = na; qa = nq; r = rr; }
        if (it % 4000 == 3999) step *= 0.5;
      }
      if (r > best) best = r;
    }
    printf("fixture %d: max core-distance / total-radius with contact %.4f\n", k, best);
    if (best > overall) overall = best;
  }
  printf("overall %.4f\n", overall);
}
