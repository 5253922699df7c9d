// hk_core.h -- per-arena physics of the hockey hot path, CDNA4 device code.
//
// One lane simulates one arena.  This is the MI355X implementation of
//   hockey/hockey_env.py:658-695  HockeyEnv.step (pre-solve laws :436-483, :610-633, obs/info/reward :485-591)
//   hockey/hockey_env.py:44-76    ContactDetector.BeginContact (goal / possession events)
//   hockey/hockey_env.py:682      world.Step(0.02, 180, 60) -> Box2D 2.3 b2World::Step semantics for this scene
//   hockey/hockey_env.py:781-833  BasicOpponent.act (fused policy)
// Float operation order follows Box2D 2.3 / the reference's numpy+pybox2d semantics exactly; the file is
// compiled with -ffp-contract=off and IEEE div/sqrt so results are bit-identical to the CPU oracle
// (tests/test_gpu_parity.py).  Scene constants (hulls, normals, masses) are computed on the host at build
// time (hk_scene.cpp via hk_scene_gen.cpp) and compiled in as a constexpr Scene.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef HK_DEV
#define HK_DEV __device__ __forceinline__
#endif

namespace hk {

// ---------------------------------------------------------------------------------------------
// Box2D 2.3 settings (b2Settings.h)
// ---------------------------------------------------------------------------------------------
constexpr float kPi = 3.14159265359f;
constexpr float kLinearSlop = 0.005f;
constexpr float kPolyRadius = 2.0f * kLinearSlop;
constexpr float kMaxTranslation = 2.0f;
constexpr float kMaxRotation = 0.5f * kPi;
constexpr float kBaumgarte = 0.2f;
constexpr float kToiBaumgarte = 0.75f;
constexpr float kMaxLinearCorrection = 0.2f;
constexpr float kVelocityThreshold = 1.0f;
constexpr float kTimeToSleep = 0.5f;
constexpr float kLinearSleepTol = 0.01f;
constexpr float kAngularSleepTol = 2.0f / 180.0f * kPi;
constexpr int kMaxSubSteps = 8;
constexpr int kMaxPolyVerts = 8;
constexpr int kStaticVerts = 4;  // every static fixture of the scene is a quad (build_scene checks)
constexpr int kVelIters = 180;
constexpr int kPosIters = 60;
constexpr float kFltMax = 3.402823466e+38f;
constexpr float kFltEps = 1.192092896e-07f;

// bodies: 3 dynamic (player1, player2, puck) + 8 static; fixtures; canonical contact pair table
enum { B_P1 = 0, B_P2, B_PK, B_WT, B_WB, B_PLT, B_PLB, B_PRT, B_PRB, B_G1, B_G2, NB };
enum { F_WT = 0, F_WB, F_PLT, F_PLB, F_PRT, F_PRB, F_G1S, F_G1, F_G2S, F_G2, F_P1, F_P2, F_PK, NF };
constexpr int NP = 27;       // contact pairs that pass the category/mask filter
constexpr int NSOLID = 25;   // non-sensor pairs (manifold slots)
constexpr int kMaxIsland = 12;  // max contacts in one solver call (geometric bound is 9)

struct Fixture {
  int circle, count, body, sensor;
  float vx[kMaxPolyVerts], vy[kMaxPolyVerts], nx[kMaxPolyVerts], ny[kMaxPolyVerts];
  float radius, friction, restitution, pad;
};

struct Scene {
  Fixture fx[NF];
  float mass[3], invMass[3], I[3], invI[3], lcx[3], lcy[3];  // dynamic bodies
  float spx[NB], spy[NB];                                      // static body origins (index by body id)
  int pairA[NP], pairB[NP];                                    // fixture ids
  int pbodyA[NP], pbodyB[NP];                                  // body ids
  int sensor[NP];
  float friction[NP], restitution[NP];
  int manslot[NP];                                             // manifold slot or -1 (sensor)
  int edges[3][10];                                            // contact edges of each dynamic body
  // broad-phase rejection data (performance only; results unchanged, see hk_arena.h pair_far_*)
  float fx_aabb[NF][4];   // world AABB of every static fixture {minx, miny, maxx, maxy}
  float rcore[3];         // max distance from a dynamic body's COM to its core (radius-free) shape
};

// rounding margin of the polygon-pair rejection (2 x total radius, hk_arena.h pair_far_collide): contacts use
// at most ~1.4 x total radius (tests/test_broadphase_bound.py), float rounding ~1e-5 m
constexpr float kFarMargin = 0.005f;
// margin of the exact distance rejections (hk_arena.h pair_far_toi, circle pairs of pair_far_collide): covers
// the float rounding of sweep interpolation, transforms and GJK distances (~1e-5 m here), far below it
constexpr float kToiMargin = 0.005f;

// ---------------------------------------------------------------------------------------------
// float32 algebra (b2Math.h)
// ---------------------------------------------------------------------------------------------
struct v2 { float x, y; };
struct rot { float s, c; };
struct xform { v2 p; rot q; };

HK_DEV v2 V(float x, float y) { v2 r; r.x = x; r.y = y; return r; }
HK_DEV v2 vadd(v2 a, v2 b) { return V(a.x + b.x, a.y + b.y); }
HK_DEV v2 vsub(v2 a, v2 b) { return V(a.x - b.x, a.y - b.y); }
HK_DEV v2 vneg(v2 a) { return V(-a.x, -a.y); }
HK_DEV v2 vs(float s, v2 a) { return V(s * a.x, s * a.y); }
HK_DEV float dot(v2 a, v2 b) { return a.x * b.x + a.y * b.y; }
HK_DEV float crs(v2 a, v2 b) { return a.x * b.y - a.y * b.x; }
HK_DEV v2 crs_vs(v2 a, float s) { return V(s * a.y, -s * a.x); }
HK_DEV v2 crs_sv(float s, v2 a) { return V(-s * a.y, s * a.x); }
HK_DEV float vlen(v2 a) { return sqrtf(a.x * a.x + a.y * a.y); }
HK_DEV float vlen2(v2 a) { return a.x * a.x + a.y * a.y; }
HK_DEV float vdist(v2 a, v2 b) { return vlen(vsub(a, b)); }
HK_DEV float vdist2(v2 a, v2 b) { v2 c = vsub(a, b); return dot(c, c); }
HK_DEV float vnormalize(v2 &a) {
  float l = vlen(a);
  if (l < kFltEps) return 0.0f;
  float inv = 1.0f / l;
  a.x *= inv;
  a.y *= inv;
  return l;
}
// Packed 2-vectors (v_pk_mul_f32 / v_pk_add_f32): per component the same IEEE fp32 operation as the
// scalar form, so results are bit-identical; one wave issues a packed op at ~1.2x the cost of a scalar
// one (scripts/micro/pk_issue.hip), i.e. ~1.7x the fp32 throughput.  Used in the hot contact-solver loops.
typedef float f2 __attribute__((vector_size(8)));  // GCC/clang vector extension (the host harness is g++)
HK_DEV f2 F2(v2 a) { return f2{a.x, a.y}; }
HK_DEV v2 V2(f2 a) { return V(a[0], a[1]); }
HK_DEV f2 bc(float s) { return f2{s, s}; }
// crs_sv(s, r) == bc(s) * perp(r) bit for bit: (-s) * y == s * (-y) (negation commutes with rounding)
HK_DEV f2 perp(f2 r) { return f2{-r[1], r[0]}; }
HK_DEV float pdot(f2 a, f2 b) { const f2 p = a * b; return p[0] + p[1]; }                // dot()
HK_DEV float pcrs(f2 a, f2 b) { const f2 p = a * f2{b[1], b[0]}; return p[0] - p[1]; }  // crs()
// mul_rv(q, v) == (c x + s (-y), c y + s x): a + (-b) == a - b and + commutes, bit for bit
HK_DEV f2 prv(rot q, f2 v) { return bc(q.c) * v + bc(q.s) * perp(v); }

HK_DEV float fmin2(float a, float b) { return a < b ? a : b; }
HK_DEV float fmax2(float a, float b) { return a > b ? a : b; }
HK_DEV float fclamp(float a, float lo, float hi) { return fmax2(lo, fmin2(a, hi)); }
HK_DEV float fabs2(float a) { return a > 0.0f ? a : -a; }

// Host harness only (hostcheck, HK_HOST_DIAG): event counts behind the algorithmic FLOP count of an env-step
// (scripts/flop_count.py multiplies them by the FLOPs each event's source performs).  No-op in the product build.
enum {
  EV_VEL1 = 0, EV_VEL2, EV_POS_PT, EV_INIT, EV_INIT_PT, EV_INIT_BLOCK, EV_WARM_PT, EV_POLY_CIRCLE, EV_POLYGONS,
  EV_GJK, EV_GJK_IT, EV_ROT, EV_TOI, EV_SEP_MIN, EV_SEP_EVAL, EV_STEP, EV_N
};
#ifdef HK_HOST_DIAG
extern unsigned long long g_hk_flop_ev[EV_N];
#define HK_EV(k, n) (g_hk_flop_ev[k] += (unsigned long long)(n))
#else
#define HK_EV(k, n) ((void)0)
#endif

// deterministic sin/cos for b2Rot::Set (bit-identical to the oracle's hk_sincosf)
HK_DEV rot rot_set(float x) {
  HK_EV(EV_ROT, 1);
  float fj = rintf(x * 0.636619772367581343f);
  int j = (int)fj;
  float r = ((x - fj * 1.5703125f) - fj * 4.837512969970703125e-4f) - fj * 7.549789954891882e-8f;
  float z = r * r;
  float sn = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * r + r;
  float cs = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z -
             0.5f * z + 1.0f;
  // quadrant j & 3: (s, c) = (sn, cs), (cs, -sn), (-sn, -cs), (-cs, sn) -- by two selects and sign flips (exact
  // negations) instead of a switch, which compiled to a branch tree with exec-mask juggling (r06, -DHK_ASM_MARKS)
  const uint32_t k = (uint32_t)j & 3u;
  const bool odd = (k & 1u) != 0u;
  const float a = odd ? cs : sn, b = odd ? sn : cs;
  rot q;
  q.s = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, a) ^ ((k & 2u) << 30));
  q.c = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, b) ^ (((k + 1u) & 2u) << 30));
  return q;
}
HK_DEV v2 mul_rv(rot q, v2 v) { return V(q.c * v.x - q.s * v.y, q.s * v.x + q.c * v.y); }
HK_DEV v2 mulT_rv(rot q, v2 v) { return V(q.c * v.x + q.s * v.y, -q.s * v.x + q.c * v.y); }
HK_DEV rot mulT_rr(rot q, rot r) { rot o; o.s = q.c * r.s - q.s * r.c; o.c = q.c * r.c + q.s * r.s; return o; }
HK_DEV v2 mul_xv(xform T, v2 v) { return V((T.q.c * v.x - T.q.s * v.y) + T.p.x, (T.q.s * v.x + T.q.c * v.y) + T.p.y); }
HK_DEV v2 mulT_xv(xform T, v2 v) {
  float px = v.x - T.p.x, py = v.y - T.p.y;
  return V(T.q.c * px + T.q.s * py, -T.q.s * px + T.q.c * py);
}
HK_DEV xform mulT_xx(xform A, xform B) {
  xform C;
  C.q = mulT_rr(A.q, B.q);
  C.p = mulT_rv(A.q, vsub(B.p, A.p));
  return C;
}

// deterministic double sin/cos (fdlibm kernels) for math.cos / math.sin / np.sin in the reference
HK_DEV uint32_t d_hi(double d) { return (uint32_t)__double2hiint(d); }
HK_DEV double ksin(double x, double y) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
HK_DEV double kcos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  uint32_t ix = d_hi(x) & 0x7fffffffu;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - (z * r - x * y));
  double qx = (ix > 0x3fe90000u) ? 0.28125 : __hiloint2double((int)(ix - 0x00200000u), 0);
  double hz = 0.5 * z - qx, a = 1.0 - qx;
  return a - (hz - (z * r - x * y));
}
HK_DEV int rem_pio2(double x, double &y0, double &y1) {
  const double invpio2 = 6.36619772367581382433e-01, pio2_1 = 1.57079632673412561417e+00,
               pio2_1t = 6.07710050650619224932e-11, pio2_2 = 6.07710050630396597660e-11,
               pio2_2t = 2.02226624879595063154e-21, pio2_3 = 2.02226624871116645580e-21,
               pio2_3t = 8.47842766036889956997e-32;
  double fn = rint(x * invpio2);
  int n = (int)fn;
  double r = x - fn * pio2_1, w = fn * pio2_1t;
  double y = r - w;
  int j = (int)((d_hi(x) >> 20) & 0x7ff);
  int i = j - (int)((d_hi(y) >> 20) & 0x7ff);
  if (i > 16) {
    double t = r;
    w = fn * pio2_2;
    r = t - w;
    w = fn * pio2_2t - ((t - r) - w);
    y = r - w;
    i = j - (int)((d_hi(y) >> 20) & 0x7ff);
    if (i > 49) {
      t = r;
      w = fn * pio2_3;
      r = t - w;
      w = fn * pio2_3t - ((t - r) - w);
      y = r - w;
    }
  }
  y0 = y;
  y1 = (r - y) - w;
  return n;
}
HK_DEV double hk_sin(double x) {
  double a, b;
  if ((d_hi(x) & 0x7fffffffu) <= 0x3fe921fbu) return ksin(x, 0.0);
  int n = rem_pio2(x, a, b);
  switch (n & 3) {
    case 0: return ksin(a, b);
    case 1: return kcos(a, b);
    case 2: return -ksin(a, b);
    default: return -kcos(a, b);
  }
}
HK_DEV double hk_cos(double x) {
  double a, b;
  if ((d_hi(x) & 0x7fffffffu) <= 0x3fe921fbu) return kcos(x, 0.0);
  int n = rem_pio2(x, a, b);
  switch (n & 3) {
    case 0: return kcos(a, b);
    case 1: return -ksin(a, b);
    case 2: return -kcos(a, b);
    default: return ksin(a, b);
  }
}

// true if the predicate holds on any active lane of the wave (a wave-uniform decision).  The host harness
// runs one lane at a time, where it is the lane's own predicate.
#if defined(__HIP_DEVICE_COMPILE__)
HK_DEV bool wave_any(bool p) { return __ballot(p) != 0ull; }
#else
HK_DEV bool wave_any(bool p) { return p; }
#endif

// A per-lane all-ones / all-zeros mask the compiler cannot see through.  `x & mask` then stays one v_and per word:
// written as `if (!c) x = 0` (or a select), LLVM sinks the computation of x into a branch on c and the structurizer
// wraps every use in exec-mask save / xor / restore plus moves (~10 issue slots per velocity iteration, the
// static-body-A reset of the one- and two-contact loops; r05, -DHK_ASM_MARKS dump).
HK_DEV uint32_t lane_mask(bool c) {
  uint32_t m = c ? 0xffffffffu : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(m));
#else
  asm volatile("" : "+r"(m));
#endif
  return m;
}
HK_DEV float mask_f(float x, uint32_t m) { return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & m); }

// Analysis build only (-DHK_ASM_MARKS): labels in the device assembly around hot regions.
#ifdef HK_ASM_MARKS
#define HK_MARK(x) asm volatile(";HKMARK " #x)
#else
#define HK_MARK(x) ((void)0)
#endif

// Diagnostic build only (make TIMERS=1): per-phase shader-clock accounting; compiled out otherwise.
#ifdef HK_PHASE_TIMERS
struct PhaseT {
  unsigned long long last, acc[16], fam[3];  // acc: phases 0-12 + the phase-0 split 13-15; fam: velocity-loop cycles in the general / two / one families
};
#define HK_FAM_T0() const unsigned long long _ft0 = __builtin_amdgcn_s_memtime()
#define HK_FAM_ADD(T, k) ((T).fam[k] += __builtin_amdgcn_s_memtime() - _ft0)
#define HK_TIC(T, k)                                              \
  do {                                                            \
    unsigned long long _t = __builtin_amdgcn_s_memtime();         \
    (T).acc[k] += _t - (T).last;                                  \
    (T).last = _t;                                                \
  } while (0)
#ifdef HK_T0_SPLIT  // analysis only: phase 0 split into scene copy / arena load / policy (own slots 13, 14, 15)
#define HK_TIC_SPLIT(T, k) HK_TIC(T, k)
#else
#define HK_TIC_SPLIT(T, k) ((void)0)
#endif
#else
struct PhaseT {};
#define HK_TIC_SPLIT(T, k) ((void)0)
#define HK_TIC(T, k) ((void)0)
#define HK_FAM_T0() ((void)0)
#define HK_FAM_ADD(T, k) ((void)0)
#endif

}  // namespace hk
