// Microbenchmark (analysis only): cycles per velocity iteration of the one- and two-contact loops of the
// step kernel's contact solver (hk_solver.h vone_chunk / vtwo_chunk), one wave, 180 iterations, no exit.
#include "../../hockey-env_amd/csrc/hk_core.h"
constexpr hk::Scene g_scene =
#include "../../hockey-env_amd/csrc/hk_scene_data.inc"
    ;
__shared__ hk::Scene g_scene_lds;
#include "../../hockey-env_amd/csrc/hk_step.h"
#include <cstdio>

using namespace hk;

HK_DEV void fill(FSlot &s, float x, int bA, int bB) {
  s.bits = 3 | (bA << 7) | (bB << 11) | (1 << 15) | (1 << 17) | (1 << 19);
  s.mA = bA < 3 ? 0.25f : 0.0f; s.mB = 0.5f; s.iA = bA < 3 ? 0.1f : 0.0f; s.iB = 0.3f; s.fr = 0.1f;
  s.nx = 0.6f; s.ny = 0.8f;
  for (int j = 0; j < 2; ++j) {
    s.rAx[j] = 0.3f + x; s.rAy[j] = -0.2f; s.rBx[j] = -0.1f; s.rBy[j] = 0.15f + x;
    s.ni[j] = 0.01f; s.ti[j] = 0.001f; s.nm[j] = 1.3f; s.tm[j] = 1.1f; s.bias[j] = 0.02f;
  }
  s.Kxx = s.Kxy = s.Kyy = s.Nxx = s.Nxy = s.Nyy = 0.0f;
  s.sn[0] = s.sn[1] = s.sn[2] = s.sn[3] = 0u;
}

template <int KIND>
__global__ void __launch_bounds__(64) kb(float *out, long long *cyc) {
  const float x = threadIdx.x * 1e-3f;
  FSlot s0, s1;
  fill(s0, x, 0, 2);
  fill(s1, x, 3, 0);
  f2 vA = f2{0.1f + x, 0.2f}, vB = f2{-0.3f, 0.4f + x};
  float wA = 0.05f, wB = -0.07f;
  uint32_t sn[10];
  for (int k = 0; k < 10; ++k) sn[k] = 0u;
  int it = 0;
  bool active = true;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (KIND == 0) vone_chunk<false, 1>(s0, true, vA, wA, vB, wB, sn, it, kVelIters, 1 << 20, active);
  if (KIND == 1) vone_chunk<true, 1>(s0, false, vA, wA, vB, wB, sn, it, kVelIters, 1 << 20, active);
  if (KIND == 2) vone_chunk<false, 0>(s0, true, vA, wA, vB, wB, sn, it, kVelIters, 1 << 20, active);
  if (KIND == 3) {
    TwoState t;
    t.vA0 = vA; t.vB0 = vB; t.vA1 = f2{0.0f, 0.0f}; t.vB1 = vA;
    t.wA0 = wA; t.wB0 = wB; t.wA1 = 0.0f; t.wB1 = wA;
    for (int k = 0; k < 20; ++k) t.sn[k] = 0u;
    bool on0 = true, on1 = true;
    vtwo_chunk<1, 1, false>(s0, s1, t, true, false, true, false, false, false, false, true, it, kVelIters, 1 << 20,
                            active, on0, on1);
    vA = t.vA0; vB = t.vB0; wA = t.wA0; wB = t.wB1;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = vA[0] + vA[1] + vB[0] + vB[1] + wA + wB + s0.ni[0] + s0.ti[0] + s1.ni[0] + (float)it;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float *o;
  long long *c, h;
  (void)hipMalloc(&o, 64 * 4);
  (void)hipMalloc(&c, 8);
  const char *names[4] = {"vone<dynamic A, 1 point>", "vone<static A, 1 point>", "vone<dynamic A, any points>",
                          "vtwo<1,1> (player-puck + wall-player)"};
  for (int rep = 0; rep < 2; ++rep)
    for (int kind = 0; kind < 4; ++kind) {
      if (kind == 0) hipLaunchKernelGGL(kb<0>, 1, 64, 0, 0, o, c);
      if (kind == 1) hipLaunchKernelGGL(kb<1>, 1, 64, 0, 0, o, c);
      if (kind == 2) hipLaunchKernelGGL(kb<2>, 1, 64, 0, 0, o, c);
      if (kind == 3) hipLaunchKernelGGL(kb<3>, 1, 64, 0, 0, o, c);
      (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-40s %8.1f cycles per iteration\n", names[kind], (double)h / kVelIters);
    }
  return 0;
}
