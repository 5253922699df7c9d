// How much of critic_step's time is its seven 256x256 layer GEMMs (hk_learner.hip gemm256)?  The same grid and
// workgroup shape as critic_step at batch 16 384 (256 workgroups x 4 waves, 16 samples per wave), the same
// workgroup-collective gemm256 on a packed operand, 7 calls per wave (the critic step's count), timed with
// events.  Build: hipcc --offload-arch=gfx950 -O3 -o learner_gemm_bench learner_gemm_bench.hip
#include "../../hockey-env_amd/csrc/hk_learner.hip"

#include <cstdio>

namespace hkl {
// candidate: three LDS fragment buffers, the next block's A fragments read into registers while this block's
// MFMAs run (one barrier per block as before)
__device__ __forceinline__ void gemm256_tb(const f4 *__restrict__ P, Tile &in, const float *__restrict__ bias,
                                           Tile &out, int lane, f4 *sfrag) {
  const int wave = threadIdx.x >> 6, q = lane >> 4;
  float *sbias = reinterpret_cast<float *>(sfrag + 3 * 1024);
  if (bias) sbias[threadIdx.x] = bias[threadIdx.x];
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) out.v[ob] = z4();
  f4 g[4];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) sfrag[kb * 1024 + (4 * wave + i) * 64 + lane] = P[((4 * wave + i) * 16 + kb) * 64 + lane];
  __syncthreads();
  f4 a[16], an[16];
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a[ob] = sfrag[ob * 64 + lane];
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) {
    if (kb + 2 < 16) {
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] = P[((4 * wave + i) * 16 + kb + 2) * 64 + lane];
    }
    if (kb + 1 < 16) {
      const f4 *nb = sfrag + ((kb + 1) % 3) * 1024;
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) an[ob] = nb[ob * 64 + lane];
    }
    if (bias) {
      const f4 bb = *reinterpret_cast<const f4 *>(sbias + 16 * kb + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) in.v[kb][r] = tanh_fast(in.v[kb][r] + bb[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float b = in.v[kb][r];
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) out.v[ob] = mfma(a[ob][r], b, out.v[ob]);
    }
    if (kb + 2 < 16) {
      f4 *wb = sfrag + ((kb + 2) % 3) * 1024;
#pragma unroll
      for (int i = 0; i < 4; ++i) wb[(4 * wave + i) * 64 + lane] = g[i];
    }
    __syncthreads();
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) a[ob] = an[ob];
  }
}

// candidate: the current two-buffer gemm256, with block kb + 1's bias + tanh computed while block kb's MFMAs run
// (block 0 before the loop), so no MFMA waits on the activation's VALU chain
__device__ __forceinline__ void gemm256_ahead(const f4 *__restrict__ P, Tile &in, const float *__restrict__ bias,
                                              Tile &out, int lane, f4 *sfrag) {
  const int wave = threadIdx.x >> 6, q = lane >> 4;
  float *sbias = reinterpret_cast<float *>(sfrag + 3 * 1024);
  if (bias) sbias[threadIdx.x] = bias[threadIdx.x];
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) out.v[ob] = z4();
  f4 g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = P[((4 * wave + i) * 16) * 64 + lane];
#pragma unroll
  for (int i = 0; i < 4; ++i) sfrag[(4 * wave + i) * 64 + lane] = g[i];
  __syncthreads();
  if (bias) {
    const f4 bb = *reinterpret_cast<const f4 *>(sbias + 4 * q);
#pragma unroll
    for (int r = 0; r < 4; ++r) in.v[0][r] = tanh_fast(in.v[0][r] + bb[r]);
  }
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) {
    const f4 *buf = sfrag + (kb & 1) * 1024;
    if (kb + 1 < 16) {
#pragma unroll
      for (int i = 0; i < 4; ++i) g[i] = P[((4 * wave + i) * 16 + kb + 1) * 64 + lane];
    }
    f4 a[16];
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) a[ob] = buf[ob * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float b = in.v[kb][r];
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) out.v[ob] = mfma(a[ob][r], b, out.v[ob]);
    }
    if (bias && kb + 1 < 16) {
      const f4 bb = *reinterpret_cast<const f4 *>(sbias + 16 * (kb + 1) + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) in.v[kb + 1][r] = tanh_fast(in.v[kb + 1][r] + bb[r]);
    }
    if (kb + 1 < 16) {
      f4 *nb = sfrag + ((kb + 1) & 1) * 1024;
#pragma unroll
      for (int i = 0; i < 4; ++i) nb[(4 * wave + i) * 64 + lane] = g[i];
    }
    __syncthreads();
  }
}

// candidate (r06): no LDS staging and no workgroup barrier -- every wave loads its own A fragments from L2 / L1 (the
// workgroup's 4 waves read the same lines, so 3 of 4 hit L1), half a k-block (8 output blocks) at a time, the next
// half's 8 loads in flight while this half's 32 MFMAs run (8 independent accumulators)
__device__ __forceinline__ void gemm256_direct(const f4 *__restrict__ P0, Tile &in, const float *__restrict__ bias,
                                               Tile &out, int lane) {
  const int q = lane >> 4;
  const f4 *P = P0;
  asm volatile("" : "+s"(P));  // a fresh operand per call, as in the kernels (no loads hoisted out of a caller's loop)
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) out.v[ob] = z4();
  f4 a[2][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[0][i] = P[(i * 16) * 64 + lane];
#pragma unroll
  for (int h = 0; h < 32; ++h) {
    const int kb = h >> 1, ob0 = (h & 1) * 8;
    if (h + 1 < 32) {
      const int kb1 = (h + 1) >> 1, ob1 = ((h + 1) & 1) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) a[(h + 1) & 1][i] = P[((ob1 + i) * 16 + kb1) * 64 + lane];
    }
    if (bias && (h & 1) == 0) {
      const f4 bb = *reinterpret_cast<const f4 *>(bias + 16 * kb + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) in.v[kb][r] = tanh_fast(in.v[kb][r] + bb[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float b = in.v[kb][r];
#pragma unroll
      for (int i = 0; i < 8; ++i) out.v[ob0 + i] = mfma(a[h & 1][i][r], b, out.v[ob0 + i]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the next halves' loads from being hoisted (registers)
  }
}
// the same with whole k-blocks: the next block's 16 fragment loads in flight during this block's 64 MFMAs
__device__ __forceinline__ void gemm256_direct16(const f4 *__restrict__ P0, Tile &in, const float *__restrict__ bias,
                                                 Tile &out, int lane) {
  const int q = lane >> 4;
  const f4 *P = P0;
  asm volatile("" : "+s"(P));
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) out.v[ob] = z4();
  f4 a[2][16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[0][i] = P[(i * 16) * 64 + lane];
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) {
    if (kb + 1 < 16) {
#pragma unroll
      for (int i = 0; i < 16; ++i) a[(kb + 1) & 1][i] = P[(i * 16 + kb + 1) * 64 + lane];
    }
    if (bias) {
      const f4 bb = *reinterpret_cast<const f4 *>(bias + 16 * kb + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) in.v[kb][r] = tanh_fast(in.v[kb][r] + bb[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float b = in.v[kb][r];
#pragma unroll
      for (int i = 0; i < 16; ++i) out.v[i] = mfma(a[kb & 1][i][r], b, out.v[i]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
__global__ void __launch_bounds__(WG, 1) gemm_direct16_kernel(const f4 *P, const float *bias, float *out, int reps) {
  const int lane = threadIdx.x & 63;
  Tile a, b;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a.v[ob] = f4{0.01f * lane, 0.02f, 0.03f, 0.04f * ob};
  for (int r = 0; r < 2 * reps; ++r) {
    gemm256_direct16(P, a, bias, b, lane);
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) a.v[ob] = b.v[ob];
  }
  float s = 0.0f;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s += a.v[ob][0] + a.v[ob][1] + a.v[ob][2] + a.v[ob][3];
  out[blockIdx.x * WG + threadIdx.x] = s;
}
__global__ void __launch_bounds__(WG, 1) gemm_direct_kernel(const f4 *P, const float *bias, float *out, int reps) {
  const int lane = threadIdx.x & 63;
  Tile a, b;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a.v[ob] = f4{0.01f * lane, 0.02f, 0.03f, 0.04f * ob};
  for (int r = 0; r < 2 * reps; ++r) {
    gemm256_direct(P, a, bias, b, lane);
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) a.v[ob] = b.v[ob];
  }
  float s = 0.0f;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s += a.v[ob][0] + a.v[ob][1] + a.v[ob][2] + a.v[ob][3];
  out[blockIdx.x * WG + threadIdx.x] = s;
}

template <int kV>
__global__ void __launch_bounds__(WG, 1) gemm_var3_kernel(const f4 *P, const float *bias, float *out, int reps) {
  __shared__ f4 sfrag[3 * 16 * 64 + 64];
  const int lane = threadIdx.x & 63;
  Tile a, b;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a.v[ob] = f4{0.01f * lane, 0.02f, 0.03f, 0.04f * ob};
  for (int r = 0; r < reps; ++r) {
    if constexpr (kV == 2) {
      gemm256_ahead(P, a, bias, b, lane, sfrag);
      gemm256_ahead(P, b, bias, a, lane, sfrag);
    } else {
      gemm256(P, a, nullptr, b, lane, sfrag);
      gemm256(P, b, nullptr, a, lane, sfrag);
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s += a.v[ob][0] + a.v[ob][1] + a.v[ob][2] + a.v[ob][3];
  out[blockIdx.x * WG + threadIdx.x] = s;
}

template <bool kTB>
__global__ void __launch_bounds__(WG, 1) gemm_var_kernel(const f4 *P, const float *bias, float *out, int reps) {
  __shared__ f4 sfrag[3 * 16 * 64 + 64];
  const int lane = threadIdx.x & 63;
  Tile a, b;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a.v[ob] = f4{0.01f * lane, 0.02f, 0.03f, 0.04f * ob};
  for (int r = 0; r < reps; ++r) {
    if constexpr (kTB) {
      gemm256_tb(P, a, bias, b, lane, sfrag);
      gemm256_tb(P, b, bias, a, lane, sfrag);
    } else {
      gemm256(P, a, bias, b, lane, sfrag);
      gemm256(P, b, bias, a, lane, sfrag);
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s += a.v[ob][0] + a.v[ob][1] + a.v[ob][2] + a.v[ob][3];
  out[blockIdx.x * WG + threadIdx.x] = s;
}

__global__ void __launch_bounds__(WG, 1) gemm7_kernel(const f4 *P, const float *bias, float *out, int reps) {
  __shared__ f4 sfrag[2 * 16 * 64 + 64];
  const int lane = threadIdx.x & 63;
  Tile a, b;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a.v[ob] = f4{0.01f * lane, 0.02f, 0.03f, 0.04f * ob};
  for (int r = 0; r < reps; ++r) {
    gemm256(P, a, bias, b, lane, sfrag);
    gemm256(P, b, bias, a, lane, sfrag);
  }
  float s = 0.0f;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s += a.v[ob][0] + a.v[ob][1] + a.v[ob][2] + a.v[ob][3];
  out[blockIdx.x * WG + threadIdx.x] = s;
}
}  // namespace hkl

int main() {
  using namespace hkl;
  f4 *P;
  float *bias, *out;
  hipMalloc(&P, sizeof(f4) * 16 * 16 * 64);
  hipMalloc(&bias, sizeof(float) * 256);
  hipMalloc(&out, sizeof(float) * 256 * WG);
  hipMemset(P, 0, sizeof(f4) * 16 * 16 * 64);
  hipMemset(bias, 0, sizeof(float) * 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int tb = 0; tb < 6; ++tb)
  for (int reps : {4, 8}) {
    auto kern = tb == 5 ? gemm_direct16_kernel : tb == 4 ? gemm_direct_kernel : tb == 1 ? gemm_var_kernel<true> : tb == 0 ? gemm_var_kernel<false>
                : tb == 2 ? gemm_var3_kernel<2> : gemm_var3_kernel<3>;
    hipLaunchKernelGGL(kern, dim3(256), dim3(WG), 0, 0, P, bias, out, reps);
    hipEventRecord(e0);
    for (int k = 0; k < 20; ++k) hipLaunchKernelGGL(kern, dim3(256), dim3(WG), 0, 0, P, bias, out, reps);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / 20, calls = 2.0 * reps;
    const double flop = calls * 2.0 * 256 * 256 * 16384;  // per launch
    printf("%s gemm256 x %d per wave: %.1f us per launch, %.2f us per gemm256 call, %.1f TFLOP/s\n",
           tb == 5 ? "direct, whole blocks (r06)" : tb == 4 ? "direct, half blocks (r06)" : tb == 1 ? "triple-buffered" : tb == 0 ? "current" : tb == 2 ? "tanh-ahead"
                                                                                         : "no-activation", (int)calls, us,
           us / calls, flop / (us * 1e-6) / 1e12);
    (void)0;
  }
  return 0;
}
