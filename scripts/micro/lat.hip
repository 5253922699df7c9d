// Microbenchmark: issue cost of packed vs scalar fp32 VALU for ONE wave per SIMD (gfx950).
// Each variant runs 1024 iterations of 16 instructions in 8 independent chains; prints cycles/instruction.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND>
__global__ void __launch_bounds__(64) k(float *out, long long *cyc, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  float b0 = a0 * 0.5f, b1 = a1 * 0.5f, b2 = a2 * 0.5f, b3 = a3 * 0.5f, b4 = a4 * .5f, b5 = a5 * .5f, b6 = a6 * .5f, b7 = a7 * .5f;
  const long long t0 = clock64();
  for (int i = 0; i < 1024; ++i) {
    if (KIND == 0) {  // scalar v_mul_f32, 16 independent-ish ops
      asm volatile(
          "v_mul_f32 %0, %0, %16\n v_mul_f32 %1, %1, %16\n v_mul_f32 %2, %2, %16\n v_mul_f32 %3, %3, %16\n"
          "v_mul_f32 %4, %4, %16\n v_mul_f32 %5, %5, %16\n v_mul_f32 %6, %6, %16\n v_mul_f32 %7, %7, %16\n"
          "v_mul_f32 %8, %8, %16\n v_mul_f32 %9, %9, %16\n v_mul_f32 %10, %10, %16\n v_mul_f32 %11, %11, %16\n"
          "v_mul_f32 %12, %12, %16\n v_mul_f32 %13, %13, %16\n v_mul_f32 %14, %14, %16\n v_mul_f32 %15, %15, %16\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+v"(b0), "+v"(b1),
            "+v"(b2), "+v"(b3), "+v"(b4), "+v"(b5), "+v"(b6), "+v"(b7)
          : "v"(s));
    } else if (KIND == 1) {  // packed v_pk_mul_f32 on register pairs: 8 instructions = 16 fp32 ops
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, q0 = {b0, b1}, q1 = {b2, b3}, q2 = {b4, b5},
         q3 = {b6, b7};
      f2 ss = {s, s};
      asm volatile(
          "v_pk_mul_f32 %0, %0, %8\n v_pk_mul_f32 %1, %1, %8\n v_pk_mul_f32 %2, %2, %8\n v_pk_mul_f32 %3, %3, %8\n"
          "v_pk_mul_f32 %4, %4, %8\n v_pk_mul_f32 %5, %5, %8\n v_pk_mul_f32 %6, %6, %8\n v_pk_mul_f32 %7, %7, %8\n"
          : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(q0), "+v"(q1), "+v"(q2), "+v"(q3)
          : "v"(ss));
      a0 = p0.x; a1 = p0.y; a2 = p1.x; a3 = p1.y; a4 = p2.x; a5 = p2.y; a6 = p3.x; a7 = p3.y;
      b0 = q0.x; b1 = q0.y; b2 = q1.x; b3 = q1.y; b4 = q2.x; b5 = q2.y; b6 = q3.x; b7 = q3.y;
    } else if (KIND == 3) {  // packed dependent chain: 8 v_pk_mul on one pair, s_nop 0 between (hazard)
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 p0 = {a0, a1};
      f2 ss = {s, s};
      asm volatile(
          "v_pk_mul_f32 %0, %0, %1\n s_nop 0\n v_pk_mul_f32 %0, %0, %1\n s_nop 0\n v_pk_mul_f32 %0, %0, %1\n s_nop 0\n"
          "v_pk_mul_f32 %0, %0, %1\n s_nop 0\n v_pk_mul_f32 %0, %0, %1\n s_nop 0\n v_pk_mul_f32 %0, %0, %1\n s_nop 0\n"
          "v_pk_mul_f32 %0, %0, %1\n s_nop 0\n v_pk_mul_f32 %0, %0, %1\n s_nop 0\n"
          : "+v"(p0)
          : "v"(ss));
      a0 = p0.x; a1 = p0.y;
    } else if (KIND == 4) {  // dependent cmp + cndmask chain (clamp-like), 8 pairs
      asm volatile(
          "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n"
          "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n"
          "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n"
          "v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n v_cmp_lt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %1, %0, vcc\n"
          : "+v"(a0)
          : "v"(s) : "vcc");
    } else if (KIND == 5) {  // dependent chain of v_mul_f32 and v_add_f32 alternating with an e64 sub (16)
      asm volatile(
          "v_mul_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_sub_f32 %0, %0, %1\n v_mul_f32 %0, %1, %0\n"
          "v_mul_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_sub_f32 %0, %0, %1\n v_mul_f32 %0, %1, %0\n"
          "v_mul_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_sub_f32 %0, %0, %1\n v_mul_f32 %0, %1, %0\n"
          "v_mul_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_sub_f32 %0, %0, %1\n v_mul_f32 %0, %1, %0\n"
          : "+v"(a0)
          : "v"(s));
    } else {  // scalar dependent chain: 16 ops on one register
      asm volatile(
          "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
          "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
          "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
          "v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n v_mul_f32 %0, %0, %1\n"
          : "+v"(a0)
          : "v"(s));
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  float *o;
  long long *c, h;
  hipMalloc(&o, 64 * 4);
  hipMalloc(&c, 8);
  const char *names[6] = {"v_mul_f32 x16 (8+8 independent)", "v_pk_mul_f32 x8 (16 fp32 ops)", "v_mul_f32 x16 dependent", "v_pk_mul_f32 x8 dependent (+s_nop 0)", "cmp+cndmask x8 dependent", "mul/add/sub x16 dependent"};
  const int ninstr[6] = {16, 8, 16, 8, 16, 16};
  for (int rep = 0; rep < 2; ++rep)
    for (int kind = 0; kind < 6; ++kind) {
      if (kind == 0) hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, o, c, 1.0f);
      if (kind == 1) hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, o, c, 1.0f);
      if (kind == 2) hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, o, c, 1.0f);
      if (kind == 3) hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, o, c, 1.0f);
      if (kind == 4) hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, o, c, 1.0f);
      if (kind == 5) hipLaunchKernelGGL(k<5>, 1, 64, 0, 0, o, c, 1.0f);
      hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
      if (rep) printf("%-36s %7.2f clock64 ticks per instruction, %7.2f per fp32 op\n", names[kind],
                      (double)h / (1024.0 * ninstr[kind]), (double)h / (1024.0 * 16));
    }
  return 0;
}
