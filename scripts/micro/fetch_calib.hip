// FETCH_SIZE / WRITE_SIZE calibration for the step kernel's own access widths (MI355X_MICROARCH.md: "Other access
// widths are uncalibrated: calibrate on a known byte count in your own access pattern").  Each kernel moves a known
// number of bytes with one of the step kernel's patterns, over the step kernel's array sizes (65 536 lanes, one lane
// per arena, 1 024 blocks of 64):
//   soa_dword   41 SoA float fields [f][N] read, 41 written (the f / i state words: global_load_dword per field)
//   soa_dword_r 41 SoA fields read, 1 written (reads alone)
//   soa_double  3 SoA double rows read and written (the BasicOpponent phase rows: global_load_dwordx2)
//   soa_quad    4 x 16-B quads per lane read and written (the guide's calibrated case: 16 B per lane)
//   byte_store  1 byte per lane written (done), 1 float per lane written (reward), nothing read
//   rec_sparse  64-B records [N][16] read (3 quads) and written (4 quads) by 40 % of lanes (the manifold records)
//   obs_dword   [N][18] floats written as 18 dword stores per lane (the step kernel's obs rows: a store
//               instruction covers every 72-B row of the wave at one word, so each 128-B line is written piecewise)
//   obs_lds     the same rows staged through LDS and written as 16-B stores of consecutive wave memory
//   info_dword  [N][4] floats as 4 dword stores per lane;  info_quad  the same as one 16-B store per lane
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip.  Run each counter in its own pass:
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- ./fetch_calib
// scripts/fetch_calib_reduce.py divides each kernel's counter by its known bytes.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int N = 65536, NF = 41, REPS = 20;

__global__ void soa_dword(const float *__restrict__ in, float *__restrict__ out) {
  const int a = blockIdx.x * 64 + threadIdx.x;
  float v[NF];
#pragma unroll
  for (int k = 0; k < NF; ++k) v[k] = in[k * N + a];
#pragma unroll
  for (int k = 0; k < NF; ++k) out[k * N + a] = v[k] * 1.0001f + v[(k + 1) % NF];
}
__global__ void soa_dword_r(const float *__restrict__ in, float *__restrict__ out) {
  const int a = blockIdx.x * 64 + threadIdx.x;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < NF; ++k) s += in[k * N + a];
  out[a] = s;
}
__global__ void soa_double(const double *__restrict__ in, double *__restrict__ out) {
  const int a = blockIdx.x * 64 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 3; ++k) out[k * N + a] = in[k * N + a] * 1.0001;
}
__global__ void soa_quad(const float4 *__restrict__ in, float4 *__restrict__ out) {
  const int a = blockIdx.x * 64 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float4 q = in[k * N + a];
    q.x *= 1.0001f;
    out[k * N + a] = q;
  }
}
__global__ void byte_store(unsigned char *__restrict__ done, float *__restrict__ rew) {
  const int a = blockIdx.x * 64 + threadIdx.x;
  done[a] = (unsigned char)(a & 1);
  rew[a] = (float)a;
}
// lanes a with (a * 2654435761u) % 10 < 4 touch their record (a hashed 40 %, as touching pairs are scattered)
__global__ void rec_sparse(float4 *__restrict__ rec) {
  const int a = blockIdx.x * 64 + threadIdx.x;
  if (((unsigned)a * 2654435761u) % 10u >= 4u) return;
  float4 *r = rec + (size_t)a * 4;
  float4 q0 = r[0], q2 = r[2], q3 = r[3];
  q0.x += 1.0f;
  r[0] = q0;
  r[1] = q2;
  r[2] = q3;
  r[3] = q0;
}

__global__ void obs_dword(float *__restrict__ obs) {
  const int a = blockIdx.x * 64 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 18; ++k) obs[(size_t)a * 18 + k] = (float)(a + k);
}
__global__ void obs_lds(float *__restrict__ obs) {
  __shared__ float st[64 * 18];
  const int t = threadIdx.x, a0 = blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 18; ++k) st[t * 18 + k] = (float)(a0 + t + k);
  __syncthreads();
  const float4 *src = reinterpret_cast<const float4 *>(st);
  float4 *dst = reinterpret_cast<float4 *>(obs + (size_t)a0 * 18);
  for (int j = t; j < 64 * 18 / 4; j += 64) dst[j] = src[j];
}
__global__ void info_dword(float *__restrict__ info) {
  const int a = blockIdx.x * 64 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) info[(size_t)a * 4 + k] = (float)(a + k);
}
__global__ void info_quad(float4 *__restrict__ info) {
  const int a = blockIdx.x * 64 + threadIdx.x;
  info[a] = float4{(float)a, (float)(a + 1), (float)(a + 2), (float)(a + 3)};
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  float *fin, *fout;
  double *din, *dout;
  float4 *qin, *qout, *rec;
  unsigned char *done;
  float *rew, *obs, *info;
  CK(hipMalloc(&fin, sizeof(float) * NF * N));
  CK(hipMalloc(&fout, sizeof(float) * NF * N));
  CK(hipMalloc(&din, sizeof(double) * 3 * N));
  CK(hipMalloc(&dout, sizeof(double) * 3 * N));
  CK(hipMalloc(&qin, sizeof(float4) * 4 * N));
  CK(hipMalloc(&qout, sizeof(float4) * 4 * N));
  CK(hipMalloc(&rec, sizeof(float4) * 4 * N));
  CK(hipMalloc(&done, N));
  CK(hipMalloc(&rew, sizeof(float) * N));
  CK(hipMalloc(&obs, sizeof(float) * 18 * N));
  CK(hipMalloc(&info, sizeof(float) * 4 * N));
  CK(hipMemset(fin, 0, sizeof(float) * NF * N));
  CK(hipMemset(din, 0, sizeof(double) * 3 * N));
  CK(hipMemset(qin, 0, sizeof(float4) * 4 * N));
  CK(hipMemset(rec, 0, sizeof(float4) * 4 * N));
  const dim3 g(N / 64), b(64);
  // each kernel REPS times back to back, as the step kernel runs in the bench
  for (int r = 0; r < REPS; ++r) soa_dword<<<g, b>>>(fin, fout);
  for (int r = 0; r < REPS; ++r) soa_dword_r<<<g, b>>>(fin, fout);
  for (int r = 0; r < REPS; ++r) soa_double<<<g, b>>>(din, dout);
  for (int r = 0; r < REPS; ++r) soa_quad<<<g, b>>>(qin, qout);
  for (int r = 0; r < REPS; ++r) byte_store<<<g, b>>>(done, rew);
  for (int r = 0; r < REPS; ++r) rec_sparse<<<g, b>>>(rec);
  for (int r = 0; r < REPS; ++r) obs_dword<<<g, b>>>(obs);
  for (int r = 0; r < REPS; ++r) obs_lds<<<g, b>>>(obs);
  for (int r = 0; r < REPS; ++r) info_dword<<<g, b>>>(info);
  for (int r = 0; r < REPS; ++r) info_quad<<<g, b>>>(reinterpret_cast<float4 *>(info));
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  int touched = 0;
  for (int a = 0; a < N; ++a) touched += ((unsigned)a * 2654435761u) % 10u < 4u;
  // known bytes per launch (read, write)
  printf("soa_dword %d %d\n", NF * N * 4, NF * N * 4);
  printf("soa_dword_r %d %d\n", NF * N * 4, N * 4);
  printf("soa_double %d %d\n", 3 * N * 8, 3 * N * 8);
  printf("soa_quad %d %d\n", 4 * N * 16, 4 * N * 16);
  printf("byte_store %d %d\n", 0, N * 5);
  printf("rec_sparse %d %d\n", touched * 48, touched * 64);
  printf("obs_dword %d %d\n", 0, N * 72);
  printf("obs_lds %d %d\n", 0, N * 72);
  printf("info_dword %d %d\n", 0, N * 16);
  printf("info_quad %d %d\n", 0, N * 16);
  hipFree(fin); hipFree(fout); hipFree(din); hipFree(dout); hipFree(qin); hipFree(qout); hipFree(rec);
  hipFree(done); hipFree(rew); hipFree(obs); hipFree(info);
  return 0;
}
