// hk_learner.hip -- the batched TD3 learner (BASELINE C5) as fused fp32 MFMA kernels for gfx950.
//
// One learner update of rl/td3/learner.py:55-218 at a large batch B (C5 draws 16 384 samples per update):
//   critic_step   target policy smoothing + clipped double-Q target (compute_target, :75-112), both critics'
//                 forward, the weighted smooth-L1 loss (rl/utils/torch_utils.py:12-24) and its backward through
//                 both critics down to the first layer -- one launch, B / 64 workgroups of 4 waves, 16 samples
//                 per wave;
//   actor_step    actor forward, Q1 of the updated critic on (s, actor(s)), -mean Q1 backward through Q1 to the
//                 action and through the actor (update_actor, :138-175) -- one launch;
//   wgrad         the weight gradients dW = dZ^T X (the reduction over the batch) as split-K MFMA tiles;
//   adam          per-parameter reduction of the gradient slabs in a fixed order + torch.optim.Adam's update
//                 (lr, betas (0.9, 0.999), eps, L2 weight decay; rl/td3/agent.py:174-182), on actor updates with
//                 soft_update (:196-218) folded in;
//   pack          re-lays the changed weights out for the MFMA operands (polyak: soft_update as its own launch).
//
// Every product is v_mfma_f32_16x16x4_f32: exact f32 fma chains (no reduced-precision path on gfx950), so the
// arithmetic is the reference's fp32 up to summation order.  Layout of a wave's activations ("Tile"): lane l holds
// sample j = l & 15 and, for each 16-neuron block ob and r = 0..3, neuron 16 ob + 4 (l >> 4) + r in v[ob][r] --
// exactly the C/D layout of the MFMA (col = lane & 15, row = 4 (lane >> 4) + reg), and, read as a B operand with
// k-step (kb, r), exactly the fragment the next layer needs (lane (j, kk = l >> 4) holds input neuron
// 16 kb + 4 kk + r).  Consecutive layers therefore chain in registers with no data movement; the weights are
// pre-packed into the matching A-operand order (pack_kernel) after every optimiser step.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hockey_learner.h"

namespace hkl {

constexpr int H = 256;   // hidden width (rl/td3/networks.py: h = 256)
constexpr int XP = 32;   // padded row of the stored first-layer inputs X0 [B][XP]
constexpr int S1 = 6;    // first-layer k-steps: inputs padded to 24
constexpr int WG = 256;  // threads of the fused kernels: 4 waves x 16 samples = 64 samples per workgroup
constexpr int CHUNK = 256;  // batch granularity; the weight-gradient kernel's split-K chunks are 256 or 512 samples

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 z4() { return f4{0.0f, 0.0f, 0.0f, 0.0f}; }

struct Tile {
  f4 v[16];
};

// tanh without branches: tanh|x| = (1 - t) / (1 + t), t = 2^(-2 log2(e) |x|) (v_exp_f32, v_rcp_f32), sign restored.
// OCML's tanhf branches between a polynomial and an exp path per lane (exec-mask juggling around ~30 VALU per
// call, a third of the critic kernel's instructions); this form is 7 VALU.  Its absolute error is a few 1e-8 near
// 0 (the 1 - t cancellation) and below 2e-7 everywhere (checked against torch.tanh in
// tests/test_gpu_learner.py), far inside the learner's stated fp32 tolerances.
__device__ __forceinline__ float tanh_fast(float x) {
  const float t = __builtin_amdgcn_exp2f(-2.8853900817779268f * fabsf(x));
  const float y = (1.0f - t) * __builtin_amdgcn_rcpf(1.0f + t);
  return copysignf(y, x);
}

// ------------------------------------------------------------------------------------------------ packed layouts
// f1 [16 ob][64 lane][8]     : W1[16 ob + (l & 15)][4 s + (l >> 4)] for k-step s < 6 (0 past the input width)
// fp [16 ob][16 kb][64 lane] : f4 over r of W2[16 ob + (l & 15)][16 kb + 4 (l >> 4) + r]        (forward)
// bp [16 ib][16 ob][64 lane] : f4 over r of W2[16 ob + 4 (l >> 4) + r][16 ib + (l & 15)]        (W2^T: backward)
// fo [16 kb][64 lane]        : f4 over r of W3[l & 15][16 kb + 4 (l >> 4) + r] (0 for rows >= n_out)
// wa [256]                   : f4 of W1[n][18..21] (a critic's action columns: dQ/da)
constexpr int kF1 = 16 * 64 * 8, kFp = 16 * 16 * 64 * 4, kBp = kFp, kFo = 16 * 64 * 4, kWa = 256 * 4;
constexpr int kPackFloats = kF1 + kFp + kBp + kFo + kWa;
static_assert(kPackFloats == HKL_PACK_FLOATS, "pack size (include/hockey_learner.h)");

struct Net {  // device view of one MLP (n_in -> 256 -> 256 -> n_out)
  const float *w1, *b1, *w2, *b2, *w3, *b3;
  const float *pk;
  int n_in, n_out;
  __device__ const float *f1() const { return pk; }
  __device__ const f4 *fp() const { return reinterpret_cast<const f4 *>(pk + kF1); }
  __device__ const f4 *bp() const { return reinterpret_cast<const f4 *>(pk + kF1 + kFp); }
  __device__ const f4 *fo() const { return reinterpret_cast<const f4 *>(pk + kF1 + kFp + kBp); }
  __device__ const f4 *wa() const { return reinterpret_cast<const f4 *>(pk + kF1 + kFp + kBp + kFo); }
};
__host__ __device__ inline Net net_of(const hkl_net &n) { return Net{n.w1, n.b1, n.w2, n.b2, n.w3, n.b3, n.pack, n.n_in, n.n_out}; }

// ------------------------------------------------------------------------------------------------ layer routines
// out = W1 x (no bias): x[s] = this lane's input for k-step s (feature 4 s + (lane >> 4)).  Workgroup-collective:
// the 32 KB first-layer pack is staged in LDS (both fragment buffers) once for the 4 waves.
__device__ __forceinline__ void gemm_in(const float *__restrict__ f1, const float (&x)[S1], Tile &out, int lane,
                                        f4 *sfrag) {
  const f4 *src = reinterpret_cast<const f4 *>(f1);
#pragma unroll
  for (int i = 0; i < 8; ++i) sfrag[threadIdx.x + i * WG] = src[threadIdx.x + i * WG];
  __syncthreads();
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const f4 lo = sfrag[(ob * 64 + lane) * 2];
    const f4 hi = sfrag[(ob * 64 + lane) * 2 + 1];
    f4 acc = z4();
    acc = mfma(lo[0], x[0], acc);
    acc = mfma(lo[1], x[1], acc);
    acc = mfma(lo[2], x[2], acc);
    acc = mfma(lo[3], x[3], acc);
    acc = mfma(hi[0], x[4], acc);
    acc = mfma(hi[1], x[5], acc);
    out.v[ob] = acc;
  }
  __syncthreads();  // the staging buffers are reused by the next collective call
}

// out = P in, P a packed 256 x 256 operand (fp: W2 in; bp: W2^T in), a workgroup-collective call (all 4 waves).
// The A fragments are the same for the workgroup's 4 waves: each 16-neuron k-block (16 KB) is loaded once per
// workgroup into one of two LDS buffers (each thread 4 x 16 B) while the waves multiply the previous one, so the
// L2 serves a quarter of the bytes.  bias != nullptr: `in` holds pre-activations and block kb is activated in
// place (tanh(in + bias)) just before its first use, so the activation's VALU work overlaps the MFMAs of the
// block before; on return `in` holds the activations.
__device__ __forceinline__ void gemm256(const f4 *__restrict__ P, Tile &in, const float *__restrict__ bias, Tile &out,
                                        int lane, f4 *sfrag) {
  const int wave = threadIdx.x >> 6, q = lane >> 4;
  float *sbias = reinterpret_cast<float *>(sfrag + 2 * 1024);  // the bias, staged once (no global wait per k-block)
  if (bias) sbias[threadIdx.x] = bias[threadIdx.x];
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) out.v[ob] = z4();
  f4 g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) g[i] = P[((4 * wave + i) * 16) * 64 + lane];
#pragma unroll
  for (int i = 0; i < 4; ++i) sfrag[(4 * wave + i) * 64 + lane] = g[i];
  __syncthreads();
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
    if (kb + 1 < 16) {
      f4 *nb = sfrag + ((kb + 1) & 1) * 1024;
#pragma unroll
      for (int i = 0; i < 4; ++i) nb[(4 * wave + i) * 64 + lane] = g[i];
    }
    __syncthreads();
  }
}

// t = tanh(t + b) (Linear bias, then the tanh activation)
__device__ __forceinline__ void bias_tanh(Tile &t, const float *__restrict__ b, int q) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const f4 bb = *reinterpret_cast<const f4 *>(b + 16 * ob + 4 * q);
#pragma unroll
    for (int r = 0; r < 4; ++r) t.v[ob][r] = tanh_fast(t.v[ob][r] + bb[r]);
  }
}

// the n_out (<= 4) outputs W3 h + b3 of this lane's sample, broadcast to every lane of the sample; a
// workgroup-collective call (the W3 fragments and the bias are staged in LDS once for the 4 waves).  bias !=
// nullptr: h holds pre-activations, activated in place (tanh(h + bias)) block by block as in gemm256.
__device__ __forceinline__ f4 gemm_out(const f4 *__restrict__ fo, Tile &h, const float *__restrict__ bias,
                                       const float *__restrict__ b3, int n_out, int lane, f4 *sfrag) {
  const int q = lane >> 4;
  float *sbias = reinterpret_cast<float *>(sfrag + 2 * 1024);
#pragma unroll
  for (int i = 0; i < 4; ++i) sfrag[threadIdx.x + i * WG] = fo[threadIdx.x + i * WG];
  if (bias) sbias[threadIdx.x] = bias[threadIdx.x];
  __syncthreads();
  f4 acc0 = z4(), acc1 = z4();
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) {
    const f4 a = sfrag[kb * 64 + lane];
    if (bias) {
      const f4 bb = *reinterpret_cast<const f4 *>(sbias + 16 * kb + 4 * q);
#pragma unroll
      for (int r = 0; r < 4; ++r) h.v[kb][r] = tanh_fast(h.v[kb][r] + bb[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (kb & 1) acc1 = mfma(a[r], h.v[kb][r], acc1);
      else acc0 = mfma(a[r], h.v[kb][r], acc0);
    }
  }
  __syncthreads();  // the staging buffers are reused by the next collective call
  const f4 acc = acc0 + acc1;  // lanes 0..15 hold outputs 0..3 of sample lane & 15
  f4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = __shfl(acc[r], lane & 15) + (r < n_out ? b3[r] : 0.0f);
  return o;
}

// A one-output head (a critic's Q): W3[0] . tanh(h + bias) + b3[0] for this lane's sample, returned to every lane of
// the sample, h activated in place as gemm_out leaves it.  VALU dot products (each lane's 64 neurons, four partial
// sums) and two cross-row shuffles instead of a 16 x 16 MFMA tile of which one row is used; no LDS staging and no
// workgroup barrier.  The 4 lanes of a sample add the same partials in commuted order, so they agree bit for bit.
__device__ __forceinline__ float head1(const float *__restrict__ w3, Tile &h, const float *__restrict__ bias,
                                       const float *__restrict__ b3, int lane) {
  const int q = lane >> 4;
  f4 acc = z4();
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const f4 bb = *reinterpret_cast<const f4 *>(bias + 16 * ob + 4 * q);
    const f4 w = *reinterpret_cast<const f4 *>(w3 + 16 * ob + 4 * q);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      h.v[ob][r] = tanh_fast(h.v[ob][r] + bb[r]);
      acc[r] += w[r] * h.v[ob][r];
    }
  }
  float v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v + b3[0];
}

// dh = W3^T dz3 (dz3: this lane's sample's n_out output gradients)
__device__ __forceinline__ void back_out(const float *__restrict__ w3, int n_out, f4 dz3, Tile &dh, int q) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    f4 s = z4();
    for (int o = 0; o < n_out; ++o) {
      const f4 w = *reinterpret_cast<const f4 *>(w3 + o * H + 16 * ob + 4 * q);
      s += w * dz3[o];
    }
    dh.v[ob] = s;
  }
}

// t = t * (1 - y^2): tanh backward (torch tanh_backward: grad * (1 - y * y))
__device__ __forceinline__ void tanh_back(Tile &t, const Tile &y) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) t.v[ob] = t.v[ob] * (1.0f - y.v[ob] * y.v[ob]);
}

// sum over the 16 samples of a wave (lanes with equal lane >> 4: one DPP row), every lane of the row gets the sum:
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror -- four v_add with a DPP source
template <int C>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), C, 0xf, 0xf, false));
}
__device__ __forceinline__ float sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}

__device__ __forceinline__ void store_tile(float *__restrict__ M, const Tile &t, int64_t row, int q) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) *reinterpret_cast<f4 *>(M + row * H + 16 * ob + 4 * q) = t.v[ob];
}
__device__ __forceinline__ void load_tile(const float *__restrict__ M, Tile &t, int64_t row, int q) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) t.v[ob] = *reinterpret_cast<const f4 *>(M + row * H + 16 * ob + 4 * q);
}

// Workgroup partial of a per-neuron sum over the workgroup's 64 samples: red[w][n] per wave, then the 4 waves in a
// fixed order.  v[ob][r] = this lane's value for neuron 16 ob + 4 q + r (summed over the wave's samples here).
__device__ __forceinline__ void wg_neuron_sum(const Tile &t, float *red, float *__restrict__ out, int wave, int lane) {
  const int q = lane >> 4;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = sum16(t.v[ob][r]);
      if ((lane & 15) == 0) red[wave * H + 16 * ob + 4 * q + r] = s;
    }
  __syncthreads();
  const int n = threadIdx.x;  // WG == H
  out[n] = ((red[n] + red[H + n]) + red[2 * H + n]) + red[3 * H + n];
  __syncthreads();
}
__device__ __forceinline__ float wg_scalar_sum(float v, float *red, int wave, int lane) {
  // v: one value per sample (lanes 0..15 of each wave carry distinct samples; other lanes ignored)
  float s = (lane < 16) ? v : 0.0f;
  s = sum16(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const float tot = ((red[0] + red[1]) + red[2]) + red[3];
  __syncthreads();
  return tot;
}

// unscale an action in [-1, 1] to the critic's input (TwinQNetwork._unscale_action): ((a - low) / range) * 2 - 1
__device__ __forceinline__ float unscale(float a, float low, float range) { return ((a - low) / range) * 2.0f - 1.0f; }

// first-layer inputs of this lane from a state row (18 features) and 4 action inputs (already unscaled, or 0)
__device__ __forceinline__ void input_frags(const float *__restrict__ srow, const f4 act, bool with_act, float (&x)[S1],
                                            int q) {
#pragma unroll
  for (int s = 0; s < S1; ++s) {
    const int f = 4 * s + q;
    float v = 0.0f;
    if (f < 18) v = srow[f];
    else if (with_act && f < 22) {
      const int c = f - 18;
      v = c == 0 ? act[0] : c == 1 ? act[1] : c == 2 ? act[2] : act[3];
    }
    x[s] = v;
  }
}

// ------------------------------------------------------------------------------------------------ sampling
// The batch's replay slots and target noise from a counter-based RNG (Philox4x32-10 keyed by the learner's seed, the
// counter = (sample, update, purpose)): uniform slots floor(u * size) with a 53-bit u (rl/replay/uniform_buffer.py's
// (rand * size).astype(int)), and the target policy smoothing noise clamp(N(0, scale), -clip, clip) by Box-Muller
// (learner.py:80-93).  The update counter lives in device memory (graph replays advance it): critic_step bumps it.
struct P4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ P4 philox(uint64_t key, P4 c) {
  uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = P4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// sample e's replay slot of update `ctr` over `size` filled slots
__device__ __forceinline__ int64_t sample_slot(uint64_t seed, int64_t e, uint64_t ctr, uint64_t size) {
  const P4 r0 = philox(seed, P4{(uint32_t)e, (uint32_t)(e >> 32), (uint32_t)ctr, (uint32_t)(ctr >> 32)});
  const uint64_t bits = (((uint64_t)r0.x << 32) | r0.y) >> 11;
  const double u = (double)bits * (1.0 / 9007199254740992.0);
  const uint64_t i = (uint64_t)(u * (double)size);
  return (int64_t)(i < size ? i : size - 1);
}
// sample e's clipped target-smoothing noise of update `ctr`
__device__ __forceinline__ f4 sample_noise(uint64_t seed, int64_t e, uint64_t ctr, float scale, float clip) {
  const P4 r1 = philox(seed ^ 0x6E6F697365ull, P4{(uint32_t)e, (uint32_t)(e >> 32), (uint32_t)ctr, (uint32_t)(ctr >> 32)});
  const uint32_t w[4] = {r1.x, r1.y, r1.z, r1.w};
  float z[4];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float u1 = ((float)(w[2 * p] >> 8) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
    const float u2 = (float)(w[2 * p + 1] >> 8) * (1.0f / 16777216.0f);
    const float rad = sqrtf(-2.0f * logf(u1));
    float sn, cs;
    sincosf(6.283185307179586f * u2, &sn, &cs);
    z[2 * p] = rad * cs;
    z[2 * p + 1] = rad * sn;
  }
  f4 nz;
#pragma unroll
  for (int c = 0; c < 4; ++c) nz[c] = fminf(fmaxf(z[c] * scale, -clip), clip);
  return nz;
}
__global__ void __launch_bounds__(256) sample_kernel(hkl_sample_io io) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= io.batch) return;
  const uint64_t ctr = (uint64_t)*io.counter, size = (uint64_t)*io.size;
  io.idx[e] = sample_slot(io.seed, e, ctr, size);
  *reinterpret_cast<f4 *>(io.noise + e * 4) = sample_noise(io.seed, e, ctr, io.scale, io.clip);
}

// ------------------------------------------------------------------------------------------------ critic step
// Q(x) of one critic network (forward only): its output for this lane's sample
__device__ __forceinline__ float q_forward(const Net &c, const float (&x)[S1], Tile &h1, Tile &h2, int lane,
                                           f4 *sfrag) {
  gemm_in(c.f1(), x, h1, lane, sfrag);
  gemm256(c.fp(), h1, c.b1, h2, lane, sfrag);
  return head1(c.w3, h2, c.b2, c.b3, lane);
}

// one critic k of update_critic: forward on x, the weighted smooth-L1 (torch_utils.py:12-24; critic_loss =
// (loss1 + loss2) * 0.5, each a batch mean) and the backward to the first layer.  Stores H1, DZ1, DZ2 for the
// weight gradients (their bias gradients are the column sums wgrad takes); dW3 / db3 as workgroup partials.
__device__ __forceinline__ void critic_one(const hkl_critic_io &io, int k, const Net &c, const float (&x)[S1], float y,
                                           float w, int64_t row, float *red, f4 *sfrag, float &td, float &loss) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4;
  Tile h1, h2;
  gemm_in(c.f1(), x, h1, lane, sfrag);
  gemm256(c.fp(), h1, c.b1, h2, lane, sfrag);
  store_tile(io.h1[k], h1, row, q);
  const float qv = head1(c.w3, h2, c.b2, c.b3, lane);
  const float diff = qv - y, ad = fabsf(diff);
  loss += ad < 1.0f ? 0.5f * w * diff * diff : (ad - 0.5f) * w;
  const float g = (ad < 1.0f ? w * diff : (diff > 0.0f ? w : diff < 0.0f ? -w : 0.0f)) * (0.5f / (float)io.batch);
  td += ad;
  // output layer: dW3 = sum_j g_j h2_j, db3 = sum_j g_j
  Tile t;
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) t.v[ob] = h2.v[ob] * g;
  wg_neuron_sum(t, red, io.p_dw3[k] + blockIdx.x * H, wave, lane);
  const float gb = wg_scalar_sum(g, red, wave, lane);
  if (threadIdx.x == 0) io.p_db3[k][blockIdx.x] = gb;
  // dz2 = (W3^T g) * (1 - h2^2)
  back_out(c.w3, 1, f4{g, 0.0f, 0.0f, 0.0f}, t, q);
  tanh_back(t, h2);
  store_tile(io.dz2[k], t, row, q);
  // dz1 = (W2^T dz2) * (1 - h1^2)
  gemm256(c.bp(), t, nullptr, h2, lane, sfrag);
  tanh_back(h2, h1);
  store_tile(io.dz1[k], h2, row, q);
}

// compute_target + update_critic's forward / loss / backward for both critics (learner.py:75-136).
__global__ void __launch_bounds__(WG, 1) critic_step_kernel(hkl_critic_io io) {
  __shared__ f4 sfrag[2 * 16 * 64 + 64];  // two fragment buffers + the staged bias
  __shared__ float red[4 * H];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, j = lane & 15;
  const int64_t row = (int64_t)blockIdx.x * 64 + wave * 16 + j;  // this lane's sample (batch row)
  const int64_t src = io.idx[row];                                // its replay slot
  const float *s_row = io.ring_s + src * 18, *s2_row = io.ring_s2 + src * 18;
  const float rwd = io.ring_r[src], dn = io.ring_d[src];
  const f4 act = *reinterpret_cast<const f4 *>(io.ring_a + src * 4);
  const f4 nz = *reinterpret_cast<const f4 *>(io.noise + row * 4);
  const float w = io.iw ? io.iw[row] : 1.0f;
  const Net ta = net_of(io.target_actor), tq[2] = {net_of(io.target_q[0]), net_of(io.target_q[1])};
  const Net cq[2] = {net_of(io.q[0]), net_of(io.q[1])};

  // ---- target: y = r + gamma (1 - d) min(Q1', Q2')(s2, clamp(actor'(s2) + noise, -1, 1))
  float x[S1];
  input_frags(s2_row, z4(), false, x, q);
  Tile h1, h2;
  gemm_in(ta.f1(), x, h1, lane, sfrag);
  gemm256(ta.fp(), h1, ta.b1, h2, lane, sfrag);
  const f4 a2 = gemm_out(ta.fo(), h2, ta.b2, ta.b3, 4, lane, sfrag);
  f4 a2u;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float t = fminf(fmaxf(tanh_fast(a2[c]) + nz[c], -1.0f), 1.0f);  // torch.clamp(target_action + noise, -1, 1)
    a2u[c] = unscale(t, io.act_low[c], io.act_range[c]);
  }
  input_frags(s2_row, a2u, true, x, q);
  const float qt0 = q_forward(tq[0], x, h1, h2, lane, sfrag), qt1 = q_forward(tq[1], x, h1, h2, lane, sfrag);
  const float y = rwd + io.gamma * (1.0f - dn) * fminf(qt0, qt1);

  // ---- critics on (s, a)
  f4 au;
#pragma unroll
  for (int c = 0; c < 4; ++c) au[c] = unscale(act[c], io.act_low[c], io.act_range[c]);
  input_frags(s_row, au, true, x, q);
  {  // X0 row (shared by both critics' dW1): 22 features, zero padded; lane q writes 8 of its sample's 32
    float *xr = io.x0 + row * XP;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = 8 * q + e;
      xr[f] = f < 18 ? s_row[f] : f < 22 ? au[f - 18] : 0.0f;
    }
  }
  float td = 0.0f, loss = 0.0f;
  critic_one(io, 0, cq[0], x, y, w, row, red, sfrag, td, loss);
  critic_one(io, 1, cq[1], x, y, w, row, red, sfrag, td, loss);
  if (io.td && q == 0) io.td[row] = td * 0.5f;  // (|q1 - y| + |q2 - y|) / 2 (learner.py:163-170)
  const float ls = wg_scalar_sum(loss, red, wave, lane);
  if (threadIdx.x == 0) io.p_loss[blockIdx.x] = ls;
  if (io.sample_counter && blockIdx.x == 0 && threadIdx.x == 0) *io.sample_counter += 1;
}

// ------------------------------------------------------------------------------------------------ actor step
// update_actor's forward / backward (learner.py:138-175): loss = -mean Q1(s, actor(s)) with the updated critic.
__global__ void __launch_bounds__(WG, 1) actor_step_kernel(hkl_actor_io io) {
  __shared__ f4 sfrag[2 * 16 * 64 + 64];  // two fragment buffers + the staged bias
  __shared__ float red[4 * H];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, j = lane & 15;
  const int64_t row = (int64_t)blockIdx.x * 64 + wave * 16 + j;
  const int64_t src = io.idx[row];
  const float *s_row = io.ring_s + src * 18;
  const Net an = net_of(io.actor), qn = net_of(io.q1);
  float x[S1];
  input_frags(s_row, z4(), false, x, q);
  {
    float *xr = io.x0 + row * XP;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = 8 * q + e;
      xr[f] = f < 18 ? s_row[f] : 0.0f;
    }
  }
  Tile h1, h2;
  gemm_in(an.f1(), x, h1, lane, sfrag);
  gemm256(an.fp(), h1, an.b1, h2, lane, sfrag);
  store_tile(io.h1, h1, row, q);
  const f4 pre = gemm_out(an.fo(), h2, an.b2, an.b3, 4, lane, sfrag);
  store_tile(io.h2, h2, row, q);
  f4 a, au;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    a[c] = tanh_fast(pre[c]);
    au[c] = unscale(a[c], io.act_low[c], io.act_range[c]);
  }
  // Q1(s, a)
  input_frags(s_row, au, true, x, q);
  gemm_in(qn.f1(), x, h1, lane, sfrag);
  gemm256(qn.fp(), h1, qn.b1, h2, lane, sfrag);
  const float qv = gemm_out(qn.fo(), h2, qn.b2, qn.b3, 1, lane, sfrag)[0];
  const float g = -1.0f / (float)io.batch;  // d(-mean q) / dq
  Tile t;
  back_out(qn.w3, 1, f4{g, 0.0f, 0.0f, 0.0f}, t, q);
  tanh_back(t, h2);
  gemm256(qn.bp(), t, nullptr, h2, lane, sfrag);
  tanh_back(h2, h1);  // dz1 of Q1
  // dQ/d(unscaled action) = W1[:, 18:22]^T dz1, summed over the 4 lanes of the sample; then the unscale chain rule
  f4 da = z4();
  const f4 *wa = qn.wa();
#pragma unroll
  for (int ob = 0; ob < 16; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) da += wa[16 * ob + 4 * q + r] * h2.v[ob][r];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float v = da[c];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    da[c] = v * (2.0f / io.act_range[c]);
  }
  // actor output layer: dz3 = da * (1 - a^2); dW3 = sum_j dz3_j h2_j; db3 = sum_j dz3_j
  f4 dz3;
#pragma unroll
  for (int c = 0; c < 4; ++c) dz3[c] = da[c] * (1.0f - a[c] * a[c]);
  load_tile(io.h2, h2, row, q);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int ob = 0; ob < 16; ++ob) t.v[ob] = h2.v[ob] * dz3[c];
    wg_neuron_sum(t, red, io.p_dw3 + ((int64_t)blockIdx.x * 4 + c) * H, wave, lane);
    const float gb = wg_scalar_sum(dz3[c], red, wave, lane);
    if (threadIdx.x == 0) io.p_db3[blockIdx.x * 4 + c] = gb;
  }
  back_out(an.w3, 4, dz3, t, q);
  tanh_back(t, h2);
  store_tile(io.dz2, t, row, q);
  gemm256(an.bp(), t, nullptr, h2, lane, sfrag);
  load_tile(io.h1, h1, row, q);
  tanh_back(h2, h1);
  store_tile(io.dz1, h2, row, q);
  const float ls = wg_scalar_sum(-qv, red, wave, lane);
  if (threadIdx.x == 0) io.p_loss[blockIdx.x] = ls;
}

// ------------------------------------------------------------------------------------------------ weight gradients
// dW[o][k] = sum_j DZ[j][o] X[j][k] over one chunk of CHUNK samples, o in 128-row tiles, k in KT-wide tiles; 4 waves
// as 2 (o) x 2 (k).  The chunk streams through two LDS buffers 32 samples at a time (the next sub-chunk's loads are
// in flight while the current one is multiplied).  Output: slab[chunk][256][ldx] (natural W layout, fp32 partial
// sums; the adam kernel adds the chunks in order).  Blocks of the first k tile also sum DZ's columns: the bias
// gradient partials bslab[chunk][256].  One launch runs up to 4 jobs (blockIdx.z = job * chunks + chunk).
struct WgJob {
  const float *dz, *x;
  float *slab, *bslab;
  int ldx;
};
struct WgJobs {
  WgJob job[4];
  int chunks, chunk_size;
};
constexpr int kWgSub = 32, kWgOt = 128, kWgPad = 4;
// One split-K tile of dW = DZ^T X: output rows [o0, o0 + 128) x k columns [k0, k0 + KT) of job jb, summed over one
// chunk of samples (sa / sb: this block's double-buffered LDS staging, [2][32][128 + 4] and [2][32][KT + 4]).
template <int KT>
__device__ __forceinline__ void wgrad_tile(const WgJobs &jobs, int bx, int by, int bz, float (*sa)[kWgSub][kWgOt + kWgPad],
                                           float (*sb)[kWgSub][KT + kWgPad]) {
  constexpr int SUB = kWgSub, OT = kWgOt;
  constexpr int NB = KT == 128 ? 4 : 1;  // 16-column blocks per wave
  constexpr int LA = SUB * OT / 4 / WG, LB = (SUB * KT / 4 + WG - 1) / WG;  // f4 loads per thread per sub-chunk
  const int jb = bz / jobs.chunks, chunk = bz % jobs.chunks;
  const float *__restrict__ dz = jobs.job[jb].dz;
  const float *__restrict__ xs = jobs.job[jb].x;
  float *__restrict__ slab = jobs.job[jb].slab;
  float *__restrict__ bslab = jobs.job[jb].bslab;
  const int ldx = jobs.job[jb].ldx;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, kk = lane >> 4, i = lane & 15;
  const int wo = wave >> 1, wk = wave & 1;
  const int o0 = bx * OT, k0 = by * KT;
  const int csize = jobs.chunk_size;
  const int64_t j0 = (int64_t)chunk * csize;
  const bool bias = bslab != nullptr && by == 0;
  f4 acc[4][NB];
#pragma unroll
  for (int bo = 0; bo < 4; ++bo)
#pragma unroll
    for (int bk = 0; bk < NB; ++bk) acc[bo][bk] = z4();
  float bsum = 0.0f;  // thread t < OT: column o0 + t of DZ
  f4 ga[LA], gb[LB];
  auto fetch = [&](int sub) {
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int e = threadIdx.x + u * WG, rr = e / (OT / 4), cc = (e % (OT / 4)) * 4;
      ga[u] = *reinterpret_cast<const f4 *>(dz + (j0 + sub + rr) * H + o0 + cc);
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = threadIdx.x + u * WG, rr = e / (KT / 4), cc = (e % (KT / 4)) * 4;
      if (e < SUB * KT / 4) gb[u] = *reinterpret_cast<const f4 *>(xs + (j0 + sub + rr) * ldx + k0 + cc);
    }
  };
  auto stash = [&](int b) {
#pragma unroll
    for (int u = 0; u < LA; ++u) {
      const int e = threadIdx.x + u * WG, rr = e / (OT / 4), cc = (e % (OT / 4)) * 4;
      *reinterpret_cast<f4 *>(&sa[b][rr][cc]) = ga[u];
    }
#pragma unroll
    for (int u = 0; u < LB; ++u) {
      const int e = threadIdx.x + u * WG, rr = e / (KT / 4), cc = (e % (KT / 4)) * 4;
      if (e < SUB * KT / 4) *reinterpret_cast<f4 *>(&sb[b][rr][cc]) = gb[u];
    }
  };
  fetch(0);
  for (int sub = 0, b = 0; sub < csize; sub += SUB, b ^= 1) {
    stash(b);
    __syncthreads();
    if (sub + SUB < csize) fetch(sub + SUB);
    if (bias && threadIdx.x < OT) {
#pragma unroll
      for (int r = 0; r < SUB; ++r) bsum += sa[b][r][threadIdx.x];
    }
#pragma unroll
    for (int s = 0; s < SUB / 4; ++s) {
      const f4 A = *reinterpret_cast<const f4 *>(&sa[b][4 * s + kk][64 * wo + 4 * i]);  // rows o = 64 wo + 4 i + bo
      f4 B;
      if constexpr (NB == 4) B = *reinterpret_cast<const f4 *>(&sb[b][4 * s + kk][64 * wk + 4 * i]);  // k = 64 wk + 4 i + bk
      else B[0] = sb[b][4 * s + kk][16 * wk + i];                                                // k = 16 wk + i
#pragma unroll
      for (int bo = 0; bo < 4; ++bo)
#pragma unroll
        for (int bk = 0; bk < NB; ++bk) acc[bo][bk] = mfma(A[bo], B[bk], acc[bo][bk]);
    }
  }
  if (bias && threadIdx.x < OT) bslab[(int64_t)chunk * H + o0 + threadIdx.x] = bsum;
  // acc[bo][bk] lane (jj = i, q = kk) reg r: o = o0 + 64 wo + 4 (4 q + r) + bo, k = k0 + (NB == 4 ? 64 wk + 4 jj + bk : 16 wk + jj)
  float *dst = slab + (int64_t)chunk * H * ldx;
#pragma unroll
  for (int bo = 0; bo < 4; ++bo)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = o0 + 64 * wo + 4 * (4 * kk + r) + bo;
      if constexpr (NB == 4) {
        const f4 v = f4{acc[bo][0][r], acc[bo][1][r], acc[bo][2][r], acc[bo][3][r]};
        *reinterpret_cast<f4 *>(dst + (int64_t)o * ldx + k0 + 64 * wk + 4 * i) = v;
      } else {
        dst[(int64_t)o * ldx + k0 + 16 * wk + i] = acc[bo][0][r];
      }
    }
}

template <int KT>
__global__ void __launch_bounds__(WG, 1) wgrad_kernel(WgJobs jobs) {
  __shared__ float sa[2][kWgSub][kWgOt + kWgPad];
  __shared__ float sb[2][kWgSub][KT + kWgPad];
  wgrad_tile<KT>(jobs, blockIdx.x, blockIdx.y, blockIdx.z, sa, sb);
}

// hkl_wgrad_pair: a network's dW2 tiles (k width 256) and dW1 tiles (k width 32) in one launch -- blocks
// [0, n_wide) take the wide jobs (grid 2 x 2 x chunks per job), the rest the narrow ones (2 x 1 x chunks), so the
// short dW1 tiles fill the SIMDs the dW2 tiles leave and one launch gap is saved.  The narrow tile's staging
// lives inside the wide one's (same LDS as a wide-only block).
__global__ void __launch_bounds__(WG, 1) wgrad_pair_kernel(WgJobs wide, WgJobs narrow, int n_wide) {
  __shared__ float sa[2][kWgSub][kWgOt + kWgPad];
  __shared__ float sb[2][kWgSub][128 + kWgPad];
  static_assert(sizeof(float[2][kWgSub][XP + kWgPad]) <= sizeof(sb), "the narrow staging fits the wide one");
  const int id = blockIdx.x;
  if (id < n_wide) {
    wgrad_tile<128>(wide, id & 1, (id >> 1) & 1, id >> 2, sa, sb);
  } else {
    const int j = id - n_wide;
    wgrad_tile<XP>(narrow, j & 1, 0, j >> 1, sa, reinterpret_cast<float(*)[kWgSub][XP + kWgPad]>(&sb[0][0][0]));
  }
}

// ------------------------------------------------------------------------------------------------ Adam
// grad(e) = sum over chunks c (in order) of src[c * stride + row(e) * ld + col(e)]; then torch.optim.Adam (L2 weight
// decay, bias-corrected moments).  step: the optimiser's step count before this update (device, advanced by pack).
__global__ void __launch_bounds__(256) adam_kernel(hkl_adam_io io) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  int sidx = -1;
  int64_t base = 0;
  for (int s = 0; s < io.n_seg; ++s) {
    const int64_t n = (int64_t)io.seg[s].rows * io.seg[s].cols;
    if (e < base + n) {
      sidx = s;
      break;
    }
    base += n;
  }
  if (sidx >= 0) {
    const hkl_seg &S = io.seg[sidx];
    const int64_t k = e - base;
    const int64_t rr = k / S.cols, cc = k % S.cols;
    const float *src = S.src + rr * S.ld + cc;
    // 16 partial sums (chunk c into p16[c & 15], in increasing c), summed in a fixed tree; up to 64 slab loads in
    // flight per thread (the reduction is bound by memory-level parallelism: ~2 workgroups per CU at the C5
    // parameter counts)
    float p16[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) p16[u] = 0.0f;
    int c = 0;
    for (; c + 64 <= S.chunks; c += 64) {  // four rounds' loads in flight at once, added in the same order
      float q[64];
#pragma unroll
      for (int u = 0; u < 64; ++u) q[u] = src[(int64_t)(c + u) * S.stride];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < 16; ++u) p16[u] += q[16 * r + u];
    }
    for (; c + 32 <= S.chunks; c += 32) {  // two rounds' loads in flight at once, added in the same order
      float q[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) q[u] = src[(int64_t)(c + u) * S.stride];
#pragma unroll
      for (int u = 0; u < 16; ++u) p16[u] += q[u];
#pragma unroll
      for (int u = 0; u < 16; ++u) p16[u] += q[16 + u];
    }
    for (; c + 16 <= S.chunks; c += 16) {
      float q[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) q[u] = src[(int64_t)(c + u) * S.stride];
#pragma unroll
      for (int u = 0; u < 16; ++u) p16[u] += q[u];
    }
    for (; c < S.chunks; ++c) p16[c & 15] += src[(int64_t)c * S.stride];
#pragma unroll
    for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
      for (int u = 0; u < h; ++u) p16[u] = p16[u] + p16[u + h];
    float g = p16[0];
    float p = S.param[k];
    if (io.wd != 0.0f) g += io.wd * p;
    const float t = (float)(*io.step + 1);
    float m = S.m[k], v = S.v[k];
    m = m + (g - m) * (1.0f - io.beta1);  // exp_avg.lerp_(grad, 1 - beta1)
    v = v * io.beta2 + (1.0f - io.beta2) * g * g;
    const float bc1 = 1.0f - powf(io.beta1, t), bc2 = 1.0f - powf(io.beta2, t);
    const float denom = sqrtf(v) / sqrtf(bc2) + io.eps;
    p = p - (io.lr / bc1) * (m / denom);
    S.m[k] = m;
    S.v[k] = v;
    S.param[k] = p;
    if (io.polyak && S.target)  // soft_update with the new parameter: target.mul_(rho).add_(tau * param)
      S.target[k] = __fadd_rn(__fmul_rn(S.target[k], io.polyak_rho), __fmul_rn(io.polyak_tau, p));
  }
  if (blockIdx.x == 0 && io.loss_src) {
    // the step's loss: the sum of the workgroup partials (scaled), into the learner's accumulator -- a fixed-order
    // tree over workgroup 0's 256 threads (one thread summing 256 dependent loads was this kernel's tail)
    __shared__ float lred[256];
    float s = 0.0f;
    for (int c = threadIdx.x; c < io.loss_chunks; c += 256) s += io.loss_src[c];
    lred[threadIdx.x] = s;
    __syncthreads();
#pragma unroll
    for (int h = 128; h >= 1; h >>= 1) {
      if ((int)threadIdx.x < h) lred[threadIdx.x] = lred[threadIdx.x] + lred[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      *io.loss_sum += (double)(lred[0] * io.loss_scale);
      *io.loss_count += 1.0;
    }
  }
}

// target <- target * rho + tau * param (learner.py:214-218: mul_(rho), add_((1 - rho) * param); tau = 1 - rho
// rounded to fp32 like the reference's scalar)
__global__ void __launch_bounds__(256) polyak_kernel(float *__restrict__ t, const float *__restrict__ p, int64_t n, float rho,
                                                     float tau) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) t[e] = t[e] * rho + tau * p[e];
}

__global__ void tanh_probe_kernel(const float *x, float *y, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) y[e] = tanh_fast(x[e]);
}

// ------------------------------------------------------------------------------------------------ packing
__global__ void __launch_bounds__(256) pack_kernel(hkl_pack_io io) {
  const hkl_net &N = io.net[blockIdx.y];
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.y == 0 && e == 0 && io.step) *io.step += 1;  // the optimiser step this pack follows
  if (e >= kPackFloats) return;
  float *pk = N.pack;
  float v = 0.0f;
  if (e < kF1) {
    const int ob = (int)(e / 512), l = (int)(e / 8 % 64), s = (int)(e % 8);
    const int o = 16 * ob + (l & 15), c = 4 * s + (l >> 4);
    v = (s < S1 && c < N.n_in) ? N.w1[o * N.n_in + c] : 0.0f;
  } else if (e < kF1 + kFp) {
    const int64_t k = e - kF1;
    const int ob = (int)(k / 4096), kb = (int)(k / 256 % 16), l = (int)(k / 4 % 64), r = (int)(k % 4);
    v = N.w2[(16 * ob + (l & 15)) * H + 16 * kb + 4 * (l >> 4) + r];
  } else if (e < kF1 + kFp + kBp) {
    const int64_t k = e - kF1 - kFp;
    const int ib = (int)(k / 4096), ob = (int)(k / 256 % 16), l = (int)(k / 4 % 64), r = (int)(k % 4);
    v = N.w2[(16 * ob + 4 * (l >> 4) + r) * H + 16 * ib + (l & 15)];
  } else if (e < kF1 + kFp + kBp + kFo) {
    const int64_t k = e - kF1 - kFp - kBp;
    const int kb = (int)(k / 256), l = (int)(k / 4 % 64), r = (int)(k % 4);
    const int o = l & 15;
    v = o < N.n_out ? N.w3[o * H + 16 * kb + 4 * (l >> 4) + r] : 0.0f;
  } else {
    const int64_t k = e - kF1 - kFp - kBp - kFo;
    const int n = (int)(k / 4), c = (int)(k % 4);
    v = N.n_in == 22 ? N.w1[n * 22 + 18 + c] : 0.0f;
  }
  pk[e] = v;
}

}  // namespace hkl

using namespace hkl;

// ------------------------------------------------------------------------------------------------ C ABI
static thread_local char g_err[256];
static int fail(hipError_t e, const char *who) {
  snprintf(g_err, sizeof g_err, "%s: %s", who, hipGetErrorString(e));
  return HKL_E_DEVICE;
}

extern "C" {

const char *hkl_last_error(void) { return g_err; }

int hkl_pack(const hkl_net *nets, int n_nets, int64_t *step, void *stream) {
  if (n_nets < 1 || n_nets > 4) return HKL_E_INVALID;
  hkl_pack_io io{};
  for (int k = 0; k < n_nets; ++k) io.net[k] = nets[k];
  io.step = step;
  hipLaunchKernelGGL(pack_kernel, dim3((kPackFloats + 255) / 256, n_nets), dim3(256), 0, (hipStream_t)stream, io);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_pack");
}

int hkl_critic_step(const hkl_critic_io *io, void *stream) {
  if (!io || io->batch <= 0 || io->batch % CHUNK) return HKL_E_INVALID;
  hipLaunchKernelGGL(critic_step_kernel, dim3(io->batch / 64), dim3(WG), 0, (hipStream_t)stream, *io);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_critic_step");
}

int hkl_actor_step(const hkl_actor_io *io, void *stream) {
  if (!io || io->batch <= 0 || io->batch % CHUNK) return HKL_E_INVALID;
  hipLaunchKernelGGL(actor_step_kernel, dim3(io->batch / 64), dim3(WG), 0, (hipStream_t)stream, *io);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_actor_step");
}

// samples per split-K chunk (include/hockey_learner.h hkl_wgrad): a single k-width-256 job has 4 x B / 512 tiles
// at 512, half the workgroups the chip holds at C5's batch, so it takes 256-sample chunks
static int wg_chunk_size(int n_jobs, int k_width, int64_t batch) {
  return (k_width == 256 && n_jobs >= 2 && batch % 512 == 0) ? 512 : 256;
}

int hkl_wgrad(const hkl_wgrad_job *jobs, int n_jobs, int k_width, int64_t batch, void *stream) {
  if (!jobs || n_jobs < 1 || n_jobs > 4 || batch <= 0 || batch % CHUNK || (k_width != 256 && k_width != XP))
    return HKL_E_INVALID;
  WgJobs J{};
  for (int k = 0; k < n_jobs; ++k) J.job[k] = WgJob{jobs[k].dz, jobs[k].x, jobs[k].slab, jobs[k].bias_slab, k_width};
  // dW2 (k width 256): 512-sample chunks when the batch allows and two or more networks fill the chip (fewer
  // partial slabs for adam to add); one network (the actor) or dW1 (k width 32, a small tile per block): 256, for
  // more blocks
  J.chunk_size = wg_chunk_size(n_jobs, k_width, batch);
  J.chunks = (int)(batch / J.chunk_size);
  const unsigned z = (unsigned)(J.chunks * n_jobs);
  if (k_width == 256) hipLaunchKernelGGL(wgrad_kernel<128>, dim3(2, 2, z), dim3(WG), 0, (hipStream_t)stream, J);
  else hipLaunchKernelGGL(wgrad_kernel<32>, dim3(2, 1, z), dim3(WG), 0, (hipStream_t)stream, J);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_wgrad");
}

static WgJobs wg_jobs(const hkl_wgrad_job *jobs, int n_jobs, int k_width, int64_t batch) {
  WgJobs J{};
  for (int k = 0; k < n_jobs; ++k) J.job[k] = WgJob{jobs[k].dz, jobs[k].x, jobs[k].slab, jobs[k].bias_slab, k_width};
  J.chunk_size = wg_chunk_size(n_jobs, k_width, batch);
  J.chunks = (int)(batch / J.chunk_size);
  return J;
}

int hkl_wgrad_pair(const hkl_wgrad_job *wide, int n_wide, const hkl_wgrad_job *narrow, int n_narrow, int64_t batch,
                   void *stream) {
  if (!wide || !narrow || n_wide < 1 || n_wide > 4 || n_narrow < 1 || n_narrow > 4 || batch <= 0 || batch % CHUNK)
    return HKL_E_INVALID;
  const WgJobs W = wg_jobs(wide, n_wide, 256, batch), N = wg_jobs(narrow, n_narrow, XP, batch);
  const int nw = 4 * W.chunks * n_wide, nn = 2 * N.chunks * n_narrow;
  hipLaunchKernelGGL(wgrad_pair_kernel, dim3((unsigned)(nw + nn)), dim3(WG), 0, (hipStream_t)stream, W, N, nw);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_wgrad_pair");
}

int hkl_adam(const hkl_adam_io *io, void *stream) {
  if (!io || io->n_seg < 1 || io->n_seg > HKL_MAX_SEG) return HKL_E_INVALID;
  if (io->loss_src && (!io->loss_sum || !io->loss_count)) return HKL_E_INVALID;  // loss partials need a destination
  for (int s = 0; s < io->n_seg; ++s)
    if (!io->seg[s].param || !io->seg[s].m || !io->seg[s].v || !io->seg[s].src || (io->polyak && !io->seg[s].target))
      return HKL_E_INVALID;
  int64_t n = 0;
  for (int s = 0; s < io->n_seg; ++s) n += (int64_t)io->seg[s].rows * io->seg[s].cols;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *io);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_adam");
}

int hkl_polyak(float *target, const float *param, int64_t n, float rho, float tau, void *stream) {
  if (n <= 0) return HKL_E_INVALID;
  hipLaunchKernelGGL(polyak_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, target, param,
                     n, rho, tau);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_polyak");
}

int hkl_pack_floats(void) { return kPackFloats; }

int hkl_sample(const hkl_sample_io *io, void *stream) {
  if (!io || io->batch <= 0) return HKL_E_INVALID;
  hipLaunchKernelGGL(sample_kernel, dim3((unsigned)((io->batch + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *io);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_sample");
}

int hkl_tanh_probe(const float *x, float *y, int64_t n, void *stream) {
  if (n <= 0) return HKL_E_INVALID;
  hipLaunchKernelGGL(tanh_probe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, x, y, n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_tanh_probe");
}

}  // extern "C"
