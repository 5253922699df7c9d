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
//                 (lr, betas (0.9, 0.999), eps, L2 weight decay; rl/td3/agent.py:174-182);
//   polyak        soft_update (:196-218), then pack re-lays the changed weights out for the MFMA operands.
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
constexpr int CHUNK = 256;  // samples per split-K chunk of the weight-gradient kernel

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 z4() { return f4{0.0f, 0.0f, 0.0f, 0.0f}; }

struct Tile {
  f4 v[16];
};

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
// out = W1 x (no bias): x[s] = this lane's input for k-step s (feature 4 s + (lane >> 4))
__device__ __forceinline__ void gemm_in(const float *__restrict__ f1, const float (&x)[S1], Tile &out, int lane) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const f4 lo = *reinterpret_cast<const f4 *>(f1 + (ob * 64 + lane) * 8);
    const f4 hi = *reinterpret_cast<const f4 *>(f1 + (ob * 64 + lane) * 8 + 4);
    f4 acc = z4();
    acc = mfma(lo[0], x[0], acc);
    acc = mfma(lo[1], x[1], acc);
    acc = mfma(lo[2], x[2], acc);
    acc = mfma(lo[3], x[3], acc);
    acc = mfma(hi[0], x[4], acc);
    acc = mfma(hi[1], x[5], acc);
    out.v[ob] = acc;
  }
}

// out = P in, P a packed 256 x 256 operand (fp: W2 in; bp: W2^T in).  The A fragments of the next 16-neuron
// k-block are loaded while the current one is multiplied.
__device__ __forceinline__ void gemm256(const f4 *__restrict__ P, const Tile &in, Tile &out, int lane) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) out.v[ob] = z4();
  f4 a[16];
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) a[ob] = P[(ob * 16) * 64 + lane];
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) {
    f4 an[16];
    if (kb + 1 < 16) {
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) an[ob] = P[(ob * 16 + kb + 1) * 64 + lane];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float b = in.v[kb][r];
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) out.v[ob] = mfma(a[ob][r], b, out.v[ob]);
    }
    if (kb + 1 < 16) {
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) a[ob] = an[ob];
    }
  }
}

// t = tanh(t + b) (Linear bias, then the tanh activation)
__device__ __forceinline__ void bias_tanh(Tile &t, const float *__restrict__ b, int q) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const f4 bb = *reinterpret_cast<const f4 *>(b + 16 * ob + 4 * q);
#pragma unroll
    for (int r = 0; r < 4; ++r) t.v[ob][r] = tanhf(t.v[ob][r] + bb[r]);
  }
}

// the n_out (<= 4) outputs W3 h + b3 of this lane's sample, broadcast to every lane of the sample
__device__ __forceinline__ f4 gemm_out(const f4 *__restrict__ fo, const Tile &h, const float *__restrict__ b3, int n_out,
                                       int lane) {
  f4 acc0 = z4(), acc1 = z4();
#pragma unroll
  for (int kb = 0; kb < 16; ++kb) {
    const f4 a = fo[kb * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (kb & 1) acc1 = mfma(a[r], h.v[kb][r], acc1);
      else acc0 = mfma(a[r], h.v[kb][r], acc0);
    }
  }
  const f4 acc = acc0 + acc1;  // lanes 0..15 hold outputs 0..3 of sample lane & 15
  f4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = __shfl(acc[r], lane & 15) + (r < n_out ? b3[r] : 0.0f);
  return o;
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

// sum over the 16 samples of a wave (lanes with equal lane >> 4)
__device__ __forceinline__ float sum16(float v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
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

// ------------------------------------------------------------------------------------------------ critic step
// Q(x) of one critic network (forward only): its output for this lane's sample
__device__ __forceinline__ float q_forward(const Net &c, const float (&x)[S1], Tile &h1, Tile &h2, int lane, int q) {
  gemm_in(c.f1(), x, h1, lane);
  bias_tanh(h1, c.b1, q);
  gemm256(c.fp(), h1, h2, lane);
  bias_tanh(h2, c.b2, q);
  return gemm_out(c.fo(), h2, c.b3, 1, lane)[0];
}

// one critic k of update_critic: forward on x, the weighted smooth-L1 (torch_utils.py:12-24; critic_loss =
// (loss1 + loss2) * 0.5, each a batch mean) and the backward to the first layer
__device__ __forceinline__ void critic_one(const hkl_critic_io &io, int k, const Net &c, const float (&x)[S1], float y,
                                           float w, int64_t row, float *red, float &td, float &loss) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4;
  Tile h1, h2;
  gemm_in(c.f1(), x, h1, lane);
  bias_tanh(h1, c.b1, q);
  gemm256(c.fp(), h1, h2, lane);
  bias_tanh(h2, c.b2, q);
  const float qv = gemm_out(c.fo(), h2, c.b3, 1, lane)[0];
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
  store_tile(io.h1[k], h1, row, q);
  wg_neuron_sum(t, red, io.p_db2[k] + blockIdx.x * H, wave, lane);
  // dz1 = (W2^T dz2) * (1 - h1^2)
  gemm256(c.bp(), t, h2, lane);
  tanh_back(h2, h1);
  store_tile(io.dz1[k], h2, row, q);
  wg_neuron_sum(h2, red, io.p_db1[k] + blockIdx.x * H, wave, lane);
}

// compute_target + update_critic's forward / loss / backward for both critics (learner.py:75-136).
__global__ void __launch_bounds__(WG, 1) critic_step_kernel(hkl_critic_io io) {
  __shared__ float red[4 * H];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, j = lane & 15;
  const int64_t g = blockIdx.x;
  const int64_t row = g * 64 + wave * 16 + j;  // this lane's sample (batch row)
  const int64_t src = io.idx[row];             // its replay slot
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
  gemm_in(ta.f1(), x, h1, lane);
  bias_tanh(h1, ta.b1, q);
  gemm256(ta.fp(), h1, h2, lane);
  bias_tanh(h2, ta.b2, q);
  f4 a2 = gemm_out(ta.fo(), h2, ta.b3, 4, lane);
  f4 a2u;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const float t = fminf(fmaxf(tanhf(a2[c]) + nz[c], -1.0f), 1.0f);  // torch.clamp(target_action + noise, -1, 1)
    a2u[c] = unscale(t, io.act_low[c], io.act_range[c]);
  }
  input_frags(s2_row, a2u, true, x, q);
  const float qt0 = q_forward(tq[0], x, h1, h2, lane, q), qt1 = q_forward(tq[1], x, h1, h2, lane, q);
  const float y = rwd + io.gamma * (1.0f - dn) * fminf(qt0, qt1);

  // ---- critics on (s, a)
  f4 au;
#pragma unroll
  for (int c = 0; c < 4; ++c) au[c] = unscale(act[c], io.act_low[c], io.act_range[c]);
  input_frags(s_row, au, true, x, q);
  if (q == 0) {  // X0 row (shared by both critics' dW1): 22 features, zero padded
    float *xr = io.x0 + row * XP;
    for (int f = 0; f < XP; ++f) xr[f] = f < 18 ? s_row[f] : f < 22 ? au[f - 18] : 0.0f;
  }
  float td = 0.0f, loss = 0.0f;
  critic_one(io, 0, cq[0], x, y, w, row, red, td, loss);
  critic_one(io, 1, cq[1], x, y, w, row, red, td, loss);
  if (io.td && q == 0) io.td[row] = td * 0.5f;  // (|q1 - y| + |q2 - y|) / 2 (learner.py:163-170)
  const float ls = wg_scalar_sum(loss, red, wave, lane);
  if (threadIdx.x == 0) io.p_loss[blockIdx.x] = ls;
}

// ------------------------------------------------------------------------------------------------ actor step
// update_actor's forward / backward (learner.py:138-175): loss = -mean Q1(s, actor(s)) with the updated critic.
__global__ void __launch_bounds__(WG, 1) actor_step_kernel(hkl_actor_io io) {
  __shared__ float red[4 * H];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, j = lane & 15;
  const int64_t row = (int64_t)blockIdx.x * 64 + wave * 16 + j;
  const int64_t src = io.idx[row];
  const float *s_row = io.ring_s + src * 18;
  const Net an = net_of(io.actor), qn = net_of(io.q1);
  float x[S1];
  input_frags(s_row, z4(), false, x, q);
  if (q == 0) {
    float *xr = io.x0 + row * XP;
    for (int f = 0; f < XP; ++f) xr[f] = f < 18 ? s_row[f] : 0.0f;
  }
  Tile h1, h2;
  gemm_in(an.f1(), x, h1, lane);
  bias_tanh(h1, an.b1, q);
  store_tile(io.h1, h1, row, q);
  gemm256(an.fp(), h1, h2, lane);
  bias_tanh(h2, an.b2, q);
  store_tile(io.h2, h2, row, q);
  const f4 pre = gemm_out(an.fo(), h2, an.b3, 4, lane);
  f4 a, au;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    a[c] = tanhf(pre[c]);
    au[c] = unscale(a[c], io.act_low[c], io.act_range[c]);
  }
  // Q1(s, a)
  input_frags(s_row, au, true, x, q);
  gemm_in(qn.f1(), x, h1, lane);
  bias_tanh(h1, qn.b1, q);
  gemm256(qn.fp(), h1, h2, lane);
  bias_tanh(h2, qn.b2, q);
  const float qv = gemm_out(qn.fo(), h2, qn.b3, 1, lane)[0];
  const float g = -1.0f / (float)io.batch;  // d(-mean q) / dq
  Tile t;
  back_out(qn.w3, 1, f4{g, 0.0f, 0.0f, 0.0f}, t, q);
  tanh_back(t, h2);
  gemm256(qn.bp(), t, h2, lane);
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
  wg_neuron_sum(t, red, io.p_db2 + (int64_t)blockIdx.x * H, wave, lane);
  gemm256(an.bp(), t, h2, lane);
  load_tile(io.h1, h1, row, q);
  tanh_back(h2, h1);
  store_tile(io.dz1, h2, row, q);
  wg_neuron_sum(h2, red, io.p_db1 + (int64_t)blockIdx.x * H, wave, lane);
  const float ls = wg_scalar_sum(-qv, red, wave, lane);
  if (threadIdx.x == 0) io.p_loss[blockIdx.x] = ls;
}

// ------------------------------------------------------------------------------------------------ weight gradients
// dW[o][k] = sum_j DZ[j][o] X[j][k] over one chunk of CHUNK samples, o in 128-row tiles, k in KT-wide tiles; 4 waves
// as 2 (o) x 2 (k).  The chunk streams through LDS 32 samples at a time.  Output: slab[chunk][256][ldx] (natural
// W layout, fp32 partial sums; the adam kernel adds the chunks in order).
template <int KT>
__global__ void __launch_bounds__(WG, 1) wgrad_kernel(const float *__restrict__ dz, const float *__restrict__ xs, int ldx,
                                                      float *__restrict__ slab) {
  constexpr int SUB = 32, OT = 128, PAD = 4;
  constexpr int NB = KT == 128 ? 4 : 1;  // 16-column blocks per wave
  __shared__ float sa[SUB][OT + PAD];
  __shared__ float sb[SUB][KT + PAD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, kk = lane >> 4, i = lane & 15;
  const int wo = wave >> 1, wk = wave & 1;
  const int o0 = blockIdx.x * OT, k0 = blockIdx.y * KT;
  const int64_t j0 = (int64_t)blockIdx.z * CHUNK;
  f4 acc[4][NB];
#pragma unroll
  for (int bo = 0; bo < 4; ++bo)
#pragma unroll
    for (int bk = 0; bk < NB; ++bk) acc[bo][bk] = z4();
  for (int sub = 0; sub < CHUNK; sub += SUB) {
    // stage DZ[j0 + sub .. +32][o0 .. o0 + 128] and X[..][k0 .. k0 + KT]
    for (int e = threadIdx.x; e < SUB * OT / 4; e += WG) {
      const int rr = e / (OT / 4), cc = (e % (OT / 4)) * 4;
      *reinterpret_cast<f4 *>(&sa[rr][cc]) = *reinterpret_cast<const f4 *>(dz + (j0 + sub + rr) * H + o0 + cc);
    }
    for (int e = threadIdx.x; e < SUB * KT / 4; e += WG) {
      const int rr = e / (KT / 4), cc = (e % (KT / 4)) * 4;
      *reinterpret_cast<f4 *>(&sb[rr][cc]) = *reinterpret_cast<const f4 *>(xs + (j0 + sub + rr) * ldx + k0 + cc);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < SUB / 4; ++s) {
      const f4 A = *reinterpret_cast<const f4 *>(&sa[4 * s + kk][64 * wo + 4 * i]);  // rows o = 64 wo + 4 i + bo
      f4 B;
      if constexpr (NB == 4) B = *reinterpret_cast<const f4 *>(&sb[4 * s + kk][64 * wk + 4 * i]);  // k = 64 wk + 4 i + bk
      else B[0] = sb[4 * s + kk][16 * wk + i];                                                // k = 16 wk + i
#pragma unroll
      for (int bo = 0; bo < 4; ++bo)
#pragma unroll
        for (int bk = 0; bk < NB; ++bk) acc[bo][bk] = mfma(A[bo], B[bk], acc[bo][bk]);
    }
    __syncthreads();
  }
  // acc[bo][bk] lane (jj = i, q = kk) reg r: o = o0 + 64 wo + 4 (4 q + r) + bo, k = k0 + (NB == 4 ? 64 wk + 4 jj + bk : 16 wk + jj)
  float *dst = slab + (int64_t)blockIdx.z * H * ldx;
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
    float g = 0.0f;
    for (int c = 0; c < S.chunks; ++c) g += src[(int64_t)c * S.stride];
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
  }
  if (e == 0 && io.loss_src) {  // the step's loss: sum of the workgroup partials / batch, into the learner's accumulator
    float s = 0.0f;
    for (int c = 0; c < io.loss_chunks; ++c) s += io.loss_src[c];
    *io.loss_sum += (double)(s * io.loss_scale);
    *io.loss_count += 1.0;
  }
}

// target <- target * rho + tau * param (learner.py:214-218: mul_(rho), add_((1 - rho) * param); tau = 1 - rho
// rounded to fp32 like the reference's scalar)
__global__ void __launch_bounds__(256) polyak_kernel(float *__restrict__ t, const float *__restrict__ p, int64_t n, float rho,
                                                     float tau) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) t[e] = t[e] * rho + tau * p[e];
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
  if (n_nets < 1 || n_nets > 3) return HKL_E_INVALID;
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

int hkl_wgrad(const float *dz, const float *x, int k_width, int64_t batch, float *slab, void *stream) {
  if (batch <= 0 || batch % CHUNK || (k_width != 256 && k_width != XP)) return HKL_E_INVALID;
  const unsigned chunks = (unsigned)(batch / CHUNK);
  if (k_width == 256)
    hipLaunchKernelGGL(wgrad_kernel<128>, dim3(2, 2, chunks), dim3(WG), 0, (hipStream_t)stream, dz, x, 256, slab);
  else
    hipLaunchKernelGGL(wgrad_kernel<32>, dim3(2, 1, chunks), dim3(WG), 0, (hipStream_t)stream, dz, x, XP, slab);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HKL_OK : fail(e, "hkl_wgrad");
}

int hkl_adam(const hkl_adam_io *io, void *stream) {
  if (!io || io->n_seg < 1 || io->n_seg > HKL_MAX_SEG) return HKL_E_INVALID;
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

}  // extern "C"
