/* hockey_learner.h -- C ABI of the fused fp32 MFMA TD3 learner (libhockey_learner.so, gfx950).
 *
 * Replaces, for large learner batches, the PyTorch ops of one rl/td3/learner.py TD3Learner.update
 * (:55-72): compute_target (:75-112), update_critic (:115-136), update_actor (:138-175) and soft_update (:196-218),
 * with Adam (rl/td3/agent.py:174-182).  hockey_amd/learner_hip.py binds it with ctypes; every pointer is a device
 * pointer (torch tensors' storage), every call is asynchronous on `stream` (a hipStream_t) and graph-capturable.
 * Batches are multiples of 256.  Returns HKL_OK or an error code; hkl_last_error() describes the last failure.
 */
#ifndef HOCKEY_LEARNER_H
#define HOCKEY_LEARNER_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HKL_OK 0
#define HKL_E_INVALID 1
#define HKL_E_DEVICE 2
#define HKL_MAX_SEG 12
/* floats of one network's MFMA operand pack (hk_learner.hip: f1, fp, bp, fo, wa) */
#define HKL_PACK_FLOATS (16 * 64 * 8 + 2 * 16 * 16 * 64 * 4 + 16 * 64 * 4 + 256 * 4)

/* one MLP n_in -> 256 -> 256 -> n_out (tanh hidden; rl/td3/networks.py ActorNetwork): torch Linear weights
 * [out][in] row-major, and its operand pack (hkl_pack writes it from the weights) */
typedef struct {
  const float *w1, *b1, *w2, *b2, *w3, *b3;
  float *pack;
  int32_t n_in, n_out;
} hkl_net;

/* compute_target + update_critic forward / backward for both critics.  Inputs: the replay ring's columns
 * (s [cap][18], a [cap][4], r [cap], s2 [cap][18], d [cap]), the sampled slots idx [B], the clipped target noise
 * [B][4], optional importance weights iw [B].  Outputs: X0 [B][32] (critic inputs), per critic k: H1, DZ1, DZ2
 * [B][256]; workgroup partials (B / 64 rows) of db1, db2, dW3 [.][256] and db3 [.]; loss partials [B / 64];
 * optional td [B] = (|q1 - y| + |q2 - y|) / 2 for prioritized replay.  (db1 / db2 come from hkl_wgrad's
 * column sums; p_db1 / p_db2 are unused.) */
typedef struct {
  int64_t batch;
  const int64_t *idx;
  const float *ring_s, *ring_a, *ring_r, *ring_s2, *ring_d;
  const float *noise, *iw;
  hkl_net target_actor, target_q[2], q[2];
  float gamma;
  float act_low[4], act_range[4];
  float *x0, *h1[2], *dz1[2], *dz2[2];
  float *p_db1[2], *p_db2[2], *p_dw3[2], *p_db3[2];
  float *p_loss, *td;
  int64_t *sample_counter; /* optional: hkl_sample's update counter, advanced by one at the end */
} hkl_critic_io;

/* update_actor forward / backward: actor(s), Q1(s, actor(s)) of the updated critic, d(-mean Q1).  Outputs: X0
 * [B][32], H1, H2, DZ1, DZ2 [B][256]; workgroup partials of dW3 [.][4][256], db3 [.][4]; loss partials
 * (p_db1 / p_db2 unused). */
typedef struct {
  int64_t batch;
  const int64_t *idx;
  const float *ring_s;
  hkl_net actor, q1;
  float act_low[4], act_range[4];
  float *x0, *h1, *h2, *dz1, *dz2;
  float *p_db1, *p_db2, *p_dw3, *p_db3;
  float *p_loss;
} hkl_actor_io;

/* one parameter tensor for hkl_adam: grad[r][c] = sum_{k < chunks} src[k * stride + r * ld + c]; target
 * (optional): the tensor's soft-update twin in the target network, updated when hkl_adam_io.polyak is set */
typedef struct {
  float *param, *m, *v;
  const float *src;
  int32_t rows, cols;
  int64_t ld;
  int32_t chunks;
  int64_t stride;
  float *target;
} hkl_seg;

typedef struct {
  hkl_seg seg[HKL_MAX_SEG];
  int32_t n_seg;
  float lr, beta1, beta2, eps, wd;
  const int64_t *step;           /* optimiser steps taken so far (device); hkl_pack advances it */
  const float *loss_src;         /* optional: loss partials; *loss_sum += their sum x loss_scale, *loss_count += 1 */
  int32_t loss_chunks;
  float loss_scale;
  double *loss_sum, *loss_count;
  /* polyak != 0: after its Adam step every parameter p with a segment target t also takes soft_update
   * (learner.py:214-218): t = t * polyak_rho + polyak_tau * p, each product rounded (torch's mul_ then add_) --
   * the same values as hkl_polyak after hkl_adam, one launch fewer */
  int32_t polyak;
  float polyak_rho, polyak_tau;
} hkl_adam_io;

typedef struct {
  hkl_net net[4];
  int64_t *step;
} hkl_pack_io;

const char *hkl_last_error(void);
int hkl_pack_floats(void);
/* re-lay the weights of 1..4 networks out as MFMA operands; advances *step by one when step != NULL */
int hkl_pack(const hkl_net *nets, int n_nets, int64_t *step, void *stream);
int hkl_critic_step(const hkl_critic_io *io, void *stream);
int hkl_actor_step(const hkl_actor_io *io, void *stream);
/* weight-gradient job: slab[c][256][k_width] = sum over the samples j of chunk c (k_width 256: 512 samples each
 * when the launch has two or more k-width-256 jobs and the batch is a multiple of 512, else 256; k_width 32: 256)
 * of dz[j][o] x[j][k]
 * (dz [B][256], x [B][k_width]); bias_slab (optional) [c][256] = the chunk's column sums of dz */
typedef struct {
  const float *dz, *x;
  float *slab, *bias_slab;
} hkl_wgrad_job;
/* 1..4 jobs of one k_width (256 or 32) in one launch */
int hkl_wgrad(const hkl_wgrad_job *jobs, int n_jobs, int k_width, int64_t batch, void *stream);
/* hkl_wgrad for n_wide k-width-256 jobs (dW2) and n_narrow k-width-32 jobs (dW1) in one launch (the same slabs as
 * the two hkl_wgrad calls, bit for bit). */
int hkl_wgrad_pair(const hkl_wgrad_job *wide, int n_wide, const hkl_wgrad_job *narrow, int n_narrow, int64_t batch,
                   void *stream);
int hkl_adam(const hkl_adam_io *io, void *stream);
/* target = target * rho + tau * param over n floats (soft_update; tau = 1 - rho) */
int hkl_polyak(float *target, const float *param, int64_t n, float rho, float tau, void *stream);

/* the batch's replay slots idx[B] (uniform over the ring's *size filled slots) and clipped target noise [B][4]
 * from Philox4x32-10 keyed by seed, counter = *counter (device; hkl_critic_step advances it) */
typedef struct {
  int64_t batch;
  uint64_t seed;
  const int64_t *counter, *size;
  int64_t *idx;
  float *noise;
  float scale, clip;
} hkl_sample_io;
int hkl_sample(const hkl_sample_io *io, void *stream);

/* y = the kernels' tanh of x (n floats; a test probe of the activation's accuracy) */
int hkl_tanh_probe(const float *x, float *y, int64_t n, void *stream);

#ifdef __cplusplus
}
#endif
#endif
