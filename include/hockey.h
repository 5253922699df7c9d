/* hockey.h -- C ABI of the MI355X-native batched hockey simulator (libhockey_hip.so).
 *
 * Drop-in boundary for the reference's per-step hot path (julilili42/hockey-env):
 *   hk_reset           replaces HockeyEnv.reset            hockey/hockey_env.py:345-418
 *   hk_step            replaces HockeyEnv.step             hockey/hockey_env.py:658-695
 *                      (+ HockeyEnv_BasicOpponent.step     hockey/hockey_env.py:882-886 via policies)
 *     io.obs2/reward2  replace obs_agent_two / get_info_agent_two / get_reward_agent_two
 *                                                          hockey/hockey_env.py:500-516, 537-540, 568-591
 *     HK_POLICY_BASIC  replaces BasicOpponent.act          hockey/hockey_env.py:781-833
 *   hk_set_state       replaces HockeyEnv.set_state        hockey/hockey_env.py:594-608 (raw-state form)
 * The reference exposes these through gymnasium (register('Hockey-v0' / 'Hockey-One-v0'),
 * hockey_env.py:889-903); the Python host layer (hockey-env_amd/hockey_amd) binds this ABI with
 * ctypes and keeps that gymnasium surface.  See INTEGRATION.md for the binding.
 *
 * Conventions: every array is DEVICE memory laid out [N, k] row-major (arena-major), N = n_arenas
 * of the context.  Calls are asynchronous on `stream` (a hipStream_t, NULL = default stream) and
 * return 0 on success or a negative HK_E* code; hk_last_error() describes the last failure of the
 * calling thread.  No C++ exceptions cross the ABI.  A context is bound to one device and is not
 * re-entrant: callers serialise calls per context.
 */
#ifndef HOCKEY_H
#define HOCKEY_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HK_OBS_DIM 18
#define HK_ACT_DIM 8
#define HK_INFO_DIM 4
#define HK_STATE_DIM 18 /* p1, p2, puck: body-origin x, y, angle, vx, vy, omega */
#define HK_AUX_DIM 5    /* has_puck1, has_puck2, time, done, winner */
#define HK_PARAM_DIM 6  /* reset placement: p2x, p2y, puckx, pucky, puck_fx, puck_fy */
#define HK_DEBUG_DIM 13 /* pre-solve F1xy, F2xy, Fpuck xy, tau1, tau2, ldamp1,2,puck, adamp1,2 */
#define HK_NUM_COUNTERS 16
#define HK_RECORD_DIM 16 /* hk_step_io.record: f64 per arena */

enum {
  HK_OK = 0,
  HK_E_INVALID = -1,  /* bad argument */
  HK_E_HIP = -2,      /* HIP runtime error */
  HK_E_NOMEM = -3,    /* device allocation failed */
  HK_E_DEVICE = -4    /* no usable gfx950 device */
};

/* per-player action source, fused into the step kernel */
enum {
  HK_POLICY_EXTERNAL = 0,     /* take io.actions[:, 4p:4p+4] */
  HK_POLICY_RANDOM = 1,       /* U(-1,1)^4 from Philox4x32-10 keyed by (seed, arena, step) */
  HK_POLICY_BASIC_WEAK = 2,   /* BasicOpponent(weak=True) on the player's own-frame obs */
  HK_POLICY_BASIC_STRONG = 3  /* BasicOpponent(weak=False) */
};

/* io.flags */
enum {
  HK_STEP_SKIP_PHYSICS = 1 /* world.Step is a no-op (golden-vector harness) */
};

/* counters (int64, accumulated on device since create / last hk_reset_counters) */
enum {
  HK_CNT_STEPS = 0,     /* env-steps simulated */
  HK_CNT_EPISODES = 1,  /* episodes finished (done edges) */
  HK_CNT_GOALS_P1 = 2,  /* episodes won by player 1 */
  HK_CNT_GOALS_P2 = 3,  /* episodes won by player 2 */
  HK_CNT_TOI = 4,       /* solved time-of-impact events */
  HK_CNT_OVERFLOW = 5,  /* island / TOI capacity overflows (must stay 0) */
  HK_CNT_LARGE_ISLANDS = 6, /* solver calls with more contacts than the register fast path holds */
  HK_CNT_BAD_POLICY = 7     /* arena-steps whose io.policy2 entry was not an HK_POLICY_* id (that player
                               acted with zeros); must stay 0 */
};

typedef struct hk_config {
  int32_t keep_mode;         /* HockeyEnv(keep_mode=True)  hockey_env.py:91 */
  int32_t mode;              /* 0 NORMAL, 1 TRAIN_SHOOTING, 2 TRAIN_DEFENSE (Mode, :78-81) */
  int32_t auto_reset;        /* 0 = reference semantics (sticky done, :685-695); 1 = an arena that is done
                                after a step is reset (device placement) at the end of that same step:
                                done / reward / info describe the terminal step, obs / obs2 the new
                                episode's first state, io.final_obs the terminal observation */
  int32_t vel_ref_semantics; /* 0 = pybox2d copy semantics (default) */
  int32_t policy[2];         /* HK_POLICY_* for player 1 and player 2 */
  uint64_t seed;             /* Philox key for device randomness */
  int64_t arena_offset;      /* global id of local arena 0: RNG streams are keyed by global arena id, so a
                                shard of a multi-GPU run reproduces the same arenas bit for bit */
  int32_t diag_flags;        /* HK_DIAG_* (0 in production): test-only routing of bit-identical slow paths */
} hk_config;

/* hk_config.diag_flags */
enum {
  HK_DIAG_LARGE_ISLANDS = 1 /* solve every island / TOI mini-island on the HBM slot file (the path islands
                               larger than the register slots take, ~1e-5 of arena-steps); same results */
};

typedef struct hk_step_io {
  const float *actions;   /* [N,8] f32 joint action (external players), may be NULL if none external */
  const double *opp_inc;  /* [N,2] f64 BasicOpponent phase increments or NULL (= Philox U(0,0.2)) */
  float *obs;             /* [N,18] f32 agent-1 observation (or NULL) */
  float *obs2;            /* [N,18] f32 agent-2 mirrored observation (or NULL) */
  float *reward;          /* [N]    f32 agent-1 reward (or NULL) */
  float *reward2;         /* [N]    f32 agent-2 reward (or NULL) */
  uint8_t *done;          /* [N]    done flag (or NULL) */
  float *info;            /* [N,4]  f32 {winner, closeness, touch, direction} (or NULL) */
  float *info2;           /* [N,4]  f32 agent-2 info (or NULL) */
  float *actions_out;     /* [N,8]  f32 joint action actually applied (or NULL) */
  float *debug;           /* [N,13] f32 pre-solve forces / torques / dampings (or NULL) */
  float *final_obs;       /* [N,18] f32 observation after the step's physics (or NULL): the terminal
                             observation of arenas that auto-reset in this step, == obs for the others */
  int32_t flags;          /* HK_STEP_* */
  const uint8_t *policy2; /* [N] u8 per-arena player-2 policy (HK_POLICY_*) for this step, overriding the
                             context's, or NULL: rl/training/opponent_manager.py:62-91 draws player 2's
                             opponent (self-play / strong / weak bot) per step.  EXTERNAL reads actions[:,4:8],
                             so io.actions must be given with an override (HK_E_INVALID otherwise); an id
                             above 3 is counted in HK_CNT_BAD_POLICY and that player acts with zeros.
                             Under an override the strong bot keeps phase row 1 and the weak bot its own row 2
                             (the reference's OpponentManager holds one BasicOpponent of each kind) */
  double *record;         /* [N,16] f64 per-step record (or NULL), the float64 values the reference's step
                             returns, written by the step kernel so a single-env caller needs one launch and
                             one copy: [0:4] info {winner, closeness, touch, direction} (_get_info), [4:8]
                             info2 (get_info_agent_two), [8] reward (get_reward(info)), [9] reward2
                             (get_reward_agent_two(info2)), [10] has_puck1, [11] has_puck2, [12] time, [13]
                             done, [14] winner -- after the step, before any auto-reset -- [15] 0.
                             hockey_env.py:542-591, 518-540, 685-693 */
} hk_step_io;

const char *hk_last_error(void);
const char *hk_version(void);

int hk_create(int device, int64_t n_arenas, const hk_config *cfg, void **ctx_out);
int hk_destroy(void *ctx);
int64_t hk_num_arenas(const void *ctx);
int hk_set_policy(void *ctx, int player, int policy);

/* Reset the arenas selected by mask ([N] u8, NULL = all).  params ([N,6] f32) is the placement drawn on
 * the host from the reference's PCG64 stream (explicit seeds); NULL = device Philox placement for the
 * context's mode.  max_t ([N] i32) NULL = mode default (250 NORMAL / 80 training); values outside [0, 65535] are
 * rejected with HK_E_INVALID (checked on the host before any launch; r06 packs max_t into 16 bits).  one_starts ([N] u8)
 * is only read when params == NULL (NORMAL puck side); NULL = toggle the per-arena flag like
 * reset(one_starting=None). */
int hk_reset(void *ctx, const uint8_t *mask, const float *params, const int32_t *max_t,
             const uint8_t *one_starts, void *stream);

int hk_step(void *ctx, const hk_step_io *io, void *stream);

/* HockeyEnv.step of a SINGLE-arena context with host buffers: the reference's deployment shape (one env, numpy
 * in and out, hockey_env.py:658-695) in one call.  The action (and BasicOpponent phase increments) go through
 * the context's pinned, device-mapped buffer and the packed result returns to `out` before the call returns.
 * By default a resident step server does the step: a one-wave kernel that stays on the GPU on a private stream
 * (started on the first call, ordered after the work already on `stream`) and serves each call's request from
 * the mapped buffer, so a step costs no kernel launch.  It exits after 20 ms without a request or 2 s in all and
 * is restarted on demand; every other entry point of the context stops it first, so context calls stay ordered
 * as on one stream.  HK_STEP_HOST_SERVER=0 launches one step kernel per call on `stream` instead (the host waits
 * on a completion word the kernel stores after its last output); HK_STEP_HOST_STAGED=1 stages through device
 * copies (A/B timing).  actions: host [1,8] f32 (NULL if no player is external); opp_inc: host [1,2] f64 or
 * NULL; flags: HK_STEP_* (as hk_step_io.flags); out: host buffer of HK_HOST_RECORD_BYTES = obs f32[18] @0,
 * obs2 f32[18] @72, done u8 @144, hk_step_io.record f64[16] @152.  HK_E_INVALID for a context with more than
 * one arena. */
#define HK_HOST_RECORD_BYTES 280
int hk_step_host(void *ctx, const float *actions, const double *opp_inc, int32_t flags, void *out, void *stream);

/* n_steps consecutive hk_step calls in ONE launch (a rollout with fused or pre-supplied actions).  Every
 * io array gains a leading [n_steps] dimension (actions [n_steps,N,8], obs [n_steps,N,18], ...); debug, if
 * given, describes the last step.  Results are bit-identical to n_steps hk_step calls; the waves of the
 * launch advance independently instead of meeting at a per-step kernel boundary. */
int hk_rollout(void *ctx, int32_t n_steps, const hk_step_io *io, void *stream);

/* Raw state access: state [N,18] f32 (body origins / angles / velocities), aux [N,5] i32 = has_puck1, has_puck2,
 * time, done, winner.  hk_set_state rejects aux rows (of the arenas the mask selects) with has_puck outside
 * [0, 255], done outside {0, 1} or winner outside {-1, 0, 1} with HK_E_INVALID before anything is launched: the
 * arena's int words are packed in HBM (r06; the reference's values are has_puck 0..15, done 0/1, winner -1/0/1).
 * hk_set_state applies pybox2d setter semantics in set_state's order (SetTransform, SetLinearVelocity wakes,
 * ...); a NaN position pair / angle / velocity pair / omega leaves that quantity's setter uncalled (the
 * reference's set_state never assigns the puck's angle or angular velocity, hockey_env.py:594-608). */
int hk_get_state(void *ctx, float *state, int32_t *aux, void *stream);
int hk_set_state(void *ctx, const uint8_t *mask, const float *state, const int32_t *aux, void *stream);

/* BasicOpponent phases ([N,2] f64 device, player 1 / player 2): copied out to phase_out (nullable), then
 * overwritten from phase_in (nullable).  BasicOpponent.__init__ draws U(0, pi) (hockey_env.py:785). */
int hk_opponent_phase(void *ctx, double *phase_out, const double *phase_in, void *stream);

/* All three phase rows ([N,3] f64 device, same copy-out-then-overwrite contract): row 0 player 1's bot, row 1
 * player 2's bot under the context policy (and the strong bot under an io.policy2 override), row 2 player 2's
 * weak bot under an override.  Rule: a step WITH an override walks row 2 for the weak bot and row 1 for the
 * strong bot; a step WITHOUT one walks row 1 for whichever bot the context policy names.  A caller that mixes
 * the two on a context whose player-2 policy is weak therefore splits that bot's phase over rows 1 and 2;
 * the C5 loop (rl/training/opponent_manager.py's mix) passes an override on every step. */
int hk_opponent_phase3(void *ctx, double *phase_out, const double *phase_in, void *stream);

/* Observation of the current state without stepping ([N,18] f32 each, either may be NULL). */
int hk_observe(void *ctx, float *obs, float *obs2, void *stream);

/* Info dicts and rewards of the current state in float64, as the reference computes them (nullable; info
 * [N,4] = {winner, closeness, touch, direction}):
 *   info / info2     replace _get_info / get_info_agent_two            hockey/hockey_env.py:542-591
 *   reward / reward2 replace get_reward(_get_info()) / get_reward_agent_two(get_info_agent_two())  :518-540 */
int hk_info(void *ctx, double *info, double *info2, double *reward, double *reward2, void *stream);

/* counters: out[HK_NUM_COUNTERS] int64 on the HOST (synchronises the stream). */
int hk_counters(void *ctx, int64_t *out, void *stream);
int hk_reset_counters(void *ctx, void *stream);

/* Launch-geometry introspection for the bench roofline (bytes moved per env-step by the step kernel:
 * algorithmic = SURVEY §8(d) accounting; implementation = what the kernel actually reads+writes). */
int hk_bytes_per_step(const void *ctx, int64_t *algorithmic, int64_t *implementation);

#ifdef __cplusplus
}
#endif
#endif
