// hk_kernels.h -- host/device shared declarations: HBM state layout and kernel launchers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hk_core.h"

namespace hk {

// per dynamic body float fields (f[b*FB + k][N])
enum { FB_PX = 0, FB_PY, FB_CX, FB_CY, FB_A, FB_VX, FB_VY, FB_W, FB_SLEEP, FB };
enum { F_PFX = 3 * FB, F_PFY, NFF };
// int fields: the 12 logical words a lane works with (registers) ...
enum { I_AWAKE = 0, I_HAS1, I_HAS2, I_TIME, I_DONE, I_WINNER, I_MAXT, I_TOUCH, I_ENABLED, I_ONE, I_EPISODE, I_STEP, NIF };
// ... and the 6 packed words they live in in HBM (r06, VERDICT r05 item 6: 48 -> 24 B read per arena-step):
//   PW_TAW  touching mask (27 pairs) | awake bits << 27 | done << 30 | one_starts << 31
//   PW_ENW  enabled mask (27 pairs) | (winner + 1) << 27
//   PW_HM   has_puck1 | has_puck2 << 8 | max_t << 16       (has_puck in [0, 255], max_t in [0, 65535])
//   PW_TIME, PW_EPISODE, PW_STEP: whole words
// hk_set_state / hk_reset reject aux / max_t values outside these ranges with HK_E_INVALID (include/hockey.h).
enum { PW_TAW = 0, PW_ENW, PW_HM, PW_TIME, PW_EPISODE, PW_STEP, NPW };
constexpr int kHasMax = 255, kMaxTMax = 65535;
HK_DEV void unpack_ints(const uint32_t (&p)[NPW], int32_t (&iw)[NIF]) {
  iw[I_TOUCH] = (int32_t)(p[PW_TAW] & 0x07ffffffu);
  iw[I_AWAKE] = (int32_t)((p[PW_TAW] >> 27) & 7u);
  iw[I_DONE] = (int32_t)((p[PW_TAW] >> 30) & 1u);
  iw[I_ONE] = (int32_t)(p[PW_TAW] >> 31);
  iw[I_ENABLED] = (int32_t)(p[PW_ENW] & 0x07ffffffu);
  iw[I_WINNER] = (int32_t)((p[PW_ENW] >> 27) & 3u) - 1;
  iw[I_HAS1] = (int32_t)(p[PW_HM] & 0xffu);
  iw[I_HAS2] = (int32_t)((p[PW_HM] >> 8) & 0xffu);
  iw[I_MAXT] = (int32_t)(p[PW_HM] >> 16);
  iw[I_TIME] = (int32_t)p[PW_TIME];
  iw[I_EPISODE] = (int32_t)p[PW_EPISODE];
  iw[I_STEP] = (int32_t)p[PW_STEP];
}
HK_DEV void pack_ints(const int32_t (&iw)[NIF], uint32_t (&p)[NPW]) {
  p[PW_TAW] = ((uint32_t)iw[I_TOUCH] & 0x07ffffffu) | (((uint32_t)iw[I_AWAKE] & 7u) << 27) |
              (((uint32_t)iw[I_DONE] & 1u) << 30) | (((uint32_t)iw[I_ONE] & 1u) << 31);
  p[PW_ENW] = ((uint32_t)iw[I_ENABLED] & 0x07ffffffu) | (((uint32_t)(iw[I_WINNER] + 1) & 3u) << 27);
  p[PW_HM] = ((uint32_t)iw[I_HAS1] & 0xffu) | (((uint32_t)iw[I_HAS2] & 0xffu) << 8) |
             (((uint32_t)iw[I_MAXT] & 0xffffu) << 16);
  p[PW_TIME] = (uint32_t)iw[I_TIME];
  p[PW_EPISODE] = (uint32_t)iw[I_EPISODE];
  p[PW_STEP] = (uint32_t)iw[I_STEP];
}
// manifold record per (solid pair, arena): 16 words = 64 B, read / written as four 16-B quads
//   q0 {meta, local normal x, y, local point x}   q1 {local point y, point0 x, y, point1 x}
//   q2 {point1 y, id0, id1, pad}                  q3 {normal impulse 0, tangent impulse 0, normal 1, tangent 1}
enum { M_META = 0, M_LNX, M_LNY, M_LPX, M_LPY, M_P0X, M_P0Y, M_P1X, M_P1Y, M_P0ID, M_P1ID, M_PAD, M_P0NI, M_P0TI,
       M_P1NI, M_P1TI, NMF };
static_assert(NMF == 16, "a manifold record is four 16-byte quads");

struct DevState {
  float *f;
  int32_t *i;  // packed int words [NPW][N] (PW_*)
  float *man;  // manifold records [NSOLID][N][NMF] (64 B per record, hk_arena.h ManRec)
  float *ws;  // large-island slot workspace [kBigC][kSlotWords][N] (hk_solver.h HbmSlots)
  double *phase;  // BasicOpponent phases [3][N]: player 1, player 2 (its policy / the strong bot under a
                  // per-arena override), player 2's weak bot under an override (hk_step_io.policy2)
  unsigned long long *counters;
  int64_t n;
};

struct KCfg {
  int keep_mode, mode, auto_reset, vel_ref;
  int policy[2];
  uint64_t seed;
  int64_t arena_offset;
  int diag;  // hk_config.diag_flags (HK_DIAG_*): bit0 routes every solve through the HBM slot file; 0 in product
};

struct StepIO {
  const float *actions;
  const double *opp_inc;
  float *obs, *obs2, *reward, *reward2;
  uint8_t *done;
  float *info, *info2, *actions_out, *debug, *final_obs;
  int flags;
  const uint8_t *policy2;  // per-arena player-2 policy override (hk_step_io.policy2) or nullptr
  double *record;          // [N,16] f64 step record (hk_step_io.record) or nullptr
  // hk_step_host only: after every output of the launch is written, arena 0's lane stores done_seq here
  // (release at system scope), so the host can wait on this word instead of a stream synchronisation
  unsigned long long *done_word;
  unsigned long long done_seq;
};

// hk_step_host's resident server (single-arena contexts): one wave stays on the GPU and serves step requests
// posted in the context's mapped host buffer, so a step costs no launch.  Protocol (hk_capi.cpp hk_step_host):
// the host writes the inputs and `args`, then the sequence number into `req` (release); the server sees
// req != its last served number (acquire at system scope), runs the step with args' flags / input pointers,
// writes the outputs and then the sequence number into `done` (release).  The server exits when `req` holds
// kServerQuit, after idle_ticks of wall clock with no request, or after life_ticks in all -- every wave reaches
// an exit, and the host relaunches a server on demand.
constexpr unsigned long long kServerQuit = ~0ull;
struct HostServer {
  const unsigned long long *req;
  unsigned long long *done;
  const int32_t *args;  // [0] HK_STEP_* flags, [1] actions given, [2] phase increments given
  unsigned long long idle_ticks, life_ticks;  // s_memrealtime (wall-clock counter) ticks
};

hipError_t launch_init(const DevState &s, const KCfg &cfg, hipStream_t st);
hipError_t launch_host_server(const DevState &s, const KCfg &cfg, const StepIO &io, const HostServer &hs,
                              hipStream_t st);
hipError_t launch_reset(const DevState &s, const KCfg &cfg, const uint8_t *mask, const float *params,
                        const int32_t *max_t, const uint8_t *one, hipStream_t st);
hipError_t launch_step(const DevState &s, const KCfg &cfg, const StepIO &io, int nsteps, hipStream_t st);
hipError_t launch_observe(const DevState &s, const KCfg &cfg, float *obs, float *obs2, hipStream_t st);
hipError_t launch_info(const DevState &s, const KCfg &cfg, double *info, double *info2, double *reward,
                       double *reward2, hipStream_t st);
hipError_t launch_get_state(const DevState &s, const KCfg &cfg, float *state, int32_t *aux, hipStream_t st);
hipError_t launch_set_state(const DevState &s, const KCfg &cfg, const uint8_t *mask, const float *state,
                            const int32_t *aux, hipStream_t st);
int64_t workspace_words_per_arena();

// host-side scene construction (hk_scene.cpp): Box2D 2.3 hull / normals / mass data of hockey_env.py's
// fixtures, and the canonical contact pair table.  Run at build time by hk_scene_gen.cpp, whose output
// (hk_scene_data.inc) is the kernels' compile-time scene.
void build_scene(Scene &sc);

}  // namespace hk
