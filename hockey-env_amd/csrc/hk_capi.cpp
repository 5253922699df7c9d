// hk_capi.cpp -- the extern "C" boundary declared in include/hockey.h.
//
// Owns the per-context device state (SoA arrays in HBM, allocated once at hk_create and sized for the
// whole arena batch), validates arguments, and launches the gfx950 kernels on the caller's stream.
// Errors are reported as negative status codes plus a thread-local message (hk_last_error); no C++
// exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>
#include <string>

#include "../../include/hockey.h"
#include "hk_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, const char *a = "", long long b = 0) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), fmt, a, b);
  g_err = buf;
  return code;
}

int hipfail(hipError_t e, const char *where) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s", where, hipGetErrorString(e));
  g_err = buf;
  return HK_E_HIP;
}

struct Ctx {
  int device = 0;
  hk::DevState s{};
  hk::KCfg cfg{};
  // hk_step_host buffer (allocated on first use): inputs and packed outputs in pinned, mapped, coherent host
  // memory.  The step kernel reads the inputs and writes the outputs through hs_map (its device address), so a
  // step costs one launch and one stream sync, with no copy commands.  HK_STEP_HOST_STAGED=1 selects the staged
  // variant instead (device buffer hs_dev, one H2D and one D2H copy per step) for A/B timing.
  uint8_t *hs_pin = nullptr, *hs_map = nullptr, *hs_dev = nullptr;
  int hs_staged = 0;
  uint64_t hs_seq = 0;  // hk_step_host steps so far (the completion word's expected value)
  // hk_step_host's resident server (mapped variant; HK_STEP_HOST_SERVER=0 launches one step kernel per call
  // instead): it runs on the device's shared server stream (SrvSlot), ordered after the caller's stream when it
  // starts, and every other entry point stops it first (server_stop), so it never runs beside another kernel of
  // this context.
  int srv_on = 0;
  hipEvent_t srv_after = nullptr;
  bool srv_running = false;  // guarded by the device's SrvSlot::mu
  std::chrono::steady_clock::time_point srv_start, srv_last;
  unsigned long long srv_idle_ticks = 0, srv_life_ticks = 0;
};

// the server's own limits (hk_kernels.h HostServer): it exits after kSrvIdleMs without a request or kSrvLifeMs in
// all; the host replaces it before either can fire mid-request (half those times), and relaunches on demand.  The
// idle limit bounds what a resident server can cost other work: a kernel that lands on the server stream's hardware
// queue (streams share the box's 4 queues) or a device-wide synchronise waits for its idle exit.
constexpr int kSrvIdleMs = 4, kSrvLifeMs = 2000;
// the longest a server-path hk_step_host call waits for its answer (the server is ordered after the caller's
// stream, so this also bounds the work queued there before the step); then it fails with HK_E_DEVICE
constexpr int kSrvWaitMs = 10000;

// At most ONE resident step server per device and process: every single-arena context's server runs on
// the device's one server stream, and a context that starts its server first stops the running one of another
// context.  So N facades stepped round-robin cost a server hand-over per step (a quit, a stream sync and a launch:
// tens of microseconds), never a kernel queued behind another context's idle server.  ``mu`` is held for a whole
// server-path hk_step_host call and by server_stop, so a hand-over never interrupts a request in flight on another
// thread.
struct SrvSlot {
  std::mutex mu;
  hipStream_t stream = nullptr;
  Ctx *owner = nullptr;
};
constexpr int kMaxDevices = 64;
SrvSlot &srv_slot(int device) {
  static SrvSlot slots[kMaxDevices];
  return slots[device];
}

// hk_step_host buffer layout per context: inputs [N,8] f32 actions + [N,2] f64 increments, outputs [N] packed
// records of HK_HOST_RECORD_BYTES (obs f32[18], obs2 f32[18], done u8 + 7 pad, record f64[16])
constexpr size_t kHostObs = 0, kHostObs2 = 72, kHostDone = 144, kHostRec = 152;
static_assert(kHostRec + 16 * 8 == HK_HOST_RECORD_BYTES, "hk_step_host record layout");
size_t host_in_bytes(int64_t n) { return (size_t)n * (8 * 4 + 2 * 8); }
constexpr size_t kHostWordBytes = 64;  // the completion word (hk_step_host), on its own 64-B line
// offset of the completion word in the pinned buffer: the inputs and the records, rounded up to a 64-B line; the
// server's request word and its argument words follow on lines of their own
size_t host_word_off(int64_t n) { return (host_in_bytes(n) + (size_t)n * HK_HOST_RECORD_BYTES + 63) & ~(size_t)63; }
size_t host_req_off(int64_t n) { return host_word_off(n) + kHostWordBytes; }
size_t host_args_off(int64_t n) { return host_word_off(n) + 2 * kHostWordBytes; }
size_t host_pin_bytes(int64_t n) { return host_word_off(n) + 3 * kHostWordBytes; }

volatile uint64_t *req_word(Ctx *c) { return reinterpret_cast<volatile uint64_t *>(c->hs_pin + host_req_off(c->s.n)); }

// stop hk_step_host's server (if one runs) and wait for it: every request it was given has been answered (a step
// returns only then), so the next server starts idle.  The caller holds srv_slot(c->device).mu.
hipError_t server_stop_locked(Ctx *c) {
  SrvSlot &slot = srv_slot(c->device);
  if (slot.owner == c) slot.owner = nullptr;
  if (!c->srv_running) return hipSuccess;
  std::atomic_thread_fence(std::memory_order_release);
  *req_word(c) = hk::kServerQuit;
  const hipError_t e = hipStreamSynchronize(slot.stream);
  *req_word(c) = c->hs_seq;
  c->srv_running = false;
  return e;
}
hipError_t server_stop(Ctx *c) {
  if (!c->srv_on) return hipSuccess;  // this context never started a server (srv_on is set by its own thread)
  std::lock_guard<std::mutex> lk(srv_slot(c->device).mu);
  return server_stop_locked(c);
}
#define HK_QUIESCE(c, who)                                               \
  do {                                                                   \
    const hipError_t qe_ = server_stop(c);                               \
    if (qe_ != hipSuccess) return hipfail(qe_, who ": step server");     \
  } while (0)


int check_policy(int p) { return p >= HK_POLICY_EXTERNAL && p <= HK_POLICY_BASIC_STRONG; }

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" {

const char *hk_last_error(void) { return g_err.c_str(); }

const char *hk_version(void) { return "hockey-mi355x 0.2 (gfx950, lane-per-arena step kernel)"; }

int hk_create(int device, int64_t n, const hk_config *cfg, void **out) {
  if (!out) return fail(HK_E_INVALID, "hk_create: out is NULL%s", "");
  *out = nullptr;
  if (n <= 0 || n > (int64_t)1 << 30) return fail(HK_E_INVALID, "hk_create: bad n_arenas %s%lld", "", n);
  if (!cfg) return fail(HK_E_INVALID, "hk_create: cfg is NULL%s");
  if (cfg->mode < 0 || cfg->mode > 2) return fail(HK_E_INVALID, "hk_create: bad mode%s");
  if (!check_policy(cfg->policy[0]) || !check_policy(cfg->policy[1]))
    return fail(HK_E_INVALID, "hk_create: bad policy%s");
  if (cfg->diag_flags & ~HK_DIAG_LARGE_ISLANDS) return fail(HK_E_INVALID, "hk_create: unknown diag_flags%s");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0) return fail(HK_E_DEVICE, "hk_create: no HIP device available%s");
  if (device < 0 || device >= ndev || device >= kMaxDevices)
    return fail(HK_E_DEVICE, "hk_create: device %s%lld out of range", "", device);
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return hipfail(e, "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(HK_E_DEVICE, "hk_create: device arch %s is not gfx950 (MI355X)", prop.gcnArchName);
  DeviceGuard g(device);
  Ctx *c = new Ctx();
  c->device = device;
  c->cfg.keep_mode = cfg->keep_mode ? 1 : 0;
  c->cfg.mode = cfg->mode;
  c->cfg.auto_reset = cfg->auto_reset ? 1 : 0;
  c->cfg.vel_ref = cfg->vel_ref_semantics ? 1 : 0;
  c->cfg.policy[0] = cfg->policy[0];
  c->cfg.policy[1] = cfg->policy[1];
  c->cfg.seed = cfg->seed;
  c->cfg.arena_offset = cfg->arena_offset;
  c->cfg.diag = cfg->diag_flags;
  c->s.n = n;
  const size_t nf = (size_t)hk::NFF * n, ni = (size_t)hk::NPW * n, nm = (size_t)hk::NSOLID * hk::NMF * n;
  const size_t nw = (size_t)hk::workspace_words_per_arena() * n;
  if ((e = hipMalloc(&c->s.f, nf * 4)) != hipSuccess || (e = hipMalloc(&c->s.i, ni * 4)) != hipSuccess ||
      (e = hipMalloc(&c->s.man, nm * 4)) != hipSuccess || (e = hipMalloc(&c->s.phase, 3 * n * 8)) != hipSuccess ||
      (e = hipMalloc(&c->s.ws, nw * 4)) != hipSuccess || (e = hipMalloc(&c->s.counters, HK_NUM_COUNTERS * 8)) != hipSuccess) {
    hk_destroy(c);
    return hipfail(e, "hk_create: hipMalloc");
  }
  if ((e = hipMemset(c->s.counters, 0, HK_NUM_COUNTERS * 8)) != hipSuccess ||
      (e = hipMemset(c->s.man, 0, nm * 4)) != hipSuccess) {
    hk_destroy(c);
    return hipfail(e, "hk_create: hipMemset");
  }
  if ((e = hk::launch_init(c->s, c->cfg, nullptr)) != hipSuccess) {
    hk_destroy(c);
    return hipfail(e, "hk_create: init kernel");
  }
  // HockeyEnv.__init__ ends with reset(one_starts=True) (hockey_env.py:155): device placement
  if ((e = hk::launch_reset(c->s, c->cfg, nullptr, nullptr, nullptr, nullptr, nullptr)) != hipSuccess ||
      (e = hipDeviceSynchronize()) != hipSuccess) {
    hk_destroy(c);
    return hipfail(e, "hk_create: initial reset");
  }
  *out = c;
  return HK_OK;
}

int hk_destroy(void *ctx) {
  if (!ctx) return HK_OK;
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  (void)server_stop(c);  // the shared server stream stays for the process's other contexts
  if (c->srv_after) (void)hipEventDestroy(c->srv_after);
  if (c->s.f) (void)hipFree(c->s.f);
  if (c->s.i) (void)hipFree(c->s.i);
  if (c->s.man) (void)hipFree(c->s.man);
  if (c->s.ws) (void)hipFree(c->s.ws);
  if (c->s.phase) (void)hipFree(c->s.phase);
  if (c->s.counters) (void)hipFree(c->s.counters);
  if (c->hs_dev) (void)hipFree(c->hs_dev);
  if (c->hs_pin) (void)hipHostFree(c->hs_pin);
  delete c;
  return HK_OK;
}

int64_t hk_num_arenas(const void *ctx) { return ctx ? ((const Ctx *)ctx)->s.n : 0; }

int hk_set_policy(void *ctx, int player, int policy) {
  if (!ctx) return fail(HK_E_INVALID, "hk_set_policy: ctx is NULL%s");
  if (player < 0 || player > 1 || !check_policy(policy)) return fail(HK_E_INVALID, "hk_set_policy: bad args%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_set_policy");  // a running server holds the old configuration
  c->cfg.policy[player] = policy;
  return HK_OK;
}

// The packed int words (hk_kernels.h PW_*) hold has_puck in [0, 255], max_t in [0, 65535], done in {0, 1} and
// winner in {-1, 0, 1}: a caller's per-arena values outside those ranges are rejected before anything is launched
// (HK_E_INVALID).  The arrays are device memory; they are copied to the host on the call's stream for the check
// (reset / set_state are not on the step path).  Only arenas the mask selects are checked.
static int check_ints(const char *who, int64_t n, int cols, const int32_t *dev, const uint8_t *mask_dev,
                      hipStream_t st) {
  std::vector<int32_t> v((size_t)n * cols);
  std::vector<uint8_t> m(mask_dev ? (size_t)n : 0);
  hipError_t e = hipMemcpyAsync(v.data(), dev, v.size() * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && mask_dev) e = hipMemcpyAsync(m.data(), mask_dev, m.size(), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hipfail(e, who);
  for (int64_t a = 0; a < n; ++a) {
    if (mask_dev && !m[a]) continue;
    const int32_t *r = v.data() + a * cols;
    if (cols == 1) {
      if (r[0] < 0 || r[0] > hk::kMaxTMax)
        return fail(HK_E_INVALID, "%s: max_t out of range [0, 65535]", who);
      continue;
    }
    if (r[0] < 0 || r[0] > hk::kHasMax || r[1] < 0 || r[1] > hk::kHasMax)
      return fail(HK_E_INVALID, "%s: aux has_puck out of range [0, 255]", who);
    if (r[3] < 0 || r[3] > 1) return fail(HK_E_INVALID, "%s: aux done not 0 or 1", who);
    if (r[4] < -1 || r[4] > 1) return fail(HK_E_INVALID, "%s: aux winner not -1, 0 or 1", who);
  }
  return HK_OK;
}

int hk_reset(void *ctx, const uint8_t *mask, const float *params, const int32_t *max_t, const uint8_t *one_starts,
             void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_reset: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_reset");
  if (max_t) {
    const int rc = check_ints("hk_reset", c->s.n, 1, max_t, mask, (hipStream_t)stream);
    if (rc != HK_OK) return rc;
  }
  hipError_t e = hk::launch_reset(c->s, c->cfg, mask, params, max_t, one_starts, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_reset");
}

static int launch_steps(const char *who, void *ctx, const hk_step_io *io, int nsteps, void *stream) {
  if (!ctx || !io) return fail(HK_E_INVALID, "%s: NULL argument", who);
  if (nsteps < 1) return fail(HK_E_INVALID, "%s: n_steps must be >= 1", who);
  Ctx *c = (Ctx *)ctx;
  if (!io->actions && (c->cfg.policy[0] == HK_POLICY_EXTERNAL || c->cfg.policy[1] == HK_POLICY_EXTERNAL))
    return fail(HK_E_INVALID, "%s: a player takes external actions but io->actions is NULL", who);
  if (io->policy2 && !io->actions)  // an override may pick HK_POLICY_EXTERNAL for any arena
    return fail(HK_E_INVALID, "%s: io->policy2 is given but io->actions is NULL", who);
  hk::StepIO s{};
  s.actions = io->actions;
  s.opp_inc = io->opp_inc;
  s.obs = io->obs;
  s.obs2 = io->obs2;
  s.reward = io->reward;
  s.reward2 = io->reward2;
  s.done = io->done;
  s.info = io->info;
  s.info2 = io->info2;
  s.actions_out = io->actions_out;
  s.debug = io->debug;
  s.final_obs = io->final_obs;
  s.flags = io->flags;
  s.policy2 = io->policy2;
  s.record = io->record;
  DeviceGuard g(c->device);
  {
    const hipError_t qe = server_stop(c);
    if (qe != hipSuccess) return hipfail(qe, who);
  }
  hipError_t e = hk::launch_step(c->s, c->cfg, s, nsteps, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, who);
}

int hk_step(void *ctx, const hk_step_io *io, void *stream) { return launch_steps("hk_step", ctx, io, 1, stream); }

int hk_step_host(void *ctx, const float *actions, const double *opp_inc, int32_t flags, void *out, void *stream) {
  if (!ctx || !out) return fail(HK_E_INVALID, "hk_step_host: NULL argument%s");
  Ctx *c = (Ctx *)ctx;
  if (c->s.n != 1) return fail(HK_E_INVALID, "hk_step_host: only single-arena contexts (n_arenas == 1)%s");
  if (!actions && (c->cfg.policy[0] == HK_POLICY_EXTERNAL || c->cfg.policy[1] == HK_POLICY_EXTERNAL))
    return fail(HK_E_INVALID, "hk_step_host: a player takes external actions but actions is NULL%s");
  DeviceGuard g(c->device);
  const int64_t n = c->s.n;
  const size_t in_b = host_in_bytes(n), out_b = (size_t)n * HK_HOST_RECORD_BYTES;
  hipError_t e = hipSuccess;
  if (!c->hs_pin) {
    const char *v = std::getenv("HK_STEP_HOST_STAGED");
    c->hs_staged = v && v[0] == '1';
    const char *sv = std::getenv("HK_STEP_HOST_SERVER");
    c->srv_on = !c->hs_staged && !(sv && sv[0] == '0');
    if (c->hs_staged && (e = hipMalloc(&c->hs_dev, in_b + out_b)) != hipSuccess)
      return hipfail(e, "hk_step_host: hipMalloc");
    const size_t pin_b = host_pin_bytes(n);
    if ((e = hipHostMalloc(&c->hs_pin, pin_b, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess ||
        (e = hipHostGetDevicePointer((void **)&c->hs_map, c->hs_pin, 0)) != hipSuccess) {
      if (c->hs_pin) (void)hipHostFree(c->hs_pin);
      if (c->hs_dev) (void)hipFree(c->hs_dev);
      c->hs_pin = c->hs_dev = nullptr;
      return hipfail(e, "hk_step_host: hipHostMalloc");
    }
    // pinned memory is not zeroed and small blocks are recycled: a stale completion word equal to the first
    // expected sequence number (1) would end the first wait before the kernel ran
    std::memset(c->hs_pin, 0, pin_b);
    c->hs_seq = 0;
    if (c->srv_on) {
      int khz = 0;
      SrvSlot &slot = srv_slot(c->device);
      {
        std::lock_guard<std::mutex> lk(slot.mu);
        if (!slot.stream && hipStreamCreateWithFlags(&slot.stream, hipStreamNonBlocking) != hipSuccess)
          slot.stream = nullptr;
      }
      if (!slot.stream || (e = hipEventCreateWithFlags(&c->srv_after, hipEventDisableTiming)) != hipSuccess ||
          (e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device)) != hipSuccess || khz <= 0) {
        // no server for this context: its steps take the launch-per-step path (still the GPU kernel)
        if (c->srv_after) (void)hipEventDestroy(c->srv_after);
        c->srv_after = nullptr;
        c->srv_on = 0;
      }
      c->srv_idle_ticks = (unsigned long long)khz * kSrvIdleMs;
      c->srv_life_ticks = (unsigned long long)khz * kSrvLifeMs;
    }
  }
  const hipStream_t st = (hipStream_t)stream;
  const size_t a_b = (size_t)n * 8 * 4, inc_b = (size_t)n * 2 * 8;
  if (c->srv_on) {
    SrvSlot &slot = srv_slot(c->device);
    std::lock_guard<std::mutex> lk(slot.mu);
    // one resident server per device: hand the slot over from another context's server first
    if (slot.owner && slot.owner != c && (e = server_stop_locked(slot.owner)) != hipSuccess)
      return hipfail(e, "hk_step_host: another context's step server");
    // A server that has idled or lived for half its limits may be about to exit on its own: replace it now
    // rather than post a request it could miss (a missed request is still served: see the wait below).
    const auto now = std::chrono::steady_clock::now();
    if (c->srv_running && (now - c->srv_last > std::chrono::microseconds(kSrvIdleMs * 500) ||
                           now - c->srv_start > std::chrono::milliseconds(kSrvLifeMs / 2))) {
      if ((e = server_stop_locked(c)) != hipSuccess) return hipfail(e, "hk_step_host: step server");
    }
    if (actions) std::memcpy(c->hs_pin, actions, a_b);
    if (opp_inc) std::memcpy(c->hs_pin + a_b, opp_inc, inc_b);
    volatile int32_t *args = reinterpret_cast<volatile int32_t *>(c->hs_pin + host_args_off(n));
    args[0] = flags;
    args[1] = actions ? 1 : 0;
    args[2] = opp_inc ? 1 : 0;
    const uint64_t seq = ++c->hs_seq;
    std::atomic_thread_fence(std::memory_order_release);
    *req_word(c) = seq;  // the request: every input word above is written first
    volatile uint64_t *word = reinterpret_cast<volatile uint64_t *>(c->hs_pin + host_word_off(n));
    for (int launches = 0;;) {
      if (!c->srv_running) {
        // start a server, ordered after the work already on the caller's stream (e.g. a reset)
        if (++launches > 2) return fail(HK_E_DEVICE, "hk_step_host: the step server exits without serving%s");
        hk::StepIO s{};
        s.actions = (const float *)c->hs_map;
        s.opp_inc = (const double *)(c->hs_map + a_b);
        uint8_t *o = c->hs_map + in_b;
        s.obs = (float *)(o + kHostObs);
        s.obs2 = (float *)(o + kHostObs2);
        s.done = o + kHostDone;
        s.record = (double *)(o + kHostRec);
        hk::HostServer hs{};
        hs.req = reinterpret_cast<const unsigned long long *>(c->hs_map + host_req_off(n));
        hs.done = reinterpret_cast<unsigned long long *>(c->hs_map + host_word_off(n));
        hs.args = reinterpret_cast<const int32_t *>(c->hs_map + host_args_off(n));
        hs.idle_ticks = c->srv_idle_ticks;
        hs.life_ticks = c->srv_life_ticks;
        if ((e = hipEventRecord(c->srv_after, st)) != hipSuccess ||
            (e = hipStreamWaitEvent(slot.stream, c->srv_after, 0)) != hipSuccess ||
            (e = hk::launch_host_server(c->s, c->cfg, s, hs, slot.stream)) != hipSuccess)
          return hipfail(e, "hk_step_host: server launch");
        c->srv_running = true;
        slot.owner = c;
        c->srv_start = std::chrono::steady_clock::now();
      }
      // Spin on the completion word; every 4096 polls ask the server's stream, so a server that faulted returns
      // its error and one that exited on its own before serving this request is replaced.  The wait is bounded
      // (ADVICE r05): the slot's lock is held here, so a server that never starts (the caller's stream blocked
      // on an event that never fires) must not hold every other facade on this device forever.  Past the deadline
      // the request is withdrawn (the quit word: a server that starts later exits without serving it), the
      // server stays recorded as running, so the next stop of this context waits for its stream, and the call
      // fails with HK_E_DEVICE.
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(kSrvWaitMs);
      uint32_t k = 1;
      for (; *word != seq; ++k) {
        if ((k & 4095u) == 0u) {
          const hipError_t q = hipStreamQuery(slot.stream);
          if (q == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() < deadline) continue;
            std::atomic_thread_fence(std::memory_order_release);
            *req_word(c) = hk::kServerQuit;
            if (*word == seq) break;  // answered while the request was being withdrawn
            return fail(HK_E_DEVICE, "hk_step_host: the step server did not answer within the wait limit "
                                     "(is the calling stream blocked?)%s");
          }
          if (q != hipSuccess) {
            c->srv_running = false;
            slot.owner = nullptr;
            return hipfail(q, "hk_step_host: step server");
          }
          if (*word == seq) break;
          c->srv_running = false;  // exited (idle / life limit) without this request: start another
          slot.owner = nullptr;
          break;
        }
      }
      if (*word == seq) break;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    c->srv_last = std::chrono::steady_clock::now();
    std::memcpy(out, c->hs_pin + in_b, out_b);
    return HK_OK;
  }
  if (actions) std::memcpy(c->hs_pin, actions, a_b);
  if (opp_inc) std::memcpy(c->hs_pin + a_b, opp_inc, inc_b);
  uint8_t *dev = c->hs_staged ? c->hs_dev : c->hs_map;
  if (c->hs_staged && (actions || opp_inc) &&
      (e = hipMemcpyAsync(c->hs_dev, c->hs_pin, in_b, hipMemcpyHostToDevice, st)) != hipSuccess)
    return hipfail(e, "hk_step_host: H2D");
  uint8_t *o = dev + in_b;
  hk::StepIO s{};
  s.actions = actions ? (const float *)dev : nullptr;
  s.opp_inc = opp_inc ? (const double *)(dev + a_b) : nullptr;
  s.obs = (float *)(o + kHostObs);
  s.obs2 = (float *)(o + kHostObs2);
  s.done = o + kHostDone;
  s.record = (double *)(o + kHostRec);
  s.flags = flags;
  // mapped variant: the kernel stores the launch's sequence number into a completion word in the same mapped
  // buffer after its last output store, and the host waits on that word instead of synchronising the stream
  volatile uint64_t *word = reinterpret_cast<volatile uint64_t *>(c->hs_pin + host_word_off(n));
  const uint64_t seq = ++c->hs_seq;
  if (!c->hs_staged) {
    s.done_word = reinterpret_cast<unsigned long long *>(c->hs_map + host_word_off(n));
    s.done_seq = seq;
  }
  if ((e = hk::launch_step(c->s, c->cfg, s, 1, st)) != hipSuccess) return hipfail(e, "hk_step_host: launch");
  if (c->hs_staged) {
    if ((e = hipMemcpyAsync(c->hs_pin + in_b, o, out_b, hipMemcpyDeviceToHost, st)) != hipSuccess)
      return hipfail(e, "hk_step_host: D2H");
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return hipfail(e, "hk_step_host: sync");
  } else {
    // Spin on the word; every 4096 polls ask the stream, so a launch that fails (or never writes the word)
    // returns its error instead of hanging the caller.
    for (uint32_t k = 1; *word != seq; ++k) {
      if ((k & 4095u) == 0u) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipErrorNotReady) continue;
        if (q != hipSuccess) return hipfail(q, "hk_step_host: step kernel");
        if (*word != seq) return fail(HK_E_DEVICE, "hk_step_host: the step finished without its completion word%s");
        break;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  std::memcpy(out, c->hs_pin + in_b, out_b);
  return HK_OK;
}

int hk_rollout(void *ctx, int32_t n_steps, const hk_step_io *io, void *stream) {
  return launch_steps("hk_rollout", ctx, io, n_steps, stream);
}

int hk_get_state(void *ctx, float *state, int32_t *aux, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_get_state: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_get_state");
  hipError_t e = hk::launch_get_state(c->s, c->cfg, state, aux, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_get_state");
}

int hk_set_state(void *ctx, const uint8_t *mask, const float *state, const int32_t *aux, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_set_state: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_set_state");
  if (aux) {
    const int rc = check_ints("hk_set_state", c->s.n, 5, aux, mask, (hipStream_t)stream);
    if (rc != HK_OK) return rc;
  }
  hipError_t e = hk::launch_set_state(c->s, c->cfg, mask, state, aux, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_set_state");
}

int hk_observe(void *ctx, float *obs, float *obs2, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_observe: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_observe");
  hipError_t e = hk::launch_observe(c->s, c->cfg, obs, obs2, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_observe");
}

int hk_info(void *ctx, double *info, double *info2, double *reward, double *reward2, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_info: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_info");
  hipError_t e = hk::launch_info(c->s, c->cfg, info, info2, reward, reward2, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_info");
}

int hk_opponent_phase(void *ctx, double *phase_out, const double *phase_in, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_opponent_phase: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_opponent_phase");
  hipError_t e = hipSuccess;
  // device layout is [3][N] (player-major); the ABI layout is [N,2]
  if (phase_out)
    e = hipMemcpy2DAsync(phase_out, 2 * sizeof(double), c->s.phase, sizeof(double), sizeof(double), c->s.n,
                         hipMemcpyDeviceToDevice, (hipStream_t)stream);
  if (e == hipSuccess && phase_out)
    e = hipMemcpy2DAsync(phase_out + 1, 2 * sizeof(double), c->s.phase + c->s.n, sizeof(double), sizeof(double),
                         c->s.n, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  if (e == hipSuccess && phase_in)
    e = hipMemcpy2DAsync(c->s.phase, sizeof(double), phase_in, 2 * sizeof(double), sizeof(double), c->s.n,
                         hipMemcpyDeviceToDevice, (hipStream_t)stream);
  if (e == hipSuccess && phase_in)
    e = hipMemcpy2DAsync(c->s.phase + c->s.n, sizeof(double), phase_in + 1, 2 * sizeof(double), sizeof(double),
                         c->s.n, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_opponent_phase");
}

int hk_opponent_phase3(void *ctx, double *phase_out, const double *phase_in, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_opponent_phase3: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_opponent_phase3");
  hipError_t e = hipSuccess;
  // device layout is [3][N] (row-major by phase row); the ABI layout is [N,3]
  for (int r = 0; r < 3 && e == hipSuccess && phase_out; ++r)
    e = hipMemcpy2DAsync(phase_out + r, 3 * sizeof(double), c->s.phase + (size_t)r * c->s.n, sizeof(double),
                         sizeof(double), c->s.n, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  for (int r = 0; r < 3 && e == hipSuccess && phase_in; ++r)
    e = hipMemcpy2DAsync(c->s.phase + (size_t)r * c->s.n, sizeof(double), phase_in + r, 3 * sizeof(double),
                         sizeof(double), c->s.n, hipMemcpyDeviceToDevice, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_opponent_phase3");
}

int hk_counters(void *ctx, int64_t *out, void *stream) {
  if (!ctx || !out) return fail(HK_E_INVALID, "hk_counters: NULL argument%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_counters");
  hipError_t e = hipMemcpyAsync(out, c->s.counters, HK_NUM_COUNTERS * 8, hipMemcpyDeviceToHost, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_counters");
}

int hk_reset_counters(void *ctx, void *stream) {
  if (!ctx) return fail(HK_E_INVALID, "hk_reset_counters: ctx is NULL%s");
  Ctx *c = (Ctx *)ctx;
  DeviceGuard g(c->device);
  HK_QUIESCE(c, "hk_reset_counters");
  hipError_t e = hipMemsetAsync(c->s.counters, 0, HK_NUM_COUNTERS * 8, (hipStream_t)stream);
  return e == hipSuccess ? HK_OK : hipfail(e, "hk_reset_counters");
}

int hk_bytes_per_step(const void *ctx, int64_t *algorithmic, int64_t *implementation) {
  if (!ctx) return fail(HK_E_INVALID, "hk_bytes_per_step: ctx is NULL%s");
  // action 32 B + body state 72 B + 4 int32 scalars 16 B read; body state 72 B,
  // scalars 16 B, obs 72 B, reward 4 B, done 1 B written = 285 B per env-step.
  if (algorithmic) *algorithmic = 285;
  // implementation (excluding manifolds, which are only touched where a pair is in contact):
  // f: 29 floats read+write, i: 6 packed int words read+write (r06; 12 before), obs 72 + reward 4 + done 1 + info 16.
  if (implementation) *implementation = (int64_t)(hk::NFF * 4 * 2 + hk::NPW * 4 * 2 + 72 + 4 + 1 + 16);
  return HK_OK;
}

}  // extern "C"
