// Sanitizer build of the CPU-side code (ASan/UBSan on host code): the oracle (oracle/hk_oracle.c)
// and the kernel's per-lane source compiled for the host (hostcheck), both under
// -fsanitize=address,undefined, stepped in lockstep over every mode and policy kind.  Test infrastructure
// only; tests/test_sanitize.py builds and runs it (make -C tests/sanitize).  Exit status 0 = no sanitizer
// report and every step bit-identical; GPU code is not sanitized (GPU ASan is not available on the pool).
#include "../../hockey-env_amd/csrc/hostcheck/hk_hostcheck.cpp"

extern "C" {
#include "../../oracle/hk_oracle.h"
}

#include <cstdio>
#include <random>

static const int kPol[][2] = {{3, 3}, {1, 1}, {0, 2}, {2, 0}};

int main() {
  int bad = 0;
  for (int mode = 0; mode < 3; ++mode) {
    for (const auto &pol : kPol) {
      const int64_t n = 48;
      const int cfg7[7] = {1, mode, 1, 0, pol[0], pol[1], 0};
      const int32_t cfg6[6] = {1, mode, 1, 0, pol[0], pol[1]};
      void *h = hkh_create(n, cfg7, 11 + mode, 100);
      hkh_reset(h, nullptr, nullptr, nullptr, nullptr);
      hkov *v = hkov_create(n, cfg6, 11 + mode, 100);
      std::mt19937 rng(mode * 10 + pol[0]);
      std::uniform_real_distribution<float> U(-1.2f, 1.2f);
      std::vector<float> act(n * 8), o1(n * 18), o2(n * 18), r1(n), r2(n), i1(n * 4), i2(n * 4), fo1(n * 18),
          fo2(n * 18);
      std::vector<uint8_t> d1(n), d2(n), p2(n);
      for (int t = 0; t < 260; ++t) {
        for (auto &x : act) x = U(rng);
        for (auto &x : p2) x = (uint8_t)(rng() % 3 == 0 ? 0 : 2 + rng() % 2);
        const uint8_t *mix = (t % 2) ? p2.data() : nullptr;
        StepIO io{};
        io.actions = act.data();
        io.obs = o1.data();
        io.reward = r1.data();
        io.done = d1.data();
        io.info = i1.data();
        io.final_obs = fo1.data();
        io.policy2 = mix;
        hkh_step(h, &io);
        hkov_step(v, act.data(), nullptr, o2.data(), nullptr, r2.data(), nullptr, d2.data(), i2.data(), nullptr,
                  nullptr, fo2.data(), mix);
        if (memcmp(o1.data(), o2.data(), o1.size() * 4) || memcmp(r1.data(), r2.data(), r1.size() * 4) ||
            memcmp(d1.data(), d2.data(), d1.size()) || memcmp(i1.data(), i2.data(), i1.size() * 4) ||
            memcmp(fo1.data(), fo2.data(), fo1.size() * 4)) {
          std::printf("mismatch: mode %d policies %d/%d step %d\n", mode, pol[0], pol[1], t);
          ++bad;
          break;
        }
      }
      hkh_destroy(h);
      hkov_destroy(v);
    }
  }
  std::printf("sanitized lockstep: %s\n", bad ? "MISMATCH" : "ok");
  return bad ? 1 : 0;
}
