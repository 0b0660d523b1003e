// Sanitizer driver for the engine's CPU build (test infrastructure, SURVEY §5 "sanitizer host
// build"): host_engine.hip compiled together with this file under AddressSanitizer +
// UndefinedBehaviorSanitizer (host code only; GPU sanitizers are not available on the pool).
// It drives every mhh_* entry point of include/msacl_host.h over all six envs — reset, >1000
// lockstep steps (terminations, truncation at step 1000, autoreset both from the Philox draws and
// from injected reset states), state get/set — and the MSACL target math on ragged shapes,
// plus the error paths. Exit status 0 = clean; a sanitizer report aborts with non-zero.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "msacl_host.h"

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
float frand(float lo, float hi) {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return lo + (hi - lo) * (float)((g_rng >> 11) * (1.0 / 9007199254740992.0));
}

int fails = 0;
void expect(bool ok, const char* what) {
  if (!ok) {
    fprintf(stderr, "FAIL: %s (%s)\n", what, mhh_last_error());
    ++fails;
  }
}

void drive_env(int id, int64_t E) {
  mhh_env_t h = nullptr;
  expect(mhh_env_create(id, E, 1234u + id, &h) == 0 && h, "create");
  if (!h) return;
  mh_env_info_t d;
  expect(mhh_env_info(id, &d) == 0, "info");
  const int D = d.obs_dim, A = d.act_dim;
  std::vector<float> obs(E * D), nxt(E * D), real(E * D), rew(E), act(E * A);
  std::vector<uint8_t> term(E), trunc(E);
  expect(mhh_env_reset(h, nullptr, obs.data()) == 0, "reset");
  int dones = 0;
  for (int t = 0; t < 1010; ++t) {
    for (auto& a : act) a = frand(-1.0f, 1.0f);
    expect(mhh_env_step(h, act.data(), nullptr, nxt.data(), real.data(), rew.data(), term.data(), trunc.data()) == 0,
           "step");
    for (int64_t e = 0; e < E; ++e) dones += term[e] | trunc[e];
  }
  expect(dones >= E, "every env ends an episode within 1010 steps");
  // NULL optional outputs
  expect(mhh_env_step(h, act.data(), nullptr, nxt.data(), nullptr, nullptr, nullptr, nullptr) == 0, "step (no outs)");
  // state round trip, then every env one step before the truncation horizon
  std::vector<float> st(E * d.state_dim);
  std::vector<double> xs(E * (d.xstate_dim > 0 ? d.xstate_dim : 1));
  std::vector<int32_t> steps(E);
  expect(mhh_env_get_state(h, st.data(), xs.data(), steps.data()) == 0, "get_state");
  expect(mhh_env_set_state(h, st.data(), xs.data(), steps.data()) == 0, "set_state");
  for (auto& s : steps) s = d.max_step - 1;
  expect(mhh_env_set_state(h, nullptr, nullptr, steps.data()) == 0, "set_state (steps)");
  expect(mhh_env_step(h, act.data(), nullptr, nxt.data(), real.data(), rew.data(), term.data(), trunc.data()) == 0,
         "step to truncation");
  for (int64_t e = 0; e < E; ++e) expect(trunc[e] || term[e], "step 1000 truncates");
  if (d.reset_dim > 0) {  // injected reset states: a reset and an autoreset from the caller's states
    std::vector<float> rs(E * d.reset_dim);
    for (auto& x : rs) x = frand(-0.5f, 0.5f);
    expect(mhh_env_reset(h, rs.data(), obs.data()) == 0, "reset (injected)");
    expect(mhh_env_step(h, act.data(), rs.data(), nxt.data(), real.data(), rew.data(), term.data(), trunc.data()) == 0,
           "step (injected resets)");
  }
  expect(mhh_env_destroy(h) == 0, "destroy");
}

void drive_msacl(int B, int n, int Dd) {
  const int64_t M = (int64_t)B * n;
  auto vec = [](int64_t k, float lo, float hi) {
    std::vector<float> v(k);
    for (auto& x : v) x = frand(lo, hi);
    return v;
  };
  auto q1 = vec(M, -2, 2), q2 = vec(M, -2, 2), q1t = vec(M, -2, 2), q2t = vec(M, -2, 2), nlp = vec(M, -3, 3);
  auto rew = vec(M, -10, 0), done = vec(M, 0, 1), w = vec(B, 0.2f, 1);
  float la = 0.3f;
  std::vector<float> backup(M), dq1(M), dq2(M), loss(1), td(B);
  expect(mhh_msacl_q_target(q1.data(), q2.data(), q1t.data(), q2t.data(), nlp.data(), rew.data(), done.data(), &la,
                            w.data(), 0.99f, B, n, backup.data(), dq1.data(), dq2.data(), loss.data(), td.data()) == 0,
         "q_target");
  expect(mhh_msacl_q_target(q1.data(), q2.data(), q1t.data(), q2t.data(), nlp.data(), rew.data(), done.data(), &la,
                            nullptr, 0.99f, B, n, backup.data(), nullptr, nullptr, nullptr, nullptr) == 0,
         "q_target (optional outputs)");
  auto lp = vec(M, -3, 1), old = vec(M, -3, 1), V = vec(M, 0, 3), V2 = vec(M, 0, 3);
  auto o = vec(M * Dd, -1, 1), o2 = vec(M * Dd, -1, 1), c = vec(n, 0.5f, 1.5f), lw = vec(n, 0, 0.2f),
       s = vec(n, 0.1f, 1);
  std::vector<float> isc(M), esl(M), ld(B), ll(1), dV(M), dV2(M);
  expect(mhh_msacl_lyapunov(lp.data(), old.data(), V.data(), V2.data(), o.data(), o2.data(), c.data(), lw.data(),
                            s.data(), 1.0f, 2.0f, 1.0f, 10.0f, B, n, Dd, isc.data(), esl.data(), ld.data(), ll.data(),
                            dV.data(), dV2.data()) == 0,
         "lyapunov");
  auto V0 = vec(B, 0, 3), V2b = vec(M, 0, 3), ratio = vec(B, 0.7f, 1.3f);
  std::vector<float> adv_raw(B), adv(B), lp_out(1), dr(B);
  double stats[2];
  expect(mhh_msacl_stability_adv(V0.data(), V2b.data(), lw.data(), s.data(), B, n, adv_raw.data(), stats) == 0,
         "stability_adv");
  if (B >= 2)
    expect(mhh_msacl_ppo_clip(ratio.data(), adv_raw.data(), stats, (double)B, 0.1f, B, adv.data(), lp_out.data(),
                              dr.data()) == 0,
           "ppo_clip");
  float ent;
  float g = 1.0f;
  std::vector<float> dl(M);
  expect(mhh_msacl_policy_loss(q1.data(), q2.data(), nlp.data(), &la, M, lp_out.data(), &ent) == 0, "policy_loss");
  expect(mhh_msacl_policy_loss_backward(q1.data(), q2.data(), &la, &g, M, dq1.data(), dq2.data(), dl.data()) == 0,
         "policy_loss_backward");
  std::vector<float> r0(B), dlp(M);
  expect(mhh_msacl_ratio0(lp.data(), old.data(), B, n, r0.data()) == 0, "ratio0");
  expect(mhh_msacl_ratio0_backward(r0.data(), dr.data(), B, n, dlp.data()) == 0, "ratio0_backward");
}

void error_paths() {
  mhh_env_t h = nullptr;
  mh_env_info_t info;
  expect(mhh_env_info(42, &info) != 0, "unknown env info rejected");
  expect(mhh_env_create(42, 4, 0, &h) != 0 && h == nullptr, "unknown env id rejected");
  expect(mhh_env_create(0, 0, 0, &h) != 0, "zero envs rejected");
  expect(mhh_env_create(0, 4, 0, nullptr) != 0, "null out rejected");
  expect(mhh_env_reset(nullptr, nullptr, nullptr) != 0, "null handle rejected");
  expect(mhh_env_step(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) != 0, "null step");
  expect(mhh_msacl_q_target(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0.99f, 0,
                            0, nullptr, nullptr, nullptr, nullptr, nullptr) != 0,
         "q_target bad args");
  double st[2] = {0, 0};
  float r = 1, a = 0, l, d;
  expect(mhh_msacl_ppo_clip(&r, &a, st, 1.0, 0.1f, 1, &a, &l, &d) != 0, "ppo_clip needs n_total >= 2");
}

}  // namespace

int main() {
  expect(mhh_abi_version() == 1, "abi");
  for (int id = 0; id < 6; ++id) {
    drive_env(id, 1);   // config 1's single env
    drive_env(id, 37);  // ragged batch
  }
  drive_msacl(1, 1, 1);
  drive_msacl(2, 3, 2);
  drive_msacl(37, 20, 12);
  drive_msacl(256, 20, 6);
  error_paths();
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("asan driver: all checks passed\n");
  return 0;
}
