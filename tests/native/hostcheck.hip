// hostcheck.hip — TEST INFRASTRUCTURE: compiles the product's env_math.h (the exact source the
// gfx950 rollout kernel inlines) for the HOST so the CPU test-suite can check the kernel math
// against the golden fixtures in a container without a GPU. Not part of the product library.
#include <vector>

#include "env_math.h"

namespace {
std::vector<double> g_tab;
const double* quad_tab() {
  if (g_tab.empty()) {
    g_tab.resize((size_t)(mh::MAX_STEP + 1) * mh::QT_ROW);
    mh::quad_fill_table(g_tab.data(), mh::MAX_STEP + 1);
  }
  return g_tab.data();
}

template <class Env>
void step_all(int64_t n, float* state, double* xstate, const int32_t* steps, const float* act, float* obs,
              float* rew) {
  for (int64_t e = 0; e < n; ++e) {
    double xs[Env::XS > 0 ? Env::XS : 1];
    for (int i = 0; i < Env::XS; ++i) xs[i] = xstate[e * Env::XS + i];
    Env::step(state + e * Env::S, xs, steps[e], act + e * Env::A, quad_tab(), obs + e * Env::D, rew + e);
    for (int i = 0; i < Env::XS; ++i) xstate[e * Env::XS + i] = xs[i];
  }
}
template <class Env>
void reset_all(int64_t n, const float* rs, float* state, double* xstate, float* obs) {
  for (int64_t e = 0; e < n; ++e) {
    double xs[Env::XS > 0 ? Env::XS : 1];
    Env::reset_from(rs + e * Env::RS, state + e * Env::S, xs, quad_tab(), obs + e * Env::D);
    for (int i = 0; i < Env::XS; ++i) xstate[e * Env::XS + i] = xs[i];
  }
}
}  // namespace

extern "C" {
// the kernel's powf(x, 2) restatement (fast exact-square path + glibc table path)
void mhc_powf2(int64_t n, const float* x, float* out) {
  for (int64_t i = 0; i < n; ++i) out[i] = mh::powf2(x[i]);
}

int mhc_env_step(int env_id, int64_t n, float* state, double* xstate, const int32_t* steps, const float* act,
                 float* obs, float* rew) {
  switch (env_id) {
    case 0: step_all<mh::VanderPol>(n, state, xstate, steps, act, obs, rew); return 0;
    case 1: step_all<mh::Pendulum>(n, state, xstate, steps, act, obs, rew); return 0;
    case 2: step_all<mh::DuctedFan>(n, state, xstate, steps, act, obs, rew); return 0;
    case 3: step_all<mh::TwoLink>(n, state, xstate, steps, act, obs, rew); return 0;
    case 4: step_all<mh::SingleTrackCar>(n, state, xstate, steps, act, obs, rew); return 0;
    case 5: step_all<mh::QuadTracking>(n, state, xstate, steps, act, obs, rew); return 0;
  }
  return -1;
}
int mhc_env_reset(int env_id, int64_t n, const float* rs, float* state, double* xstate, float* obs) {
  switch (env_id) {
    case 0: reset_all<mh::VanderPol>(n, rs, state, xstate, obs); return 0;
    case 1: reset_all<mh::Pendulum>(n, rs, state, xstate, obs); return 0;
    case 2: reset_all<mh::DuctedFan>(n, rs, state, xstate, obs); return 0;
    case 3: reset_all<mh::TwoLink>(n, rs, state, xstate, obs); return 0;
    case 4: reset_all<mh::SingleTrackCar>(n, rs, state, xstate, obs); return 0;
    case 5: reset_all<mh::QuadTracking>(n, rs, state, xstate, obs); return 0;
  }
  return -1;
}
void mhc_quad_table(double* out) {
  const double* t = quad_tab();
  for (size_t i = 0; i < g_tab.size(); ++i) out[i] = t[i];
}
int mhc_np_sum12(const float* a, float* out) { *out = mh::np_sum<12>(a); return 0; }
int mhc_polar3(const float* in, float* out) { mh::polar3(in, out); return 0; }
}
