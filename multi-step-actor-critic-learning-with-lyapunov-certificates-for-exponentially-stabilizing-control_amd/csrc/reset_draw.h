// reset_draw.h — the six envs' reset distributions as counter-based Philox draws, shared by
// the gfx950 rollout kernels (rollout.hip) and the host engine (host_engine.hip), so a CPU run
// and a GPU run with the same (seed, env, counter) draw the same uniforms.
#pragma once
#include "env_math.h"
#include "philox.h"

namespace mh {

// Uniform draws evaluated like Generator.uniform(low, high) -> float64 -> astype(float32).
MH_HD float uni(double u, float lo, float hi) {
  return (float)((double)lo + ((double)hi - (double)lo) * u);
}

template <class Env>
struct ResetDraw;

template <>
struct ResetDraw<VanderPol> {  // VanderPol.py:79-82, U(-5, 5)^2
  MH_HD static void draw(const Rng& r, float* rs) {
    u32x4 q = r.draw(1);
    rs[0] = uni(u01(q.x), -5.0f, 5.0f);
    rs[1] = uni(u01(q.y), -5.0f, 5.0f);
  }
};
template <>
struct ResetDraw<Pendulum> {  // Pendulum.py:83-86, uniform over the observation box
  MH_HD static void draw(const Rng& r, float* rs) {
    u32x4 q = r.draw(1);
    rs[0] = uni(u01(q.x), Pendulum::obs_lo(0), Pendulum::obs_hi(0));
    rs[1] = uni(u01(q.y), Pendulum::obs_lo(1), Pendulum::obs_hi(1));
  }
};
template <int N>
MH_HD void draw_box(const Rng& r, float* rs, float half) {
  for (int i = 0; i < N; i += 4) {
    u32x4 q = r.draw(1 + i / 4);
    uint32_t v[4] = {q.x, q.y, q.z, q.w};
    for (int j = 0; j < 4 && i + j < N; ++j) rs[i + j] = uni(u01(v[j]), -half, half);
  }
}
template <>
struct ResetDraw<DuctedFan> {  // DuctedFan.py:89-92
  MH_HD static void draw(const Rng& r, float* rs) { draw_box<6>(r, rs, 0.5f); }
};
template <>
struct ResetDraw<TwoLink> {  // TwoLink.py:81-84
  MH_HD static void draw(const Rng& r, float* rs) { draw_box<4>(r, rs, 0.5f); }
};
template <>
struct ResetDraw<SingleTrackCar> {  // SingleTrackCar.py:121-124
  MH_HD static void draw(const Rng& r, float* rs) { draw_box<7>(r, rs, 0.5f); }
};
template <>
struct ResetDraw<QuadTracking> {  // QuadTracking.py:169-186
  MH_HD static void draw(const Rng& r, float* rs) {
    u32x4 q0 = r.draw(1), q1 = r.draw(2), q2 = r.draw(3);
    const uint32_t v[12] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
    for (int i = 0; i < 6; ++i) rs[i] = uni(u01(v[i]), -0.01f, 0.01f);       // x, v
    for (int i = 0; i < 3; ++i) rs[15 + i] = uni(u01(v[6 + i]), -0.01f, 0.01f);  // Omega
    float nz[4];
    r.normal4f(4, nz);
    // scipy Rotation.from_rotvec(rv).as_matrix() via the unit quaternion, in float32 (the reset
    // draw itself is distribution-matched, not sample-matched, so f32 rounding is immaterial)
    const float rv[3] = {nz[0] * 0.01f, nz[1] * 0.01f, nz[2] * 0.01f};  // rotvec ~ N(0, 0.01^2)
    const float th = sqrtf(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]);
    float sh, ch;
    sincosf(0.5f * th, &sh, &ch);
    const float sc = th <= 1e-3f ? 0.5f - th * th / 48.0f : sh / th;
    const float x = sc * rv[0], y = sc * rv[1], z = sc * rv[2], w = ch;
    const float Rm[9] = {1 - 2 * (y * y + z * z), 2 * (x * y - z * w),     2 * (x * z + y * w),
                         2 * (x * y + z * w),     1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
                         2 * (x * z - y * w),     2 * (y * z + x * w),     1 - 2 * (x * x + y * y)};
    for (int i = 0; i < 9; ++i) rs[6 + i] = Rm[i];
  }
};

}  // namespace mh
