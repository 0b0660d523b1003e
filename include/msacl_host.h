/*
 * msacl_host.h — C ABI of the engine's CPU build (libmsacl_host.so, csrc/host_engine.hip):
 * BASELINE.json config 1 ("VanderPol, 1 env, MSACL off_serial_trainer on CPU reference sampler
 * (plumbing, no GPU)"). Same env math (env_math.h), reset distributions and Philox streams
 * (reset_draw.h) as the gfx950 library; every pointer is a HOST pointer; calls run synchronously
 * on the calling thread. Error codes and env ids are those of msacl_hip.h.
 *
 * It is selected explicitly (device="cpu" in the Python layer); the GPU path never routes
 * through it.
 */
#ifndef MSACL_HOST_H
#define MSACL_HOST_H

#include <stdint.h>

#include "msacl_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void* mhh_env_t;

int mhh_abi_version(void);
const char* mhh_last_error(void);

/* The env's spaces and dims (what init_args reads, RL/utils/init_args.py:33-46), as mh_env_info */
int mhh_env_info(int32_t env_id, mh_env_info_t* out);

/* gym.vector.SyncVectorEnv([make_env(env_id, ...)] * num_envs) on the host
 * (RL/create_pkg/create_envs.py:24-32, RL/env/make_env.py:10-41); resets draw from the env's
 * reset distribution with Philox keyed by (seed, env index, per-env counter), as the device. */
int mhh_env_create(int32_t env_id, int64_t num_envs, uint64_t seed, mhh_env_t* out);
int mhh_env_destroy(mhh_env_t h);
/* env.reset() of every env (reset_states: [E][reset_dim] injected start states, or NULL) */
int mhh_env_reset(mhh_env_t h, const float* reset_states, float* obs);
/* SyncVectorEnv.step (gymnasium 0.28.1): env.step of every env (RL/env/<Name>.py step), then
 * autoreset of finished envs; real_next_obs = the pre-reset observation (info["final_observation"]
 * rows), reward = the env's float reward; reset_states as in mhh_env_reset. */
int mhh_env_step(mhh_env_t h, const float* act, const float* reset_states, float* next_obs, float* real_next_obs,
                 float* reward, uint8_t* terminated, uint8_t* truncated);
int mhh_env_get_state(mhh_env_t h, float* state, double* xstate, int32_t* steps);
int mhh_env_set_state(mhh_env_t h, const float* state, const double* xstate, const int32_t* steps);

/* MSACL target / certificate math (RL/algorithm/msacl.py), the host twins of mh_msacl_* in
 * msacl_hip.h (same arguments minus the stream): */
int mhh_msacl_q_target(const float* q1, const float* q2, const float* q1t, const float* q2t, const float* next_logp,
                       const float* rew, const float* done, const float* log_alpha, const float* weight, float gamma,
                       int32_t B, int32_t n, float* backup, float* dq1, float* dq2, float* loss_out, float* abs_td);
int mhh_msacl_lyapunov(const float* logp, const float* old_logp, const float* lya_obs, const float* lya_obs2,
                       const float* obs, const float* obs2, const float* c, const float* w, const float* s,
                       float alpha1, float alpha2, float pos_scale, float diff_scale, int32_t B, int32_t n, int32_t D,
                       float* is_clip, float* esl, float* lya_diff, float* loss_out, float* d_lya_obs,
                       float* d_lya_obs2);
int mhh_msacl_stability_adv(const float* lya_obs0, const float* lya_obs2, const float* w, const float* s, int32_t B,
                            int32_t n, float* adv_raw, double* stats_out);
int mhh_msacl_ppo_clip(const float* ratio, const float* adv_raw, const double* stats, double n_total, float clip_eps,
                       int32_t B, float* adv, float* loss_out, float* d_ratio);
int mhh_msacl_policy_loss(const float* q1, const float* q2, const float* logp, const float* log_alpha, int64_t N,
                          float* loss_out, float* entropy_out);
int mhh_msacl_policy_loss_backward(const float* q1, const float* q2, const float* log_alpha, const float* g_loss,
                                   int64_t N, float* dq1, float* dq2, float* dlogp);
int mhh_msacl_ratio0(const float* logp_new, const float* old_logp, int32_t B, int32_t n, float* ratio_out);
int mhh_msacl_ratio0_backward(const float* ratio, const float* g_ratio, int32_t B, int32_t n, float* d_logp_new);

#ifdef __cplusplus
}
#endif

#endif /* MSACL_HOST_H */
