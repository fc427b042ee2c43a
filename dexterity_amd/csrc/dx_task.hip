// dx_task.hip -- batched task logic on the device: the task kernels
// that bracket the step kernel when the task logic is not fused into it (reach, whose
// sampling pass runs between them; or DX_NO_FUSE=1), the MT19937 seeding kernels and the
// bench / RL helpers.  The task logic itself is dx_task.h.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dx_task.h"

__device__ __forceinline__ float urand(uint64_t seed, int env, int episode, int draw) {
  return dx_urand(seed, env, episode, draw);
}
// Seeds every env's two MT19937 streams with seed + env (numpy RandomState(seed + env)
// and np.random.seed(seed + env) of the env's process in the reference); the host passes
// seed + env0 for a shard whose env 0 is the job's env env0.
extern "C" __global__ void dx_mt_seed_kernel(int nenv, uint64_t seed, uint32_t* mt_env, uint32_t* mt_goal) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= nenv) return;
  const uint32_t s = (uint32_t)(seed + (uint64_t)env);
  dx_mt_seed(mt_env, nenv, env, s);
  dx_mt_seed(mt_goal, nenv, env, s);
}

// Reach: env e's RandomState(seed + e) as a contiguous block (state, pos = 624, no
// cached gaussian).
extern "C" __global__ void dx_mtw_seed_kernel(int nenv, uint64_t seed, uint32_t* mt) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= nenv) return;
  uint32_t* s = mt + (size_t)env * DX_MTW_WORDS;
  uint32_t v = (uint32_t)(seed + (uint64_t)env);
  for (int k = 0; k < 624; k++) {
    s[k] = v;
    v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)(k + 1);
  }
  s[624] = 624;
  s[625] = 0;
  s[626] = 0;
  s[627] = 0;
}

extern "C" __global__ void dx_task_pre_kernel(TaskParams P, TaskState S, DevBatch B, const float* qpos0,
                                              const float* action) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= P.nenv) return;
  // action -> ctrl (effectors/mujoco_actuation.py:33; MuJoCo clamps internally)
  if (action)
    for (int i = 0; i < P.nu; i++) B.ctrl[(size_t)env * P.nu + i] = action[(size_t)env * P.nu + i];
  if (task_pre<false>(P, S, B, qpos0, env))
    for (int i = 0; i < P.nu; i++) B.ctrl[(size_t)env * P.nu + i] = 0;  // mj_resetData
}

// One 64-lane wave per env: lane 0 does the bookkeeping, all lanes write the
// observation (coalesced; a thread per env wrote 123 floats 492 B apart).
extern "C" __global__ void dx_task_post_kernel(TaskParams P, TaskState S, DevBatch B) {
  const int env = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (env >= P.nenv) return;
  const bool bad = B.bad && B.bad[env];
  task_post(P, S, B, env, lane, S.skip[env] != 0, bad, B.nstep[env]);
  if (lane == 0 && bad) B.bad[env] = 0;  // consumed (the env's episode ended with it)
}

// Uniform random actions within the actuator ctrlrange: the synthetic agent of
// manipulation_test.py:44-45 (random_state.uniform(spec.minimum, spec.maximum)).
// Keyed by the job-wide env index env0 + env, so a shard draws what the same envs of
// one unsharded batch draw.
extern "C" __global__ void dx_sample_actions_kernel(int nenv, int nu, const float* ctrlrange, uint64_t seed,
                                                    int step, int env0, float* out) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nenv * nu) return;
  int env = t / nu, i = t % nu;
  float u = urand(seed, env0 + env, step, 1000 + i);
  float lo = ctrlrange[2 * i], hi = ctrlrange[2 * i + 1];
  out[t] = lo + (hi - lo) * u;
}

extern "C" __global__ void dx_pack_outputs_kernel(int nenv, int obs_dim, const float* obs, const float* rew,
                                                  const float* disc, const int* st, float* dst) {
  int t = blockIdx.x * blockDim.x + threadIdx.x;
  int w = obs_dim + 3;
  if (t >= nenv * w) return;
  int env = t / w, k = t % w;
  float v;
  if (k < obs_dim) v = obs[(size_t)env * obs_dim + k];
  else if (k == obs_dim) v = rew[env];
  else if (k == obs_dim + 1) v = disc[env];
  else v = (float)st[env];
  dst[t] = v;
}
