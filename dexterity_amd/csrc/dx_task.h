// dx_task.h -- the per-env task logic as device functions.
//
// The reference runs these per environment in Python around every control step
// (composer hooks):
//   GoalTask.before_step       task.py:154-165   goal change after >5 successes
//   GoalTask.after_step        task.py:167-185   distance, success counters, per-goal timeout
//   ReOrient.after_step        reorient.py:201-209 + _is_prop_fallen :229-235
//   should_terminate_episode   task.py:187-193, reorient.py:211-213
//   get_discount               task.py:195-204, reorient.py:222-225
//   get_reward                 reorient.py:215-220 -> _get_shaped_reorientation_reward :238-284
//   observables                dexterous_hand.py:250-310 (sin/cos, qvel, fingertip pos/vel),
//                              prop pose sensors, goal task.py:207-216
//   initialize_episode         reorient.py:182-188 (PropPlacer bbox :70-78, UniformQuaternion goal)
// task_pre (before_step / initialize_episode) and task_post (after_step, reward, discount,
// termination, observation) run either as the two small kernels of dx_task.hip around the
// step kernel, or fused into the step kernel itself (dx_step.hip, DevBatch::fuse): task_pre
// in the first physics-step task of the env, task_post in its last, so a control step is
// one step-kernel launch plus the overflow tier's.
//
// dm_env semantics: after a LAST step the next step() of that env resets it and returns
// FIRST (composer.Environment.step), done by task_pre + the physics kernel's skip mask.
#pragma once
#include "dx_internal.h"

enum { TS_FIRST = 0, TS_MID = 1, TS_LAST = 2 };  // dm_env StepType

// Stores of task state.  Plain in the task kernels (the next kernel sees them).  Fused
// into the step kernel, what task_pre writes is read by the env's later tasks, which may
// run on another XCD: those stores are write-through (sc1), the substep queue's hand-off
// form (cdna_hip_programming.md Guideline 16 R1; the consumer task acquires before its
// loads).  The array base is wave-uniform, the element offset per lane.
template <bool WT>
struct TaskStore {
  template <class T>
  __device__ static __forceinline__ void st(T* base, size_t i, T v) {
    if constexpr (!WT) {
      base[i] = v;
    } else {
      const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
      if constexpr (sizeof(T) == 8) {
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 d = {(unsigned)u, (unsigned)(u >> 32)};
        __builtin_amdgcn_raw_buffer_store_b64(d, rsrc, (int)(i * 8), 0, 16);
      } else {
        unsigned u;
        __builtin_memcpy(&u, &v, 4);
        __builtin_amdgcn_raw_buffer_store_b32(u, rsrc, (int)(i * 4), 0, 16);
      }
    }
  }
};

// orientation distance || axisangle(quat_diff_active(cur, goal)) || = 2 acos(|<goal, cur>|)
// (prop_orientation.py:40-50, [3P] dm_robotics quat_diff_active / quat_to_axisangle)
__device__ __forceinline__ float quat_distance(const float* g, const float* c) {
  float n = sqrtf(c[0] * c[0] + c[1] * c[1] + c[2] * c[2] + c[3] * c[3]);
  float d = fabsf(g[0] * c[0] + g[1] * c[1] + g[2] * c[2] + g[3] * c[3]) / fmaxf(n, 1e-20f);
  return 2.0f * acosf(fminf(1.0f, d));
}

// tanh_squared(x, margin, 0.95) of manipulation/shared/rewards.py:18-28
__device__ __forceinline__ float tanh_squared(float x, float margin) {
  const float w = 2.178272210300875f / margin;  // arctanh(sqrt(0.95))
  float t = tanhf(w * x);
  return t * t;
}

// Uniform random actions within the actuator ctrlrange: the synthetic agent of
// manipulation_test.py:44-45 (random_state.uniform(spec.minimum, spec.maximum)), keyed by
// (seed, job-wide env, step, actuator).
__device__ __forceinline__ float random_action(const float* ctrlrange, uint64_t seed, int genv, int step, int i) {
  const float u = dx_urand(seed, genv, step, 1000 + i);
  const float lo = ctrlrange[2 * i], hi = ctrlrange[2 * i + 1];
  return lo + (hi - lo) * u;
}

// before_step / initialize_episode of one env (one thread).  The action is already in
// B.ctrl; a reset zeroes ctrl (mj_resetData), which the caller does (the return value).
// Returns 1 when the env was (re)initialised: it is observed only this step (S.skip).
template <bool WT>
__device__ __forceinline__ int task_pre(const TaskParams& P, const TaskState& S, const DevBatch& B,
                                        const float* qpos0, int env) {
  using W = TaskStore<WT>;
  const int st = S.step_type[env];
  if (st == TS_LAST || S.episode[env] < 0) {
    // initialize_episode from a reset physics state (mj_resetData)
    S.episode[env] = S.episode[env] + 1;  // (read only by later task_pre calls)
    float* q = B.qpos + (size_t)env * P.nq;
    for (int i = 0; i < P.nq; i++) q[i] = qpos0[i];
    for (int i = 0; i < P.nv; i++) {
      B.qvel[(size_t)env * P.nv + i] = 0;
      B.qacc_ws[(size_t)env * P.nv + i] = 0;
    }
    B.time[env] = 0;
    if (B.nstep) B.nstep[env] = 0;
    if (P.kind != DX_KIND_REACH) {
      // reorient.py:182-188 in the reference's draw order: the goal first
      // (GoalTask.initialize_episode, task.py:137-152 -> PropOrientation.next_goal,
      // prop_orientation.py:34-38, whose sampler gets the RandomState positionally
      // and so draws from numpy's global stream), then PropPlacer (reorient.py:143-151)
      // on the env's RandomState: position uniform in the bbox (3 draws), then a
      // uniform quaternion (3 draws).  A spawn never touches the hand (the box is above
      // it, tests/test_host_logic.py), so PropPlacer's first attempt is always kept.
      float g[4];
      if (P.kind == DX_KIND_HANDOVER) {  // the cube spawns over the first hand, handed to the second
        for (int k = 0; k < 3; k++) g[k] = P.hand_target[1][k];
        g[3] = 1.f;
      } else {
        dx_mt_uniform_quat(S.mt_goal, P.nenv, env, g);
      }
      for (int k = 0; k < 4; k++) W::st(S.goal, (size_t)P.goal_dim * env + k, g[k]);
      if (P.prop_qadr >= 0) {
        uint32_t w[12];  // position (3 doubles) then the quaternion (3 doubles), one fetch
        dx_mt_take<12>(S.mt_env, P.nenv, env, w);
        for (int k = 0; k < 3; k++)
          // random_uniform: low + (high - low) * u, rounded as numpy does (no fma)
          q[P.prop_qadr + k] = (float)__dadd_rn(P.bbox_lo_d[k], __dmul_rn(P.bbox_hi_d[k] - P.bbox_lo_d[k],
                                                                          dx_mt_double2(w[2 * k], w[2 * k + 1])));
        dx_mt_quat_from(w + 6, q + P.prop_qadr + 3);
      }
    } else {
      // reach.py:155-168: fingertip goal (physics rollouts) and collision-free joint
      // angles, both drawn by the sampling pass of the step kernel (mode 2)
      S.need[env] = 3;
      S.goalnum[env] = 0;
    }
    W::st(S.successes, env, 0);
    W::st(S.counter, env, 0);
    W::st(S.registered, env, 0);
    W::st(S.exceeded, env, 0);
    W::st(S.failure, env, 0);
    W::st(S.solve_start, env, 0.f);
    W::st(S.time_d, env, 0.0);
    W::st(S.nsub_d, env, 0);
    W::st(S.solve_start_d, env, 0.0);
    W::st(S.solve_n, env, -1);
    W::st(S.skip, env, 1);
    return 1;
  }
  W::st(S.skip, env, 0);
  // GoalTask.before_step (task.py:154-165)
  if (S.counter[env] > P.steps_before_change) {
    if (P.kind != DX_KIND_REACH) {
      float g[4];
      if (P.kind == DX_KIND_HANDOVER) {  // the goal switches to the other hand: the cube goes back
        const int h = S.goal[(size_t)P.goal_dim * env + 3] > 0.5f ? 0 : 1;
        for (int k = 0; k < 3; k++) g[k] = P.hand_target[h][k];
        g[3] = (float)h;
      } else {
        dx_mt_uniform_quat(S.mt_goal, P.nenv, env, g);  // numpy's global stream
      }
      for (int k = 0; k < 4; k++) W::st(S.goal, (size_t)P.goal_dim * env + k, g[k]);
      W::st(S.counter, env, 0);
      W::st(S.exceeded, env, 0);
      W::st(S.solve_start, env, B.time[env]);
      W::st(S.solve_start_d, env, S.time_d[env]);
      W::st(S.registered, env, 0);
    } else {
      S.need[env] = 1;  // next_goal and the bookkeeping run in the sampling pass
    }
  }
  return 0;
}

// after_step, reward, discount, termination and the observation of one env, by one
// 64-lane wave (lane 0 the bookkeeping, every lane the observation).  `skip`: the env
// was reset by this step's task_pre (FIRST); `bad`: a physics step diverged and reset
// the env (dx_step.hip health_check); `nsteps`: physics steps since the episode's
// mj_resetData (fp64 time below).  Reads the env's physics outputs from the batch.
__device__ __forceinline__ void task_post(const TaskParams& P, const TaskState& S, const DevBatch& B, int env,
                                          int lane, bool skip, bool bad, int nsteps) {
  const float* q = B.qpos + (size_t)env * P.nq;
  const float* v = B.qvel + (size_t)env * P.nv;
  const float* g = S.goal + P.goal_dim * env;
  const bool reach = P.kind == DX_KIND_REACH;
  float cur[4] = {1, 0, 0, 0};
  if (P.prop_qadr >= 0)
    for (int k = 0; k < 4; k++) cur[k] = q[P.prop_qadr + 3 + k];
  // goal distance: orientation (prop_orientation.py:40-50) or per-fingertip
  // Cartesian distances (fingertip_position.py:127-137)
  float dist = 0, dtip[DX_MAX_TIPS];
  bool all_close = true;
  float rsum = 0;
  if (reach) {
    for (int t = 0; t < P.ntips; t++) {
      const float* x = B.site_xpos + ((size_t)env * P.nsite + P.tip_sites[t]) * 3;
      float d0 = g[3 * t] - x[0], d1 = g[3 * t + 1] - x[1], d2 = g[3 * t + 2] - x[2];
      dtip[t] = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
      bool close = dtip[t] <= P.threshold;
      all_close = all_close && close;
      // reach.py:196-210: dense -tanh^2(d, 0.1), sparse -1, 0 within the threshold
      rsum += close ? 0.f : (P.dense ? -tanh_squared(dtip[t], 0.1f) : -1.f);
    }
  } else if (P.kind == DX_KIND_HANDOVER) {
    // the cube's distance to the receiving hand's target point
    const float d0 = q[P.prop_qadr] - g[0], d1 = q[P.prop_qadr + 1] - g[1], d2 = q[P.prop_qadr + 2] - g[2];
    dist = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    all_close = dist <= P.threshold;
  } else {
    dist = quat_distance(g, cur);
    all_close = dist <= P.threshold;
  }
  if (lane == 0) {
    if (skip) {
      S.step_type[env] = TS_FIRST;
      S.reward[env] = 0;
      S.discount[env] = 1;
    } else if (bad) {
      // a substep diverged and the physics reset the env (dx_step.hip health_check):
      // [3P] composer.Environment.step with a PhysicsError it does not raise ends the
      // episode with reward 0 and discount 0; the next step re-initialises the env
      S.step_type[env] = TS_LAST;
      S.reward[env] = 0;
      S.discount[env] = 0;
    } else {
      // physics time in fp64, as MuJoCo accumulates d->time (time += h per mj_step): the
      // fp64 sum is advanced by one addition per physics step taken since the reset (the
      // reach sampling pass's accepted rollouts included, an integer count that travels
      // with the state); the goal's start time is taken at the substep the pass recorded
      const int n_now = nsteps;
      int n = S.nsub_d[env];
      double time = S.time_d[env];
      const int sn = S.solve_n[env];
      if (sn >= 0 && sn <= n) S.solve_start_d[env] = time;
      for (; n < n_now; n++) {
        time = __dadd_rn(time, P.h_d);
        if (n + 1 == sn) S.solve_start_d[env] = time;
      }
      S.solve_n[env] = -1;
      S.nsub_d[env] = n;
      S.time_d[env] = time;
      // GoalTask.after_step (task.py:167-185)
      if (all_close) {
        S.counter[env] += 1;
        if (!S.registered[env]) { S.successes[env] += 1; S.registered[env] = 1; }
      } else if (P.max_time_d > 0 && time - S.solve_start_d[env] > P.max_time_d) {
        S.exceeded[env] = 1;
      }
      // ReOrient.after_step: fall detection (prop-ground contact at the new state)
      int failure = !reach && P.fall_termination && B.watch && B.watch[env];
      S.failure[env] = failure;
      bool success_done = S.successes[env] >= P.successes_needed;
      // composer.Environment.step: should_terminate_episode or time >= time_limit
      // (a time-limit truncation keeps the task's discount)
      bool terminate = success_done || S.exceeded[env] || failure || time >= P.time_limit_d;
      float r;
      if (reach) {
        r = rsum / (float)P.ntips;
      } else {
        // reorient.py:238-284: 1/(d+eps) + 800*[d<=thr] - 0.1*|ctrl|^2 (handover: the same
        // shape on the cube's distance to the target point, with the task's weights)
        float cn = 0;
        for (int i = 0; i < P.nu; i++) {
          float c = B.ctrl[(size_t)env * P.nu + i];
          cn += c * c;
        }
        r = P.w_orient * (1.0f / (dist + P.eps)) + P.w_success * (dist <= P.threshold ? 1.0f : 0.0f) + P.w_action * cn;
      }
      S.reward[env] = r;
      // discount (reorient.py:222-225, task.py:195-204)
      S.discount[env] = failure ? 1.0f : (success_done ? 0.0f : 1.0f);
      S.step_type[env] = terminate ? TS_LAST : TS_MID;
    }
  }
  // observation (STATE_ONLY), flat layout:
  // [sin/cos(qpos_hand) 2*hand_nq | qvel_hand | tip pos 3*ntips | tip linvel 3*ntips |
  //  reorient: prop pos 3 | prop quat 4 | prop linvel 3 | prop angvel 3 | target quat 4 |
  //  goal (4 quaternion, or 3*ntips fingertip positions for reach; handover: the prop block
  //  without the target quaternion, goal = target point + receiving hand)]
  float* o = S.obs + (size_t)env * P.obs_dim;
  const float n = sqrtf(cur[0] * cur[0] + cur[1] * cur[1] + cur[2] * cur[2] + cur[3] * cur[3]);
  for (int k = lane; k < P.obs_dim; k += 64) {
    int e = k;
    float val = 0.f;
    if (e < 2 * P.hand_nq) {
      float sn, cs;
      sincosf(q[e >> 1], &sn, &cs);
      val = (e & 1) ? cs : sn;
    } else if ((e -= 2 * P.hand_nq) < P.hand_nv) {
      val = v[e];
    } else if ((e -= P.hand_nv) < 3 * P.ntips) {
      val = B.site_xpos[((size_t)env * P.nsite + P.tip_sites[e / 3]) * 3 + e % 3];
    } else if ((e -= 3 * P.ntips) < 3 * P.ntips) {
      val = B.site_vel[((size_t)env * P.nsite + P.tip_sites[e / 3]) * 6 + e % 3];
    } else {
      e -= 3 * P.ntips;
      if (P.prop_qadr >= 0) {
        if (e < 3) {
          val = q[P.prop_qadr + e];
        } else if (e < 7) {  // cur[e - 3], read from qpos: a lane-indexed cur[] would live in scratch
          val = q[P.prop_qadr + e] / n;
        } else if (e < 10) {
          val = v[P.prop_dadr + e - 7];
        } else if (e < 13) {
          // frameangvel: world-frame angular velocity = R(quat) * local omega
          const float w0 = cur[0] / n, x = cur[1] / n, y = cur[2] / n, z = cur[3] / n;
          const float* wl = v + P.prop_dadr + 3;
          const int r = e - 10;
          const float R0 = r == 0 ? 1 - 2 * (y * y + z * z) : (r == 1 ? 2 * (x * y + w0 * z) : 2 * (x * z - w0 * y));
          const float R1 = r == 0 ? 2 * (x * y - w0 * z) : (r == 1 ? 1 - 2 * (x * x + z * z) : 2 * (y * z + w0 * x));
          const float R2 = r == 0 ? 2 * (x * z + w0 * y) : (r == 1 ? 2 * (y * z - w0 * x) : 1 - 2 * (x * x + y * y));
          val = R0 * wl[0] + R1 * wl[1] + R2 * wl[2];
        } else if (P.kind == DX_KIND_HANDOVER) {
          val = g[e - 13];  // goal_state (no hint prop)
        } else if (e < 17) {
          val = g[e - 13];  // target_prop/orientation (hint cube = goal)
        } else {
          val = g[e - 17];  // goal_state
        }
      } else {
        val = g[e];  // goal_state
      }
    }
    o[k] = val;
  }
}
