/*
 * dx.h -- C ABI of the MI355X batched physics step (libdx.so).
 *
 * This is the drop-in boundary for the reference's hot path.  In the reference
 * (v-wewei/dexterity) every environment owns one MuJoCo mjModel/mjData pair behind
 * dm_control's `mjcf.Physics`, and the path is driven through these calls
 * ([3P] MuJoCo C API):
 *
 *   physics.step()            -> mj_step2(m,d); mj_step1(m,d)   (composer substep loop,
 *                                 reorient.py:58,61,168 / reach.py:54,59,139)
 *   physics.forward()         -> mj_forward(m,d)                (fingertip_position.py:95)
 *   physics.bind(acts).ctrl=  -> d->ctrl                        (effectors/mujoco_actuation.py:33)
 *   bind(joints).qpos/.qvel   -> d->qpos / d->qvel              (shadow_hand_e.py:121, reorient.py:187)
 *   xfrc_applied[:] = -m g    -> d->xfrc_applied                (utils/mujoco_utils.py:91-99)
 *   bind(sites).xpos          -> d->site_xpos                   (dexterous_hand.py:286-291)
 *   physics.data.contact      -> d->contact, d->ncon            (utils/mujoco_collisions.py:95-119)
 *
 * Here one handle (`dx_batch`) owns B environments that share one compiled model;
 * all state stays resident in HBM and one call advances every environment.
 *
 * Conventions:
 *  - every function returns 0 on success or a negative DX_E* code; the message of
 *    the last failure on the calling thread is in dx_last_error();
 *  - state arrays are float32, environment-major: field[env][n];
 *  - pointers passed to dx_set_field / dx_get_field may be host or device memory
 *    (resolved through HIP's unified addressing);
 *  - calls on one dx_batch are serialised on its own HIP stream; a dx_batch is not
 *    thread-safe; different handles are independent;
 *  - the library owns all device memory it allocates.
 */
#ifndef DX_H
#define DX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DX_ABI_VERSION 1

typedef struct dx_model dx_model;
typedef struct dx_batch dx_batch;

enum dx_error {
  DX_OK = 0,
  DX_EINVAL = -1,   /* bad argument                        */
  DX_EMODEL = -2,   /* malformed or unsupported model blob */
  DX_EHIP = -3,     /* HIP runtime failure                 */
  DX_ENOMEM = -4,   /* allocation failure                  */
  DX_ELIMIT = -5    /* model exceeds kernel limits         */
};

/* Per-environment fields addressable through dx_set_field / dx_get_field /
 * dx_field_ptr.  Widths are per environment. */
enum dx_field {
  DX_QPOS = 0,          /* nq                                    rw */
  DX_QVEL = 1,          /* nv                                    rw */
  DX_CTRL = 2,          /* nu                                    rw */
  DX_QACC_WARMSTART = 3,/* nv                                    rw */
  DX_QACC = 4,          /* nv   last solved acceleration         r  */
  DX_TIME = 5,          /* 1                                     rw */
  DX_SITE_XPOS = 6,     /* 3*nsite  (after dx_step / dx_forward) r  */
  DX_SITE_VEL = 7,      /* 6*nsite  linear(3) + angular(3), world frame, at site r */
  DX_XPOS = 8,          /* 3*nbody                               r  */
  DX_XQUAT = 9,         /* 4*nbody                               r  */
  DX_NCON = 10,         /* 1  (int32 bits)                       r  */
  DX_GROUND_CONTACT = 11, /* 1 (int32 bits): any contact involving geom
                           `ground_geom` with dist <= 1e-8 (reorient.py:229-235) */
  DX_NITER = 12,        /* 1  (int32 bits) solver iterations of the last substep */
  DX_NCAND = 13,        /* 1  (int32 bits) narrowphase candidates of the last collision pass */
  DX_STEP_COST = 14,    /* 1  (uint32 bits) shader cycles / 1024 the env's last dx_step took
                           (feeds the longest-first dispatch order; 0 if disabled) */
  DX_SENSOR_TORQUE = 15,/* 3*nbody  r  (after dx_sensor_enable): 3-axis `torque` sensor of a
                           site at each body's origin, in the body frame -- the joint torque
                           sensors of shadow_hand_e.py:176-196 / adroit_hand.py:153-172
                           (mj_rnePostConstraint + mj_sensorAcc of the last substep, before
                           its integration, as after dm_control's physics.step()) */
  DX_DIVERGED = 16,     /* 1  (int32 bits) r: the env's state diverged during the last dx_step /
                           dx_forward (a non-finite qpos / qvel / qacc, or |qacc| > 1e10: MuJoCo's
                           BADQACC, [3P] mj_checkAcc) and was reset to qpos0 (mj_resetData) */
  DX_NFIELD
};

/* Model ------------------------------------------------------------------ */
/* Loads a compiled-model blob (dexterity_amd/blob.py).  The blob is copied. */
dx_model* dx_model_load(const void* blob, size_t nbytes);
void dx_model_free(dx_model* m);
/* Sizes: out[0..11] = nq nv nbody njnt ngeom nsite nu ntendon nbpair ngpair ncon_max nefc_max
 * (ncon_max / nefc_max: the contact pool and constraint-row capacity of a physics step,
 * DX_NCON_HI = 256 contacts with the overflow tier) */
int dx_model_sizes(const dx_model* m, int32_t out[12]);
/* Bytes of LDS one environment (one 64-lane workgroup) of dx_step uses. */
int dx_model_lds_bytes(const dx_model* m);
/* Test hook: index of the vertex the device's support scan returns for hull `mesh`
   along local direction dir (direction-binned hulls); info =
   [vertex, cube-map cells per face edge (0: not binned), cell capacity]. */
int dx_hull_support(const dx_model* m, int32_t mesh, const float dir[3], int32_t info[3]);
/* Build hook: the per-env LDS layout (dx_internal.h Lds, in words) followed by 16
   model dimensions, for compile-time kernel specialization; returns the count. */
int dx_model_layout(const dx_model* m, int32_t* out, int32_t n);
/* Width (in 4-byte words per environment) of a dx_field. */
int dx_field_width(const dx_model* m, int field);

/* Batch ------------------------------------------------------------------ */
/* Allocates nenv environments on HIP device `device`, reset to qpos0. */
dx_batch* dx_batch_create(const dx_model* m, int32_t nenv, int32_t device);
void dx_batch_destroy(dx_batch* b);
int dx_batch_nenv(const dx_batch* b);
/* Resets environments [env0, env0+n) to qpos0, zero velocity, zero ctrl. */
int dx_reset(dx_batch* b, int32_t env0, int32_t n);

/* Copies n environments' worth of a field, starting at env0. */
int dx_set_field(dx_batch* b, int field, const void* src, int32_t env0, int32_t n);
int dx_get_field(dx_batch* b, int field, void* dst, int32_t env0, int32_t n);
/* Device pointer of a field's [nenv][width] array (zero-copy access). */
int dx_field_ptr(dx_batch* b, int field, void** devptr);
/* Batch-shared applied body wrench xfrc_applied[nbody][6] (force, torque), the
 * gravity-compensation write of utils/mujoco_utils.py:91-99. */
int dx_set_xfrc(dx_batch* b, const float* xfrc, int32_t nbody);
/* Geom whose contacts set DX_GROUND_CONTACT (-1 disables). */
int dx_set_ground_geom(dx_batch* b, int32_t geom);
/* DX_GROUND_CONTACT watches contacts between `geom` and any geom of `body`
 * (reorient.py:229-235: prop geoms vs the arena ground). */
int dx_set_watch(dx_batch* b, int32_t geom, int32_t body);

/* Stepping --------------------------------------------------------------- */
/* Advances every environment by nsubstep physics steps (ctrl held constant),
 * then recomputes position-dependent outputs (site poses, velocities, ground
 * contact) at the new state: the step2->step1 contract of dm_control. */
int dx_step(dx_batch* b, int32_t nsubstep);
/* mj_forward equivalent: outputs at the current state, no integration. */
int dx_forward(dx_batch* b);
/* Stream the batch's kernels are enqueued on (hipStream_t) and a blocking sync. */
void* dx_stream(dx_batch* b);
int dx_sync(dx_batch* b);

/* Whether dx_step / dx_forward write the body poses DX_XPOS / DX_XQUAT (default 1 for
 * a dx_batch, 0 for the batch of a dx_env, whose tasks never read them: 28 B per body
 * and env-step of HBM writes saved). */
int dx_set_outputs(dx_batch* b, int bodies);

/* Sensors ---------------------------------------------------------------- */
/* Enables DX_SENSOR_TORQUE: dx_step / dx_forward then also compute every body's torque
 * sensor (one extra small kernel per call; nothing when disabled). */
int dx_sensor_enable(dx_batch* b, int enable);

/* Health (always on) ----------------------------------------------------- */
/* Counters of capacity overflows and divergences since the batch was created or last
 * cleared, out[0 .. min(n, DX_HEALTH_WORDS)):
 *   0 env-substeps that found more contacts than the contact pool holds, DX_NCON_HI = 256
 *     (above the Shadow scenes' nconmax = 200, shadow_hand_series_e.xml:8): the first 256
 *     in generation (candidate) order are kept, as MuJoCo fills its pool and drops the
 *     rest with mjWARN_CONTACTFULL
 *   1 env-substeps whose broadphase / narrowphase candidate lists overflowed
 *   2 contacts whose Jacobian spans more than DX_DOFMAX dofs (truncated)
 *   3 env-substeps with more constraint rows than the LDS block holds (truncated)
 *   4 env-substeps that diverged (DX_DIVERGED) and reset their env
 *   5 the most contacts one env-substep found, when above 16 (else 0)
 *   6 env-substeps that found more than the 32 contacts the step kernel keeps in LDS and
 *     were therefore run by a larger pool -- the mid tier (64 contacts, beside a queued
 *     step launch on a side stream) or the overflow tier (256, behind the launch), the
 *     same physics: not a truncation
 *   7 mid-tier launches that stopped waiting for deferrals before their step launch ended
 *     (~14 ms without a finished task: a serialised dispatch order or an aborted launch)
 *   8 step-kernel deferrals run by the overflow tier behind the launch instead of by the
 *     mid tier beside it (words 7 and 8: speed only, the same physics)
 * then, when the histogram is on (dx_ncon_histogram), out[16 .. 16 + 65): env-substeps
 * by contacts found (bins 0..63, then >= 64).  Synchronises the batch's stream. */
#define DX_HEALTH_WORDS 16
#define DX_NCON_HIST 65
int dx_health(dx_batch* b, uint32_t* out, int32_t n);
int dx_health_clear(dx_batch* b);
int dx_ncon_histogram(dx_batch* b, int enable);

/* Debug / parity -------------------------------------------------------- */
/* When enabled, dx_forward/dx_step record per-env intermediates of the LAST
 * substep: qacc_smooth, qfrc_bias(+applied), qfrc_actuator, M (nv*nv), contacts. */
int dx_debug_enable(dx_batch* b, int enable);
/* name: "qacc_smooth" "qfrc_smooth" "M" "contact" (16 floats/contact: pos3 frame9
 * dist geom1 geom2 condim) "efc_count" ; dst is host memory for all envs.
 * "health" (no dx_debug_enable needed): dx_health's words, as uint32 bits.
 * "queue_timeouts" (1 word, int32 bits, no dx_debug_enable needed): nonzero if a
 * task of the substep queue ever stopped waiting for its predecessor. */
int dx_debug_get(dx_batch* b, const char* name, float* dst, size_t nfloats);

/* Environments: a dx_batch plus on-device task logic ------------------- */
/* One dx_env is B copies of a reference task (composer.Environment + Task,
 * environment.py:9-34, task.py:137-204): dx_env_step = GoalTask.before_step,
 * n_sub_steps physics steps, after_step, reward, discount, termination and the
 * observation vector, for every env, with dm_env auto-reset (an env that returned
 * LAST is re-initialised by its next step and returns FIRST). */
typedef struct dx_env dx_env;
enum dx_task_kind { DX_TASK_REORIENT = 0, DX_TASK_REACH = 1, DX_TASK_HANDOVER = 2 };
/* Reorient params (float[26], or float[38] with the fp64 bbox), reorient.py:40-78 / task.py:120-135:
 *  0 n_sub_steps  1 hand_nq  2 hand_nv  3 prop_qposadr  4 prop_dofadr
 *  5 first fingertip site  6 n fingertips  7 successes_needed
 *  8 steps_before_changing_goal  9 fall_termination  10 success_threshold
 *  11 orientation_eps  12 w_orientation  13 w_success  14 w_action
 *  15 max_time_per_goal  16-18 prop bbox lower  19-21 prop bbox upper
 *  22 ground geom  23 prop body  24-25 reserved
 *  26-37 (optional) the bbox in fp64: raw bits of lower[3], upper[3] (two words each)
 * Randomness: env e draws from numpy-compatible MT19937 streams seeded with
 * seed + e -- its RandomState (PropPlacer) and numpy's global stream (goals, which
 * the reference's PropOrientation draws from np.random: prop_orientation.py:38). */
#define DX_REORIENT_NPARAMS 26
/* Reach params (float[26 + 3*nq + nu*nq]), reach.py:43-70, task.py:120-135,
 * fingertip_position.py:21-35, dexterous_hand.py:120-168:
 *  0 n_sub_steps  1 hand_nq (= nq)  2 hand_nv  3 n fingertips  4-8 fingertip sites
 *  9 successes_needed  10 steps_before_changing_goal  11 success_threshold
 *  12 max_time_per_goal  13 dense reward (1) / sparse (0)  14 init joint range fraction
 *  15 goal sampling scale  16 max rejection samples  17 n coupled joint pairs
 *  18-25 coupled pairs (joint, source joint): qpos[joint] = qpos[source]
 *  26..  joint midrange [nq], lower [nq], upper [nq], position->control [nu][nq]
 *  then, optionally, six fp64 arrays [nq] as raw bits (two words each): the goal
 *  sampler's mean (joint midrange) and scale (0.1 x range), the joint limits, and the
 *  initial-joint bounds (range_fraction x limits).  With them env e draws from a
 *  numpy-compatible RandomState(seed + e) in the reference's order (goal normals with
 *  numpy's cached polar gaussians, then the uniform joint angles); without them, from a
 *  counter-based stream. */
#define DX_REACH_NPARAMS_HEAD 26
/* Handover params (float[44]): a two-hand scene (BASELINE config 5; the reference has no
 * bimanual task -- its pattern is Juggle's two hands and effectors, juggle.py:147-177,
 * arenas/arena.py:58-105), the cube handed from palm to palm behind the GoalTask surface.
 * 0-37 as reorient's, with hand_nq / hand_nv / fingertips counting both hands and the
 * bbox the giving (first) hand's spawn box; then 38-40 / 41-43 the target points above
 * the first / second hand's palm.  The goal is [target xyz, receiving hand]: at reset
 * the second hand's target; after steps_before_changing_goal successes it switches to
 * the other hand (the cube handed back).  Reward reorient.py:238-284's shape on the
 * cube-to-target distance d: w_orientation / (d + eps) + w_success [d <= threshold] +
 * w_action |ctrl|^2; the cube touching the ground ends the episode (discount 1). */
#define DX_HANDOVER_NPARAMS 44
enum dx_env_out { DX_OUT_OBS = 0, DX_OUT_REWARD = 1, DX_OUT_DISCOUNT = 2, DX_OUT_STEP_TYPE = 3,
                  DX_OUT_GOAL = 4, DX_OUT_SUCCESSES = 5, DX_OUT_GOAL_FAILURES = 6,
                  DX_OUT_GOAL_QPOS = 7 /* reach: [nenv][nq] f32, FingertipCartesianPosition.qpos
                                          (fingertip_position.py:136-139) */ };
dx_env* dx_env_create(const dx_model* m, int32_t nenv, int32_t device, int32_t task, uint64_t seed,
                      const float* params, int32_t nparams);
/* One shard of a job's environments: this handle's env e is the job's env env0 + e.
 * Every per-env stream is keyed by the job-wide index (numpy-compatible MT19937 seeded
 * with seed + env0 + e, dx_env_sample_actions keyed by env0 + e), so shard r of a
 * sharded job behaves exactly like envs [env0, env0 + nenv) of one unsharded batch --
 * the reference's one-RandomState-per-env seed contract (manipulation/__init__.py:56-86)
 * with env i seeded seed + i.  dx_env_create(...) = dx_env_create_shard(..., 0, ...). */
dx_env* dx_env_create_shard(const dx_model* m, int32_t nenv, int32_t device, int32_t task, uint64_t seed,
                            int64_t env0, const float* params, int32_t nparams);
void dx_env_destroy(dx_env* e);
dx_batch* dx_env_batch(dx_env* e);
int dx_env_obs_dim(const dx_env* e);
/* Goal width: 4 (reorient quaternion) or 3 * n fingertips (reach positions). */
int dx_env_goal_dim(const dx_env* e);
/* Re-initialises every env (initialize_episode) and computes FIRST observations. */
int dx_env_reset(dx_env* e);
/* One control step for every env; action is [nenv][nu] float32, device memory.  The
 * reorient task's before_step / after_step / reward / observation run inside the step
 * kernel: a control step is the step kernel, the mid contact tier beside it (a side
 * stream) and the overflow tier's launch after it, which also orders the next launch. */
int dx_env_step(dx_env* e, const float* action);
/* composer.Environment's time_limit (manipulation/__init__.py:61,83): an episode also
 * ends (LAST, with the task's discount) once its physics time reaches `seconds`.
 * Default: none (task.time_limit = inf). */
int dx_env_set_time_limit(dx_env* e, double seconds);
/* max_time_per_goal (task.py:120-135, 180-183) in fp64; default: the float in the task
 * params.  Both limits compare against the env's time accumulated in fp64 as MuJoCo
 * accumulates d->time (one += timestep per physics step), so a limit on a control-step
 * boundary ends the episode at the same step as the reference. */
int dx_env_set_goal_time_limit(dx_env* e, double seconds);
/* Device pointers of the outputs: obs [nenv][obs_dim] f32, reward/discount [nenv] f32,
 * step_type [nenv] i32 (0 FIRST, 1 MID, 2 LAST), goal [nenv][goal_dim] f32, successes i32,
 * goal failures i32 (the GoalInitializationErrors the reference would have raised: goal
 * draws that exhausted max_rejection_samples, fingertip_position.py:112-117; like
 * GoalEnvironment, environment.py:14-34, the env retries -- the step's goal draw, or the
 * whole reset -- from its continuing RandomState, up to 64 times per goal). */
int dx_env_output(dx_env* e, int which, void** devptr);
/* Library-owned [nenv][nu] device action buffer, and a fill of it with actions
 * drawn uniformly within each actuator's ctrlrange (the random agent of
 * manipulation_test.py:44-45), keyed by (seed, env, step). */
int dx_env_action_buffer(dx_env* e, void** devptr);
int dx_env_sample_actions(dx_env* e, uint64_t seed, int32_t step);
/* dx_env_step with the actions dx_env_sample_actions(e, seed, step) would draw, drawn
 * inside the step kernel (no action buffer, no extra launch): the random agent of the
 * reference's environment tests and of the benchmark. */
int dx_env_step_random(dx_env* e, uint64_t seed, int32_t step);

/* Checkpoint / resume.  An env's state is the set of device arrays that carry from one
 * control step to the next (physics and task state, the numpy-compatible MT19937 streams,
 * the dispatch order).  dx_env_save(e, NULL, 0) returns the state's size in bytes;
 * dx_env_save copies it to dst (host or device memory), dx_env_load restores it into an
 * env of the same task, model and batch size: the run then continues bit for bit as the
 * saved one would have.  dx_env_state_field(e, i, ...) describes field i (name, byte
 * offset in the saved buffer, bytes; i < 0: the count) and returns the field count. */
int dx_env_save(dx_env* e, void* dst, size_t nbytes);
int dx_env_load(dx_env* e, const void* src, size_t nbytes);
int dx_env_state_field(dx_env* e, int32_t i, const char** name, size_t* offset, size_t* nbytes);

/* Packs [obs | reward | discount | step_type] per env into dst ([nenv][obs_dim+3]
 * f32, device memory) on the env's stream: the shard an RCCL all-gather collates. */
int dx_env_pack_outputs(dx_env* e, float* dst_dev);
/* The reference's call shape, GoalEnvironment.step(action) -> TimeStep
 * (environment.py:25-34, task.py:63-73): action_host [nenv][nu] f32 and out_host
 * [nenv][obs_dim+3] f32 ([obs | reward | discount | step_type as float]) are host memory
 * (page-locked for asynchronous DMA); upload, control step, pack and download run on the
 * env's stream, and the call returns once out_host holds the TimeStep. */
int dx_env_step_host(dx_env* e, const float* action_host, float* out_host);

/* Multi-GPU observation collation over RCCL -------- */
/* The reference runs one environment per process and has no collective; here each
 * process (one per GPU) owns a dx_env shard of the job's environments and the only
 * exchange is one all-gather of the packed outputs per control step, over xGMI.
 * Bootstrap: rank 0 calls dx_comm_unique_id and hands the DX_COMM_ID_BYTES bytes to
 * every rank (file, env var, socket: the caller's choice) before dx_comm_init. */
typedef struct dx_comm dx_comm;
#define DX_COMM_ID_BYTES 128
int dx_comm_unique_id(void* id /* DX_COMM_ID_BYTES */);
/* Collective over nranks processes (ncclCommInitRank); device = this rank's GPU. */
dx_comm* dx_comm_init(const void* id, int32_t nranks, int32_t rank, int32_t device);
void dx_comm_destroy(dx_comm* c);
int dx_comm_rank(const dx_comm* c);
int dx_comm_size(const dx_comm* c);
/* All-gather of every rank's packed [obs | reward | discount | step_type] rows into
 * dst ([nranks * nenv][obs_dim + 3] f32, device memory on this rank's GPU): rank r's
 * environments land at rows [r * nenv, (r + 1) * nenv).  Enqueued on the env's stream
 * after its step (no host synchronisation); every rank must pass an env with the same
 * nenv and obs_dim. */
int dx_allgather_obs(dx_env* e, dx_comm* c, float* dst_dev);
/* Blocking max over ranks of a host scalar (also a barrier): the bench's job time. */
int dx_comm_allreduce_max(dx_comm* c, double* value);
int dx_comm_barrier(dx_comm* c);

/* Kinematic queries and batched inverse kinematics ---------------------- */
/* mj_jacSite (utils/mujoco_utils.py:67-73, compute_object_6d_jacobian) for every env
 * at its current qpos (kinematics + com positions are recomputed first; the batch's
 * state is not modified).  jacp / jacr: [nenv][nsite][3][nv] f32, host or device
 * memory; either may be null. */
int dx_jac_site(dx_batch* b, const int32_t* sites, int32_t nsite, float* jacp, float* jacr);

/* IKSolver.solve (inverse_kinematics/ik_solver.py:71-167) for every env of a batch.
 * Each attempt integrates damped-least-squares joint velocities
 * (controllers/dls/dls.py:43-77: (J^T J + reg I) qdot = J^T twist, twist = gain *
 * (target - site) / 1 s) with mj_integratePos over dt = 1 s, clips the solved
 * joints to their range, and re-runs kinematics, for at most max_steps steps
 * (ik_solver.py:169-236; early stop when every site is within linear_tol, abort
 * when error / progress > progress_threshold for any site).  Attempt 0 starts the
 * solved joints at their midrange, attempt a > 0 at numpy's a-th
 * np.random.uniform(*range.T) over the passed joints (ik_solver.py:127-130), env e
 * replaying a global stream seeded np.random.seed(seed + e) bit for bit; the other
 * qpos entries come from the batch.  The attempts run in parallel, one wavefront
 * each; the selection follows ik_solver.py:132-152: among attempts with every
 * error <= linear_tol, the first one (stop_on_first_successful_attempt) or the one
 * closest to the midrange (first on ties).  3 * nsite <= 32, njoint <= 64. */
typedef struct dx_ik_options {
  float linear_tol;          /* 1e-3  (ik_solver.py:73)                 */
  float regularization;      /* 1e-5  (_REGULARIZATION_WEIGHT, :24)     */
  float gain;                /* 0.95  (_LINEAR_VELOCITY_GAIN, :18)      */
  float progress_threshold;  /* 20    (_PROGRESS_THRESHOLD, :29)        */
  int32_t max_steps;         /* 100                                     */
  int32_t early_stop;        /* 0                                       */
  int32_t num_attempts;      /* 30                                      */
  int32_t stop_on_first;     /* 0 (stop_on_first_successful_attempt)    */
  uint64_t seed;
} dx_ik_options;
/* targets [nenv][nsite][3]; outputs (host or device memory, any may be null):
 * qpos_out [nenv][njoint] (the selected attempt's solved joints; when no attempt
 * succeeded -- the reference returns None -- the last attempt's), success [nenv]
 * (int32 0/1), linear_err [nenv][nsite] (of the returned joints), attempt [nenv]
 * (int32 index of the returned attempt), steps [nenv] (int32 integration steps it
 * took). */
int dx_ik_solve(dx_batch* b, const dx_ik_options* opt, const int32_t* sites, int32_t nsite,
                const int32_t* joints, int32_t njoint, const float* targets, float* qpos_out,
                int32_t* success, float* linear_err, int32_t* attempt, int32_t* steps);

/* Timing ---------------------------------------------------------------- */
/* When enabled, HIP events bracket the step-kernel launches on the batch stream -- every
 * launch (enable = 1) or every enable-th one (enable > 1: the events' own packets cost
 * ~5 us per bracketed launch); dx_timing_read syncs, returns the summed kernel time and
 * the count of bracketed launches, and clears. */
int dx_timing_enable(dx_batch* b, int enable);
int dx_timing_read(dx_batch* b, double* total_ms, int32_t* count);
/* Per-stage shader-clock accounting inside the fused step kernel (diagnostics):
 * out[k] = summed s_memtime cycles of stage k over all envs since the last read
 * (n < nenv * 40), or out[env * 40 + k] per env (n >= nenv * 40). */
int dx_stage_timing(dx_batch* b, int enable);
int dx_stage_read(dx_batch* b, uint64_t* out, int32_t n);
/* Test hook: overwrites the LDS of every CU on `device` with NaN patterns. */
int dx_debug_poison_lds(int32_t device);

const char* dx_last_error(void);
/* The hash of the sources the library was built from (dexterity_amd/build.py source_key):
 * the Python layer refuses an in-tree library whose sources have changed since. */
const char* dx_build_key(void);
int dx_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
