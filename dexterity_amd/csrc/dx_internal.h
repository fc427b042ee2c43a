// dx_internal.h -- device-side model / batch / LDS layout of libdx.so (gfx950).
//
// One 64-lane wavefront (= one 64-thread workgroup) advances one environment.
// Everything per-env lives in LDS for the whole launch; the model (shared by all
// environments, ~150-300 KB) is read from global memory and stays L2-resident.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DX_WAVE 64
// Contact pool, two tiers.  The step kernel keeps DX_NCON_MAX = 32 contacts per env and
// physics step in LDS; a physics step that finds more is not truncated but deferred, from
// its unchanged state, to the overflow tier (dx_step.hip compiled with -DDX_TIER_HI, pool
// DX_NCON_HI = 256, above the reference scenes' nconmax 200, shadow_hand_series_e.xml:8).
// A pool that still overflows keeps its first contacts in candidate (generation) order.
#define DX_NCON_HI 256
// The mid tier (-DDX_TIER_MID, pool DX_NCON_MID) runs beside a queued step-kernel launch, in
// the LDS one step-kernel workgroup leaves free on a CU, and takes the deferred physics
// steps as they are published (dx_step.hip dx_step_mid_kernel); a step beyond its pool
// goes on to the overflow tier after the launch.
#define DX_NCON_MID 64
#ifndef DX_NCON_MAX
#define DX_NCON_MAX 32    // contacts kept per env per substep by this translation unit
#endif
#define DX_NCON_SPARE 4   // extra record slots: the crossing candidate's contacts in a pool cut
// contact chunks of DX_WAVE (lane = contact) the constraint / Hessian passes walk
#define DX_NCH ((DX_NCON_MAX + DX_WAVE - 1) / DX_WAVE)
// first step of the shuffle search over a chunk's contacts (5 steps for <= 32 contacts)
#define DX_SEARCH0 (DX_NCON_MAX > 32 ? 32 : 16)
#ifndef DX_CAND_MAX
#define DX_CAND_MAX 768   // collision candidate-list words per env (dx_api.hip LDS layout)
#endif
#define DX_DOFMAX 14      // max dofs in a contact Jacobian (|chain(b1) xor chain(b2)|; checked at load)
#define DX_CON_STRIDE 20  // words per contact record in LDS:
// 0-2 pos, 3-11 frame (normal, tangents), 12 dist, 13 geom pair, 14 nnz | nrows << 8
// (key while sorting), 15 first efc row, 16-17 friction (mu1, mu2), 18-19 dof support mask
#define DX_MAX_NV 64      // dof bitmasks are uint64
#define DX_QUEUES 8         // substep queues: one per XCD (MI355X: 8 XCDs)
#define DX_QHEAD_STRIDE 64  // words between two queue heads (each on its own 256-B span)
#define DX_SEP_SLOTS 64   // per-env MPR separating-direction cache, slot = geom pair & 63
#ifndef DX_SEP_WT
#define DX_SEP_WT 0       // 1: cache entries stored write-through (sc1), the round-2 form
#endif
// 1: a cached separating direction that still separates stays in the cache (0: the
// round-3 code cleared it after every such verdict, so the cache hit every other substep)
#ifndef DX_SEP_KEEP
#define DX_SEP_KEEP 1
#endif
#define DX_LDL_SLOTS 16   // tree-sparse LDL^T items: at most 16 x 64 (dx_device.h tree_solve)
#ifndef DX_SWEEP_PK
#define DX_SWEEP_PK 1     // sweep: pivot-column zeroing by packed multiplies (0: one select per entry)
#endif
#ifndef DX_SWEEP
#define DX_SWEEP 1        // dense solves n <= 30 by the MFMA sweep operator (else Cholesky)
#endif

// narrowphase lane groups per wave: 8 of 8 lanes, or 16 of 4 lanes when a substep has
// more than 8 candidates (dx_step.hip narrow_pass); the LDS layout reserves the portal
// points of the larger count
#define DX_NGRP_MAX 16
#define DX_GOAL_RETRIES 64  // reach goal sampling: GoalInitializationError retries per goal (bounded)

enum { DXG_PLANE = 0, DXG_SPHERE = 2, DXG_CAPSULE = 3, DXG_BOX = 6, DXG_MESH = 7 };
enum { DXJ_FREE = 0, DXJ_HINGE = 3 };
enum { DXR_FRIC = 0, DXR_LIMJ = 1, DXR_LIMT = 2, DXR_CON = 3, DXR_CONFL = 4 };

// Model arrays are read-only for a launch; on the device the pointers carry the
// constant address space, so uniform accesses compile to scalar (s_load) loads
// and divergent ones to global loads -- never generic flat loads.
#ifdef __HIP_DEVICE_COMPILE__
#define DXG __attribute__((address_space(4)))
#else
#define DXG
#endif

struct DevModel {
  int nq, nv, nbody, njnt, ngeom, nsite, nu, ntendon, nwrap, nbpair, ngpair;
  int iterations, disable_contact, any_damping, nlevel, nroot, nfric, nlimj, nlimt;
  int solver;  // [3P] mjtSolver: 0 PGS, 1 CG, 2 Newton (default)
  float timestep, tolerance, impratio, meaninertia;
  float gravity[3];
  // bodies
  const DXG int *body_parent, *body_rootidx, *body_jntnum, *body_jntadr, *body_dofnum, *body_dofadr;
  const DXG int *lvl_adr, *lvl_body, *root_body;
  const DXG uint64_t* body_chain;  // dofs on the path body -> root
  const DXG float *body_pos, *body_quat, *body_ipos, *body_imat, *body_mass, *body_inertia;
  const DXG float *body_bsphere, *body_invweight0;
  // joints / dofs
  const DXG int *jnt_type, *jnt_bodyid, *jnt_qposadr, *jnt_dofadr;
  const DXG float *jnt_pos, *jnt_axis, *jnt_range, *jnt_margin, *jnt_solref, *jnt_solimp, *qpos0;
  const DXG int *limj_jnt;  // limited hinge joints
  const DXG int *dof_bodyid, *dof_parentid, *dof_jntid, *fric_dof, *dof_fricrow;
  const DXG float *dof_armature, *dof_damping, *dof_frictionloss, *dof_solref, *dof_solimp,
      *dof_invweight0;
  // geoms / meshes
  const DXG int *geom_type, *geom_bodyid, *geom_dataid;
  const DXG float *geom_size, *geom_pos, *geom_mat, *geom_center, *geom_bsphere, *geom_bsphere_b, *geom_obb_b;
  const DXG int *mesh_vertadr, *mesh_vertnum;
  const DXG float4* mesh_vert4;  // hull vertices (x, y, z, index in the mesh as int bits)
  // direction-binned hulls (dx_api.hip build_hull_bins): cube map of binn x binn cells
  // per face, bincap = DX_HULL_K float4 (x, y, z, vertex index bits; -1 = padding) per cell
  const DXG int *mesh_binn, *mesh_bincap, *mesh_binadr;
  const DXG float4* mesh_bin4;
  // narrowphase setup records: geom_rec [ngeom][8] float4 = {type, body, nvert, bin_n,
  // bin_cap, vert4 offset, bin4 offset, -}{size, -}{pos, -}{mat 9, center 3, -};
  // gpair_rec [ngpair] = {g1, g2, margin, primitive-pair flag}
  const DXG float4 *geom_rec, *gpair_rec;
  // culling records (dx_api.hip): geom_crec [ngeom][6], bpair_rec [nbpair][7] float4
  const DXG float4 *geom_crec, *bpair_rec;
  // tree records (dx_api.hip): body_rec [nbody][8] float4, dof_rec [nv][2] float4
  const DXG float4 *body_rec, *dof_rec;
  // tree-sparse LDL^T of M (dx_api.hip): [ldl_nslot][64] items k | i << 8 | j << 16
  // (-1: none) grouped by level, bit s of ldl_sync ends a level; nslot 0: dense solver
  int ldl_nslot;
  unsigned ldl_sync;
  const DXG int* ldl_tab;
  // sites
  const DXG int* site_bodyid;
  const DXG float *site_pos, *site_mat;
  // tendons (fixed) and actuators
  const DXG int *tendon_adr, *tendon_num, *wrap_dof, *wrap_qadr, *limt_ten;
  const DXG float *tendon_range, *tendon_margin, *tendon_solref, *tendon_solimp, *tendon_invweight0,
      *wrap_coef, *tendon_J;
  const DXG int *actuator_trntype, *actuator_trnid, *actuator_biastype, *actuator_ctrllimited,
      *actuator_forcelimited;
  const DXG float *actuator_gear, *actuator_gainprm, *actuator_biasprm, *actuator_ctrlrange,
      *actuator_forcerange;
  // collision pairs
  const DXG int *bpair_body, *bpair_adr, *bpair_num, *bpair_plane, *gpair_geom, *gpair_condim;
  const DXG float* bpair_sphere;  // [nbpair][8]: sphere of side 1, side 2 (body frames)
  const DXG float *gpair_friction, *gpair_solref, *gpair_solimp, *gpair_margin;
};

struct TaskParams;
struct TaskState;
struct DevBatch {
  int nenv;
  float *qpos, *qvel, *ctrl, *qacc_ws, *qacc, *time;
  float *site_xpos, *site_vel, *xpos, *xquat;
  int *ncon, *watch, *niter, *ncand;
  const float* xfrc;  // [nbody*6], shared by all envs (may be null)
  int out_bodies;     // write DX_XPOS / DX_XQUAT after each step (dx_set_outputs)
  const int* skip;    // [nenv] nonzero: env was just reset, observe only (may be null)
  int watch_geom, watch_body;
  const int* watch_pairs;  // body pairs that can hold a watched contact (dx_set_watch), or null
  int watch_npairs;
  // debug (null when disabled)
  float *dbg_qacc_smooth, *dbg_qfrc_smooth, *dbg_M, *dbg_con;
  int* dbg_nefc;
  unsigned long long* stage_acc;  // [DX_NSTAGE] s_memtime cycles per stage (null: off)
  float4* sepcache;               // [nenv][DX_SEP_SLOTS] (dir, pair + 1) of separated pairs
  const int* order;               // [nenv] workgroup -> env (heaviest first), or null
  unsigned* cost;                 // [nenv] shader cycles / 1024 of the env's last step, or null
  const TaskParams* tp;           // device copies, reach sampling pass only (mode 2)
  const TaskState* ts;
  // substep queue (mode 3, dx_step.hip step_queue): one task counter per queue
  // ([DX_QUEUES][DX_QHEAD_STRIDE], zeroed on the stream before each queued launch),
  // per-env progress tags (epoch * 32 + substeps done), launch epoch, the number of
  // queues in use (1 or DX_QUEUES: one per XCD), timeout mark
  unsigned* qhead;
  unsigned* progress;
  unsigned epoch;
  int nqueue;
  int* qerr;
  // the state an env's task hands to its next substep's task: [nenv][hand_stride]
  // floats = qpos | qvel | warm start | time | cost so far | nstep | flags, each record on
  // whole 128-B lines (hand_stride a multiple of 32), so a hand-off writes back and reads
  // only its own lines
  float* hand;
  int hand_stride;
  // torque sensors (dx_sensor.hip): the last substep's pre-integration state, solved
  // qacc and contact forces, [nenv][dx_sensor_stash_words]; null when the field is off
  float* sen_stash;
  // always-on health counters ([DX_HEALTH_WORDS], include/dx.h dx_health), the optional
  // histogram of contacts found per env-substep ([DX_NCON_HIST], null: off) and the
  // per-env divergence flag (set when a substep produced a non-finite or runaway state
  // and the env was reset, MuJoCo's BADQACC; cleared by the task post kernel)
  unsigned* health;
  unsigned* ncon_hist;
  int* bad;
  int* nstep;  // [nenv] physics steps since the env's last mj_resetData (fp64 time = nstep additions of h)
  // narrowphase group size: sixteen 4-lane groups when a substep has more than np_wide
  // candidates, else eight 8-lane groups (DX_WAVE / 8; DX_NP_WIDE overrides it, the
  // group-size invisibility test forces either layout)
  int np_wide;
  // physics steps deferred by the step kernel (dx_step.hip env_defer): [0] the count, [1]
  // the epoch of the queued launch that published the entries (the mid tier claims only its
  // own launch's), [2 ..] entries (DX_DEFER_*), emptied by the overflow kernel's last workgroup
  unsigned* defer;
  // with the mid tier running beside a queued launch (mid = 1): the step kernel publishes
  // each deferral (state in the env's hand-off record, entry | DX_DEFER_VALID stored after
  // it), its workgroups count themselves in qdone[0] as they exit, and the mid tier's own
  // deferrals go to defer2 (same layout, batch arrays) for the overflow tier
  unsigned* defer2;
  unsigned* qdone;  // [0] exits of queued workgroups (never reset), [1] deferral entries finished this launch
  int mid, mid_defer_at;
  int defer_at;  // defer a physics step with more contacts than this (DX_NCON_MAX; DX_DEFER_AT for tests)
  // longest-first key: 1 (default) the control step's last physics step's cost x nsub, 0
  // the whole control step's cost (measured same-box: 1 is 0.4 % faster), 2 their mean
  int order_last;
  // Task logic fused into the step kernel (dx_task.h; DevBatch::tp / ts): task_pre in the
  // env's first physics-step task, with ctrl = the action (`action`, [nenv][nu], or drawn
  // in the kernel by the random agent when act_random: dx_urand(act_seed, env0 + env,
  // act_step)), task_post in its last.  0: the task kernels of dx_task.hip run instead.
  int fuse;
  const float* action;
  int act_random, act_step;
  uint64_t act_seed;
  // Longest-first dispatch order for the next launch, built without a kernel of its own:
  // an env's last task of a launch that sets onext counts its cost bucket in
  // ohist[opar][256] (descending cost) and keeps its rank in okey[env] (bucket <<
  // DX_OKEY_RANK_BITS | rank); the overflow tier's launch then places every env at its bucket's prefix +
  // rank in `order` and its last workgroup zeroes ohist[opar] and the queue heads.
  unsigned *ohist, *okey;
  int opar, onext;
};
#define DX_OKEY_RANK_BITS 24  // rank within a cost bucket: a whole batch (nenv <= 2^20) fits one bucket
// deferral entries: env (bits 0-19) | physics step << 20 (bits 20-27) | flags
#define DX_DEFER_ENV_BITS 20
#define DX_DEFER_FWD (1u << 28)      // forward only (dx_forward)
#define DX_DEFER_CLAIMED (1u << 29)  // taken by the mid tier or the overflow tier (compare-and-swap)
#define DX_DEFER_VALID (1u << 31)    // published (beside a mid-tier launch)
#define DX_HEALTH_WORDS 16
#define DX_NCON_HIST 65   // bins 0..63, and >= 64
#define DX_MAXVAL 1e10f   // mjMAXVAL: |qacc| beyond this is a diverged state (mj_checkAcc)
#define DX_NSTAGE 48
// slots of a hull's support block: a cube-map cell (one 128-B line), or the first
// vertices of a hull scanned whole; a hull with more vertices is binned
#define DX_HULL_K 8

// Offsets (in 4-byte words) of every per-env LDS array.
struct Lds {
  int qpos, qvel, ctrl, qacc, qacc_smooth, qfrc_smooth, qfrc_con;
  int v1, v2, v3, v4, v5;  // nv-sized scratch vectors (Ma, grad, dir, Mdir, tmp)
  int xpos, xquat, xmat, xipos, xanchor, xaxis, rcom, cinert, cdof, cvel, cdof_dot, scr;
  int M, H, ten_len, act_len, act_force;
  int con, cj_idx, cj_val, cq, cw;
  int efc_meta, efc_D, efc_aref, efc_fl, efc_Rf, efc_jar, efc_jv;
  int tri;   // ushort lower-triangle index table (nv > 32 only)
  int ints;  // misc int scalars
  int tsm;   // smooth-solve Cholesky transpose
  int cand;  // collision candidate lists
  int cgv;   // CG solver: M^-1 grad (nv words, free space during the solve)
  int nefc_max, cand_max;
  int total;
};

// Task parameters and per-env task state, see dx_task.hip.
enum { DX_KIND_REORIENT = 0, DX_KIND_REACH = 1, DX_KIND_HANDOVER = 2 };
#define DX_MAX_TIPS 16  // fingertip sites a task observes (two hands: 10)
struct TaskParams {
  int kind;                 // DX_KIND_*
  int nenv, nq, nv, nu, nsite;
  int hand_nq, hand_nv;     // hand joints are qpos[0:hand_nq], qvel[0:hand_nv]
  int prop_qadr, prop_dadr; // free joint of the prop (reorient), -1 otherwise
  int ntips;                // fingertip sites
  int tip_sites[DX_MAX_TIPS];
  int obs_dim, goal_dim;
  int successes_needed, steps_before_change, fall_termination;
  float threshold, eps, w_orient, w_success, w_action, max_time, timestep_ctrl;
  float time_limit;         // composer Environment time_limit (s); +inf: none
  float bbox_lo[3], bbox_hi[3];
  float hand_target[2][3];  // handover: the point above each palm the cube is handed to
  double bbox_lo_d[3], bbox_hi_d[3];  // the same box in fp64 (the reference's values)
  // reach (fingertip_position.py / dexterous_hand.py samplers)
  int dense, max_reject, ncoupled;
  int coupled[8][2];        // qpos[c[0]] = qpos[c[1]] after uniform joint sampling
  float range_frac, goal_scale;
  const float* tdata;       // device: ref[nq] | lo[nq] | hi[nq] | position->control [nu][nq]
                            // [| fp64 raw bits: ref, normal scale, lo, hi, uniform lower, upper]
  int tdata_f64;            // the fp64 block is present (numpy-compatible draws)
  uint64_t seed;
  int env0;                 // global index of this batch's env 0 (a shard of a sharded job):
                            // env e is the job's env env0 + e and draws from seed + env0 + e
  // fp64 time bookkeeping, as MuJoCo's d->time (mjtNum): the physics timestep, the
  // per-goal limit (max_time_per_goal) and composer's time_limit (+inf: none)
  double h_d, max_time_d, time_limit_d;
};

struct TaskState {
  float *goal, *solve_start, *reward, *discount, *obs;
  int *successes, *counter, *registered, *exceeded, *step_type, *episode, *skip, *failure;
  int *need, *goalnum, *goalfail;  // reach: bit0 next_goal, bit1 joint init; goals drawn; rejected-out goals
  float* goal_qpos;                // reach: [nenv][nq] joints that placed the goal (FingertipCartesianPosition.qpos)
  // reorient: numpy-compatible MT19937 streams per env (dx_mt_*): the env's RandomState
  // (PropPlacer draws) and numpy's global stream (the goal draws), [625][nenv] each
  uint32_t *mt_env, *mt_goal;
  // reach: the env's RandomState as one contiguous block per env, [nenv][DX_MTW_WORDS]
  // (state[624], pos, has_gauss, gauss as fp64), drawn wave-cooperatively in the step
  // kernel (dx_step.hip mtw_*)
  uint32_t* mt_reach;
  // fp64 time (TaskParams::h_d): the env's time as MuJoCo accumulates it (time += h per
  // physics step, from 0 at the episode's mj_resetData), the substeps it covers, the
  // time the current goal was set, and (reach) the substep at which the sampling pass
  // set it (-1: none pending)
  double *time_d, *solve_start_d;
  int *nsub_d, *solve_n;
};

// numpy.random.RandomState-compatible MT19937 ([3P] numpy legacy seeding and
// random_sample: mt19937_seed, mt19937_gen, legacy_double), one stream per env kept in
// HBM interleaved over the envs -- word k of env e at k * nenv + e (k < 624), the read
// position at 624 * nenv + e -- so the rare twist (every 624 words) is a coalesced
// sweep across a wave's envs.  Pinned against numpy in tests/test_host_logic.py and
// tests/test_gpu_env.py.
#define DX_MT_WORDS 625
#define DX_MTW_WORDS 628
// tempering of an MT19937 state word (mt19937_genrand output stage)
__device__ __forceinline__ uint32_t dx_mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  return y ^ (y >> 18);
}
__device__ __forceinline__ void dx_mt_seed(uint32_t* s, int nenv, int env, uint32_t seed) {
  for (int k = 0; k < 624; k++) {
    s[(size_t)k * nenv + env] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(k + 1);
  }
  s[(size_t)624 * nenv + env] = 624;
}
__device__ __forceinline__ uint32_t dx_mt_next(uint32_t* s, int nenv, int env) {
  uint32_t pos = s[(size_t)624 * nenv + env];
  if (pos >= 624) {
    for (int k = 0; k < 624; k++) {
      const uint32_t a = s[(size_t)k * nenv + env], b = s[(size_t)((k + 1) % 624) * nenv + env];
      const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
      s[(size_t)k * nenv + env] = s[(size_t)((k + 397) % 624) * nenv + env] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    pos = 0;
  }
  const uint32_t y = s[(size_t)pos * nenv + env];
  s[(size_t)624 * nenv + env] = pos + 1;
  return dx_mt_temper(y);
}
// RandomState.random_sample: 53-bit double from two outputs
__device__ __forceinline__ double dx_mt_double2(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}
__device__ __forceinline__ double dx_mt_double(uint32_t* s, int nenv, int env) {
  const uint32_t a = dx_mt_next(s, nenv, env), b = dx_mt_next(s, nenv, env);
  return dx_mt_double2(a, b);
}
// The next N outputs at once: one load of the position, then the N state words as
// independent loads (one memory round trip instead of two per output), unless the
// block crosses a twist -- then one output at a time.
template <int N>
__device__ __forceinline__ void dx_mt_take(uint32_t* s, int nenv, int env, uint32_t (&out)[N]) {
  const uint32_t pos = s[(size_t)624 * nenv + env];
  if (pos + N <= 624) {
#pragma unroll
    for (int k = 0; k < N; k++) out[k] = dx_mt_temper(s[(size_t)(pos + k) * nenv + env]);
    s[(size_t)624 * nenv + env] = pos + N;
  } else {
    for (int k = 0; k < N; k++) out[k] = dx_mt_next(s, nenv, env);
  }
}
// [3P] dm_control composer.variation.rotations.UniformQuaternion:
// u1, u2, u3 = random_state.uniform([0, 0, 0], [1, 2 pi, 2 pi]);
// q = [sqrt(1-u1) sin u2, sqrt(1-u1) cos u2, sqrt(u1) sin u3, sqrt(u1) cos u3]
// (computed in double, then rounded to the fp32 state)
__device__ __forceinline__ void dx_mt_quat_from(const uint32_t* w, float* q) {
  const double twopi = 6.283185307179586;
  const double u1 = dx_mt_double2(w[0], w[1]);
  const double u2 = twopi * dx_mt_double2(w[2], w[3]);
  const double u3 = twopi * dx_mt_double2(w[4], w[5]);
  const double a = sqrt(1.0 - u1), b = sqrt(u1);
  q[0] = (float)(a * sin(u2));
  q[1] = (float)(a * cos(u2));
  q[2] = (float)(b * sin(u3));
  q[3] = (float)(b * cos(u3));
}
__device__ __forceinline__ void dx_mt_uniform_quat(uint32_t* s, int nenv, int env, float* q) {
  uint32_t w[6];
  dx_mt_take<6>(s, nenv, env, w);
  dx_mt_quat_from(w, q);
}

// Counter-based RNG: splitmix64 over (seed, env, episode, draw).
__device__ __forceinline__ uint64_t dx_mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float dx_urand(uint64_t seed, int env, int episode, int draw) {
  uint64_t h = dx_mix64(seed ^ dx_mix64(((uint64_t)env << 32) ^ (uint64_t)(uint32_t)episode) ^
                        dx_mix64(0x51ed27ull + (uint64_t)(uint32_t)draw));
  return (float)((h >> 40) * (1.0 / 16777216.0));
}

// dx_step.hip: specialized-kernel lookup and launch (host side)
int dx_spec_find(const DevModel& d, const Lds& L);
bool dx_spec_reach(int spec);  // the specialization fuses the reach sampling pass
int dx_step_occupancy(int spec, size_t lds);
hipError_t dx_launch_step(int spec, int grid, size_t lds, hipStream_t stream, const DevModel* mdev, const DevBatch& B,
                          const Lds& L, int nsub, int mode);
hipError_t dx_launch_order(int nenv, hipStream_t stream, const unsigned* cost, int* order, unsigned* qhead);
// the overflow tier (dx_step.hip, DX_TIER_HI): the physics steps deferred by the last launch
hipError_t dx_launch_step_hi(int grid, size_t lds, hipStream_t stream, const DevModel* mdev, const DevBatch& B,
                             const Lds& L, int nsub);
// the mid tier (dx_step.hip, DX_TIER_MID): beside the queued launch after which qdone[0]
// reaches `target`
hipError_t dx_launch_step_mid(int grid, size_t lds, hipStream_t stream, const DevModel* mdev, const DevBatch& B,
                              const Lds& L, int nsub, unsigned target);

// dx_sensor.hip: joint torque sensors from the step kernel's stash (host side)
hipError_t dx_launch_sensor(int nenv, size_t lds, hipStream_t stream, const DevModel* mdev, const DevBatch& B,
                            const Lds& L, float* out);

// dx_ik.hip: site Jacobians and batched damped-least-squares IK (host side).
struct IkDev {
  int mode;                  // 0: IK attempts (one wave per (env, attempt)); 1: site Jacobians
  int nsite, njoint, max_steps, early_stop, nattempt, stop_on_first;
  float tol, reg, gain, progress;
  uint64_t seed;
  int blk;                   // LDS word offset of the IK block (after the model's layout)
  const int* sites;          // [nsite]
  const int* joints;         // [njoint]
  const float* targets;      // [nenv][nsite][3]
  float* att_qpos;           // [nenv][nattempt][njoint]
  float* att_err;            // [nenv][nattempt][nsite]
  int* att_steps;            // [nenv][nattempt]
  float *jacp, *jacr;        // mode 1: [nenv][nsite][3][nv] (either may be null)
  const float* starts;       // [nenv][nattempt - 1][njoint]: attempts >= 1 start here
};
hipError_t dx_launch_ik_starts(int nenv, int natt, int njoint, uint64_t seed, const double* range, uint32_t* mt,
                               float* out, hipStream_t stream);
int dx_ik_lds_words(const DevModel& d, int nsite);
hipError_t dx_launch_ik(int nwave, size_t lds, hipStream_t stream, const DevModel* mdev, const DevBatch& B,
                        const Lds& L, const IkDev& P);
hipError_t dx_launch_ik_select(int nenv, hipStream_t stream, const DevModel& m, const IkDev& P, float* qpos_out,
                               int* success, float* err_out, int* attempt_out, int* steps_out);
