// dx_device.h -- device toolkit shared by the step kernel (dx_step.hip) and the
// kinematic-query / inverse-kinematics kernels (dx_ik.hip): wave primitives, small
// 3D / spatial algebra, the per-env context, the tree passes (kinematics, com
// positions, tendons, CRB) and the wave / matrix-core Cholesky solvers.
#pragma once
#include "dx_internal.h"

#include <math.h>
#include <string.h>

// The lane id is laundered through an empty volatile asm at every use: the compiler
// can then neither hoist lane-dependent address arithmetic out of the substep loop
// nor keep it alive across the stages (it did, and spilled those values to scratch).
__device__ __forceinline__ int lane_id() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}
#define LANE (lane_id())
// A workgroup is exactly one wavefront, and a wavefront's LDS instructions execute
// in issue order, so cross-lane LDS hand-offs need only a compiler-level barrier
// (no s_barrier, and no s_waitcnt on outstanding global stores).
#define SYNC() __builtin_amdgcn_wave_barrier()

// ------------------------------------------------------------------------ //
// wave helpers
// ------------------------------------------------------------------------ //
// DPP row reductions (gfx9 family): quad_perm, row_half_mirror, row_mirror, then
// row_bcast15 / row_bcast31 carry the partial results up to lane 63.  With every row
// enabled (the in-row patterns, where each lane's source exists) the move has no "old"
// operand (mov_dpp, bound_ctrl): the compiler then folds it into the consuming add /
// integer min / max / or as one v_*_dpp instruction -- with update_dpp(old = x) every
// step was a copy, the DPP move and the operation.  The masked broadcasts keep x in the
// rows they skip.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i(int x) {
  if (ROWMASK == 0xF) return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);
  return __builtin_amdgcn_update_dpp(x, x, CTRL, ROWMASK, 0xF, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(dpp_i<CTRL, ROWMASK>(__float_as_int(x)));
}
// fp32 <-> a signed integer of the same order (for max / min reductions on the integer
// DPP path: fmaxf on a DPP operand also re-canonicalises it, two more instructions per
// step).  Finite values and infinities only; an involution.
__device__ __forceinline__ int f2ord(float f) {
  const int b = __float_as_int(f + 0.0f);  // (-0 -> +0: the two compare equal as floats)
  return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float ord2f(int k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }
// Sums: quad, half-row, row sums by DPP, then rows carried up to lane 63 (each lane
// contributes exactly once), broadcast with readlane.  The two row broadcasts run with
// every row enabled, so they fold into their operation too: rows 0-2 may read a source
// that does not exist, but lane 63 reads only lane 47 (row 2's sum) and then lane 31
// (rows 0 + 1), whatever the other rows hold -- and only lane 63 is read.
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1, 0xF>(v);
  v += dpp_f<0x4E, 0xF>(v);
  v += dpp_f<0x141, 0xF>(v);
  v += dpp_f<0x140, 0xF>(v);
  v += dpp_f<0x142, 0xF>(v);
  v += dpp_f<0x143, 0xF>(v);
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ int wave_sum_i(int v) {
  v += dpp_i<0xB1, 0xF>(v);
  v += dpp_i<0x4E, 0xF>(v);
  v += dpp_i<0x141, 0xF>(v);
  v += dpp_i<0x140, 0xF>(v);
  v += dpp_i<0x142, 0xF>(v);
  v += dpp_i<0x143, 0xF>(v);
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_max_i(int m) {
  m = max(m, dpp_i<0xB1, 0xF>(m));
  m = max(m, dpp_i<0x4E, 0xF>(m));
  m = max(m, dpp_i<0x141, 0xF>(m));
  m = max(m, dpp_i<0x140, 0xF>(m));
  m = max(m, dpp_i<0x142, 0xF>(m));
  m = max(m, dpp_i<0x143, 0xF>(m));
  return __builtin_amdgcn_readlane(m, 63);
}
__device__ __forceinline__ float wave_max_f(float m) { return ord2f(wave_max_i(f2ord(m))); }
__device__ __forceinline__ int wave_min_i(int m) {
  m = min(m, dpp_i<0xB1, 0xF>(m));
  m = min(m, dpp_i<0x4E, 0xF>(m));
  m = min(m, dpp_i<0x141, 0xF>(m));
  m = min(m, dpp_i<0x140, 0xF>(m));
  m = min(m, dpp_i<0x142, 0xF>(m));
  m = min(m, dpp_i<0x143, 0xF>(m));
  return __builtin_amdgcn_readlane(m, 63);
}
// index of the first (lowest-index) maximum over lanes' (best, index) pairs
__device__ __forceinline__ int wave_argmax_first(float best, int bi) {
  float vmax = wave_max_f(best);
  return wave_min_i(best == vmax ? bi : 0x7fffffff);
}

// Inclusive prefix sum over the wave by DPP: Hillis-Steele within each 16-lane row
// (row_shr 1, 2, 4, 8 with zero fill), then row_bcast:15 / row_bcast:31 carry the
// row totals upwards.  No LDS round trip.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i0(int x) {  // lanes without a source read 0
  if (ROWMASK == 0xF) return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, true);  // (bound_ctrl: 0)
  return __builtin_amdgcn_update_dpp(0, x, CTRL, ROWMASK, 0xF, false);
}
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += dpp_i0<0x111, 0xF>(x);  // row_shr:1
  x += dpp_i0<0x112, 0xF>(x);  // row_shr:2
  x += dpp_i0<0x114, 0xF>(x);  // row_shr:4
  x += dpp_i0<0x118, 0xF>(x);  // row_shr:8
  x += dpp_i0<0x142, 0xA>(x);  // row_bcast:15 -> rows 1, 3
  x += dpp_i0<0x143, 0xC>(x);  // row_bcast:31 -> rows 2, 3
  return x;
}
// exclusive prefix sum over lanes
__device__ __forceinline__ int wave_excl_scan(int v) { return wave_incl_scan(v) - v; }

// ------------------------------------------------------------------------ //
// small math
// ------------------------------------------------------------------------ //
__device__ __forceinline__ float dot3(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
__device__ __forceinline__ void cross3(float* r, const float* a, const float* b) {
  float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ void sub3(float* r, const float* a, const float* b) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
__device__ __forceinline__ float norm3(const float* a) { return sqrtf(dot3(a, a)); }
__device__ __forceinline__ void normalize3(float* a) {
  float n = norm3(a);
  if (n > 1e-20f) { float s = 1.0f / n; a[0] *= s; a[1] *= s; a[2] *= s; }
}
__device__ __forceinline__ void matvec3(float* r, const float* R, const float* v) {
  float t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  float t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  float t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ void mattvec3(float* r, const float* R, const float* v) {
  float t0 = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  float t1 = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  float t2 = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ __forceinline__ void matmul3(float* r, const float* A, const float* B) {
  float t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = t[i];
}
__device__ __forceinline__ void quat2mat(float* R, const float* q) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
__device__ __forceinline__ void quatmul(float* r, const float* a, const float* b) {
  float t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
__device__ __forceinline__ void quatnorm(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < 1e-20f) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  float s = 1.0f / n;
  q[0] *= s; q[1] *= s; q[2] *= s; q[3] *= s;
}
// spatial algebra: [angular; linear] about the root-com frame origin
__device__ __forceinline__ void mul_inert(float* r, const float* I, const float* v) {
  const float* w = v;
  const float* l = v + 3;
  const float* mc = I + 6;
  float m = I[9];
  r[0] = I[0] * w[0] + I[3] * w[1] + I[4] * w[2] + (mc[1] * l[2] - mc[2] * l[1]);
  r[1] = I[3] * w[0] + I[1] * w[1] + I[5] * w[2] + (mc[2] * l[0] - mc[0] * l[2]);
  r[2] = I[4] * w[0] + I[5] * w[1] + I[2] * w[2] + (mc[0] * l[1] - mc[1] * l[0]);
  r[3] = m * l[0] - (mc[1] * w[2] - mc[2] * w[1]);
  r[4] = m * l[1] - (mc[2] * w[0] - mc[0] * w[2]);
  r[5] = m * l[2] - (mc[0] * w[1] - mc[1] * w[0]);
}
__device__ __forceinline__ void cross_motion(float* r, const float* v, const float* m) {
  float a[3], b[3], c[3];
  cross3(a, v, m);
  cross3(b, v, m + 3);
  cross3(c, v + 3, m);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
__device__ __forceinline__ void cross_force(float* r, const float* v, const float* f) {
  float a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
__device__ __forceinline__ float dot6(const float* a, const float* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

// ------------------------------------------------------------------------ //
// per-env context
// ------------------------------------------------------------------------ //
// The model's dimensions and the LDS layout come either from the launch (generic
// kernel) or from a compile-time model specialization (dx_specs.inc, generated by
// build.py for the shipped scenes): then every LDS offset is an immediate, loop
// bounds are constants, and far fewer scalar registers stay live (the generic
// kernel spills its ~60 layout/dimension scalars into VGPR lanes).
#define DX_DIMS(X) X(nq) X(nv) X(nbody) X(njnt) X(nu) X(ntendon) X(nsite) X(nlevel) X(nroot) \
  X(nfric) X(nlimj) X(nlimt) X(nbpair) X(any_damping) X(disable_contact) X(iterations) X(solver)
struct SpecRT {
  static constexpr bool reach_task = false;  // (the generic kernel: no fused reach sampling pass)
};
// Stages take the model through c.mdl().  (Laundering that reference per stage, so
// each stage re-loads its table pointers instead of the kernel keeping ~100 of them
// live, cut the SGPR spills 408 -> 331 but not the step time; it is a plain
// reference.)
template <class SP>
struct CtxT {
  static constexpr bool is_spec = true;  // a scene specialization (dims and layout constant)
  const DevModel& m;
  static constexpr Lds L = SP::L;
#define DX_X(n) static constexpr int n = SP::n;
  DX_DIMS(DX_X)
#undef DX_X
  float* S;
  int* I;  // misc ints
  unsigned long long* stage_acc;
  float4* sep = nullptr;  // this env's separating-direction cache (DX_SEP_SLOTS), or null
  int np_wide = DX_WAVE / 8;  // narrowphase: 4-lane groups above this many candidates
  bool defer = false;         // a full contact pool defers the physics step (I_DEFER)
  int defer_at = DX_NCON_MAX; // ... or more contacts than this (DX_DEFER_AT: tests, probes)
  __device__ CtxT(const DevModel& m_, const Lds&, float* S_, int* I_, unsigned long long* acc)
      : m(m_), S(S_), I(I_), stage_acc(acc) {}
  __device__ float* f(int off) const { return S + off; }
  __device__ const DevModel& mdl() const { return m; }
};
template <>
struct CtxT<SpecRT> {
  static constexpr bool is_spec = false;
  const DevModel& m;
  const Lds& L;
#define DX_X(n) int n;
  DX_DIMS(DX_X)
#undef DX_X
  float* S;
  int* I;
  unsigned long long* stage_acc;
  float4* sep = nullptr;
  int np_wide = DX_WAVE / 8;
  bool defer = false;
  int defer_at = DX_NCON_MAX;
  __device__ CtxT(const DevModel& m_, const Lds& L_, float* S_, int* I_, unsigned long long* acc)
      : m(m_), L(L_),
#define DX_X(n) n(m_.n),
        DX_DIMS(DX_X)
#undef DX_X
        S(S_), I(I_), stage_acc(acc) {}
  __device__ float* f(int off) const { return S + off; }
  __device__ const DevModel& mdl() const { return m; }
};
// Per-stage cycle accounting (runtime-gated by DevBatch::stage_acc, lane 0 only).
enum {
  ST_KIN = 0, ST_CRB, ST_BROAD, ST_MID, ST_NARROW, ST_CON, ST_VEL, ST_SMOOTH, ST_NEWTON_EVAL,
  ST_NEWTON_GRAD, ST_NEWTON_HESS, ST_NEWTON_CHOL, ST_NEWTON_LS, ST_QFRC, ST_EULER, ST_OBSERVE, ST_IO,
  ST_MATVEC, ST_NP_MPR, ST_JACVEC,
  CNT_PLANE_BOX = 20, CNT_PLANE_CONVEX, CNT_CAPSULE, CNT_MPR, CNT_SUPPORT, CNT_MPR_HIT,
  CNT_MPR_MAXIT, CNT_NEWTON_IT, CNT_LS_IT, CNT_SOLVE, CNT_NEFC, CNT_NP_TRIPS, CNT_BROAD_KEEP, CNT_MID_PAIRS,
  CNT_MID_KEEP,  // event counters, not cycles
  CNT_QWAIT,     // substep queue: cycles a claimed task waited for the env's previous physics step
  // the narrowphase loop's trips split (DX_NP_MARKS builds only, dx_step.hip NpClock): loop
  // bookkeeping and contact writes, new pairs' set-up, a support's cell load up to its
  // first use, the support's reductions and world transform, the portal arithmetic
  ST_NP_LOOP = 36, ST_NP_FRESH, ST_NP_SUPLOAD, ST_NP_SUPRED, ST_NP_PORTAL
};
// The accumulators are this env's own global slots, updated by no-return atomics: a
// read-modify-write would put a memory round trip on the wave's path at every mark
// (and every in-loop count), charged to the stage after it.
template <class P>
__device__ __forceinline__ void stage_add(P p, unsigned long long v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class Ctx>
__device__ __forceinline__ void stage_mark(const Ctx& c, int k) {
  if (c.stage_acc && LANE == 0) {
    unsigned long long t = __builtin_amdgcn_s_memtime();
    unsigned long long* last = (unsigned long long*)(c.I + 10);
    stage_add(c.stage_acc + k, t - *last);
    *last = t;
  }
}
#ifndef DX_NP_MARKS
#define DX_NP_MARKS 0
#endif
template <class Ctx>
__device__ __forceinline__ void stage_count(const Ctx& c, int k, int n = 1) {
  if (c.stage_acc && LANE == 0) stage_add(c.stage_acc + k, (unsigned long long)n);
}
// misc int slots
// I_OVF: capacity bits of the substep (1 candidates, 2 contacts, 4 Jacobian dofs, 8 rows);
// I_NRAW: most contacts any collision pass of the substep found (before the DX_NCON_MAX cap)
// I_DEFER: the substep's contacts exceed this tier's pool; it is redone by the overflow tier
enum { I_NCON = 0, I_NEFC, I_NCAND, I_NBC, I_OVF, I_NITER, I_WATCH, I_NLIM, I_NRAW, I_DEFER, I_NINT };
// (words 10-11: the stage clock; carried between an env's physics-step tasks:)
// I_NSTEP: physics steps since the env's last mj_resetData (the fp64 time's addition count);
// I_FLAGS: bit 0 -- a physics step of this control step diverged and reset the env
enum { I_NSTEP = 12, I_FLAGS = 13 };

// ------------------------------------------------------------------------ //
// position stage
// ------------------------------------------------------------------------ //
// Per-body model data of lane b = body (nbody <= 64), loaded in one memory round trip
// at the start of a tree pass (dx_api.hip body_rec); the level loops then touch only
// LDS.  Joint fields are the body's first joint (Shadow / Adroit bodies have <= 1).
struct BodyRec {
  int parent, depth, ja, jn, jtype, qadr, dofadr, dofnum, jdof, rootidx;
  float pos[3], quat[4], ipos[3], jpos[3], jaxis[3], q0, mass, inert[3];
};
template <class Ctx>
__device__ __forceinline__ bool load_body(const Ctx& c, BodyRec& r) {
  const int b = LANE;
  const bool act = b >= 1 && b < c.nbody;
  const DXG float4* R = c.mdl().body_rec + 8 * (act ? b : 0);
  const float4 a = R[0], p = R[1], q = R[2], i = R[3], jp = R[4], jx = R[5], d = R[6], in = R[7];
  r.inert[0] = in.x; r.inert[1] = in.y; r.inert[2] = in.z;
  r.parent = __float_as_int(a.x);
  r.depth = act ? __float_as_int(a.y) : -1;
  r.ja = __float_as_int(a.z);
  r.jn = __float_as_int(a.w);
  r.pos[0] = p.x; r.pos[1] = p.y; r.pos[2] = p.z;
  r.jtype = __float_as_int(p.w);
  r.quat[0] = q.x; r.quat[1] = q.y; r.quat[2] = q.z; r.quat[3] = q.w;
  r.ipos[0] = i.x; r.ipos[1] = i.y; r.ipos[2] = i.z;
  r.rootidx = __float_as_int(i.w);
  r.jpos[0] = jp.x; r.jpos[1] = jp.y; r.jpos[2] = jp.z;
  r.qadr = __float_as_int(jp.w);
  r.jaxis[0] = jx.x; r.jaxis[1] = jx.y; r.jaxis[2] = jx.z;
  r.q0 = jx.w;
  r.dofadr = __float_as_int(d.x);
  r.dofnum = __float_as_int(d.y);
  r.mass = d.z;
  r.jdof = __float_as_int(d.w);
  return act;
}

// Forward kinematics (mj_kinematics) as chain compositions instead of one tree level
// after another.  Phase 1 (lane = body, all bodies at once): the body's pose in its
// parent's frame, L_b = body offset o joint rotations (the sincos / normalise work),
// as an 8-float record {pos, parent, quat} in the xmat slots, plus every joint's
// anchor/axis in the body's own frame.  Phase 2: x_b = L_root o ... o L_parent o L_b,
// walking the parent links upward (p <- L_a.pos + L_a.rot p, q <- L_a.quat q): a
// chain of cheap compositions with no barrier per level.  Phase 3: rotation matrix,
// inertial frame, joint anchors and axes in the world frame.
template <class Ctx>
__device__ __forceinline__ void kinematics_impl(const Ctx& c, const BodyRec& br, const bool act) {
  const DevModel& m = c.mdl();
  float* qpos = c.f(c.L.qpos);
  float* xpos = c.f(c.L.xpos);
  float* xquat = c.f(c.L.xquat);
  float* xmat = c.f(c.L.xmat);
  float* xipos = c.f(c.L.xipos);
  float* xanchor = c.f(c.L.xanchor);
  float* xaxis = c.f(c.L.xaxis);
  const int b = LANE, ja = br.ja, jn = br.jn;
  const bool fr = act && jn > 0 && br.jtype == DXJ_FREE;
  float lp[3] = {br.pos[0], br.pos[1], br.pos[2]};
  float lq[4] = {br.quat[0], br.quat[1], br.quat[2], br.quat[3]};
  if (act) {
    if (fr) {
      const float* q = qpos + br.qadr;
      lp[0] = q[0]; lp[1] = q[1]; lp[2] = q[2];
      lq[0] = q[3]; lq[1] = q[4]; lq[2] = q[5]; lq[3] = q[6];
      quatnorm(lq);
    } else {
      for (int jj = 0; jj < jn; jj++) {
        const int j = ja + jj;
        float jp[3], ja3[3], q0;
        int qa;
        if (jj == 0) {
          for (int k = 0; k < 3; k++) { jp[k] = br.jpos[k]; ja3[k] = br.jaxis[k]; }
          qa = br.qadr;
          q0 = br.q0;
        } else {
          for (int k = 0; k < 3; k++) { jp[k] = m.jnt_pos[3 * j + k]; ja3[k] = m.jnt_axis[3 * j + k]; }
          qa = m.jnt_qposadr[j];
          q0 = m.qpos0[qa];
        }
        float R[9], t[3];
        quat2mat(R, lq);
        matvec3(t, R, jp);
        const float anc[3] = {t[0] + lp[0], t[1] + lp[1], t[2] + lp[2]};
        if (jj + 1 < jn) {  // anchor / axis in the parent frame, moved to the body frame below
          float ax[3];
          matvec3(ax, R, ja3);
          for (int k = 0; k < 3; k++) { xanchor[3 * j + k] = anc[k]; xaxis[3 * j + k] = ax[k]; }
        }
        float sn, co;
        sincosf(0.5f * (qpos[qa] - q0), &sn, &co);
        const float ql[4] = {co, ja3[0] * sn, ja3[1] * sn, ja3[2] * sn};
        quatmul(lq, lq, ql);
        quatnorm(lq);
        quat2mat(R, lq);
        matvec3(t, R, jp);
        lp[0] = anc[0] - t[0]; lp[1] = anc[1] - t[1]; lp[2] = anc[2] - t[2];
      }
      if (jn > 1) {  // all but the last joint: parent frame -> body frame (L_b^-1)
        float R[9];
        quat2mat(R, lq);
        for (int jj = 0; jj + 1 < jn; jj++) {
          const int j = ja + jj;
          float d[3] = {xanchor[3 * j] - lp[0], xanchor[3 * j + 1] - lp[1], xanchor[3 * j + 2] - lp[2]};
          float ab[3], xb[3];
          mattvec3(ab, R, d);
          mattvec3(xb, R, xaxis + 3 * j);
          for (int k = 0; k < 3; k++) { xanchor[3 * j + k] = ab[k]; xaxis[3 * j + k] = xb[k]; }
        }
      }
    }
    float* rec = xmat + 9 * b;
    rec[0] = lp[0]; rec[1] = lp[1]; rec[2] = lp[2];
    rec[3] = __int_as_float(br.parent);
    rec[4] = lq[0]; rec[5] = lq[1]; rec[6] = lq[2]; rec[7] = lq[3];
  }
  SYNC();
  float xp[3] = {lp[0], lp[1], lp[2]}, xq[4] = {lq[0], lq[1], lq[2], lq[3]};
  if (act) {
    int a = br.parent;
    while (a > 0) {
      const float* r = xmat + 9 * a;
      const float ap[3] = {r[0], r[1], r[2]};
      const int an = __float_as_int(r[3]);
      const float aq[4] = {r[4], r[5], r[6], r[7]};
      // xp <- ap + rot(aq) xp ; xq <- aq xq
      float t[3];
      t[0] = 2.f * (aq[2] * xp[2] - aq[3] * xp[1]);
      t[1] = 2.f * (aq[3] * xp[0] - aq[1] * xp[2]);
      t[2] = 2.f * (aq[1] * xp[1] - aq[2] * xp[0]);
      const float v0 = xp[0] + aq[0] * t[0] + (aq[2] * t[2] - aq[3] * t[1]);
      const float v1 = xp[1] + aq[0] * t[1] + (aq[3] * t[0] - aq[1] * t[2]);
      const float v2 = xp[2] + aq[0] * t[2] + (aq[1] * t[1] - aq[2] * t[0]);
      xp[0] = ap[0] + v0; xp[1] = ap[1] + v1; xp[2] = ap[2] + v2;
      quatmul(xq, aq, xq);
      a = an;
    }
    quatnorm(xq);
  }
  SYNC();
  if (LANE == 0) {
    xpos[0] = xpos[1] = xpos[2] = 0;
    xquat[0] = 1; xquat[1] = xquat[2] = xquat[3] = 0;
    for (int k = 0; k < 9; k++) xmat[k] = (k % 4 == 0) ? 1.f : 0.f;
    xipos[0] = xipos[1] = xipos[2] = 0;
  }
  if (act) {
    float R[9], t[3];
    quat2mat(R, xq);
    for (int e = 0; e < 3; e++) xpos[3 * b + e] = xp[e];
    for (int e = 0; e < 4; e++) xquat[4 * b + e] = xq[e];
    for (int e = 0; e < 9; e++) xmat[9 * b + e] = R[e];
    matvec3(t, R, br.ipos);
    for (int e = 0; e < 3; e++) xipos[3 * b + e] = xp[e] + t[e];
    if (fr) {
      xanchor[3 * ja] = xp[0]; xanchor[3 * ja + 1] = xp[1]; xanchor[3 * ja + 2] = xp[2];
      xaxis[3 * ja] = 0; xaxis[3 * ja + 1] = 0; xaxis[3 * ja + 2] = 1;
    } else {
      for (int jj = 0; jj < jn; jj++) {
        const int j = ja + jj;
        float ab[3], xb[3];
        if (jj + 1 == jn) {  // the last joint's anchor and axis are its own, in the body frame
          if (jj == 0) {
            for (int k = 0; k < 3; k++) { ab[k] = br.jpos[k]; xb[k] = br.jaxis[k]; }
          } else {
            for (int k = 0; k < 3; k++) { ab[k] = m.jnt_pos[3 * j + k]; xb[k] = m.jnt_axis[3 * j + k]; }
          }
        } else {
          for (int k = 0; k < 3; k++) { ab[k] = xanchor[3 * j + k]; xb[k] = xaxis[3 * j + k]; }
        }
        float aw[3], xw[3];
        matvec3(aw, R, ab);
        matvec3(xw, R, xb);
        for (int k = 0; k < 3; k++) { xanchor[3 * j + k] = xp[k] + aw[k]; xaxis[3 * j + k] = xw[k]; }
      }
    }
  }
  SYNC();
}

template <class Ctx>
__device__ __forceinline__ void kinematics(const Ctx& c) {
  BodyRec br;
  const bool act = load_body(c, br);
  kinematics_impl(c, br, act);
}

// Per-lane model data of com_pos beyond the body record: the body's inertia frame
// (lane = body) and the dof record (lane = dof).  Loaded with the body record before
// kinematics, so no model-table round trip follows a barrier.
struct ComPre {
  float imat[9];
  float4 dof0;
};
template <class Ctx>
__device__ __forceinline__ void load_com_pre(const Ctx& c, ComPre& p) {
  const DevModel& m = c.mdl();
  const int b = min(LANE, c.nbody - 1);
#pragma unroll
  for (int k = 0; k < 9; k++) p.imat[k] = m.body_imat[9 * b + k];
  p.dof0 = m.dof_rec[2 * min(LANE, c.nv - 1)];
}

template <class Ctx>
__device__ __forceinline__ void com_pos_impl(const Ctx& c, const BodyRec& br, const bool act, const ComPre& pre) {
  const DevModel& m = c.mdl();
  float* xipos = c.f(c.L.xipos);
  float* xmat = c.f(c.L.xmat);
  float* rcom = c.f(c.L.rcom);
  // subtree com of every root (only roots are needed as com-frame origins); lane = body
  for (int r = 0; r < c.nroot; r++) {
    float s0 = 0, s1 = 0, s2 = 0, sm = 0;
    if (act && br.rootidx == r) {
      const int b = LANE;
      const float ms = br.mass;
      s0 = ms * xipos[3 * b]; s1 = ms * xipos[3 * b + 1]; s2 = ms * xipos[3 * b + 2]; sm = ms;
    }
    s0 = wave_sum(s0); s1 = wave_sum(s1); s2 = wave_sum(s2); sm = wave_sum(sm);
    if (LANE == 0) {
      int rb = m.root_body[r];
      if (sm > 1e-15f) { rcom[3 * r] = s0 / sm; rcom[3 * r + 1] = s1 / sm; rcom[3 * r + 2] = s2 / sm; }
      else { rcom[3 * r] = xipos[3 * rb]; rcom[3 * r + 1] = xipos[3 * rb + 1]; rcom[3 * r + 2] = xipos[3 * rb + 2]; }
    }
  }
  SYNC();
  float* cinert = c.f(c.L.cinert);
  if (act) {
    const int b = LANE;
    float Rb[9];
    matmul3(Rb, xmat + 9 * b, pre.imat);
    const float* I = br.inert;
    float mass = br.mass;
    const float* rc = rcom + 3 * br.rootidx;
    float off[3] = {xipos[3 * b] - rc[0], xipos[3 * b + 1] - rc[1], xipos[3 * b + 2] - rc[2]};
    float Iw[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        Iw[3 * i + j] = Rb[3 * i] * I[0] * Rb[3 * j] + Rb[3 * i + 1] * I[1] * Rb[3 * j + 1] +
                        Rb[3 * i + 2] * I[2] * Rb[3 * j + 2];
    float dd = dot3(off, off);
    float* ci = cinert + 10 * b;
    ci[0] = Iw[0] + mass * (dd - off[0] * off[0]);
    ci[1] = Iw[4] + mass * (dd - off[1] * off[1]);
    ci[2] = Iw[8] + mass * (dd - off[2] * off[2]);
    ci[3] = Iw[1] - mass * off[0] * off[1];
    ci[4] = Iw[2] - mass * off[0] * off[2];
    ci[5] = Iw[5] - mass * off[1] * off[2];
    ci[6] = mass * off[0]; ci[7] = mass * off[1]; ci[8] = mass * off[2];
    ci[9] = mass;
  }
  float* cdof = c.f(c.L.cdof);
  float* xanchor = c.f(c.L.xanchor);
  float* xaxis = c.f(c.L.xaxis);
  for (int d = LANE; d < c.nv; d += DX_WAVE) {
    const float4 dr = pre.dof0;
    const int b = __float_as_int(dr.x), j = __float_as_int(dr.y), tk = __float_as_int(dr.w);
    const float* rc = rcom + 3 * __float_as_int(dr.z);
    float off[3] = {rc[0] - xanchor[3 * j], rc[1] - xanchor[3 * j + 1], rc[2] - xanchor[3 * j + 2]};
    float* cd = cdof + 6 * d;
    if ((tk & 255) == DXJ_FREE) {
      int k = tk >> 8;
      if (k < 3) {
        for (int e = 0; e < 6; e++) cd[e] = 0;
        cd[3 + k] = 1;
      } else {
        const float* R = xmat + 9 * b;
        float ax[3] = {R[k - 3], R[3 + k - 3], R[6 + k - 3]};
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(cd + 3, ax, off);
      }
    } else {
      const float* ax = xaxis + 3 * j;
      cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
      cross3(cd + 3, ax, off);
    }
  }
  SYNC();
}

template <class Ctx>
__device__ __forceinline__ void com_pos(const Ctx& c) {
  BodyRec br;
  const bool act = load_body(c, br);
  ComPre pre;
  load_com_pre(c, pre);
  com_pos_impl(c, br, act, pre);
}
// mj_kinematics + mj_comPos with every model-table load issued up front
template <class Ctx>
__device__ __forceinline__ void kin_com(const Ctx& c) {
  BodyRec br;
  const bool act = load_body(c, br);
  ComPre pre;
  load_com_pre(c, pre);
  kinematics_impl(c, br, act);
  com_pos_impl(c, br, act, pre);
}

// Tendon wrap tables of lane t = LANE (first two wraps), loaded before kinematics.
struct TenPre {
  int adr, num, q0, q1, atrn, aidx;
  float c0, c1, ag;
};
template <class Ctx>
__device__ __forceinline__ void load_ten_pre(const Ctx& c, TenPre& p) {
  const DevModel& m = c.mdl();
  const bool ok = LANE < c.ntendon;
  const int t = ok ? LANE : 0;
  p.adr = ok ? m.tendon_adr[t] : 0;
  p.num = ok ? m.tendon_num[t] : 0;
  p.c0 = p.num > 0 ? m.wrap_coef[p.adr] : 0.f;
  p.q0 = p.num > 0 ? m.wrap_qadr[p.adr] : 0;
  p.c1 = p.num > 1 ? m.wrap_coef[p.adr + 1] : 0.f;
  p.q1 = p.num > 1 ? m.wrap_qadr[p.adr + 1] : 0;
  // actuator lane: gear, transmission, and its joint's qpos address or its tendon
  const bool aok = LANE < c.nu;
  const int a = aok ? LANE : 0;
  p.ag = aok ? m.actuator_gear[a] : 0.f;
  p.atrn = aok ? m.actuator_trntype[a] : 1;
  const int id = aok ? m.actuator_trnid[a] : 0;
  p.aidx = p.atrn == 0 ? m.jnt_qposadr[id] : id;
}
template <class Ctx>
__device__ __forceinline__ void tendon_lengths(const Ctx& c, const TenPre& p) {
  const DevModel& m = c.mdl();
  float* qpos = c.f(c.L.qpos);
  float* tl = c.f(c.L.ten_len);
  for (int t = LANE; t < c.ntendon; t += DX_WAVE) {
    const bool own = t == LANE;  // first pass: the preloaded wraps
    const int adr = own ? p.adr : m.tendon_adr[t], num = own ? p.num : m.tendon_num[t];
    float len = 0;
    for (int w = 0; w < num; w++) {
      const float wc = (own && w == 0) ? p.c0 : ((own && w == 1) ? p.c1 : m.wrap_coef[adr + w]);
      const int wq = (own && w == 0) ? p.q0 : ((own && w == 1) ? p.q1 : m.wrap_qadr[adr + w]);
      len += wc * qpos[wq];
    }
    tl[t] = len;
  }
  SYNC();
  // actuator lengths (position actuators' bias), lane = actuator (nu <= 64)
  float* al = c.f(c.L.act_len);
  if (LANE < c.nu) al[LANE] = p.atrn == 0 ? p.ag * qpos[p.aidx] : p.ag * tl[p.aidx];
}

// Symmetric nv x nv matrices (M, the Newton Hessian, Cholesky factors) are stored
// as packed lower triangles, row-major: (i, j <= i) -> ti(i) + j.
__device__ __forceinline__ int ti(int i) { return (i * (i + 1)) >> 1; }

template <class Ctx>
__device__ __forceinline__ void crb_mass(const Ctx& c) {
  const DevModel& m = c.mdl();
  int nv = c.nv;
  float* crb = c.f(c.L.scr);
  float* cinert = c.f(c.L.cinert);
  float* M = c.f(c.L.M);
  float* cdof = c.f(c.L.cdof);
  // model records first: their L2 round trips overlap the level passes below
  // (a load after a barrier is a full round trip on the wave's critical path)
  BodyRec br;
  const bool act = load_body(c, br);
  const int i0 = min(LANE, nv - 1);  // nv <= 64 (model check): one dof per lane
  const float4 d0r = m.dof_rec[2 * i0], d1r = m.dof_rec[2 * i0 + 1];
  for (int k = LANE; k < 10 * c.nbody; k += DX_WAVE) crb[k] = cinert[k];
  for (int k = LANE; k < ti(nv); k += DX_WAVE) M[k] = 0;
  SYNC();
  for (int lv = c.nlevel; lv >= 2; lv--) {
    if (act && br.depth == lv && br.parent > 0)
      for (int e = 0; e < 10; e++) atomicAdd(crb + 10 * br.parent + e, crb[10 * LANE + e]);
    SYNC();
  }
  // row i: j over the dof's ancestors (incl. itself), a bit mask from dof_rec
  for (int i = LANE; i < nv; i += DX_WAVE) {
    const float4 d0 = d0r, d1 = d1r;
    float f[6];
    mul_inert(f, crb + 10 * __float_as_int(d0.x), cdof + 6 * i);
    uint64_t anc = (uint64_t)(uint32_t)__float_as_int(d1.z) | ((uint64_t)(uint32_t)__float_as_int(d1.w) << 32);
    while (anc) {
      int j = __ffsll((long long)anc) - 1;
      anc &= anc - 1;
      M[ti(i) + j] = dot6(cdof + 6 * j, f);
    }
    M[ti(i) + i] += d1.x;
  }
  SYNC();
}

// In-place dense Cholesky (lower, row-major) of the n x n matrix A, one wave.
// Column k: lanes scale the sub-diagonal of column k, then update the trailing
// lower triangle; entry t of a w x w trailing triangle maps to (ii, jj) through
// the LDS table tri[t] = ii << 8 | jj (built once per launch), so the update is
// branch-free and balanced over the 64 lanes.  Two barriers per column.
__device__ __forceinline__ void wave_cholesky(float* A, int n, const unsigned short* tri) {
  for (int k = 0; k < n; k++) {
    float d = sqrtf(fmaxf(A[ti(k) + k], 1e-30f));
    float inv = 1.0f / d;
    for (int i = k + 1 + LANE; i < n; i += DX_WAVE) A[ti(i) + k] *= inv;
    SYNC();
    if (LANE == 0) A[ti(k) + k] = d;
    int w = n - k - 1;
    int tot = w * (w + 1) / 2;
    for (int t = LANE; t < tot; t += DX_WAVE) {
      int e = tri[t];
      int i = k + 1 + (e >> 8), j = k + 1 + (e & 255);
      A[ti(i) + j] -= A[ti(i) + k] * A[ti(j) + k];
    }
    SYNC();
  }
}
// Solve (L L^T) x = b; x holds b on entry (LDS).  Lane i keeps x_i in a register;
// the dependent chain uses readlane broadcasts and no barriers.  n <= 64.
__device__ __forceinline__ void wave_chol_solve(const float* A, float* x, int n) {
  float xi = LANE < n ? x[LANE] : 0.f;
  for (int k = 0; k < n; k++) {
    float lik = LANE > k && LANE < n ? A[ti(LANE) + k] : 0.f;
    float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xi), k)) / A[ti(k) + k];
    if (LANE == k) xi = v;
    xi -= lik * v;
  }
  for (int k = n - 1; k >= 0; k--) {
    float lki = LANE < k ? A[ti(k) + LANE] : 0.f;
    float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xi), k)) / A[ti(k) + k];
    if (LANE == k) xi = v;
    xi -= lki * v;
  }
  SYNC();
  if (LANE < n) x[LANE] = xi;
  SYNC();
}

// Cholesky solve for n <= 32 on the matrix cores.  The matrix, padded to 32 x 32 with
// an identity block, lives in the 16 accumulator VGPRs of v_mfma_f32_32x32x2_f32
// (lane l, VGPR v holds C[8 (v/4) + 4 (l/32) + v%4][l%32]; probe:
// tools/probes/mfma_layout.hip).  Right-looking, two columns per step: rows k, k+1
// are one VGPR pair in one half-wave, broadcast to both halves by v_permlane32_swap
// (symmetry makes them the columns); the 2 x 2 diagonal block is factored from
// three readlanes; the panel (L[:,k], L[:,k+1]) is the 32 x 2 A operand and its
// transpose the B operand of ONE MFMA that applies the rank-2 update to the whole
// trailing matrix.  16 steps instead of 32 columns of ~31 readlanes each.  The
// substitutions then run on lane rows of L (lane i holds L[i][k] in Lr[k]) with
// readlane/writelane; the backward one reads L's columns after an LDS transpose
// through T (packed, may alias A).
// A (+ hs*dadd on the diagonal, if dadd) -> x = A^-1 x.
__device__ __forceinline__ float rl(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
// llvm.amdgcn.writelane (no clang builtin in this toolchain)
extern "C" __device__ int dx_writelane_i32(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");
__device__ __forceinline__ float wl(float v, float s, int k) {  // v with lane k := s
  return __int_as_float(dx_writelane_i32(__float_as_int(s), k, __float_as_int(v)));
}
typedef float dx_f16v __attribute__((ext_vector_type(16)));
typedef float dx_f2v __attribute__((ext_vector_type(2)));
// v with its lower (up = false) or upper (up = true) half-wave copied into both halves
__device__ __forceinline__ float half_dup(float v, bool up) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(up ? r[1] : r[0]);
}
__device__ __forceinline__ void mfma_chol_solve32(const float* A, int n, float dj, float* x, float* T) {
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  dx_f16v C;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    const int ra = max(i, j), rb = min(i, j);
    const bool in = i < n && j < n;
    float e = in ? A[ti(ra) + rb] : (i == j ? 1.f : 0.f);
    if (i == j && in) e += dj;
    C[v] = e;
  }
  float b = l < n ? x[l] : 0.f;
  SYNC();  // A may alias T
  float Lr[32];  // lane j: L[j][k], strictly below the diagonal
  float dinv = 0.f;
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C[vk], up), rk1 = half_dup(C[vk + 1], up);  // C[k][j], C[k+1][j]
    const float i11 = __builtin_amdgcn_rsqf(fmaxf(rl(C[vk], k + (up ? 32 : 0)), 1e-30f));
    const float l21 = rl(C[vk + 1], k + (up ? 32 : 0)) * i11;
    const float i22 = __builtin_amdgcn_rsqf(fmaxf(rl(C[vk + 1], k + 1 + (up ? 32 : 0)) - l21 * l21, 1e-30f));
    dinv = wl(dinv, i11, k);
    dinv = wl(dinv, i22, k + 1);
    const float lk = rk * i11;                  // L[j][k]   (j > k)
    const float lk1 = (rk1 - lk * l21) * i22;   // L[j][k+1] (j > k + 1)
    Lr[k] = j > k ? lk : 0.f;
    Lr[k + 1] = j > k + 1 ? lk1 : 0.f;
    const float p = j > k + 1 ? (hi ? lk1 : lk) : 0.f;  // panel: A[j][hi], B[hi][j]
    C = __builtin_amdgcn_mfma_f32_32x32x2f32(-p, p, C, 0, 0, 0);
  }
  // strictly-lower row -> T (packed).  Lanes with nothing to store write T[0], the
  // (0, 0) diagonal slot, which the substitutions never read: no exec-mask branches.
  const int i = l;
#pragma unroll
  for (int k = 0; k < 32; k++) T[(k < i && i < n) ? ti(i) + k : 0] = Lr[k];
  // forward: L y = b
  float y = 0.f;
#pragma unroll
  for (int k = 0; k < 32; k++) {
    float yk = rl(b, k) * rl(dinv, k);
    y = wl(y, yk, k);
    b = fmaf(-Lr[k], yk, b);
  }
  SYNC();
  // column i of L (below the diagonal) -> Lr; rows >= n of T are never written
  const int ic = min(i, n - 1);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    float v = T[ti(k) + ic];
    Lr[k] = ic < k && k < n ? v : 0.f;
  }
  // backward: L^T x = y
  float xo = 0.f;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    float xk = rl(y, k) * rl(dinv, k);
    xo = wl(xo, xk, k);
    y = fmaf(-Lr[k], xk, y);
  }
  if (i < n) x[i] = xo;
  SYNC();
}

// Cholesky solve for 32 < n <= 64 on the matrix cores (two-hand scenes, nv 54).  The
// padded 64 x 64 matrix is three 32 x 32 accumulator tiles: C11 (rows/cols 0-31),
// C12 (rows 0-31, cols 32-63, i.e. the transpose of the lower off-diagonal block)
// and C22 (rows/cols 32-63, identity padding past n).  Right-looking, two columns
// per step as in mfma_chol_solve32: for k < 32 rows k, k+1 of C11 give the panel's
// rows 0-31 and rows k, k+1 of C12 its rows 32-63 (symmetry again), and three MFMAs
// apply the rank-2 update to C11, C12 and C22; columns 32-63 then factor C22 alone.
// L goes to T (packed rows, ti(n) words, may alias A) as it is produced, and both
// substitutions run with lane = row (0-63) on readlane / writelane chains.
__device__ __forceinline__ void mfma_chol_solve64(const float* A, int n, float dj1, float dj2, float* x,
                                                  float* T) {
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  dx_f16v C11, C12, C22;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    {  // C11: A[i][j]
      const int ra = max(i, j), rb = min(i, j);
      float e = A[ti(ra) + rb];  // i, j < 32 < n
      if (i == j) e += dj1;
      C11[v] = e;
    }
    // (clamped in-range addresses, selected after: no exec-mask branch per load)
    {  // C12: A[i][32 + j] = A[32 + j][i]
      const int r = 32 + j;
      const float e = A[ti(min(r, n - 1)) + i];
      C12[v] = r < n ? e : 0.f;
    }
    {  // C22: A[32 + i][32 + j]
      const int ri = 32 + i, rj = 32 + j;
      const bool in = ri < n && rj < n;
      const int ca = min(max(ri, rj), n - 1), cb = min(min(ri, rj), n - 1);
      const float av = A[ti(ca) + cb];
      float e = in ? av : (i == j ? 1.f : 0.f);
      if (i == j && in) e += dj2;
      C22[v] = e;
    }
  }
  const float bx = x[min(l, n - 1)];
  float b = l < n ? bx : 0.f;
  SYNC();  // A may alias T
  float dinv = 0.f;  // lane k: 1 / L[k][k]
  // columns 0..31
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C11[vk], up), rk1 = half_dup(C11[vk + 1], up);  // A[j][k], A[j][k+1]
    const float sk = half_dup(C12[vk], up), sk1 = half_dup(C12[vk + 1], up);  // A[32+j][k], A[32+j][k+1]
    const float i11 = __builtin_amdgcn_rsqf(fmaxf(rl(rk, k), 1e-30f));
    const float l21 = rl(rk1, k) * i11;
    const float i22 = __builtin_amdgcn_rsqf(fmaxf(rl(rk1, k + 1) - l21 * l21, 1e-30f));
    dinv = wl(dinv, i11, k);
    dinv = wl(dinv, i22, k + 1);
    const float lk = rk * i11, lk1 = (rk1 - lk * l21) * i22;  // L[j][k], L[j][k+1]
    const float mk = sk * i11, mk1 = (sk1 - mk * l21) * i22;  // L[32+j][k], L[32+j][k+1]
    {  // L out (lanes with nothing to store write the never-read diagonal slot T[0])
      const int r = hi ? 32 + j : j;
      const bool v0 = hi ? r < n : j > k, v1 = hi ? r < n : j > k + 1;
      T[v0 ? ti(r) + k : 0] = hi ? mk : lk;
      T[v1 ? ti(r) + k + 1 : 0] = hi ? mk1 : lk1;
    }
    const float pa = j > k + 1 ? (hi ? lk1 : lk) : 0.f;
    const float pb = hi ? mk1 : mk;
    C11 = __builtin_amdgcn_mfma_f32_32x32x2f32(-pa, pa, C11, 0, 0, 0);
    C12 = __builtin_amdgcn_mfma_f32_32x32x2f32(-pa, pb, C12, 0, 0, 0);
    C22 = __builtin_amdgcn_mfma_f32_32x32x2f32(-pb, pb, C22, 0, 0, 0);
  }
  // columns 32..63: the trailing tile alone
#pragma unroll
  for (int k = 0; k < 32; k += 2) {
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C22[vk], up), rk1 = half_dup(C22[vk + 1], up);
    const float i11 = __builtin_amdgcn_rsqf(fmaxf(rl(C22[vk], k + (up ? 32 : 0)), 1e-30f));
    const float l21 = rl(C22[vk + 1], k + (up ? 32 : 0)) * i11;
    const float i22 = __builtin_amdgcn_rsqf(fmaxf(rl(C22[vk + 1], k + 1 + (up ? 32 : 0)) - l21 * l21, 1e-30f));
    dinv = wl(dinv, i11, 32 + k);
    dinv = wl(dinv, i22, 32 + k + 1);
    const float lk = rk * i11, lk1 = (rk1 - lk * l21) * i22;  // L[32+j][32+k], L[32+j][32+k+1]
    {
      const bool ok = hi == 0 && 32 + j < n;
      T[ok && j > k ? ti(32 + j) + 32 + k : 0] = lk;
      T[ok && j > k + 1 ? ti(32 + j) + 32 + k + 1 : 0] = lk1;
    }
    const float p = j > k + 1 ? (hi ? lk1 : lk) : 0.f;
    C22 = __builtin_amdgcn_mfma_f32_32x32x2f32(-p, p, C22, 0, 0, 0);
  }
  SYNC();
  const int i = l;
  // forward: L y = b (lane i holds b_i, then y_i).  L's entries come from LDS eight
  // columns at a time, loaded before the eight dependent steps that use them.
  float y = 0.f;
  for (int k0 = 0; k0 < n; k0 += 8) {
    float lc[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = k0 + u;
      const float t = T[ti(min(i, n - 1)) + min(k, n - 1)];
      lc[u] = i > k && i < n ? t : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = min(k0 + u, 63);
      const float yk = rl(b, k) * rl(dinv, k);
      if (k0 + u < n) {
        y = wl(y, yk, k);
        b = fmaf(-lc[u], yk, b);
      }
    }
  }
  // backward: L^T x = y
  float xo = 0.f;
  for (int k1 = n - 1; k1 >= 0; k1 -= 8) {
    float lc[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = k1 - u;
      const float t = T[ti(max(k, 0)) + min(i, max(k, 0))];
      lc[u] = k >= 0 && i < k ? t : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int k = max(k1 - u, 0);
      const float xk = rl(y, k) * rl(dinv, k);
      if (k1 - u >= 0) {
        xo = wl(xo, xk, k);
        y = fmaf(-lc[u], xk, y);
      }
    }
  }
  SYNC();
  if (i < n) x[i] = xo;
  SYNC();
}

// Solve for n <= 30 by the symmetric sweep operator on the matrix cores: the bordered
// matrix [[A, b], [b^T, 0]] (b in row/column 31, identity padding between) sits in the
// v_mfma_f32_32x32x2_f32 accumulator as in mfma_chol_solve32.  Sweeping the pivot pair
// {k, k+1} of a symmetric S maps it to [[-P^-1, P^-1 U^T], [U P^-1, S' - U P^-1 U^T]]
// (P the 2 x 2 pivot block, U the other rows of the pivot columns); once every pivot of
// A is swept, column 31 holds A^-1 b.  One step = the pivot rows and columns zeroed, then
// one rank-2 MFMA S -= V W V^T with W = P^-1 and V = U with -I in the pivot rows: that
// writes U W into the pivot columns and -W into the pivot block without the cancellation
// an in-place update would suffer when |P| >> |W|.  Only the entries read later are
// zeroed: a pivot column below the pair (rows read as future pivot rows) and the pivot
// rows (their column-31 entries are the answer).  The pivots are the Cholesky Schur
// complements (Gauss-Jordan on an SPD matrix in pivot pairs): 15 dependent steps and no
// triangular substitutions (mfma_chol_solve32's two 32-step readlane chains and its LDS
// transpose).  A (+ dj on the diagonal) -> x = A^-1 x.  tests/test_sweep_solve.py
// restates it in numpy.
__device__ __forceinline__ void mfma_sweep_solve30(const float* A, int n, float dj, float* x) {
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  // Every lane loads in-range addresses (indices clamped to n - 1) and selects after:
  // a guarded load compiles to an exec-mask branch with its own LDS wait, 32 in a row.
  const int jc = min(j, n - 1);
  const float bj = j < n ? x[jc] : 0.f;
  float av[16], xv[16];
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int ic = min(8 * (v >> 2) + 4 * hi + (v & 3), n - 1);
    av[v] = A[ti(max(ic, jc)) + min(ic, jc)];
    xv[v] = x[ic];
  }
  dx_f16v C;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    const bool in = i < n && j < n;
    float e = in ? av[v] : (i == j && i < 31 ? 1.f : 0.f);
    if (i == j && in) e += dj;
    if (i == 31) e = bj;              // row 31: b_j (0 at (31, 31))
    if (j == 31 && i < n) e = xv[v];  // column 31: b_i
    C[v] = e;
  }
#pragma unroll
  for (int k = 0; k < 30; k += 2) {
    if (k >= n) continue;  // identity padding (a uniform branch; break would block the unroll)
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C[vk], up), rk1 = half_dup(C[vk + 1], up);  // S[k][j], S[k+1][j]
    // the pivot block straight from the accumulator (lane k + 32 up holds column k of rows
    // k, k + 1): the readlanes and the 2 x 2 inverse do not wait for the half swaps
    const int kl = k + (up ? 32 : 0);
    const float p00 = rl(C[vk], kl), p10 = rl(C[vk + 1], kl), p11 = rl(C[vk + 1], kl + 1);
    const float id = 1.0f / (p00 * p11 - p10 * p10);
    const float w00 = p11 * id, w01 = -p10 * id, w11 = p00 * id;
    const bool pc = j == k || j == k + 1;  // a pivot column
    const float v0 = pc ? (j == k ? -1.f : 0.f) : rk;
    const float v1 = pc ? (j == k ? 0.f : -1.f) : rk1;
    const float a = hi ? v1 : v0;                                             // A: V[j][hi]
    const float b = hi ? fmaf(w01, v0, w11 * v1) : fmaf(w00, v0, w01 * v1);  // B: (W V^T)[hi][j]
#if DX_SWEEP_PK
    // two accumulator entries per packed multiply (v_pk_mul_f32) by 0 on the pivot
    // columns' lanes, 1 elsewhere: half the instructions of one select per entry
    const dx_f2v mk = {pc ? 0.f : 1.f, pc ? 0.f : 1.f};
#pragma unroll
    for (int v = 0; v < 16; v += 2) {
      const bool z0 = 8 * (v >> 2) + 4 + (v & 3) >= k + 2, z1 = 8 * ((v + 1) >> 2) + 4 + ((v + 1) & 3) >= k + 2;
      if (z0 && z1) {
        dx_f2v t = {C[v], C[v + 1]};
        t = t * mk;
        C[v] = t.x;
        C[v + 1] = t.y;
      } else if (z0) {
        C[v] = pc ? 0.f : C[v];
      } else if (z1) {
        C[v + 1] = pc ? 0.f : C[v + 1];
      }
    }
#else
#pragma unroll
    for (int v = 0; v < 16; v++)
      if (8 * (v >> 2) + 4 + (v & 3) >= k + 2) C[v] = pc ? 0.f : C[v];
#endif
    const bool ph = hi == (up ? 1 : 0);
    C[vk] = ph ? 0.f : C[vk];
    C[vk + 1] = ph ? 0.f : C[vk + 1];
    C = __builtin_amdgcn_mfma_f32_32x32x2f32(-a, b, C, 0, 0, 0);
  }
  // column 31 -> x (lane 31 of each half writes its half's rows)
  SYNC();
  if (j == 31) {
#pragma unroll
    for (int v = 0; v < 16; v++) {
      const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
      if (i < n) x[i] = C[v];
    }
  }
  SYNC();
}

// The inverse of an n <= 30 SPD matrix by the same sweep: sweeping every pivot of A
// leaves -A^-1 in the accumulator.  Unlike mfma_sweep_solve30 every entry is kept exact
// (the pivot rows and columns are zeroed whole before each rank-2 update), and -C is
// written to Ainv as a packed lower triangle (may not alias A).  For repeated solves with
// one matrix: CG's M^-1 grad, one matrix-vector product per iteration instead of a sweep.
__device__ __forceinline__ void mfma_sweep_inverse30(const float* A, int n, float* Ainv) {
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  const int jc = min(j, n - 1);
  float av[16];
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int ic = min(8 * (v >> 2) + 4 * hi + (v & 3), n - 1);
    av[v] = A[ti(max(ic, jc)) + min(ic, jc)];
  }
  dx_f16v C;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    C[v] = i < n && j < n ? av[v] : (i == j ? 1.f : 0.f);
  }
#pragma unroll
  for (int k = 0; k < 30; k += 2) {
    if (k >= n) continue;  // identity padding (a uniform branch)
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C[vk], up), rk1 = half_dup(C[vk + 1], up);  // S[k][j], S[k+1][j]
    // the pivot block straight from the accumulator (lane k + 32 up holds column k of rows
    // k, k + 1): the readlanes and the 2 x 2 inverse do not wait for the half swaps
    const int kl = k + (up ? 32 : 0);
    const float p00 = rl(C[vk], kl), p10 = rl(C[vk + 1], kl), p11 = rl(C[vk + 1], kl + 1);
    const float id = 1.0f / (p00 * p11 - p10 * p10);
    const float w00 = p11 * id, w01 = -p10 * id, w11 = p00 * id;
    const bool pc = j == k || j == k + 1;  // a pivot column
    const float v0 = pc ? (j == k ? -1.f : 0.f) : rk;
    const float v1 = pc ? (j == k ? 0.f : -1.f) : rk1;
    const float a = hi ? v1 : v0;
    const float b = hi ? fmaf(w01, v0, w11 * v1) : fmaf(w00, v0, w01 * v1);
    const dx_f2v mk = {pc ? 0.f : 1.f, pc ? 0.f : 1.f};
#pragma unroll
    for (int v = 0; v < 16; v += 2) {  // the pivot columns, every row
      dx_f2v t = {C[v], C[v + 1]};
      t = t * mk;
      C[v] = t.x;
      C[v + 1] = t.y;
    }
    const bool ph = hi == (up ? 1 : 0);  // the pivot rows, every column
    C[vk] = ph ? 0.f : C[vk];
    C[vk + 1] = ph ? 0.f : C[vk + 1];
    C = __builtin_amdgcn_mfma_f32_32x32x2f32(-a, b, C, 0, 0, 0);
  }
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    if (i < n && j <= i) Ainv[ti(i) + j] = -C[v];
  }
  SYNC();
}

// Diagonal additions hs * dadd for chol_solve, one pair per lane (columns l % 32 and
// 32 + l % 32).  Load them early, before the caller's barriers: a model-table load
// issued after a barrier is a whole L2 round trip on the wave's critical path.
struct DiagAdd { float d1, d2; };
__device__ __forceinline__ DiagAdd diag_add(const DXG float* dadd, float hs, int n) {
  const int j = LANE & 31;
  DiagAdd d;
  d.d1 = j < n ? hs * dadd[j] : 0.f;
  d.d2 = 32 + j < n ? hs * dadd[32 + j] : 0.f;
  return d;
}
// x <- (A + diag(dd))^-1 x for a packed lower-triangle A (LDS), n <= 64;
// T: ti(max(n, 32)) words of LDS scratch, may alias A.
__device__ __forceinline__ void chol_solve(const float* A, int n, DiagAdd dd, float* x, float* T) {
  if (DX_SWEEP && n <= 30) mfma_sweep_solve30(A, n, dd.d1, x);
  else if (n <= 32) mfma_chol_solve32(A, n, dd.d1, x, T);
  else mfma_chol_solve64(A, n, dd.d1, dd.d2, x, T);
}
__device__ __forceinline__ void chol_solve(const float* A, int n, float* x, float* T) {
  chol_solve(A, n, DiagAdd{0.f, 0.f}, x, T);
}

// The Cholesky factor of an n <= 30 SPD matrix, in place: A (packed lower triangle,
// LDS) -> G (packed lower triangle with its diagonal), G G' = A.  The factorisation of
// mfma_chol_solve32 (two columns per step, one rank-2 MFMA on the trailing matrix),
// storing each column pair as it is produced; A is read whole before the first store.
__device__ __forceinline__ void mfma_chol_factor30(float* A, int n) {
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  const int jc = min(j, n - 1);
  float av[16];
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int ic = min(8 * (v >> 2) + 4 * hi + (v & 3), n - 1);
    av[v] = A[ti(max(ic, jc)) + min(ic, jc)];
  }
  dx_f16v C;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    C[v] = i < n && j < n ? av[v] : (i == j ? 1.f : 0.f);
  }
  SYNC();
#pragma unroll
  for (int k = 0; k < 30; k += 2) {
    if (k >= n) continue;  // identity padding (a uniform branch)
    const int vk = 4 * (k >> 3) + (k & 3);
    const bool up = (k & 7) >= 4;
    const float rk = half_dup(C[vk], up), rk1 = half_dup(C[vk + 1], up);  // C[k][j], C[k+1][j]
    const float i11 = __builtin_amdgcn_rsqf(fmaxf(rl(C[vk], k + (up ? 32 : 0)), 1e-30f));
    const float l21 = rl(C[vk + 1], k + (up ? 32 : 0)) * i11;
    const float i22 = __builtin_amdgcn_rsqf(fmaxf(rl(C[vk + 1], k + 1 + (up ? 32 : 0)) - l21 * l21, 1e-30f));
    const float lk = rk * i11;                 // G[j][k]   (j >= k; the diagonal at j = k)
    const float lk1 = (rk1 - lk * l21) * i22;  // G[j][k+1] (j >= k + 1)
    if (hi == 0 && j >= k && j < n) A[ti(j) + k] = lk;
    if (hi == 0 && j > k && j < n) A[ti(j) + k + 1] = lk1;
    const float p = j > k + 1 ? (hi ? lk1 : lk) : 0.f;
    C = __builtin_amdgcn_mfma_f32_32x32x2f32(-p, p, C, 0, 0, 0);
  }
  SYNC();
}

// The Gram matrix P P' of the wave's 64 rows on the matrix cores: lane k holds row k of
// P (30 entries, zero past nv); out[r] in lane k is P_r . P_k, plus diag (this lane's
// value) on the diagonal -- lane k holds column k.  Rows 0-31 and 32-63 are the two row
// tiles: one v_permlane32_swap of (P[2s], P[2s+1]) gives both tiles' A operands of k step
// s (lanes 0-31 supply P[i][2s], lanes 32-63 P[i][2s+1] of the tile's row i), and B = A'
// is the same operand, so the four 32 x 32 tiles take 15 v_mfma_f32_32x32x2_f32 each
// (`full`: rows past 32 exist; else tile (0, 0) alone).  The accumulator holds C[i][j] in
// lane j + 32 b for the rows i with bit 2 = b; one more swap per register pair gives
// every lane its whole column.
__device__ __forceinline__ void pgs_gram64(const float (&P)[30], float diag, bool full, float (&out)[64]) {
  const int l = LANE;
  const int j = l & 31, hi = l >> 5;
  const float d0 = half_dup(diag, false), d1 = half_dup(diag, true);  // diag of rows j and 32 + j
  dx_f16v C00, C10, C01, C11;
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int i = 8 * (v >> 2) + 4 * hi + (v & 3);
    C00[v] = i == j ? d0 : 0.f;
    C11[v] = i == j ? d1 : 0.f;
    C10[v] = 0.f;
    C01[v] = 0.f;
  }
  if (full) {
#pragma unroll
    for (int s = 0; s < 15; s++) {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(P[2 * s]), __float_as_uint(P[2 * s + 1]), false, false);
      const float a0 = __uint_as_float(sw[0]), a1 = __uint_as_float(sw[1]);
      C00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a0, C00, 0, 0, 0);
      C10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, a0, C10, 0, 0, 0);
      C01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a1, C01, 0, 0, 0);
      C11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, a1, C11, 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < 15; s++) {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(P[2 * s]), __float_as_uint(P[2 * s + 1]), false, false);
      const float a0 = __uint_as_float(sw[0]);
      C00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, a0, C00, 0, 0, 0);
    }
    C11 = C10;  // (zero)
  }
  // lane j (< 32) keeps its rows of tiles (., 0) and takes lane j + 32's; lane j + 32
  // keeps its rows of tiles (., 1) and takes lane j's: after the swap sw[0] holds the
  // rows with bit 2 clear of this lane's column, sw[1] those with bit 2 set
#pragma unroll
  for (int v = 0; v < 16; v++) {
    const int r = 8 * (v >> 2) + (v & 3);
    const auto s0 = __builtin_amdgcn_permlane32_swap(__float_as_uint(C00[v]), __float_as_uint(C01[v]), false, false);
    out[r] = __uint_as_float(s0[0]);
    out[r + 4] = __uint_as_float(s0[1]);
    const auto s1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(C10[v]), __float_as_uint(C11[v]), false, false);
    out[32 + r] = __uint_as_float(s1[0]);
    out[32 + r + 4] = __uint_as_float(s1[1]);
  }
}

// Reduce-scatter of 32-vectors over the wave: each lane holds t[0..31]; returns, in lane
// L, component c = L >> 1 of the sum over all 64 lanes (lanes 2c and 2c + 1 hold it).  A
// permlane32 swap halves the vectors across the half-waves (16 adds), a permlane16 swap
// across the rows (8), then row_mirror, row_half_mirror and two quad_perms within the
// rows (4 + 2 + 1 + 1): 32 adds and 70 instructions in all, against 32 wave sums.
__device__ __forceinline__ float wave_reduce_scatter32(const float (&t)[32]) {
  float u[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {  // u[i]: component i + 16 b5
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(t[i]), __float_as_uint(t[16 + i]), false, false);
    u[i] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {  // v[i]: component i + 8 b4 + 16 b5
    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(u[i]), __float_as_uint(u[8 + i]), false, false);
    v[i] = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const int L = LANE;
  const bool b3 = (L >> 3) & 1, b2 = (L >> 2) & 1, b1 = (L >> 1) & 1;
  float x[4];
#pragma unroll
  for (int i = 0; i < 4; i++)  // + 4 b3; the partner 15 - L (row_mirror) has b3 flipped
    x[i] = (b3 ? v[4 + i] : v[i]) + dpp_f<0x140, 0xF>(b3 ? v[i] : v[4 + i]);
  float y[2];
#pragma unroll
  for (int i = 0; i < 2; i++)  // + 2 b2; the partner 7 - L within the half-row (row_half_mirror)
    y[i] = (b2 ? x[2 + i] : x[i]) + dpp_f<0x141, 0xF>(b2 ? x[i] : x[2 + i]);
  const float z = (b1 ? y[1] : y[0]) + dpp_f<0x4E, 0xF>(b1 ? y[0] : y[1]);  // + b1; partner L ^ 2
  return z + dpp_f<0xB1, 0xF>(z);                                          // partner L ^ 1
}

// x <- (M + diag(dd))^-1 x for a matrix with the kinematic tree's sparsity (M, and
// M + h·D in the Euler step): entry (i, j < i) is nonzero only when dof j is an
// ancestor of dof i.  [3P] MuJoCo's mj_factorM / mj_solveM: M = L^T D L with L unit
// lower, eliminated leaves first, which fills in nothing.
// Factorisation: the dofs of one height level above the leaves are never ancestors of
// one another, so a level is a set of independent items (k, i, j) -- A[i][j] -=
// A[k][i] A[k][j] / A[k][k] for i a proper ancestor of k and j = i or an ancestor of
// i -- spread over the lanes (DevModel::ldl_tab, loaded before the first barrier) and
// summed into the shared ancestors with LDS float atomics.  The level's reads (rows k)
// are never its targets.  Shadow hand + cube: 8 slots of 64 items in 6 levels,
// against 16 rank-2 MFMA steps of the dense factorisation.
// Substitutions, lane = dof, one readlane + one FMA per step (no writelanes): lane i
// keeps u_i = y_i / D_i, so w = D^-1 L^-T y comes out of the k-descending chain over
// the columns of L, and x = L^-1 w out of the ascending chain over its rows.
// T: ti(n) words of LDS scratch (not aliasing A or x).
template <class Ctx>
__device__ __forceinline__ void tree_solve(const Ctx& c, const float* A, float dj, float* x, float* T) {
  const DevModel& m = c.mdl();
  const int n = c.nv;
  const int ns = m.ldl_nslot;
  const unsigned lvend = m.ldl_sync;
  int item[DX_LDL_SLOTS];
#pragma unroll
  for (int s = 0; s < DX_LDL_SLOTS; s++) item[s] = s < ns ? m.ldl_tab[s * DX_WAVE + LANE] : -1;
  for (int k = LANE; k < ti(n); k += DX_WAVE) T[k] = A[k];
  SYNC();
  if (LANE < n) T[ti(LANE) + LANE] += dj;
  SYNC();
#pragma unroll
  for (int s = 0; s < DX_LDL_SLOTS; s++) {
    if (s < ns) {
      const int t = item[s];
      if (t >= 0) {
        const int k = t & 255, i = (t >> 8) & 255, j = t >> 16;
        const float akk = T[ti(k) + k], aki = T[ti(k) + i], akj = T[ti(k) + j];
        atomicAdd(T + ti(i) + j, -aki * (akj / akk));
      }
      if ((lvend >> s) & 1u) SYNC();
    }
  }
  SYNC();
  const int l = LANE;
  const float dinv = l < n ? 1.0f / T[ti(l) + l] : 0.f;
  // w = D^-1 L^-T b: lane i holds u_i = y_i / D_i; step k (descending) takes the final
  // w_k = u_k, and L[k][i] z_k / D_i = (A[k][i] / D_k) (w_k D_k) / D_i = A[k][i] / D_i w_k
  float u = l < n ? x[l] * dinv : 0.f;
  for (int k1 = n - 1; k1 >= 0; k1 -= 8) {
    float lc[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int k = k1 - q;
      lc[q] = k >= 0 && l < k ? T[ti(k) + l] * dinv : 0.f;  // A[k][i] / D_i
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int k = max(k1 - q, 0);
      if (k1 - q >= 0) u = fmaf(-lc[q], rl(u, k), u);
    }
  }
  // x = L^-1 w: lane k holds v_k = w_k - sum_i A[k][i] / D_k x_i; step i (ascending)
  // takes x_i = v_i
  float v = u;
  for (int i0 = 0; i0 < n; i0 += 8) {
    float lr[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int i = i0 + q;
      lr[q] = l > i && l < n ? T[ti(l) + i] * dinv : 0.f;  // A[k][i] / D_k
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int i = min(i0 + q, 63);
      if (i0 + q < n) v = fmaf(-lr[q], rl(v, i), v);
    }
  }
  SYNC();
  if (l < n) x[l] = v;
  SYNC();
}
// M (+ diag) solve: n <= 30 by the MFMA sweep operator (15 dependent steps, no
// substitutions: same-box 2.60 -> 2.67 M env-steps/s on Shadow reorient against the tree
// LDL^T, whose six level barriers and two 30-step readlane chains cost more), larger n by
// the tree-sparse LDL^T when the model has its item table, else the dense Cholesky.
template <class Ctx>
__device__ __forceinline__ void m_solve(const Ctx& c, const float* A, DiagAdd dd, float* x, float* T) {
  if (DX_SWEEP && c.nv <= 30) mfma_sweep_solve30(A, c.nv, dd.d1, x);
  else if (c.mdl().ldl_nslot > 0) tree_solve(c, A, LANE < 32 ? dd.d1 : dd.d2, x, T);
  else chol_solve(A, c.nv, dd, x, T);
}
