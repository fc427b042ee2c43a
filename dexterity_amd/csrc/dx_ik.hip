// dx_ik.hip -- site Jacobians and batched damped-least-squares inverse kinematics
// for CDNA4 (gfx950).
//
// Reference: dexterity/inverse_kinematics/ik_solver.py (IKSolver.solve / _solve_ik /
// _update_physics_data), dexterity/controllers/dls/dls.py (DampedLeastSquaresMapper)
// and utils/mujoco_utils.py:38-73 (compute_object_6d_jacobian = mj_jacSite [3P]).
//
// One 64-lane wavefront runs one IK attempt of one environment: the reference runs
// its attempts one after another, but they are independent given their starting
// joints, so here every (env, attempt) pair is its own workgroup and a selection
// kernel applies the reference's choice rule afterwards (ik_solver.py:132-152).
// Per integration step the wave recomputes kinematics + com positions (the tree
// passes of the step kernel, dx_device.h), stacks the 3 * nsite site-Jacobian rows
// in LDS, forms J J^T + reg I (3 * nsite <= 32) and solves it on the matrix cores
// (mfma_chol_solve32), then qdot = J^T y.  That is dls.py's (J^T J + reg I) qdot =
// J^T twist by the push-through identity (J^T J + reg I)^-1 J^T = J^T (J J^T +
// reg I)^-1: a 15 x 15 system instead of nv x nv, with the same solution.
#include "dx_device.h"

// IK block in LDS (words), appended after the model's own layout at P.blk.
struct IkLds {
  int J, H, y, pt, pv, tg, qd, total;
};
__host__ __device__ inline IkLds ik_lds(int blk, int nv) {
  IkLds k;
  int o = blk;
  k.J = o;  o += 32 * nv;   // stacked site-Jacobian rows [3 * nsite][nv]
  k.H = o;  o += 528;       // packed lower triangle of J J^T + reg I; Cholesky scratch (ti(32))
  k.y = o;  o += 32;        // twist -> multipliers
  k.pt = o; o += 32;        // site positions at the current qpos
  k.pv = o; o += 32;        // site positions before the last step
  k.tg = o; o += 32;        // targets
  k.qd = o; o += DX_MAX_NV; // joint velocities
  k.total = o;
  return k;
}
int dx_ik_lds_words(const DevModel& d, int) { return ik_lds(0, d.nv).total; }

// lane t < 3 * nsite: coordinate t % 3 of site t / 3 at the current kinematics
// (site_xpos, as geometry.PoseStamped(frame=site).get_world_pose reads it)
template <class Ctx>
__device__ __forceinline__ void sites_to_lds(const Ctx& c, const IkDev& P, float* pt) {
  const DevModel& m = c.mdl();
  if (LANE < 3 * P.nsite) {
    const int s = LANE / 3, e = LANE - 3 * s;
    const int sid = P.sites[s];
    const int b = m.site_bodyid[sid];
    const float* xp = c.f(c.L.xpos) + 3 * b;
    const float* xm = c.f(c.L.xmat) + 9 * b;
    const DXG float* sp = m.site_pos + 3 * sid;
    pt[LANE] = xp[e] + xm[3 * e] * sp[0] + xm[3 * e + 1] * sp[1] + xm[3 * e + 2] * sp[2];
  }
  SYNC();
}

// mj_jacSite rows [3 * nsite][nv]: translational (rot = false) or rotational.  Column
// d of a site on body b is non-zero when dof d is on b's path to the root; then
// jacp = cdof_lin + cdof_ang x (site - subtree_com[root]), jacr = cdof_ang.
template <class Ctx>
__device__ __forceinline__ void site_jacobian(const Ctx& c, const IkDev& P, const float* pt, float* J, bool rot) {
  const DevModel& m = c.mdl();
  const int nv = c.nv, n = 3 * P.nsite * nv;
  const float* cdof = c.f(c.L.cdof);
  const float* rcom = c.f(c.L.rcom);
  for (int k = LANE; k < n; k += DX_WAVE) {
    const int r = k / nv, d = k - r * nv, s = r / 3, e = r - 3 * s;
    const int b = m.site_bodyid[P.sites[s]];
    float v = 0.f;
    if ((m.body_chain[b] >> d) & 1ull) {
      const float* cd = cdof + 6 * d;
      if (rot) {
        v = cd[e];
      } else {
        const float* rc = rcom + 3 * m.body_rootidx[b];
        const float o0 = pt[3 * s] - rc[0], o1 = pt[3 * s + 1] - rc[1], o2 = pt[3 * s + 2] - rc[2];
        const float cr = e == 0 ? cd[1] * o2 - cd[2] * o1 : e == 1 ? cd[2] * o0 - cd[0] * o2 : cd[0] * o1 - cd[1] * o0;
        v = cd[3 + e] + cr;
      }
    }
    J[k] = v;
  }
  SYNC();
}

// mj_integratePos(qpos, qdot, h) followed by mj_normalizeQuat, then the clip of the
// solved joints to their range (ik_solver.py:189-194 and 238-250).
template <class Ctx>
__device__ __forceinline__ void ik_integrate(const Ctx& c, const IkDev& P, const float* v, float h) {
  const DevModel& m = c.mdl();
  float* qpos = c.f(c.L.qpos);
  for (int j = LANE; j < c.njnt; j += DX_WAVE) {
    const int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j];
    if (m.jnt_type[j] == DXJ_FREE) {
      for (int k = 0; k < 3; k++) qpos[qa + k] += h * v[da + k];
      float* q = qpos + qa + 3;
      const float* w = v + da + 3;
      const float wn = norm3(w);
      if (wn > 1e-20f) {
        float s, co;
        sincosf(0.5f * h * wn, &s, &co);
        const float dq[4] = {co, w[0] / wn * s, w[1] / wn * s, w[2] / wn * s};
        quatmul(q, q, dq);
      }
      quatnorm(q);
    } else {
      qpos[qa] += h * v[da];
    }
  }
  SYNC();
  for (int k = LANE; k < P.njoint; k += DX_WAVE) {
    const int j = P.joints[k];
    const int qa = m.jnt_qposadr[j];
    qpos[qa] = fminf(fmaxf(qpos[qa], m.jnt_range[2 * j]), m.jnt_range[2 * j + 1]);
  }
  SYNC();
}

// mode 0: one IK attempt per workgroup (blockIdx = env * nattempt + attempt);
// mode 1: the site Jacobians of env blockIdx at its current qpos.
extern "C" __global__ void __launch_bounds__(64) dx_ik_kernel(const DevModel* __restrict__ mp, DevBatch B, Lds L, IkDev P) {
  extern __shared__ float smem[];
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  const int w = (int)blockIdx.x;
  const int env = P.mode == 0 ? w / P.nattempt : w;
  const int att = P.mode == 0 ? w - env * P.nattempt : 0;
  if (env >= B.nenv) return;
  CtxT<SpecRT> c(m, L, smem, nullptr, nullptr);
  c.I = (int*)(smem + L.ints);
  const IkLds K = ik_lds(P.blk, m.nv);
  // the Cholesky solve reads padding words of its packed triangles (times exact zeros)
  for (int k = LANE; k < K.total; k += DX_WAVE) smem[k] = 0.f;
  SYNC();
  const int nv = m.nv, n3 = 3 * P.nsite;
  float* qpos = c.f(L.qpos);
  for (int i = LANE; i < m.nq; i += DX_WAVE) qpos[i] = B.qpos[(size_t)env * m.nq + i];
  SYNC();
  if (P.mode == 0) {
    // ik_solver.py:122-129: attempt 0 from the nullspace reference (joint midrange),
    // later attempts from np.random.uniform over the joint ranges (dx_ik_starts_kernel)
    for (int k = LANE; k < P.njoint; k += DX_WAVE) {
      const int j = P.joints[k];
      const float lo = m.jnt_range[2 * j], hi = m.jnt_range[2 * j + 1];
      qpos[m.jnt_qposadr[j]] =
          att == 0 ? 0.5f * (lo + hi) : P.starts[((size_t)env * (P.nattempt - 1) + att - 1) * P.njoint + k];
    }
    SYNC();
  }
  kin_com(c);
  float* pt = c.f(K.pt);
  float* J = c.f(K.J);
  sites_to_lds(c, P, pt);
  if (P.mode == 1) {
    const size_t base = (size_t)env * n3 * nv;
    if (P.jacp) {
      site_jacobian(c, P, pt, J, false);
      for (int k = LANE; k < n3 * nv; k += DX_WAVE) P.jacp[base + k] = J[k];
      SYNC();
    }
    if (P.jacr) {
      site_jacobian(c, P, pt, J, true);
      for (int k = LANE; k < n3 * nv; k += DX_WAVE) P.jacr[base + k] = J[k];
    }
    return;
  }
  float* H = c.f(K.H);
  float* y = c.f(K.y);
  float* pv = c.f(K.pv);
  float* tg = c.f(K.tg);
  float* qd = c.f(K.qd);
  if (LANE < n3) {
    tg[LANE] = P.targets[(size_t)env * n3 + LANE];
    pv[LANE] = pt[LANE];
  }
  SYNC();
  float err = 0.f;  // lane s < nsite: linear error of site s after the last step
  int it = 0;
  while (it < P.max_steps) {
    // _compute_twist (ik_solver.py:253-261) over a 1 s integration step
    if (LANE < n3) y[LANE] = P.gain * (tg[LANE] - pt[LANE]);
    site_jacobian(c, P, pt, J, false);
    // J J^T + reg I, packed lower triangle
    for (int t = LANE; t < ti(n3); t += DX_WAVE) {
      int i = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
      while (ti(i + 1) <= t) i++;
      while (ti(i) > t) i--;
      const int j = t - ti(i);
      float s = 0.f;
      for (int d = 0; d < nv; d++) s = fmaf(J[i * nv + d], J[j * nv + d], s);
      H[t] = s + (i == j ? P.reg : 0.f);
    }
    SYNC();
    mfma_chol_solve32(H, n3, 0.f, y, H);
    for (int d = LANE; d < nv; d += DX_WAVE) {
      float s = 0.f;
      for (int r = 0; r < n3; r++) s = fmaf(J[r * nv + d], y[r], s);
      qd[d] = s;
    }
    SYNC();
    ik_integrate(c, P, qd, 1.0f);
    kin_com(c);
    sites_to_lds(c, P, pt);
    it++;
    // ik_solver.py:201-233: per-site error and progress, then the break conditions
    int far = 0, stuck = 0;
    if (LANE < P.nsite) {
      const int s3 = 3 * LANE;
      const float e0 = tg[s3] - pt[s3], e1 = tg[s3 + 1] - pt[s3 + 1], e2 = tg[s3 + 2] - pt[s3 + 2];
      const float c0 = pt[s3] - pv[s3], c1 = pt[s3 + 1] - pv[s3 + 1], c2 = pt[s3 + 2] - pv[s3 + 2];
      err = sqrtf(e0 * e0 + e1 * e1 + e2 * e2);
      const float chg = sqrtf(c0 * c0 + c1 * c1 + c2 * c2);
      far = err > P.tol;
      stuck = err / (chg + 1e-10f) > P.progress;
    }
    SYNC();
    if (LANE < n3) pv[LANE] = pt[LANE];
    SYNC();
    const bool close = !__any(far);
    const bool no_progress = __any(stuck) != 0;
    if ((P.early_stop && close) || no_progress) break;
  }
  const size_t a = (size_t)env * P.nattempt + att;
  for (int k = LANE; k < P.njoint; k += DX_WAVE) P.att_qpos[a * P.njoint + k] = qpos[m.jnt_qposadr[P.joints[k]]];
  if (LANE < P.nsite) P.att_err[a * P.nsite + LANE] = err;
  if (LANE == 0) P.att_steps[a] = it;
}

// IKSolver.solve's choice among the attempts (ik_solver.py:132-152), one thread per env.
extern "C" __global__ void dx_ik_select_kernel(int nenv, IkDev P, const DXG float* jnt_range,
                                               float* qpos_out, int* success, float* err_out, int* attempt_out,
                                               int* steps_out) {
  const int env = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (env >= nenv) return;
  int best = -1;
  float best_d = INFINITY;
  for (int a = 0; a < P.nattempt; a++) {
    const size_t k = (size_t)env * P.nattempt + a;
    bool ok = true;
    for (int s = 0; s < P.nsite; s++) ok = ok && P.att_err[k * P.nsite + s] <= P.tol;
    if (!ok) continue;
    float d2 = 0.f;
    for (int q = 0; q < P.njoint; q++) {
      const int j = P.joints[q];
      const float dq = P.att_qpos[k * P.njoint + q] - 0.5f * (jnt_range[2 * j] + jnt_range[2 * j + 1]);
      d2 = fmaf(dq, dq, d2);
    }
    const float d = sqrtf(d2);
    if (d < best_d) { best_d = d; best = a; }
    if (P.stop_on_first) break;
  }
  const int sel = best >= 0 ? best : P.nattempt - 1;
  const size_t k = (size_t)env * P.nattempt + sel;
  if (qpos_out)
    for (int q = 0; q < P.njoint; q++) qpos_out[(size_t)env * P.njoint + q] = P.att_qpos[k * P.njoint + q];
  if (err_out)
    for (int s = 0; s < P.nsite; s++) err_out[(size_t)env * P.nsite + s] = P.att_err[k * P.nsite + s];
  if (success) success[env] = best >= 0;
  if (attempt_out) attempt_out[env] = sel;
  if (steps_out) steps_out[env] = P.att_steps[k];
}

hipError_t dx_launch_ik(int nwave, size_t lds, hipStream_t stream, const DevModel* m, const DevBatch& B, const Lds& L,
                        const IkDev& P) {
  hipLaunchKernelGGL(dx_ik_kernel, dim3(nwave), dim3(64), lds, stream, m, B, L, P);
  return hipGetLastError();
}

hipError_t dx_launch_ik_select(int nenv, hipStream_t stream, const DevModel& m, const IkDev& P, float* qpos_out,
                               int* success, float* err_out, int* attempt_out, int* steps_out) {
  hipLaunchKernelGGL(dx_ik_select_kernel, dim3((nenv + 255) / 256), dim3(256), 0, stream, nenv, P, m.jnt_range,
                     qpos_out, success, err_out, attempt_out, steps_out);
  return hipGetLastError();
}

// Random restarts of IKSolver.solve (ik_solver.py:127-130): attempt a >= 1 starts at
// np.random.uniform(*range.T) -- numpy's global stream, which env e's process seeded with
// np.random.seed(seed + e) -- so attempt a takes draws (a - 1) * njoint .. a * njoint - 1,
// one per joint in order: low + (high - low) * random_sample(), in fp64 as numpy computes
// it (no fma), then rounded to the fp32 state.  One thread per env; its MT19937 state is
// interleaved over the envs (dx_mt_* in dx_internal.h).
extern "C" __global__ void dx_ik_starts_kernel(int nenv, int natt, int nj, uint64_t seed, const double* range,
                                               uint32_t* mt, float* out) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= nenv) return;
  dx_mt_seed(mt, nenv, env, (uint32_t)(seed + (uint64_t)env));
  for (int a = 0; a < natt; a++)
    for (int k = 0; k < nj; k++) {
      const double lo = range[2 * k], hi = range[2 * k + 1];
      const double u = dx_mt_double(mt, nenv, env);
      out[((size_t)env * natt + a) * nj + k] = (float)__dadd_rn(lo, __dmul_rn(hi - lo, u));
    }
}

hipError_t dx_launch_ik_starts(int nenv, int natt, int njoint, uint64_t seed, const double* range, uint32_t* mt,
                               float* out, hipStream_t stream) {
  hipLaunchKernelGGL(dx_ik_starts_kernel, dim3((nenv + 63) / 64), dim3(64), 0, stream, nenv, natt, njoint, seed, range,
                     mt, out);
  return hipGetLastError();
}
