// dx_sensor.hip -- joint torque sensors (mj_rnePostConstraint + mj_sensorAcc) for CDNA4.
//
// The reference puts a 3-axis `torque` sensor on a site at the origin of every
// joint's body (models/hands/shadow_hand_e.py:176-196, adroit_hand.py:153-172) and
// projects it on the joint axis for the `joint_torques` observable
// (dexterous_hand.py:266-275).  MuJoCo computes it in mj_step2 after the constraint
// solve and before integration [3P]: the internal spatial force cfrc_int of the body
// (its subtree's inertial + bias forces minus the external forces: xfrc_applied and
// the contact forces) moved to the site and rotated into the site frame.
//
// The step kernel only stashes what that needs at its last substep (pre-integration
// qpos / qvel, the solved qacc, and each contact's bodies, point and world-frame force:
// dx_step.hip sensor_stash), so the hot path pays nothing when the field is off.  This
// kernel rebuilds the tree quantities from the stash, one 64-lane wave per env,
// lane = body (nbody <= 64), and writes the sensor of every body:
//   DX_SENSOR_TORQUE [nenv][nbody][3]  (site at the body origin, body frame).
#include "dx_device.h"

// Stash layout per env (floats): qpos [nq] | qvel [nv] | qacc [nv] | ncon (int bits) |
// DX_NCON_HI x {b1, b2 (int bits), pos[3], force[3] (world, acting on b2)}.
__host__ __device__ inline int dx_sensor_stash_words(int nq, int nv) { return nq + 2 * nv + 1 + 8 * DX_NCON_HI; }

extern "C" __global__ void __launch_bounds__(64) dx_sensor_kernel(const DevModel* __restrict__ mp, DevBatch B, Lds L,
                                                                  float* out) {
  extern __shared__ float smem[];
  const DevModel& m = *(const DevModel*)(const DXG DevModel*)mp;
  const int env = (int)blockIdx.x;
  if (env >= B.nenv) return;
  CtxT<SpecRT> c(m, L, smem, nullptr, nullptr);
  c.I = (int*)(smem + L.ints);
  for (int k = LANE; k < L.total + 6 * DX_MAX_NV; k += DX_WAVE) smem[k] = 0.f;
  SYNC();
  const int nq = c.nq, nv = c.nv, nb = c.nbody;
  const float* st = B.sen_stash + (size_t)env * dx_sensor_stash_words(nq, nv);
  float* qpos = c.f(L.qpos);
  float* qvel = c.f(L.qvel);
  float* qacc = c.f(L.qacc);
  for (int i = LANE; i < nq; i += DX_WAVE) qpos[i] = st[i];
  for (int i = LANE; i < nv; i += DX_WAVE) {
    qvel[i] = st[nq + i];
    qacc[i] = st[nq + nv + i];
  }
  SYNC();
  kin_com(c);  // xpos, xmat, xipos, cinert, cdof, subtree com (rcom) at the stashed qpos
  float* cdof = c.f(L.cdof);
  float* cdd = c.f(L.cdof_dot);
  float* cinert = c.f(L.cinert);
  const float* xpos = c.f(L.xpos);
  const float* xmat = c.f(L.xmat);
  const float* xipos = c.f(L.xipos);
  const float* rcom = c.f(L.rcom);
  // cdof_dot, lane = dof (mj_comVel as chain sums, as dx_step.hip velocity_stage)
  for (int d = LANE; d < nv; d += DX_WAVE) {
    const float4 d0 = m.dof_rec[2 * d], d1 = m.dof_rec[2 * d + 1];
    const int tk = __float_as_int(d0.w), k = tk >> 8;
    const bool fr = (tk & 255) == DXJ_FREE;
    const uint64_t anc = (uint64_t)(uint32_t)__float_as_int(d1.z) | ((uint64_t)(uint32_t)__float_as_int(d1.w) << 32);
    uint64_t mask = anc & ((1ull << (fr ? d - k + 3 : d)) - 1ull);
    float cv[6] = {0, 0, 0, 0, 0, 0};
    for (; mask; mask &= mask - 1) {
      const int e = __ffsll((long long)mask) - 1;
      for (int x = 0; x < 6; x++) cv[x] += cdof[6 * e + x] * qvel[e];
    }
    float o[6];
    cross_motion(o, cv, cdof + 6 * d);
    for (int x = 0; x < 6; x++) cdd[6 * d + x] = fr && k < 3 ? 0.f : o[x];
  }
  SYNC();
  // lane = body: cfrc_body - cfrc_ext, com frame of the body's tree
  float* acc = smem + L.total;  // [nbody][6]
  const int ncon = __float_as_int(st[nq + 2 * nv]);
  const float* cs = st + nq + 2 * nv + 1;
  const int b = LANE;
  if (b >= 1 && b < nb) {
    const uint64_t ch = m.body_chain[b];
    const float* rc = rcom + 3 * m.body_rootidx[b];
    float cv[6] = {0, 0, 0, 0, 0, 0};
    float ca[6] = {0, 0, 0, -m.gravity[0], -m.gravity[1], -m.gravity[2]};
    for (uint64_t mask = ch; mask; mask &= mask - 1) {
      const int e = __ffsll((long long)mask) - 1;
      for (int x = 0; x < 6; x++) {
        cv[x] += cdof[6 * e + x] * qvel[e];
        ca[x] += cdd[6 * e + x] * qvel[e] + cdof[6 * e + x] * qacc[e];
      }
    }
    float t1[6], t2[6], t3[6], f[6];
    mul_inert(t1, cinert + 10 * b, ca);
    mul_inert(t2, cinert + 10 * b, cv);
    cross_force(t3, cv, t2);
    for (int x = 0; x < 6; x++) f[x] = t1[x] + t3[x];
    if (B.xfrc) {  // applied wrench at the body com (xfrc rows: force, torque)
      const float* x6 = B.xfrc + 6 * b;
      const float off[3] = {xipos[3 * b] - rc[0], xipos[3 * b + 1] - rc[1], xipos[3 * b + 2] - rc[2]};
      float tq[3];
      cross3(tq, off, x6);
      f[0] -= x6[3] + tq[0]; f[1] -= x6[4] + tq[1]; f[2] -= x6[5] + tq[2];
      f[3] -= x6[0]; f[4] -= x6[1]; f[5] -= x6[2];
    }
    for (int ci = 0; ci < ncon; ci++) {  // contact force: on b2, its reaction on b1
      const float* r = cs + 8 * ci;
      const int b1 = __float_as_int(r[0]), b2 = __float_as_int(r[1]);
      if (b != b1 && b != b2) continue;
      const float s = b == b2 ? 1.f : -1.f;
      const float off[3] = {r[2] - rc[0], r[3] - rc[1], r[4] - rc[2]};
      float tq[3];
      cross3(tq, off, r + 5);
      f[0] -= s * tq[0]; f[1] -= s * tq[1]; f[2] -= s * tq[2];
      f[3] -= s * r[5]; f[4] -= s * r[6]; f[5] -= s * r[7];
    }
    for (int x = 0; x < 6; x++) acc[6 * b + x] = f[x];
  }
  SYNC();
  // cfrc_int: subtree sums, children before parents (bodies are in DFS order)
  if (LANE == 0)
    for (int k = nb - 1; k > 0; k--) {
      const int p = m.body_parent[k];
      if (p > 0)
        for (int x = 0; x < 6; x++) acc[6 * p + x] += acc[6 * k + x];
    }
  SYNC();
  // torque sensor on a site at the body origin: R^T (torque - (xpos - com) x force)
  if (b < nb) {
    float sv[3] = {0, 0, 0};
    if (b >= 1) {
      const float* f = acc + 6 * b;
      const float* rc = rcom + 3 * m.body_rootidx[b];
      const float dif[3] = {xpos[3 * b] - rc[0], xpos[3 * b + 1] - rc[1], xpos[3 * b + 2] - rc[2]};
      float cr[3];
      cross3(cr, dif, f + 3);
      const float t[3] = {f[0] - cr[0], f[1] - cr[1], f[2] - cr[2]};
      mattvec3(sv, xmat + 9 * b, t);
    }
    float* o = out + ((size_t)env * nb + b) * 3;
    o[0] = sv[0]; o[1] = sv[1]; o[2] = sv[2];
  }
}

hipError_t dx_launch_sensor(int nenv, size_t lds, hipStream_t stream, const DevModel* mdev, const DevBatch& B,
                            const Lds& L, float* out) {
  hipLaunchKernelGGL(dx_sensor_kernel, dim3(nenv), dim3(64), lds, stream, mdev, B, L, out);
  return hipGetLastError();
}
