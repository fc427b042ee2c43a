/*
 * dx_oracle.c -- TEST INFRASTRUCTURE ONLY (see dx_oracle.h).
 *
 * fp64 scalar restatement of MuJoCo's mj_step (Euler) for the dexterity scenes.
 * Pipeline and the reference file that configures each stage:
 *   kinematics / comPos ........ body tree of shadow_hand_series_e.xml:270-665,
 *                                adroit_hand.xml:61-230, cube free joint reorient.py:134
 *   tendon / transmission ...... shadow_hand_position_actuators.xml:4-21, adroit_hand.xml:252-397
 *   CRB + dense Cholesky ....... armature shadow_hand_series_e.xml:227
 *   collision .................. contype/exclude shadow_hand_series_e.xml:667-694, ground
 *                                models/arenas/standard.py:16-23, fall test reorient.py:229-235
 *   constraints ................ frictionloss/limits shadow_hand_series_e.xml:227, contacts
 *   smooth dynamics ............ actuators shadow_hand_position_actuators.xml:25-54,
 *                                gravity compensation utils/mujoco_utils.py:91-99
 *   Newton solver .............. [3P] MuJoCo default solver (no solver= in any reference XML);
 *                                CG and PGS for <option solver=...> ([3P] mj_solCG, mj_solPGS)
 *   Euler (implicit damping) ... [3P] MuJoCo default integrator, dt from reorient.py:58 / reach.py:54
 * MuJoCo itself is third-party and absent: every [3P] semantic restated here is
 * listed in DESIGN.md §3 ("parity unpinned" against real MuJoCo).
 */
#include "dx_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MINVAL 1e-15
#define NCON_MAX 256
#define MPR_TOL 1e-6
#define MPR_ITER 50

enum { GEOM_PLANE = 0, GEOM_SPHERE = 2, GEOM_CAPSULE = 3, GEOM_BOX = 6, GEOM_MESH = 7 };
enum { JNT_FREE = 0, JNT_HINGE = 3 };
enum { EFC_FRIC_DOF = 0, EFC_LIM_JNT = 2, EFC_LIM_TEN = 3, EFC_CON_PYR = 4, EFC_CON_FL = 5 };

/* ------------------------------------------------------------------------ */
/* model                                                                     */
/* ------------------------------------------------------------------------ */
struct dxo_model {
  unsigned char* blob;
  size_t nbytes;
  int nq, nv, nbody, njnt, ngeom, nsite, nu, ntendon, nwrap, nmesh, nbpair, ngpair;
  int iterations, disable_contact, any_damping, solver;
  double timestep, tolerance, impratio, meaninertia;
  const double* gravity;
  const int *body_parent, *body_rootid, *body_weldid, *body_jntnum, *body_jntadr, *body_dofnum,
      *body_dofadr;
  const double *body_pos, *body_quat, *body_ipos, *body_iquat, *body_mass, *body_inertia,
      *body_bsphere, *body_invweight0;
  const int *jnt_type, *jnt_bodyid, *jnt_qposadr, *jnt_dofadr, *jnt_limited;
  const double *jnt_pos, *jnt_axis, *jnt_range, *jnt_margin, *jnt_solref, *jnt_solimp, *qpos0;
  const int *dof_bodyid, *dof_jntid, *dof_parentid;
  const double *dof_armature, *dof_damping, *dof_frictionloss, *dof_solref, *dof_solimp,
      *dof_invweight0;
  const int *geom_type, *geom_bodyid, *geom_dataid;
  const double *geom_size, *geom_pos, *geom_quat, *geom_center, *geom_bsphere, *geom_aabb;
  const int *mesh_vertadr, *mesh_vertnum;
  const double* mesh_vert;
  const int* site_bodyid;
  const double *site_pos, *site_quat;
  const int *tendon_adr, *tendon_num, *tendon_limited, *wrap_dof;
  const double *tendon_range, *tendon_margin, *tendon_solref, *tendon_solimp, *tendon_invweight0,
      *wrap_coef;
  const int *actuator_trntype, *actuator_trnid, *actuator_biastype, *actuator_ctrllimited,
      *actuator_forcelimited;
  const double *actuator_gear, *actuator_gainprm, *actuator_biasprm, *actuator_ctrlrange,
      *actuator_forcerange;
  const int *bpair_body, *bpair_adr, *bpair_num, *bpair_plane, *gpair_geom, *gpair_condim;
  const double* bpair_sphere;
  const double *gpair_friction, *gpair_solref, *gpair_solimp, *gpair_margin;
};

static const void* blob_find(const unsigned char* blob, size_t nbytes, const char* name, int dtype,
                             long* count) {
  long n = *(const long*)(blob + 8);
  const unsigned char* p = blob + 16;
  for (long i = 0; i < n; i++, p += 72) {
    if (strncmp((const char*)p, name, 48) == 0) {
      int code = *(const int*)(p + 48);
      long cnt = *(const long*)(p + 56);
      long off = *(const long*)(p + 64);
      if (code != dtype || off < 0 || (size_t)off > nbytes) return NULL;
      if (count) *count = cnt;
      return blob + off;
    }
  }
  return NULL;
}

#define GETI(field)                                                                     \
  do {                                                                                  \
    m->field = (const int*)blob_find(m->blob, nbytes, #field, 0, &cnt);                 \
    if (!m->field) { fprintf(stderr, "dxo: missing %s\n", #field); ok = 0; }            \
  } while (0)
#define GETD(field)                                                                     \
  do {                                                                                  \
    m->field = (const double*)blob_find(m->blob, nbytes, #field, 1, &cnt);              \
    if (!m->field) { fprintf(stderr, "dxo: missing %s\n", #field); ok = 0; }            \
  } while (0)

dxo_model* dxo_model_load(const void* blob, size_t nbytes) {
  if (nbytes < 16 || memcmp(blob, "DXMBLOB1", 8) != 0) return NULL;
  dxo_model* m = (dxo_model*)calloc(1, sizeof(dxo_model));
  m->blob = (unsigned char*)malloc(nbytes);
  memcpy(m->blob, blob, nbytes);
  m->nbytes = nbytes;
  long cnt = 0;
  int ok = 1;
  const int* s;
#define SCALARI(name)                                              \
  s = (const int*)blob_find(m->blob, nbytes, #name, 0, &cnt);     \
  if (!s) { fprintf(stderr, "dxo: missing %s\n", #name); ok = 0; } \
  else m->name = s[0];
  SCALARI(nq) SCALARI(nv) SCALARI(nbody) SCALARI(njnt) SCALARI(ngeom) SCALARI(nsite) SCALARI(nu)
  SCALARI(ntendon) SCALARI(nwrap) SCALARI(nmesh) SCALARI(nbpair) SCALARI(ngpair)
  SCALARI(iterations) SCALARI(disable_contact)
#undef SCALARI
  const double* sd;
#define SCALARD(name)                                              \
  sd = (const double*)blob_find(m->blob, nbytes, #name, 1, &cnt); \
  if (!sd) { fprintf(stderr, "dxo: missing %s\n", #name); ok = 0; } \
  else m->name = sd[0];
  SCALARD(timestep) SCALARD(tolerance) SCALARD(impratio) SCALARD(meaninertia)
#undef SCALARD
  GETD(gravity);
  GETI(body_parent); GETI(body_rootid); GETI(body_weldid); GETI(body_jntnum); GETI(body_jntadr);
  GETI(body_dofnum); GETI(body_dofadr);
  GETD(body_pos); GETD(body_quat); GETD(body_ipos); GETD(body_iquat); GETD(body_mass);
  GETD(body_inertia); GETD(body_bsphere); GETD(body_invweight0);
  GETI(jnt_type); GETI(jnt_bodyid); GETI(jnt_qposadr); GETI(jnt_dofadr); GETI(jnt_limited);
  GETD(jnt_pos); GETD(jnt_axis); GETD(jnt_range); GETD(jnt_margin); GETD(jnt_solref);
  GETD(jnt_solimp); GETD(qpos0);
  GETI(dof_bodyid); GETI(dof_jntid); GETI(dof_parentid);
  GETD(dof_armature); GETD(dof_damping); GETD(dof_frictionloss); GETD(dof_solref);
  GETD(dof_solimp); GETD(dof_invweight0);
  GETI(geom_type); GETI(geom_bodyid); GETI(geom_dataid);
  GETD(geom_size); GETD(geom_pos); GETD(geom_quat); GETD(geom_center); GETD(geom_bsphere); GETD(geom_aabb);
  GETI(mesh_vertadr); GETI(mesh_vertnum); GETD(mesh_vert);
  GETI(site_bodyid); GETD(site_pos); GETD(site_quat);
  GETI(tendon_adr); GETI(tendon_num); GETI(tendon_limited); GETI(wrap_dof);
  GETD(tendon_range); GETD(tendon_margin); GETD(tendon_solref); GETD(tendon_solimp);
  GETD(tendon_invweight0); GETD(wrap_coef);
  GETI(actuator_trntype); GETI(actuator_trnid); GETI(actuator_biastype);
  GETI(actuator_ctrllimited); GETI(actuator_forcelimited);
  GETD(actuator_gear); GETD(actuator_gainprm); GETD(actuator_biasprm); GETD(actuator_ctrlrange);
  GETD(actuator_forcerange);
  GETI(bpair_body); GETI(bpair_adr); GETI(bpair_num); GETI(bpair_plane); GETD(bpair_sphere);
  GETI(gpair_geom); GETI(gpair_condim);
  GETD(gpair_friction); GETD(gpair_solref); GETD(gpair_solimp); GETD(gpair_margin);
  if (!ok) {
    dxo_model_free(m);
    return NULL;
  }
  /* optional <option solver>: 0 PGS (dual), 1 CG, 2 Newton (MuJoCo's default; absent
     in every reference scene) */
  s = (const int*)blob_find(m->blob, nbytes, "solver", 0, &cnt);
  m->solver = s ? s[0] : 2;
  if (m->solver < 0 || m->solver > 2) {
    fprintf(stderr, "dxo: solver %d not supported (PGS = 0, CG = 1, Newton = 2)\n", m->solver);
    dxo_model_free(m);
    return NULL;
  }
  m->any_damping = 0;
  for (int i = 0; i < m->nv; i++)
    if (m->dof_damping[i] > 0) m->any_damping = 1;
  return m;
}

void dxo_model_free(dxo_model* m) {
  if (!m) return;
  free(m->blob);
  free(m);
}

/* ------------------------------------------------------------------------ */
/* data                                                                      */
/* ------------------------------------------------------------------------ */
typedef struct {
  double pos[3], frame[9], dist, friction[5], solref[2], solimp[5], margin;
  int geom1, geom2, condim;
} OContact;

struct dxo_data {
  double time;
  double *qpos, *qvel, *ctrl, *qacc, *qacc_warmstart, *qacc_smooth, *xfrc_applied;
  double *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis;
  double *geom_xpos, *geom_xmat, *site_xpos, *site_xmat;
  double *subtree_com, *cinert, *cdof, *cvel, *cdof_dot, *crb, *cacc, *cfrc;
  double *cfrc_ext, *cfrc_int, *cacc_post, *sensor_torque;
  double *ten_length, *ten_J, *actuator_length, *actuator_moment, *actuator_force;
  double *M, *L, *H;
  double *qfrc_bias, *qfrc_passive, *qfrc_actuator, *qfrc_applied, *qfrc_smooth, *qfrc_constraint;
  int ncon;
  OContact* contact;
  int nefc, nefc_max;
  int *efc_type, *efc_id, *efc_state;
  double *efc_J, *efc_pos, *efc_margin, *efc_floss, *efc_diag, *efc_R, *efc_D, *efc_K, *efc_B,
      *efc_imp, *efc_vel, *efc_aref, *efc_jar, *efc_force, *efc_jv;
  double *tmp1, *tmp2, *tmp3, *tmp4, *tmp5, *mcom, *msum;
  int niter;
  double flops[DXO_NSTAGE];
  const dxo_model* model;
  int ncon_fixed;      /* test helper dxo_set_contacts: < 0 = run the narrowphase */
  double* con_fixed;   /* [ncon_fixed][16] records in dxo_contact's layout */
};

dxo_data* dxo_data_create(const dxo_model* m) {
  dxo_data* d = (dxo_data*)calloc(1, sizeof(dxo_data));
  d->model = m;
  int nq = m->nq, nv = m->nv, nb = m->nbody, ng = m->ngeom, ns = m->nsite;
  d->qpos = calloc(nq, 8); d->qvel = calloc(nv, 8); d->ctrl = calloc(m->nu > 0 ? m->nu : 1, 8);
  d->qacc = calloc(nv, 8); d->qacc_warmstart = calloc(nv, 8); d->qacc_smooth = calloc(nv, 8);
  d->xfrc_applied = calloc(6 * nb, 8);
  d->xpos = calloc(3 * nb, 8); d->xquat = calloc(4 * nb, 8); d->xmat = calloc(9 * nb, 8);
  d->xipos = calloc(3 * nb, 8); d->ximat = calloc(9 * nb, 8);
  d->xanchor = calloc(3 * (m->njnt + 1), 8); d->xaxis = calloc(3 * (m->njnt + 1), 8);
  d->geom_xpos = calloc(3 * (ng + 1), 8); d->geom_xmat = calloc(9 * (ng + 1), 8);
  d->site_xpos = calloc(3 * (ns + 1), 8); d->site_xmat = calloc(9 * (ns + 1), 8);
  d->subtree_com = calloc(3 * nb, 8); d->cinert = calloc(10 * nb, 8); d->cdof = calloc(6 * nv, 8);
  d->cvel = calloc(6 * nb, 8); d->cdof_dot = calloc(6 * nv, 8); d->crb = calloc(10 * nb, 8);
  d->cacc = calloc(6 * nb, 8); d->cfrc = calloc(6 * nb, 8);
  d->cfrc_ext = calloc(6 * nb, 8); d->cfrc_int = calloc(6 * nb, 8); d->cacc_post = calloc(6 * nb, 8);
  d->sensor_torque = calloc(3 * nb, 8);
  d->ten_length = calloc(m->ntendon + 1, 8); d->ten_J = calloc((m->ntendon + 1) * nv, 8);
  d->actuator_length = calloc(m->nu + 1, 8); d->actuator_moment = calloc((m->nu + 1) * nv, 8);
  d->actuator_force = calloc(m->nu + 1, 8);
  d->M = calloc(nv * nv, 8); d->L = calloc(nv * nv, 8); d->H = calloc(nv * nv, 8);
  d->qfrc_bias = calloc(nv, 8); d->qfrc_passive = calloc(nv, 8); d->qfrc_actuator = calloc(nv, 8);
  d->qfrc_applied = calloc(nv, 8); d->qfrc_smooth = calloc(nv, 8); d->qfrc_constraint = calloc(nv, 8);
  d->contact = calloc(NCON_MAX, sizeof(OContact));
  int ne = 4 * NCON_MAX + 2 * nv + 2 * m->ntendon + 8;
  d->nefc_max = ne;
  d->efc_type = calloc(ne, 4); d->efc_id = calloc(ne, 4); d->efc_state = calloc(ne, 4);
  d->efc_J = calloc((size_t)ne * nv, 8);
  d->efc_pos = calloc(ne, 8); d->efc_margin = calloc(ne, 8); d->efc_floss = calloc(ne, 8);
  d->efc_diag = calloc(ne, 8); d->efc_R = calloc(ne, 8); d->efc_D = calloc(ne, 8);
  d->efc_K = calloc(ne, 8); d->efc_B = calloc(ne, 8); d->efc_imp = calloc(ne, 8);
  d->efc_vel = calloc(ne, 8); d->efc_aref = calloc(ne, 8); d->efc_jar = calloc(ne, 8);
  d->efc_force = calloc(ne, 8); d->efc_jv = calloc(ne, 8);
  int nt = nv > 16 ? nv : 16;
  d->tmp1 = calloc(nt * 6, 8); d->tmp2 = calloc(nt * 6, 8); d->tmp3 = calloc(nt * 6, 8);
  d->tmp4 = calloc(nt * 6, 8); d->tmp5 = calloc(nt * 6, 8);
  d->mcom = calloc(3 * nb, 8); d->msum = calloc(nb, 8);
  d->ncon_fixed = -1;
  d->con_fixed = calloc(16 * NCON_MAX, 8);
  dxo_reset(m, d);
  return d;
}

void dxo_data_free(dxo_data* d) {
  if (!d) return;
  void* ptrs[] = {d->qpos, d->qvel, d->ctrl, d->qacc, d->qacc_warmstart, d->qacc_smooth,
                  d->xfrc_applied, d->xpos, d->xquat, d->xmat, d->xipos, d->ximat, d->xanchor,
                  d->xaxis, d->geom_xpos, d->geom_xmat, d->site_xpos, d->site_xmat,
                  d->subtree_com, d->cinert, d->cdof, d->cvel, d->cdof_dot, d->crb, d->cacc,
                  d->cfrc, d->cfrc_ext, d->cfrc_int, d->cacc_post, d->sensor_torque, d->ten_length, d->ten_J, d->actuator_length, d->actuator_moment,
                  d->actuator_force, d->M, d->L, d->H, d->qfrc_bias, d->qfrc_passive,
                  d->qfrc_actuator, d->qfrc_applied, d->qfrc_smooth, d->qfrc_constraint,
                  d->contact, d->efc_type, d->efc_id, d->efc_state, d->efc_J, d->efc_pos,
                  d->efc_margin, d->efc_floss, d->efc_diag, d->efc_R, d->efc_D, d->efc_K,
                  d->efc_B, d->efc_imp, d->efc_vel, d->efc_aref, d->efc_jar, d->efc_force,
                  d->efc_jv, d->tmp1, d->tmp2, d->tmp3, d->tmp4, d->tmp5, d->mcom, d->msum,
                  d->con_fixed};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); i++) free(ptrs[i]);
  free(d);
}

void dxo_reset(const dxo_model* m, dxo_data* d) {
  memcpy(d->qpos, m->qpos0, 8 * m->nq);
  memset(d->qvel, 0, 8 * m->nv);
  memset(d->qacc_warmstart, 0, 8 * m->nv);
  memset(d->ctrl, 0, 8 * (m->nu > 0 ? m->nu : 1));
  memset(d->xfrc_applied, 0, 8 * 6 * m->nbody);
  d->time = 0;
  d->ncon = 0;
  d->nefc = 0;
}

/* ------------------------------------------------------------------------ */
/* small vector helpers                                                      */
/* ------------------------------------------------------------------------ */
static inline double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static inline void cross3(double* r, const double* a, const double* b) {
  double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2],
         t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static inline double norm3(const double* a) { return sqrt(dot3(a, a)); }
static inline void sub3(double* r, const double* a, const double* b) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
static inline void add3(double* r, const double* a, const double* b) {
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
}
static inline void scl3(double* r, const double* a, double s) {
  r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s;
}
static inline double normalize3(double* a) {
  double n = norm3(a);
  if (n > MINVAL) { a[0] /= n; a[1] /= n; a[2] /= n; }
  return n;
}
static void quat2mat(double* R, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
static void quatmul(double* r, const double* a, const double* b) {
  double t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, 32);
}
static void quatnorm(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < MINVAL) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}
static void matvec3(double* r, const double* R, const double* v) {
  double t0 = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  double t1 = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  double t2 = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void mattvec3(double* r, const double* R, const double* v) {
  double t0 = R[0] * v[0] + R[3] * v[1] + R[6] * v[2];
  double t1 = R[1] * v[0] + R[4] * v[1] + R[7] * v[2];
  double t2 = R[2] * v[0] + R[5] * v[1] + R[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void matmul3(double* r, const double* A, const double* B) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(r, t, 72);
}

/* spatial algebra, vectors [angular(3); linear(3)], com-based frame */
static void mul_inert(double* r, const double* I, const double* v) {
  /* I = [Ixx Iyy Izz Ixy Ixz Iyz mcx mcy mcz m] about the com-frame origin */
  const double* w = v;
  const double* l = v + 3;
  const double* mc = I + 6;
  double m = I[9];
  r[0] = I[0] * w[0] + I[3] * w[1] + I[4] * w[2] + (mc[1] * l[2] - mc[2] * l[1]);
  r[1] = I[3] * w[0] + I[1] * w[1] + I[5] * w[2] + (mc[2] * l[0] - mc[0] * l[2]);
  r[2] = I[4] * w[0] + I[5] * w[1] + I[2] * w[2] + (mc[0] * l[1] - mc[1] * l[0]);
  r[3] = m * l[0] - (mc[1] * w[2] - mc[2] * w[1]);
  r[4] = m * l[1] - (mc[2] * w[0] - mc[0] * w[2]);
  r[5] = m * l[2] - (mc[0] * w[1] - mc[1] * w[0]);
}
static void cross_motion(double* r, const double* v, const double* m) {
  double a[3], b[3], c[3];
  cross3(a, v, m);
  cross3(b, v, m + 3);
  cross3(c, v + 3, m);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static void cross_force(double* r, const double* v, const double* f) {
  double a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
static inline double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

/* ------------------------------------------------------------------------ */
/* kinematics, com, cdof                                                     */
/* ------------------------------------------------------------------------ */
static void kinematics(const dxo_model* m, dxo_data* d) {
  d->xquat[0] = 1; d->xquat[1] = d->xquat[2] = d->xquat[3] = 0;
  quat2mat(d->xmat, d->xquat);
  memset(d->xpos, 0, 24);
  memcpy(d->xipos, d->xpos, 24);
  memcpy(d->ximat, d->xmat, 72);
  for (int b = 1; b < m->nbody; b++) {
    int p = m->body_parent[b], ja = m->body_jntadr[b], jn = m->body_jntnum[b];
    double* xp = d->xpos + 3 * b;
    double* xq = d->xquat + 4 * b;
    if (jn > 0 && m->jnt_type[ja] == JNT_FREE) {
      const double* q = d->qpos + m->jnt_qposadr[ja];
      xp[0] = q[0]; xp[1] = q[1]; xp[2] = q[2];
      memcpy(xq, q + 3, 32);
      quatnorm(xq);
      memcpy(d->xanchor + 3 * ja, xp, 24);
      d->xaxis[3 * ja] = 0; d->xaxis[3 * ja + 1] = 0; d->xaxis[3 * ja + 2] = 1;
      d->flops[DXO_ST_KIN] += 12;
    } else {
      double t[3];
      matvec3(t, d->xmat + 9 * p, m->body_pos + 3 * b);
      add3(xp, d->xpos + 3 * p, t);
      quatmul(xq, d->xquat + 4 * p, m->body_quat + 4 * b);
      d->flops[DXO_ST_KIN] += 15 + 28;
      for (int j = ja; j < ja + jn; j++) {
        double R[9], qloc[4];
        quat2mat(R, xq);
        matvec3(t, R, m->jnt_pos + 3 * j);
        add3(d->xanchor + 3 * j, t, xp);
        matvec3(d->xaxis + 3 * j, R, m->jnt_axis + 3 * j);
        double ang = d->qpos[m->jnt_qposadr[j]] - m->qpos0[m->jnt_qposadr[j]];
        double s = sin(0.5 * ang);
        qloc[0] = cos(0.5 * ang);
        qloc[1] = m->jnt_axis[3 * j] * s; qloc[2] = m->jnt_axis[3 * j + 1] * s;
        qloc[3] = m->jnt_axis[3 * j + 2] * s;
        quatmul(xq, xq, qloc);
        quatnorm(xq);
        quat2mat(R, xq);
        matvec3(t, R, m->jnt_pos + 3 * j);
        sub3(xp, d->xanchor + 3 * j, t);
        d->flops[DXO_ST_KIN] += 100;
      }
    }
    quat2mat(d->xmat + 9 * b, xq);
    double t[3], Ri[9];
    matvec3(t, d->xmat + 9 * b, m->body_ipos + 3 * b);
    add3(d->xipos + 3 * b, xp, t);
    quat2mat(Ri, m->body_iquat + 4 * b);
    matmul3(d->ximat + 9 * b, d->xmat + 9 * b, Ri);
    d->flops[DXO_ST_KIN] += 20 + 15 + 20 + 45;
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    double t[3], Rg[9];
    matvec3(t, d->xmat + 9 * b, m->geom_pos + 3 * g);
    add3(d->geom_xpos + 3 * g, d->xpos + 3 * b, t);
    quat2mat(Rg, m->geom_quat + 4 * g);
    matmul3(d->geom_xmat + 9 * g, d->xmat + 9 * b, Rg);
    d->flops[DXO_ST_KIN] += 15 + 20 + 45;
  }
  for (int s = 0; s < m->nsite; s++) {
    int b = m->site_bodyid[s];
    double t[3], Rs[9];
    matvec3(t, d->xmat + 9 * b, m->site_pos + 3 * s);
    add3(d->site_xpos + 3 * s, d->xpos + 3 * b, t);
    quat2mat(Rs, m->site_quat + 4 * s);
    matmul3(d->site_xmat + 9 * s, d->xmat + 9 * b, Rs);
    d->flops[DXO_ST_KIN] += 80;
  }
}

static void com_pos(const dxo_model* m, dxo_data* d) {
  int nb = m->nbody;
  double* mc = d->mcom;
  double* ms = d->msum;
  for (int b = 0; b < nb; b++) {
    ms[b] = m->body_mass[b];
    scl3(mc + 3 * b, d->xipos + 3 * b, m->body_mass[b]);
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0) {
      ms[p] += ms[b];
      add3(mc + 3 * p, mc + 3 * p, mc + 3 * b);
    }
  }
  for (int b = 0; b < nb; b++) {
    if (ms[b] > MINVAL)
      scl3(d->subtree_com + 3 * b, mc + 3 * b, 1.0 / ms[b]);
    else
      memcpy(d->subtree_com + 3 * b, d->xipos + 3 * b, 24);
  }
  d->flops[DXO_ST_KIN] += 10.0 * nb;
  /* cinert: inertia about subtree com of the root, world orientation */
  memset(d->cinert, 0, 80);
  for (int b = 1; b < nb; b++) {
    const double* R = d->ximat + 9 * b;
    const double* I = m->body_inertia + 3 * b;
    double mass = m->body_mass[b];
    double off[3];
    sub3(off, d->xipos + 3 * b, d->subtree_com + 3 * m->body_rootid[b]);
    double Iw[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        Iw[3 * i + j] = R[3 * i] * I[0] * R[3 * j] + R[3 * i + 1] * I[1] * R[3 * j + 1] +
                        R[3 * i + 2] * I[2] * R[3 * j + 2];
    double dd = dot3(off, off);
    double* ci = d->cinert + 10 * b;
    ci[0] = Iw[0] + mass * (dd - off[0] * off[0]);
    ci[1] = Iw[4] + mass * (dd - off[1] * off[1]);
    ci[2] = Iw[8] + mass * (dd - off[2] * off[2]);
    ci[3] = Iw[1] - mass * off[0] * off[1];
    ci[4] = Iw[2] - mass * off[0] * off[2];
    ci[5] = Iw[5] - mass * off[1] * off[2];
    ci[6] = mass * off[0]; ci[7] = mass * off[1]; ci[8] = mass * off[2];
    ci[9] = mass;
    d->flops[DXO_ST_KIN] += 45 + 30;
  }
  /* cdof */
  for (int j = 0; j < m->njnt; j++) {
    int b = m->jnt_bodyid[j], da = m->jnt_dofadr[j];
    double off[3];
    sub3(off, d->subtree_com + 3 * m->body_rootid[b], d->xanchor + 3 * j);
    if (m->jnt_type[j] == JNT_FREE) {
      for (int k = 0; k < 3; k++) {
        double* c = d->cdof + 6 * (da + k);
        memset(c, 0, 48);
        c[3 + k] = 1;
      }
      for (int k = 0; k < 3; k++) {
        double* c = d->cdof + 6 * (da + 3 + k);
        const double* R = d->xmat + 9 * b;
        double ax[3] = {R[k], R[3 + k], R[6 + k]};
        memcpy(c, ax, 24);
        cross3(c + 3, ax, off);
      }
      d->flops[DXO_ST_KIN] += 30;
    } else {
      double* c = d->cdof + 6 * da;
      memcpy(c, d->xaxis + 3 * j, 24);
      cross3(c + 3, d->xaxis + 3 * j, off);
      d->flops[DXO_ST_KIN] += 12;
    }
  }
}

/* tendon lengths / jacobians and actuator transmission */
static void tendon_transmission(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  for (int t = 0; t < m->ntendon; t++) {
    double len = 0;
    double* J = d->ten_J + t * nv;
    memset(J, 0, 8 * nv);
    for (int w = m->tendon_adr[t]; w < m->tendon_adr[t] + m->tendon_num[t]; w++) {
      int dof = m->wrap_dof[w];
      int qa = m->jnt_qposadr[m->dof_jntid[dof]];
      len += m->wrap_coef[w] * d->qpos[qa];
      J[dof] += m->wrap_coef[w];
    }
    d->ten_length[t] = len;
    d->flops[DXO_ST_CRB] += 2.0 * m->tendon_num[t];
  }
  for (int i = 0; i < m->nu; i++) {
    double* mom = d->actuator_moment + i * nv;
    memset(mom, 0, 8 * nv);
    double g = m->actuator_gear[i];
    if (m->actuator_trntype[i] == 0) {
      int j = m->actuator_trnid[i];
      d->actuator_length[i] = g * d->qpos[m->jnt_qposadr[j]];
      mom[m->jnt_dofadr[j]] = g;
    } else {
      int t = m->actuator_trnid[i];
      d->actuator_length[i] = g * d->ten_length[t];
      for (int k = 0; k < nv; k++) mom[k] = g * d->ten_J[t * nv + k];
    }
  }
}

/* composite rigid body mass matrix (dense) + armature, then Cholesky */
static int cholesky(double* L, const double* A, int n, double* flops) {
  if (L != A) memcpy(L, A, 8 * n * n);
  for (int j = 0; j < n; j++) {
    double s = L[j * n + j];
    for (int k = 0; k < j; k++) s -= L[j * n + k] * L[j * n + k];
    if (s <= MINVAL) s = MINVAL;
    double ljj = sqrt(s);
    L[j * n + j] = ljj;
    for (int i = j + 1; i < n; i++) {
      double v = L[i * n + j];
      for (int k = 0; k < j; k++) v -= L[i * n + k] * L[j * n + k];
      L[i * n + j] = v / ljj;
    }
    for (int i = 0; i < j; i++) L[i * n + j] = 0;
  }
  *flops += (double)n * n * n / 3.0;
  return 0;
}
static void chol_solve(const double* L, double* x, const double* b, int n, double* flops) {
  for (int i = 0; i < n; i++) {
    double v = b[i];
    for (int k = 0; k < i; k++) v -= L[i * n + k] * x[k];
    x[i] = v / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double v = x[i];
    for (int k = i + 1; k < n; k++) v -= L[k * n + i] * x[k];
    x[i] = v / L[i * n + i];
  }
  *flops += 2.0 * n * n;
}


static void crb(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  memcpy(d->crb, d->cinert, 80 * m->nbody);
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[10 * p + k] += d->crb[10 * b + k];
  }
  memset(d->M, 0, 8 * nv * nv);
  for (int i = 0; i < nv; i++) {
    double f[6];
    mul_inert(f, d->crb + 10 * m->dof_bodyid[i], d->cdof + 6 * i);
    d->flops[DXO_ST_CRB] += 36;
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      double v = dot6(d->cdof + 6 * j, f);
      d->M[i * nv + j] = v;
      d->M[j * nv + i] = v;
      d->flops[DXO_ST_CRB] += 11;
    }
    d->M[i * nv + i] += m->dof_armature[i];
  }
  cholesky(d->L, d->M, nv, &d->flops[DXO_ST_CRB]);
}

/* ------------------------------------------------------------------------ */
/* velocity stage: comVel, passive, RNE, actuation, applied, qacc_smooth     */
/* ------------------------------------------------------------------------ */
static void com_vel(const dxo_model* m, dxo_data* d) {
  memset(d->cvel, 0, 48);
  for (int b = 1; b < m->nbody; b++) {
    double* cv = d->cvel + 6 * b;
    memcpy(cv, d->cvel + 6 * m->body_parent[b], 48);
    int ja = m->body_jntadr[b], jn = m->body_jntnum[b];
    for (int j = ja; j < ja + jn; j++) {
      int da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == JNT_FREE) {
        for (int k = 0; k < 3; k++) memset(d->cdof_dot + 6 * (da + k), 0, 48);
        for (int k = 0; k < 3; k++)
          for (int e = 0; e < 6; e++) cv[e] += d->cdof[6 * (da + k) + e] * d->qvel[da + k];
        for (int k = 3; k < 6; k++) cross_motion(d->cdof_dot + 6 * (da + k), cv, d->cdof + 6 * (da + k));
        for (int k = 3; k < 6; k++)
          for (int e = 0; e < 6; e++) cv[e] += d->cdof[6 * (da + k) + e] * d->qvel[da + k];
        d->flops[DXO_ST_SMOOTH] += 6 * 12 + 3 * 30;
      } else {
        cross_motion(d->cdof_dot + 6 * da, cv, d->cdof + 6 * da);
        for (int e = 0; e < 6; e++) cv[e] += d->cdof[6 * da + e] * d->qvel[da];
        d->flops[DXO_ST_SMOOTH] += 30 + 12;
      }
    }
  }
}

static void rne(const dxo_model* m, dxo_data* d) {
  double* cacc = d->cacc;
  double* cfrc = d->cfrc;
  memset(cacc, 0, 48);
  cacc[3] = -m->gravity[0]; cacc[4] = -m->gravity[1]; cacc[5] = -m->gravity[2];
  for (int b = 1; b < m->nbody; b++) {
    double* ca = cacc + 6 * b;
    memcpy(ca, cacc + 6 * m->body_parent[b], 48);
    for (int j = m->body_dofadr[b]; j >= 0 && j < m->body_dofadr[b] + m->body_dofnum[b]; j++)
      for (int e = 0; e < 6; e++) ca[e] += d->cdof_dot[6 * j + e] * d->qvel[j];
    double t1[6], t2[6], t3[6];
    mul_inert(t1, d->cinert + 10 * b, ca);
    mul_inert(t2, d->cinert + 10 * b, d->cvel + 6 * b);
    cross_force(t3, d->cvel + 6 * b, t2);
    for (int e = 0; e < 6; e++) cfrc[6 * b + e] = t1[e] + t3[e];
    d->flops[DXO_ST_SMOOTH] += 12.0 * m->body_dofnum[b] + 36 + 36 + 30 + 6;
  }
  for (int b = m->nbody - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0)
      for (int e = 0; e < 6; e++) cfrc[6 * p + e] += cfrc[6 * b + e];
  }
  for (int j = 0; j < m->nv; j++) d->qfrc_bias[j] = dot6(d->cdof + 6 * j, cfrc + 6 * m->dof_bodyid[j]);
  d->flops[DXO_ST_SMOOTH] += 6.0 * m->nbody + 11.0 * m->nv;
}

/* jacobian columns of a point on body b: jacp[3*nv] jacr[3*nv] (zeroed first) */
static void jac_point(const dxo_model* m, const dxo_data* d, int b, const double* point,
                      double* jacp, double* jacr) {
  int nv = m->nv;
  if (jacp) memset(jacp, 0, 24 * nv);
  if (jacr) memset(jacr, 0, 24 * nv);
  int bb = b;
  while (bb > 0 && m->body_dofnum[bb] == 0) bb = m->body_parent[bb];
  if (bb == 0) return;
  int j = m->body_dofadr[bb] + m->body_dofnum[bb] - 1;
  double off[3];
  sub3(off, point, d->subtree_com + 3 * m->body_rootid[b]);
  for (; j >= 0; j = m->dof_parentid[j]) {
    const double* c = d->cdof + 6 * j;
    double t[3];
    cross3(t, c, off);
    if (jacp) { jacp[j] = c[3] + t[0]; jacp[nv + j] = c[4] + t[1]; jacp[2 * nv + j] = c[5] + t[2]; }
    if (jacr) { jacr[j] = c[0]; jacr[nv + j] = c[1]; jacr[2 * nv + j] = c[2]; }
  }
}

static void smooth_forces(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  /* passive: joint damping (no springs in these scenes) */
  for (int i = 0; i < nv; i++) d->qfrc_passive[i] = -m->dof_damping[i] * d->qvel[i];
  /* actuation: affine position servos, [3P] mj_fwdActuation */
  memset(d->qfrc_actuator, 0, 8 * nv);
  for (int i = 0; i < m->nu; i++) {
    double c = d->ctrl[i];
    if (m->actuator_ctrllimited[i]) {
      if (c < m->actuator_ctrlrange[2 * i]) c = m->actuator_ctrlrange[2 * i];
      if (c > m->actuator_ctrlrange[2 * i + 1]) c = m->actuator_ctrlrange[2 * i + 1];
    }
    const double* mom = d->actuator_moment + i * nv;
    double vel = 0;
    for (int k = 0; k < nv; k++) vel += mom[k] * d->qvel[k];
    double force = m->actuator_gainprm[3 * i] * c;
    if (m->actuator_biastype[i] == 1)
      force += m->actuator_biasprm[3 * i] + m->actuator_biasprm[3 * i + 1] * d->actuator_length[i] +
               m->actuator_biasprm[3 * i + 2] * vel;
    if (m->actuator_forcelimited[i]) {
      if (force < m->actuator_forcerange[2 * i]) force = m->actuator_forcerange[2 * i];
      if (force > m->actuator_forcerange[2 * i + 1]) force = m->actuator_forcerange[2 * i + 1];
    }
    d->actuator_force[i] = force;
    for (int k = 0; k < nv; k++) d->qfrc_actuator[k] += mom[k] * force;
    d->flops[DXO_ST_SMOOTH] += 4.0 * nv + 8;
  }
  /* applied: xfrc at body com (gravity compensation, mujoco_utils.py:91-99) */
  memset(d->qfrc_applied, 0, 8 * nv);
  double* jp = d->tmp3;
  double* jr = d->tmp4;
  for (int b = 1; b < m->nbody; b++) {
    const double* f = d->xfrc_applied + 6 * b;
    if (f[0] == 0 && f[1] == 0 && f[2] == 0 && f[3] == 0 && f[4] == 0 && f[5] == 0) continue;
    jac_point(m, d, b, d->xipos + 3 * b, jp, jr);
    for (int k = 0; k < nv; k++)
      d->qfrc_applied[k] += jp[k] * f[0] + jp[nv + k] * f[1] + jp[2 * nv + k] * f[2] +
                            jr[k] * f[3] + jr[nv + k] * f[4] + jr[2 * nv + k] * f[5];
    d->flops[DXO_ST_SMOOTH] += 12.0 * nv;
  }
  for (int i = 0; i < nv; i++)
    d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i] + d->qfrc_applied[i] + d->qfrc_actuator[i];
  chol_solve(d->L, d->qacc_smooth, d->qfrc_smooth, nv, &d->flops[DXO_ST_SMOOTH]);
}

/* ------------------------------------------------------------------------ */
/* collision                                                                 */
/* ------------------------------------------------------------------------ */
typedef struct {
  int type;
  const double *pos, *mat, *size;
  const double* vert; /* mesh hull vertices (local) */
  int nvert;
  double center[3];   /* world interior point */
  double margin;      /* half the pair margin (inflation) */
} Shape;

static void make_shape(const dxo_model* m, const dxo_data* d, int g, double half_margin, Shape* s) {
  s->type = m->geom_type[g];
  s->pos = d->geom_xpos + 3 * g;
  s->mat = d->geom_xmat + 9 * g;
  s->size = m->geom_size + 3 * g;
  s->vert = NULL;
  s->nvert = 0;
  if (s->type == GEOM_MESH) {
    int mid = m->geom_dataid[g];
    s->vert = m->mesh_vert + 3 * m->mesh_vertadr[mid];
    s->nvert = m->mesh_vertnum[mid];
  }
  double t[3];
  matvec3(t, s->mat, m->geom_center + 3 * g);
  add3(s->center, s->pos, t);
  s->margin = half_margin;
}

/* support point of a shape in world direction dir (not necessarily unit) */
static void support(const Shape* s, const double* dir, double* out, double* flops) {
  double ld[3];
  mattvec3(ld, s->mat, dir);
  double lp[3] = {0, 0, 0};
  switch (s->type) {
    case GEOM_BOX:
      for (int k = 0; k < 3; k++) lp[k] = (ld[k] >= 0 ? s->size[k] : -s->size[k]);
      *flops += 15;
      break;
    case GEOM_SPHERE: {
      double n = norm3(ld);
      if (n > MINVAL) scl3(lp, ld, s->size[0] / n);
      *flops += 10;
      break;
    }
    case GEOM_CAPSULE: {
      double n = norm3(ld);
      if (n > MINVAL) scl3(lp, ld, s->size[0] / n);
      lp[2] += (ld[2] >= 0 ? s->size[1] : -s->size[1]);
      *flops += 12;
      break;
    }
    case GEOM_MESH: {
      double best = -1e300;
      int bi = 0;
      for (int i = 0; i < s->nvert; i++) {
        double v = dot3(s->vert + 3 * i, ld);
        if (v > best) { best = v; bi = i; }
      }
      memcpy(lp, s->vert + 3 * bi, 24);
      /* 5 FLOP per vertex; an efficient support reads ~16 vertices (the kernel's binned
         cell block; MuJoCo hill-climbs the hull graph), the rest of this exhaustive scan
         goes to DXO_ST_SCAN (flops points at flops[DXO_ST_COL]) */
      const int eff = s->nvert < 16 ? s->nvert : 16;
      *flops += 5.0 * eff;
      flops[DXO_ST_SCAN - DXO_ST_COL] += 5.0 * (s->nvert - eff);
      break;
    }
  }
  matvec3(out, s->mat, lp);
  add3(out, out, s->pos);
  if (s->margin > 0) {
    double n = norm3(dir);
    if (n > MINVAL)
      for (int k = 0; k < 3; k++) out[k] += dir[k] / n * s->margin;
  }
  *flops += 18;
}

/* Minkowski portal refinement on A - B ([3P] libccd ccdMPRPenetration, as used by
 * MuJoCo's mjc_Convex).  Returns 1 with depth/normal/pos on penetration. */
typedef struct { double v[3], a[3], b[3]; } MPoint;

static void mpr_support(const Shape* A, const Shape* B, const double* dir, MPoint* p, double* fl) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  support(A, dir, p->a, fl);
  support(B, nd, p->b, fl);
  sub3(p->v, p->a, p->b);
}
static int is_zero(double x) { return fabs(x) < 1e-14; }

static void portal_dir(const MPoint* P, double* dir) {
  double a[3], b[3];
  sub3(a, P[2].v, P[1].v);
  sub3(b, P[3].v, P[1].v);
  cross3(dir, a, b);
  normalize3(dir);
}
static int portal_reach_tol(const MPoint* P, const MPoint* v4, const double* dir) {
  double dv4 = dot3(v4->v, dir);
  double d1 = dv4 - dot3(P[1].v, dir), d2 = dv4 - dot3(P[2].v, dir), d3 = dv4 - dot3(P[3].v, dir);
  double mn = d1 < d2 ? d1 : d2;
  mn = mn < d3 ? mn : d3;
  return mn <= MPR_TOL;
}
static void expand_portal(MPoint* P, const MPoint* v4) {
  double v4v0[3];
  cross3(v4v0, v4->v, P[0].v);
  if (dot3(P[1].v, v4v0) > 0) {
    if (dot3(P[2].v, v4v0) > 0) P[1] = *v4;
    else P[3] = *v4;
  } else {
    if (dot3(P[3].v, v4v0) > 0) P[2] = *v4;
    else P[1] = *v4;
  }
}
static double tri_point_dist2(const double* P, const double* a, const double* b, const double* c,
                              double* closest) {
  /* closest point on triangle abc to P (Ericson, Real-Time Collision Detection 5.1.5) */
  double ab[3], ac[3], ap[3];
  sub3(ab, b, a); sub3(ac, c, a); sub3(ap, P, a);
  double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  double q[3];
  if (d1 <= 0 && d2 <= 0) { memcpy(q, a, 24); goto done; }
  double bp[3]; sub3(bp, P, b);
  double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { memcpy(q, b, 24); goto done; }
  double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) {
    double v = d1 / (d1 - d3);
    for (int k = 0; k < 3; k++) q[k] = a[k] + v * ab[k];
    goto done;
  }
  double cp[3]; sub3(cp, P, c);
  double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { memcpy(q, c, 24); goto done; }
  double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) {
    double w = d2 / (d2 - d6);
    for (int k = 0; k < 3; k++) q[k] = a[k] + w * ac[k];
    goto done;
  }
  double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) q[k] = b[k] + w * (c[k] - b[k]);
    goto done;
  }
  {
    double denom = 1.0 / (va + vb + vc);
    double v = vb * denom, w = vc * denom;
    for (int k = 0; k < 3; k++) q[k] = a[k] + ab[k] * v + ac[k] * w;
  }
done:
  memcpy(closest, q, 24);
  double dd[3];
  sub3(dd, q, P);
  return dot3(dd, dd);
}
static void find_pos(const MPoint* P, double* pos) {
  double dir[3];
  portal_dir(P, dir);
  double b[4], t[3];
  cross3(t, P[2].v, P[3].v); b[0] = dot3(P[1].v, t);
  cross3(t, P[2].v, P[0].v); b[1] = dot3(P[3].v, t);
  cross3(t, P[1].v, P[3].v); b[2] = dot3(P[0].v, t);
  cross3(t, P[1].v, P[0].v); b[3] = dot3(P[2].v, t);
  double sum = b[0] + b[1] + b[2] + b[3];
  if (sum <= 0) {
    b[0] = 0;
    cross3(t, P[3].v, dir); b[1] = dot3(P[2].v, t);
    cross3(t, P[1].v, dir); b[2] = dot3(P[3].v, t);
    cross3(t, P[2].v, dir); b[3] = dot3(P[1].v, t);
    sum = b[1] + b[2] + b[3];
  }
  double inv = 1.0 / sum;
  double p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 3; k++) {
      p1[k] += b[i] * P[i].a[k];
      p2[k] += b[i] * P[i].b[k];
    }
  for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p1[k] + p2[k]) * inv;
}

static int mpr_penetration(const Shape* A, const Shape* B, double* depth, double* normal,
                           double* pos, double* fl) {
  MPoint P[4];
  /* discover portal */
  sub3(P[0].v, A->center, B->center);
  memcpy(P[0].a, A->center, 24);
  memcpy(P[0].b, B->center, 24);
  if (is_zero(P[0].v[0]) && is_zero(P[0].v[1]) && is_zero(P[0].v[2])) P[0].v[0] += 1e-10 * 10;
  double dir[3] = {-P[0].v[0], -P[0].v[1], -P[0].v[2]};
  normalize3(dir);
  mpr_support(A, B, dir, &P[1], fl);
  double dt = dot3(P[1].v, dir);
  if (is_zero(dt) || dt < 0) return 0;
  cross3(dir, P[0].v, P[1].v);
  if (is_zero(dot3(dir, dir))) {
    if (is_zero(P[1].v[0]) && is_zero(P[1].v[1]) && is_zero(P[1].v[2])) {
      /* origin on v1: touching contact */
      *depth = 0;
      normal[0] = normal[1] = 0; normal[2] = 1;
      for (int k = 0; k < 3; k++) pos[k] = 0.5 * (P[1].a[k] + P[1].b[k]);
      return 1;
    }
    /* origin on segment v0-v1 */
    *depth = norm3(P[1].v);
    memcpy(normal, P[1].v, 24);
    normalize3(normal);
    for (int k = 0; k < 3; k++) pos[k] = 0.5 * (P[1].a[k] + P[1].b[k]);
    return 1;
  }
  normalize3(dir);
  mpr_support(A, B, dir, &P[2], fl);
  dt = dot3(P[2].v, dir);
  if (is_zero(dt) || dt < 0) return 0;
  double va[3], vb[3];
  sub3(va, P[1].v, P[0].v);
  sub3(vb, P[2].v, P[0].v);
  cross3(dir, va, vb);
  normalize3(dir);
  if (dot3(dir, P[0].v) > 0) {
    MPoint t = P[1]; P[1] = P[2]; P[2] = t;
    scl3(dir, dir, -1);
  }
  for (int it = 0;; it++) {
    if (it > 1000) return 0;
    mpr_support(A, B, dir, &P[3], fl);
    dt = dot3(P[3].v, dir);
    if (is_zero(dt) || dt < 0) return 0;
    int cont = 0;
    cross3(va, P[1].v, P[3].v);
    dt = dot3(va, P[0].v);
    if (dt < 0 && !is_zero(dt)) { P[2] = P[3]; cont = 1; }
    if (!cont) {
      cross3(va, P[3].v, P[2].v);
      dt = dot3(va, P[0].v);
      if (dt < 0 && !is_zero(dt)) { P[1] = P[3]; cont = 1; }
    }
    if (cont) {
      sub3(va, P[1].v, P[0].v);
      sub3(vb, P[2].v, P[0].v);
      cross3(dir, va, vb);
      normalize3(dir);
    } else {
      break;
    }
  }
  /* refine portal until it encloses the origin */
  for (int it = 0;; it++) {
    portal_dir(P, dir);
    if (dot3(dir, P[1].v) >= 0) break; /* origin inside */
    MPoint v4;
    mpr_support(A, B, dir, &v4, fl);
    if (dot3(v4.v, dir) < 0 || portal_reach_tol(P, &v4, dir) || it > MPR_ITER) return 0;
    expand_portal(P, &v4);
  }
  /* find penetration */
  for (int it = 0;; it++) {
    portal_dir(P, dir);
    MPoint v4;
    mpr_support(A, B, dir, &v4, fl);
    if (portal_reach_tol(P, &v4, dir) || it > MPR_ITER) {
      double origin[3] = {0, 0, 0}, cl[3];
      double d2 = tri_point_dist2(origin, P[1].v, P[2].v, P[3].v, cl);
      *depth = sqrt(d2);
      if (*depth > MINVAL) {
        scl3(normal, cl, 1.0 / *depth);
      } else {
        memcpy(normal, dir, 24);
      }
      find_pos(P, pos);
      *fl += 200;
      return 1;
    }
    expand_portal(P, &v4);
    *fl += 60;
  }
}

static int add_contact(dxo_data* d, const dxo_model* m, int gp, int g1, int g2, const double* pos,
                       const double* normal, double dist) {
  if (d->ncon >= NCON_MAX) return 0;
  OContact* c = d->contact + d->ncon++;
  memcpy(c->pos, pos, 24);
  /* frame: normal, then tangents ([3P] mju_makeFrame) */
  memcpy(c->frame, normal, 24);
  double* y = c->frame + 3;
  if (fabs(normal[1]) < 0.5) { y[0] = 0; y[1] = 1; y[2] = 0; }
  else { y[0] = 0; y[1] = 0; y[2] = 1; }
  double t = dot3(normal, y);
  for (int k = 0; k < 3; k++) y[k] -= t * normal[k];
  normalize3(y);
  cross3(c->frame + 6, normal, y);
  c->dist = dist;
  c->geom1 = g1;
  c->geom2 = g2;
  c->condim = m->gpair_condim[gp];
  memcpy(c->friction, m->gpair_friction + 5 * gp, 40);
  memcpy(c->solref, m->gpair_solref + 2 * gp, 16);
  memcpy(c->solimp, m->gpair_solimp + 5 * gp, 40);
  c->margin = m->gpair_margin[gp];
  return 1;
}

static void collide_plane_box(const dxo_model* m, dxo_data* d, int gp, int g1, int g2,
                              double margin) {
  const double* pp = d->geom_xpos + 3 * g1;
  const double* pm = d->geom_xmat + 9 * g1;
  double n[3] = {pm[2], pm[5], pm[8]};
  const double* bp = d->geom_xpos + 3 * g2;
  const double* bm = d->geom_xmat + 9 * g2;
  const double* sz = m->geom_size + 3 * g2;
  double rel[3];
  sub3(rel, bp, pp);
  double cdist = dot3(rel, n);
  double ext = 0;
  for (int k = 0; k < 3; k++) ext += fabs(bm[k] * n[0] + bm[3 + k] * n[1] + bm[6 + k] * n[2]) * sz[k];
  d->flops[DXO_ST_COL] += 30;
  if (cdist > margin + ext) return;
  int cnt = 0;
  for (int i = 0; i < 8 && cnt < 4; i++) {
    double v[3];
    double s0 = (i & 1) ? sz[0] : -sz[0], s1 = (i & 2) ? sz[1] : -sz[1], s2 = (i & 4) ? sz[2] : -sz[2];
    for (int k = 0; k < 3; k++) v[k] = bp[k] + bm[3 * k] * s0 + bm[3 * k + 1] * s1 + bm[3 * k + 2] * s2;
    double r[3];
    sub3(r, v, pp);
    double dist = dot3(r, n);
    d->flops[DXO_ST_COL] += 30;
    if (dist <= margin) {
      double pos[3];
      for (int k = 0; k < 3; k++) pos[k] = v[k] - 0.5 * dist * n[k];
      if (add_contact(d, m, gp, g1, g2, pos, n, dist)) cnt++;
    }
  }
}

static void collide_plane_convex(const dxo_model* m, dxo_data* d, int gp, int g1, int g2,
                                 double margin) {
  const double* pp = d->geom_xpos + 3 * g1;
  const double* pm = d->geom_xmat + 9 * g1;
  double n[3] = {pm[2], pm[5], pm[8]};
  Shape s;
  make_shape(m, d, g2, 0, &s);
  double nd[3] = {-n[0], -n[1], -n[2]};
  double sp[3];
  support(&s, nd, sp, &d->flops[DXO_ST_COL]);
  double r[3];
  sub3(r, sp, pp);
  double dist = dot3(r, n);
  if (dist > margin) return;
  double pos[3];
  for (int k = 0; k < 3; k++) pos[k] = sp[k] - 0.5 * dist * n[k];
  add_contact(d, m, gp, g1, g2, pos, n, dist);
}

static void collide_convex(const dxo_model* m, dxo_data* d, int gp, int g1, int g2, double margin) {
  Shape A, B;
  make_shape(m, d, g1, 0.5 * margin, &A);
  make_shape(m, d, g2, 0.5 * margin, &B);
  double depth, normal[3], pos[3];
  if (mpr_penetration(&A, &B, &depth, normal, pos, &d->flops[DXO_ST_COL])) {
    add_contact(d, m, gp, g1, g2, pos, normal, margin - depth);
  }
}

/* segment-segment closest points, for capsule-capsule (Adroit explicit pairs) */
static void collide_capsules(const dxo_model* m, dxo_data* d, int gp, int g1, int g2, double margin) {
  const double *p1 = d->geom_xpos + 3 * g1, *m1 = d->geom_xmat + 9 * g1;
  const double *p2 = d->geom_xpos + 3 * g2, *m2 = d->geom_xmat + 9 * g2;
  double r1 = m->geom_size[3 * g1], h1 = m->geom_size[3 * g1 + 1];
  double r2 = m->geom_size[3 * g2], h2 = m->geom_size[3 * g2 + 1];
  double a1[3] = {m1[2] * h1, m1[5] * h1, m1[8] * h1}, a2[3] = {m2[2] * h2, m2[5] * h2, m2[8] * h2};
  /* segments p1 +- a1, p2 +- a2; minimize over s,t in [-1,1] */
  double dvec[3];
  sub3(dvec, p1, p2);
  double ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
  double u = -dot3(a1, dvec), v = dot3(a2, dvec);
  double det = ma * mc - mb * mb;
  double s, t;
  if (det > 1e-12) {
    s = (u * mc - mb * v) / det;
    t = (ma * v - mb * u) / det;
  } else {
    s = 0; t = 0;
  }
  for (int it = 0; it < 3; it++) {
    if (s < -1) s = -1; if (s > 1) s = 1;
    t = (v - mb * s) / (mc > 1e-12 ? mc : 1e-12);
    if (t < -1) t = -1; if (t > 1) t = 1;
    s = (u - mb * t) / (ma > 1e-12 ? ma : 1e-12);
    if (s < -1) s = -1; if (s > 1) s = 1;
  }
  double q1[3], q2[3];
  for (int k = 0; k < 3; k++) { q1[k] = p1[k] + s * a1[k]; q2[k] = p2[k] + t * a2[k]; }
  double diff[3];
  sub3(diff, q2, q1);
  double len = norm3(diff);
  double dist = len - r1 - r2;
  d->flops[DXO_ST_COL] += 80;
  if (dist > margin) return;
  double n[3];
  if (len > MINVAL) scl3(n, diff, 1.0 / len);
  else { n[0] = 1; n[1] = 0; n[2] = 0; }
  double pos[3];
  for (int k = 0; k < 3; k++) pos[k] = q1[k] + n[k] * (r1 + 0.5 * dist);
  add_contact(d, m, gp, g1, g2, pos, n, dist);
}

/* separating-axis test of the geoms' oriented bounding boxes (geom-frame AABBs);
 * conservative, so it only removes pairs MPR would reject. */
static int obb_overlap(const dxo_model* m, const dxo_data* d, int g1, int g2, double margin, double* fl) {
  double ca[3], cb[3];
  const double* a1 = m->geom_aabb + 6 * g1;
  const double* a2 = m->geom_aabb + 6 * g2;
  const double* Ra = d->geom_xmat + 9 * g1;
  const double* Rb = d->geom_xmat + 9 * g2;
  matvec3(ca, Ra, a1); add3(ca, ca, d->geom_xpos + 3 * g1);
  matvec3(cb, Rb, a2); add3(cb, cb, d->geom_xpos + 3 * g2);
  const double* ea = a1 + 3;
  const double* eb = a2 + 3;
  double t0[3], t[3], R[9], AR[9];
  sub3(t0, cb, ca);
  for (int i = 0; i < 3; i++) {
    t[i] = Ra[i] * t0[0] + Ra[3 + i] * t0[1] + Ra[6 + i] * t0[2];
    for (int j = 0; j < 3; j++) {
      R[3 * i + j] = Ra[i] * Rb[j] + Ra[3 + i] * Rb[3 + j] + Ra[6 + i] * Rb[6 + j];
      AR[3 * i + j] = fabs(R[3 * i + j]) + 1e-6;
    }
  }
  *fl += 150;
  for (int i = 0; i < 3; i++)
    if (fabs(t[i]) > ea[i] + eb[0] * AR[3 * i] + eb[1] * AR[3 * i + 1] + eb[2] * AR[3 * i + 2] + margin) return 0;
  for (int j = 0; j < 3; j++) {
    double tj = t[0] * R[j] + t[1] * R[3 + j] + t[2] * R[6 + j];
    if (fabs(tj) > ea[0] * AR[j] + ea[1] * AR[3 + j] + ea[2] * AR[6 + j] + eb[j] + margin) return 0;
  }
  for (int i = 0; i < 3; i++) {
    int i1 = (i + 1) % 3, i2 = (i + 2) % 3;
    for (int j = 0; j < 3; j++) {
      int j1 = (j + 1) % 3, j2 = (j + 2) % 3;
      double ra = ea[i1] * AR[3 * i2 + j] + ea[i2] * AR[3 * i1 + j];
      double rb = eb[j1] * AR[3 * i + j2] + eb[j2] * AR[3 * i + j1];
      double tt = t[i2] * R[3 * i1 + j] - t[i1] * R[3 * i2 + j];
      if (fabs(tt) > ra + rb + margin) return 0;
    }
  }
  return 1;
}

static int sphere_overlap(const double* c1, double r1, const double* c2, double r2, double margin) {
  double t[3];
  sub3(t, c1, c2);
  double rr = r1 + r2 + margin;
  return dot3(t, t) <= rr * rr;
}

/* Test helper (dxo_set_contacts): the contact list given instead of the narrowphase's --
 * point, normal, depth and geom pair from each record; frame, condim, friction, solref,
 * solimp and margin from the pair, as add_contact sets them for a found contact. */
static void fixed_contacts(const dxo_model* m, dxo_data* d) {
  for (int i = 0; i < d->ncon_fixed; i++) {
    const double* r = d->con_fixed + 16 * i;
    const int g1 = (int)r[13], g2 = (int)r[14];
    for (int gp = 0; gp < m->ngpair; gp++)
      if (m->gpair_geom[2 * gp] == g1 && m->gpair_geom[2 * gp + 1] == g2) {
        double n[3] = {r[3], r[4], r[5]};
        normalize3(n);
        add_contact(d, m, gp, g1, g2, r, n, r[12]);
        break;
      }
  }
}

static void collision(const dxo_model* m, dxo_data* d) {
  d->ncon = 0;
  if (m->disable_contact) return;
  if (d->ncon_fixed >= 0) {
    fixed_contacts(m, d);
    return;
  }
  for (int bp = 0; bp < m->nbpair; bp++) {
    int b1 = m->bpair_body[2 * bp], b2 = m->bpair_body[2 * bp + 1];
    const double* s1 = m->bpair_sphere + 8 * bp;
    const double* s2 = s1 + 4;
    double maxmargin = 0;
    for (int gp = m->bpair_adr[bp]; gp < m->bpair_adr[bp] + m->bpair_num[bp]; gp++)
      if (m->gpair_margin[gp] > maxmargin) maxmargin = m->gpair_margin[gp];
    if (s2[3] >= 0) {
      double c2[3];
      matvec3(c2, d->xmat + 9 * b2, s2); add3(c2, c2, d->xpos + 3 * b2);
      d->flops[DXO_ST_COL] += 20;
      int pg = m->bpair_plane[bp];
      if (pg >= 0) {
        const double* pm = d->geom_xmat + 9 * pg;
        double n[3] = {pm[2], pm[5], pm[8]}, r[3];
        sub3(r, c2, d->geom_xpos + 3 * pg);
        if (dot3(r, n) > s2[3] + maxmargin) continue;
      } else if (s1[3] >= 0) {
        double c1[3];
        matvec3(c1, d->xmat + 9 * b1, s1); add3(c1, c1, d->xpos + 3 * b1);
        d->flops[DXO_ST_COL] += 20;
        if (!sphere_overlap(c1, s1[3], c2, s2[3], maxmargin)) continue;
      }
    }
    for (int gp = m->bpair_adr[bp]; gp < m->bpair_adr[bp] + m->bpair_num[bp]; gp++) {
      int g1 = m->gpair_geom[2 * gp], g2 = m->gpair_geom[2 * gp + 1];
      int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
      double margin = m->gpair_margin[gp];
      /* mid-phase: geom bounding spheres (planes: signed distance) */
      const double* gs2 = m->geom_bsphere + 4 * g2;
      double c2[3];
      matvec3(c2, d->geom_xmat + 9 * g2, gs2); add3(c2, c2, d->geom_xpos + 3 * g2);
      d->flops[DXO_ST_COL] += 20;
      if (t1 == GEOM_PLANE) {
        const double* pm = d->geom_xmat + 9 * g1;
        double n[3] = {pm[2], pm[5], pm[8]}, r[3];
        sub3(r, c2, d->geom_xpos + 3 * g1);
        if (dot3(r, n) > gs2[3] + margin) continue;
        if (t2 == GEOM_BOX) collide_plane_box(m, d, gp, g1, g2, margin);
        else collide_plane_convex(m, d, gp, g1, g2, margin);
        continue;
      }
      const double* gs1 = m->geom_bsphere + 4 * g1;
      double c1[3];
      matvec3(c1, d->geom_xmat + 9 * g1, gs1); add3(c1, c1, d->geom_xpos + 3 * g1);
      d->flops[DXO_ST_COL] += 20;
      if (!sphere_overlap(c1, gs1[3], c2, gs2[3], margin)) continue;
      if (!obb_overlap(m, d, g1, g2, margin, &d->flops[DXO_ST_COL])) continue;
      if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) collide_capsules(m, d, gp, g1, g2, margin);
      else collide_convex(m, d, gp, g1, g2, margin);
    }
  }
}

/* ------------------------------------------------------------------------ */
/* constraints                                                               */
/* ------------------------------------------------------------------------ */
static double impedance(const double* solimp, double violation) {
  double d0 = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (d0 < 0.0001) d0 = 0.0001; if (d0 > 0.9999) d0 = 0.9999;
  if (dmax < 0.0001) dmax = 0.0001; if (dmax > 0.9999) dmax = 0.9999;
  if (width <= MINVAL || d0 == dmax) return 0.5 * (d0 + dmax);
  double x = fabs(violation) / width;
  if (x >= 1) return dmax;
  double y;
  if (power == 1) {
    y = x;
  } else if (x <= mid) {
    y = pow(x, power) / pow(mid, power - 1);
  } else {
    y = 1 - pow(1 - x, power) / pow(1 - mid, power - 1);
  }
  return d0 + y * (dmax - d0);
}

static int add_row(const dxo_model* m, dxo_data* d, int type, int id, double pos, double margin,
                   double floss, double diag, const double* solref, const double* solimp) {
  if (d->nefc >= d->nefc_max) return -1;
  int r = d->nefc++;
  d->efc_type[r] = type;
  d->efc_id[r] = id;
  d->efc_pos[r] = pos;
  d->efc_margin[r] = margin;
  d->efc_floss[r] = floss;
  d->efc_diag[r] = diag;
  double imp = impedance(solimp, pos - margin);
  double tc = solref[0], dr = solref[1];
  double dmax = solimp[1];
  if (dmax < 0.0001) dmax = 0.0001; if (dmax > 0.9999) dmax = 0.9999;
  if (tc < 2 * m->timestep) tc = 2 * m->timestep; /* refsafe */
  d->efc_K[r] = 1.0 / fmax(MINVAL, dmax * dmax * tc * tc * dr * dr);
  d->efc_B[r] = 2.0 / fmax(MINVAL, dmax * tc);
  d->efc_imp[r] = imp;
  d->efc_R[r] = fmax(MINVAL, (1 - imp) / imp * diag);
  memset(d->efc_J + (size_t)r * m->nv, 0, 8 * m->nv);
  return r;
}

static void make_constraint(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  d->nefc = 0;
  /* dof friction loss */
  for (int i = 0; i < nv; i++) {
    if (m->dof_frictionloss[i] <= 0) continue;
    int r = add_row(m, d, EFC_FRIC_DOF, i, 0, 0, m->dof_frictionloss[i], m->dof_invweight0[i],
                    m->dof_solref + 2 * i, m->dof_solimp + 5 * i);
    if (r >= 0) d->efc_J[(size_t)r * nv + i] = 1;
  }
  /* joint limits */
  for (int j = 0; j < m->njnt; j++) {
    if (!m->jnt_limited[j] || m->jnt_type[j] != JNT_HINGE) continue;
    double q = d->qpos[m->jnt_qposadr[j]];
    int dof = m->jnt_dofadr[j];
    for (int side = 0; side < 2; side++) {
      double dist = side == 0 ? q - m->jnt_range[2 * j] : m->jnt_range[2 * j + 1] - q;
      if (dist < m->jnt_margin[j]) {
        int r = add_row(m, d, EFC_LIM_JNT, j, dist, m->jnt_margin[j], 0, m->dof_invweight0[dof],
                        m->jnt_solref + 2 * j, m->jnt_solimp + 5 * j);
        if (r >= 0) d->efc_J[(size_t)r * nv + dof] = side == 0 ? 1 : -1;
      }
    }
  }
  /* tendon limits */
  for (int t = 0; t < m->ntendon; t++) {
    if (!m->tendon_limited[t]) continue;
    double len = d->ten_length[t];
    for (int side = 0; side < 2; side++) {
      double dist = side == 0 ? len - m->tendon_range[2 * t] : m->tendon_range[2 * t + 1] - len;
      if (dist < m->tendon_margin[t]) {
        int r = add_row(m, d, EFC_LIM_TEN, t, dist, m->tendon_margin[t], 0,
                        m->tendon_invweight0[t], m->tendon_solref + 2 * t,
                        m->tendon_solimp + 5 * t);
        if (r >= 0)
          for (int k = 0; k < nv; k++)
            d->efc_J[(size_t)r * nv + k] = (side == 0 ? 1 : -1) * d->ten_J[t * nv + k];
      }
    }
  }
  d->flops[DXO_ST_CON] += 40.0 * d->nefc;
  /* contacts */
  double* j1 = d->tmp1;
  double* j2 = d->tmp2;
  for (int c = 0; c < d->ncon; c++) {
    OContact* con = d->contact + c;
    int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
    jac_point(m, d, b1, con->pos, j1, NULL);
    jac_point(m, d, b2, con->pos, j2, NULL);
    double Jc[3 * 64];
    double* Jf = nv <= 64 ? Jc : (double*)malloc(24 * nv);
    for (int k = 0; k < nv; k++) {
      double dx = j2[k] - j1[k], dy = j2[nv + k] - j1[nv + k], dz = j2[2 * nv + k] - j1[2 * nv + k];
      for (int r = 0; r < 3; r++)
        Jf[r * nv + k] = con->frame[3 * r] * dx + con->frame[3 * r + 1] * dy + con->frame[3 * r + 2] * dz;
    }
    d->flops[DXO_ST_CON] += 24.0 * nv;
    double tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
    if (con->condim == 1) {
      int r = add_row(m, d, EFC_CON_FL, c, con->dist, con->margin, 0, tran, con->solref, con->solimp);
      if (r >= 0) memcpy(d->efc_J + (size_t)r * nv, Jf, 8 * nv);
    } else {
      /* pyramidal cone, edges J_n +- mu_k J_tk; R_edge = 2 mu_0^2 R_n / impratio */
      double mu0 = con->friction[0];
      for (int k = 1; k < 3; k++) {
        for (int sgn = 0; sgn < 2; sgn++) {
          int r = add_row(m, d, EFC_CON_PYR, c, con->dist, con->margin, 0, tran, con->solref,
                          con->solimp);
          if (r < 0) break;
          double mu = con->friction[k - 1] * (sgn == 0 ? 1 : -1);
          for (int q = 0; q < nv; q++) d->efc_J[(size_t)r * nv + q] = Jf[q] + mu * Jf[k * nv + q];
          d->efc_R[r] = fmax(MINVAL, 2 * mu0 * mu0 * d->efc_R[r] / m->impratio);
        }
      }
      d->flops[DXO_ST_CON] += 8.0 * nv;
    }
    if (Jf != Jc) free(Jf);
  }
  /* velocities and reference accelerations */
  for (int r = 0; r < d->nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    double v = 0;
    for (int k = 0; k < nv; k++) v += J[k] * d->qvel[k];
    d->efc_vel[r] = v;
    d->efc_D[r] = 1.0 / d->efc_R[r];
    double viol = d->efc_type[r] == EFC_FRIC_DOF ? 0 : d->efc_pos[r] - d->efc_margin[r];
    d->efc_aref[r] = -d->efc_B[r] * v - d->efc_K[r] * d->efc_imp[r] * viol;
  }
  d->flops[DXO_ST_CON] += (2.0 * nv + 10) * d->nefc;
}

/* ------------------------------------------------------------------------ */
/* Newton solver on MuJoCo's primal problem                                  */
/* ------------------------------------------------------------------------ */
/* cost of constraint row at jar; returns cost and writes force, hessian weight */
static double row_cost(const dxo_data* d, int r, double jar, double* force, double* hw) {
  double D = d->efc_D[r];
  int type = d->efc_type[r];
  if (type == EFC_FRIC_DOF) {
    double f = d->efc_floss[r], Rf = d->efc_R[r] * f;
    if (jar <= -Rf) { *force = f; *hw = 0; return -f * jar - 0.5 * Rf * f; }
    if (jar >= Rf) { *force = -f; *hw = 0; return f * jar - 0.5 * Rf * f; }
    *force = -D * jar; *hw = D; return 0.5 * D * jar * jar;
  }
  if (jar < 0) { *force = -D * jar; *hw = D; return 0.5 * D * jar * jar; }
  *force = 0; *hw = 0; return 0;
}

/* total cost at qacc (+ fills jar, force, Ma) */
static double eval_cost(const dxo_model* m, dxo_data* d, const double* qacc, double* Ma) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int k = 0; k < nv; k++) s += d->M[i * nv + k] * qacc[k];
    Ma[i] = s;
  }
  double gauss = 0;
  for (int i = 0; i < nv; i++) gauss += 0.5 * (qacc[i] - d->qacc_smooth[i]) * (Ma[i] - d->qfrc_smooth[i]);
  double cost = gauss;
  for (int r = 0; r < d->nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    double jv = 0;
    for (int k = 0; k < nv; k++) jv += J[k] * qacc[k];
    d->efc_jar[r] = jv - d->efc_aref[r];
    double f, hw;
    cost += row_cost(d, r, d->efc_jar[r], &f, &hw);
    d->efc_force[r] = f;
    d->efc_state[r] = hw > 0;
  }
  d->flops[DXO_ST_SOLVE] += 2.0 * nv * nv + 4.0 * nv + (2.0 * nv + 8) * d->nefc;
  return cost;
}

/* exact line search along dir: minimise f(a) = cost(qacc + a*dir) (convex, piecewise quadratic) */
static double line_search(const dxo_model* m, dxo_data* d, const double* qacc, const double* Ma,
                          const double* dir) {
  int nv = m->nv;
  double* Mdir = d->tmp5;
  for (int i = 0; i < nv; i++) {
    double s = 0;
    for (int k = 0; k < nv; k++) s += d->M[i * nv + k] * dir[k];
    Mdir[i] = s;
  }
  double qa = 0, qb = 0;
  for (int i = 0; i < nv; i++) {
    qa += dir[i] * Mdir[i];
    qb += dir[i] * (Ma[i] - d->qfrc_smooth[i]);
  }
  for (int r = 0; r < d->nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    double jv = 0;
    for (int k = 0; k < nv; k++) jv += J[k] * dir[k];
    d->efc_jv[r] = jv;
  }
  d->flops[DXO_ST_SOLVE] += 2.0 * nv * nv + 4.0 * nv + 2.0 * nv * d->nefc;
  /* derivative and curvature at alpha */
  double lo = 0, hi = -1, alpha = 0;
  double g0 = 0;
  for (int it = 0; it < 60; it++) {
    double g = qa * alpha + qb, h = qa;
    for (int r = 0; r < d->nefc; r++) {
      double jv = d->efc_jv[r];
      if (jv == 0) continue;
      double x = d->efc_jar[r] + alpha * jv;
      double f, hw;
      row_cost(d, r, x, &f, &hw);
      g += -f * jv;
      h += hw * jv * jv;
    }
    d->flops[DXO_ST_SOLVE] += 10.0 * d->nefc;
    if (it == 0) g0 = g;
    if (fabs(g) <= 1e-12 * fabs(g0) + 1e-300) break;
    if (g < 0) lo = alpha; else hi = alpha;
    double next = h > 0 ? alpha - g / h : alpha + 1;
    if (hi >= 0 && (next <= lo || next >= hi)) next = 0.5 * (lo + hi);
    if (hi < 0 && next <= lo) next = lo + 1;
    if (fabs(next - alpha) <= 1e-15 * (fabs(alpha) + 1e-30)) break;
    alpha = next;
  }
  return alpha;
}

static void solve_newton(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  double* Ma = d->tmp1;
  double* grad = d->tmp2;
  double* dir = d->tmp3;
  double* qacc = d->qacc;
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  /* warm start: pick the better of qacc_warmstart and qacc_smooth */
  memcpy(qacc, d->qacc_warmstart, 8 * nv);
  double cost = eval_cost(m, d, qacc, Ma);
  double cost_smooth = eval_cost(m, d, d->qacc_smooth, Ma);
  if (cost_smooth < cost) {
    memcpy(qacc, d->qacc_smooth, 8 * nv);
    cost = cost_smooth;
  } else {
    cost = eval_cost(m, d, qacc, Ma);
  }
  d->niter = 0;
  if (d->nefc == 0) {
    memcpy(qacc, d->qacc_smooth, 8 * nv);
    return;
  }
  for (int it = 0; it < m->iterations; it++) {
    /* gradient and Hessian */
    for (int i = 0; i < nv; i++) grad[i] = Ma[i] - d->qfrc_smooth[i];
    memcpy(d->H, d->M, 8 * nv * nv);
    for (int r = 0; r < d->nefc; r++) {
      const double* J = d->efc_J + (size_t)r * nv;
      for (int k = 0; k < nv; k++) grad[k] -= J[k] * d->efc_force[r];
      if (!d->efc_state[r]) continue;
      double D = d->efc_D[r];
      for (int i = 0; i < nv; i++) {
        if (J[i] == 0) continue;
        double a = D * J[i];
        for (int k = 0; k < nv; k++) d->H[i * nv + k] += a * J[k];
      }
    }
    d->flops[DXO_ST_SOLVE] += 2.0 * nv * d->nefc + 2.0 * nv * nv * d->nefc * 0.5;
    double gnorm = 0;
    for (int i = 0; i < nv; i++) gnorm += grad[i] * grad[i];
    gnorm = sqrt(gnorm) * scale;
    if (gnorm < m->tolerance) break;
    cholesky(d->H, d->H, nv, &d->flops[DXO_ST_SOLVE]);
    chol_solve(d->H, dir, grad, nv, &d->flops[DXO_ST_SOLVE]);
    for (int i = 0; i < nv; i++) dir[i] = -dir[i];
    double alpha = line_search(m, d, qacc, Ma, dir);
    for (int i = 0; i < nv; i++) qacc[i] += alpha * dir[i];
    double newcost = eval_cost(m, d, qacc, Ma);
    d->niter++;
    double improvement = scale * (cost - newcost);
    cost = newcost;
    if (improvement < m->tolerance) break;
  }
}

/* [3P] MuJoCo's primal CG (mj_solCG): the same cost, warm start and exact line search
 * as the Newton solver, with the search direction from Polak-Ribiere nonlinear
 * conjugate gradients preconditioned by M (Mgrad = M^-1 grad through M's factor), and
 * the same convergence tests (scaled improvement or scaled gradient < tolerance).  A
 * direction that is not a descent direction restarts along -Mgrad. */
static void solve_cg(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  double* Ma = d->tmp1;
  double* grad = d->tmp2;
  double* dir = d->tmp3;
  double* Mg = d->tmp4;
  double* Mg_old = d->H;  /* nv doubles of scratch (H is unused by CG) */
  double* qacc = d->qacc;
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  memcpy(qacc, d->qacc_warmstart, 8 * nv);
  double cost = eval_cost(m, d, qacc, Ma);
  double cost_smooth = eval_cost(m, d, d->qacc_smooth, Ma);
  if (cost_smooth < cost) {
    memcpy(qacc, d->qacc_smooth, 8 * nv);
    cost = cost_smooth;
  } else {
    cost = eval_cost(m, d, qacc, Ma);
  }
  d->niter = 0;
  if (d->nefc == 0) {
    memcpy(qacc, d->qacc_smooth, 8 * nv);
    return;
  }
  /* gradient = M qacc - qfrc_smooth - J^T force; Mgrad = M^-1 gradient */
#define CG_GRAD()                                                                   \
  do {                                                                              \
    for (int i = 0; i < nv; i++) grad[i] = Ma[i] - d->qfrc_smooth[i];               \
    for (int r = 0; r < d->nefc; r++) {                                             \
      const double* J = d->efc_J + (size_t)r * nv;                                  \
      for (int k = 0; k < nv; k++) grad[k] -= J[k] * d->efc_force[r];               \
    }                                                                               \
    chol_solve(d->L, Mg, grad, nv, &d->flops[DXO_ST_SOLVE]);                        \
    d->flops[DXO_ST_SOLVE] += 2.0 * nv * d->nefc;                                   \
  } while (0)
  CG_GRAD();
  double gMg_old = 0;
  for (int i = 0; i < nv; i++) { dir[i] = -Mg[i]; gMg_old += grad[i] * Mg[i]; }
  for (int it = 0; it < m->iterations; it++) {
    double alpha = line_search(m, d, qacc, Ma, dir);
    if (alpha == 0) break;
    for (int i = 0; i < nv; i++) qacc[i] += alpha * dir[i];
    double newcost = eval_cost(m, d, qacc, Ma);
    d->niter++;
    double improvement = scale * (cost - newcost);
    cost = newcost;
    memcpy(Mg_old, Mg, 8 * nv);
    CG_GRAD();
    double gnorm = 0;
    for (int i = 0; i < nv; i++) gnorm += grad[i] * grad[i];
    gnorm = sqrt(gnorm) * scale;
    if (improvement < m->tolerance || gnorm < m->tolerance) break;
    double num = 0, gMg = 0;
    for (int i = 0; i < nv; i++) { num += grad[i] * (Mg[i] - Mg_old[i]); gMg += grad[i] * Mg[i]; }
    double beta = num / fmax(MINVAL, gMg_old);
    if (beta < 0) beta = 0;
    gMg_old = gMg;
    double slope = 0;
    for (int i = 0; i < nv; i++) {
      dir[i] = -Mg[i] + beta * dir[i];
      slope += grad[i] * dir[i];
    }
    /* not a descent direction (the line search is exact only to its tolerance): restart
       along -M^-1 grad */
    if (!(slope < 0))
      for (int i = 0; i < nv; i++) dir[i] = -Mg[i];
    d->flops[DXO_ST_SOLVE] += 8.0 * nv;
  }
#undef CG_GRAD
}

/* [3P] MuJoCo's PGS (mj_solPGS): projected Gauss-Seidel on the dual problem
 *   min_f 0.5 f'(A + R) f + f'b,  A = J M^-1 J',  b = J qacc_smooth - aref,
 * friction-loss rows boxed to [-floss, floss], limit and (pyramidal) contact rows
 * f >= 0, rows visited in order, each a scalar update f_r -= res_r / AR_rr followed by
 * its projection.  Restated matrix-free: qacc = qacc_smooth + M^-1 J'f is kept current
 * (qacc += delta M^-1 J_r' per changed row), so res_r = J_r qacc - aref_r + R_r f_r and
 * no nefc x nefc matrix is formed -- the same iterates as the AR form.  Warm start: the
 * primal forces at qacc_warmstart, kept only when their dual cost is below that of
 * f = 0 (zero).  Stops after `iterations` sweeps or when a sweep's scaled dual-cost
 * decrease is below `tolerance`.  The oracle for dx_step.hip solve_pgs. */
static void solve_pgs(const dxo_model* m, dxo_data* d) {
  int nv = m->nv, nefc = d->nefc;
  double* Ma = d->tmp1;
  double* g = d->tmp2;
  double* u = d->tmp4;
  double* qacc = d->qacc;
  double* f = d->efc_force;
  double* ard = d->efc_jv;
  const double* a0 = d->qacc_smooth;
  double scale = 1.0 / (m->meaninertia * (nv > 1 ? nv : 1));
  d->niter = 0;
  if (nefc == 0) {
    memcpy(qacc, a0, 8 * nv);
    return;
  }
  /* warm start: primal forces at qacc_warmstart (eval_cost fills efc_force) */
  eval_cost(m, d, d->qacc_warmstart, Ma);
  memset(g, 0, 8 * nv);
  double dc = 0;
  for (int r = 0; r < nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    for (int k = 0; k < nv; k++) g[k] += J[k] * f[r];
    dc += 0.5 * d->efc_R[r] * f[r] * f[r] - f[r] * d->efc_aref[r];
  }
  chol_solve(d->L, u, g, nv, &d->flops[DXO_ST_SOLVE]);
  for (int k = 0; k < nv; k++) dc += 0.5 * g[k] * u[k] + g[k] * a0[k];
  if (dc < 0) {
    for (int k = 0; k < nv; k++) qacc[k] = a0[k] + u[k];
  } else {
    memset(f, 0, 8 * nefc);
    memcpy(qacc, a0, 8 * nv);
  }
  /* diagonal of AR */
  for (int r = 0; r < nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    chol_solve(d->L, u, J, nv, &d->flops[DXO_ST_SOLVE]);
    double s = 0;
    for (int k = 0; k < nv; k++) s += J[k] * u[k];
    ard[r] = s + d->efc_R[r];
  }
  for (int it = 0; it < m->iterations; it++) {
    double impr = 0;
    for (int r = 0; r < nefc; r++) {
      const double* J = d->efc_J + (size_t)r * nv;
      double jq = 0;
      for (int k = 0; k < nv; k++) jq += J[k] * qacc[k];
      double res = jq - d->efc_aref[r] + d->efc_R[r] * f[r];
      double fn = f[r] - res / ard[r];
      if (d->efc_type[r] == EFC_FRIC_DOF) {
        double fl = d->efc_floss[r];
        fn = fn < -fl ? -fl : (fn > fl ? fl : fn);
      } else if (fn < 0) {
        fn = 0;
      }
      double dl = fn - f[r];
      if (dl != 0) {
        chol_solve(d->L, u, J, nv, &d->flops[DXO_ST_SOLVE]);
        for (int k = 0; k < nv; k++) qacc[k] += dl * u[k];
        f[r] = fn;
        impr -= 0.5 * ard[r] * dl * dl + dl * res;
      }
      d->flops[DXO_ST_SOLVE] += 4.0 * nv + 10;
    }
    d->niter++;
    if (scale * impr < m->tolerance) break;
  }
}

static void finish_constraint(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  memset(d->qfrc_constraint, 0, 8 * nv);
  for (int r = 0; r < d->nefc; r++) {
    const double* J = d->efc_J + (size_t)r * nv;
    for (int k = 0; k < nv; k++) d->qfrc_constraint[k] += J[k] * d->efc_force[r];
  }
}

/* ------------------------------------------------------------------------ */
/* mj_rnePostConstraint + torque sensors (mj_sensorAcc) [3P]                 */
/* ------------------------------------------------------------------------ */
/* The reference puts a 3-axis `torque` sensor on a site at the origin of every
 * joint's body (shadow_hand_e.py:176-196, adroit_hand.py:153-172); the sensor reads
 * the internal force of the body on its parent, cfrc_int, at the site, in the site
 * frame.  cfrc_int needs the full acceleration (qacc after the constraint solve) and
 * the external forces: xfrc_applied and the contact forces decoded from the pyramid
 * rows (mju_decodePyramid).  Computed after the solve of every forward pass, before
 * integration (mj_step2 -> mj_sensorAcc); not part of the FLOP counters (the GPU
 * computes it only when the sensor field is enabled). */
static void shift_force(double* res, const double* f, const double* newpos, const double* oldpos) {
  /* mju_transformSpatial, force: torque_new = torque - (newpos - oldpos) x force */
  double dif[3], cr[3];
  sub3(dif, newpos, oldpos);
  cross3(cr, dif, f + 3);
  res[0] = f[0] - cr[0]; res[1] = f[1] - cr[1]; res[2] = f[2] - cr[2];
  res[3] = f[3]; res[4] = f[4]; res[5] = f[5];
}

static void rne_post_constraint(const dxo_model* m, dxo_data* d) {
  int nb = m->nbody;
  memset(d->cfrc_ext, 0, 48 * nb);
  for (int b = 1; b < nb; b++) {
    const double* x = d->xfrc_applied + 6 * b;
    if (x[0] == 0 && x[1] == 0 && x[2] == 0 && x[3] == 0 && x[4] == 0 && x[5] == 0) continue;
    double f[6] = {x[3], x[4], x[5], x[0], x[1], x[2]}, fc[6];
    shift_force(fc, f, d->subtree_com + 3 * m->body_rootid[b], d->xipos + 3 * b);
    for (int e = 0; e < 6; e++) d->cfrc_ext[6 * b + e] += fc[e];
  }
  for (int r = 0; r < d->nefc;) {
    int type = d->efc_type[r];
    if (type != EFC_CON_PYR && type != EFC_CON_FL) { r++; continue; }
    const OContact* con = d->contact + d->efc_id[r];
    double lf[3] = {0, 0, 0};
    if (type == EFC_CON_FL) {
      lf[0] = d->efc_force[r];
      r += 1;
    } else {
      for (int e = 0; e < 4; e++) lf[0] += d->efc_force[r + e];
      lf[1] = (d->efc_force[r] - d->efc_force[r + 1]) * con->friction[0];
      lf[2] = (d->efc_force[r + 2] - d->efc_force[r + 3]) * con->friction[1];
      r += 4;
    }
    /* world force = frame^T lf (frame rows: normal, tangent1, tangent2) */
    double f[6] = {0, 0, 0, 0, 0, 0}, fc[6];
    for (int k = 0; k < 3; k++) f[3 + k] = con->frame[k] * lf[0] + con->frame[3 + k] * lf[1] + con->frame[6 + k] * lf[2];
    int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
    if (b1) {
      shift_force(fc, f, d->subtree_com + 3 * m->body_rootid[b1], con->pos);
      for (int e = 0; e < 6; e++) d->cfrc_ext[6 * b1 + e] -= fc[e];
    }
    if (b2) {
      shift_force(fc, f, d->subtree_com + 3 * m->body_rootid[b2], con->pos);
      for (int e = 0; e < 6; e++) d->cfrc_ext[6 * b2 + e] += fc[e];
    }
  }
  double* ca = d->cacc_post;
  memset(ca, 0, 48);
  ca[3] = -m->gravity[0]; ca[4] = -m->gravity[1]; ca[5] = -m->gravity[2];
  memset(d->cfrc_int, 0, 48);
  for (int b = 1; b < nb; b++) {
    double* a = ca + 6 * b;
    memcpy(a, ca + 6 * m->body_parent[b], 48);
    for (int j = m->body_dofadr[b]; j >= 0 && j < m->body_dofadr[b] + m->body_dofnum[b]; j++)
      for (int e = 0; e < 6; e++) a[e] += d->cdof_dot[6 * j + e] * d->qvel[j] + d->cdof[6 * j + e] * d->qacc[j];
    double t1[6], t2[6], t3[6];
    mul_inert(t1, d->cinert + 10 * b, a);
    mul_inert(t2, d->cinert + 10 * b, d->cvel + 6 * b);
    cross_force(t3, d->cvel + 6 * b, t2);
    for (int e = 0; e < 6; e++) d->cfrc_int[6 * b + e] = t1[e] + t3[e] - d->cfrc_ext[6 * b + e];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m->body_parent[b];
    if (p > 0)
      for (int e = 0; e < 6; e++) d->cfrc_int[6 * p + e] += d->cfrc_int[6 * b + e];
  }
  /* torque sensor on a site at body b's origin (site frame = body frame) */
  memset(d->sensor_torque, 0, 24);
  for (int b = 1; b < nb; b++) {
    double t[6];
    shift_force(t, d->cfrc_int + 6 * b, d->xpos + 3 * b, d->subtree_com + 3 * m->body_rootid[b]);
    mattvec3(d->sensor_torque + 3 * b, d->xmat + 9 * b, t);
  }
}

/* mj_objectVelocity (utils/mujoco_utils.py:27-34), world orientation: the com-based
 * cvel of the object's body moved to the object position; res = [lin(3), ang(3)]
 * (the order get_site_velocity returns).  objtype 0: body inertial frame (xipos,
 * what frame*vel sensors of objtype "body" read), 1: site, 2: body frame (xpos). */
void dxo_object_velocity(const dxo_model* m, const dxo_data* d, int objtype, int id, double res[6]) {
  int b = objtype == 1 ? m->site_bodyid[id] : id;
  const double* pos = objtype == 1 ? d->site_xpos + 3 * id : objtype == 0 ? d->xipos + 3 * b : d->xpos + 3 * b;
  const double* cv = d->cvel + 6 * b;
  double off[3], w[3];
  sub3(off, pos, d->subtree_com + 3 * m->body_rootid[b]);
  cross3(w, cv, off);
  res[0] = cv[3] + w[0]; res[1] = cv[4] + w[1]; res[2] = cv[5] + w[2];
  res[3] = cv[0]; res[4] = cv[1]; res[5] = cv[2];
}

/* ------------------------------------------------------------------------ */
/* Euler with implicit joint damping                                         */
/* ------------------------------------------------------------------------ */
static void euler(const dxo_model* m, dxo_data* d) {
  int nv = m->nv;
  double h = m->timestep;
  memcpy(d->qacc_warmstart, d->qacc, 8 * nv);
  double* qacc = d->tmp1;
  if (m->any_damping) {
    double* rhs = d->tmp2;
    memcpy(d->H, d->M, 8 * nv * nv);
    for (int i = 0; i < nv; i++) d->H[i * nv + i] += h * m->dof_damping[i];
    for (int i = 0; i < nv; i++) rhs[i] = d->qfrc_smooth[i] + d->qfrc_constraint[i];
    cholesky(d->H, d->H, nv, &d->flops[DXO_ST_INT]);
    chol_solve(d->H, qacc, rhs, nv, &d->flops[DXO_ST_INT]);
  } else {
    memcpy(qacc, d->qacc, 8 * nv);
  }
  for (int i = 0; i < nv; i++) d->qvel[i] += h * qacc[i];
  /* integrate positions with the new velocity */
  for (int j = 0; j < m->njnt; j++) {
    int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (m->jnt_type[j] == JNT_FREE) {
      for (int k = 0; k < 3; k++) d->qpos[qa + k] += h * d->qvel[da + k];
      double* q = d->qpos + qa + 3;
      const double* w = d->qvel + da + 3;
      double wn = norm3(w);
      if (wn > MINVAL) {
        double ang = h * wn;
        double s = sin(0.5 * ang);
        double dq[4] = {cos(0.5 * ang), w[0] / wn * s, w[1] / wn * s, w[2] / wn * s};
        quatmul(q, q, dq);
      }
      quatnorm(q);
    } else {
      d->qpos[qa] += h * d->qvel[da];
    }
  }
  d->time += h;
  d->flops[DXO_ST_INT] += 4.0 * nv + 60;
}

/* ------------------------------------------------------------------------ */
/* public entry points                                                       */
/* ------------------------------------------------------------------------ */
static void position_stage(const dxo_model* m, dxo_data* d) {
  kinematics(m, d);
  com_pos(m, d);
  tendon_transmission(m, d);
  crb(m, d);
  collision(m, d);
  make_constraint(m, d);
}

int dxo_forward(const dxo_model* m, dxo_data* d) {
  position_stage(m, d);
  com_vel(m, d);
  rne(m, d);
  smooth_forces(m, d);
  /* constraint velocities were computed in make_constraint with current qvel */
  if (m->solver == 1)
    solve_cg(m, d);
  else if (m->solver == 0)
    solve_pgs(m, d);
  else
    solve_newton(m, d);
  finish_constraint(m, d);
  rne_post_constraint(m, d);
  return 0;
}

/* Observation-time pass at the current state (no forces): kinematics, com, site
 * poses and cvel -- what the observables read after dm_control's step1. */
int dxo_observe(const dxo_model* m, dxo_data* d) {
  kinematics(m, d);
  com_pos(m, d);
  com_vel(m, d);
  return 0;
}

int dxo_step(const dxo_model* m, dxo_data* d) {
  dxo_forward(m, d);
  euler(m, d);
  for (int i = 0; i < m->nq; i++)
    if (!isfinite(d->qpos[i])) return -1;
  return 0;
}

int dxo_kinematics(const dxo_model* m, dxo_data* d) {
  kinematics(m, d);
  com_pos(m, d);
  collision(m, d);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* kinematic queries and IK (inverse_kinematics/ik_solver.py, controllers/dls)  */
/* ------------------------------------------------------------------------ */
int dxo_fk(const dxo_model* m, dxo_data* d) {
  kinematics(m, d);
  com_pos(m, d);
  return 0;
}

/* mj_jacSite (utils/mujoco_utils.py:67-73): [3][nv] each, after dxo_fk */
void dxo_jac_site(const dxo_model* m, const dxo_data* d, int site, double* jacp, double* jacr) {
  jac_point(m, d, m->site_bodyid[site], d->site_xpos + 3 * site, jacp, jacr);
}

/* One IKSolver._solve_ik attempt (ik_solver.py:169-236) from d->qpos: DLS joint
 * velocities (dls.py:43-77, (J^T J + reg I) qdot = J^T twist, solved densely as the
 * reference does), mj_integratePos over 1 s, clip of the solved joints to their
 * range, mj_normalizeQuat, mj_kinematics + mj_comPos (ik_solver.py:238-250).
 * opts = {linear_tol, regularization, gain, progress_threshold}.  Returns the steps
 * taken; err_out[nsite] = the last step's linear errors. */
int dxo_ik_attempt(const dxo_model* m, dxo_data* d, int nsite, const int* sites, int njoint, const int* joints,
                   const double* targets, const double* opts, int max_steps, int early_stop, double* err_out) {
  const int nv = m->nv, nr = 3 * nsite;
  double* J = (double*)calloc((size_t)nr * nv, 8);
  double* H = (double*)calloc((size_t)nv * nv, 8);
  double* jp = (double*)calloc(3 * (size_t)nv, 8);
  double* rhs = (double*)calloc(nv, 8);
  double* qd = (double*)calloc(nv, 8);
  double* prev = (double*)calloc(nr, 8);
  double* tw = (double*)calloc(nr, 8);
  double fl = 0;
  dxo_fk(m, d);
  for (int s = 0; s < nsite; s++) memcpy(prev + 3 * s, d->site_xpos + 3 * sites[s], 24);
  int it = 0;
  while (it < max_steps) {
    for (int s = 0; s < nsite; s++)
      for (int e = 0; e < 3; e++) tw[3 * s + e] = opts[2] * (targets[3 * s + e] - d->site_xpos[3 * sites[s] + e]) / 1.0;
    for (int s = 0; s < nsite; s++) {
      dxo_jac_site(m, d, sites[s], jp, NULL);
      memcpy(J + (size_t)3 * s * nv, jp, 24 * (size_t)nv);
    }
    for (int i = 0; i < nv; i++) {
      for (int j = 0; j < nv; j++) {
        double v = 0;
        for (int r = 0; r < nr; r++) v += J[r * nv + i] * J[r * nv + j];
        H[i * nv + j] = v + (i == j ? opts[1] : 0.0);
      }
      double v = 0;
      for (int r = 0; r < nr; r++) v += J[r * nv + i] * tw[r];
      rhs[i] = v;
    }
    cholesky(H, H, nv, &fl);
    chol_solve(H, qd, rhs, nv, &fl);
    /* mj_integratePos(qpos, qd, 1) */
    for (int j = 0; j < m->njnt; j++) {
      int qa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
      if (m->jnt_type[j] == JNT_FREE) {
        for (int k = 0; k < 3; k++) d->qpos[qa + k] += qd[da + k];
        double* q = d->qpos + qa + 3;
        const double* w = qd + da + 3;
        double wn = norm3(w);
        if (wn > MINVAL) {
          double sn = sin(0.5 * wn);
          double dq[4] = {cos(0.5 * wn), w[0] / wn * sn, w[1] / wn * sn, w[2] / wn * sn};
          quatmul(q, q, dq);
        }
        quatnorm(q);
      } else {
        d->qpos[qa] += qd[da];
      }
    }
    for (int k = 0; k < njoint; k++) {
      int j = joints[k], qa = m->jnt_qposadr[j];
      double lo = m->jnt_range[2 * j], hi = m->jnt_range[2 * j + 1];
      d->qpos[qa] = d->qpos[qa] < lo ? lo : d->qpos[qa] > hi ? hi : d->qpos[qa];
    }
    dxo_fk(m, d);
    it++;
    int close = 1, stuck = 0;
    for (int s = 0; s < nsite; s++) {
      const double* p = d->site_xpos + 3 * sites[s];
      double e[3], c[3];
      sub3(e, targets + 3 * s, p);
      sub3(c, p, prev + 3 * s);
      double err = norm3(e), chg = norm3(c);
      err_out[s] = err;
      if (err > opts[0]) close = 0;
      if (err / (chg + 1e-10) > opts[3]) stuck = 1;
      memcpy(prev + 3 * s, p, 24);
    }
    if ((early_stop && close) || stuck) break;
  }
  free(J); free(H); free(jp); free(rhs); free(qd); free(prev); free(tw);
  return it;
}

double* dxo_field(dxo_data* d, const char* name, int* len) {
  const dxo_model* m = d->model;
  int nv = m->nv, nb = m->nbody;
#define F(nm, ptr, n) \
  if (strcmp(name, nm) == 0) { if (len) *len = (n); return (ptr); }
  F("time", &d->time, 1);
  F("qpos", d->qpos, m->nq);
  F("qvel", d->qvel, nv);
  F("ctrl", d->ctrl, m->nu);
  F("qacc", d->qacc, nv);
  F("qacc_warmstart", d->qacc_warmstart, nv);
  F("qacc_smooth", d->qacc_smooth, nv);
  F("qfrc_bias", d->qfrc_bias, nv);
  F("qfrc_passive", d->qfrc_passive, nv);
  F("qfrc_actuator", d->qfrc_actuator, nv);
  F("qfrc_applied", d->qfrc_applied, nv);
  F("qfrc_smooth", d->qfrc_smooth, nv);
  F("qfrc_constraint", d->qfrc_constraint, nv);
  F("xfrc_applied", d->xfrc_applied, 6 * nb);
  F("xpos", d->xpos, 3 * nb);
  F("xquat", d->xquat, 4 * nb);
  F("xmat", d->xmat, 9 * nb);
  F("xipos", d->xipos, 3 * nb);
  F("subtree_com", d->subtree_com, 3 * nb);
  F("cinert", d->cinert, 10 * nb);
  F("cdof", d->cdof, 6 * nv);
  F("cvel", d->cvel, 6 * nb);
  F("cfrc_int", d->cfrc_int, 6 * nb);
  F("cfrc_ext", d->cfrc_ext, 6 * nb);
  F("sensor_torque", d->sensor_torque, 3 * nb);
  F("geom_xpos", d->geom_xpos, 3 * m->ngeom);
  F("geom_xmat", d->geom_xmat, 9 * m->ngeom);
  F("site_xpos", d->site_xpos, 3 * m->nsite);
  F("site_xmat", d->site_xmat, 9 * m->nsite);
  F("M", d->M, nv * nv);
  F("actuator_force", d->actuator_force, m->nu);
  F("actuator_length", d->actuator_length, m->nu);
  F("ten_length", d->ten_length, m->ntendon);
  F("efc_force", d->efc_force, d->nefc);
  F("efc_aref", d->efc_aref, d->nefc);
  F("efc_R", d->efc_R, d->nefc);
  F("efc_pos", d->efc_pos, d->nefc);
  F("efc_J", d->efc_J, d->nefc * nv);
#undef F
  if (len) *len = 0;
  return NULL;
}

/* Test helper: the solver's scaled primal cost scale * f(qacc) (the quantity whose
 * improvement solve_newton compares with the tolerance) of the constraint problem the
 * last dxo_forward built, at an arbitrary qacc -- how optimal another solver's
 * acceleration is in this problem.  Overwrites efc_force / efc_state / efc_jar. */
double dxo_solver_cost(const dxo_model* m, dxo_data* d, const double* qacc) {
  const double scale = 1.0 / (m->meaninertia * (m->nv > 1 ? m->nv : 1));
  return scale * eval_cost(m, d, qacc, d->tmp1);
}

/* Test helper: every later collision pass of d yields these n contacts (records in
 * dxo_contact's layout: pos, frame -- only its normal row is read -- dist, geom1, geom2,
 * condim) instead of running the narrowphase; n < 0 restores the narrowphase.  Lets a
 * test run the oracle's dynamics on another implementation's contact list. */
int dxo_set_contacts(dxo_data* d, int n, const double* recs) {
  if (n > NCON_MAX) return -1;
  d->ncon_fixed = n;
  if (n > 0) memcpy(d->con_fixed, recs, sizeof(double) * 16 * (size_t)n);
  return 0;
}

int dxo_ncon(const dxo_data* d) { return d->ncon; }
void dxo_contact(const dxo_data* d, int i, double out[16]) {
  const OContact* c = d->contact + i;
  memcpy(out, c->pos, 24);
  memcpy(out + 3, c->frame, 72);
  out[12] = c->dist;
  out[13] = c->geom1;
  out[14] = c->geom2;
  out[15] = c->condim;
}
int dxo_nefc(const dxo_data* d) { return d->nefc; }
int dxo_solver_niter(const dxo_data* d) { return d->niter; }
void dxo_flops(const dxo_data* d, double out[DXO_NSTAGE]) { memcpy(out, d->flops, sizeof(d->flops)); }
void dxo_flops_reset(dxo_data* d) { memset(d->flops, 0, sizeof(d->flops)); }

int dxo_batch_step(const dxo_model* m, int nenv, int nsub, double* qpos, double* qvel,
                   const double* ctrl, double* qacc_warmstart, const double* xfrc, int nthreads) {
  return dxo_batch_step_counted(m, nenv, nsub, qpos, qvel, ctrl, qacc_warmstart, xfrc, nthreads, NULL);
}

int dxo_batch_step_counted(const dxo_model* m, int nenv, int nsub, double* qpos, double* qvel,
                           const double* ctrl, double* qacc_warmstart, const double* xfrc, int nthreads,
                           double* flops) {
  return dxo_batch_step_watch(m, nenv, nsub, qpos, qvel, ctrl, qacc_warmstart, xfrc, nthreads, flops, -1, -1, NULL);
}

/* any contact at the current collision pass between geom wg and a geom of body wb with
   dist <= 1e-8: mujoco_collisions.has_collision (utils/mujoco_collisions.py:95-119) as
   ReOrient._is_prop_fallen calls it (reorient.py:229-235) */
static int watch_contact(const dxo_model* m, const dxo_data* d, int wg, int wb) {
  for (int i = 0; i < d->ncon; i++) {
    const OContact* c = d->contact + i;
    const int other = c->geom1 == wg ? c->geom2 : (c->geom2 == wg ? c->geom1 : -1);
    if (other >= 0 && m->geom_bodyid[other] == wb && c->dist <= 1e-8) return 1;
  }
  return 0;
}

int dxo_batch_step_watch(const dxo_model* m, int nenv, int nsub, double* qpos, double* qvel,
                         const double* ctrl, double* qacc_warmstart, const double* xfrc, int nthreads,
                         double* flops, int watch_geom, int watch_body, int* watch) {
  int err = 0;
  double fs[DXO_NSTAGE] = {0};
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel reduction(| : err) reduction(+ : fs[:DXO_NSTAGE])
#endif
  {
    dxo_data* d = dxo_data_create(m);
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int e = 0; e < nenv; e++) {
      memcpy(d->qpos, qpos + (size_t)e * m->nq, 8 * m->nq);
      memcpy(d->qvel, qvel + (size_t)e * m->nv, 8 * m->nv);
      memcpy(d->ctrl, ctrl + (size_t)e * m->nu, 8 * m->nu);
      memcpy(d->qacc_warmstart, qacc_warmstart + (size_t)e * m->nv, 8 * m->nv);
      if (xfrc) memcpy(d->xfrc_applied, xfrc, 48 * m->nbody);
      for (int s = 0; s < nsub; s++) err |= dxo_step(m, d) != 0;
      if (watch) {  /* the new state's contacts (dm_control's step ends with mj_step1) */
        dxo_kinematics(m, d);
        watch[e] = watch_contact(m, d, watch_geom, watch_body);
      }
      memcpy(qpos + (size_t)e * m->nq, d->qpos, 8 * m->nq);
      memcpy(qvel + (size_t)e * m->nv, d->qvel, 8 * m->nv);
      memcpy(qacc_warmstart + (size_t)e * m->nv, d->qacc_warmstart, 8 * m->nv);
    }
    for (int k = 0; k < DXO_NSTAGE; k++) fs[k] += d->flops[k];
    dxo_data_free(d);
  }
  if (flops) memcpy(flops, fs, sizeof(fs));
  return err ? -1 : 0;
}
