/*
 * dx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * fp64, single-environment, scalar C restatement of the MuJoCo `mj_step`
 * pipeline as configured by the dexterity scenes.  It is the parity oracle for
 * the HIP kernels in dexterity_amd/csrc and the `cpu_baseline` leg of bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it;
 * nothing on the product path links or calls it.
 *
 * PARITY STATUS vs the reference: the reference path is MuJoCo's C library
 * ([3P], absent from /root/reference and not installable here).  This file
 * restates MuJoCo's published pipeline from the model data the
 * reference configures; it is pinned only by the reference's own known-answer
 * tests restated under tests/ (reorient_test.py:13-50 reward KAT,
 * hands_test.py:26-31 projections, physical invariants).  Dynamics parity against
 * real MuJoCo is UNPINNED.
 */
#ifndef DX_ORACLE_H
#define DX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dxo_model dxo_model;
typedef struct dxo_data dxo_data;

/* Stage FLOP counters (flops counted as mul/add/div/sqrt = 1). */
enum {
  DXO_ST_KIN = 0,   /* kinematics + com + cdof                        */
  DXO_ST_CRB,       /* tendon, transmission, CRB, factorization       */
  DXO_ST_COL,       /* broadphase + narrowphase                       */
  DXO_ST_CON,       /* constraint assembly (J, R, aref)               */
  DXO_ST_SMOOTH,    /* comVel, passive, RNE, actuation, qacc_smooth   */
  DXO_ST_SOLVE,     /* Newton solver                                  */
  DXO_ST_INT,       /* implicit-damping Euler                         */
  DXO_ST_SCAN,      /* mesh supports: the full hull scan's vertices beyond the 16 an
                       efficient support reads (a direction-binned cell block, as the
                       kernel does, or a hill climb) -- reported apart, not part of the
                       algorithmic count                                  */
  DXO_NSTAGE
};

dxo_model* dxo_model_load(const void* blob, size_t nbytes);
void dxo_model_free(dxo_model* m);
dxo_data* dxo_data_create(const dxo_model* m);
void dxo_data_free(dxo_data* d);
void dxo_reset(const dxo_model* m, dxo_data* d);

/* mj_forward: everything up to and including the constraint solve. */
int dxo_forward(const dxo_model* m, dxo_data* d);
/* mj_step with the Euler integrator: forward + implicit-damping Euler. */
int dxo_step(const dxo_model* m, dxo_data* d);
/* Position-only pass (kinematics + collision), as used for observations. */
int dxo_kinematics(const dxo_model* m, dxo_data* d);

/* Observation pass: mj_kinematics + mj_comPos + mj_comVel at the current state. */
int dxo_observe(const dxo_model* m, dxo_data* d);
/* mj_objectVelocity, world orientation, res = [lin(3), ang(3)] at the object:
 * objtype 0 body inertial frame (xipos), 1 site, 2 body frame (xpos). */
void dxo_object_velocity(const dxo_model* m, const dxo_data* d, int objtype, int id, double res[6]);

/* mj_kinematics + mj_comPos (no collision). */
int dxo_fk(const dxo_model* m, dxo_data* d);
/* mj_jacSite after dxo_fk: jacp / jacr [3][nv] (either may be NULL). */
void dxo_jac_site(const dxo_model* m, const dxo_data* d, int site, double* jacp, double* jacr);
/* One IKSolver._solve_ik attempt from d->qpos (ik_solver.py:169-250, dls.py:43-77).
 * opts = {linear_tol, regularization, gain, progress_threshold}; returns the steps
 * taken, err_out[nsite] = last linear errors; d->qpos holds the result. */
int dxo_ik_attempt(const dxo_model* m, dxo_data* d, int nsite, const int* sites, int njoint, const int* joints,
                   const double* targets, const double* opts, int max_steps, int early_stop, double* err_out);

/* Field access: returns a pointer to the named double array and its length.
 * Names: qpos qvel ctrl qacc qacc_warmstart qacc_smooth qfrc_bias qfrc_passive
 * qfrc_actuator qfrc_applied qfrc_smooth qfrc_constraint xfrc_applied xpos xquat
 * xmat xipos site_xpos M actuator_force actuator_length ten_length cvel
 * efc_force efc_aref efc_R efc_pos efc_J time cfrc_int cfrc_ext sensor_torque
 * (sensor_torque [nbody][3]: the `torque` sensor of a site at each body's origin,
 * site frame, from the last forward pass: mj_rnePostConstraint + mj_sensorAcc).  */
double* dxo_field(dxo_data* d, const char* name, int* len);

int dxo_ncon(const dxo_data* d);
/* contact i: out[0:3]=pos, [3:12]=frame, [12]=dist, [13]=geom1, [14]=geom2, [15]=condim */
void dxo_contact(const dxo_data* d, int i, double out[16]);
int dxo_nefc(const dxo_data* d);
int dxo_solver_niter(const dxo_data* d);
double dxo_solver_cost(const dxo_model* m, dxo_data* d, const double* qacc);
int dxo_set_contacts(dxo_data* d, int n, const double* recs);
void dxo_flops(const dxo_data* d, double out[DXO_NSTAGE]);
void dxo_flops_reset(dxo_data* d);

/* Batched CPU stepping for the baseline timing: nenv independent envs,
 * OpenMP over envs when built with -fopenmp. state arrays are [nenv, n]. */
int dxo_batch_step(const dxo_model* m, int nenv, int nsub, double* qpos, double* qvel,
                   const double* ctrl, double* qacc_warmstart, const double* xfrc,
                   int nthreads);
/* Same, also returning the FLOP counters summed over all envs and substeps, per stage
   (flops: double[DXO_NSTAGE]). */
int dxo_batch_step_counted(const dxo_model* m, int nenv, int nsub, double* qpos, double* qvel,
                           const double* ctrl, double* qacc_warmstart, const double* xfrc,
                           int nthreads, double* flops);
/* Same, and (watch != NULL) watch[e] = 1 when env e's state after the steps has a contact
   between geom watch_geom and a geom of body watch_body with dist <= 1e-8 (the fall test
   of reorient.py:229-235). */
int dxo_batch_step_watch(const dxo_model* m, int nenv, int nsub, double* qpos, double* qvel,
                         const double* ctrl, double* qacc_warmstart, const double* xfrc, int nthreads,
                         double* flops, int watch_geom, int watch_body, int* watch);

#ifdef __cplusplus
}
#endif
#endif
