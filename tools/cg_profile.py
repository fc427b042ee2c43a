"""CG (<option solver="CG">, [3P] MuJoCo's mj_solCG at its defaults: 100 iterations, tol 1e-8)
on config 3 (reorient, 4096 envs): per-stage cycles of the step kernel, and the solver's
iteration counts per env beside the fp64 oracle's CG -- and both solvers' Newton -- on the
same states (diagnostics for VERDICT r3 item 5: is CG's cost its iteration count, or the
kernel's cost per iteration?).

usage: python tools/cg_profile.py [nenv] [oracle_sample] [CG|PGS]   -> gpurun_out/<solver>_profile.json
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import _lib, manipulation, physics  # noqa: E402
from oracle import oracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NS = int(sys.argv[2]) if len(sys.argv) > 2 else 512
SOLVER = sys.argv[3] if len(sys.argv) > 3 else "CG"
L = _lib.load()
out = {}


def stage_profile(solver, steps=5):
    t = manipulation.ReOrient()
    if solver:
        t.compiled = t.compiled.with_solver(solver)
    env = manipulation.GoalEnvironment(t, num_envs=B, seed=7)
    env.reset()
    for i in range(10):
        env.step_random(i)
    env.physics.sync()
    _lib.check(L.dx_stage_timing(env.physics.ptr, 1))
    buf = (ctypes.c_uint64 * (_lib.NSTAGE * B))()
    _lib.check(L.dx_stage_read(env.physics.ptr, buf, _lib.NSTAGE * B))
    t0 = time.perf_counter()
    for i in range(steps):
        env.step_random(10 + i)
    env.physics.sync()
    dt = (time.perf_counter() - t0) / steps
    _lib.check(L.dx_stage_read(env.physics.ptr, buf, _lib.NSTAGE * B))
    _lib.check(L.dx_stage_timing(env.physics.ptr, 0))
    per_env = np.frombuffer(buf, dtype=np.uint64).reshape(B, _lib.NSTAGE).astype(np.float64)
    n = B * steps * 5
    cyc = per_env.sum(axis=0)
    cnt = {name: cyc[k] / n for k, name in _lib.COUNTERS.items()}
    cyc[list(_lib.COUNTERS)] = 0
    stages = {name: cyc[k] / n for k, name in enumerate(_lib.STAGES)}
    solver_cyc = sum(stages[s] for s in ("newton_eval", "newton_grad", "newton_hessian", "newton_chol",
                                         "newton_linesearch", "matvec", "jacvec"))
    # the state mix the solvers are compared on
    ph = env.physics
    cost = ph.get(_lib.STEP_COST)[:, 0].astype(np.float64) * 1024
    ncon = ph.get(_lib.NCON)[:, 0]
    top = np.argsort(-cost)[:12]
    log.append(f"[{solver or 'Newton'} last step] per-env cycles p50 {np.median(cost):.3e} p99 {np.percentile(cost, 99):.3e} "
               f"max {cost.max():.3e}; heaviest envs (cycles, ncon, niter): "
               + ", ".join(f"({cost[e]:.2e}, {ncon[e]}, {ph.get(_lib.NITER)[e, 0]})" for e in top))
    st = (ph.qpos, ph.qvel, ph.get(_lib.QACC_WARMSTART), ph.get(_lib.CTRL))
    xfrc = t.gravity_compensation
    env.close()
    return dict(ms_per_step=dt * 1e3, cycles_per_env_substep=sum(stages.values()), stages=stages, counters=cnt,
                solver_cycles_per_env_substep=solver_cyc,
                solver_cycles_per_iteration=solver_cyc / max(cnt["newton_iter"], 1e-9)), st, xfrc, t.compiled


log = []
for solver in (SOLVER, None):
    prof, st, xfrc, cm = stage_profile(solver)
    out["profile_" + (solver or "Newton")] = prof
    log.append(f"[{solver or 'Newton'}] {prof['ms_per_step']:.3f} ms/step, "
               f"{prof['cycles_per_env_substep']:.0f} cyc/env-substep, solver "
               f"{prof['solver_cycles_per_env_substep']:.0f} cyc/env-substep = "
               f"{prof['counters']['newton_iter']:.2f} iterations x {prof['solver_cycles_per_iteration']:.0f} cyc, "
               f"line-search iterations {prof['counters']['linesearch_iter']:.2f}, nefc {prof['counters']['nefc']:.1f}")
    log.append("   stages: " + ", ".join(f"{k} {v:.0f}" for k, v in sorted(prof["stages"].items(), key=lambda x: -x[1])[:10]))
    if solver == SOLVER:
        states, xfrc_cg, cm_cg = st, xfrc, cm

# iteration counts on the same states (the CG env's state mix): one forward (= one solve)
qpos, qvel, ws, ctrl = states
cm_newton = manipulation.ReOrient().compiled
res = {}
for name, cm in ((SOLVER, cm_cg), ("Newton", cm_newton)):
    model = physics.Model(cm)
    ph = physics.BatchedPhysics(model, B)
    ph.set_xfrc(xfrc_cg)
    for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws), (_lib.CTRL, ctrl)):
        ph.set(f, v)
    ph.debug(True)
    ph.forward()
    nefc = ph.debug_get("efc_count")[:, 0]
    log.append(f"[{name} state mix] nefc mean {nefc.mean():.1f} p50 {np.median(nefc):.0f} p99 "
               f"{np.percentile(nefc, 99):.0f} max {nefc.max()}; > 64 rows: {(nefc > 64).mean():.4f} of the envs")
    gpu_it = ph.get(_lib.NITER)[:, 0].copy()
    gpu_qacc = ph.qacc
    ph.close()
    om = O.OracleModel(model.blob)
    idx = np.linspace(0, B - 1, NS).astype(int)
    ora_it, dq = [], []
    for e in idx:
        d = O.OracleData(om)
        d.xfrc_applied[:] = np.asarray(xfrc_cg, dtype=np.float32).astype(np.float64).ravel()
        d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = qpos[e], qvel[e], ws[e], ctrl[e]
        d.forward()
        ora_it.append(d.niter)
        dq.append(np.abs(gpu_qacc[e] - d.qacc).max() / max(1.0, np.abs(d.qacc_smooth).max()))
    ora_it = np.array(ora_it)
    res[name] = dict(gpu_mean=float(gpu_it.mean()), gpu_p50=float(np.median(gpu_it)), gpu_p99=float(np.percentile(gpu_it, 99)),
                     gpu_max=int(gpu_it.max()), gpu_hist=np.bincount(gpu_it, minlength=1).tolist(),
                     gpu_sample_mean=float(gpu_it[idx].mean()), oracle_sample_mean=float(ora_it.mean()),
                     oracle_p50=float(np.median(ora_it)), oracle_p99=float(np.percentile(ora_it, 99)),
                     oracle_max=int(ora_it.max()), oracle_hist=np.bincount(ora_it, minlength=1).tolist(),
                     per_env_ratio_mean=float((gpu_it[idx] / np.maximum(ora_it, 1)).mean()),
                     qacc_err_of_scale_p50=float(np.median(dq)), qacc_err_of_scale_max=float(np.max(dq)))
    log.append(f"[{name} iterations, one solve per env] GPU mean {gpu_it.mean():.2f} (p50 {np.median(gpu_it):.0f}, "
               f"p99 {np.percentile(gpu_it, 99):.0f}, max {gpu_it.max()}); oracle fp64 on {NS} of the states: mean "
               f"{ora_it.mean():.2f} (p50 {np.median(ora_it):.0f}, p99 {np.percentile(ora_it, 99):.0f}, max "
               f"{ora_it.max()}) vs GPU on the same {gpu_it[idx].mean():.2f}; qacc err / scale p50 {np.median(dq):.1e}")
out["iterations"] = res
print("\n".join(log), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"{SOLVER.lower()}_profile.json"), "w"), indent=1)
