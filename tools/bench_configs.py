#!/usr/bin/env python3
"""Throughput of every GPU configuration of BASELINE.json on one MI355X (diagnostics).

bench.py measures the headline (config 3); this script adds the other single-GPU
configs, one JSON line each:
  config 2  reach_shadow.state_dense (contacts disabled), 1024 envs; also Adroit reach
  config 3  reorient.state_dense, 4096 envs (same workload as bench.py)
  config 5  bimanual handover physics (two Shadow hands + cube, nv 54), 4096 envs,
            random actions held for 5 physics substeps per control step
Timed regions hold inputs in HBM (device-side actions), as in bench.py.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _kernel_ms(L, ptr):
    kt, kn = ctypes.c_double(), ctypes.c_int32()
    L.dx_timing_read(ptr, ctypes.byref(kt), ctypes.byref(kn))
    return kt.value / max(1, kn.value), kn.value


def env_config(name, domain, task, nenv, steps=50, warmup=10, solver=None):
    from dexterity_amd import _lib, manipulation

    L = _lib.load()
    if solver is None:
        env = manipulation.load(domain, task, seed=7, num_envs=nenv)
    else:  # the same task on the model compiled with <option solver=...> (MuJoCo's defaults otherwise)
        t = manipulation.SUITE[(domain, task)]()
        t.compiled = t.compiled.with_solver(solver)
        env = manipulation.GoalEnvironment(t, num_envs=nenv, seed=7)
    env.reset()
    for i in range(warmup):
        env.step_random(i)
    env.physics.sync()
    L.dx_timing_enable(env.physics.ptr, 1)
    _kernel_ms(L, env.physics.ptr)
    env.physics.health_clear()
    t = time.perf_counter()
    for i in range(steps):
        env.step_random(warmup + i)
    env.physics.sync()
    dt = time.perf_counter() - t
    kms, kn = _kernel_ms(L, env.physics.ptr)
    h = env.physics.health()  # the deferral tiers over the timed region (include/dx.h dx_health)
    env.close()
    return {"config": name, "envs": nenv, "solver": solver or "Newton", "env_steps_per_s": round(nenv * steps / dt, 1),
            "ms_per_step": round(dt / steps * 1e3, 4), "step_kernel_ms_avg": round(kms, 4),
            "step_kernel_launches_per_step": kn / steps,
            "deferred": {k: h[k] for k in ("contact_deferred", "mid_tier_gave_up", "deferred_behind_launch")}}


def bimanual(nenv=4096, steps=30, warmup=5, nsub=5):
    """Config 5 as raw physics (no task): random ctrl held for 5 substeps, uploaded once
    into a hipMalloc'd device buffer (libdx's HIP runtime, no PyTorch)."""
    from dexterity_amd import _lib, physics
    from dexterity_amd.manipulation import _copy_h2d, _hip_runtime
    from dexterity_amd.mjcf.compiler import CompiledModel

    L = _lib.load()
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "bimanual_handover.npz"))
    model = physics.Model(cm)
    phys = physics.BatchedPhysics(model, nenv)
    phys.set_xfrc(physics.gravity_compensation(cm, "shadow_hand_"))
    q0 = np.tile(cm.qpos0, (nenv, 1))
    q0[:, 48:51] += np.random.RandomState(0).uniform(-0.02, 0.02, size=(nenv, 3)) * [1, 1, 0]
    phys.set(_lib.QPOS, q0)
    lo, hi = cm.actuator_ctrlrange.T
    acts = np.random.RandomState(1).uniform(lo, hi, size=(warmup + steps, nenv, cm.nu)).astype(np.float32)
    dev = ctypes.c_void_p()
    assert _hip_runtime().hipMalloc(ctypes.byref(dev), acts.nbytes) == 0
    _copy_h2d(dev.value, acts)
    row = nenv * cm.nu * 4

    def one(i):
        phys.set_device(_lib.CTRL, dev.value + i * row, 0, nenv)
        phys.step(nsub)

    for i in range(warmup):
        one(i)
    phys.sync()
    L.dx_timing_enable(phys.ptr, 1)
    _kernel_ms(L, phys.ptr)
    t = time.perf_counter()
    for i in range(steps):
        one(warmup + i)
    phys.sync()
    dt = time.perf_counter() - t
    kms, _ = _kernel_ms(L, phys.ptr)
    ncon = phys.get(_lib.NCON)[:, 0]
    ok = bool(np.isfinite(phys.qpos).all())
    phys.close()
    _hip_runtime().hipFree(dev)
    return {"config": "5p bimanual handover physics only (nv 54)", "envs": nenv,
            "env_steps_per_s": round(nenv * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 4),
            "step_kernel_ms_avg": round(kms, 4), "substeps": nsub, "mean_ncon": float(ncon.mean()),
            "finite": ok}


def main():
    """Every config, or (arguments) only those whose key is given: 1 1' 2 2' 3 3' 3'' 5 5p."""
    from bench import cpu_baseline_reach_1env

    runs = {
        "1": lambda: {"config": "1 reach (Shadow hand, contacts disabled), 1 env, CPU",
                      **cpu_baseline_reach_1env(4.0, "shadow")},
        "1'": lambda: {"config": "1' reach (Adroit hand), 1 env, CPU", **cpu_baseline_reach_1env(4.0, "adroit")},
        "2": lambda: env_config("2 reach_shadow.state_dense (no contacts)", "reach_shadow", "state_dense", 1024,
                                steps=400, warmup=40),
        "2'": lambda: env_config("2' reach.state_dense (Adroit)", "reach", "state_dense", 1024, steps=200),
        "3": lambda: env_config("3 reorient.state_dense", "reorient", "state_dense", 4096),
        "3'": lambda: env_config("3' reorient.state_dense, CG solver at MuJoCo's defaults", "reorient",
                                 "state_dense", 4096, solver="CG"),
        "3''": lambda: env_config("3'' reorient.state_dense, PGS solver at MuJoCo's defaults", "reorient",
                                  "state_dense", 4096, solver="PGS"),
        "5": lambda: env_config("5 bimanual.state_dense (two-hand handover task)", "bimanual", "state_dense", 4096),
        "5p": bimanual,
    }
    for k in (sys.argv[1:] or list(runs)):
        print(json.dumps(runs[k]()), flush=True)


if __name__ == "__main__":
    main()
