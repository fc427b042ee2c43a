"""Per-stage cycle breakdown of dx_step_kernel (s_memtime, lane 0 of every env)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dexterity_amd import _lib, manipulation  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
domain = sys.argv[3] if len(sys.argv) > 3 else "reorient"  # e.g. reach_shadow (BASELINE config 2)
solver = sys.argv[4] if len(sys.argv) > 4 else None  # CG / PGS: <option solver=...> at MuJoCo's defaults
if solver is None:
    env = manipulation.load(domain, "state_dense", seed=3, num_envs=B)
else:
    task = manipulation.SUITE[(domain, "state_dense")]()
    task.compiled = task.compiled.with_solver(solver)
    env = manipulation.GoalEnvironment(task, num_envs=B, seed=3)
L = _lib.load()
env.reset()
for i in range(10):
    env.step_random(i)
env.physics.sync()
_lib.check(L.dx_stage_timing(env.physics.ptr, 1))
buf = (ctypes.c_uint64 * (_lib.NSTAGE * B))()
_lib.check(L.dx_stage_read(env.physics.ptr, buf, _lib.NSTAGE * B))
t = time.perf_counter()
for i in range(steps):
    env.step_random(100 + i)
env.physics.sync()
dt = time.perf_counter() - t
_lib.check(L.dx_stage_read(env.physics.ptr, buf, _lib.NSTAGE * B))
per_env = np.frombuffer(buf, dtype=np.uint64).reshape(B, _lib.NSTAGE).astype(np.float64)
cyc = per_env.sum(axis=0)
cnt = {name: cyc[k] / (B * steps * 5) for k, name in _lib.COUNTERS.items()}
cyc[list(_lib.COUNTERS)] = 0
tot = cyc.sum()
per = cyc / (B * steps * 5)
out = {}
print(f"B={B} steps={steps}: {dt/steps*1e3:.2f} ms/step; total cycles per env-substep {tot/(B*steps*5):.0f}")
for k, name in enumerate(_lib.STAGES):
    print(f"  {name:20s} {100*cyc[k]/tot:6.2f}%  {per[k]:12.0f} cyc/env-substep")
    out[name] = per[k]
np_parts = {name: per_env[:, k].sum() / (B * steps * 5) for k, name in _lib.NP_STAGES.items()}
if sum(np_parts.values()) > 0:  # a DX_NP_MARKS build: the narrowphase trip split
    trips = cnt["np_trips"]
    print("narrowphase trip split (cycles per env-substep, per trip):",
          ", ".join(f"{n} {v:.0f} ({v / max(trips, 1e-9):.0f})" for n, v in np_parts.items()))
print("narrowphase calls per env-substep", {k: round(v, 3) for k, v in cnt.items()})
# the heaviest environments bound the launch (longest-first dispatch): their stages
stage_cols = [k for k in range(len(_lib.STAGES))]
tot_env = per_env[:, stage_cols].sum(axis=1)
order = np.argsort(tot_env)
top = order[-max(1, B // 100):]
mid = order[B // 2 - B // 100: B // 2 + B // 100]
print(f"heaviest 1% envs: {tot_env[top].mean() / (steps * 5):.0f} cyc/substep, median band "
      f"{tot_env[mid].mean() / (steps * 5):.0f}")
for k in np.argsort(-per_env[top][:, stage_cols].mean(axis=0))[:12]:
    print(f"  {_lib.STAGES[k]:20s} top1% {per_env[top, k].mean() / (steps * 5):10.0f}   median {per_env[mid, k].mean() / (steps * 5):10.0f}")
for k, name in _lib.COUNTERS.items():
    print(f"  {name:16s} top1% {per_env[top, k].mean() / (steps * 5):8.2f}   median {per_env[mid, k].mean() / (steps * 5):8.2f}")
# the four heaviest single environments (with steps = 1: the heaviest env-steps)
for e in order[-4:][::-1]:
    parts = sorted(((per_env[e, k] / (steps * 5), _lib.STAGES[k]) for k in stage_cols), reverse=True)[:6]
    cnts = {name: round(per_env[e, k] / (steps * 5), 1) for k, name in _lib.COUNTERS.items()
            if name in ("mpr", "mpr_support", "mpr_hit", "np_trips", "newton_iter", "linesearch_iter", "nefc")}
    print(f"  env {e}: {tot_env[e] / (steps * 5):.0f} cyc/substep;", ", ".join(f"{n} {v:.0f}" for v, n in parts), cnts)
# substep queue: slot-time spent waiting for an env's previous physics step, against the
# tasks' own cycles (both in s_memtime cycles; 2.39 GHz shader clock under the bench)
wait = per_env[:, 35].sum()
busy = per_env[:, stage_cols].sum()
slots = 2047
print(f"queue waits {wait / (B * steps * 5):.0f} cyc/env-substep = {100 * wait / (busy + wait):.1f}% of slot time in "
      f"tasks; slot utilisation at 2.39 GHz ~ {(busy + wait) / (slots * dt / steps * 2.39e9 * steps):.3f}")
niter = env.physics.get(_lib.NITER)[:, 0]
ncon = env.physics.get(_lib.NCON)[:, 0]
print("niter hist", np.bincount(niter), "ncon mean", ncon.mean(), "max", ncon.max())
ncand = env.physics.get(_lib.NCAND)[:, 0]
print("ncand (observation pass) mean", ncand.mean(), "max", ncand.max())
json.dump({"B": B, "ms_per_step": dt / steps * 1e3, "cycles_per_env_substep": out}, open("gpurun_out/stages.json", "w"))
