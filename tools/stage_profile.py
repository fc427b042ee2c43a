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
env = manipulation.load("reorient", "state_dense", seed=3, num_envs=B)
L = _lib.load()
env.reset()
for i in range(10):
    env.step(env.sample_actions(i), device_action=True)
env.physics.sync()
_lib.check(L.dx_stage_timing(env.physics.ptr, 1))
buf = (ctypes.c_uint64 * _lib.NSTAGE)()
_lib.check(L.dx_stage_read(env.physics.ptr, buf, _lib.NSTAGE))
t = time.perf_counter()
for i in range(steps):
    env.step(env.sample_actions(100 + i), device_action=True)
env.physics.sync()
dt = time.perf_counter() - t
_lib.check(L.dx_stage_read(env.physics.ptr, buf, _lib.NSTAGE))
cyc = np.array(list(buf), dtype=np.float64)
cnt = {name: cyc[k] / (B * steps * 5) for k, name in _lib.COUNTERS.items()}
cyc[list(_lib.COUNTERS)] = 0
tot = cyc.sum()
per = cyc / (B * steps * 5)
out = {}
print(f"B={B} steps={steps}: {dt/steps*1e3:.2f} ms/step; total cycles per env-substep {tot/(B*steps*5):.0f}")
for k, name in enumerate(_lib.STAGES):
    print(f"  {name:20s} {100*cyc[k]/tot:6.2f}%  {per[k]:12.0f} cyc/env-substep")
    out[name] = per[k]
print("narrowphase calls per env-substep", {k: round(v, 3) for k, v in cnt.items()})
niter = env.physics.get(_lib.NITER)[:, 0]
ncon = env.physics.get(_lib.NCON)[:, 0]
print("niter hist", np.bincount(niter), "ncon mean", ncon.mean(), "max", ncon.max())
ncand = env.physics.get(_lib.NCAND)[:, 0]
print("ncand (observation pass) mean", ncand.mean(), "max", ncand.max())
json.dump({"B": B, "ms_per_step": dt / steps * 1e3, "cycles_per_env_substep": out}, open("gpurun_out/stages.json", "w"))
