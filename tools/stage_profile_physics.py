#!/usr/bin/env python3
"""Per-stage cycle profile of the step kernel on a physics-level scene (diagnostics).

usage: python tools/stage_profile_physics.py <asset> [nenv] [steps]
e.g.   python tools/stage_profile_physics.py bimanual_handover 4096 5
Random actions within ctrlrange held for 5 physics substeps per control step, the
hands gravity-compensated (the prefix of every hand body starts with "shadow_hand").
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import _lib, physics  # noqa: E402
from dexterity_amd.mjcf.compiler import CompiledModel  # noqa: E402

asset = sys.argv[1] if len(sys.argv) > 1 else "bimanual_handover"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
cm = CompiledModel.load(os.path.join(ROOT, "assets", f"{asset}.npz"))
model = physics.Model(cm)
phys = physics.BatchedPhysics(model, B)
phys.set_xfrc(physics.gravity_compensation(cm, "shadow_hand"))
lo, hi = cm.actuator_ctrlrange.T
rng = np.random.RandomState(1)
L = _lib.load()
for i in range(5):
    phys.set(_lib.CTRL, rng.uniform(lo, hi, size=(B, cm.nu)))
    phys.step(5)
phys.sync()
_lib.check(L.dx_stage_timing(phys.ptr, 1))
buf = (ctypes.c_uint64 * (_lib.NSTAGE * B))()
_lib.check(L.dx_stage_read(phys.ptr, buf, _lib.NSTAGE * B))
t = time.perf_counter()
for i in range(steps):
    phys.set(_lib.CTRL, rng.uniform(lo, hi, size=(B, cm.nu)))
    phys.step(5)
phys.sync()
dt = time.perf_counter() - t
_lib.check(L.dx_stage_read(phys.ptr, buf, _lib.NSTAGE * B))
per_env = np.frombuffer(buf, dtype=np.uint64).reshape(B, _lib.NSTAGE).astype(np.float64)
cyc = per_env.sum(axis=0)
n = B * steps * 5
cols = list(range(len(_lib.STAGES)))
tot = cyc[cols].sum()
print(f"{asset} B={B} steps={steps}: {dt / steps * 1e3:.2f} ms/step (host ctrl upload included); "
      f"{tot / n:.0f} cycles per env-substep")
for k in np.argsort(-cyc[cols]):
    print(f"  {_lib.STAGES[k]:20s} {100 * cyc[k] / tot:6.2f}%  {cyc[k] / n:10.0f} cyc/env-substep")
print({name: round(cyc[k] / n, 2) for k, name in _lib.COUNTERS.items()})
phys.close()
