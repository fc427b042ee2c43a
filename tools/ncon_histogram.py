"""Contacts found per env-substep over a long random-action run of the bench workload
(reorient.state_dense, 4096 envs): the histogram that sizes DX_NCON_MAX, and the health
counters (include/dx.h dx_health) of the same run.  Writes gpurun_out/ncon_hist.json.

  python tools/ncon_histogram.py [envs] [control steps] [scene: reorient | bimanual]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import _lib, manipulation, physics  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 500
scene = sys.argv[3] if len(sys.argv) > 3 else "reorient"
t0 = time.perf_counter()
if scene == "reorient":
    env = manipulation.load("reorient", "state_dense", seed=12345, num_envs=B)
    ph = env.physics
    ph.ncon_histogram(True)
    env.reset()
    ph.health_clear()
    for i in range(steps):
        env.step_random(i)
        if i % 100 == 99:
            print(f"step {i + 1}: {ph.health()}", flush=True)
    nsub = env.task.config.n_sub_steps
else:  # bimanual handover physics (config 5), random ctrl, no task resets
    from dexterity_amd.mjcf.compiler import CompiledModel

    cm = CompiledModel.load(os.path.join(ROOT, "assets", "bimanual_handover.npz"))
    ph = physics.BatchedPhysics(physics.Model(cm), B)
    ph.set_xfrc(physics.gravity_compensation(cm, "shadow_hand_"))
    ph.ncon_histogram(True)
    ph.health_clear()
    rng = np.random.RandomState(0)
    lo, hi = cm.actuator_ctrlrange.T
    nsub = 5
    for i in range(steps):
        ph.set(_lib.CTRL, rng.uniform(lo, hi, size=(B, cm.nu)).astype(np.float32))
        ph.step(nsub)
h = ph.health()
hist = h.pop("ncon_hist")
n = int(hist.sum())
nz = np.nonzero(hist)[0]
out = {"scene": scene, "envs": B, "control_steps": steps, "env_substeps": n, "expected_env_substeps": B * steps * nsub,
       "health": h, "ncon_hist": {int(k): int(hist[k]) for k in nz},
       "mean": float((hist * np.arange(len(hist))).sum() / max(n, 1)),
       "p99": int(np.searchsorted(np.cumsum(hist), 0.99 * n)), "p999999": int(np.searchsorted(np.cumsum(hist), (1 - 1e-6) * n)),
       "max": int(nz.max()) if len(nz) else 0, "over_32": int(hist[33:].sum()), "seconds": time.perf_counter() - t0}
print(json.dumps(out), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
with open(os.path.join(ROOT, "gpurun_out", f"ncon_hist_{scene}.json"), "w") as f:
    json.dump(out, f, indent=1)
