"""Mid-tier debugging: the contact-pool test's box field, 16 envs, one 5-substep step with
and without the mid tier; per-env ncon, time and health (-> stdout)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dexterity_amd import _lib, physics  # noqa: E402
from tests.test_gpu_contact_pool import _states, box_field  # noqa: E402

cm = box_field(10)
states = _states(cm, 16, np.random.RandomState(1), 4)
for nomid in (False, True, False):
    if nomid:
        os.environ["DX_NO_MID"] = "1"
    else:
        os.environ.pop("DX_NO_MID", None)
    for nstep in (1, 5, 2, 3):
        ph = physics.BatchedPhysics(physics.Model(cm), len(states))
        ph.set(_lib.QPOS, np.stack([s[0] for s in states]))
        ph.set(_lib.QVEL, np.stack([s[1] for s in states]))
        ph.health_clear()
        ph.step(nstep)
        h = ph.health()
        print(f"nomid={nomid} nstep={nstep}: ncon {ph.get(_lib.NCON)[:, 0].tolist()} time "
              f"{np.round(ph.get(_lib.TIME)[:, 0], 4).tolist()} deferred {h['contact_deferred']} "
              f"timeouts {ph.debug_get('queue_timeouts')[0]}", flush=True)
        ph.close()
