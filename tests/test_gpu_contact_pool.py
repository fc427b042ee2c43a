"""The contact pool (include/dx.h dx_health words 0 and 6).

The step kernel keeps 32 contacts per env and physics step in LDS.  A physics step that
finds more is deferred, from the state it started from, to the overflow tier (dx_step.hip
env_defer -> dx_step_hi_kernel: the same physics with a 256-contact pool, above the
reference scenes' nconmax = 200, shadow_hand_series_e.xml:8), so nothing is dropped below
the reference's pool.  A pool that still overflows keeps its first contacts in candidate
(generation) order, as MuJoCo fills its contact buffer -- and as the oracle does with its
256-contact pool (oracle/dx_oracle.c NCON_MAX).  Both are compared with the fp64 oracle
here: contact lists element by element, the constrained accelerations, one physics step
and five.  The scenes are built from the compiler's own primitives (a ground plane and
free cubes resting 1 mm into it, four plane-box corners each), so they compile on the GPU
box."""

import numpy as np
import pytest

from dexterity_amd import _lib, blob

pytestmark = pytest.mark.gpu


def _ground(s):
    s.add_world_geom("ground", "plane", (1, 1, 0.1), friction="0.4 0.005 0.0001", solimp="0.95 0.99 0.001",
                     solref="0.002 1")


def box_field(n_boxes):
    """`n_boxes` separate cubes (half-size 2 cm) on the ground: 4 contacts each."""
    from dexterity_amd.mjcf.compiler import Scene

    s = Scene(timestep=0.005)
    _ground(s)
    for i in range(n_boxes):
        s.add_free_box(f"box{i}", 0.02, [0.1 * (i % 5) - 0.2, 0.1 * (i // 5), 0.019])
    return s.compile()


def bar_field(n_bars=10, n_parts=8):
    """`n_bars` compound bodies of `n_parts` cubes in a row on the ground: 4 contacts per
    cube, 320 for the default -- beyond the 256-contact pool."""
    from dexterity_amd.mjcf.compiler import Scene

    s = Scene(timestep=0.005)
    _ground(s)
    for i in range(n_bars):
        s.add_free_box(f"bar{i}", 0.02, [0.5 * (i % 2) - 0.5, 0.2 * (i // 2) - 0.4, 0.019],
                       parts=[(0.05 * k, 0.0, 0.0) for k in range(1, n_parts)])
    return s.compile()


def _states(cm, n, rng, lift_max):
    """Env e: the resting field with up to `lift_max` free bodies lifted 5 cm (out of
    contact; env 0 lifts none) and small random velocities everywhere."""
    nb = cm.nq // 7
    out = []
    for e in range(n):
        q = cm.qpos0.copy()
        k = 0 if e == 0 else rng.randint(0, lift_max + 1)
        for b in rng.choice(nb, size=k, replace=False):
            q[7 * b + 2] += 0.05
        v = rng.uniform(-0.05, 0.05, size=cm.nv)
        out.append((q, v))
    return out


def _oracle(oracle_mod, om, q, v, nstep):
    d = oracle_mod.OracleData(om)
    d.qpos[:] = np.asarray(q, np.float32)
    d.qvel[:] = np.asarray(v, np.float32)
    if nstep == 0:
        d.forward()
    for _ in range(nstep):
        d.step()
    return d


def _check_contacts(rec, n, d):
    """GPU contact records (debug "contact": pos 3, frame 9, dist, geom1, geom2, condim)
    against the oracle's list, element by element (both in candidate order)."""
    oc = d.contacts()
    assert n == len(oc)
    r = rec[:n].astype(np.float64)
    np.testing.assert_array_equal(r[:, 13:15], oc[:, 13:15])
    np.testing.assert_allclose(r[:, 12], oc[:, 12], atol=2e-6)
    np.testing.assert_allclose(r[:, 0:3], oc[:, 0:3], atol=2e-5)
    np.testing.assert_allclose(r[:, 3:12], oc[:, 3:12], atol=1e-5)


def _run(gpu_phys, cm, states, nstep, debug=False):
    from dexterity_amd import physics

    ph = physics.BatchedPhysics(physics.Model(cm), len(states))
    ph.set(_lib.QPOS, np.stack([s[0] for s in states]))
    ph.set(_lib.QVEL, np.stack([s[1] for s in states]))
    if debug:
        ph.debug(True)
    ph.health_clear()
    if nstep == 0:
        ph.forward()
    else:
        ph.step(nstep)
    return ph


@pytest.mark.parametrize("nstep", [0, 1, 5])
def test_pool_beyond_step_kernel_matches_oracle(oracle_mod, nstep):
    """10 cubes (40 contacts when all rest on the ground, down to 24): the envs with more
    than 32 go to the overflow tier, none is truncated, and contacts, qacc (forward), one
    physics step and five (the substep queue's deferral mid-step) match the oracle."""
    cm = box_field(10)
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    rng = np.random.RandomState(1)
    states = _states(cm, 16, rng, 4)
    ph = _run(None, cm, states, nstep, debug=(nstep == 0))
    h = ph.health()
    ncon = ph.get(_lib.NCON)[:, 0]
    assert h["contact_overflow"] == 0 and h["diverged"] == 0, h
    ds = [_oracle(oracle_mod, om, q, v, nstep) for q, v in states]
    expect_deferred = 0
    for e, d in enumerate(ds):
        assert ncon[e] == d.ncon, (e, ncon[e], d.ncon)
    if nstep == 0:
        rec = ph.debug_get("contact")
        qacc = ph.qacc
        for e, d in enumerate(ds):
            _check_contacts(rec[e], ncon[e], d)
            scale = max(1.0, np.abs(d.qacc_smooth).max())
            np.testing.assert_allclose(qacc[e], d.qacc, atol=5e-4 * scale)
            expect_deferred += d.ncon > 32
        assert expect_deferred >= 3 and expect_deferred < len(states), expect_deferred
        assert h["contact_deferred"] == expect_deferred, h
    else:
        assert h["contact_deferred"] >= 3, h
        qpos, qvel = ph.qpos, ph.qvel
        tol_q = 1e-6 if nstep == 1 else 1e-5
        for e, d in enumerate(ds):
            np.testing.assert_allclose(qpos[e], d.qpos, atol=tol_q)
            np.testing.assert_allclose(qvel[e], d.qvel, atol=5e-4 * max(1.0, np.abs(d.qvel).max()))
    assert (ncon > 32).any() and (ncon <= 32).any()
    ph.close()


def test_steps_beyond_mid_tier_match_oracle(oracle_mod):
    """A queued physics step with 256 contacts (10 bars of 8 cubes, two lifted) passes the
    step kernel (32) and the mid tier running beside it (64, dx_step_mid_kernel) and ends
    in the overflow tier (256): one step and three match the oracle, nothing is cut."""
    cm = bar_field()
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    q1 = cm.qpos0.copy()
    q1[7 * 3 + 2] += 0.05
    q1[7 * 6 + 2] += 0.05
    rng = np.random.RandomState(3)
    states = [(q1, rng.uniform(-0.01, 0.01, size=cm.nv)) for _ in range(3)]
    for nstep in (1, 3):
        ph = _run(None, cm, states, nstep)
        h = ph.health()
        assert h["contact_overflow"] == 0 and h["diverged"] == 0 and h["contact_deferred"] >= 3, h
        qpos, qvel = ph.qpos, ph.qvel
        for e, (q, v) in enumerate(states):
            d = _oracle(oracle_mod, om, q, v, nstep)
            np.testing.assert_allclose(qpos[e], d.qpos, atol=1e-6 if nstep == 1 else 1e-5)
            np.testing.assert_allclose(qvel[e], d.qvel, atol=5e-4 * max(1.0, np.abs(d.qvel).max()))
        ph.close()


_SERIAL_SNIPPET = """
import sys, numpy as np
sys.path.insert(0, {root!r})
from dexterity_amd import _lib, physics
from tests.test_gpu_contact_pool import box_field, _states
cm = box_field(10)
states = _states(cm, 16, np.random.RandomState(1), 4)
ph = physics.BatchedPhysics(physics.Model(cm), len(states))
ph.set(_lib.QPOS, np.stack([s[0] for s in states]))
ph.set(_lib.QVEL, np.stack([s[1] for s in states]))
for _ in range(3):
    ph.step(5)
np.save(sys.argv[1], np.concatenate([ph.qpos, ph.qvel], axis=1))
print("deferred", ph.health()["contact_deferred"])
"""


def test_tiers_under_serialised_kernels(tmp_path):
    """The mid tier and the overflow tier never wait for each other to start: with every
    kernel serialised (AMD_SERIALIZE_KERNEL=3, as a profiler's counter collection does),
    deferred physics steps still complete -- the overflow tier takes the entries the mid
    tier has not -- and the results equal the concurrent run's bit for bit."""
    import os
    import subprocess
    import sys

    from tests.conftest import ROOT

    outs = []
    for serial in (False, True):
        env = dict(os.environ)
        if serial:
            env["AMD_SERIALIZE_KERNEL"] = "3"
        f = str(tmp_path / f"out_{int(serial)}.npy")
        r = subprocess.run([sys.executable, "-c", _SERIAL_SNIPPET.format(root=ROOT), f], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        assert int(r.stdout.split()[-1]) >= 3
        outs.append(np.load(f))
    np.testing.assert_array_equal(outs[0], outs[1])


def test_pool_cut_keeps_candidate_order(oracle_mod):
    """10 bars of 8 cubes on the ground: 320 contacts, beyond the 256-contact pool.  The
    first 256 in candidate order are kept -- the oracle's list, whose pool (256) fills
    in the same generation order -- the truncation is counted, and the constrained
    accelerations on the kept set match.  With two bars lifted (256 contacts exactly)
    nothing is cut."""
    cm = bar_field()
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    q0 = cm.qpos0.copy()
    q1 = cm.qpos0.copy()
    q1[7 * 3 + 2] += 0.05
    q1[7 * 6 + 2] += 0.05
    states = [(q0, np.zeros(cm.nv)), (q1, np.zeros(cm.nv))]
    ph = _run(None, cm, states, 0, debug=True)
    h = ph.health()
    ncon = ph.get(_lib.NCON)[:, 0]
    assert list(ncon) == [256, 256]
    assert h["contact_overflow"] == 1 and h["ncon_max"] == 320, h
    rec = ph.debug_get("contact")
    qacc = ph.qacc
    for e, (q, v) in enumerate(states):
        d = _oracle(oracle_mod, om, q, v, 0)
        _check_contacts(rec[e], ncon[e], d)
        scale = max(1.0, np.abs(d.qacc_smooth).max())
        np.testing.assert_allclose(qacc[e], d.qacc, atol=5e-4 * scale)
    ph.close()
