"""The reference's own physics known-answer tests, run through the C ABI on the GPU
(and, as the checker, on the fp64 oracle):

  * hands_test.py:159-193  joint torque sensors at static equilibrium: Adroit hand
    alone, contact / gravity / actuation disabled, a torque tau in {0, -6, 5} applied
    on the body of joint {0, 2, 4} about the joint axis; step until the joint stops
    (|qvel| <= 1e-2); the joint torque observable must read -tau within 1e-2;
  * hands_test.py:195-228  five golden Adroit fingertip positions reached by the IK
    solver (linear_tol 1e-3, early stop, first successful attempt) and confirmed by
    forward kinematics within atol 1e-3;
and two contact known answers from physics rather than the restatement: the inclined
plane (Coulomb stick / slide) and the resting cube's equilibrium penetration (MuJoCo's
published soft-contact model).
"""

import os

import numpy as np
import pytest

from dexterity_amd import _lib, blob
from dexterity_amd.mjcf.compiler import CompiledModel
from tests.conftest import RESTING_CASES, ROOT

pytestmark = pytest.mark.gpu

# hands_test.py:196-205
FINGERTIP_GOLDEN = np.array([
    [-0.003572, -0.020904, 0.371999],
    [-0.028277, -0.036063, 0.391271],
    [-0.052305, -0.006066, 0.393481],
    [-0.089808, -0.042816, 0.423813],
    [0.026246, -0.017261, 0.416314],
])


@pytest.fixture(scope="module")
def gpu():
    from dexterity_amd import build, physics

    build.build()
    return physics


@pytest.fixture(scope="module")
def adroit_hand():
    return CompiledModel.load(os.path.join(ROOT, "assets", "adroit_hand.npz"))


def _applied_torque(cm, xmat, joint, tau):
    """physics.bind(joint.parent).xfrc_applied[3:] = tau * physics.bind(joint).xaxis."""
    b = int(cm.jnt_bodyid[joint])
    xaxis = xmat.reshape(-1, 3, 3)[b] @ np.asarray(cm.jnt_axis[joint], dtype=np.float64)
    x = np.zeros((cm.nbody, 6))
    x[b, 3:] = tau * xaxis
    return x


@pytest.mark.parametrize("joint,tau", [(j, t) for j in (0, 2, 4) for t in (0.0, -6.0, 5.0)])
def test_joint_torque_sensor_equilibrium_kat(gpu, oracle_mod, adroit_hand, joint, tau):
    cm = adroit_hand.disabled("contact", "gravity", "actuation")
    b = int(cm.jnt_bodyid[joint])
    da = int(cm.jnt_dofadr[joint])
    axis = np.asarray(cm.jnt_axis[joint], dtype=np.float64)
    # oracle (fp64)
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    d = oracle_mod.OracleData(om)
    d.fk()
    xfrc = _applied_torque(cm, d.xmat, joint, tau)
    d.xfrc_applied[:] = xfrc.ravel()
    d.step()
    n_or = 1
    while abs(d.qvel[da]) > 1e-2 and n_or < 5000:
        d.step()
        n_or += 1
    torque_or = -(d.sensor_torque.reshape(-1, 3)[b] @ axis)
    assert abs(torque_or - tau) <= 1e-2
    # GPU (fp32), same procedure through the C ABI
    model = gpu.Model(cm)
    ph = gpu.BatchedPhysics(model, 1)
    ph.set_xfrc(xfrc)
    ph.enable_sensors(True)
    ph.step(1)
    n = 1
    while abs(ph.qvel[0, da]) > 1e-2 and n < 5000:
        ph.step(1)
        n += 1
    torque = -ph.joint_torques([b], axis[None, :])[0, 0]
    ph.close()
    assert abs(torque - tau) <= 1e-2, (torque, tau, n)
    assert abs(n - n_or) <= max(2, 0.05 * n_or)
    assert abs(torque - torque_or) <= 2e-3


def test_torque_sensors_match_oracle_with_contacts(gpu, oracle_mod):
    """Every body's torque sensor after a forward pass at contact-rich reorient states
    (contact forces, gravity compensation and actuation all enter cfrc_int), GPU fp32
    vs oracle fp64, within 2e-3 of the largest sensor reading of the state."""
    from tests.test_gpu_parity import _load_states, _oracle_forward, _oracle_states

    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    xfrc = gpu.gravity_compensation(cm, "shadow_hand_e/")
    om, states = _oracle_states(oracle_mod, cm, xfrc)
    model = gpu.Model(cm)
    ph = _load_states(gpu, model, xfrc, states)
    ph.enable_sensors(True)
    ph.forward()
    s = ph.get(_lib.SENSOR_TORQUE).reshape(len(states), cm.nbody, 3)
    with_contacts = 0
    for e, st in enumerate(states):
        d = _oracle_forward(oracle_mod, om, cm, xfrc, st)
        so = d.sensor_torque.reshape(cm.nbody, 3)
        scale = max(np.abs(so).max(), 1e-3)
        assert np.abs(s[e] - so).max() <= 2e-3 * scale, (e, np.abs(s[e] - so).max(), scale)
        with_contacts += d.ncon > 0
    assert with_contacts >= 6
    ph.close()


def test_adroit_fingertip_golden_ik(gpu, oracle_mod, adroit_hand):
    from dexterity_amd.inverse_kinematics import IKSolver

    model = gpu.Model(adroit_hand)
    solver = IKSolver(model, hand="adroit")
    qpos = solver.solve(target_positions=FINGERTIP_GOLDEN, linear_tol=1e-3, early_stop=True,
                        stop_on_first_successful_attempt=True)
    assert qpos is not None
    lo, hi = adroit_hand.jnt_range[solver.joints].T
    assert np.all(qpos >= lo - 1e-6) and np.all(qpos <= hi + 1e-6)
    # hand.set_joint_angles + fingertip_positions observable, in fp64
    om = oracle_mod.OracleModel(blob.pack(adroit_hand.arrays))
    d = oracle_mod.OracleData(om)
    d.qpos[adroit_hand.jnt_qposadr[solver.joints]] = qpos
    d.fk()
    tips = d.site_xpos.reshape(-1, 3)[solver.sites]
    np.testing.assert_allclose(tips, FINGERTIP_GOLDEN, atol=1e-3)
    solver.close()


@pytest.mark.parametrize("condim,mu,solref", RESTING_CASES)
def test_resting_contact_depth_kat(gpu, condim, mu, solref):
    """The resting-contact known answer on the fp32 kernel (tests/test_oracle.py has it
    on the oracle): a cube left on a level plane settles at the penetration MuJoCo's
    published soft-contact model gives (tests/conftest.py resting_depth: K, d(r), R with
    frictionless or pyramidal rows), within 1e-3 of it (fp32 position near 0.02 m:
    ulp 1.9e-9 against depths of 1.4e-5 .. 1.2e-3 m), at rest (|qvel| < 1e-5) after 2 s."""
    from tests.conftest import resting_box_scene, resting_depth

    cm = resting_box_scene(condim, mu, solref)
    ph = gpu.BatchedPhysics(gpu.Model(cm), 4)
    for _ in range(5):  # (at most 255 physics steps per call)
        ph.step(200)
    q = ph.qpos.astype(np.float64)
    v = ph.qvel.astype(np.float64)
    ph.close()
    r = resting_depth(condim, mu, solref)
    assert np.abs(v).max() < 1e-5, np.abs(v).max()
    assert np.all(np.abs((0.02 - q[:, 2]) - r) <= 1e-3 * r), (0.02 - q[:, 2], r)


@pytest.mark.parametrize("tilt", [5.0, 10.0, 15.0, 25.0, 30.0])
def test_inclined_plane_friction_kat(gpu, oracle_mod, tilt):
    """The inclined-plane known answer on the fp32 kernel (tests/test_oracle.py has it on
    the oracle): below tan^-1(0.4) the cube sticks, above it slides with
    a = g (sin - mu cos) within 5 %; and the kernel's velocity stays within 2 % (of the
    sliding speed, or 2e-4 m/s when sticking) of the oracle's over the same 0.6 s."""
    from tests.conftest import inclined_box_scene

    cm = inclined_box_scene(tilt)
    model = gpu.Model(cm)
    ph = gpu.BatchedPhysics(model, 4)
    ph.step(100)
    v0 = ph.qvel[:, 0].astype(np.float64)
    ph.step(200)
    v = ph.qvel.astype(np.float64)
    q = ph.qpos.astype(np.float64)
    a = (v[:, 0] - v0) / (200 * 0.002)
    th, mu, g = np.radians(tilt), 0.4, 9.81
    if np.tan(th) < mu:
        assert np.all(np.abs(v[:, 0]) < 2e-3) and np.all(np.abs(a) < 1e-2), (tilt, v[:, 0], a)
    else:
        expect = g * (np.sin(th) - mu * np.cos(th))
        assert np.all(np.abs(a - expect) <= 0.05 * expect), (tilt, a, expect)
    assert np.all(np.abs(q[:, 2] - 0.02) < 1e-3)
    d = oracle_mod.OracleData(oracle_mod.OracleModel(model.blob))
    d.qpos[:] = cm.qpos0
    for _ in range(300):
        d.step()
    assert np.all(np.abs(v[:, 0] - d.qvel[0]) <= max(2e-4, 0.02 * abs(d.qvel[0]))), (v[:, 0], d.qvel[0])
    ph.close()
