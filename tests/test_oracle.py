"""CPU oracle checks: physical invariants and an independent numpy restatement.

The oracle's dynamics cannot be compared with real MuJoCo here (absent, SURVEY.md
§8 c1: parity unpinned).  These tests pin what can be pinned without it:
  * kinematics + CRB mass matrix against the independent numpy implementation in
    dexterity_amd/mjcf/setconst.py (different code, same physics);
  * gravity torques against J^T(m g) built from numpy jacobians;
  * Coriolis power identity v.C(q,v)v = 1/2 v.dM/dt v;
  * gravity compensation (utils/mujoco_utils.py:91-99) cancels gravity exactly;
  * free fall, contact resting equilibrium (sum of normal forces = m g; a cube's
    penetration = the one MuJoCo's published soft-contact model gives), energy
    conservation of a frictionless undamped system, 100 steps without divergence
    (hands_test.py:52-57).
"""

import os

import numpy as np
import pytest

from dexterity_amd import blob
from dexterity_amd.mjcf import setconst
from dexterity_amd.physics import gravity_compensation
from tests.conftest import RESTING_CASES, ROOT, random_hand_state


def _data(oracle_mod, compiled):
    m = oracle_mod.OracleModel(blob.pack(compiled.arrays))
    return m, oracle_mod.OracleData(m)


@pytest.mark.parametrize("scene", ["reorient_compiled", "adroit_compiled"])
def test_mass_matrix_matches_numpy(oracle_mod, scene, request):
    cm = request.getfixturevalue(scene)
    m, d = _data(oracle_mod, cm)
    rng = np.random.RandomState(1)
    for _ in range(4):
        qpos, qvel = random_hand_state(cm, rng, frac=1.0)
        d.qpos[:] = qpos
        d.qvel[:] = qvel
        d.forward()
        M = d.M.reshape(cm.nv, cm.nv)
        Mref = setconst.mass_matrix(cm.arrays, qpos)[0]
        np.testing.assert_allclose(M, Mref, rtol=1e-10, atol=1e-14)
        assert np.all(np.linalg.eigvalsh(M) > 0)


def test_gravity_bias_matches_jacobian_transpose(oracle_mod, reorient_compiled):
    cm = reorient_compiled
    m, d = _data(oracle_mod, cm)
    rng = np.random.RandomState(2)
    qpos, _ = random_hand_state(cm, rng)
    d.qpos[:] = qpos
    d.qvel[:] = 0
    d.forward()
    A = cm.arrays
    M, cdof, com, xipos = setconst.mass_matrix(A, qpos)
    g = np.zeros(cm.nv)
    for b in range(1, cm.nbody):
        jp, _ = setconst.body_jacobian(A, cdof, com, b, xipos[b])
        g -= jp.T @ (cm.body_mass[b] * cm.gravity)
    np.testing.assert_allclose(d.qfrc_bias, g, rtol=1e-9, atol=1e-12)


def test_coriolis_power_identity(oracle_mod, reorient_compiled):
    cm = reorient_compiled
    arrays = dict(cm.arrays)
    arrays["gravity"] = np.zeros(3)
    m = oracle_mod.OracleModel(blob.pack(arrays))
    d = oracle_mod.OracleData(m)
    rng = np.random.RandomState(4)
    qpos, qvel = random_hand_state(cm, rng, vel=2.0)
    qvel[24:] = 0  # keep the free joint's quaternion velocity mapping out of the FD
    d.qpos[:] = qpos
    d.qvel[:] = qvel
    d.forward()
    cv = d.qfrc_bias.copy()
    h = 1e-6
    dq = np.zeros(cm.nq)
    dq[:24] = qvel[:24]
    Mp = setconst.mass_matrix(cm.arrays, qpos + h * dq)[0]
    Mm = setconst.mass_matrix(cm.arrays, qpos - h * dq)[0]
    Mdot = (Mp - Mm) / (2 * h)
    assert qvel @ cv == pytest.approx(0.5 * qvel @ Mdot @ qvel, rel=1e-5, abs=1e-10)


def test_gravity_compensation_cancels_hand_gravity(oracle_mod, reorient_compiled):
    cm = reorient_compiled
    m, d = _data(oracle_mod, cm)
    d.xfrc_applied[:] = gravity_compensation(cm, "shadow_hand_e/").ravel()
    rng = np.random.RandomState(5)
    qpos, _ = random_hand_state(cm, rng)
    d.qpos[:] = qpos
    # servo targets at the current joint positions -> zero actuator force
    from dexterity_amd import hands

    d.ctrl[:] = hands.shadow_joint_positions_to_control(qpos[:24])
    d.forward()
    assert np.abs(d.qfrc_actuator).max() < 1e-12
    assert np.abs(d.qacc_smooth[:24]).max() < 1e-9
    np.testing.assert_allclose(d.qacc_smooth[24:], [0, 0, -9.81, 0, 0, 0], atol=1e-9)


def test_cube_rests_on_palm(oracle_mod, reorient_compiled):
    """Drop the cube at the spawn-box centre: it settles on the palm, contacts
    carry its weight, nothing diverges (hands_test.py:52-57 style)."""
    cm = reorient_compiled
    m, d = _data(oracle_mod, cm)
    d.xfrc_applied[:] = gravity_compensation(cm, "shadow_hand_e/").ravel()
    for _ in range(200):
        assert d.step() == 0
    assert d.ncon > 0
    assert np.all(np.isfinite(d.qpos)) and np.all(np.isfinite(d.qvel))
    assert np.abs(d.qvel[24:27]).max() < 1e-2
    # contact normal forces balance the cube's weight (the hand is compensated)
    d.forward()
    J = d.efc_J.reshape(d.nefc, cm.nv)
    f = d.efc_force
    fz_cube = (J[:, 24:27].T @ f)[2]
    assert fz_cube == pytest.approx(0.064 * 9.81, rel=0.05)


def test_energy_conserved_without_dissipation(oracle_mod, reorient_compiled):
    cm = reorient_compiled
    arrays = dict(cm.arrays)
    arrays["gravity"] = np.zeros(3)
    arrays["dof_damping"] = np.zeros(cm.nv)
    arrays["dof_frictionloss"] = np.zeros(cm.nv)
    arrays["jnt_limited"] = np.zeros_like(cm.jnt_limited)
    arrays["disable_contact"] = np.array([1], np.int32)
    arrays["actuator_gainprm"] = np.zeros_like(cm.actuator_gainprm)
    arrays["actuator_biasprm"] = np.zeros_like(cm.actuator_biasprm)
    arrays["timestep"] = np.array([1e-4])
    m = oracle_mod.OracleModel(blob.pack(arrays))
    d = oracle_mod.OracleData(m)
    rng = np.random.RandomState(6)
    qpos, qvel = random_hand_state(cm, rng, vel=1.0)
    d.qpos[:] = qpos
    d.qvel[:] = qvel

    def energy():
        d.forward()
        M = d.M.reshape(cm.nv, cm.nv)
        return 0.5 * d.qvel @ M @ d.qvel

    e0 = energy()
    for _ in range(200):
        d.step()
    assert energy() == pytest.approx(e0, rel=2e-3)


def test_free_fall(oracle_mod, reorient_compiled):
    cm = reorient_compiled
    m, d = _data(oracle_mod, cm)
    d.qpos[24:27] = [0.5, 0.5, 1.0]  # far from the hand and the ground
    for _ in range(10):
        d.step()
    t = 10 * cm.timestep
    # semi-implicit Euler: z = z0 - g h^2 n(n+1)/2
    assert d.qpos[26] == pytest.approx(1.0 - 9.81 * cm.timestep**2 * 10 * 11 / 2, rel=1e-12)
    assert d.qvel[26] == pytest.approx(-9.81 * t, rel=1e-12)
    assert d.ncon == 0


def test_adroit_hundred_steps(oracle_mod, adroit_compiled):
    cm = adroit_compiled
    m, d = _data(oracle_mod, cm)
    d.xfrc_applied[:] = gravity_compensation(cm, "adroit_hand/").ravel()
    rng = np.random.RandomState(7)
    lo, hi = cm.actuator_ctrlrange.T
    for _ in range(100):
        d.ctrl[:] = rng.uniform(lo, hi)
        assert d.step() == 0
    assert np.all(np.isfinite(d.qpos))
    assert d.nefc > 0  # tendon coupling limits are active


def test_flop_counters_populated(oracle_mod, reorient_compiled):
    m, d = _data(oracle_mod, reorient_compiled)
    d.flops_reset()
    d.step()
    fl = d.flops()
    assert fl.shape == (8,) and np.all(fl[[0, 1, 4, 6]] > 0) and fl[7] >= 0


def test_flop_counters_split_full_hull_scan(oracle_mod, reorient_compiled):
    """Mesh supports are charged at an efficient support's 16 vertices; the exhaustive
    scan's surplus goes to the separate "scan" stage (not algorithmic work)."""
    from dexterity_amd.physics import gravity_compensation

    m, d = _data(oracle_mod, reorient_compiled)
    cm = reorient_compiled
    d.xfrc_applied[:] = gravity_compensation(cm, "shadow_hand_e/").ravel()
    d.qpos[24:27] = (0.0, -0.13, 0.16)  # the cube falls into the palm: mesh-box MPR
    for _ in range(60):
        d.step()
    d.flops_reset()
    d.step()
    fl = d.flops()
    assert fl[2] > 0 and fl[7] > 0


# --------------------------------------------------------------------------- #
# the reference's physics known-answer tests, on the fp64 oracle (CPU)
# --------------------------------------------------------------------------- #
@pytest.mark.parametrize("joint,tau", [(j, t) for j in (0, 2, 4) for t in (0.0, -6.0, 5.0)])
def test_oracle_joint_torque_sensor_kat(oracle_mod, joint, tau):
    """hands_test.py:159-193 on the standalone Adroit hand: contact, gravity and
    actuation disabled, tau about joint `joint`'s axis on its body, step until the
    joint stops; the torque sensor projected on the axis reads -tau within 1e-2."""
    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel

    cm = CompiledModel.load(os.path.join(ROOT, "assets", "adroit_hand.npz")).disabled("contact", "gravity", "actuation")
    d = oracle_mod.OracleData(oracle_mod.OracleModel(blob.pack(cm.arrays)))
    d.fk()
    b, da = int(cm.jnt_bodyid[joint]), int(cm.jnt_dofadr[joint])
    axis = np.asarray(cm.jnt_axis[joint], dtype=np.float64)
    x = np.zeros((cm.nbody, 6))
    x[b, 3:] = tau * (d.xmat.reshape(-1, 3, 3)[b] @ axis)
    d.xfrc_applied[:] = x.ravel()
    d.step()
    n = 1
    while abs(d.qvel[da]) > 1e-2 and n < 5000:
        d.step()
        n += 1
    assert n < 5000
    assert abs(-(d.sensor_torque.reshape(-1, 3)[b] @ axis) - tau) <= 1e-2


def test_oracle_adroit_fingertip_golden_ik(oracle_mod):
    """hands_test.py:195-228: the five golden fingertip positions are reachable by the
    IK attempt loop (ik_solver.py:155-228) within 1e-3; starts at the joint midrange,
    then uniform random starts (the reference's attempts) until one succeeds."""
    from dexterity_amd import blob, hands
    from dexterity_amd.mjcf.compiler import CompiledModel

    golden = np.array([[-0.003572, -0.020904, 0.371999], [-0.028277, -0.036063, 0.391271],
                       [-0.052305, -0.006066, 0.393481], [-0.089808, -0.042816, 0.423813],
                       [0.026246, -0.017261, 0.416314]])
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "adroit_hand.npz"))
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    sites = [cm.names["site"].index("adroit_hand/" + s) for s in hands.ADROIT_FINGERTIP_SITES]
    joints = [cm.names["joint"].index("adroit_hand/" + j) for j in hands.SHADOW_JOINTS]
    lo, hi = np.asarray(cm.jnt_range)[joints].T
    rng = np.random.RandomState(0)
    for attempt in range(30):
        d = oracle_mod.OracleData(om)
        d.qpos[cm.jnt_qposadr[joints]] = (lo + hi) / 2 if attempt == 0 else rng.uniform(lo, hi)
        steps, err = d.ik_attempt(sites, joints, golden, early_stop=True)
        if np.all(err <= 1e-3):
            break
    assert np.all(err <= 1e-3)
    d.fk()
    np.testing.assert_allclose(d.site_xpos.reshape(-1, 3)[sites], golden, atol=1e-3)


def test_oracle_cg_reaches_the_newton_optimum(oracle_mod, reorient_compiled):
    """`<option solver="CG">` ([3P] MuJoCo's primal Polak-Ribiere CG) minimises the same
    convex constraint cost as Newton: on contact-rich states both reach the same
    acceleration (to the solvers' tolerance) and cost."""
    from dexterity_amd import blob

    cm = reorient_compiled
    xfrc = gravity_compensation(cm, "shadow_hand_e/")
    newton = oracle_mod.OracleModel(blob.pack(cm.arrays))
    cg = oracle_mod.OracleModel(blob.pack(cm.with_solver("CG", iterations=1000, tolerance=1e-10).arrays))
    rng = np.random.RandomState(3)
    d = oracle_mod.OracleData(newton)
    d.xfrc_applied[:] = xfrc.ravel()
    d.qpos[24:27] += [0.01, -0.01, 0]
    lo, hi = cm.actuator_ctrlrange.T
    checked = 0
    for s in range(120):
        d.ctrl[:] = 0.3 * rng.uniform(lo, hi)
        d.step()
        if s % 20 != 19:
            continue
        a = oracle_mod.OracleData(newton)
        b = oracle_mod.OracleData(cg)
        for x in (a, b):
            x.xfrc_applied[:] = xfrc.ravel()
            x.qpos[:], x.qvel[:], x.ctrl[:], x.qacc_warmstart[:] = d.qpos, d.qvel, d.ctrl, d.qacc_warmstart
            x.forward()
        assert a.nefc == b.nefc and a.nefc > 24
        scale = max(1.0, np.abs(a.qacc_smooth).max())
        assert np.abs(a.qacc - b.qacc).max() <= 1e-4 * scale, np.abs(a.qacc - b.qacc).max()
        assert b.niter >= 1
        checked += a.ncon > 0
    assert checked >= 3


def test_oracle_pgs_reaches_the_newton_optimum(oracle_mod, reorient_compiled):
    """`<option solver="PGS">` ([3P] MuJoCo's dual projected Gauss-Seidel) solves the
    dual of the primal problem Newton minimises: run to convergence, its acceleration
    qacc_smooth + M^-1 J'f is Newton's (the restatement's anchor: MuJoCo itself is not
    in the reference, so PGS's iterates are pinned only through this optimum).  At
    MuJoCo's defaults (100 sweeps, 1e-8) it stops within the sweep budget."""
    from dexterity_amd import blob

    cm = reorient_compiled
    xfrc = gravity_compensation(cm, "shadow_hand_e/")
    newton = oracle_mod.OracleModel(blob.pack(cm.arrays))
    pgs = oracle_mod.OracleModel(blob.pack(cm.with_solver("PGS", iterations=20000, tolerance=1e-15).arrays))
    pgs_d = oracle_mod.OracleModel(blob.pack(cm.with_solver("PGS").arrays))
    rng = np.random.RandomState(3)
    d = oracle_mod.OracleData(newton)
    d.xfrc_applied[:] = xfrc.ravel()
    d.qpos[24:27] += [0.01, -0.01, 0]
    lo, hi = cm.actuator_ctrlrange.T
    checked = 0
    for s in range(120):
        d.ctrl[:] = 0.3 * rng.uniform(lo, hi)
        d.step()
        if s % 20 != 19:
            continue
        a = oracle_mod.OracleData(newton)
        b = oracle_mod.OracleData(pgs)
        c = oracle_mod.OracleData(pgs_d)
        for x in (a, b, c):
            x.xfrc_applied[:] = xfrc.ravel()
            x.qpos[:], x.qvel[:], x.ctrl[:], x.qacc_warmstart[:] = d.qpos, d.qvel, d.ctrl, d.qacc_warmstart
            x.forward()
        assert a.nefc == b.nefc and a.nefc > 24
        scale = max(1.0, np.abs(a.qacc_smooth).max())
        assert np.abs(a.qacc - b.qacc).max() <= 1e-5 * scale, np.abs(a.qacc - b.qacc).max()
        assert 1 <= b.niter < 20000
        assert 1 <= c.niter <= 100
        # (100 sweeps do not reach the optimum on the light cube's dofs: Gauss-Seidel's
        # slow tail, which MuJoCo's PGS has as well)
        assert np.all(np.isfinite(c.qacc))
        checked += a.ncon > 0
    assert checked >= 3


@pytest.mark.parametrize("tilt", [5.0, 10.0, 15.0, 25.0, 30.0])
def test_oracle_inclined_plane_friction_kat(oracle_mod, tilt):
    """Contact physics against a physical law rather than the restatement: a cube on a
    plane tilted below tan^-1(mu) stays put (|v| < 2e-3 m/s after 0.6 s: MuJoCo's soft
    contacts creep slightly), and above it slides with a = g (sin - mu cos) within 5 %
    (the soft constraint's regularisation makes friction a little weaker than Coulomb's).
    tests/test_gpu_kat.py runs the same case on the GPU kernel."""
    from dexterity_amd import blob
    from tests.conftest import inclined_box_scene

    cm = inclined_box_scene(tilt)
    d = oracle_mod.OracleData(oracle_mod.OracleModel(blob.pack(cm.arrays)))
    d.qpos[:] = cm.qpos0
    for _ in range(100):
        d.step()
    v0 = d.qvel[0]
    for _ in range(200):
        d.step()
    a = (d.qvel[0] - v0) / (200 * 0.002)
    th, mu, g = np.radians(tilt), 0.4, 9.81
    if np.tan(th) < mu:
        assert abs(d.qvel[0]) < 2e-3 and abs(a) < 1e-2, (tilt, d.qvel[0], a)
    else:
        expect = g * (np.sin(th) - mu * np.cos(th))
        assert abs(a - expect) <= 0.05 * expect, (tilt, a, expect)
    assert abs(d.qpos[2] - 0.02) < 1e-3  # still resting on a face


@pytest.mark.parametrize("condim,mu,solref", RESTING_CASES)
def test_oracle_resting_contact_depth_kat(oracle_mod, condim, mu, solref):
    """Contact dynamics against MuJoCo's published soft-contact model rather than the
    restatement: a cube left on a level plane settles (|qvel| < 1e-9 after 2 s) at the
    penetration tests/conftest.py resting_depth derives from K, d(r) and R alone, within
    1e-6 of it; four contacts (one per bottom corner).  tests/test_gpu_kat.py runs the
    same cases on the GPU kernel."""
    from tests.conftest import resting_box_scene, resting_depth

    cm = resting_box_scene(condim, mu, solref)
    assert abs(cm.body_invweight0[1][0] - 1.0 / 0.064) < 1e-9  # A = 1 / m
    d = oracle_mod.OracleData(oracle_mod.OracleModel(blob.pack(cm.arrays)))
    d.qpos[:] = cm.qpos0
    for _ in range(1000):
        d.step()
    r = resting_depth(condim, mu, solref)
    assert d.ncon == 4
    assert np.abs(d.qvel).max() < 1e-9
    assert abs((0.02 - d.qpos[2]) - r) <= 1e-6 * r, (0.02 - d.qpos[2], r)


def test_batch_step_watch_is_the_fall_test(oracle_mod, reorient_compiled):
    """batch_step_watch's flag is ReOrient._is_prop_fallen (reorient.py:229-235): a
    prop-ground contact (dist <= 1e-8) at the state after the steps -- set for a cube
    resting on the ground, clear for one held above it (the CPU baseline's reset rule)."""
    from dexterity_amd.physics import gravity_compensation

    cm = reorient_compiled
    om = oracle_mod.OracleModel(__import__("dexterity_amd.blob", fromlist=["pack"]).pack(cm.arrays))
    q = np.tile(cm.qpos0, (2, 1))
    q[0, 24:27] = (0.3, 0.3, 0.0195)  # on the ground, away from the hand
    q[1, 24:27] = (0.0, -0.13, 0.16)   # the spawn point above the palm
    z = np.zeros((2, cm.nv))
    ctrl = np.zeros((2, cm.nu))
    g = cm.names["geom"].index("ground")
    b = cm.names["body"].index("prop/")
    rc, _, _, _, fell = oracle_mod.batch_step_watch(om, q, z.copy(), ctrl, z.copy(),
                                                    gravity_compensation(cm, "shadow_hand_e/"), 5, g, b)
    assert rc == 0 and fell.tolist() == [True, False]
