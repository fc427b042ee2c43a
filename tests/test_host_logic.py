"""Host logic vs the reference's own values (tests/golden/reference_host.json).

Pins: hands_test.py:26-31 (P2C @ C2P == I), the Shadow/Adroit joint and actuator
orderings, rewards.tanh_squared (reach dense reward), rewards.weighted_average,
the STATE_ONLY observable set (observations.py:96-120), and the reward KAT of
reorient_test.py:13-50 restated on the oracle's task functions.
"""

import numpy as np
import pytest

from dexterity_amd import hands
from oracle import task_ref


def test_projection_matrices_match_reference(golden):
    g = golden["shadow"]
    np.testing.assert_array_equal(hands.POSITION_TO_CONTROL, np.array(g["position_to_control"]))
    np.testing.assert_array_equal(hands.CONTROL_TO_POSITION, np.array(g["control_to_position"]))
    assert hands.COUPLED_JOINT_IDS == g["coupled_joint_ids"]
    # hands_test.py:26-31
    np.testing.assert_array_equal(
        hands.POSITION_TO_CONTROL @ hands.CONTROL_TO_POSITION, np.eye(len(hands.SHADOW_ACTUATORS))
    )


def test_joint_and_actuator_orderings(golden, reorient_compiled, adroit_compiled):
    assert list(hands.SHADOW_JOINTS) == golden["shadow"]["joints"]
    assert list(hands.SHADOW_ACTUATORS) == golden["shadow"]["actuators"]
    assert list(hands.ADROIT_JOINTS) == golden["adroit"]["joints"]
    assert list(hands.ADROIT_ACTUATORS) == golden["adroit"]["actuators"]
    # compiled scenes order joints/actuators exactly like the reference hand classes
    sj = [n.split("/")[-1] for n in reorient_compiled.names["joint"] if n.startswith("shadow_hand_e/")]
    assert sj == golden["shadow"]["joints"]
    sa = [n.split("/")[-1] for n in reorient_compiled.names["actuator"]]
    assert sa == golden["shadow"]["actuators"]
    aa = [n.split("/")[-1] for n in adroit_compiled.names["actuator"]]
    assert aa == golden["adroit"]["actuators"]


def test_control_joint_roundtrip():
    rng = np.random.RandomState(0)
    ctrl = rng.uniform(-1, 1, size=(7, 20))
    q = hands.shadow_control_to_joint_positions(ctrl)
    np.testing.assert_allclose(hands.shadow_joint_positions_to_control(q), ctrl, atol=1e-12)
    with pytest.raises(ValueError):
        hands.shadow_control_to_joint_positions(np.zeros(3))
    with pytest.raises(ValueError):
        hands.shadow_joint_positions_to_control(np.zeros(3))


def test_tanh_squared_matches_reference(golden):
    for row in golden["tanh_squared"]:
        assert task_ref.tanh_squared(row["x"], row["margin"]) == pytest.approx(row["value"], rel=1e-12, abs=1e-15)
    for row in golden["tanh_squared_vector"]:
        assert task_ref.tanh_squared(np.array(row["x"]), row["margin"]) == pytest.approx(row["value"], rel=1e-12)
    with pytest.raises(ValueError):
        task_ref.tanh_squared(0.1, margin=0.0)


def test_weighted_average_matches_reference(golden):
    g = golden["weighted_average"]
    assert task_ref.weighted_average(g["components"]) == pytest.approx(g["value"], rel=1e-15)


def test_reorient_reward_kat():
    """reorient_test.py:13-50: prop at the goal -> components exactly 10, 1, |ctrl|^2."""
    rng = np.random.RandomState(12345)
    goal = task_ref.uniform_quaternion(rng)
    ctrl = rng.uniform(-1, 1, size=20)
    d = task_ref.goal_distance(goal, goal)
    comps = task_ref.shaped_reorientation_reward(d, ctrl)
    assert comps["orientation"][0] == 1 / 0.1
    assert comps["success_bonus"][0] == 1.0
    assert comps["action_smoothing"][0] == np.linalg.norm(ctrl) ** 2


def test_goal_distance_properties():
    rng = np.random.RandomState(3)
    for _ in range(20):
        a = task_ref.uniform_quaternion(rng)
        b = task_ref.uniform_quaternion(rng)
        d = task_ref.goal_distance(a, b)
        assert 0 <= d <= np.pi + 1e-12
        assert d == pytest.approx(task_ref.goal_distance(a, -b))  # double cover
        assert task_ref.goal_distance(a, a) == pytest.approx(0.0, abs=1e-12)


def test_observation_set_matches_reference(golden):
    from dexterity_amd import manipulation

    g = golden["observations"]["hand_observables"]
    assert set(g["privileged_proprio"]) | set(g["proprio"]) == {
        "joint_velocities", "fingertip_positions", "fingertip_linear_velocities", "joint_positions_sin_cos"
    }
    opts = golden["observations"]["state_only_options"]
    assert all(o["enabled"] and o["update_interval"] == 1 for o in opts.values())
    layout = manipulation.observation_layout(24, 24, 5, True, "shadow_hand_e")
    sizes = {k: s.stop - s.start for k, s in layout.items()}
    # 24 + 15 + 15 + 48 (hand) + 13 (prop) + 4 (target) + 4 (goal) = 123
    assert sum(sizes.values()) == 123
    for name in g["privileged_proprio"] + g["proprio"]:
        assert f"shadow_hand_e/{name}" in layout


def test_action_spec_from_ctrlrange(reorient_compiled):
    from dexterity_amd import effectors

    spec = effectors.create_action_spec(reorient_compiled, list(range(20)), "shadow_hand_e_joint")
    assert spec.shape == (20,)
    assert np.all(np.isfinite(spec.minimum)) and np.all(np.isfinite(spec.maximum))
    # shadow_hand_position_actuators.xml:25-26
    assert spec.minimum[0] == pytest.approx(-0.488692) and spec.maximum[0] == pytest.approx(0.139626)
    names = spec.name.split("\t")
    assert names[0] == "shadow_hand_e_joint0" and len(names) == 20
    eff = effectors.HandEffector(list(range(20)), "shadow_hand_e")
    mask = effectors.find_effector_indices(eff, spec)
    assert all(mask)


def test_merge_specs():
    from dexterity_amd.specs import BoundedArray, merge_specs

    a = BoundedArray((2,), np.float32, [-1, -2], [1, 2], name="a0\ta1")
    b = BoundedArray((1,), np.float32, [0], [3], name="b0")
    m = merge_specs([a, b])
    assert m.shape == (3,)
    np.testing.assert_array_equal(m.minimum, [-1, -2, 0])
    assert m.name == "a0\ta1\tb0"


def test_reorient_config_constants():
    from dexterity_amd.manipulation import ReOrientConfig

    c = ReOrientConfig()
    assert c.n_sub_steps == 5  # reorient.py:58,61
    assert c.max_time_per_goal == pytest.approx(7.5)  # reorient.py:67-68


# --------------------------------------------------------------------------- #
# numpy-compatible resets
# --------------------------------------------------------------------------- #
def mt19937_doubles(seed: int, n: int) -> np.ndarray:
    """Plain restatement of numpy's legacy MT19937 (mt19937_seed / mt19937_gen /
    legacy_double): the algorithm dx_internal.h dx_mt_* runs on the device."""
    mt = [0] * 624
    s = seed & 0xFFFFFFFF
    for k in range(624):
        mt[k] = s
        s = (1812433253 * (s ^ (s >> 30)) + k + 1) & 0xFFFFFFFF
    pos = 624
    out = []

    def nxt():
        nonlocal pos
        if pos >= 624:
            for k in range(624):
                y = (mt[k] & 0x80000000) | (mt[(k + 1) % 624] & 0x7FFFFFFF)
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
            pos = 0
        y = mt[pos]
        pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        return y ^ (y >> 18)

    for _ in range(n):
        a, b = nxt() >> 5, nxt() >> 6
        out.append((a * 67108864.0 + b) / 9007199254740992.0)
    return np.array(out)


@pytest.mark.parametrize("seed", [0, 12345, 2**32 - 1])
def test_mt19937_restatement_matches_numpy(seed):
    np.testing.assert_array_equal(mt19937_doubles(seed, 1300), np.random.RandomState(seed).random_sample(1300))


def test_uniform_quaternion_draw_is_three_random_samples():
    """[3P] UniformQuaternion draws random_state.uniform([0]*3, [1, 2pi, 2pi]): three
    random_sample values scaled -- the form the device evaluates."""
    a = np.random.RandomState(5).uniform([0.0] * 3, [1.0, 2 * np.pi, 2 * np.pi])
    u = np.random.RandomState(5).random_sample(3)
    np.testing.assert_array_equal(a, u * [1.0, 2 * np.pi, 2 * np.pi])


def test_reorient_params_carry_the_fp64_box():
    from dexterity_amd.manipulation import ReOrient

    p = ReOrient().params()
    box = np.array((-0.025, -0.155, 0.16, 0.025, -0.105, 0.16))
    np.testing.assert_array_equal(p[26:38].view(np.float64), box)
    np.testing.assert_array_equal(p[16:22], box.astype(np.float32))


def test_prop_spawn_never_touches_the_hand(oracle_mod, reorient_compiled):
    """PropPlacer (reorient.py:143-151) redraws a pose that collides; the spawn box
    (z = 0.16, reorient.py:72-78) lies above the hand at qpos0, so the first attempt is
    always kept and every reset consumes exactly 6 draws of the env's stream.  Bound:
    the cube's lowest point (0.16 - 0.02 sqrt 3) is above every hand geom's bounding
    sphere; and no sampled spawn produces a contact with the prop."""
    from dexterity_amd import blob

    cm = reorient_compiled
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    prop = cm.names["body"].index("prop/")
    gb = np.asarray(cm.geom_bodyid)
    d = oracle_mod.OracleData(om)
    d.kinematics()
    gx, gm = d.geom_xpos.reshape(-1, 3), d.geom_xmat.reshape(-1, 3, 3)
    bs = np.asarray(cm.geom_bsphere, dtype=np.float64).reshape(-1, 4)  # local centre, radius
    hand = np.nonzero((gb > 0) & (gb < prop))[0]
    rc = 0.02 * np.sqrt(3)  # the cube's circumscribed radius
    lo, hi = np.array([-0.025, -0.155]), np.array([0.025, -0.105])
    top = -np.inf
    V = np.asarray(cm.mesh_vert, dtype=np.float64).reshape(-1, 3)
    for g in hand:  # hand geoms whose bounding sphere reaches over the spawn footprint
        c = gx[g] + gm[g] @ bs[g, :3]
        if np.linalg.norm(c[:2] - np.clip(c[:2], lo, hi)) >= bs[g, 3] + rc:
            continue
        if int(cm.geom_type[g]) == 7:  # mesh: its highest hull vertex
            m = int(cm.geom_dataid[g])
            v = V[cm.mesh_vertadr[m]: cm.mesh_vertadr[m] + cm.mesh_vertnum[m]]
            top = max(top, (gx[g] + v @ gm[g].T)[:, 2].max())
        else:
            top = max(top, c[2] + bs[g, 3])
    assert top < 0.16 - rc, top
    rs = np.random.RandomState(0)
    for _ in range(300):
        d = oracle_mod.OracleData(om)
        d.qpos[24:27] = rs.uniform([-0.025, -0.155, 0.16], [0.025, -0.105, 0.16])
        u1, u2, u3 = rs.uniform([0.0] * 3, [1.0, 2 * np.pi, 2 * np.pi])
        d.qpos[27:31] = [np.sqrt(1 - u1) * np.sin(u2), np.sqrt(1 - u1) * np.cos(u2), np.sqrt(u1) * np.sin(u3),
                         np.sqrt(u1) * np.cos(u3)]
        d.kinematics()
        assert not any(gb[int(c[13])] == prop or gb[int(c[14])] == prop for c in d.contacts())


def test_loader_constants():
    """loader_test.py:8-12 and manipulation/__init__.py:47-53."""
    from dexterity_amd import manipulation

    assert manipulation.ALL_TASKS and manipulation.ALL_NAMES and manipulation.TASKS_BY_DOMAIN
    assert ("reorient", "state_dense") in manipulation.ALL_TASKS
    assert manipulation.TASKS_BY_DOMAIN["reach"] == ("state_dense", "state_sparse")
    assert "reorient.state_dense" in manipulation.ALL_NAMES
    with pytest.raises(ValueError):
        manipulation.load("nope", "state_dense")
    with pytest.raises(ValueError):
        manipulation.load("reorient", "nope")
