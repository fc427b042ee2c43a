"""GPU (libdx.so, fp32) vs the fp64 CPU oracle on identical inputs.

Tolerances (fp32 kernel vs fp64 oracle, SURVEY.md §8 c4 proposal):
  * mass matrix: relative 1e-5 of max|M|;
  * qacc_smooth: 1e-5 of the forcing scale max|qacc_smooth|;
  * contacts: identical geom-pair sets; |dist| 2e-5 m, |pos| 2e-4 m, normal max(2e-3, 1e-7/|dist|);
  * constrained qacc after the Newton solve: 5e-4 of max(1, |qacc_smooth|) (soft
    contacts are stiff; both iterate to the model's tolerance 1e-8, the kernel in
    fp32, so its Newton stops at fp32 resolution of the cost);
  * one substep: qpos 1e-6 rad/m absolute;
  * contact-free trajectory, 10 control steps: qpos 1e-4 rad;
  * determinism: bit-identical outputs for identical inputs.
"""

import os

import numpy as np
import pytest

from dexterity_amd import _lib, blob
from dexterity_amd.mjcf.compiler import CompiledModel
from tests.conftest import ROOT, random_hand_state

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    from dexterity_amd import build, physics

    build.build()
    return physics


def _f32(st):
    """A state as the GPU holds it: every array rounded to fp32, widened back."""
    return tuple(np.asarray(x, dtype=np.float32).astype(np.float64) for x in st)


def _oracle_states(oracle_mod, cm, xfrc, n_traj=3, seed=0):
    """States along oracle trajectories: cube dropped on the palm, random servo targets."""
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    rng = np.random.RandomState(seed)
    states = []
    lo, hi = cm.actuator_ctrlrange.T
    for t in range(n_traj):
        d = oracle_mod.OracleData(om)
        d.xfrc_applied[:] = xfrc.ravel()
        d.qpos[24:27] += rng.uniform(-0.02, 0.02, size=3) * [1, 1, 0]
        ctrl = rng.uniform(lo, hi) * 0.3
        for s in range(120):
            d.ctrl[:] = ctrl
            d.step()
            if s in (45, 80, 119):
                states.append((d.qpos.copy(), d.qvel.copy(), d.qacc_warmstart.copy(), ctrl.copy()))
    # contact-free: hand in random poses, cube far away
    for _ in range(3):
        qpos, qvel = random_hand_state(cm, rng)
        qpos[24:27] = [0.3, 0.3, 0.5]
        states.append((qpos, qvel, np.zeros(cm.nv), rng.uniform(lo, hi)))
    return om, states


def _oracle_forward(oracle_mod, om, cm, xfrc, st):
    d = oracle_mod.OracleData(om)
    d.xfrc_applied[:] = xfrc.ravel()
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = st
    d.forward()
    return d


def _oracle_pair(oracle_mod, om, cm, xfrc, st):
    """The oracle's forward pass at the fp64 state and at the state the GPU holds
    (`_f32`).  MPR's contact normal and depth are not continuous functions of the
    state: over the wide sample, three fp64 contacts move under the fp32 rounding of
    the state alone (a 2.9 mm hand-hand penetration by 4.7e-5 m and 0.13 rad, cube
    contacts by 2.2e-2 and 0.42 rad).  A GPU result that matches either pass is the
    reference algorithm's answer within the fp32 resolution of its input."""
    return (_oracle_forward(oracle_mod, om, cm, xfrc, st),
            _oracle_forward(oracle_mod, om, cm, np.asarray(xfrc, dtype=np.float32).astype(np.float64), _f32(st)))


@pytest.fixture(scope="module")
def reorient_setup(gpu, oracle_mod):
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    xfrc = gpu.gravity_compensation(cm, "shadow_hand_e/")
    om, states = _oracle_states(oracle_mod, cm, xfrc)
    model = gpu.Model(cm)
    return cm, xfrc, om, states, model


def _qacc_on_gpu_contacts(oracle_mod, om, xfrc, st, recs):
    """The oracle's constrained qacc at the state the GPU holds (`_f32`) with the GPU's
    contact list `recs` in place of its own narrowphase (dxo_set_contacts): what a tie
    state's accelerations must equal if the tie (MPR's choice of point or normal) is the
    whole difference."""
    d = oracle_mod.OracleData(om)
    d.xfrc_applied[:] = np.asarray(xfrc, dtype=np.float32).astype(np.float64).ravel()
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = _f32(st)
    d.set_contacts(np.asarray(recs, dtype=np.float64))
    d.forward()
    return d.qacc.copy()


def _geom_points(cm, d, g):
    """World-frame vertices of a box or mesh geom (a mesh collides as the convex hull of
    its vertices) at the oracle state d."""
    gx = d.geom_xpos.reshape(-1, 3)[g]
    gm = d.geom_xmat.reshape(-1, 3, 3)[g]
    t = int(cm.geom_type[g])
    if t == 7:
        m = int(cm.geom_dataid[g])
        a, n = int(cm.mesh_vertadr[m]), int(cm.mesh_vertnum[m])
        v = np.asarray(cm.mesh_vert, dtype=np.float64).reshape(-1, 3)[a:a + n]
    elif t == 6:
        h = np.asarray(cm.geom_size, dtype=np.float64).reshape(-1, 3)[g]
        v = np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]) * h
    else:
        raise NotImplementedError(f"geom type {t}")
    return gx + v @ gm.T


def _separation(cm, d, g1, g2, n):
    """Signed distance of geom2 from geom1 along the unit normal n (geom1 -> geom2), in
    fp64: min over geom2 of w.n - max over geom1 of v.n.  For the normal of a converged
    MPR portal this is the contact's dist (the portal is a face of the Minkowski
    difference); any other direction gives less."""
    n = np.asarray(n, dtype=np.float64)
    n = n / np.linalg.norm(n)
    return (_geom_points(cm, d, g2) @ n).min() - (_geom_points(cm, d, g1) @ n).max()


def _load_states(gpu, model, xfrc, states):
    phys = gpu.BatchedPhysics(model, len(states))
    phys.set_xfrc(xfrc)
    phys.set(_lib.QPOS, np.stack([s[0] for s in states]))
    phys.set(_lib.QVEL, np.stack([s[1] for s in states]))
    phys.set(_lib.QACC_WARMSTART, np.stack([s[2] for s in states]))
    phys.set(_lib.CTRL, np.stack([s[3] for s in states]))
    return phys


def _normal_tol(dist):
    """Normal tolerance of a contact at depth |dist| (see _contact_tie), capped at 0.05 rad
    so a very shallow contact cannot excuse an arbitrary normal."""
    return min(0.05, max(2e-3, 1e-7 / max(abs(dist), 1e-12)))


def _contact_match(r, o):
    return (abs(r[12] - o[12]) < 2e-5 and np.abs(r[0:3] - o[0:3]).max() < 2e-4
            and np.abs(r[3:6] - o[3:6]).max() < _normal_tol(o[12]))


def _contact_tie(cm, ds, r):
    """Compare one GPU contact record r with the oracle passes ds (`_oracle_pair`) for
    the same geom pair.  Returns False when r matches either pass within the
    tolerances below.  Otherwise r is a tie -- a contact whose point or normal fp32
    and fp64 MPR legitimately resolve differently -- checked against the fp64 pass for
    what a tie must still satisfy, and True is returned; the state's accelerations are
    then not compared tightly.

    * depth: 2e-5 m always;
    * normal: the direction of a vector of length |dist| built from world coordinates
      of ~0.2 m (fp32 ulp 1.5e-8 m); after the hull transform and the portal cross
      products the points carry a few ulp, so it is good to max(2e-3, 1e-7/|dist|) rad;
    * point: 2e-4 m.
    Ties:
    * flat-on-flat pairs (cube face on a palm facet): the contact point is any point
      of the shared face, picked by support ties.  It must stay on the face: the
      displacement is orthogonal to the normal within 2e-4 m, and at most 5 cm;
    * portal ties: the fp32 portal stops on a neighbouring Minkowski face.  The
      normal is still within 0.05 rad, and the geoms' fp64 separation along the GPU
      normal is within 5e-4 m of the contact's depth (`_separation`: an exact face
      normal gives the depth itself)."""
    key = (int(r[13]), int(r[14]))
    os_ = [{(int(c[13]), int(c[14])): c for c in d.contacts()}.get(key) for d in ds]
    assert os_[0] is not None or os_[1] is not None, key
    if any(o is not None and _contact_match(r, o) for o in os_):
        return False
    d, o = (ds[0], os_[0]) if os_[0] is not None else (ds[1], os_[1])
    assert abs(r[12] - o[12]) < 2e-5
    tie = False
    nerr = np.abs(r[3:6] - o[3:6]).max()
    if nerr >= _normal_tol(o[12]):
        assert nerr < 0.05
        assert _separation(cm, d, int(o[13]), int(o[14]), r[3:6]) - o[12] > -5e-4
        tie = True
    delta = r[0:3] - o[0:3]
    if np.abs(delta).max() >= 2e-4:
        assert abs(np.dot(delta, o[3:6])) < 2e-4
        assert np.linalg.norm(delta) < 0.05
        tie = True
    return tie


def _check_forward(gpu, oracle_mod, cm, xfrc, om, states, model):
    phys = _load_states(gpu, model, xfrc, states)
    phys.debug(True)
    phys.forward()
    phys.sync()
    M = phys.debug_get("M")
    a0 = phys.debug_get("qacc_smooth")
    con = phys.debug_get("contact")
    cnt = phys.debug_get("efc_count")
    qacc = phys.qacc
    ncontact_states = 0
    degenerate = 0
    for e, st in enumerate(states):
        ds = _oracle_pair(oracle_mod, om, cm, xfrc, st)
        d = ds[0]
        Mo = d.M.reshape(cm.nv, cm.nv)
        assert np.abs(M[e] - Mo).max() <= 1e-5 * np.abs(Mo).max()
        scale = np.abs(d.qacc_smooth).max()
        assert np.abs(a0[e] - d.qacc_smooth).max() <= 1e-5 * scale
        oc = d.contacts()
        n = cnt[e, 0]
        gc = con[e, : (con[e, :, 15] != 0).sum()]
        assert cnt[e, 1] == 0, "overflow flag set"
        assert len(gc) == len(oc)
        ok = {(int(r[13]), int(r[14])): r for r in oc}
        ties = 0
        for r in gc:
            assert (int(r[13]), int(r[14])) in ok
            ties += _contact_tie(cm, ds, r)
        assert ties <= 2
        degenerate += ties > 0
        assert n == d.nefc
        ncontact_states += len(oc) > 0
        # qacc from one oracle pass (either side of an MPR discontinuity, _oracle_pair)
        err = min((np.abs(qacc[e] - dd.qacc) for dd in ds), key=lambda x: x.max())
        sc = max(1.0, scale)
        if ties == 0:
            # the cube's own six dofs get the bimanual test's 3e-3: a shallow contact's
            # normal carries the fp32 error of _contact_tie (5e-3 rad at 11 um), which
            # tilts that contact's force and the cube's angular acceleration with it
            assert err[: cm.nv - 6].max() <= 5e-4 * sc, f"env {e}"
            assert err[cm.nv - 6 :].max() <= 3e-3 * sc, f"env {e}"
        else:
            # a tied contact sits elsewhere on the shared face (or on a neighbouring
            # Minkowski face): its force acts at another point, so the accelerations are
            # held to a looser bound instead of being skipped
            TIE_ERR.append(float(err.max() / sc))
            assert err[: cm.nv - 6].max() <= TIE_QACC_HAND * sc, (f"tie env {e}", err.max() / sc)
            assert err[cm.nv - 6 :].max() <= TIE_QACC_CUBE * sc, (f"tie env {e}", err.max() / sc)
            # and the tie is the whole difference: on the GPU's own contacts the oracle's
            # accelerations equal the GPU's within the tight bound
            fix = np.abs(qacc[e] - _qacc_on_gpu_contacts(oracle_mod, om, xfrc, st, gc))
            assert fix.max() <= 5e-4 * sc, (f"tie env {e} on the GPU's contacts", fix.max() / sc)
    return ncontact_states, degenerate


# Tie states (_contact_tie): qacc within these fractions of max(1, |qacc_smooth|) --
# hand dofs / cube dofs -- and one-substep qpos within TIE_QPOS.  Their errors are
# recorded here and printed by the wide-sample test.
# Measured (r3, test_forward_and_substep_parity_wide_sample's output): one tie state in
# 63, its qacc error 1.3e-3 of the scale, its one-step errors qpos 3e-7 / qvel 6e-6.
TIE_QACC_HAND, TIE_QACC_CUBE, TIE_QPOS = 5e-3, 2e-2, 1e-5
TIE_ERR, TIE_STEP_ERR = [], []
# states with a tie, at most, over the wide sample of 63 states (measured: 1)
WIDE_TIES_MAX = 3


def test_forward_parity_reorient(gpu, oracle_mod, reorient_setup):
    cm, xfrc, om, states, model = reorient_setup
    ncontact_states, degenerate = _check_forward(gpu, oracle_mod, cm, xfrc, om, states, model)
    assert ncontact_states >= 6
    assert degenerate <= 2


def _check_substep(gpu, oracle_mod, cm, xfrc, om, states, model):
    # states with a contact tie (_contact_tie) get the looser tie bound in the one-step
    # comparison
    probe = _load_states(gpu, model, xfrc, states)
    probe.debug(True)
    probe.forward()
    con = probe.debug_get("contact")
    skip = set()
    for e, st in enumerate(states):
        ds = _oracle_pair(oracle_mod, om, cm, xfrc, st)
        for r in con[e, : (con[e, :, 15] != 0).sum()]:
            if _contact_tie(cm, ds, r):
                skip.add(e)
    probe.close()
    phys = _load_states(gpu, model, xfrc, states)
    phys.step(1)
    qpos, qvel = phys.qpos, phys.qvel
    for e, st in enumerate(states):
        errs = []
        for x, y in ((xfrc, st), (np.asarray(xfrc, dtype=np.float32).astype(np.float64), _f32(st))):
            d = oracle_mod.OracleData(om)
            d.xfrc_applied[:] = x.ravel()
            d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = y
            d.step()
            errs.append((np.abs(qpos[e] - d.qpos).max(),
                         np.abs(qvel[e] - d.qvel).max() / max(1.0, np.abs(d.qacc_smooth).max())))
        # either side of an MPR discontinuity (_oracle_pair), qpos and qvel from the same
        # pass: qpos 1e-6, qvel 5e-4 of the scale (a tie state: the looser tie bounds)
        qt, vt = (TIE_QPOS, TIE_QACC_CUBE) if e in skip else (1e-6, 5e-4)
        if e in skip:
            TIE_STEP_ERR.append(min(errs, key=lambda qv: qv[0]))
            # on the GPU's own contacts the oracle's step equals the GPU's tightly
            d = oracle_mod.OracleData(om)
            d.xfrc_applied[:] = np.asarray(xfrc, dtype=np.float32).astype(np.float64).ravel()
            d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = _f32(st)
            d.set_contacts(con[e, : (con[e, :, 15] != 0).sum()].astype(np.float64))
            d.step()
            assert np.abs(qpos[e] - d.qpos).max() < 1e-6, (e, "on the GPU's contacts")
        assert any(q < qt and v < vt for q, v in errs), (e, e in skip, errs)
    return skip


def test_single_substep_parity(gpu, oracle_mod, reorient_setup):
    skip = _check_substep(gpu, oracle_mod, *reorient_setup)
    assert len(skip) <= 2


def test_forward_and_substep_parity_wide_sample(gpu, oracle_mod, reorient_setup):
    """The same two checks over 20 oracle trajectories (60 contact-rich states plus 3
    contact-free ones), with the flat-on-flat face-tie allowance scaled to the sample:
    at most 1 in 6 states may place a contact point elsewhere on the tied face."""
    cm, xfrc, _, _, model = reorient_setup
    om, states = _oracle_states(oracle_mod, cm, xfrc, n_traj=20, seed=7)
    ncontact_states, degenerate = _check_forward(gpu, oracle_mod, cm, xfrc, om, states, model)
    assert ncontact_states >= 40
    skip = _check_substep(gpu, oracle_mod, cm, xfrc, om, states, model)
    print(f"tie states: forward {degenerate} / substep {len(skip)} of {len(states)}; "
          f"tie qacc errors (of scale) {sorted(round(x, 5) for x in TIE_ERR)}; "
          f"tie one-step (qpos, qvel) errors {[(float(f'{q:.2e}'), float(f'{v:.2e}')) for q, v in TIE_STEP_ERR]}")
    assert degenerate <= WIDE_TIES_MAX and len(skip) <= WIDE_TIES_MAX


def test_contact_free_trajectory_parity(gpu, oracle_mod):
    """Config 2 (reach, Shadow hand, contact-free): 10 control steps, qpos <= 1e-4 rad."""
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reach.npz"))
    xfrc = gpu.gravity_compensation(cm, "shadow_hand_e/")
    model = gpu.Model(cm)
    om = oracle_mod.OracleModel(model.blob)
    rng = np.random.RandomState(12345)
    B = 8
    q0 = []
    for _ in range(B):
        q, _ = random_hand_state(cm, rng)
        q0.append(q)
    q0 = np.stack(q0)
    lo, hi = cm.actuator_ctrlrange.T
    ctrls = rng.uniform(lo, hi, size=(10, B, cm.nu))
    phys = gpu.BatchedPhysics(model, B)
    phys.set_xfrc(xfrc)
    phys.set(_lib.QPOS, q0)
    ds = []
    for e in range(B):
        d = oracle_mod.OracleData(om)
        d.xfrc_applied[:] = xfrc.ravel()
        d.qpos[:] = q0[e]
        ds.append(d)
    for t in range(10):
        phys.set(_lib.CTRL, ctrls[t])
        phys.step(1)
        for e in range(B):
            ds[e].ctrl[:] = ctrls[t, e]
            ds[e].step()
    qpos = phys.qpos
    for e in range(B):
        assert np.abs(qpos[e] - ds[e].qpos).max() < 1e-4


def test_adroit_forward_parity(gpu, oracle_mod):
    """Adroit: 44 limited fixed tendons (coupling rows) + capsule pairs (condim 1)."""
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "adroit_reach.npz"))
    xfrc = gpu.gravity_compensation(cm, "adroit_hand/")
    model = gpu.Model(cm)
    om = oracle_mod.OracleModel(model.blob)
    rng = np.random.RandomState(9)
    states = []
    lo, hi = cm.actuator_ctrlrange.T
    for _ in range(6):
        q, v = random_hand_state(cm, rng, frac=1.0)
        states.append((q, v, np.zeros(cm.nv), rng.uniform(lo, hi)))
    phys = _load_states(gpu, model, xfrc, states)
    phys.debug(True)
    phys.forward()
    qacc = phys.qacc
    cnt = phys.debug_get("efc_count")
    for e, st in enumerate(states):
        d = _oracle_forward(oracle_mod, om, cm, xfrc, st)
        assert cnt[e, 0] == d.nefc
        scale = np.abs(d.qacc_smooth).max()
        assert np.abs(qacc[e] - d.qacc).max() <= 5e-4 * max(1.0, scale)


def _tendon_limit_rows(cm, q):
    """Active tendon-limit rows at qpos q ([3P] mj_instantiateLimit: a limited fixed
    tendon whose length is within its margin of either end of its range)."""
    n = 0
    for t in range(int(cm.ntendon)):
        if not cm.tendon_limited[t]:
            continue
        a, k = int(cm.tendon_adr[t]), int(cm.tendon_num[t])
        length = sum(float(cm.wrap_coef[w]) * q[int(cm.jnt_qposadr[int(cm.dof_jntid[int(cm.wrap_dof[w])])])]
                     for w in range(a, a + k))
        lo, hi = cm.tendon_range[t]
        m = float(cm.tendon_margin[t])
        n += int(length - lo < m) + int(hi - length < m)
    return n


def test_adroit_incremental_newton_parity(gpu, oracle_mod):
    """The incremental-Hessian Newton path on a model with limited tendons (Adroit, 44
    coupling tendons): the kernel takes it whenever a solve has no tendon-limit row
    (dx_step.hip solve: `limt`), so states with none are chosen on the host -- which pins
    the path taken -- and qacc and one substep are held to the tight bounds against the
    oracle (qacc 5e-4 of the scale, qpos 1e-6)."""
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "adroit_reach.npz"))
    xfrc = gpu.gravity_compensation(cm, "adroit_hand/")
    model = gpu.Model(cm)
    om = oracle_mod.OracleModel(model.blob)
    rng = np.random.RandomState(21)
    lo, hi = cm.actuator_ctrlrange.T
    states = []
    while len(states) < 8:
        # (near qpos0: the coupling tendons' ranges are +-0.032, so a wide sample always
        # activates some; this one has friction-loss, joint-limit and contact rows)
        q, v = random_hand_state(cm, rng, frac=0.1)
        if _tendon_limit_rows(cm, q) == 0:
            states.append((q, v, np.zeros(cm.nv), rng.uniform(lo, hi)))
    phys = _load_states(gpu, model, xfrc, states)
    phys.debug(True)
    phys.forward()
    qacc = phys.qacc
    cnt = phys.debug_get("efc_count")
    phys.close()
    nrows = 0
    for e, st in enumerate(states):
        d = _oracle_forward(oracle_mod, om, cm, xfrc, st)
        assert cnt[e, 0] == d.nefc
        nrows += d.nefc
        scale = max(1.0, np.abs(d.qacc_smooth).max())
        assert np.abs(qacc[e] - d.qacc).max() <= 5e-4 * scale, e
    assert nrows > 0  # (constraint rows other than tendon limits: friction loss, joint limits)
    phys = _load_states(gpu, model, xfrc, states)
    phys.step(1)
    qpos = phys.qpos
    phys.close()
    for e, st in enumerate(states):
        d = oracle_mod.OracleData(om)
        d.xfrc_applied[:] = np.asarray(xfrc).ravel()
        d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = st
        d.step()
        assert np.abs(qpos[e] - d.qpos).max() <= 1e-6, e


def test_deterministic_replay(gpu, reorient_setup):
    cm, xfrc, om, states, model = reorient_setup
    outs = []
    for _ in range(2):
        phys = _load_states(gpu, model, xfrc, states)
        phys.step(5)
        outs.append((phys.qpos, phys.qvel, phys.get(_lib.SITE_XPOS)))
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_independent_of_stale_lds(gpu, reorient_setup):
    """Results must not depend on LDS contents left by earlier workgroups: a run
    after every CU's LDS was filled with NaN patterns is bit-identical."""
    cm, xfrc, om, states, model = reorient_setup
    L = _lib.load()
    outs = []
    for poison in (False, True):
        phys = _load_states(gpu, model, xfrc, states)
        if poison:
            _lib.check(L.dx_debug_poison_lds(0))
        phys.step(5)
        q = phys.qpos
        assert np.all(np.isfinite(q))
        outs.append((q, phys.qvel, phys.get(_lib.NITER)))
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_env_step_rewards_match_host_restatement(gpu):
    from dexterity_amd import manipulation
    from oracle import task_ref

    env = manipulation.load("reorient", "state_dense", seed=12345, num_envs=64)
    ts = env.reset()
    assert np.all(ts.first())
    spec = env.action_spec()
    rng = np.random.RandomState(12345)
    for step in range(12):
        action = rng.uniform(spec.minimum, spec.maximum, size=(64, spec.shape[0])).astype(np.float32)
        ts = env.step(action)
        obs = ts.observation
        for e in range(64):
            if ts.step_type[e] == 0:
                assert ts.reward[e] == 0 and ts.discount[e] == 1
                continue
            d = task_ref.goal_distance(obs["goal_state"][e], obs["prop/orientation"][e])
            r = task_ref.reorient_reward(d, action[e])
            assert ts.reward[e] == pytest.approx(r, rel=2e-4, abs=2e-3)
            assert ts.discount[e] in (0.0, 1.0)
        for k, v in obs.items():
            assert np.all(np.isfinite(v)), k
    # observation spec coherent with the data (manipulation_test.py:48-55)
    for name, spec_ in env.observation_spec().items():
        assert ts.observation[name].shape[1:] == spec_.shape
    env.close()


def test_success_kat_on_gpu(gpu):
    """reorient_test.py:13-50 on the device: prop placed at the goal -> success."""
    from dexterity_amd import manipulation

    env = manipulation.load("reorient", "state_dense", seed=7, num_envs=16)
    env.reset()
    goals = env.goals()
    qpos = env.physics.qpos
    qpos[:, 27:31] = goals
    env.physics.set(_lib.QPOS, qpos)
    env.physics.set(_lib.QVEL, np.zeros((16, env.model.nv)))
    ts = env.step(np.zeros((16, env.model.nu), np.float32))
    d = np.array([2 * np.arccos(min(1.0, abs(float(np.dot(g, q))))) for g, q in
                  zip(goals, ts.observation["prop/orientation"])])
    assert np.all(d < 0.1)
    np.testing.assert_allclose(ts.reward, 1 / (d + 0.1) + 800.0, rtol=1e-4)
    assert np.all(ts.last()) and np.all(ts.discount == 0.0)
    assert np.all(env.successes() == 1)
    env.close()


def _nearest_perturbed(oracle_mod, om, xfrc32, st, nsub, gq, gv, scale, k=32, rel=6e-8, seed=0):
    """The GPU's result (gq, gv) against the nearest of k oracle runs from the state
    perturbed at fp32 resolution (relative `rel` on qpos and qvel; run 0 unperturbed):
    (qpos err, qvel err / scale).  MPR is discontinuous at deep or flat contacts -- the
    fp64 oracle's own contact normal jumps by up to 0.16 rad under 6e-8 relative input
    perturbations in 4 of 60 deep-contact states (round 4) -- so a GPU result equal to one
    of these runs is the reference algorithm's answer for an input within the fp32
    rounding of the GPU's (the generalisation of _oracle_pair)."""
    rng = np.random.RandomState(seed)
    q, v, w, c = (np.asarray(x, dtype=np.float64) for x in st)
    Q = np.tile(q, (k, 1))
    V = np.tile(v, (k, 1))
    Q[1:] *= 1 + rng.standard_normal(Q[1:].shape) * rel
    V[1:] *= 1 + rng.standard_normal(V[1:].shape) * rel
    rc, oq, ov, _ = oracle_mod.batch_step(om, Q, V, np.tile(c, (k, 1)), np.tile(w, (k, 1)), xfrc32, nsub=nsub)
    assert rc == 0
    eq = np.abs(oq - gq).max(axis=1)
    ev = np.abs(ov - gv).max(axis=1) / scale
    i = int(np.argmin(eq + 1e-3 * ev))
    return eq[i], ev[i]


def _min_penetration(cm, d, g1, g2, starts):
    """The geoms' minimum penetration depth in fp64 (the largest separation over directions,
    negative when they overlap), by a local search from the given normals: the quantity
    MPR approximates with the portal it stops on."""
    from scipy.optimize import minimize

    best = -np.inf
    for n0 in starts:
        n0 = np.asarray(n0, dtype=np.float64)
        r = minimize(lambda v: -_separation(cm, d, g1, g2, v / max(np.linalg.norm(v), 1e-12)), n0,
                     method="Nelder-Mead", options={"xatol": 1e-7, "fatol": 1e-9, "maxiter": 2000})
        best = max(best, -r.fun, _separation(cm, d, g1, g2, n0))
    return best


def _contact_lists_agree(d, recs, cm=None, deep=None, divergent=False):
    """The GPU's contact records `recs` against the oracle's contacts at the same state
    (d after forward): the same geom pairs with the same multiplicity, except contacts
    within the depth tolerance of existing (|dist| < 2e-5 m, on either side); for each
    record (paired with the same pair's oracle contact nearest to it) the depth within
    max(2e-5 m, 3 % of the depth), the normal within 0.1 rad, the point within 2e-4 m or
    displaced along the contact face (orthogonal to the normal within 2e-4 m, at most
    5 cm).  MPR reports the direction to the closest point of its final portal; which
    portal fp32 and fp64 end on can differ while both satisfy its stopping test, so the
    normal of a shallow or rounded contact is not pinned tighter than this.  Returns
    (None or the first disagreement, tie contacts).

    Deep mesh-mesh contacts (|dist| > 0.1 mm; `cm` and the list `deep` given): MPR stops
    on a portal within its tolerance of the Minkowski boundary, and for a deep overlap of
    two rounded hulls fp32 and fp64 can stop on different portals, either closer to the
    true minimum penetration.  Such a contact is accepted, and appended to `deep`, when its
    depth is within 3 % of the geoms' minimum penetration depth (_min_penetration, fp64),
    i.e. when it is as good an answer as MPR gives -- or when its portal lies on the
    Minkowski boundary: the fp64 separation of the two hulls along the GPU's own normal
    equals the GPU's depth (within max(2e-5 m, 3 %)), i.e. the GPU's (normal, depth) is
    an exact support-based answer, a terminal portal of MPR from another start (deep
    finger-finger overlaps of the two-hand scene, where MPR's answer is discontinuous).

    `divergent` (the last resort of _account_full_batch): a deep hull-hull or box-hull
    contact (|dist| > 0.5 mm) whose (normal, depth) is the reference algorithm's answer in
    fp32 -- the
    oracle's MPR restated with the arithmetic type as a parameter (oracle/mpr_ref.py),
    evaluated in fp32 from the geoms' poses perturbed at the fp32 forward kinematics'
    resolution, reproduces the GPU's contact to 1e-4 rad and 1e-4 of the depth
    (fp32_reproduces) -- also passes: at a deep overlap of two curved hulls fp32 and fp64
    MPR stop on different portals (another normal, a depth 4-11 % apart), and the fp32
    one is what the kernel computes.  Appended to `deep` with rule "fp32 portal".  Round 6
    replaced round 5's window (any normal, depth within 15 %) by this reproduction; the
    states that needed it are committed fixtures (tests/golden/fullbatch_*_fp32_portal.npz,
    tests/test_mpr_precision.py)."""
    oc = d.contacts()
    ties = 0

    def deep_ok(r, o):
        if cm is None or deep is None or abs(o[12]) <= 1e-4:
            return False
        g1, g2 = int(o[13]), int(o[14])
        t1, t2 = int(cm.geom_type[g1]), int(cm.geom_type[g2])
        if t1 not in (6, 7) or t2 not in (6, 7):
            return False
        if t1 != 7 or t2 != 7:  # a box against a hull: the fp32 portal rule alone
            return fp32_portal(r, o, g1, g2)
        pen = _min_penetration(cm, d, g1, g2, (r[3:6], o[3:6]))
        if abs(r[12] - pen) <= 0.03 * abs(pen):
            deep.append((int(o[13]), int(o[14]), float(r[12]), float(o[12]), float(pen), "min"))
            return True
        sep = _separation(cm, d, g1, g2, r[3:6])
        if abs(sep - r[12]) <= max(2e-5, 0.03 * abs(r[12])):
            deep.append((int(o[13]), int(o[14]), float(r[12]), float(o[12]), float(sep), "boundary"))
            return True
        return fp32_portal(r, o, g1, g2)

    def fp32_portal(r, o, g1, g2):
        if divergent and abs(o[12]) > 5e-4:
            from oracle.mpr_ref import fp32_reproduces

            ok, ang, dr, _ = fp32_reproduces(cm, d, g1, g2, r)
            if ok:
                deep.append((g1, g2, float(r[12]), float(o[12]), float(ang), "fp32 portal"))
                return True
        return False

    used = np.zeros(len(oc), dtype=bool)
    for r in recs:
        idx = np.flatnonzero((oc[:, 13] == r[13]) & (oc[:, 14] == r[14]) & ~used)
        if len(idx) == 0:
            if abs(r[12]) < 2e-5:
                continue
            return f"GPU contact {r[13]:.0f}-{r[14]:.0f} dist {r[12]:.2e} not in the oracle's list", ties
        i = idx[np.argmin(np.abs(oc[idx, 0:3] - r[0:3]).max(axis=1))]
        used[i] = True
        o = oc[i]
        if abs(r[12] - o[12]) > max(2e-5, 0.03 * abs(o[12])):
            if deep_ok(r, o):
                continue
            return f"contact {r[13]:.0f}-{r[14]:.0f} dist {r[12]:.3e} vs {o[12]:.3e}", ties
        if _contact_match(r, o):
            continue
        ties += 1
        nerr = np.abs(r[3:6] - o[3:6]).max()
        if nerr > max(0.1, 1e-6 / max(abs(o[12]), 1e-12)):
            if deep_ok(r, o):
                continue
            return f"contact {r[13]:.0f}-{r[14]:.0f} (dist {o[12]:.2e}) normal off by {nerr:.3f}", ties
        delta = r[0:3] - o[0:3]
        if np.abs(delta).max() >= 2e-4 and (abs(np.dot(delta, o[3:6])) >= 2e-4 or np.linalg.norm(delta) >= 0.05):
            return f"contact {r[13]:.0f}-{r[14]:.0f} point off by {delta}", ties
    for o in oc[~used]:
        if abs(o[12]) >= 2e-5:
            return f"oracle contact {o[13]:.0f}-{o[14]:.0f} dist {o[12]:.2e} not in the GPU's list", ties
    return None, ties


def _oracle_on_contacts(oracle_mod, om, x32, st, recs, gqacc):
    """The oracle's step from state st with the GPU's contact list `recs` in place of its
    narrowphase: (qpos, qvel, relative cost excess of the GPU's qacc in that constraint
    problem, i.e. (f(qacc_gpu) - f(qacc_oracle)) / |f(qacc_oracle)|)."""
    d = oracle_mod.OracleData(om)
    d.xfrc_applied[:] = x32
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = (np.asarray(x, dtype=np.float64) for x in st)
    d.set_contacts(recs)
    d.forward()
    oa = d.qacc.copy()
    c0 = d.solver_cost(oa)
    excess = (d.solver_cost(gqacc) - c0) / max(abs(c0), 1e-30)
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = (np.asarray(x, dtype=np.float64) for x in st)
    d.step()
    return d.qpos.copy(), d.qvel.copy(), excess


def _account_full_batch(oracle_mod, om, compiled, x32, h, states, gpu_out, label, solver="Newton"):
    """The full-batch accounting of test_full_batch_parity: every env's GPU step (gq, gv)
    against the oracle's from the same fp32 state (oq, ov); a state outside the tight bound
    (qpos 1e-6, qvel 5e-4 of the scale) must be explained as an MPR discontinuity, contact
    geometry or solver resolution.  Returns (tight mask, category counts, tie contacts,
    deep mesh-mesh contacts, unexplained states)."""
    qpos, qvel, ws, ctrl = states
    gq, gv, gqacc, con, scale, oq, ov = gpu_out
    eq = np.abs(gq - oq).max(axis=1)
    ev = np.abs(gv - ov).max(axis=1) / scale
    tight = (eq <= 1e-6) & (ev <= 5e-4)
    kinds = {"perturbed": 0, "geometry": 0, "solver": 0, "divergent": 0}
    ties = 0
    deep = []  # deep mesh-mesh contacts judged on geometry (_contact_lists_agree)
    unexplained = []
    divergent = []  # states of the "divergent" rule, dumped for a CPU-side fixture
    # a CG / PGS step stops short of the optimum (100 iterations / sweeps), where fp32 and
    # fp64 walk the same iteration apart: their "equal" is the solver bound
    tq, tv = (1e-6, 5e-4) if solver == "Newton" else (FULL_SOLVER_QPOS, FULL_SOLVER_QVEL)
    for e in np.flatnonzero(~tight):
        st = (qpos[e], qvel[e], ws[e], ctrl[e])
        if solver != "Newton" and eq[e] <= tq and ev[e] <= tv:
            kinds["solver"] += 1  # the oracle's same solver from the same state and warm start
            continue
        pq, pv = _nearest_perturbed(oracle_mod, om, x32, st, 1, gq[e], gv[e], scale[e])
        if pq <= tq and pv <= tv:
            kinds["perturbed"] += 1
            continue
        recs = con[e][con[e][:, 15] != 0]
        cq, cv, excess = _oracle_on_contacts(oracle_mod, om, x32, st, recs, gqacc[e])
        sq, sv = np.abs(cq - gq[e]).max(), np.abs(cv - gv[e]).max() / scale[e]
        # the oracle's contacts at the state, else at one of its perturbations at fp32
        # resolution -- of the input (6e-8) and of the fp32 forward kinematics that places
        # the geoms (1e-6: seven-level chains of fp32 transforms) -- since MPR's path, and
        # so its normal and depth, is discontinuous in the input
        rng = np.random.RandomState(int(e))
        for p in range(33):
            rel = 6e-8 if p <= 16 else 1e-6
            pst = st if p == 0 else (qpos[e] * (1 + rng.standard_normal(qpos.shape[1]) * rel),
                                     qvel[e] * (1 + rng.standard_normal(qvel.shape[1]) * rel), ws[e], ctrl[e])
            why, t = _contact_lists_agree(_oracle_forward(oracle_mod, om, None, x32, pst), recs)
            if why is None:
                break
        if why is not None:  # at the state itself, with deep mesh-mesh contacts judged on geometry
            dp = []
            why, t = _contact_lists_agree(_oracle_forward(oracle_mod, om, None, x32, st), recs, compiled, dp)
            deep += dp
        if why is not None and sq <= tq and sv <= tv:  # the last resort: a deep fp32 portal
            dp = []
            why, t = _contact_lists_agree(_oracle_forward(oracle_mod, om, None, x32, st), recs, compiled, dp, True)
            if why is None:
                deep += dp
                kinds["divergent"] += 1
                divergent.append(int(e))
                continue
        if why is None and sq <= tq and sv <= tv:
            kinds["geometry"] += 1
            ties += t
        elif why is None and solver == "Newton" and excess <= 1e-7 and sv <= 5e-4 and sq <= h * 5e-4 * scale[e]:
            kinds["solver"] += 1
        elif why is None and solver != "Newton" and sq <= FULL_SOLVER_QPOS and sv <= FULL_SOLVER_QVEL:
            kinds["solver"] += 1
        elif why is None and solver == "CG" and excess <= 1e-6 and sv <= FULL_SOLVER_QVEL:
            # CG is a primal method: its iterate after the same budget is as good, in the
            # oracle's fp64 cost, as the oracle's own fp64 CG's (to 1e-6 of the cost)
            kinds["solver"] += 1
        else:
            unexplained.append((int(e), float(eq[e]), float(sq), float(sv), float(excess), why))
    # the states and the GPU's contacts, for a CPU-side look with the oracle
    for tag, ids in (("unexplained", [u[0] for u in unexplained]), ("divergent", divergent)):
        if ids:
            os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
            ids = np.array(ids)
            np.savez(os.path.join(ROOT, "gpurun_out", f"fullbatch_{label}_{tag}.npz"), ids=ids, qpos=qpos[ids],
                     qvel=qvel[ids], ws=ws[ids], ctrl=ctrl[ids], con=con[ids], gq=gq[ids], gv=gv[ids], x32=x32)
    print(f"{label} full batch: {(~tight).sum()} of {len(qpos)} states outside the tight bound (max qpos err {eq.max():.2e}, "
          f"max qvel err / scale {ev.max():.2e}; tight set {eq[tight].max():.2e} / {ev[tight].max():.2e}); {kinds}, "
          f"{ties} tie contacts; deep mesh-mesh contacts on geometry (pair, GPU dist, oracle dist, fp64 minimum "
          f"penetration or separation along the GPU normal, rule) {deep}; unexplained {unexplained[:10]}")
    return tight, kinds, ties, deep, unexplained


# Full-batch bounds per solver (test_full_batch_parity).  "solver" for CG and PGS: their
# MuJoCo defaults (100 iterations / sweeps, tolerance 1e-8) stop short of the optimum, so
# the primal-cost rule does not apply; instead the oracle's own CG / PGS run on the GPU's
# contact list from the same warm start must reproduce the GPU's step within
# FULL_SOLVER_QPOS (qpos) and FULL_SOLVER_QVEL (qvel / scale) -- fp32 and fp64 walk the
# same iteration from the same start, and stop on the same test.
# (measured, round 6: CG 2.5e-5 / 6.7e-5 qpos on the two states of its own trajectory's mix
# that needed it, 100 iterations stopping on a linearly converging path)
FULL_SOLVER_QPOS, FULL_SOLVER_QVEL = 1e-4, 5e-3


@pytest.mark.parametrize("solver", ["Newton", "CG", "PGS"])
def test_full_batch_parity(gpu, oracle_mod, solver):
    """BASELINE config 3 at full size, on each configuration's own bench state mix: 4096
    reorient envs after 40 control steps of the random agent (auto-resets, falls, deep
    contact-rich grasps, the overflow tier included), with each of the three solvers at
    MuJoCo's defaults -- the headline's Newton, and CG / PGS (config 3' / 3'', their own
    kernel specializations), each stepping its own trajectory.  Every env's fp32 state then
    takes one physics step on the GPU and in the fp64 oracle with the same solver (OpenMP
    over envs).  Tight: qpos within 1e-6 and qvel within 5e-4 of max(1, |qacc_smooth|).
    Every state outside it must be accounted for, one of these ways, and none may remain:
      * MPR discontinuity: the GPU equals (tight) one of the oracle's runs from the state
        perturbed at fp32 resolution (_nearest_perturbed);
      * contact geometry: the oracle's dynamics run on the GPU's own contact list
        (dxo_set_contacts) reproduce the GPU's step tightly, and that list agrees with the
        oracle's at the state or at one of 16 fp32-rounding perturbations of it
        (_contact_lists_agree) -- the whole difference is fp32 MPR's choice of normal, the
        constraints, solver and integrator are the oracle's;
      * solver resolution: Newton -- on the GPU's contacts, the GPU's qacc is optimal in
        the oracle's fp64 cost to within 1e-7 of the cost (the fp32 resolution of the cost
        the kernel's Newton stops at), qvel within the tight bound and qpos within that
        bound integrated over the step (h x 5e-4 of the scale); CG and PGS -- the oracle's
        same solver from the same state and warm start (or on the GPU's contacts)
        reproduces the GPU's step within FULL_SOLVER_QPOS / FULL_SOLVER_QVEL, their
        "tight" (100 iterations / sweeps stop short of the optimum, where fp32 and fp64
        walk the same iteration apart); CG, a primal method, also when its iterate is as
        good in the oracle's fp64 cost as the oracle's own CG's (to 1e-6 of the cost);
      * fp32 portal (the last resort): every contact list difference is a deep box-hull or
        hull-hull contact that the reference MPR evaluated in fp32 reproduces
        (_contact_lists_agree `divergent`, oracle/mpr_ref.py)."""
    from dexterity_amd import manipulation

    n = 4096
    if solver == "Newton":
        env = manipulation.load("reorient", "state_dense", seed=1, num_envs=n)
    else:  # config 3' / 3'': <option solver=...> at MuJoCo's defaults (tools/bench_configs.py)
        t = manipulation.SUITE[("reorient", "state_dense")]()
        t.compiled = t.compiled.with_solver(solver)
        env = manipulation.GoalEnvironment(t, num_envs=n, seed=1)
    env.reset()
    for step in range(40):
        env.step_random(step)
    ts = env.timestep()
    for k, v in ts.observation.items():
        assert np.all(np.isfinite(v)), k
    assert np.all(np.isfinite(ts.reward))
    assert env.physics.debug_get("queue_timeouts")[0] == 0
    ph = env.physics
    qpos, qvel = ph.qpos, ph.qvel
    ws, ctrl = ph.get(_lib.QACC_WARMSTART), ph.get(_lib.CTRL)
    ncon = ph.get(_lib.NCON)[:, 0]
    assert (ncon > 0).mean() > 0.5
    xfrc = env.task.gravity_compensation
    model = env.model
    env.close()
    # the GPU: the forward pass (contacts, qacc, and qacc_smooth for the error scale), then
    # one physics step from exactly these states
    phys = gpu.BatchedPhysics(model, n)
    phys.set_xfrc(xfrc)
    for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws), (_lib.CTRL, ctrl)):
        phys.set(f, v)
    phys.debug(True)
    phys.forward()
    scale = np.maximum(1.0, np.abs(phys.debug_get("qacc_smooth")).max(axis=1))
    con = phys.debug_get("contact").astype(np.float64)
    gqacc = phys.qacc.astype(np.float64)
    for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws)):
        phys.set(f, v)
    phys.debug(False)
    phys.step(1)
    gq, gv = phys.qpos, phys.qvel
    phys.close()
    # the oracle from the same fp32 states
    om = oracle_mod.OracleModel(model.blob)
    h = float(model.compiled.timestep)  # the physics step (s)
    x32 = np.asarray(xfrc, dtype=np.float32).astype(np.float64).ravel()
    rc, oq, ov, _ = oracle_mod.batch_step(om, qpos.astype(np.float64), qvel.astype(np.float64),
                                          ctrl.astype(np.float64), ws.astype(np.float64), x32, nsub=1)
    assert rc == 0
    tight, kinds, ties, deep, unexplained = _account_full_batch(
        oracle_mod, om, model.compiled, x32, h, (qpos, qvel, ws, ctrl), (gq, gv, gqacc, con, scale, oq, ov),
        f"reorient_{solver.lower()}", solver=solver)
    # pinned near the measured rates, so a regression in any category shows (Newton, this
    # state mix: round 4 212 of 4096 outside the tight bound -- 172 perturbed, 38 geometry,
    # 2 solver; round 5, MPR's final closest point in fp64: 182 -- 170 perturbed, 9
    # geometry, 3 solver; 0 unexplained)
    cap = FULL_CEILINGS[solver]
    assert (~tight).mean() <= cap["outside"]
    assert kinds["perturbed"] <= cap["perturbed"] and kinds["geometry"] <= 20 and kinds["solver"] <= cap["solver"], kinds
    assert kinds["divergent"] <= cap["fp32_portal"], kinds
    assert not unexplained
    # ("min": the GPU's depth within 3 % of the fp64 minimum penetration -- as good an
    # answer as MPR gives; the other rules are the ones held to a count)
    assert sum(dp[-1] != "min" for dp in deep) <= max(2, n // 1000), deep


# test_full_batch_parity's ceilings per solver, pinned near the measured rates (round 6 on
# the headline mix: CG 316 outside the tight bound -- 184 solver (its 100 iterations stop
# short on a linearly converging path, fp32 and fp64 apart), 125 perturbed, 5 geometry, 2
# divergent; PGS 204 -- 71 solver, 126 perturbed, 5 geometry, 2 divergent; 0 unexplained)
FULL_CEILINGS = {"Newton": dict(outside=0.06, perturbed=220, solver=8, fp32_portal=2),
                 "CG": dict(outside=0.09, perturbed=300, solver=240, fp32_portal=6),
                 "PGS": dict(outside=0.07, perturbed=220, solver=120, fp32_portal=6)}


def test_ground_contact_watch_matches_oracle(gpu, oracle_mod, reorient_setup):
    """DX_GROUND_CONTACT (ReOrient._is_prop_fallen, reorient.py:229-235 ->
    has_collision, utils/mujoco_collisions.py:95-119: a prop-ground contact with
    dist <= 1e-8) against the oracle's contact list, for cubes resting on, sunk into,
    hovering over and far above the ground, and on the palm."""
    from dexterity_amd import manipulation

    cm, xfrc, om, states, model = reorient_setup
    task = manipulation.ReOrient()
    ground, prop_body = task.ground_geom, task.prop_body
    pq = task.prop_qadr
    rs = np.random.RandomState(4)
    qs = []
    for z in (0.0199, 0.0195, 0.02, 0.0201, 0.021, 0.03, 0.1):
        for _ in range(3):
            q = cm.qpos0.copy()
            q[pq:pq + 3] = [0.3 + rs.uniform(-0.05, 0.05), 0.3 + rs.uniform(-0.05, 0.05), z]
            if z < 0.05:  # axis-aligned: a face (four corners) on the ground
                q[pq + 3:pq + 7] = [1, 0, 0, 0]
            else:
                qq = rs.randn(4)
                q[pq + 3:pq + 7] = qq / np.linalg.norm(qq)
            qs.append(q)
    qs.append(states[0][0])  # the cube on the palm
    qs = np.stack(qs)
    phys = gpu.BatchedPhysics(model, len(qs))
    phys.set_watch(ground, prop_body)
    phys.set(_lib.QPOS, qs)
    phys.forward()
    flag = phys.get(_lib.GROUND_CONTACT)[:, 0]
    prop_geoms = {g for g in range(cm.ngeom) if cm.geom_bodyid[g] == prop_body}
    expect = []
    for q in qs:
        d = oracle_mod.OracleData(om)
        d.qpos[:] = q.astype(np.float32)
        d.kinematics()
        hit = False
        for con in d.contacts():
            g1, g2 = int(con[13]), int(con[14])
            if {g1, g2} & {ground} and ({g1, g2} & prop_geoms) and con[12] <= 1e-8:
                hit = True
        expect.append(hit)
    np.testing.assert_array_equal(flag.astype(bool), np.array(expect))
    assert np.array(expect).any() and not np.array(expect).all()
    phys.close()


def test_substep_queue_matches_per_env_launch(gpu, monkeypatch):
    """The substep queue (one task per env and physics step, state handed over through
    HBM between workgroups, dx_step.hip step_queue) gives bit-identical trajectories to
    one workgroup per env for the whole control step (DX_NO_QUEUE=1), auto-resets,
    rewards and observations included: 4096 envs, 25 control steps."""
    from dexterity_amd import manipulation

    outs = []
    for no_queue in (False, True):
        if no_queue:
            monkeypatch.setenv("DX_NO_QUEUE", "1")
        env = manipulation.load("reorient", "state_dense", seed=5, num_envs=4096)
        env.reset()
        for step in range(25):
            env.step(env.sample_actions(step), device_action=True)
        ts = env.timestep()
        outs.append((env.physics.qpos, env.physics.qvel, env.physics.get(_lib.QACC_WARMSTART), ts.reward,
                     np.concatenate([v.reshape(4096, -1) for v in ts.observation.values()], axis=1)))
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        env.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_narrowphase_group_size_is_invisible(gpu, monkeypatch):
    """The narrowphase's 4-lane groups (sixteen pairs per wave, dx_step.hip narrow_pass<4>,
    used above eight candidates) and its 8-lane groups give bit-identical trajectories:
    every pair's support scan, first-maximiser rule and portal arithmetic are the same,
    and the separating-direction cache -- whose slots two pairs share, so which pair owns
    one depends on the order the groups finish -- never decides a verdict MPR would not
    (mpr_init, DX_SEP_CLEAR).  DX_NP_WIDE=0 forces 4-lane groups on every substep, 64
    never; 4096 envs, 15 control steps of random actions, contacts included, no
    allowance for any env to differ."""
    from dexterity_amd import manipulation

    outs = []
    for wide in ("0", "64"):
        monkeypatch.setenv("DX_NP_WIDE", wide)
        env = manipulation.load("reorient", "state_dense", seed=7, num_envs=4096)
        env.reset()
        for step in range(15):
            env.step(env.sample_actions(step), device_action=True)
        ts = env.timestep()
        ncon = env.physics.get(_lib.NCON)[:, 0]
        outs.append((env.physics.qpos, env.physics.qvel, env.physics.get(_lib.QACC_WARMSTART), ncon, ts.reward))
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        env.close()
    assert (outs[0][3] > 0).mean() > 0.5
    differ = np.zeros(4096, dtype=bool)
    for a, b in zip(*outs):
        differ |= (np.asarray(a).reshape(4096, -1) != np.asarray(b).reshape(4096, -1)).any(axis=1)
    assert differ.sum() == 0, np.flatnonzero(differ)


def test_contact_tiers_are_invisible(gpu, monkeypatch):
    """Which tier runs a physics step changes nothing: the step kernel with the mid tier
    beside it (the default: deferred steps run while the launch goes on), without it
    (DX_NO_MID=1: the overflow tier after the launch), and with every step that has a
    contact deferred to the mid tier (DX_DEFER_AT=0) give bit-identical trajectories --
    1024 envs, 12 control steps of random actions, outputs and task logic included."""
    from dexterity_amd import manipulation

    outs = []
    for env_vars in ({}, {"DX_NO_MID": "1"}, {"DX_DEFER_AT": "0"}):
        for k in ("DX_NO_MID", "DX_DEFER_AT"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env_vars.items():
            monkeypatch.setenv(k, v)
        env = manipulation.load("reorient", "state_dense", seed=5, num_envs=1024)
        env.reset()
        for step in range(12):
            env.step_random(step)
        ts = env.timestep()
        h = env.physics.health()
        outs.append((env.physics.qpos, env.physics.qvel, env.physics.get(_lib.QACC_WARMSTART), ts.reward,
                     ts.observation["shadow_hand_e/joint_positions"] if "shadow_hand_e/joint_positions" in ts.observation
                     else next(iter(ts.observation.values()))))
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        assert h["contact_overflow"] == 0 and h["diverged"] == 0
        if env_vars.get("DX_DEFER_AT") == "0":
            assert h["contact_deferred"] > 2000, h
        env.close()
    for o in outs[1:]:
        differ = np.zeros(1024, dtype=bool)
        for a, b in zip(outs[0], o):
            differ |= (np.asarray(a).reshape(1024, -1) != np.asarray(b).reshape(1024, -1)).any(axis=1)
        assert differ.sum() == 0, np.flatnonzero(differ)


def test_mixed_launches_with_deferrals(gpu, monkeypatch):
    """Deferral entries belong to their launch (list[1] = the launch's epoch; the mid tier
    claims only its own launch's entries, with its own nsub and task-logic mode): fused
    5-substep control steps alternating with raw 1- and 3-substep physics launches, every
    contact step deferred (DX_DEFER_AT=0), are bit-identical with and without the mid tier
    (DX_NO_MID=1: every entry run by its own launch's overflow tier)."""
    from dexterity_amd import manipulation

    n = 512
    outs = []
    for env_vars in ({"DX_DEFER_AT": "0"}, {"DX_DEFER_AT": "0", "DX_NO_MID": "1"}):
        monkeypatch.delenv("DX_NO_MID", raising=False)
        for k, v in env_vars.items():
            monkeypatch.setenv(k, v)
        env = manipulation.load("reorient", "state_dense", seed=8, num_envs=n)
        env.reset()
        for step in range(9):
            env.step_random(step)
            env.physics.step(1 + 2 * (step % 2))  # no task logic, another nsub
        env.physics.sync()
        h = env.physics.health()
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        assert h["contact_overflow"] == 0 and h["diverged"] == 0
        assert h["contact_deferred"] > 500, h
        outs.append((env.physics.qpos, env.physics.qvel, env.physics.get(_lib.QACC_WARMSTART),
                     env.timestep().reward, env.physics.get(_lib.TIME)))
        env.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


def test_order_key_beyond_16_bit_rank(gpu):
    """The longest-first order keeps an env's rank within its cost bucket in 24 bits: after
    a reset every env of a 70,000-env batch is an observe-only env of about the same cost
    (one bucket, > 65,536 ranks), and the next launches must still run every env exactly
    once.  Env e's trajectory does not depend on the batch size or the order, so the first
    1,024 envs equal a 1,024-env batch of the same seed bit for bit."""
    from dexterity_amd import manipulation

    outs = []
    for n in (70000, 1024):
        env = manipulation.load("reorient", "state_dense", seed=13, num_envs=n)
        env.reset()
        for step in range(4):
            env.step_random(step)
        env.physics.sync()
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        outs.append((env.physics.qpos[:1024], env.physics.qvel[:1024], env.timestep().reward[:1024],
                     env.physics.get(_lib.TIME)[:1024]))
        env.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


def _check_reach_rewards(env, ts, dense):
    from oracle import task_ref

    obs = ts.observation
    hand = env.task.hand_name
    for e in range(env.num_envs):
        if ts.step_type[e] == 0:
            assert ts.reward[e] == 0 and ts.discount[e] == 1
            continue
        r = task_ref.reach_reward(obs["goal_state"][e], obs[f"{hand}/fingertip_positions"][e], dense=dense)
        assert ts.reward[e] == pytest.approx(r, rel=1e-4, abs=1e-5)
        assert ts.discount[e] in (0.0, 1.0)


@pytest.mark.parametrize("task", ["state_dense", "state_sparse"])
def test_reach_adroit_env(gpu, task):
    """Reach (reference task, Adroit hand): rewards equal the fp64 restatement of
    reach.py:196-210 on the step's own observation; episodes start inside half the
    joint range (reach.py:34, dexterous_hand.py:120-142) after the goal rollouts
    advanced time by two physics steps (fingertip_position.py:93-111)."""
    from dexterity_amd import manipulation

    n = 64
    env = manipulation.load("reach", task, seed=3, num_envs=n)
    ts = env.reset()
    assert np.all(ts.first())
    lo, hi = env.task.joint_range.T
    q = env.physics.qpos
    assert np.all(q >= 0.5 * lo - 1e-6) and np.all(q <= 0.5 * hi + 1e-6)
    t = env.physics.get(_lib.TIME)[:, 0]
    np.testing.assert_allclose(t, 0.04, atol=1e-6)
    goals = env.goals()
    assert goals.shape == (n, 15) and np.all(np.isfinite(goals))
    tips0 = ts.observation[f"{env.task.hand_name}/fingertip_positions"]
    d0 = np.linalg.norm((goals - tips0).reshape(n, 5, 3), axis=2)
    assert np.all(d0 < 0.25) and d0.mean() > 1e-3  # reachable, not the start pose
    assert len({tuple(np.round(g, 5)) for g in goals}) == n  # per-env draws
    spec = env.action_spec()
    rng = np.random.RandomState(12345)
    for step in range(12):
        action = rng.uniform(spec.minimum, spec.maximum, size=(n, spec.shape[0])).astype(np.float32)
        ts = env.step(action)
        _check_reach_rewards(env, ts, dense=task == "state_dense")
        for k, v in ts.observation.items():
            assert np.all(np.isfinite(v)), k
    assert env.goal_failures().sum() == 0
    for name, spec_ in env.observation_spec().items():
        assert ts.observation[name].shape[1:] == spec_.shape
    assert env.obs_dim == 117
    env.close()


def test_reach_shadow_config2(gpu):
    """BASELINE config 2: reach with the Shadow hand, contact-free, 1024 envs.
    Coupled joints equal after the initial sampling (shadow_hand_e.py:124-129);
    rewards match the restatement; 30 control steps stay finite."""
    from dexterity_amd import hands, manipulation

    n = 1024
    env = manipulation.load("reach_shadow", "state_dense", seed=11, num_envs=n)
    env.reset()
    q = env.physics.qpos
    for ids in hands.COUPLED_JOINT_IDS:
        np.testing.assert_array_equal(q[:, ids[0]], q[:, ids[-1]])
    for step in range(30):
        env.step(env.sample_actions(step), device_action=True)
    ts = env.timestep()
    _check_reach_rewards(env, ts, dense=True)
    assert np.all(np.isfinite(env.physics.qpos))
    env.close()


def _bimanual_states(oracle_mod, cm, xfrc, n_traj=3, seed=5):
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    rng = np.random.RandomState(seed)
    lo, hi = cm.actuator_ctrlrange.T
    states = []
    for t in range(n_traj):
        d = oracle_mod.OracleData(om)
        d.xfrc_applied[:] = xfrc.ravel()
        d.qpos[48:51] += rng.uniform(-0.02, 0.02, size=3) * [1, 1, 0]
        ctrl = rng.uniform(lo, hi) * 0.3
        for s in range(100):
            d.ctrl[:] = ctrl
            d.step()
            if s in (40, 99):
                states.append((d.qpos.copy(), d.qvel.copy(), d.qacc_warmstart.copy(), ctrl.copy()))
    return om, states


@pytest.fixture(scope="module")
def bimanual_setup(gpu, oracle_mod):
    """BASELINE config 5 scene: two Shadow hands (nv 54, the n > 32 Cholesky path)."""
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "bimanual_handover.npz"))
    xfrc = gpu.gravity_compensation(cm, "shadow_hand_")
    om, states = _bimanual_states(oracle_mod, cm, xfrc)
    model = gpu.Model(cm)
    return cm, xfrc, om, states, model


def _check_bimanual_forward(gpu, oracle_mod, cm, xfrc, om, states, model):
    phys = _load_states(gpu, model, xfrc, states)
    phys.debug(True)
    phys.forward()
    phys.sync()
    M = phys.debug_get("M")
    a0 = phys.debug_get("qacc_smooth")
    con = phys.debug_get("contact")
    cnt = phys.debug_get("efc_count")
    qacc = phys.qacc
    with_contacts = 0
    ties = 0
    for e, st in enumerate(states):
        ds = _oracle_pair(oracle_mod, om, cm, xfrc, st)
        d = ds[0]
        Mo = d.M.reshape(cm.nv, cm.nv)
        assert np.abs(M[e] - Mo).max() <= 1e-5 * np.abs(Mo).max()
        scale = np.abs(d.qacc_smooth).max()
        assert np.abs(a0[e] - d.qacc_smooth).max() <= 1e-5 * scale
        oc = d.contacts()
        gc = con[e, : (con[e, :, 15] != 0).sum()]
        assert cnt[e, 1] == 0, "overflow flag set"
        assert {(int(r[13]), int(r[14])) for r in gc} == {(int(r[13]), int(r[14])) for r in oc}
        with_contacts += len(oc) > 0
        tie = sum(_contact_tie(cm, ds, r) for r in gc) > 0
        ties += tie
        sc = max(1.0, scale)
        if not tie:
            err = np.minimum(np.abs(qacc[e] - ds[0].qacc), np.abs(qacc[e] - ds[1].qacc))
            assert err[:48].max() <= 5e-4 * sc, f"env {e}"
            assert err[48:].max() <= 3e-3 * sc, f"env {e}"
        else:
            # a tie state is not skipped: on the GPU's own contacts the oracle's
            # accelerations equal the GPU's within the tight bound (the tie is the whole
            # difference), and the difference itself stays within the tie bounds
            fix = np.abs(qacc[e] - _qacc_on_gpu_contacts(oracle_mod, om, xfrc, st, gc))
            assert fix.max() <= 5e-4 * sc, (f"tie env {e} on the GPU's contacts", fix.max() / sc)
            err = min((np.abs(qacc[e] - dd.qacc) for dd in ds), key=lambda x: x.max())
            BIMANUAL_TIE_ERR.append(float(err.max() / sc))
            assert err[:48].max() <= TIE_QACC_HAND * sc, (f"tie env {e}", err.max() / sc)
            assert err[48:].max() <= TIE_QACC_CUBE * sc, (f"tie env {e}", err.max() / sc)
    phys.close()
    return with_contacts, ties


def test_bimanual_forward_parity(gpu, oracle_mod, bimanual_setup):
    """Mass matrix, smooth and constrained accelerations and the contact set of the
    two-hand scene match the fp64 oracle.  Tolerances as the reorient test, except the
    cube's own dofs: its contact points may differ by up to 2e-4 m (where fp32 and
    fp64 MPR stop refining the portal), which on a 2 cm cube is a ~1 % lever-arm
    change of its angular acceleration, so those six dofs get 3e-3 of the scale."""
    with_contacts, _ = _check_bimanual_forward(gpu, oracle_mod, *bimanual_setup)
    assert with_contacts >= 3


def test_bimanual_pgs_forward(gpu, oracle_mod, bimanual_setup):
    """PGS at MuJoCo's defaults on the two-hand scene (nv 54: M^-1 J_r' by the LDS
    Cholesky, not the sweep's inverse): kernel vs the oracle's PGS, one forward pass.
    A state whose contact set ties (MPR's choice under fp32 rounding) is held to the
    same bound on the GPU's own contacts (dxo_set_contacts)."""
    cm, xfrc, _, states, _ = bimanual_setup
    pg = cm.with_solver("PGS")
    om = oracle_mod.OracleModel(blob.pack(pg.arrays))
    phys = _load_states(gpu, gpu.Model(pg), xfrc, states)
    phys.debug(True)
    phys.forward()
    phys.sync()
    con = phys.debug_get("contact")
    qacc = phys.qacc
    phys.close()
    errs = []
    for e, st in enumerate(states):
        ds = _oracle_pair(oracle_mod, om, pg, xfrc, st)
        sc = max(1.0, np.abs(ds[0].qacc_smooth).max())
        err = min((np.abs(qacc[e] - d.qacc) for d in ds), key=lambda x: x.max())
        if err.max() > PGS_BIMANUAL_HAND * sc:
            gc = con[e, : (con[e, :, 15] != 0).sum()]
            err = np.abs(qacc[e] - _qacc_on_gpu_contacts(oracle_mod, om, xfrc, st, gc))
        errs.append((err[:48].max() / sc, err[48:].max() / sc))
    errs = np.array(errs)
    print(f"bimanual PGS: |qacc| err / scale, hands max {errs[:, 0].max():.2e}, cube max {errs[:, 1].max():.2e}")
    assert errs[:, 0].max() <= PGS_BIMANUAL_HAND and errs[:, 1].max() <= PGS_BIMANUAL_CUBE


# measured (r4): hands max 4.0e-6, cube max 9.6e-4 (3.1e-5 on another box) of the scale (the cube's contact
# points, as Newton's bimanual bound)
PGS_BIMANUAL_HAND, PGS_BIMANUAL_CUBE = 5e-5, 3e-3

BIMANUAL_TIE_ERR = []


def test_bimanual_forward_parity_wide_sample(gpu, oracle_mod, bimanual_setup):
    """As above over 12 trajectories (24 states).  Tie states are held to the tie bounds
    and, on the GPU's own contacts, to the tight bound (_check_bimanual_forward); at most
    1 of the 24 (measured round 4: none)."""
    cm, xfrc, _, _, model = bimanual_setup
    om, states = _bimanual_states(oracle_mod, cm, xfrc, n_traj=12, seed=11)
    BIMANUAL_TIE_ERR.clear()
    with_contacts, ties = _check_bimanual_forward(gpu, oracle_mod, cm, xfrc, om, states, model)
    print(f"bimanual wide sample: {with_contacts} of {len(states)} states in contact, {ties} tie states, "
          f"their qacc errors / scale {BIMANUAL_TIE_ERR}")
    assert with_contacts >= 15
    assert ties <= 1


def test_bimanual_substep(gpu, oracle_mod, bimanual_setup):
    """One substep vs the oracle (qpos 1e-5)."""
    cm, xfrc, om, states, model = bimanual_setup
    phys = _load_states(gpu, model, xfrc, states)
    phys.step(1)
    qpos = phys.qpos
    for e, st in enumerate(states):
        d = oracle_mod.OracleData(om)
        d.xfrc_applied[:] = xfrc.ravel()
        d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = st
        d.step()
        assert np.abs(qpos[e] - d.qpos).max() < 1e-5


def test_bimanual_full_batch_parity(gpu, oracle_mod, bimanual_setup):
    """BASELINE config 5 at full size with test_full_batch_parity's accounting: 4096
    two-hand envs (nv 54: the LDS Cholesky path; the 64- and 256-contact tiers at the
    scene's contact counts) after 20 control steps of random actions from randomised cube
    positions; every env's fp32 state then takes one physics step on the GPU and in the
    fp64 oracle, and every state outside the tight bound is explained (MPR discontinuity,
    contact geometry or solver resolution), none left."""
    cm, xfrc, om, _, model = bimanual_setup
    n = 4096
    big = gpu.BatchedPhysics(model, n)
    big.set_xfrc(xfrc)
    q0 = np.tile(cm.qpos0, (n, 1))
    q0[:, 48:51] += np.random.RandomState(0).uniform(-0.02, 0.02, size=(n, 3)) * [1, 1, 0]
    big.set(_lib.QPOS, q0)
    lo, hi = cm.actuator_ctrlrange.T
    rng = np.random.RandomState(1)
    for step in range(20):
        big.set(_lib.CTRL, rng.uniform(lo, hi, size=(n, cm.nu)).astype(np.float32))
        big.step(5)
    qpos, qvel = big.qpos, big.qvel
    ws, ctrl = big.get(_lib.QACC_WARMSTART), big.get(_lib.CTRL)
    assert np.all(np.isfinite(qpos)) and np.all(np.isfinite(qvel))
    assert (big.get(_lib.NCON)[:, 0] > 0).mean() > 0.5
    h = big.health()
    assert h["contact_overflow"] == 0 and h["diverged"] == 0, h
    assert big.debug_get("queue_timeouts")[0] == 0
    big.debug(True)
    big.forward()
    scale = np.maximum(1.0, np.abs(big.debug_get("qacc_smooth")).max(axis=1))
    con = big.debug_get("contact").astype(np.float64)
    gqacc = big.qacc.astype(np.float64)
    for f, v in ((_lib.QPOS, qpos), (_lib.QVEL, qvel), (_lib.QACC_WARMSTART, ws)):
        big.set(f, v)
    big.debug(False)
    big.step(1)
    gq, gv = big.qpos, big.qvel
    big.close()
    x32 = np.asarray(xfrc, dtype=np.float32).astype(np.float64).ravel()
    rc, oq, ov, _ = oracle_mod.batch_step(om, qpos.astype(np.float64), qvel.astype(np.float64),
                                          ctrl.astype(np.float64), ws.astype(np.float64), x32, nsub=1)
    assert rc == 0
    tight, kinds, ties, deep, unexplained = _account_full_batch(
        oracle_mod, om, cm, x32, float(cm.timestep), (qpos, qvel, ws, ctrl), (gq, gv, gqacc, con, scale, oq, ov),
        "bimanual")
    # measured (round 5): 235 of 4096 outside the tight bound -- 222 perturbed, 10
    # geometry, 1 solver, 2 divergent deep finger-finger portals (ring distal / little
    # middle of one hand, 0.9-1.9 mm deep: same contact point, depth 4-8 % apart)
    assert (~tight).mean() <= 0.08
    assert kinds["perturbed"] <= 300 and kinds["geometry"] <= 30 and kinds["solver"] <= 8, kinds
    assert kinds["divergent"] <= 4, kinds
    assert not unexplained
    assert len(deep) <= 16


def test_cg_solver_parity(gpu, oracle_mod, reorient_setup):
    """<option solver="CG"> ([3P] MuJoCo's primal CG): the kernel's CG (dx_step.hip
    solve_cg) against the oracle's (dx_oracle.c solve_cg) on the contact-rich states,
    and both against the Newton optimum; then a few CG substeps stay finite."""
    cm, xfrc, om, states, _ = reorient_setup
    # CG converges linearly, and fp32 and fp64 CG take different paths: both run to
    # the optimum (tight tolerance, ample iterations) and are compared there
    cg = cm.with_solver("CG", iterations=1000, tolerance=1e-10)
    model = gpu.Model(cg)
    om_cg = oracle_mod.OracleModel(blob.pack(cg.arrays))
    phys = _load_states(gpu, model, xfrc, states)
    phys.forward()
    qacc = phys.qacc
    for e, st in enumerate(states):
        # either side of an MPR discontinuity (_oracle_pair)
        d_cg = _oracle_pair(oracle_mod, om_cg, cg, xfrc, st)
        d_nt = _oracle_pair(oracle_mod, om, cm, xfrc, st)
        scale = max(1.0, np.abs(d_nt[0].qacc_smooth).max())
        err_cg = min(np.abs(qacc[e] - d.qacc).max() for d in d_cg)
        err_nt = min(np.abs(qacc[e] - d.qacc).max() for d in d_nt)
        assert err_cg <= 5e-4 * scale, (e, err_cg, scale)
        assert err_nt <= 5e-4 * scale
    phys.close()
    # MuJoCo's defaults (100 iterations, 1e-8) with CG on both sides: kernel CG vs the
    # oracle's CG at identical settings, one substep and three, per state
    cgd = cm.with_solver("CG")
    om_d = oracle_mod.OracleModel(blob.pack(cgd.arrays))
    for nsub in (1, 3):
        phys = _load_states(gpu, gpu.Model(cgd), xfrc, states)
        phys.step(nsub)
        qpos, qvel = phys.qpos, phys.qvel
        assert np.all(np.isfinite(qpos))
        eq, ev = [], []
        for e, st in enumerate(states):
            best = None
            for x, y in ((xfrc, st), (np.asarray(xfrc, dtype=np.float32).astype(np.float64), _f32(st))):
                d = oracle_mod.OracleData(om_d)
                d.xfrc_applied[:] = x.ravel()
                d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = y
                for _ in range(nsub):
                    d.step()
                sc = max(1.0, np.abs(d.qacc_smooth).max())
                q, v = np.abs(qpos[e] - d.qpos).max(), np.abs(qvel[e] - d.qvel).max() / sc
                best = (q, v) if best is None or q < best[0] else best
            if best[0] > CG_QPOS_MAX * nsub or best[1] > CG_QVEL_MAX:
                # a contact tie along the way (MPR's discontinuities): the nearest of the
                # oracle's runs from fp32-resolution perturbations of the state
                pq, pv = _nearest_perturbed(oracle_mod, om_d, np.asarray(xfrc, dtype=np.float32).astype(np.float64).ravel(),
                                            _f32(st), nsub, qpos[e], qvel[e], sc)
                best = min(best, (pq, pv))
            eq.append(best[0])
            ev.append(best[1])
        eq, ev = np.array(eq), np.array(ev)
        print(f"CG defaults, {nsub} substep(s): |qpos| err median {np.median(eq):.2e} max {eq.max():.2e}; "
              f"|qvel|/scale median {np.median(ev):.2e} max {ev.max():.2e}")
        assert np.median(eq) <= 1e-6 and eq.max() <= CG_QPOS_MAX * nsub
        assert np.median(ev) <= 1e-5 and ev.max() <= CG_QVEL_MAX
        phys.close()


def test_pgs_solver_parity(gpu, oracle_mod, reorient_setup):
    """<option solver="PGS"> ([3P] MuJoCo's dual projected Gauss-Seidel): the kernel's
    PGS (dx_step.hip solve_pgs) against the oracle's (dx_oracle.c solve_pgs) on the
    contact-rich states -- run to convergence, both at the Newton optimum (the primal
    problem's solution, the restatement's anchor); at MuJoCo's defaults (100 sweeps,
    1e-8), kernel vs oracle at identical settings, one forward pass and 1 / 3 substeps."""
    cm, xfrc, om, states, _ = reorient_setup
    pg = cm.with_solver("PGS", iterations=3000, tolerance=1e-13)
    om_pg = oracle_mod.OracleModel(blob.pack(pg.arrays))
    phys = _load_states(gpu, gpu.Model(pg), xfrc, states)
    phys.forward()
    qacc = phys.qacc
    e_pg, e_nt = [], []
    for e, st in enumerate(states):
        d_pg = _oracle_pair(oracle_mod, om_pg, pg, xfrc, st)
        d_nt = _oracle_pair(oracle_mod, om, cm, xfrc, st)
        scale = max(1.0, np.abs(d_nt[0].qacc_smooth).max())
        e_pg.append(min(np.abs(qacc[e] - d.qacc).max() for d in d_pg) / scale)
        e_nt.append(min(np.abs(qacc[e] - d.qacc).max() for d in d_nt) / scale)
    phys.close()
    e_pg, e_nt = np.array(e_pg), np.array(e_nt)
    print(f"PGS converged: |qacc| err / scale vs oracle PGS max {e_pg.max():.2e}, vs Newton max {e_nt.max():.2e}")
    assert e_pg.max() <= PGS_CONV_MAX and e_nt.max() <= PGS_CONV_MAX
    # MuJoCo's defaults on both sides
    pgd = cm.with_solver("PGS")
    om_d = oracle_mod.OracleModel(blob.pack(pgd.arrays))
    phys = _load_states(gpu, gpu.Model(pgd), xfrc, states)
    phys.forward()
    qacc = phys.qacc
    ea = []
    for e, st in enumerate(states):
        d_pg = _oracle_pair(oracle_mod, om_d, pgd, xfrc, st)
        scale = max(1.0, np.abs(d_pg[0].qacc_smooth).max())
        ea.append(min(np.abs(qacc[e] - d.qacc).max() for d in d_pg) / scale)
    phys.close()
    ea = np.array(ea)
    print(f"PGS defaults, forward: |qacc| err / scale median {np.median(ea):.2e} max {ea.max():.2e}")
    assert np.median(ea) <= PGS_QACC_MED and ea.max() <= PGS_QACC_MAX
    for nsub in (1, 3):
        phys = _load_states(gpu, gpu.Model(pgd), xfrc, states)
        phys.step(nsub)
        qpos, qvel = phys.qpos, phys.qvel
        assert np.all(np.isfinite(qpos)) and np.all(np.isfinite(qvel))
        eq, ev = [], []
        for e, st in enumerate(states):
            best = None
            for x, y in ((xfrc, st), (np.asarray(xfrc, dtype=np.float32).astype(np.float64), _f32(st))):
                d = oracle_mod.OracleData(om_d)
                d.xfrc_applied[:] = x.ravel()
                d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = y
                for _ in range(nsub):
                    d.step()
                sc = max(1.0, np.abs(d.qacc_smooth).max())
                q, v = np.abs(qpos[e] - d.qpos).max(), np.abs(qvel[e] - d.qvel).max() / sc
                best = (q, v) if best is None or q < best[0] else best
            eq.append(best[0])
            ev.append(best[1])
        eq, ev = np.array(eq), np.array(ev)
        print(f"PGS defaults, {nsub} substep(s): |qpos| err median {np.median(eq):.2e} max {eq.max():.2e}; "
              f"|qvel|/scale median {np.median(ev):.2e} max {ev.max():.2e}")
        assert eq.max() <= PGS_QPOS_MAX * nsub and ev.max() <= PGS_QVEL_MAX
        phys.close()


def test_pgs_tail_rows_parity(gpu, oracle_mod):
    """PGS past 128 constraint rows: the AR path's tail rows (dx_step.hip solve_pgs, rows
    128+ one at a time on qacc after the two register blocks).  The reorient envs of the
    bench's state mix with 27 or more contacts (24 friction-loss rows + 4 pyramid edges per
    contact: more than 128 rows, the envs that set the PGS launch) take one forward pass
    with <option solver="PGS">: run to convergence, kernel vs the oracle's PGS
    within PGS_CONV_MAX (test_pgs_solver_parity); at MuJoCo's defaults (100 sweeps, not
    converged on these states), kernel vs oracle within PGS_TAIL_MAX.  Both on the GPU's
    own contact list (dxo_set_contacts)."""
    from dexterity_amd import manipulation

    n = 4096
    env = manipulation.load("reorient", "state_dense", seed=1, num_envs=n)
    env.reset()
    states = []
    for step in range(80):
        env.step_random(step)
        ph = env.physics
        sel = np.nonzero(ph.get(_lib.NCON)[:, 0] >= 27)[0][:3]
        if len(sel):
            q, v, w, u = ph.qpos, ph.qvel, ph.get(_lib.QACC_WARMSTART), ph.get(_lib.CTRL)
            states += [tuple(np.asarray(x[e], dtype=np.float64) for x in (q, v, w, u)) for e in sel]
        if len(states) >= 6:
            break
    xfrc = env.task.gravity_compensation
    cm = env.task.compiled
    env.close()
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    nefc = [_oracle_forward(oracle_mod, om, cm, xfrc, st).nefc for st in states]
    print("tail states: nefc", nefc)
    assert sum(k > 128 for k in nefc) >= 2, nefc
    # on the GPU's own contact list (dxo_set_contacts): the deep contacts of these grasps
    # move under fp32 MPR (the full-batch test's "geometry" states); the solver is the test
    def run(model_cm):
        phys = _load_states(gpu, gpu.Model(model_cm), xfrc, states)
        phys.debug(True)
        phys.forward()
        phys.sync()
        con, qacc = phys.debug_get("contact"), phys.qacc
        phys.close()
        return con, qacc

    def err(om_x, con, qacc, e, st):
        gc = con[e, : (con[e, :, 15] != 0).sum()]
        d = _oracle_forward(oracle_mod, om, cm, xfrc, st)
        scale = max(1.0, np.abs(d.qacc_smooth).max())
        return np.abs(qacc[e] - _qacc_on_gpu_contacts(oracle_mod, om_x, xfrc, st, gc)).max() / scale

    pg = cm.with_solver("PGS", iterations=3000, tolerance=1e-13)
    om_pg = oracle_mod.OracleModel(blob.pack(pg.arrays))
    con, qacc = run(pg)
    e_pg = np.array([err(om_pg, con, qacc, e, st) for e, st in enumerate(states)])
    e_nt = np.array([err(om, con, qacc, e, st) for e, st in enumerate(states)])
    print(f"PGS tail, converged: |qacc| err / scale vs oracle PGS {np.round(e_pg, 7).tolist()}, "
          f"vs Newton {np.round(e_nt, 7).tolist()}")
    pgd = cm.with_solver("PGS")
    om_d = oracle_mod.OracleModel(blob.pack(pgd.arrays))
    con, qacc = run(pgd)
    ea = np.array([err(om_d, con, qacc, e, st) for e, st in enumerate(states)])
    print(f"PGS tail, defaults: |qacc| err / scale {np.round(ea, 7).tolist()}")
    ok = np.array([k > 128 for k in nefc])
    # (3000 sweeps do not reach the Newton optimum on every one of these states -- the
    # oracle's own PGS stays as far from it -- so Newton is reported, not asserted)
    assert e_pg[ok].max() <= PGS_CONV_MAX
    assert ea[ok].max() <= PGS_TAIL_MAX


# PGS bounds.  Measured (r4) over the 12 states: converged (3000 sweeps, 1e-13) qacc
# within 2.9e-4 x scale of both the oracle's PGS and the Newton optimum (fp32's floor
# here, CG's bound); defaults, one forward: median 4.4e-5, max 1.9e-4; 1 / 3 substeps:
# qpos max 9.3e-8 / 1.5e-7, qvel / scale max 9.2e-7 / 6.7e-7
PGS_CONV_MAX = 5e-4
PGS_QACC_MED, PGS_QACC_MAX = 2e-4, 1e-3
PGS_QPOS_MAX, PGS_QVEL_MAX = 1e-6, 1e-5
# tail states (r5, 7 states, nefc 128-144, on the GPU's contacts): converged max 2.4e-5,
# defaults max 2.9e-5 of the scale
PGS_TAIL_MAX = 1e-4


# CG at MuJoCo's defaults stops after 100 iterations or at 1e-8 on a linearly converging
# path that fp32 and fp64 walk differently.  Measured (r3) over the contact-rich states:
# qpos median 9e-8 / max 2.1e-6 (1 substep), 5.9e-5 (3 substeps); qvel / scale median
# 1.1e-6, max 2.8e-5
CG_QPOS_MAX, CG_QVEL_MAX = 4e-5, 1e-4
