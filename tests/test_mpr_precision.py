"""The full-batch parity accounting's "fp32 portal" rule, pinned on CPU by the states that
needed it (tests/golden/fullbatch_*_fp32_portal.npz: the states and the GPU's contact
records, dumped by test_full_batch_parity / test_bimanual_full_batch_parity on the GPU).

At a deep overlap of two curved hulls (or a box and a hull) fp32 and fp64 MPR stop on
different portals: another normal, a depth 4-11 % apart.  These tests show the kernel's
answer is the reference algorithm's answer in fp32, not a kernel defect:
  * the restated MPR (oracle/mpr_ref.py) in fp64 equals the C oracle's contact (1e-12);
  * the fp64 oracle is continuous in the state there (its answer moves < 1e-3 rad under
    fp32-scale perturbations of qpos): the difference is not an input discontinuity;
  * the restated MPR in fp32, from the geoms' poses perturbed at the fp32 forward
    kinematics' resolution, reproduces the GPU's contact to 1e-4 rad and 1e-4 of the depth.
"""
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
FIXTURES = [("fullbatch_reorient_fp32_portal.npz", "shadow_reorient.npz"),
            ("fullbatch_bimanual_fp32_portal.npz", "bimanual_handover.npz")]


def _deep_mismatches(oracle_mod, fixture, asset):
    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel

    cm = CompiledModel.load(os.path.join(ROOT, "assets", asset))
    om = oracle_mod.OracleModel(blob.pack(cm.arrays))
    z = np.load(os.path.join(GOLDEN, fixture))
    out = []
    for k, e in enumerate(z["ids"]):
        st = [np.asarray(z[f][k], dtype=np.float64) for f in ("qpos", "qvel", "ws", "ctrl")]
        d = oracle_mod.OracleData(om)
        d.xfrc_applied[:] = z["x32"]
        d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = st
        d.forward()
        oc = d.contacts()
        con = z["con"][k]
        for r in con[con[:, 15] != 0]:
            if abs(r[12]) <= 5e-4:
                continue
            m = (oc[:, 13] == r[13]) & (oc[:, 14] == r[14])
            assert m.any(), (e, r[13:15])
            o = oc[m][np.argmin(np.abs(oc[m][:, 0:3] - r[0:3]).max(axis=1))]
            if float(np.arccos(np.clip(o[3:6] @ r[3:6], -1, 1))) > 0.05:
                out.append((cm, om, z, k, st, d, o, r))
    return out


@pytest.mark.parametrize("fixture,asset", FIXTURES)
def test_fp32_portal_fixtures(oracle_mod, fixture, asset):
    from oracle.mpr_ref import fp32_reproduces, mpr, pair_inputs

    cases = _deep_mismatches(oracle_mod, fixture, asset)
    assert len(cases) >= 2
    for cm, om, z, k, st, d, o, r in cases:
        g1, g2 = int(r[13]), int(r[14])
        # the restatement in fp64 is the C oracle
        (p1, m1, v1, c1), (p2, m2, v2, c2), hm = pair_inputs(cm, d, g1, g2)
        res = mpr(p1, m1, v1, c1, p2, m2, v2, c2, hm, np.float64)
        assert abs((2 * hm - res[0]) - o[12]) <= 1e-12 and np.abs(res[1] - o[3:6]).max() <= 1e-12
        # the fp64 oracle is continuous here
        rng = np.random.RandomState(int(z["ids"][k]))
        for _ in range(24):
            dp = oracle_mod.OracleData(om)
            dp.xfrc_applied[:] = z["x32"]
            dp.qpos[:] = st[0] * (1 + rng.standard_normal(st[0].shape) * 1e-6)
            dp.qvel[:], dp.qacc_warmstart[:], dp.ctrl[:] = st[1:]
            dp.forward()
            pc = dp.contacts()
            pm = pc[(pc[:, 13] == g1) & (pc[:, 14] == g2)]
            q = pm[np.argmin(np.abs(pm[:, 0:3] - o[0:3]).max(axis=1))]
            assert float(np.arccos(np.clip(q[3:6] @ o[3:6], -1, 1))) < 1e-3
        # the fp32 evaluation of the same algorithm lands on the GPU's portal
        ok, ang, dr, draws = fp32_reproduces(cm, d, g1, g2, r)
        assert ok, (fixture, int(z["ids"][k]), g1, g2, ang, dr)
