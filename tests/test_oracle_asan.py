"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5's
race / memory-error detection, host side: GPU sanitizers are not available on this pool).

oracle/Makefile's asan-driver target compiles dx_oracle.c into an instrumented executable
(oracle/asan_driver.c), which steps each shipped scene -- and the headline scene with
each solver -- from qpos0 through contact-rich control steps; any sanitizer report fails
the run, and the qpos checksum must equal the uninstrumented library's."""

import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def driver():
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    subprocess.run(["make", "-s", "-C", ORACLE, "asan-driver"], check=True, capture_output=True)
    return os.path.join(ORACLE, "_build", "asan_driver")


def _scenes():
    from dexterity_amd.mjcf.compiler import CompiledModel

    rc = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    return [
        ("reorient", rc, 5),
        ("reorient_cg", rc.with_solver("CG"), 5),
        ("reorient_pgs", rc.with_solver("PGS"), 5),
        ("bimanual", CompiledModel.load(os.path.join(ROOT, "assets", "bimanual_handover.npz")), 5),
        ("adroit_reach", CompiledModel.load(os.path.join(ROOT, "assets", "adroit_reach.npz")), 1),
    ]


@pytest.mark.parametrize("scene", ["reorient", "reorient_cg", "reorient_pgs", "bimanual", "adroit_reach"])
def test_oracle_clean_under_sanitizers(driver, oracle_mod, tmp_path, scene):
    from dexterity_amd import blob

    name, cm, nsub = next(s for s in _scenes() if s[0] == scene)
    data = blob.pack(cm.arrays)
    path = tmp_path / f"{name}.blob"
    path.write_bytes(data)
    nstep = 24
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:abort_on_error=0:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([driver, str(path), str(nstep), str(nsub)], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    rc, total, ncon, nefc = r.stdout.split()
    # the same sequence on the uninstrumented library (-O2, OpenMP build)
    om = oracle_mod.OracleModel(data)
    d = oracle_mod.OracleData(om)
    for s in range(nstep):
        d.ctrl[:] = 0.5 * np.sin(0.7 * s + 1.3 * np.arange(cm.nu))
        for _ in range(nsub):
            d.step()
    assert int(rc) == 0
    np.testing.assert_allclose(float(total), float(np.sum(d.qpos)), rtol=1e-9, atol=1e-12)
    if scene.startswith("reorient") or scene == "bimanual":
        assert int(ncon) > 0  # the run went through the contact and solver code
