import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdx.so on the device)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


@pytest.fixture(scope="session")
def reorient_compiled():
    from dexterity_amd.mjcf.compiler import CompiledModel

    return CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))


@pytest.fixture(scope="session")
def reach_compiled():
    from dexterity_amd.mjcf.compiler import CompiledModel

    return CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reach.npz"))


@pytest.fixture(scope="session")
def adroit_compiled():
    from dexterity_amd.mjcf.compiler import CompiledModel

    return CompiledModel.load(os.path.join(ROOT, "assets", "adroit_reach.npz"))


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_host.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


def random_hand_state(compiled, rng, frac=0.5, vel=0.5):
    """qpos within `frac` of every joint range (reach.py:40), small random qvel."""
    qpos = compiled.qpos0.copy()
    for j in range(compiled.njnt):
        if compiled.jnt_type[j] == 3 and compiled.jnt_limited[j]:
            lo, hi = compiled.jnt_range[j]
            qpos[compiled.jnt_qposadr[j]] = rng.uniform(frac * lo, frac * hi)
    qvel = rng.uniform(-vel, vel, size=compiled.nv)
    return qpos, qvel
