"""Generates tests/golden/reference_host.json from the reference's importable modules.

Run where /root/reference exists:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Only the reference's pure-numpy modules import here (their package __init__s pull
dm_control, which is absent), so they are loaded by file path -- SURVEY.md §8 c2.
The output is data (inputs and the reference's outputs); the GPU box and the test
suite read only the JSON.
"""

from __future__ import annotations

import dataclasses
import importlib.util
import json
import os
import sys

import numpy as np

REF = os.environ.get("DEXTERITY_REFERENCE", "/root/reference")
PKG = os.path.join(REF, "dexterity")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_host.json")


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(PKG, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    sys.path.insert(0, REF)  # `import dexterity` (for _SRC_ROOT) only imports pathlib
    rewards = _load("ref_rewards", "manipulation/shared/rewards.py")
    shadow = _load("ref_shadow_consts", "models/hands/shadow_hand_e_constants.py")
    adroit = _load("ref_adroit_consts", "models/hands/adroit_hand_constants.py")
    obs = _load("ref_observations", "manipulation/shared/observations.py")

    rng = np.random.RandomState(12345)
    xs = np.concatenate([[0.0, 0.01, 0.05, 0.1, 0.2, 1.0], rng.uniform(0, 0.3, size=26)])
    margins = [0.1, 0.05, 0.2]
    tanh = [
        {"x": float(x), "margin": m, "value": float(rewards.tanh_squared(x, margin=m))}
        for x in xs
        for m in margins
    ]
    vecs = rng.uniform(-0.1, 0.1, size=(8, 3))
    tanh_vec = [
        {"x": v.tolist(), "margin": 0.1, "value": float(rewards.tanh_squared(v, margin=0.1))}
        for v in vecs
    ]
    Reward = rewards.Reward
    comps = {"a": Reward(2.0, 0.5), "b": Reward(-1.5, 800.0), "c": Reward(0.25, -0.1)}
    wavg = float(rewards.weighted_average(comps))

    golden = {
        "source": "reference modules loaded by file path: manipulation/shared/rewards.py, "
        "models/hands/shadow_hand_e_constants.py, models/hands/adroit_hand_constants.py, "
        "manipulation/shared/observations.py",
        "tanh_squared": tanh,
        "tanh_squared_vector": tanh_vec,
        "weighted_average": {"components": [[2.0, 0.5], [-1.5, 800.0], [0.25, -0.1]], "value": wavg},
        "shadow": {
            "joints": list(shadow.JOINTS),
            "actuators": list(shadow.ACTUATORS),
            "fingertips": list(shadow.FINGERTIP_NAMES),
            "position_to_control": shadow.POSITION_TO_CONTROL.tolist(),
            "control_to_position": shadow.CONTROL_TO_POSITION.tolist(),
            "coupled_joint_ids": shadow.COUPLED_JOINT_IDS,
            "actuator_joint_mapping": {k: list(v) for k, v in shadow.ACTUATOR_JOINT_MAPPING.items()},
        },
        "adroit": {
            "joints": list(adroit.JOINTS),
            "actuators": list(adroit.ACTUATORS),
            "fingertip_sites": list(adroit.FINGERTIP_SITE_NAMES),
        },
        "observations": {
            "hand_observables": dataclasses.asdict(obs.HAND_OBSERVABLES),
            "state_only_options": {
                k: (dataclasses.asdict(v) if dataclasses.is_dataclass(v) else dict(v))
                for k, v in obs.make_options(obs.ObservationSet.STATE_ONLY.value, obs.HAND_OBSERVABLES).items()
            },
        },
    }
    with open(OUT, "w") as f:
        json.dump(golden, f, indent=1, default=str)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
