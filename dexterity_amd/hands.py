"""Hand constants restated from the reference (models/hands/*_constants.py).

The joint / actuator orderings and the control<->joint projection matrices are
pinned against the reference's own values in tests/golden/reference_host.json
(tests/test_host_logic.py), the known-answer `P2C @ C2P == I` of
hands_test.py:26-31.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

# shadow_hand_e_constants.py:43-68
SHADOW_JOINTS: Tuple[str, ...] = (
    "WRJ1", "WRJ0",
    "FFJ3", "FFJ2", "FFJ1", "FFJ0",
    "MFJ3", "MFJ2", "MFJ1", "MFJ0",
    "RFJ3", "RFJ2", "RFJ1", "RFJ0",
    "LFJ4", "LFJ3", "LFJ2", "LFJ1", "LFJ0",
    "THJ4", "THJ3", "THJ2", "THJ1", "THJ0",
)
# shadow_hand_e_constants.py:90-111
SHADOW_ACTUATORS: Tuple[str, ...] = (
    "A_WRJ1", "A_WRJ0",
    "A_FFJ3", "A_FFJ2", "A_FFJ1",
    "A_MFJ3", "A_MFJ2", "A_MFJ1",
    "A_RFJ3", "A_RFJ2", "A_RFJ1",
    "A_LFJ4", "A_LFJ3", "A_LFJ2", "A_LFJ1",
    "A_THJ4", "A_THJ3", "A_THJ2", "A_THJ1", "A_THJ0",
)
# shadow_hand_e_constants.py:127-156: the J1 actuator of each finger drives J1+J0 via a tendon.
SHADOW_ACTUATOR_JOINTS: Dict[str, Tuple[str, ...]] = {
    a: ((a[2:],) if a[2:] not in ("FFJ1", "MFJ1", "RFJ1", "LFJ1") else (a[2:], a[2:4] + "J0"))
    for a in SHADOW_ACTUATORS
}
SHADOW_FINGERTIPS: Tuple[str, ...] = ("fftip", "mftip", "rftip", "lftip", "thtip")

# adroit_hand_constants.py: fully actuated, joint i <-> actuator i.
ADROIT_JOINTS: Tuple[str, ...] = SHADOW_JOINTS
ADROIT_ACTUATORS: Tuple[str, ...] = tuple("A_" + j for j in SHADOW_JOINTS)
ADROIT_FINGERTIP_SITES: Tuple[str, ...] = ("S_fftip", "S_mftip", "S_rftip", "S_lftip", "S_thtip")


def _projection() -> Tuple[np.ndarray, np.ndarray, List[List[int]]]:
    """shadow_hand_e_constants.py:162-187 restated."""
    nu, nj = len(SHADOW_ACTUATORS), len(SHADOW_JOINTS)
    p2c = np.zeros((nu, nj))
    c2p = np.zeros((nj, nu))
    coupled = []
    jid = {j: i for i, j in enumerate(SHADOW_JOINTS)}
    for a, act in enumerate(SHADOW_ACTUATORS):
        joints = SHADOW_ACTUATOR_JOINTS[act]
        ids = [jid[j] for j in joints]
        if len(ids) > 1:
            coupled.append(ids)
        p2c[a, ids] = 1.0
        c2p[ids, a] = 1.0 / len(ids)
    return p2c, c2p, coupled


POSITION_TO_CONTROL, CONTROL_TO_POSITION, COUPLED_JOINT_IDS = _projection()


def shadow_joint_positions_to_control(qpos: np.ndarray) -> np.ndarray:
    """shadow_hand_e.py:113-126 (batched over a leading axis)."""
    qpos = np.asarray(qpos)
    if qpos.shape[-1] != len(SHADOW_JOINTS):
        raise ValueError(f"Expected qpos of shape (..., {len(SHADOW_JOINTS)}), got {qpos.shape}")
    return qpos @ POSITION_TO_CONTROL.T


def shadow_control_to_joint_positions(control: np.ndarray) -> np.ndarray:
    """shadow_hand_e.py:100-111 (batched over a leading axis)."""
    control = np.asarray(control)
    if control.shape[-1] != len(SHADOW_ACTUATORS):
        raise ValueError(f"Expected control of shape (..., {len(SHADOW_ACTUATORS)}), got {control.shape}")
    return control @ CONTROL_TO_POSITION.T
