"""fp64 restatement of the reference's per-step task arithmetic -- TEST INFRASTRUCTURE ONLY.

Used by tests/ to check dx_task.hip.  Each function cites the reference it follows.
`tanh_squared` / `weighted_average` are pinned to the reference's own outputs
(tests/golden/reference_host.json); the quaternion helpers restate
[3P] dm_robotics.transformations (absent here) and are pinned only by the KAT of
reorient_test.py:13-50.
"""

from __future__ import annotations

import numpy as np


def tanh_squared(x, margin: float, loss_at_margin: float = 0.95) -> float:
    """manipulation/shared/rewards.py:18-28."""
    if not margin > 0:
        raise ValueError("`margin` must be positive.")
    if not 0.0 < loss_at_margin < 1.0:
        raise ValueError("`loss_at_margin` must be between 0 and 1.")
    error = np.linalg.norm(x)
    w = np.arctanh(np.sqrt(loss_at_margin)) / margin
    s = np.tanh(w * error)
    return s * s


def weighted_average(components) -> float:
    """manipulation/shared/rewards.py:13-15 over (value, weight) pairs."""
    return sum(v * w for v, w in components)


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
        w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
    ])


def quat_conj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def quat_diff_active(source_quat, target_quat):
    """[3P] dm_robotics: q such that target = q * source."""
    return quat_mul(target_quat, quat_conj(source_quat))


def quat_to_axisangle(quat):
    """[3P] dm_robotics: axis * angle with the angle wrapped to [-pi, pi]."""
    quat = np.asarray(quat, dtype=np.float64)
    angle = 2 * np.arccos(np.clip(quat[0], -1.0, 1.0))
    if angle < 1e-12:
        return np.zeros(3)
    qn = np.sin(angle / 2)
    angle = (angle + np.pi) % (2 * np.pi) - np.pi
    return quat[1:4] / qn * angle


def goal_distance(goal, current) -> float:
    """manipulation/goals/prop_orientation.py:40-50."""
    err = quat_diff_active(current, goal)
    return float(np.linalg.norm(quat_to_axisangle(err)))


def uniform_quaternion(rng) -> np.ndarray:
    """Shoemake's uniform unit quaternion ([3P] dm_control rotations.UniformQuaternion)."""
    u1, u2, u3 = rng.uniform(size=3)
    a, b = np.sqrt(1 - u1), np.sqrt(u1)
    return np.array([b * np.cos(2 * np.pi * u3), a * np.sin(2 * np.pi * u2), a * np.cos(2 * np.pi * u2),
                     b * np.sin(2 * np.pi * u3)])


def shaped_reorientation_reward(distance: float, ctrl) -> dict:
    """reorient.py:238-284 -> {name: (value, weight)}."""
    return {
        "orientation": (1.0 / (distance + 0.1), 1.0),
        "success_bonus": (1.0 if 0.0 <= distance <= 0.1 else 0.0, 800.0),  # tolerance(bounds=(0,.1), margin=0)
        "action_smoothing": (np.linalg.norm(ctrl) ** 2, -0.1),
    }


def reorient_reward(distance: float, ctrl) -> float:
    """reorient.py:215-220."""
    return weighted_average(shaped_reorientation_reward(distance, ctrl).values())


def fingertip_distances(goal, tips):
    """FingertipCartesianPosition.goal_distance (fingertip_position.py:127-137)."""
    return np.linalg.norm(np.asarray(goal, float).reshape(-1, 3) - np.asarray(tips, float).reshape(-1, 3), axis=1)


def reach_reward(goal, tips, dense: bool = True, threshold: float = 0.01) -> float:
    """Reach.get_reward (reach.py:196-210)."""
    d = fingertip_distances(goal, tips)
    if dense:
        return float(np.mean(np.where(d <= threshold, 0.0, [-tanh_squared(x, margin=0.1) for x in d])))
    return float(np.mean(np.where(d <= threshold, 0.0, -1.0)))
