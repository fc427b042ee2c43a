"""Batched fingertip inverse kinematics: the counterpart of
`dexterity/inverse_kinematics/ik_solver.py` (IKSolver) and
`dexterity/controllers/dls/dls.py` (DampedLeastSquaresMapper), run on the GPU.

`IKSolver.solve` keeps the reference's signature, defaults, errors and return value
(a joint vector, or None when no attempt reaches `linear_tol`).  `solve_batch`
solves one target set per environment of a batch in one call: every (env,
attempt) pair is one wavefront of `dx_ik_kernel` (dexterity_amd/csrc/dx_ik.hip).
There is no CPU fallback: without libdx.so the constructor raises DxError.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from dexterity_amd import _lib, hands, physics
from dexterity_amd.mjcf.compiler import CompiledModel

# ik_solver.py:16-29
_LINEAR_VELOCITY_GAIN = 0.95
_INTEGRATION_TIMESTEP_SEC = 1.0  # the device integrates over exactly 1 s
_REGULARIZATION_WEIGHT = 1e-5
_PROGRESS_THRESHOLD = 20.0


@dataclass
class IKResult:
    """Per-env outcome of `IKSolver.solve_batch`."""

    qpos: np.ndarray        # [B, njoint] solved joints (the last attempt's when not successful)
    success: np.ndarray     # [B] bool: some attempt had every fingertip within linear_tol
    linear_err: np.ndarray  # [B, nsite] fingertip errors of the returned joints
    attempt: np.ndarray     # [B] index of the returned attempt
    steps: np.ndarray       # [B] integration steps of the returned attempt


def hand_elements(compiled: CompiledModel, hand: str):
    """(fingertip site ids, hand joint ids) of `hand` ("adroit" or "shadow") in a compiled
    scene: DexterousHand.fingertip_sites / .joints (adroit_hand.py, shadow_hand_e.py)."""
    sites, joints = compiled.names["site"], compiled.names["joint"]
    if hand == "adroit":
        prefix, tips = "adroit_hand/", [s for s in hands.ADROIT_FINGERTIP_SITES]
    elif hand == "shadow":
        prefix, tips = "shadow_hand_e/", [f"{t}_site" for t in hands.SHADOW_FINGERTIPS]
    else:
        raise ValueError(f"unknown hand {hand!r}")
    site_ids = [sites.index(prefix + t) for t in tips]
    joint_ids = [joints.index(prefix + j) for j in hands.SHADOW_JOINTS]
    return site_ids, joint_ids


class IKSolver:
    """Inverse kinematics solver for a dexterous hand (ik_solver.py:40-69), batched.

    `model` is a `physics.Model` of a scene holding the hand; `sites` / `joints`
    default to the hand's fingertip sites and joints (`hand_elements`).  The joints
    not solved for (e.g. a prop's free joint) stay at the batch's qpos, which starts
    at qpos0 and can be set through `self.physics`.
    """

    def __init__(self, model: physics.Model, hand: str = "adroit", num_envs: int = 1, device: int = 0,
                 sites: Optional[Sequence[int]] = None, joints: Optional[Sequence[int]] = None):
        dsites, djoints = hand_elements(model.compiled, hand) if sites is None or joints is None else (None, None)
        self.sites = np.asarray(dsites if sites is None else sites, dtype=np.int32)
        self.joints = np.asarray(djoints if joints is None else joints, dtype=np.int32)
        self.model = model
        self.physics = physics.BatchedPhysics(model, num_envs, device)
        rng = model.compiled.jnt_range[self.joints]
        self.joint_range = np.asarray(rng, dtype=np.float64)
        # ik_solver.py:57-58: the midrange of the joints is the nullspace reference
        self._nullspace_reference = self.joint_range.mean(axis=1)

    @property
    def num_envs(self) -> int:
        return self.physics.nenv

    def close(self):
        self.physics.close()

    def solve_batch(self, target_positions: np.ndarray, linear_tol: float = 1e-3, max_steps: int = 100,
                    early_stop: bool = False, num_attempts: int = 30,
                    stop_on_first_successful_attempt: bool = False, seed: int = 0) -> IKResult:
        """One IK problem per env: target_positions [B, nsite, 3] (or [B, 3 * nsite])."""
        B, ns = self.num_envs, len(self.sites)
        t = np.asarray(target_positions, dtype=np.float32).reshape(B, -1)
        if t.shape[1] != 3 * ns:
            raise ValueError("The number of target positions must be equal to the number of end-effector sites.")
        t = np.ascontiguousarray(t)
        opt = _lib.IkOptions(linear_tol, _REGULARIZATION_WEIGHT, _LINEAR_VELOCITY_GAIN, _PROGRESS_THRESHOLD,
                             int(max_steps), int(early_stop), int(num_attempts),
                             int(stop_on_first_successful_attempt), int(seed))
        nj = len(self.joints)
        qpos = np.zeros((B, nj), np.float32)
        ok = np.zeros(B, np.int32)
        err = np.zeros((B, ns), np.float32)
        att = np.zeros(B, np.int32)
        steps = np.zeros(B, np.int32)
        _lib.check(_lib.load().dx_ik_solve(
            self.physics.ptr, ctypes.byref(opt), self.sites.ctypes.data, ns, self.joints.ctypes.data, nj,
            t.ctypes.data, qpos.ctypes.data, ok.ctypes.data, err.ctypes.data, att.ctypes.data, steps.ctypes.data))
        return IKResult(qpos, ok.astype(bool), err, att, steps)

    def solve(self, target_positions: np.ndarray, linear_tol: float = 1e-3, max_steps: int = 100,
              early_stop: bool = False, num_attempts: int = 30,
              stop_on_first_successful_attempt: bool = False, seed: int = 0) -> Optional[np.ndarray]:
        """IKSolver.solve (ik_solver.py:71-167) for env 0: the joint vector or None."""
        target_positions = np.asarray(target_positions).reshape(-1, 3)
        if target_positions.shape[0] != len(self.sites):
            raise ValueError(
                "The number of target positions must be equal to the number of end-effector sites.")
        t = np.broadcast_to(target_positions.reshape(1, -1), (self.num_envs, target_positions.size))
        r = self.solve_batch(t, linear_tol, max_steps, early_stop, num_attempts,
                             stop_on_first_successful_attempt, seed)
        return r.qpos[0].astype(np.float64) if r.success[0] else None
