"""Effectors: the action boundary (effector.py:8-34, effectors/*.py in the reference).

`Effector.set_control` is where the reference writes `physics.bind(actuators).ctrl`
(effectors/mujoco_actuation.py:30-33).  Here the write is a device-to-device copy
into the batch's ctrl array (or, inside `dx_env_step`, a fused copy in the task
pre-kernel); MuJoCo's internal ctrl clamping is done by the step kernel.
"""

from __future__ import annotations

import abc
import re
from typing import List, Sequence

import numpy as np

from dexterity_amd import _lib
from dexterity_amd.specs import BoundedArray, merge_specs


class Effector(abc.ABC):
    @abc.abstractmethod
    def action_spec(self, physics) -> BoundedArray: ...

    @abc.abstractmethod
    def set_control(self, physics, command) -> None: ...

    @property
    @abc.abstractmethod
    def prefix(self) -> str: ...

    def after_compile(self, mjcf_model) -> None:
        del mjcf_model

    def initialize_episode(self, physics, random_state) -> None:
        del physics, random_state


def create_action_spec(compiled, actuator_ids: Sequence[int], prefix: str = "") -> BoundedArray:
    """mujoco_actuation.py:48-67: bounds from ctrlrange where ctrllimited, else +-inf."""
    n = len(actuator_ids)
    names = [f"{prefix}{i}" for i in range(n)]
    lo = np.full(n, -np.inf, dtype=np.float32)
    hi = np.full(n, np.inf, dtype=np.float32)
    rng = compiled.actuator_ctrlrange[list(actuator_ids)]
    lim = compiled.actuator_ctrllimited[list(actuator_ids)].astype(bool)
    lo[lim], hi[lim] = rng[lim].T
    return BoundedArray((n,), np.float32, lo, hi, name="\t".join(names))


class MujocoEffector(Effector):
    """A generic effector over a set of actuators (mujoco_actuation.py:11-46)."""

    def __init__(self, actuator_ids: Sequence[int], prefix: str = ""):
        self._ids = list(actuator_ids)
        self._prefix = prefix
        self._spec = None

    def action_spec(self, physics) -> BoundedArray:
        if self._spec is None:
            self._spec = create_action_spec(physics.model.compiled, self._ids, self._prefix)
        return self._spec

    def set_control(self, physics, command) -> None:
        """physics.bind(actuators).ctrl = command (mujoco_actuation.py:30-33), batched:
        command is [B, len(actuators)].  An effector over every actuator in order (the
        hand effector of every suite task) writes ctrl straight to the device; a subset
        reads the other actuators' ctrl back first."""
        command = np.asarray(command, dtype=np.float32)
        nu = physics.model.nu
        if self._ids == list(range(nu)):
            physics.set(_lib.CTRL, command.reshape(physics.nenv, nu))
            return
        ctrl = physics.get(_lib.CTRL)
        ctrl[:, self._ids] = command.reshape(ctrl.shape[0], -1)
        physics.set(_lib.CTRL, ctrl)

    @property
    def prefix(self) -> str:
        return self._prefix


class HandEffector(Effector):
    """effectors/hand_effector.py:11-36: prefix `<hand_name>_joint`."""

    def __init__(self, actuator_ids: Sequence[int], hand_name: str):
        self._prefix = f"{hand_name}_joint"
        self._mujoco_effector = MujocoEffector(actuator_ids, prefix=self._prefix)

    def action_spec(self, physics) -> BoundedArray:
        return self._mujoco_effector.action_spec(physics)

    def set_control(self, physics, command) -> None:
        self._mujoco_effector.set_control(physics, command)

    @property
    def prefix(self) -> str:
        return self._mujoco_effector.prefix


def find_effector_indices(effector: Effector, action_spec: BoundedArray) -> List[bool]:
    """task.py:39-45: which entries of the merged action belong to an effector."""
    names = action_spec.name.split("\t")
    expr = re.compile(effector.prefix)
    return [re.match(expr, n) is not None for n in names]


__all__ = ["Effector", "MujocoEffector", "HandEffector", "create_action_spec", "find_effector_indices", "merge_specs"]
