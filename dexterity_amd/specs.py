"""Minimal dm_env-compatible specs and TimeStep (dm_env is not installed here).

Mirrors the parts of `dm_env` the reference's API surface returns:
`specs.Array`, `specs.BoundedArray` (effectors/mujoco_actuation.py:48-67,
prop_orientation.py:22-23) and `TimeStep` / `StepType` (environment.py:14-34).
Every field of a batched TimeStep carries a leading environment axis.
"""

from __future__ import annotations

import enum
from typing import Any, NamedTuple

import numpy as np


class Array:
    def __init__(self, shape, dtype, name: str = ""):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.name = name

    def validate(self, value):
        value = np.asarray(value)
        if value.shape != self.shape:
            raise ValueError(f"{self.name}: expected shape {self.shape}, got {value.shape}")
        return value

    def generate_value(self):
        return np.zeros(self.shape, dtype=self.dtype)

    def __repr__(self):
        return f"Array(shape={self.shape}, dtype={self.dtype}, name={self.name!r})"


class BoundedArray(Array):
    def __init__(self, shape, dtype, minimum, maximum, name: str = ""):
        super().__init__(shape, dtype, name)
        self.minimum = np.broadcast_to(np.asarray(minimum, dtype=self.dtype), self.shape).copy()
        self.maximum = np.broadcast_to(np.asarray(maximum, dtype=self.dtype), self.shape).copy()

    def validate(self, value):
        value = super().validate(value)
        if np.any(value < self.minimum) or np.any(value > self.maximum):
            raise ValueError(f"{self.name}: values out of bounds")
        return value

    def __repr__(self):
        return f"BoundedArray(shape={self.shape}, dtype={self.dtype}, name={self.name!r})"


class StepType(enum.IntEnum):
    FIRST = 0
    MID = 1
    LAST = 2


class TimeStep(NamedTuple):
    """Batched dm_env.TimeStep: step_type/reward/discount are [nenv] arrays."""

    step_type: Any
    reward: Any
    discount: Any
    observation: Any

    def first(self):
        return np.asarray(self.step_type) == StepType.FIRST

    def mid(self):
        return np.asarray(self.step_type) == StepType.MID

    def last(self):
        return np.asarray(self.step_type) == StepType.LAST


def merge_specs(action_specs):
    """utils/spec_utils.py:10-37: concatenate bounded action specs, names tab-joined."""
    mins = np.concatenate([s.minimum for s in action_specs])
    maxs = np.concatenate([s.maximum for s in action_specs])
    name = "\t".join(s.name for s in action_specs)
    return BoundedArray(mins.shape, action_specs[0].dtype, mins, maxs, name=name)
