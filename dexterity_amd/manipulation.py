"""Task suite and batched environments (manipulation/__init__.py in the reference).

`load(domain, task, seed, num_envs, device)` mirrors `manipulation.load`
(manipulation/__init__.py:56-86) and returns a `GoalEnvironment` whose
`reset()` / `step(action)` follow dm_env semantics for every one of `num_envs`
environments at once (batched TimeStep, leading env axis).  The physics and the
task logic run on the GPU (dx_env_* in include/dx.h); these classes hold the
reference's constants and the host-side API.

Suite (names as in the reference):
  reorient.state_dense   manipulation/tasks/reorient.py:367-371  (Shadow hand + cube)
  reach.state_dense      manipulation/tasks/reach.py:252-259     (Adroit hand, fingertip goals)
  reach.state_sparse     manipulation/tasks/reach.py:262-269
  reach_shadow.state_dense  BASELINE.json config 2: reach with the Shadow hand,
                         contact-free smooth dynamics (not a reference suite entry)
  bimanual.state_dense   BASELINE.json config 5: two Shadow hands hand the cube over
                         (Handover; not a reference suite entry)
"""

from __future__ import annotations

import collections
import ctypes
import dataclasses
import os
from typing import Dict, Optional

import numpy as np

from dexterity_amd import _lib
from dexterity_amd import effectors as effectors_lib
from dexterity_amd import hands as hands_lib
from dexterity_amd import physics as physics_lib
from dexterity_amd.mjcf.compiler import CompiledModel
from dexterity_amd.specs import Array, BoundedArray, StepType, TimeStep

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


@dataclasses.dataclass(frozen=True)
class ReOrientConfig:
    """Constants of manipulation/tasks/reorient.py:40-78 and GoalTask defaults."""

    physics_timestep: float = 0.005  # reorient.py:58
    control_timestep: float = 0.025  # reorient.py:61
    orientation_eps: float = 0.1  # reorient.py:50
    orientation_threshold: float = 0.1  # reorient.py:52
    orientation_weight: float = 1.0  # reorient.py:54
    success_bonus_weight: float = 800.0  # reorient.py:55
    action_smoothing_weight: float = -0.1  # reorient.py:56
    successes_needed: int = 1  # reorient.py:64
    max_steps_single_solve: int = 300  # reorient.py:67
    steps_before_moving_target: int = 5  # reorient.py:70
    fall_termination: bool = True  # reorient.py:103
    prop_bbox_lower: tuple = (-0.025, -0.155, 0.16)  # reorient.py:72-78
    prop_bbox_upper: tuple = (0.025, -0.105, 0.16)

    @property
    def n_sub_steps(self) -> int:
        return int(round(self.control_timestep / self.physics_timestep))

    @property
    def max_time_per_goal(self) -> float:
        return self.max_steps_single_solve * self.control_timestep


def observation_layout(hand_nq: int, hand_nv: int, ntips: int, with_prop: bool, hand: str,
                       goal_dim: int = 4) -> "collections.OrderedDict[str, slice]":
    """Named slices of the flat observation vector written by dx_task_post_kernel."""
    out = collections.OrderedDict()
    k = 0

    def add(name, n):
        nonlocal k
        out[name] = slice(k, k + n)
        k += n

    add(f"{hand}/joint_positions_sin_cos", 2 * hand_nq)
    add(f"{hand}/joint_velocities", hand_nv)
    add(f"{hand}/fingertip_positions", 3 * ntips)
    add(f"{hand}/fingertip_linear_velocities", 3 * ntips)
    if with_prop:
        add("prop/position", 3)
        add("prop/orientation", 4)
        add("prop/linear_velocity", 3)
        add("prop/angular_velocity", 3)
        add("target_prop/orientation", 4)
    add("goal_state", goal_dim)
    return out


class ReOrient:
    """Batched counterpart of `ReOrient` (reorient.py:90-235)."""

    domain = "reorient"
    kind = _lib.TASK_REORIENT

    def __init__(self, config: ReOrientConfig = ReOrientConfig(), asset: str = "shadow_reorient.npz"):
        self.config = config
        self.compiled = CompiledModel.load(os.path.join(ASSETS, asset))
        cm = self.compiled
        if abs(cm.timestep - config.physics_timestep) > 1e-12:
            raise ValueError("asset timestep does not match the task's physics timestep")
        self.hand_name = "shadow_hand_e"
        names = cm.names
        self.hand_joint_ids = [i for i, n in enumerate(names["joint"]) if n.startswith(self.hand_name + "/")]
        self.hand_nq = len(self.hand_joint_ids)
        self.hand_nv = self.hand_nq
        prop_j = names["joint"].index("prop/")
        self.prop_qadr = int(cm.jnt_qposadr[prop_j])
        self.prop_dadr = int(cm.jnt_dofadr[prop_j])
        self.prop_body = names["body"].index("prop/")
        self.ground_geom = names["geom"].index("ground")
        tip_sites = [f"{self.hand_name}/{t}_site" for t in ("fftip", "mftip", "rftip", "lftip", "thtip")]
        self.tip_site0 = names["site"].index(tip_sites[0])
        assert [names["site"].index(s) for s in tip_sites] == list(range(self.tip_site0, self.tip_site0 + 5))
        self.ntips = 5
        self.actuator_ids = list(range(cm.nu))
        self.hand_effector = effectors_lib.HandEffector(self.actuator_ids, self.hand_name)
        self.gravity_compensation = physics_lib.gravity_compensation(cm, self.hand_name + "/")

    def params(self) -> np.ndarray:
        c = self.config
        p = np.zeros(38, dtype=np.float32)
        p[0] = c.n_sub_steps
        p[1], p[2] = self.hand_nq, self.hand_nv
        p[3], p[4] = self.prop_qadr, self.prop_dadr
        p[5], p[6] = self.tip_site0, self.ntips
        p[7], p[8], p[9] = c.successes_needed, c.steps_before_moving_target, int(c.fall_termination)
        p[10], p[11] = c.orientation_threshold, c.orientation_eps
        p[12], p[13], p[14] = c.orientation_weight, c.success_bonus_weight, c.action_smoothing_weight
        p[15] = c.max_time_per_goal
        p[16:19] = c.prop_bbox_lower
        p[19:22] = c.prop_bbox_upper
        p[22], p[23] = self.ground_geom, self.prop_body
        # the box in fp64 for the numpy-compatible spawn draws: raw bits in 26-37
        box = np.array(c.prop_bbox_lower + c.prop_bbox_upper, dtype=np.float64)
        p[26:38] = box.view(np.float32)
        return p

    def observation_layout(self):
        return observation_layout(self.hand_nq, self.hand_nv, self.ntips, True, self.hand_name)


@dataclasses.dataclass(frozen=True)
class HandoverConfig:
    """BASELINE.json config 5 as a task (synthetic: the reference has no bimanual task; its
    two-hand pattern is Juggle's hands and effectors, juggle.py:147-177 with
    arenas/arena.py:58-105).  Two Shadow hands palm-up side by side (mjcf/scenes.py
    bimanual_handover), the reorient cube spawned over the first (left) hand and handed to
    the target point above the other palm; GoalTask bookkeeping, reward in the shape of
    reorient.py:238-284 on the cube-to-target distance, fall termination of
    reorient.py:229-235.  Timesteps as reorient's."""

    physics_timestep: float = 0.005
    control_timestep: float = 0.025
    distance_eps: float = 0.05  # 1 / (d + eps), d in metres
    success_threshold: float = 0.02  # the cube within 2 cm of the receiving palm's target
    distance_weight: float = 1.0
    success_bonus_weight: float = 800.0  # reorient.py:55
    action_smoothing_weight: float = -0.1  # reorient.py:56
    successes_needed: int = 3  # handovers (there and back, and there again)
    max_steps_single_solve: int = 300  # reorient.py:67
    steps_before_moving_target: int = 5  # task.py's goal change: the cube goes back
    fall_termination: bool = True
    # the reorient spawn box (reorient.py:72-78) over the left hand (+0.12 m in x)
    prop_bbox_lower: tuple = (0.095, -0.155, 0.16)
    prop_bbox_upper: tuple = (0.145, -0.105, 0.16)
    # where the cube comes to rest on each palm from the spawn box's centre (the fp64
    # oracle: 0.1308 m high, 0.13 m in front of the forearms), left then right
    hand_targets: tuple = ((0.12, -0.13, 0.131), (-0.12, -0.13, 0.131))

    @property
    def n_sub_steps(self) -> int:
        return int(round(self.control_timestep / self.physics_timestep))

    @property
    def max_time_per_goal(self) -> float:
        return self.max_steps_single_solve * self.control_timestep


class Handover(ReOrient):
    """The two-hand cube handover behind the Task / Effector / Environment surface
    (HandoverConfig).  Both hands' joints, velocities and fingertips are the hand block of
    the observation (left then right, as the scene orders them), then the cube's pose and
    velocities and the goal [target xyz, receiving hand]."""

    domain = "bimanual"
    kind = _lib.TASK_HANDOVER

    def __init__(self, config: HandoverConfig = HandoverConfig(), asset: str = "bimanual_handover.npz"):
        self.config = config
        self.compiled = CompiledModel.load(os.path.join(ASSETS, asset))
        cm = self.compiled
        if abs(cm.timestep - config.physics_timestep) > 1e-12:
            raise ValueError("asset timestep does not match the task's physics timestep")
        names = cm.names
        self.hand_names = ("shadow_hand_left", "shadow_hand_right")
        self.hand_name = "bimanual"
        self.hand_joint_ids = [i for i, n in enumerate(names["joint"]) if n.startswith("shadow_hand_")]
        self.hand_nq = len(self.hand_joint_ids)
        self.hand_nv = self.hand_nq
        prop_j = names["joint"].index("prop/")
        self.prop_qadr = int(cm.jnt_qposadr[prop_j])
        self.prop_dadr = int(cm.jnt_dofadr[prop_j])
        if self.prop_qadr != self.hand_nq:  # the hands' joints first, then the cube's
            raise ValueError("bimanual scene: hand joints must precede the prop's")
        self.prop_body = names["body"].index("prop/")
        self.ground_geom = names["geom"].index("ground")
        tips = [f"{h}/{t}_site" for h in self.hand_names for t in ("fftip", "mftip", "rftip", "lftip", "thtip")]
        self.tip_site0 = names["site"].index(tips[0])
        assert [names["site"].index(s) for s in tips] == list(range(self.tip_site0, self.tip_site0 + 10))
        self.ntips = 10
        self.actuator_ids = list(range(cm.nu))
        self.hand_effector = effectors_lib.HandEffector(self.actuator_ids, self.hand_name)
        self.gravity_compensation = physics_lib.gravity_compensation(cm, "shadow_hand_")

    def params(self) -> np.ndarray:
        c = self.config
        p = np.zeros(44, dtype=np.float32)
        p[0] = c.n_sub_steps
        p[1], p[2] = self.hand_nq, self.hand_nv
        p[3], p[4] = self.prop_qadr, self.prop_dadr
        p[5], p[6] = self.tip_site0, self.ntips
        p[7], p[8], p[9] = c.successes_needed, c.steps_before_moving_target, int(c.fall_termination)
        p[10], p[11] = c.success_threshold, c.distance_eps
        p[12], p[13], p[14] = c.distance_weight, c.success_bonus_weight, c.action_smoothing_weight
        p[15] = c.max_time_per_goal
        p[16:19] = c.prop_bbox_lower
        p[19:22] = c.prop_bbox_upper
        p[22], p[23] = self.ground_geom, self.prop_body
        box = np.array(c.prop_bbox_lower + c.prop_bbox_upper, dtype=np.float64)
        p[26:38] = box.view(np.float32)
        p[38:44] = np.asarray(c.hand_targets, dtype=np.float32).ravel()
        return p

    def observation_layout(self):
        """Per-hand keys: the scene orders the left hand's joints, dofs and fingertips
        before the right's, so each hand's block is a contiguous slice."""
        out = collections.OrderedDict()
        nh, k = self.hand_nq // 2, 0
        blocks = (("joint_positions_sin_cos", 2 * nh), ("joint_velocities", nh), ("fingertip_positions", 15),
                  ("fingertip_linear_velocities", 15))
        for name, n in blocks:
            for h in self.hand_names:
                out[f"{h}/{name}"] = slice(k, k + n)
                k += n
        for name, n in (("prop/position", 3), ("prop/orientation", 4), ("prop/linear_velocity", 3),
                        ("prop/angular_velocity", 3), ("goal_state", 4)):
            out[name] = slice(k, k + n)
            k += n
        return out


@dataclasses.dataclass(frozen=True)
class ReachConfig:
    """Constants of manipulation/tasks/reach.py:30-70 and fingertip_position.py:21-35."""

    physics_timestep: float = 0.02  # reach.py:54
    control_timestep: float = 0.02  # reach.py:59
    success_threshold: float = 0.01  # reach.py:47 (_DISTANCE_TO_TARGET_THRESHOLD)
    successes_needed: int = 50  # reach.py:62
    steps_before_moving_target: int = 5  # reach.py:37
    max_steps_single_solve: int = 150  # reach.py:65
    init_joint_range_fraction: float = 0.5  # reach.py:34
    goal_scale: float = 0.1  # fingertip_position.py:26
    max_rejection_samples: int = 100  # fingertip_position.py:25
    dense_reward: bool = True  # reach.py:252-269 (state_dense / state_sparse)

    @property
    def n_sub_steps(self) -> int:
        return int(round(self.control_timestep / self.physics_timestep))

    @property
    def max_time_per_goal(self) -> float:
        return self.max_steps_single_solve * self.control_timestep


class Reach:
    """Batched counterpart of `Reach` (reach.py:73-210) over `GoalTask`.

    Goals come from the batched `FingertipCartesianPosition.next_goal`
    (fingertip_position.py:72-125: joint targets ~ N(midrange, 0.1 * range), two
    physics steps, rejected while the hand self-collides) and episodes start from
    `sample_collision_free_joint_angles(range_fraction=0.5)` (dexterous_hand.py:
    120-168); both run on the device inside the step kernel (dx_step.hip reach_prep).
    """

    domain = "reach"
    kind = _lib.TASK_REACH

    def __init__(self, config: ReachConfig = ReachConfig(), hand: str = "adroit"):
        self.config = config
        asset = {"adroit": "adroit_reach.npz", "shadow": "shadow_reach.npz"}[hand]
        self.compiled = CompiledModel.load(os.path.join(ASSETS, asset))
        cm = self.compiled
        if abs(cm.timestep - config.physics_timestep) > 1e-12:
            raise ValueError("asset timestep does not match the task's physics timestep")
        names = cm.names
        if hand == "adroit":
            self.hand_name = "adroit_hand"
            tips = [f"{self.hand_name}/{s}" for s in hands_lib.ADROIT_FINGERTIP_SITES]
            self.position_to_control = np.eye(cm.nu, cm.nq)  # adroit_hand.py:106-112
            coupled = []
        else:
            self.hand_name = "shadow_hand_e"
            tips = [f"{self.hand_name}/{t}_site" for t in hands_lib.SHADOW_FINGERTIPS]
            self.position_to_control = hands_lib.POSITION_TO_CONTROL  # shadow_hand_e.py:109-119
            coupled = [(ids[0], ids[-1]) for ids in hands_lib.COUPLED_JOINT_IDS]  # shadow_hand_e.py:124-129
        self.tip_sites = [names["site"].index(t) for t in tips]
        self.coupled = coupled
        self.hand_nq = cm.nq
        self.hand_nv = cm.nv
        self.ntips = len(self.tip_sites)
        self.actuator_ids = list(range(cm.nu))
        self.hand_effector = effectors_lib.HandEffector(self.actuator_ids, self.hand_name)
        # FingertipCartesianPosition.initialize_episode (fingertip_position.py:55-62)
        self.gravity_compensation = physics_lib.gravity_compensation(cm, self.hand_name + "/")
        rng = np.asarray(cm.arrays["jnt_range"], dtype=np.float64).reshape(-1, 2)[: cm.nq]
        self.joint_range = rng

    def params(self) -> np.ndarray:
        c, cm = self.config, self.compiled
        head = np.zeros(_lib.REACH_NPARAMS_HEAD, dtype=np.float32)
        head[0] = c.n_sub_steps
        head[1], head[2], head[3] = self.hand_nq, self.hand_nv, self.ntips
        head[4:4 + self.ntips] = self.tip_sites
        head[9], head[10] = c.successes_needed, c.steps_before_moving_target
        head[11], head[12] = c.success_threshold, c.max_time_per_goal
        head[13] = 1.0 if c.dense_reward else 0.0
        head[14], head[15], head[16] = c.init_joint_range_fraction, c.goal_scale, c.max_rejection_samples
        head[17] = len(self.coupled)
        for k, (j, src) in enumerate(self.coupled):
            head[18 + 2 * k], head[19 + 2 * k] = j, src
        lo, hi = self.joint_range[:, 0], self.joint_range[:, 1]
        mid = self.joint_range.mean(axis=1)  # fingertip_position.py:80-82
        tail = np.concatenate([mid, lo, hi, np.asarray(self.position_to_control, dtype=np.float64).ravel()])
        assert tail.size == 3 * cm.nq + cm.nu * cm.nq
        # fp64 draw constants, as the reference computes them (raw bits): the goal's
        # normal(loc=midrange, scale=0.1 * range) and clip (fingertip_position.py:67-86),
        # the initial joints' uniform(range_fraction * limits) (dexterous_hand.py:137-142)
        f64 = np.concatenate([mid, c.goal_scale * (hi - lo), lo, hi, c.init_joint_range_fraction * lo,
                              c.init_joint_range_fraction * hi]).astype(np.float64)
        return np.concatenate([head, tail.astype(np.float32), f64.view(np.float32)])

    def observation_layout(self):
        return observation_layout(self.hand_nq, self.hand_nv, self.ntips, False, self.hand_name, 3 * self.ntips)


class GoalEnvironment:
    """Batched `GoalEnvironment` (environment.py:9-34) over `num_envs` environments.

    `step(action)` accepts a host array [num_envs, nu] or, with `device_action=True`,
    the integer address of a device buffer; outputs stay on the device unless read
    through `timestep()` / `observation()`.
    """

    def __init__(self, task: ReOrient, num_envs: int, seed: Optional[int] = None, device: int = 0,
                 time_limit: Optional[float] = None, strip_singleton_obs_buffer_dim: bool = True,
                 env_offset: int = 0):
        self.task = task
        self.num_envs = int(num_envs)
        # this batch's env e is env env_offset + e of the job (a shard of a sharded
        # job, dexterity_amd.distributed.env_shard); it draws from seed + env_offset + e
        self.env_offset = int(env_offset)
        # composer.Environment(time_limit=..., strip_singleton_obs_buffer_dim=...)
        # (manipulation/__init__.py:81-86): `time_limit or task.time_limit`, so None and 0
        # both mean the task's own limit, inf for every suite task
        self.time_limit = float(time_limit) if time_limit else float("inf")
        self.strip_singleton_obs_buffer_dim = bool(strip_singleton_obs_buffer_dim)
        self.model = physics_lib.Model(task.compiled)
        L = _lib.load()
        p = task.params()
        self._seed = 0 if seed is None else int(seed)
        self.ptr = L.dx_env_create_shard(self.model.ptr, self.num_envs, device, task.kind,
                                         self._seed, self.env_offset, p.ctypes.data, len(p))
        if not self.ptr:
            raise _lib.DxError(f"dx_env_create_shard failed: {L.dx_last_error().decode()}")
        batch_ptr = L.dx_env_batch(self.ptr)
        self.physics = physics_lib.BatchedPhysics.borrowed(self.model, batch_ptr, self.num_envs, device)
        # gravity compensation (shadow_hand_e.py:35-41 in initialize_episode)
        self.physics.set_xfrc(task.gravity_compensation)
        self.obs_dim = _lib.check(L.dx_env_obs_dim(self.ptr))
        self.goal_dim = _lib.check(L.dx_env_goal_dim(self.ptr))
        self._layout = task.observation_layout()
        self._action_spec = task.hand_effector.action_spec(self.physics)
        self._host_action = np.zeros((self.num_envs, self.model.nu), dtype=np.float32)
        self._dev_action = self._out(-1)
        self._pins = []  # page-locked host buffers of step() (freed by close)
        self._pin_act = self._pin_out = None
        if np.isfinite(self.time_limit):
            _lib.check(L.dx_env_set_time_limit(self.ptr, self.time_limit))
        # max_time_per_goal in fp64 (the params carry it as a float)
        _lib.check(L.dx_env_set_goal_time_limit(self.ptr, float(task.config.max_time_per_goal)))

    def close(self):
        for p in getattr(self, "_pins", ()):
            _hip_runtime().hipHostFree(ctypes.c_void_p(p))
        self._pins = []
        self._pin_act = self._pin_out = None
        if getattr(self, "physics", None) is not None:
            self.physics.ptr = None
        if getattr(self, "ptr", None) and _lib._lib is not None:
            _lib._lib.dx_env_destroy(self.ptr)
        self.ptr = None

    def __del__(self):
        self.close()

    def _out(self, which: int) -> int:
        p = ctypes.c_void_p()
        L = _lib.load()
        if which < 0:
            _lib.check(L.dx_env_action_buffer(self.ptr, ctypes.byref(p)))
        else:
            _lib.check(L.dx_env_output(self.ptr, which, ctypes.byref(p)))
        return p.value

    # ---------------------------------------------------------------- specs
    def action_spec(self) -> BoundedArray:
        return self._action_spec

    def observation_spec(self) -> "collections.OrderedDict[str, Array]":
        lead = () if self.strip_singleton_obs_buffer_dim else (1,)
        return collections.OrderedDict(
            (k, Array(lead + (s.stop - s.start,), np.float64, name=k)) for k, s in self._layout.items()
        )

    # ---------------------------------------------------------------- stepping
    def reset(self) -> TimeStep:
        _lib.check(_lib.load().dx_env_reset(self.ptr))
        return self.timestep(first=True)

    def step(self, action, device_action: bool = False) -> Optional[TimeStep]:
        L = _lib.load()
        if device_action:
            _lib.check(L.dx_env_step(self.ptr, ctypes.c_void_p(int(action))))
            return None
        a = np.asarray(action, dtype=np.float32).reshape(self.num_envs, -1)
        if a.shape[1] != self.model.nu:
            raise ValueError(f"action must be [{self.num_envs}, {self.model.nu}], got {a.shape}")
        # the reference's call shape (environment.py:25-34): host actions in, the host
        # TimeStep out, through page-locked buffers -- dx_env_step_host uploads them into
        # the library's action buffer (the step kernel writes ctrl from it:
        # mujoco_actuation.py:33), steps, packs [obs | reward | discount | step_type] and
        # downloads it, all on the env's stream with one synchronisation
        if self._pin_act is None:
            self._pin_act = _pinned((self.num_envs, self.model.nu), np.float32, self._pins)
            self._pin_out = _pinned((self.num_envs, self.obs_dim + 3), np.float32, self._pins)
        np.copyto(self._pin_act, a)
        _lib.check(L.dx_env_step_host(self.ptr, self._pin_act.ctypes.data, self._pin_out.ctypes.data))
        return self._timestep_packed(self._pin_out)

    def _timestep_packed(self, packed: np.ndarray) -> TimeStep:
        """A TimeStep (copies) from the packed [obs | reward | discount | step_type] rows."""
        d = self.obs_dim
        observation = collections.OrderedDict(
            (k, packed[:, s].astype(np.float64) if self.strip_singleton_obs_buffer_dim
             else packed[:, None, s].astype(np.float64)) for k, s in self._layout.items()
        )
        return TimeStep(packed[:, d + 2].astype(np.int32), packed[:, d].astype(np.float64),
                        packed[:, d + 1].astype(np.float64), observation)

    def step_random(self, step: int) -> None:
        """One control step under the random agent: the actions `sample_actions(step)`
        would draw (manipulation_test.py:44-45), drawn inside the step kernel."""
        _lib.check(_lib.load().dx_env_step_random(self.ptr, self._seed, step))

    def sample_actions(self, step: int) -> int:
        """Fills the device action buffer with uniform actions; returns its address."""
        _lib.check(_lib.load().dx_env_sample_actions(self.ptr, self._seed, step))
        return self._dev_action

    # ---------------------------------------------------------------- checkpoint
    # dtype of the state fields that are not float32 (include/dx.h dx_env_save)
    _STATE_DTYPES = {"nstep": np.int32, "diverged": np.int32, "successes": np.int32, "counter": np.int32,
                     "registered": np.int32, "exceeded": np.int32, "step_type": np.int32, "episode": np.int32,
                     "skip": np.int32, "failure": np.int32, "need": np.int32, "goalnum": np.int32,
                     "goalfail": np.int32, "time_d": np.float64, "solve_start_d": np.float64,
                     "nsub_d": np.int32, "solve_n": np.int32, "mt_env": np.uint32, "mt_goal": np.uint32,
                     "mt_reach": np.uint32, "step_cost": np.uint32, "order": np.int32}

    def _state_fields(self):
        L = _lib.load()
        name, off, nb = ctypes.c_char_p(), ctypes.c_size_t(), ctypes.c_size_t()
        n = _lib.check(L.dx_env_state_field(self.ptr, -1, ctypes.byref(name), ctypes.byref(off), ctypes.byref(nb)))
        out = []
        for i in range(n):
            _lib.check(L.dx_env_state_field(self.ptr, i, ctypes.byref(name), ctypes.byref(off), ctypes.byref(nb)))
            out.append((name.value.decode(), off.value, nb.value))
        return out

    def save(self, path: str) -> None:
        """Checkpoint every env's state (physics, task, RNG streams, dispatch order) to an
        .npz of named [num_envs, ...] arrays (SURVEY.md §5 checkpoint / resume); `load`
        into an env of the same task and size continues the run bit for bit."""
        L = _lib.load()
        nbytes = _lib.check(L.dx_env_save(self.ptr, None, 0))
        buf = np.empty(nbytes, dtype=np.uint8)
        _lib.check(L.dx_env_save(self.ptr, buf.ctypes.data, nbytes))
        arrays = {}
        for name, off, nb in self._state_fields():
            a = buf[off:off + nb].view(self._STATE_DTYPES.get(name, np.float32))
            arrays[name] = a.reshape(self.num_envs, -1) if name not in ("mt_env", "mt_goal") else a.reshape(-1, self.num_envs)
        meta = np.array([self.num_envs, self.model.nq, self.model.nv, self.model.nu, self.obs_dim, self.env_offset],
                        dtype=np.int64)
        # the random agent's key (dx_env_step_random / sample_actions draw from it), so a
        # load into an env created with another seed continues the same action stream
        np.savez(path, __meta__=meta, __agent_seed__=np.array([self._seed], dtype=np.int64), **arrays)

    def load(self, path: str) -> None:
        """Restores a checkpoint written by `save` (same task, model and num_envs),
        including the random agent's key."""
        L = _lib.load()
        with np.load(path, allow_pickle=False) as z:
            meta = z["__meta__"]
            want = [self.num_envs, self.model.nq, self.model.nv, self.model.nu, self.obs_dim, self.env_offset]
            if list(meta) != want:
                raise ValueError(f"checkpoint is for (num_envs, nq, nv, nu, obs_dim, env_offset) = {list(meta)}, "
                                 f"this env is {want}")
            if "__agent_seed__" in z.files:
                self._seed = int(z["__agent_seed__"][0])
            fields = self._state_fields()
            nbytes = sum(nb for _, _, nb in fields)
            buf = np.empty(nbytes, dtype=np.uint8)
            for name, off, nb in fields:
                a = np.ascontiguousarray(z[name])
                if a.nbytes != nb:
                    raise ValueError(f"checkpoint field {name}: {a.nbytes} bytes, expected {nb}")
                buf[off:off + nb] = a.view(np.uint8).ravel()
        self.physics.sync()
        _lib.check(L.dx_env_load(self.ptr, buf.ctypes.data, nbytes))

    def _read(self, which: int, dtype, width: int) -> np.ndarray:
        out = np.empty((self.num_envs, width), dtype=dtype)
        ptr = self._out(which)
        self.physics.sync()
        _copy_d2h(out, ptr)
        return out

    def timestep(self, first: bool = False) -> TimeStep:
        obs = self._read(_lib.OUT_OBS, np.float32, self.obs_dim)
        st = self._read(_lib.OUT_STEP_TYPE, np.int32, 1)[:, 0]
        rew = self._read(_lib.OUT_REWARD, np.float32, 1)[:, 0].astype(np.float64)
        disc = self._read(_lib.OUT_DISCOUNT, np.float32, 1)[:, 0].astype(np.float64)
        # an observation buffer of size 1 per observable (dm_control observation
        # updater); kept as [B, 1, n] unless strip_singleton_obs_buffer_dim
        observation = collections.OrderedDict(
            (k, obs[:, s].astype(np.float64) if self.strip_singleton_obs_buffer_dim
             else obs[:, None, s].astype(np.float64)) for k, s in self._layout.items()
        )
        return TimeStep(st.astype(np.int32), rew, disc, observation)

    def goals(self) -> np.ndarray:
        return self._read(_lib.OUT_GOAL, np.float32, self.goal_dim)

    def goal_qpos(self) -> np.ndarray:
        """Reach: the joints that placed each env's goal (FingertipCartesianPosition.qpos,
        fingertip_position.py:136-139)."""
        return self._read(_lib.OUT_GOAL_QPOS, np.float32, self.model.nq)

    def goal_failures(self) -> np.ndarray:
        return self._read(_lib.OUT_GOAL_FAILURES, np.int32, 1)[:, 0]

    def successes(self) -> np.ndarray:
        return self._read(_lib.OUT_SUCCESSES, np.int32, 1)[:, 0]


def _hip_runtime():
    """The HIP runtime libdx is linked against (for plain host<->device copies)."""
    global _hip
    if _hip is None:
        try:
            _hip = ctypes.CDLL("libamdhip64.so.7")
        except OSError:
            _hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
        _hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        _hip.hipHostFree.argtypes = [ctypes.c_void_p]
    return _hip


def _pinned(shape, dtype, owner: list) -> np.ndarray:
    """A page-locked host array (hipHostMalloc); its address is appended to `owner`."""
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    p = ctypes.c_void_p()
    rc = _hip_runtime().hipHostMalloc(ctypes.byref(p), nbytes, 0)
    if rc != 0 or not p.value:
        raise _lib.DxError(f"hipHostMalloc failed ({rc})")
    owner.append(p.value)
    buf = (ctypes.c_byte * nbytes).from_address(p.value)
    return np.frombuffer(buf, dtype=dtype).reshape(shape)


def _copy_d2h(out: np.ndarray, devptr: int) -> None:
    rc = _hip_runtime().hipMemcpy(out.ctypes.data, ctypes.c_void_p(devptr), out.nbytes, 2)  # DeviceToHost
    if rc != 0:
        raise _lib.DxError(f"hipMemcpy failed ({rc})")


def _copy_h2d(devptr: int, src: np.ndarray) -> None:
    rc = _hip_runtime().hipMemcpy(ctypes.c_void_p(devptr), src.ctypes.data, src.nbytes, 1)  # HostToDevice
    if rc != 0:
        raise _lib.DxError(f"hipMemcpy failed ({rc})")


_hip = None

SUITE = {
    ("reorient", "state_dense"): ReOrient,
    ("reach", "state_dense"): lambda: Reach(ReachConfig(dense_reward=True), hand="adroit"),
    ("reach", "state_sparse"): lambda: Reach(ReachConfig(dense_reward=False), hand="adroit"),
    ("reach_shadow", "state_dense"): lambda: Reach(ReachConfig(dense_reward=True), hand="shadow"),
    ("bimanual", "state_dense"): Handover,
}
ALL_TASKS = tuple(sorted(SUITE))
ALL_NAMES = [".".join(t) for t in ALL_TASKS]
# manipulation/__init__.py:53 (_get_tasks_by_domain)
TASKS_BY_DOMAIN = {d: tuple(t for dd, t in ALL_TASKS if dd == d) for d in sorted({d for d, _ in ALL_TASKS})}


def load(domain_name: str, task_name: str, seed: Optional[int] = None,
         strip_singleton_obs_buffer_dim: bool = True, time_limit: Optional[float] = None,
         num_envs: int = 1, device: int = 0, env_offset: int = 0) -> GoalEnvironment:
    """manipulation/__init__.py:56-86, batched: the reference's arguments in its order,
    then the batch size and the GPU.  `time_limit=None` keeps the task's own limit
    (inf for every suite task).  Env e of the batch is the reference's environment
    loaded with seed `seed + env_offset + e`; `env_offset` places a shard of a sharded
    job (distributed.env_shard) in the job's env numbering."""
    key = (domain_name, task_name)
    if domain_name not in {d for d, _ in SUITE}:
        raise ValueError(f"Unknown domain: {domain_name}")
    if key not in SUITE:
        raise ValueError(f"Unknown task: {task_name}")
    return GoalEnvironment(SUITE[key](), num_envs=num_envs, seed=seed, device=device, time_limit=time_limit,
                           strip_singleton_obs_buffer_dim=strip_singleton_obs_buffer_dim, env_offset=env_offset)


__all__ = ["load", "GoalEnvironment", "ReOrient", "ReOrientConfig", "Reach", "ReachConfig", "ALL_TASKS",
           "ALL_NAMES", "TASKS_BY_DOMAIN", "StepType"]
