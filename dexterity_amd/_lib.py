"""ctypes binding of libdx.so (include/dx.h).

The library is built in-tree (`dexterity_amd/libdx.so`, see `build.py`).  There is
deliberately no fallback: if the HIP library is missing or cannot reach a GPU,
every entry point raises.
"""

from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DX_LIB") or os.path.join(_HERE, "libdx.so")  # DX_LIB: A/B-test a variant build

# dx_field
QPOS, QVEL, CTRL, QACC_WARMSTART, QACC, TIME = 0, 1, 2, 3, 4, 5
SITE_XPOS, SITE_VEL, XPOS, XQUAT, NCON, GROUND_CONTACT, NITER, NCAND, STEP_COST = 6, 7, 8, 9, 10, 11, 12, 13, 14
SENSOR_TORQUE, DIVERGED = 15, 16
INT_FIELDS = (NCON, GROUND_CONTACT, NITER, NCAND, STEP_COST, DIVERGED)
HEALTH_WORDS, NCON_HIST = 16, 65
HEALTH = ("contact_overflow", "candidate_overflow", "jacobian_dof_overflow", "row_overflow", "diverged",
          "ncon_max", "contact_deferred", "mid_tier_gave_up", "deferred_behind_launch")

EXPORTS = (
    "dx_model_load", "dx_model_free", "dx_model_sizes", "dx_model_lds_bytes", "dx_field_width",
    "dx_batch_create", "dx_batch_destroy", "dx_batch_nenv", "dx_reset",
    "dx_set_field", "dx_get_field", "dx_field_ptr", "dx_set_xfrc", "dx_set_ground_geom",
    "dx_set_watch", "dx_step", "dx_forward", "dx_stream", "dx_sync",
    "dx_debug_enable", "dx_debug_get", "dx_last_error", "dx_abi_version",
    "dx_env_create", "dx_env_destroy", "dx_env_batch", "dx_env_obs_dim", "dx_env_reset",
    "dx_env_step", "dx_env_output", "dx_env_action_buffer", "dx_env_sample_actions",
    "dx_env_pack_outputs", "dx_timing_enable", "dx_timing_read", "dx_stage_timing", "dx_stage_read",
    "dx_debug_poison_lds", "dx_hull_support", "dx_model_layout", "dx_env_goal_dim",
    "dx_jac_site", "dx_ik_solve",
    "dx_comm_unique_id", "dx_comm_init", "dx_comm_destroy", "dx_comm_rank", "dx_comm_size",
    "dx_allgather_obs", "dx_comm_allreduce_max", "dx_comm_barrier", "dx_sensor_enable",
    "dx_env_set_time_limit", "dx_set_outputs", "dx_env_create_shard",
    "dx_health", "dx_health_clear", "dx_ncon_histogram", "dx_env_set_goal_time_limit",
    "dx_env_step_random", "dx_env_save", "dx_env_load", "dx_env_state_field", "dx_env_step_host",
    "dx_build_key",
)
COMM_ID_BYTES = 128
STAGES = ("kinematics", "crb", "broadphase", "midphase", "narrowphase", "constraints", "velocity",
          "smooth_solve", "newton_eval", "newton_grad", "newton_hessian", "newton_chol", "newton_linesearch",
          "qfrc_constraint", "euler", "observe", "io", "matvec", "np_mpr", "jacvec")
COUNTERS = {20: "plane_box", 21: "plane_convex", 22: "capsule", 23: "mpr", 24: "mpr_support", 25: "mpr_hit",
            26: "mpr_maxit", 27: "newton_iter", 28: "linesearch_iter", 29: "solves", 30: "nefc",
            31: "np_trips", 32: "broad_keep", 33: "mid_pairs", 34: "mid_keep", 35: "queue_wait"}
NSTAGE = 48
# the narrowphase trip's parts (DX_NP_MARKS builds only)
NP_STAGES = {36: "np_loop", 37: "np_fresh", 38: "np_supload", 39: "np_supred", 40: "np_portal"}
OUT_OBS, OUT_REWARD, OUT_DISCOUNT, OUT_STEP_TYPE, OUT_GOAL, OUT_SUCCESSES, OUT_GOAL_FAILURES, OUT_GOAL_QPOS = range(8)
TASK_REORIENT, TASK_REACH, TASK_HANDOVER = 0, 1, 2
REACH_NPARAMS_HEAD = 26

_lib = None


class DxError(RuntimeError):
    pass


class IkOptions(ctypes.Structure):
    """struct dx_ik_options (include/dx.h)."""

    _fields_ = [
        ("linear_tol", ctypes.c_float),
        ("regularization", ctypes.c_float),
        ("gain", ctypes.c_float),
        ("progress_threshold", ctypes.c_float),
        ("max_steps", ctypes.c_int32),
        ("early_stop", ctypes.c_int32),
        ("num_attempts", ctypes.c_int32),
        ("stop_on_first", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
    ]


def load(path: str = LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DxError(
            f"{path} not found: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')"
        )
    L = ctypes.CDLL(path)
    if hasattr(L, "dx_build_key"):
        L.dx_build_key.restype = ctypes.c_char_p
    if path == os.path.join(_HERE, "libdx.so") and os.path.isdir(os.path.join(_HERE, "csrc")):
        # the in-tree library must have been built from the sources beside it (a GPU box
        # runs the library that travelled with the tree, without rebuilding)
        from dexterity_amd import build as _build

        want, have = _build.source_key(), L.dx_build_key().decode()
        if want != have:
            raise DxError(f"{path} was built from other sources (key {have}, sources {want}): rebuild it "
                          "(python -c 'import __graft_entry__ as g; g.build()')")
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_size_t
    L.dx_model_load.restype = vp
    L.dx_model_load.argtypes = [ctypes.c_char_p, sz]
    L.dx_model_free.argtypes = [vp]
    L.dx_model_sizes.argtypes = [vp, ctypes.POINTER(i32)]
    L.dx_model_lds_bytes.argtypes = [vp]
    L.dx_field_width.argtypes = [vp, ctypes.c_int]
    L.dx_model_layout.argtypes = [vp, ctypes.POINTER(i32), i32]
    L.dx_hull_support.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(i32)]
    L.dx_batch_create.restype = vp
    L.dx_batch_create.argtypes = [vp, i32, i32]
    L.dx_batch_destroy.argtypes = [vp]
    L.dx_batch_nenv.argtypes = [vp]
    L.dx_reset.argtypes = [vp, i32, i32]
    L.dx_set_field.argtypes = [vp, ctypes.c_int, vp, i32, i32]
    L.dx_get_field.argtypes = [vp, ctypes.c_int, vp, i32, i32]
    L.dx_field_ptr.argtypes = [vp, ctypes.c_int, ctypes.POINTER(vp)]
    L.dx_set_xfrc.argtypes = [vp, vp, i32]
    L.dx_set_ground_geom.argtypes = [vp, i32]
    L.dx_set_watch.argtypes = [vp, i32, i32]
    L.dx_step.argtypes = [vp, i32]
    L.dx_forward.argtypes = [vp]
    L.dx_stream.restype = vp
    L.dx_stream.argtypes = [vp]
    L.dx_sync.argtypes = [vp]
    L.dx_debug_enable.argtypes = [vp, ctypes.c_int]
    L.dx_sensor_enable.argtypes = [vp, ctypes.c_int]
    L.dx_set_outputs.argtypes = [vp, ctypes.c_int]
    L.dx_debug_get.argtypes = [vp, ctypes.c_char_p, vp, sz]
    L.dx_last_error.restype = ctypes.c_char_p
    L.dx_abi_version.restype = ctypes.c_int
    L.dx_env_create.restype = vp
    L.dx_env_create.argtypes = [vp, i32, i32, i32, ctypes.c_uint64, vp, i32]
    L.dx_health.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), i32]
    L.dx_health_clear.argtypes = [vp]
    L.dx_ncon_histogram.argtypes = [vp, ctypes.c_int]
    L.dx_env_create_shard.restype = vp
    L.dx_env_create_shard.argtypes = [vp, i32, i32, i32, ctypes.c_uint64, ctypes.c_int64, vp, i32]
    L.dx_env_destroy.argtypes = [vp]
    L.dx_env_batch.restype = vp
    L.dx_env_batch.argtypes = [vp]
    L.dx_env_obs_dim.argtypes = [vp]
    L.dx_env_goal_dim.argtypes = [vp]
    L.dx_env_reset.argtypes = [vp]
    L.dx_env_step.argtypes = [vp, vp]
    L.dx_env_set_time_limit.argtypes = [vp, ctypes.c_double]
    L.dx_env_set_goal_time_limit.argtypes = [vp, ctypes.c_double]
    L.dx_env_output.argtypes = [vp, ctypes.c_int, ctypes.POINTER(vp)]
    L.dx_env_action_buffer.argtypes = [vp, ctypes.POINTER(vp)]
    L.dx_env_sample_actions.argtypes = [vp, ctypes.c_uint64, i32]
    L.dx_env_step_random.argtypes = [vp, ctypes.c_uint64, i32]
    L.dx_env_save.argtypes = [vp, vp, sz]
    L.dx_env_load.argtypes = [vp, vp, sz]
    L.dx_env_state_field.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz),
                                     ctypes.POINTER(sz)]
    L.dx_env_pack_outputs.argtypes = [vp, vp]
    if hasattr(L, "dx_env_step_host"):  # (round 6; an older variant library for A/B lacks it)
        L.dx_env_step_host.argtypes = [vp, vp, vp]
    L.dx_timing_enable.argtypes = [vp, ctypes.c_int]
    L.dx_timing_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]
    L.dx_stage_timing.argtypes = [vp, ctypes.c_int]
    L.dx_stage_read.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), i32]
    L.dx_debug_poison_lds.argtypes = [i32]
    L.dx_jac_site.argtypes = [vp, vp, i32, vp, vp]
    L.dx_ik_solve.argtypes = [vp, ctypes.POINTER(IkOptions), vp, i32, vp, i32, vp, vp, vp, vp, vp, vp]
    L.dx_comm_unique_id.argtypes = [vp]
    L.dx_comm_init.restype = vp
    L.dx_comm_init.argtypes = [ctypes.c_char_p, i32, i32, i32]
    L.dx_comm_destroy.argtypes = [vp]
    L.dx_comm_rank.argtypes = [vp]
    L.dx_comm_size.argtypes = [vp]
    L.dx_allgather_obs.argtypes = [vp, vp, vp]
    L.dx_comm_allreduce_max.argtypes = [vp, ctypes.POINTER(ctypes.c_double)]
    L.dx_comm_barrier.argtypes = [vp]
    _lib = L
    return L


def check(rc: int) -> int:
    if rc < 0:
        raise DxError(f"libdx error {rc}: {load().dx_last_error().decode()}")
    return rc
