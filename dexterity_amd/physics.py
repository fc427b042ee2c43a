"""Batched physics handle: the MI355X counterpart of dm_control's `mjcf.Physics`.

One `BatchedPhysics` owns B environments that share a compiled model and live in
HBM.  The methods mirror the parts of `mjcf.Physics` the reference uses on its hot
path: `step()` (composer substep loop, reorient.py:168 /
reach.py:139), `forward()`, and reads/writes of qpos / qvel / ctrl /
xfrc_applied / site xpos / contacts -- every one batched over environments.
"""

from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from dexterity_amd import _lib
from dexterity_amd import blob as blob_lib
from dexterity_amd.mjcf.compiler import CompiledModel


class Model:
    """A compiled scene loaded into libdx (shared by any number of batches)."""

    def __init__(self, compiled: CompiledModel):
        self.compiled = compiled
        self.blob = blob_lib.pack(compiled.arrays)
        L = _lib.load()
        self.ptr = L.dx_model_load(self.blob, len(self.blob))
        if not self.ptr:
            raise _lib.DxError(f"dx_model_load failed: {L.dx_last_error().decode()}")
        sizes = (ctypes.c_int32 * 12)()
        _lib.check(L.dx_model_sizes(self.ptr, sizes))
        (self.nq, self.nv, self.nbody, self.njnt, self.ngeom, self.nsite, self.nu,
         self.ntendon, self.nbpair, self.ngpair, self.ncon_max, self.nefc_max) = list(sizes)
        self.lds_bytes = _lib.check(L.dx_model_lds_bytes(self.ptr))

    @staticmethod
    def from_file(path: str) -> "Model":
        return Model(CompiledModel.load(path))

    def width(self, field: int) -> int:
        return _lib.check(_lib.load().dx_field_width(self.ptr, field))

    def __del__(self):
        if getattr(self, "ptr", None) and _lib._lib is not None:
            _lib._lib.dx_model_free(self.ptr)
            self.ptr = None


class BatchedPhysics:
    """B environments on one GPU; state resident in HBM."""

    def __init__(self, model: Model, nenv: int, device: int = 0):
        L = _lib.load()
        self.model = model
        self.nenv = int(nenv)
        self.device = device
        self.ptr = L.dx_batch_create(model.ptr, self.nenv, device)
        self._owned = True
        if not self.ptr:
            raise _lib.DxError(f"dx_batch_create failed: {L.dx_last_error().decode()}")

    @classmethod
    def borrowed(cls, model: Model, ptr: int, nenv: int, device: int) -> "BatchedPhysics":
        """A view of a batch owned elsewhere (e.g. by a dx_env); never destroyed here."""
        self = cls.__new__(cls)
        self.model, self.ptr, self.nenv, self.device, self._owned = model, ptr, int(nenv), device, False
        return self

    def close(self):
        if getattr(self, "ptr", None) and getattr(self, "_owned", False) and _lib._lib is not None:
            _lib._lib.dx_batch_destroy(self.ptr)
        self.ptr = None

    def __del__(self):
        self.close()

    # ------------------------------------------------------------------ #
    def step(self, nsubstep: int = 1) -> None:
        _lib.check(_lib.load().dx_step(self.ptr, nsubstep))

    def forward(self) -> None:
        _lib.check(_lib.load().dx_forward(self.ptr))

    def sync(self) -> None:
        _lib.check(_lib.load().dx_sync(self.ptr))

    def reset(self, env0: int = 0, n: Optional[int] = None) -> None:
        n = self.nenv - env0 if n is None else n
        _lib.check(_lib.load().dx_reset(self.ptr, env0, n))

    # ------------------------------------------------------------------ #
    def set(self, field: int, values, env0: int = 0) -> None:
        w = self.model.width(field)
        a = np.ascontiguousarray(values, dtype=np.float32).reshape(-1, w)
        _lib.check(_lib.load().dx_set_field(self.ptr, field, a.ctypes.data, env0, a.shape[0]))
        self.sync()  # host buffer must outlive the async copy

    def set_device(self, field: int, devptr: int, env0: int, n: int) -> None:
        """Device-to-device copy from a raw device pointer (no host sync)."""
        _lib.check(_lib.load().dx_set_field(self.ptr, field, ctypes.c_void_p(devptr), env0, n))

    def get(self, field: int, env0: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.nenv - env0 if n is None else n
        w = self.model.width(field)
        dt = np.int32 if field in _lib.INT_FIELDS else np.float32
        out = np.empty((n, w), dtype=dt)
        _lib.check(_lib.load().dx_get_field(self.ptr, field, out.ctypes.data, env0, n))
        return out

    def field_ptr(self, field: int) -> int:
        p = ctypes.c_void_p()
        _lib.check(_lib.load().dx_field_ptr(self.ptr, field, ctypes.byref(p)))
        return p.value

    def set_xfrc(self, xfrc) -> None:
        a = None if xfrc is None else np.ascontiguousarray(xfrc, dtype=np.float32).reshape(-1, 6)
        if a is None:
            _lib.check(_lib.load().dx_set_xfrc(self.ptr, None, 0))
        else:
            _lib.check(_lib.load().dx_set_xfrc(self.ptr, a.ctypes.data, a.shape[0]))
        self.sync()

    def set_watch(self, geom: int, body: int) -> None:
        _lib.check(_lib.load().dx_set_watch(self.ptr, geom, body))

    def jac_site(self, sites, rotational: bool = True):
        """mj_jacSite for every env at its current qpos (utils/mujoco_utils.py:38-73,
        compute_object_6d_jacobian): (jacp, jacr) of shape [B, nsite, 3, nv]."""
        s = np.ascontiguousarray(sites, dtype=np.int32).reshape(-1)
        shape = (self.nenv, len(s), 3, self.model.nv)
        jp = np.empty(shape, np.float32)
        jr = np.empty(shape, np.float32) if rotational else None
        _lib.check(_lib.load().dx_jac_site(self.ptr, s.ctypes.data, len(s), jp.ctypes.data,
                                           None if jr is None else jr.ctypes.data))
        return jp, jr

    def enable_sensors(self, enable: bool = True) -> None:
        """Joint torque sensors (DX_SENSOR_TORQUE) computed by every step / forward."""
        _lib.check(_lib.load().dx_sensor_enable(self.ptr, int(enable)))

    def joint_torques(self, joints, axes) -> np.ndarray:
        """`DexterousHandObservables.joint_torques` (dexterous_hand.py:266-275): each
        joint's 3-axis torque sensor (a site at its body origin) projected on the
        joint axis; joints are (body id) per joint, axes [njoint, 3] in the body frame."""
        s = self.get(_lib.SENSOR_TORQUE).reshape(self.nenv, -1, 3)
        bodies = np.asarray(joints, dtype=int)
        return np.einsum("ejk,jk->ej", s[:, bodies, :], np.asarray(axes, dtype=np.float64))

    def debug(self, enable: bool = True) -> None:
        _lib.check(_lib.load().dx_debug_enable(self.ptr, int(enable)))

    def health(self) -> dict:
        """The always-on health counters (include/dx.h dx_health): capacity overflows,
        diverged env-substeps, the most contacts one env-substep found and, when
        `ncon_histogram(True)` is on, the histogram of contacts per env-substep."""
        out = np.zeros(_lib.HEALTH_WORDS + _lib.NCON_HIST, dtype=np.uint32)
        _lib.check(_lib.load().dx_health(self.ptr, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), out.size))
        h = {k: int(out[i]) for i, k in enumerate(_lib.HEALTH)}
        h["ncon_hist"] = out[_lib.HEALTH_WORDS:].astype(np.int64)
        return h

    def health_clear(self) -> None:
        _lib.check(_lib.load().dx_health_clear(self.ptr))

    def ncon_histogram(self, enable: bool = True) -> None:
        _lib.check(_lib.load().dx_ncon_histogram(self.ptr, int(enable)))

    def debug_get(self, name: str) -> np.ndarray:
        nv = self.model.nv
        sizes = {
            "qacc_smooth": (self.nenv, nv),
            "qfrc_smooth": (self.nenv, nv),
            "M": (self.nenv, nv, nv),
            "contact": (self.nenv, self.model.ncon_max, 16),
            "efc_count": (self.nenv, 2),
        }
        if name in ("queue_timeouts", "queue_slots"):
            out = np.zeros(1, dtype=np.int32)
            _lib.check(_lib.load().dx_debug_get(self.ptr, name.encode(), out.ctypes.data, 1))
            return out
        shape = sizes[name]
        out = np.empty(shape, dtype=np.float32)
        _lib.check(_lib.load().dx_debug_get(self.ptr, name.encode(), out.ctypes.data, out.size))
        if name == "efc_count":
            return out.view(np.int32)
        return out

    # convenience views (host copies)
    @property
    def qpos(self) -> np.ndarray:
        return self.get(_lib.QPOS)

    @property
    def qvel(self) -> np.ndarray:
        return self.get(_lib.QVEL)

    @property
    def qacc(self) -> np.ndarray:
        return self.get(_lib.QACC)


def gravity_compensation(compiled: CompiledModel, prefix: str) -> np.ndarray:
    """xfrc_applied rows = -m_b g for bodies whose name starts with prefix.

    utils/mujoco_utils.py:91-99 (called from shadow_hand_e.py:35-41 and
    adroit_hand.py:30-36 in initialize_episode).
    """
    xfrc = np.zeros((compiled.nbody, 6))
    for i, n in enumerate(compiled.names["body"]):
        if n.startswith(prefix):
            xfrc[i, :3] = -compiled.gravity * compiled.body_mass[i]
    return xfrc
