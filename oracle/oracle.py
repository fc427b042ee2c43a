"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, `__graft_entry__.smoke()` and bench.py's cpu_baseline leg.
Parity status: see dx_oracle.h (MuJoCo dynamics parity unpinned).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

NSTAGE = 8
STAGES = ("kinematics", "crb", "collision", "constraint", "smooth", "solver", "integrate", "scan")


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, sz, ip = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        dp = ctypes.POINTER(ctypes.c_double)
        L.dxo_model_load.restype = vp
        L.dxo_model_load.argtypes = [ctypes.c_char_p, sz]
        L.dxo_model_free.argtypes = [vp]
        L.dxo_data_create.restype = vp
        L.dxo_data_create.argtypes = [vp]
        L.dxo_data_free.argtypes = [vp]
        L.dxo_reset.argtypes = [vp, vp]
        for fn in ("dxo_forward", "dxo_step", "dxo_kinematics"):
            getattr(L, fn).argtypes = [vp, vp]
            getattr(L, fn).restype = ip
        L.dxo_field.restype = dp
        L.dxo_field.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ip)]
        L.dxo_ncon.argtypes = [vp]
        L.dxo_ncon.restype = ip
        L.dxo_nefc.argtypes = [vp]
        L.dxo_nefc.restype = ip
        L.dxo_solver_niter.argtypes = [vp]
        L.dxo_solver_niter.restype = ip
        L.dxo_solver_cost.argtypes = [vp, vp, dp]
        L.dxo_solver_cost.restype = ctypes.c_double
        L.dxo_set_contacts.argtypes = [vp, ip, dp]
        L.dxo_set_contacts.restype = ip
        L.dxo_contact.argtypes = [vp, ip, dp]
        L.dxo_flops.argtypes = [vp, dp]
        L.dxo_flops_reset.argtypes = [vp]
        L.dxo_batch_step.argtypes = [vp, ip, ip, dp, dp, dp, dp, dp, ip]
        L.dxo_batch_step.restype = ip
        L.dxo_batch_step_counted.argtypes = [vp, ip, ip, dp, dp, dp, dp, dp, ip, dp]
        L.dxo_batch_step_counted.restype = ip
        L.dxo_batch_step_watch.argtypes = [vp, ip, ip, dp, dp, dp, dp, dp, ip, dp, ip, ip, vp]
        L.dxo_batch_step_watch.restype = ip
        L.dxo_observe.argtypes = [vp, vp]
        L.dxo_observe.restype = ip
        L.dxo_object_velocity.argtypes = [vp, vp, ip, ip, dp]
        L.dxo_fk.argtypes = [vp, vp]
        L.dxo_fk.restype = ip
        L.dxo_jac_site.argtypes = [vp, vp, ip, dp, dp]
        L.dxo_ik_attempt.argtypes = [vp, vp, ip, vp, ip, vp, dp, dp, ip, ip, dp]
        L.dxo_ik_attempt.restype = ip
        _lib = L
    return _lib


class OracleModel:
    def __init__(self, blob: bytes):
        self._blob = blob
        self.ptr = lib().dxo_model_load(blob, len(blob))
        if not self.ptr:
            raise RuntimeError("oracle failed to load model blob")

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.dxo_model_free(self.ptr)
            self.ptr = None


class OracleData:
    """One environment's state, with numpy views onto the oracle's arrays."""

    def __init__(self, model: OracleModel):
        self.model = model
        self.ptr = lib().dxo_data_create(model.ptr)

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.dxo_data_free(self.ptr)
            self.ptr = None

    def field(self, name: str) -> np.ndarray:
        n = ctypes.c_int(0)
        p = lib().dxo_field(self.ptr, name.encode(), ctypes.byref(n))
        if not p:
            raise KeyError(name)
        if n.value == 0:
            return np.zeros(0)
        return np.ctypeslib.as_array(p, shape=(n.value,))

    def __getattr__(self, item):
        if item in ("model", "ptr"):
            raise AttributeError(item)
        return self.field(item)

    def reset(self):
        lib().dxo_reset(self.model.ptr, self.ptr)

    def forward(self):
        return lib().dxo_forward(self.model.ptr, self.ptr)

    def step(self):
        return lib().dxo_step(self.model.ptr, self.ptr)

    def kinematics(self):
        return lib().dxo_kinematics(self.model.ptr, self.ptr)

    @property
    def ncon(self) -> int:
        return lib().dxo_ncon(self.ptr)

    @property
    def nefc(self) -> int:
        return lib().dxo_nefc(self.ptr)

    @property
    def niter(self) -> int:
        return lib().dxo_solver_niter(self.ptr)

    def set_contacts(self, recs):
        """Every later collision pass yields these contacts ([n][16] records in
        `contacts()`'s layout) instead of the narrowphase's; None restores it."""
        if recs is None:
            lib().dxo_set_contacts(self.ptr, -1, None)
            return
        r = np.ascontiguousarray(recs, dtype=np.float64).reshape(-1, 16)
        self._fixed = r
        if lib().dxo_set_contacts(self.ptr, len(r), r.ctypes.data_as(ctypes.POINTER(ctypes.c_double))) != 0:
            raise ValueError("too many contacts")

    def solver_cost(self, qacc) -> float:
        """Scaled primal cost of the last forward's constraint problem at `qacc`."""
        q = np.ascontiguousarray(qacc, dtype=np.float64)
        return lib().dxo_solver_cost(self.model.ptr, self.ptr, q.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))

    def contacts(self) -> np.ndarray:
        out = np.zeros((self.ncon, 16))
        buf = (ctypes.c_double * 16)()
        for i in range(self.ncon):
            lib().dxo_contact(self.ptr, i, buf)
            out[i] = np.frombuffer(buf, dtype=np.float64)
        return out

    def fk(self):
        return lib().dxo_fk(self.model.ptr, self.ptr)

    def observe(self):
        """Kinematics + com + cvel at the current state (dm_control's step1 outputs)."""
        return lib().dxo_observe(self.model.ptr, self.ptr)

    def object_velocity(self, objtype: str, idx: int) -> np.ndarray:
        """mj_objectVelocity in the world frame, [lin, ang] (mujoco_utils.py:10-35);
        objtype "body" (inertial frame), "site" or "xbody"."""
        res = np.zeros(6)
        code = {"body": 0, "site": 1, "xbody": 2}[objtype]
        lib().dxo_object_velocity(self.model.ptr, self.ptr, code, int(idx),
                                  res.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return res

    def jac_site(self, site: int):
        """mj_jacSite after fk(): (jacp [3, nv], jacr [3, nv])."""
        nv = self.qvel.shape[0]
        jp, jr = np.zeros((3, nv)), np.zeros((3, nv))
        dp = ctypes.POINTER(ctypes.c_double)
        lib().dxo_jac_site(self.model.ptr, self.ptr, site, jp.ctypes.data_as(dp), jr.ctypes.data_as(dp))
        return jp, jr

    def ik_attempt(self, sites, joints, targets, linear_tol=1e-3, regularization=1e-5, gain=0.95,
                   progress_threshold=20.0, max_steps=100, early_stop=False):
        """One IKSolver._solve_ik attempt from the current qpos; returns (steps, errors)."""
        s = np.ascontiguousarray(sites, dtype=np.int32)
        j = np.ascontiguousarray(joints, dtype=np.int32)
        t = np.ascontiguousarray(targets, dtype=np.float64).reshape(-1)
        o = np.array([linear_tol, regularization, gain, progress_threshold], dtype=np.float64)
        err = np.zeros(len(s))
        dp = ctypes.POINTER(ctypes.c_double)
        steps = lib().dxo_ik_attempt(self.model.ptr, self.ptr, len(s), s.ctypes.data, len(j), j.ctypes.data,
                                     t.ctypes.data_as(dp), o.ctypes.data_as(dp), max_steps, int(early_stop),
                                     err.ctypes.data_as(dp))
        return steps, err

    def flops(self) -> np.ndarray:
        buf = (ctypes.c_double * NSTAGE)()
        lib().dxo_flops(self.ptr, buf)
        return np.frombuffer(buf, dtype=np.float64).copy()

    def flops_reset(self):
        lib().dxo_flops_reset(self.ptr)


def batch_step(model: OracleModel, qpos, qvel, ctrl, qacc_warmstart, xfrc, nsub: int, nthreads: int = 0,
               flops: list = None):
    """Steps nenv independent envs nsub times (OpenMP over envs). Arrays are updated in
    place (when already contiguous float64). With `flops` (a list), appends the FLOP
    counters summed over every env and substep, per stage (STAGES): the algorithmic
    count is the sum without "scan" (the exhaustive mesh scan's surplus)."""
    dp = ctypes.POINTER(ctypes.c_double)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (qpos, qvel, ctrl, qacc_warmstart)]
    x = None if xfrc is None else np.ascontiguousarray(xfrc, dtype=np.float64)
    fl = np.zeros(len(STAGES), dtype=np.float64)
    rc = lib().dxo_batch_step_counted(
        model.ptr,
        arrs[0].shape[0],
        nsub,
        arrs[0].ctypes.data_as(dp),
        arrs[1].ctypes.data_as(dp),
        arrs[2].ctypes.data_as(dp),
        arrs[3].ctypes.data_as(dp),
        None if x is None else x.ctypes.data_as(dp),
        nthreads,
        fl.ctypes.data_as(dp),
    )
    if flops is not None:
        flops.append(fl)
    return rc, arrs[0], arrs[1], arrs[3]


def batch_step_watch(model: OracleModel, qpos, qvel, ctrl, qacc_warmstart, xfrc, nsub: int, watch_geom: int,
                     watch_body: int, nthreads: int = 0):
    """batch_step, plus per env whether the state after the steps has a contact between
    geom watch_geom and a geom of body watch_body with dist <= 1e-8 (the prop-ground fall
    test of reorient.py:229-235).  Returns (rc, qpos, qvel, qacc_warmstart, fell)."""
    dp = ctypes.POINTER(ctypes.c_double)
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (qpos, qvel, ctrl, qacc_warmstart)]
    x = None if xfrc is None else np.ascontiguousarray(xfrc, dtype=np.float64)
    fell = np.zeros(arrs[0].shape[0], dtype=np.int32)
    rc = lib().dxo_batch_step_watch(model.ptr, arrs[0].shape[0], nsub, *(a.ctypes.data_as(dp) for a in arrs),
                                    None if x is None else x.ctypes.data_as(dp), nthreads, None, int(watch_geom),
                                    int(watch_body), fell.ctypes.data)
    return rc, arrs[0], arrs[1], arrs[3], fell.astype(bool)
