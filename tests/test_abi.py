"""The C-ABI library loads and exports every symbol include/dx.h declares (no GPU).

Host-side entry points (model parsing, sizes, field widths, error reporting) are
exercised; nothing here launches a kernel.
"""

import ctypes
import os
import re

import numpy as np
import pytest

from dexterity_amd import _lib, blob, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    build.build()
    return _lib.load()


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "dx.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dx_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(lib):
    syms = _declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"libdx.so does not export {s}"
    assert set(_lib.EXPORTS) <= set(syms)


def test_abi_version(lib):
    assert lib.dx_abi_version() == 1


def test_model_load_and_sizes(lib, reorient_compiled):
    b = blob.pack(reorient_compiled.arrays)
    m = lib.dx_model_load(b, len(b))
    assert m
    sizes = (ctypes.c_int32 * 12)()
    assert lib.dx_model_sizes(m, sizes) == 0
    nq, nv, nbody, njnt, ngeom, nsite, nu, nten, nbp, ngp, ncon_max, nefc_max = list(sizes)
    assert (nq, nv, nu, nten) == (31, 30, 20, 4)
    assert ngeom == reorient_compiled.ngeom and ngp == reorient_compiled.ngpair
    assert lib.dx_field_width(m, _lib.QPOS) == 31
    assert lib.dx_field_width(m, _lib.SITE_VEL) == 6 * nsite
    assert lib.dx_field_width(m, 999) < 0
    lib.dx_model_free(m)


def test_bad_blob_reports_error(lib):
    assert not lib.dx_model_load(b"garbage-not-a-blob", 18)
    assert b"malformed" in lib.dx_last_error()
    arrays = {"nq": np.array([1], np.int32)}
    b = blob.pack(arrays)
    assert not lib.dx_model_load(b, len(b))
    assert b"missing" in lib.dx_last_error()


def test_blob_roundtrip(reorient_compiled):
    b = blob.pack(reorient_compiled.arrays)
    back = blob.unpack(b)
    for k, v in reorient_compiled.arrays.items():
        np.testing.assert_array_equal(back[k], np.asarray(v).ravel().astype(back[k].dtype))


def test_null_arguments_are_rejected(lib):
    assert lib.dx_step(None, 1) < 0
    assert lib.dx_env_step(None, None) < 0
    assert lib.dx_set_field(None, 0, None, 0, 1) < 0


@pytest.mark.parametrize("asset", ["shadow_reorient", "adroit_reach"])
def test_binned_hull_support_matches_full_scan(lib, asset):
    """Direction-binned hulls (dx_api.hip build_hull_bins) return the vertex the full
    serial scan returns -- the first maximiser -- for random and axis-aligned
    directions, including cell edges and faces.  A different index is accepted only
    for a tie at fp32 resolution (two vertices whose fp64 dots differ by < 1e-6 R,
    ordered differently by fp32 rounding)."""
    from dexterity_amd.mjcf.compiler import CompiledModel
    from dexterity_amd.physics import Model

    cm = CompiledModel.load(os.path.join(ROOT, "assets", f"{asset}.npz"))
    model = Model(cm)
    a = cm.arrays
    nvert = np.asarray(a["mesh_vertnum"])
    adr = np.asarray(a["mesh_vertadr"])
    V = np.asarray(a["mesh_vert"], dtype=np.float64).reshape(-1, 3)
    info = (ctypes.c_int32 * 3)()
    d = (ctypes.c_float * 3)()
    rng = np.random.RandomState(7)
    checked = binned = 0
    for mesh in np.nonzero(nvert > 8)[0]:
        vv = V[adr[mesh]: adr[mesh] + nvert[mesh]]
        R = np.linalg.norm(vv, axis=1).max()
        dirs = rng.randn(400, 3).astype(np.float32)
        dirs[::4, rng.randint(3)] = 0.0          # on cube-map cell edges
        dirs[1::4] = np.round(dirs[1::4] * 2) / 2  # exact face / corner ratios
        for dv in dirs:
            d[:] = dv
            assert lib.dx_hull_support(model.ptr, int(mesh), d, info) == 0
            # every hull with more than DX_HULL_K = 8 vertices is binned, 8 slots per cell
            assert info[1] > 0 and info[2] == 8
            binned += info[1] > 0
            dots = vv @ dv.astype(np.float64)
            ref = int(np.argmax(dots))
            tie = dots[info[0]] >= dots[ref] - 1e-6 * R * np.linalg.norm(dv)
            assert info[0] == ref or tie, (mesh, dv)
            checked += 1
    assert checked > 0
    assert binned == checked
