"""In-tree build of libdx.so (HIP, gfx950) -- no JIT cache, the .so travels with the repo.

The step kernel is also compiled once per shipped scene with that scene's dimensions
and LDS layout as compile-time constants (csrc/dx_specs.inc, regenerated here from
the assets through the library's own layout code).  At dx_batch_create the library
launches the specialization whose layout equals the model's, else the generic kernel.
"""

from __future__ import annotations

import concurrent.futures
import glob
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdx.so")
SPECS = os.path.join(CSRC, "dx_specs.inc")
SOURCES = ("dx_step.hip", "dx_ik.hip", "dx_task.hip", "dx_sensor.hip", "dx_api.hip")
HEADERS = ("dx_internal.h", "dx_device.h", "dx_task.h")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
DIMS = ("nq", "nv", "nbody", "njnt", "nu", "ntendon", "nsite", "nlevel", "nroot", "nfric", "nlimj", "nlimt",
        "nbpair", "any_damping", "disable_contact", "iterations", "solver")  # dx_device.h DX_DIMS


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "dx.h"))
    deps += glob.glob(os.path.join(ROOT, "assets", "*.npz"))
    return any(os.path.getmtime(p) > t for p in deps)


FLAGS = (
    # fp32 division / sqrt as v_rcp / v_sqrt (<= 1 ulp) instead of the correctly
    # rounded ~10-instruction sequences: the kernels are latency bound and the
    # parity tolerances are orders of magnitude above 1 ulp
    "-O3", f"--offload-arch={ARCH}", "-fPIC", "-std=c++17",
    "-fno-hip-fp32-correctly-rounded-divide-sqrt",
    # no SLP packing of scalar fp32 math into v_pk_* (the operand shuffles cost
    # more than the packing saves here), denormals flushed (no range scaling
    # around v_sqrt / v_rcp)
    "-fno-slp-vectorize", "-fgpu-flush-denormals-to-zero",
)
OBJ = os.path.join(ROOT, "build", "obj")
SOLVER_SPECS = ("shadow_reorient",)  # scenes specialised for CG and PGS too (spec_text)


def _spec_names() -> list:
    if not os.path.exists(SPECS):
        return []
    m = re.search(r"#define DX_SPECS\(X\)(.*)", open(SPECS).read())
    return re.findall(r"X\((\w+)\)", m.group(1)) if m else []


def _units() -> list:
    """(object name, source, extra flags): every source once, plus dx_step.hip once per
    scene specialization (-DDX_SPEC_ONLY), so the kernels compile in parallel."""
    units = [(os.path.splitext(s)[0], s, ()) for s in SOURCES]
    # a PGS specialization runs one wave per SIMD: AR's diagonal blocks and the rows' P
    # take ~430 VGPRs (dx_step.hip solve_pgs_ar), which two waves per SIMD would spill
    # (CG too: its launch is bound by its slowest envs' chains, which run faster alone on a
    # SIMD -- config 3' 0.872 -> 0.900 M env-steps/s same-box, round 6)
    # (reach: DX_REACH_WAVES, an experiment -- config 2's 1024 envs fill half the slots)
    waves = {"_pgs": os.environ.get("DX_PGS_WAVES", "1"), "_cg": os.environ.get("DX_CG_WAVES", "1"),
             "_reach": os.environ.get("DX_REACH_WAVES", "")}

    def spec_flags(n):
        w = next((v for k, v in waves.items() if n.endswith(k) and v), None)
        return (f"-DDX_SPEC_ONLY={n}",) + ((f"-DDX_STEP_WAVES={w}",) if w else ())

    units += [(f"dx_step_{n}", "dx_step.hip", spec_flags(n)) for n in _spec_names()]
    # the overflow tier: the step kernel's physics with the DX_NCON_HI contact pool
    units.append(("dx_step_hi", "dx_step.hip", ("-DDX_TIER_HI", "-DDX_NCON_MAX=DX_NCON_HI")))
    # the mid tier: the same physics with the DX_NCON_MID pool, beside queued launches
    units.append(("dx_step_mid", "dx_step.hip", ("-DDX_TIER_MID", "-DDX_NCON_MAX=DX_NCON_MID")))
    return units


def _compile(out: str, verbose: bool) -> None:
    # one build of a tree at a time (several ranks, or pytest beside bench.py): the
    # object cache and its clean-up below are shared
    import fcntl

    os.makedirs(OBJ, exist_ok=True)
    with open(os.path.join(OBJ, ".lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        _compile_locked(out, verbose)


def source_key(csrc: str = None) -> str:
    """Hash of everything a libdx.so is built from (sources, headers, the scene
    specializations, the C ABI header, the flags).  The library carries it
    (dx_build_key), and _lib.load refuses an in-tree library built from other sources."""
    csrc = csrc or CSRC
    h = hashlib.sha1()
    for f in sorted(SOURCES + HEADERS + ("dx_specs.inc",)):
        path = os.path.join(csrc, f)
        if os.path.exists(path):
            h.update(f.encode() + open(path, "rb").read())
    h.update(open(os.path.join(ROOT, "include", "dx.h"), "rb").read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:16]


def _compile_locked(out: str, verbose: bool) -> None:
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    key = source_key()
    jobs, objs = [], []
    for name, src, extra in _units():
        if src == "dx_api.hip":
            extra = extra + (f'-DDX_BUILD_KEY="{key}"',)
        xk = hashlib.sha1(" ".join(extra).encode()).hexdigest()[:6]  # (per-unit flags: DX_PGS_WAVES)
        obj = os.path.join(OBJ, f"{name}.{key}{xk}.o")
        objs.append(obj)
        if not os.path.exists(obj):
            jobs.append(([hipcc, *FLAGS, *extra, "-c", os.path.join(CSRC, src), "-o", f"{obj}.{os.getpid()}.tmp"], obj))

    def run(job):
        cmd, obj = job
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(cmd[-1], obj)

    nproc = int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))
    with concurrent.futures.ThreadPoolExecutor(max_workers=max(1, min(nproc, 8))) as ex:
        for f in [ex.submit(run, j) for j in jobs]:
            f.result()
    cmd = [hipcc, f"--offload-arch={ARCH}", "-fPIC", "-shared", *objs, "-L/opt/rocm/lib", "-lrccl", "-o", out]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    for old in glob.glob(os.path.join(OBJ, "*.o")):  # objects of other source versions
        if old not in objs:
            os.remove(old)


def spec_text(lib_path: str, dims: tuple = DIMS, solver_specs: tuple = None) -> str:
    """dx_specs.inc for every asset, from the layout the library at lib_path computes."""
    if solver_specs is None:
        solver_specs = SOLVER_SPECS
    import ctypes

    import numpy as np

    sys.path.insert(0, ROOT)
    from dexterity_amd import blob as blob_mod
    from dexterity_amd.mjcf.compiler import CompiledModel

    L = ctypes.CDLL(lib_path)
    L.dx_model_load.restype = ctypes.c_void_p
    L.dx_model_load.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
    L.dx_model_free.argtypes = [ctypes.c_void_p]
    L.dx_model_layout.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32]
    seen = {}
    models = []
    for path in sorted(glob.glob(os.path.join(ROOT, "assets", "*.npz"))):
        name = os.path.splitext(os.path.basename(path))[0]
        cm = CompiledModel.load(path)
        models.append((name, cm))
        # the headline scene also with the two other solvers at MuJoCo's defaults
        # (BASELINE config 3 names "PGS"; <option solver=...>): their own kernels, so the
        # Newton kernel carries neither (the solver is a specialization dimension)
        if name in solver_specs:
            models += [(f"{name}_{sv.lower()}", cm.with_solver(sv)) for sv in ("CG", "PGS")]
    for name, cm in models:
        data = blob_mod.pack(cm.arrays)
        m = L.dx_model_load(data, len(data))
        if not m:
            continue
        buf = (ctypes.c_int32 * 256)()
        n = L.dx_model_layout(m, buf, 256)
        L.dx_model_free(m)
        if n <= 0:
            continue
        key = tuple(buf[:n])
        seen.setdefault(key, name)
    lines = ["// generated by dexterity_amd/build.py from assets/*.npz -- do not edit"]
    names = []
    for key, name in seen.items():
        nl = len(key) - len(dims)
        ident = "DxSpec_" + "".join(ch if ch.isalnum() else "_" for ch in name)
        names.append(ident)
        lines.append(f"struct {ident} {{")
        lines.append(f"  static constexpr Lds L = {{{', '.join(str(v) for v in key[:nl])}}};")
        lines.append("  static constexpr int " + ", ".join(f"{d} = {v}" for d, v in zip(dims, key[nl:])) + ";")
        # a reach scene's kernel carries the reach sampling pass (dx_step.hip fused_reach_prep)
        lines.append(f"  static constexpr bool reach_task = {'true' if 'reach' in name else 'false'};")
        lines.append("};")
    lines.append("#define DX_SPECS(X) " + " ".join(f"X({n})" for n in names))
    del np
    return "\n".join(lines) + "\n"


def build(force: bool = False, verbose: bool = False) -> str:
    # on a GPU box (gpurun exports GRAFT_REPO_ROOT) the library travels prebuilt: tests
    # use it as it is instead of rebuilding from sources whose times the copy may change
    if not force and os.path.exists(OUT) and (os.environ.get("GRAFT_REPO_ROOT") or not _stale()):
        return OUT
    tmp = f"{OUT}.{os.getpid()}.tmp"
    _compile(tmp, verbose)
    # regenerate the specializations with the layout code just built (in a child
    # process: this one may load libdx.so afterwards)
    text = subprocess.run(
        [sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); "
         f"from dexterity_amd.build import spec_text; sys.stdout.write(spec_text({tmp!r}, {DIMS!r}, {SOLVER_SPECS!r}))"],
        check=True, capture_output=True, text=True).stdout
    old = open(SPECS).read() if os.path.exists(SPECS) else ""
    if text != old:
        with open(SPECS, "w") as f:
            f.write(text)
        if verbose:
            print(f"wrote {SPECS}; rebuilding with the specializations")
        _compile(tmp, verbose)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
