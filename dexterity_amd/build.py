"""In-tree build of libdx.so (HIP, gfx950) -- no JIT cache, the .so travels with the repo."""

from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libdx.so")
SOURCES = ("dx_step.hip", "dx_task.hip", "dx_api.hip")
HEADERS = ("dx_internal.h",)
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "dx.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [
        # fp32 division / sqrt as v_rcp / v_sqrt (<= 1 ulp) instead of the correctly
        # rounded ~10-instruction sequences: the kernels are latency bound and the
        # parity tolerances are orders of magnitude above 1 ulp
        hipcc, "-O3", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-std=c++17",
        "-fno-hip-fp32-correctly-rounded-divide-sqrt",
        *[os.path.join(CSRC, s) for s in SOURCES], "-o", OUT + ".tmp",
    ]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
