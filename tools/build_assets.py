"""Compiles the reference scenes into assets/<scene>.npz (run where /root/reference exists).

The runtime and the GPU box only read these compiled blobs; nothing at run time
reads the reference checkout.  Shadow-hand derived data (hull vertices) is
GPL-2.0 like its source meshes, see assets/README.md.
"""

from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dexterity_amd.mjcf import scenes  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def main(names=None):
    os.makedirs(OUT, exist_ok=True)
    for name in names or scenes.SCENES:
        model = scenes.SCENES[name]()
        path = os.path.join(OUT, name + ".npz")
        model.save(path)
        print(f"{name}: nq={model.nq} nv={model.nv} nbody={model.nbody} ngeom={model.ngeom} "
              f"ngpair={model.ngpair} -> {path} ({os.path.getsize(path)} B)")


if __name__ == "__main__":
    main(sys.argv[1:] or None)
