#!/usr/bin/env python3
"""CLI over oracle/mpr_ref.py: the oracle's MPR restated with the arithmetic type as a
parameter, on one geom pair of a dumped full-batch state (gpurun_out/fullbatch_*.npz,
tests/golden/fullbatch_*.npz), in fp64 (the C oracle's answer) and in fp32 (the kernel's
precision, with a search over fp32-resolution pose perturbations).

  python tools/mpr_precision.py FIXTURE.npz ENV_INDEX G1 G2 [asset]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.mpr_ref import fp32_reproduces, mpr, pair_inputs  # noqa: E402


def main(path, e, g1, g2, asset="shadow_reorient.npz"):
    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel
    from oracle import oracle as O

    O.build()
    cm = CompiledModel.load(os.path.join(ROOT, "assets", asset))
    om = O.OracleModel(blob.pack(cm.arrays))
    z = np.load(path)
    k = int(np.flatnonzero(z["ids"] == e)[0])
    d = O.OracleData(om)
    d.xfrc_applied[:] = z["x32"]
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = (np.asarray(z[f][k], dtype=np.float64)
                                                            for f in ("qpos", "qvel", "ws", "ctrl"))
    d.forward()
    (p1, m1, v1, c1), (p2, m2, v2, c2), hm = pair_inputs(cm, d, g1, g2)
    oc = d.contacts()
    o = oc[(oc[:, 13] == g1) & (oc[:, 14] == g2)]
    con = z["con"][k]
    r = con[(con[:, 15] != 0) & (con[:, 13] == g1) & (con[:, 14] == g2)]
    print("oracle (C, fp64):", o[:, 12], o[:, 3:6])
    print("GPU (fp32 kernel):", r[:, 12], r[:, 3:6])
    for T in (np.float64, np.float32):
        res = mpr(p1, m1, v1, c1, p2, m2, v2, c2, hm, T)
        depth, normal = res[0], res[1]
        print(f"restated MPR in {T.__name__}: dist {2 * hm - depth:.6e} normal {normal} trips {res[3]}")
    print("fp32 from perturbed poses (ok, angle, depth err, draws):", fp32_reproduces(cm, d, g1, g2, r[0]))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]), int(a[2]), int(a[3]), *(a[4:5]))
