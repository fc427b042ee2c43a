#!/usr/bin/env python3
"""CPU-side look at full-batch parity states the accounting dumped (gpurun_out/fullbatch_*_{divergent,
unexplained}.npz): for each deep GPU contact (|dist| > 0.5 mm), the fp64 oracle's contact of the same geom
pair at the state and over fp32-scale perturbations of the state (relative 1e-7 ... 3e-6 on qpos), so the
oracle's own discontinuity there can be compared with the GPU's answer.

  python tools/divergent_repro.py gpurun_out/fullbatch_reorient_newton_divergent.npz [asset] [solver]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def oracle_contacts(O, om, x32, q, v, w, c):
    d = O.OracleData(om)
    d.xfrc_applied[:] = x32
    d.qpos[:], d.qvel[:], d.qacc_warmstart[:], d.ctrl[:] = q, v, w, c
    d.forward()
    return d.contacts()


def survey(path, asset="shadow_reorient.npz", solver=None, nper=200, seed=0):
    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel
    from oracle import oracle as O

    O.build()
    cm = CompiledModel.load(os.path.join(ROOT, "assets", asset))
    if solver:
        cm = cm.with_solver(solver)
    om = O.OracleModel(blob.pack(cm.arrays))
    z = np.load(path)
    out = []
    for k, e in enumerate(z["ids"]):
        st = [np.asarray(z[f][k], dtype=np.float64) for f in ("qpos", "qvel", "ws", "ctrl")]
        con = z["con"][k]
        recs = con[con[:, 15] != 0]
        base = oracle_contacts(O, om, z["x32"], *st)
        rng = np.random.RandomState(seed + int(e))
        pert = []
        for p in range(nper):
            rel = 10 ** rng.uniform(-7, np.log10(3e-6))
            q = st[0] * (1 + rng.standard_normal(st[0].shape) * rel)
            pert.append(oracle_contacts(O, om, z["x32"], q, *st[1:]))
        for r in recs:
            if abs(r[12]) <= 5e-4:
                continue
            g1, g2 = r[13], r[14]

            def nearest(cs):
                m = (cs[:, 13] == g1) & (cs[:, 14] == g2)
                if not m.any():
                    return None
                c = cs[m]
                return c[np.argmin(np.abs(c[:, 0:3] - r[0:3]).max(axis=1))]

            o = nearest(base)
            if o is None:
                continue
            ang = lambda a, b: float(np.arccos(np.clip(np.dot(a, b) / np.linalg.norm(a) / np.linalg.norm(b), -1, 1)))
            ps = [nearest(c) for c in pert]
            ps = [p for p in ps if p is not None]
            pang = [ang(p[3:6], o[3:6]) for p in ps]
            pdep = [p[12] for p in ps]
            gang = ang(r[3:6], o[3:6])
            # the nearest perturbed oracle answer to the GPU's
            best = min(ps, key=lambda p: ang(p[3:6], r[3:6]) + abs(p[12] - r[12]) / abs(r[12]))
            row = dict(env=int(e), pair=(int(g1), int(g2)), gpu_dist=float(r[12]), oracle_dist=float(o[12]),
                       depth_rel=float(abs(r[12] - o[12]) / abs(o[12])), gpu_normal_angle=gang,
                       point_diff=float(np.abs(r[0:3] - o[0:3]).max()),
                       oracle_pert_max_angle=float(max(pang)), oracle_pert_depth=(float(min(pdep)), float(max(pdep))),
                       nearest_pert_angle=ang(best[3:6], r[3:6]), nearest_pert_depth_rel=float(abs(best[12] - r[12]) / abs(r[12])))
            out.append(row)
            print(row, flush=True)
    return out


if __name__ == "__main__":
    a = sys.argv[1:]
    survey(a[0], *(a[1:3]))
