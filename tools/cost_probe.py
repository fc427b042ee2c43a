#!/usr/bin/env python3
"""Per-env step-cost distribution of the reorient benchmark (diagnostics).

Reads DX_STEP_COST (shader cycles / 1024 per env of the last control step) after a
warm-up, and estimates how much of the launch the wave slots sit idle: with S wave
slots (8 per CU) and longest-first dispatch the makespan is bounded below by both
sum(cost) / S and max(cost).
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dexterity_amd import _lib, manipulation  # noqa: E402


def main(nenv=4096, steps=60, domain="reorient", solver=None):
    if solver is None:
        env = manipulation.load(domain, "state_dense", seed=1, num_envs=nenv, device=0)
    else:  # <option solver=...> at MuJoCo's defaults (tools/bench_configs.py configs 3' / 3'')
        t = manipulation.SUITE[(domain, "state_dense")]()
        t.compiled = t.compiled.with_solver(solver)
        env = manipulation.GoalEnvironment(t, num_envs=nenv, seed=1)
    env.reset()
    costs = []
    ncons = []
    L = _lib.load()
    kms = []
    for i in range(steps):
        if i >= 10:
            _lib.check(L.dx_timing_enable(env.physics.ptr, 1))
            _lib.check(L.dx_timing_read(env.physics.ptr, ctypes.byref(ctypes.c_double()), ctypes.byref(ctypes.c_int32())))
        env.step_random(i)
        if i >= 10:
            costs.append(env.physics.get(_lib.STEP_COST).ravel().astype(np.float64) * 1024)
            ncons.append(env.physics.get(_lib.NCON).ravel().astype(np.int64))
            kt, kn = ctypes.c_double(), ctypes.c_int32()
            _lib.check(L.dx_timing_read(env.physics.ptr, ctypes.byref(kt), ctypes.byref(kn)))
            kms.append(kt.value / max(kn.value, 1))
    c = np.array(costs)
    os.makedirs("gpurun_out", exist_ok=True)
    np.save("gpurun_out/costs.npy", c.astype(np.float32))
    slots = 256 * 8  # (the queued reorient batch; a contact-free batch that fits runs one workgroup per env)
    per = c.mean(axis=0)
    print(f"cycles per env-step: mean {c.mean():.3e} p50 {np.median(c):.3e} p90 {np.percentile(c, 90):.3e} "
          f"p99 {np.percentile(c, 99):.3e} max {c.max():.3e}")
    print(f"per-step sum/slots {np.mean(c.sum(axis=1) / slots):.3e}  per-step max {np.mean(c.max(axis=1)):.3e}")
    clk = float(os.environ.get("DX_CLOCK_MHZ", "2394")) * 1e6
    km = float(np.mean(kms))
    print(f"step kernel {km:.4f} ms = {km * 1e-3 * clk:.3e} cycles at {clk / 1e6:.0f} MHz; "
          f"slot utilisation sum(cost)/(slots x kernel) = {np.mean(c.sum(axis=1)) / (slots * km * 1e-3 * clk):.3f}")
    print("per-env mean cost deciles:", np.round(np.percentile(per, np.arange(0, 101, 10)) / 1e6, 3))
    # how well the last step's cost predicts this step's (what longest-first relies on)
    cc = [np.corrcoef(c[t], c[t - 1])[0, 1] for t in range(1, len(c))]
    print(f"corr(cost_t, cost_t-1) mean {np.mean(cc):.3f}")
    ranks = []
    for t in range(1, len(c)):
        prev_rank = np.argsort(np.argsort(-c[t - 1]))
        ranks.extend(prev_rank[np.argsort(-c[t])[:20]].tolist())
    print("previous-step rank of each step's 20 heaviest envs: median", np.median(ranks),
          "p90", np.percentile(ranks, 90))
    nc = np.array(ncons)
    top = np.argsort(-c.ravel())[:12]
    print("heaviest env-steps (Mcycles, contacts at the step's end):",
          [(round(c.ravel()[k] / 1e6, 2), int(nc.ravel()[k])) for k in top])
    print(f"per-step max / kernel cycles {np.mean(c.max(axis=1)) / (km * 1e-3 * clk):.3f}")
    hist, edges = np.histogram(c.ravel() / 1e6, bins=20)
    print("hist (Mcycles):", list(zip(np.round(edges[:-1], 2).tolist(), hist.tolist())))
    env.close()


if __name__ == "__main__":
    # cost_probe.py [nenv] [steps] [domain] [solver]
    main(*[int(a) for a in sys.argv[1:3]], *sys.argv[3:5])
