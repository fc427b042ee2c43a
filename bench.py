#!/usr/bin/env python3
"""Benchmark: env-steps/s of Shadow-hand cube reorient (BASELINE.json config 3/4).

One step = one control step of `reorient.state_dense` for every environment:
GoalTask.before_step, 5 physics substeps (dt 0.005, reorient.py:58,61,168),
after_step, reward / discount / termination, the 123-float STATE_ONLY observation,
and dm_env auto-reset -- all on the GPU (dx_env_step).  Actions are drawn on the
device uniformly within each actuator's ctrlrange (the random agent of
manipulation_test.py:44-45).  Inputs are resident in HBM; nothing crosses PCIe in
the timed region.

N=1: 4096 envs on one MI355X.  N>1 (torchrun, one process per GPU): 4096 envs per
GPU (weak scaling, 32768 on 8 GPUs = config 4) and an RCCL all-gather of the packed
[obs | reward | discount | step_type] shards every control step.

Prints ONE JSON line (rank 0).  See DESIGN.md §5 for the roofline accounting.
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# bytes per env-step that one control step must move through HBM with state
# resident: read ctrl 20 + qpos 31 + qvel 30 + warmstart 30 floats,
# write qpos 31 + qvel 30 + warmstart 30 + obs 123 + reward/discount/done 3 floats.
ALGO_BYTES_PER_ENV_STEP = (20 + 31 + 30 + 30 + 31 + 30 + 30 + 123 + 3) * 4  # 1312 B
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: peak FP32 (vector)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs-per-gpu", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def cpu_baseline(seconds: float, flops_per_env_step_box: list):
    """The fp64 oracle (oracle/dx_oracle.c) timed on this box's host cores, OpenMP over envs."""
    import numpy as np

    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel
    from dexterity_amd.physics import gravity_compensation
    from oracle import oracle as O

    O.build()
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    om = O.OracleModel(blob.pack(cm.arrays))
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    nenv = threads * 8
    rng = np.random.RandomState(12345)
    qpos = np.tile(cm.qpos0, (nenv, 1))
    qpos[:, 24:27] += rng.uniform(-0.025, 0.025, size=(nenv, 3)) * [1, 1, 0]
    qvel = np.zeros((nenv, cm.nv))
    ws = np.zeros((nenv, cm.nv))
    xfrc = gravity_compensation(cm, "shadow_hand_e/")
    lo, hi = cm.actuator_ctrlrange.T
    # per-env-step FLOPs from the instrumented oracle on the same scene (5 substeps)
    d = O.OracleData(om)
    d.xfrc_applied[:] = xfrc.ravel()
    for _ in range(40):  # settle the cube first so the sample includes contacts
        d.step()
    d.flops_reset()
    for _ in range(5):
        d.step()
    flops_per_env_step_box.append(float(d.flops().sum()))
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ctrl = rng.uniform(lo, hi, size=(nenv, cm.nu))
        rc, qpos, qvel, ws = O.batch_step(om, qpos, qvel, ctrl, ws, xfrc, nsub=5, nthreads=threads)
        steps += 1
    dt = time.perf_counter() - t0
    return {
        "value": nenv * steps / dt,
        "unit": "env-steps/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"fp64 C oracle (oracle/dx_oracle.c), same scene, {nenv} envs x {steps} control steps "
        f"(5 substeps each), random ctrl, OpenMP {threads} threads, {dt:.1f} s",
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    import torch  # imported before libdx so both share one HIP runtime

    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from dexterity_amd import _lib, distributed, manipulation

    B = args.envs_per_gpu
    env = manipulation.load("reorient", "state_dense", seed=distributed.rank_seed(12345, rank), num_envs=B,
                            device=local)
    L = _lib.load()
    obs_w = env.obs_dim + 3
    if world > 1:
        collator = distributed.OutputCollator(B, obs_w, device=f"cuda:{local}")

    def one_step(i):
        a = env.sample_actions(i)
        env.step(a, device_action=True)
        if world > 1:
            _lib.check(L.dx_env_pack_outputs(env.ptr, ctypes.c_void_p(collator.shard.data_ptr())))
            env.physics.sync()
            collator.gather()

    env.reset()
    for i in range(args.warmup):
        one_step(i)
    env.physics.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    _lib.check(L.dx_timing_enable(env.physics.ptr, 1))
    _lib.check(L.dx_timing_read(env.physics.ptr, ctypes.byref(ctypes.c_double()), ctypes.byref(ctypes.c_int32())))
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(args.warmup + i)
    env.physics.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kt, kn = ctypes.c_double(), ctypes.c_int32()
    _lib.check(L.dx_timing_read(env.physics.ptr, ctypes.byref(kt), ctypes.byref(kn)))
    _lib.check(L.dx_timing_enable(env.physics.ptr, 0))
    if world > 1:
        elapsed = distributed.max_over_ranks(elapsed, f"cuda:{local}")
    total_env_steps = world * B * args.steps
    value = total_env_steps / elapsed
    kernel_ms = kt.value / max(1, kn.value)
    out = None
    if rank == 0:
        achieved = ALGO_BYTES_PER_ENV_STEP * B / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_step_kernel.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                p = json.load(f)
            if p.get("envs") == B:
                traffic = p.get("hbm_bytes_per_launch")
        flops_box = []
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_seconds, flops_box)
        out = {
            "metric": "env-steps/sec (whole node), Shadow-hand cube reorient @4096 envs, 1/2/4/8 GPUs",
            "value": round(value, 1),
            "unit": "env-steps/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: random actions within ctrlrange, device RNG; cube spawn/goals per reorient.py",
            "config": {
                "workload": "reorient.state_dense, Shadow hand + cube, full contact + Newton solver",
                "envs_per_gpu": B,
                "global_envs": world * B,
                "substeps_per_env_step": 5,
                "physics_dt": 0.005,
                "parallelism": f"env-sharded x{world}" + (", RCCL obs all-gather" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "kernel": "dx_step_kernel",
                "kernel_ms_avg": round(kernel_ms, 4),
                "algo_bytes_per_env_step": ALGO_BYTES_PER_ENV_STEP,
            },
            "cpu_baseline": cpu,
        }
        if flops_box:
            fl = flops_box[0]
            out["roofline"]["valu_fp32"] = {
                "flops_per_env_step": round(fl),
                "achieved_tflops": round(fl * B / (kernel_ms * 1e-3) / 1e12, 4),
                "peak_tflops": FP32_PEAK_TFLOPS,
            }
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
