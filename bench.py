#!/usr/bin/env python3
"""Benchmark: env-steps/s of Shadow-hand cube reorient (BASELINE.json config 3/4).

One step = one control step of `reorient.state_dense` for every environment:
GoalTask.before_step, 5 physics substeps (dt 0.005, reorient.py:58,61,168),
after_step, reward / discount / termination, the 123-float STATE_ONLY observation,
and dm_env auto-reset -- all on the GPU (dx_env_step).  Actions are drawn on the
device uniformly within each actuator's ctrlrange (the random agent of
manipulation_test.py:44-45).  Inputs are resident in HBM; nothing crosses PCIe in
the timed region.

N=1: 4096 envs on one MI355X.  N>1 (torch.distributed.run launches one process per
GPU; only its RANK / WORLD_SIZE / LOCAL_RANK / MASTER_PORT environment is used):
4096 envs per GPU (weak scaling, 32768 on 8 GPUs = config 4) and, every control
step, the RCCL all-gather of the packed [obs | reward | discount | step_type] shards
(dx_allgather_obs: librccl called from libdx).  No PyTorch.

Prints ONE JSON line (rank 0).  Roofline accounting: DESIGN.md §5.4.
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
FLOP_SAMPLE_ENVS = 4096  # every env of the batch (≈0.1 s of oracle time): the per-sample spread of a 256-env sample was ±3 %


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--envs-per-gpu", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (all threads)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--host-api-steps", type=int, default=50, help="extra line: the host-action call shape (0: off)")
    return p.parse_args()


def host_threads() -> int:
    """Host cores this process may use: the affinity mask, bounded by the job's CPU
    share when the launcher states one (OMP_NUM_THREADS; 16 per GPU on the MI355X
    boxes, whose `nproc` counts the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def oracle_flops_per_env_step(states, nsub: int):
    """FLOPs of one control step on the oracle's per-stage counters, averaged over
    environment states sampled from the GPU batch at the end of the timed region (so
    the contact mix is the bench workload's).  Returns the per-stage counts per
    env-step (oracle.STAGES): the algorithmic count is every stage but "scan", the
    surplus of the oracle's exhaustive mesh-support scan over an efficient support's
    16 vertices (DXO_ST_SCAN in oracle/dx_oracle.c)."""
    import numpy as np

    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel
    from dexterity_amd.physics import gravity_compensation
    from oracle import oracle as O

    O.build()
    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    om = O.OracleModel(blob.pack(cm.arrays))
    xfrc = gravity_compensation(cm, "shadow_hand_e/")
    qpos, qvel, ws, ctrl = (np.asarray(a, dtype=np.float64) for a in states)
    fl = []
    O.batch_step(om, qpos, qvel, ctrl, ws, xfrc, nsub=nsub, nthreads=host_threads(), flops=fl)
    return dict(zip(O.STAGES, (float(v) for v in fl[0] / qpos.shape[0])))


def cpu_baseline(seconds: float, threads: int, states, nsub: int):
    """The fp64 oracle (oracle/dx_oracle.c, "port") timed on this box's host cores,
    OpenMP over environments, on the same scene and the bench's own state mix: the
    sample starts from environment states taken from the GPU batch, draws random
    actions within ctrlrange each control step, and restarts an env from its initial
    state on the task's fall rule: a prop-ground contact at the new state
    (reorient.py:229-235, the collision pass the reference's step ends with)."""
    import numpy as np

    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel
    from dexterity_amd.physics import gravity_compensation
    from oracle import oracle as O

    cm = CompiledModel.load(os.path.join(ROOT, "assets", "shadow_reorient.npz"))
    om = O.OracleModel(blob.pack(cm.arrays))
    xfrc = gravity_compensation(cm, "shadow_hand_e/")
    q0, v0, w0 = (np.array(a, dtype=np.float64) for a in states[:3])
    n = q0.shape[0]
    qpos, qvel, ws = q0.copy(), v0.copy(), w0.copy()
    lo, hi = cm.actuator_ctrlrange.T
    names = cm.names
    ground, prop = names["geom"].index("ground"), names["body"].index("prop/")
    rng = np.random.RandomState(12345)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        ctrl = rng.uniform(lo, hi, size=(n, cm.nu))
        rc, qpos, qvel, ws, down = O.batch_step_watch(om, qpos, qvel, ctrl, ws, xfrc, nsub, ground, prop,
                                                      nthreads=threads)
        qpos[down], qvel[down], ws[down] = q0[down], v0[down], w0[down]
        steps += 1
    dt = time.perf_counter() - t0
    return {
        "value": n * steps / dt,
        "unit": "env-steps/sec",
        "cores": threads,
        "kind": "port",
        "sample": f"fp64 C oracle (oracle/dx_oracle.c), reorient scene, {n} env states taken from the GPU batch "
        f"x {steps} control steps (5 substeps each) with the task's fall test (prop-ground contact), random ctrl, "
        f"fallen cubes restarted, OpenMP {threads} "
        f"threads, {dt:.1f} s",
    }


def cpu_baseline_reach_1env(seconds: float, hand: str = "adroit"):
    """BASELINE.json config 1: reach, 1 env, 1 thread, dt 0.02 x 1 substep, uniform
    random actions (manipulation_test.py:44-45); the Adroit hand is the reference task's
    hand (reach.py:231), the Shadow hand is BASELINE.md's naming (contacts disabled)."""
    import numpy as np

    from dexterity_amd import blob
    from dexterity_amd.mjcf.compiler import CompiledModel
    from dexterity_amd.physics import gravity_compensation
    from oracle import oracle as O

    asset, prefix = {"adroit": ("adroit_reach.npz", "adroit_hand/"), "shadow": ("shadow_reach.npz", "shadow_hand_e/")}[hand]
    cm = CompiledModel.load(os.path.join(ROOT, "assets", asset))
    om = O.OracleModel(blob.pack(cm.arrays))
    d = O.OracleData(om)
    d.xfrc_applied[:] = gravity_compensation(cm, prefix).ravel()
    lo, hi = cm.actuator_ctrlrange.T
    rng = np.random.RandomState(12345)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        d.ctrl[:] = rng.uniform(lo, hi)
        d.step()
        steps += 1
    dt = time.perf_counter() - t0
    return {
        "value": steps / dt,
        "unit": "env-steps/sec",
        "cores": 1,
        "kind": "port",
        "sample": f"config 1: fp64 C oracle, reach ({hand.capitalize()} hand), 1 env, 1 thread, {steps} control steps "
        f"(1 substep each, dt 0.02), random ctrl, {dt:.1f} s (Python call per step included)",
    }


def host_api_line(env, steps: int, warmup: int):
    """The reference's own call shape at the headline size: `GoalEnvironment.step` with a
    host action np.float32[B, nu] and the host TimeStep back every control step
    (environment.py:25-34, task.py:63-73) -- dx_env_step_host through page-locked buffers,
    then the dm_env-style float64 observation dict.  The random actions are drawn before
    the timed region (the agent is not the environment's cost)."""
    import numpy as np

    from dexterity_amd import _lib

    L = _lib.load()
    B, nu = env.num_envs, env.model.nu
    lo, hi = env.task.compiled.actuator_ctrlrange.T
    acts = np.random.RandomState(7).uniform(lo, hi, size=(warmup + steps, B, nu)).astype(np.float32)
    for i in range(warmup):
        env.step(acts[i])
    pin_a, pin_o = env._pin_act, env._pin_out
    t_call = t_ts = 0.0
    t0 = time.perf_counter()
    for i in range(steps):
        a = time.perf_counter()
        np.copyto(pin_a, acts[warmup + i])
        _lib.check(L.dx_env_step_host(env.ptr, pin_a.ctypes.data, pin_o.ctypes.data))
        b = time.perf_counter()
        ts = env._timestep_packed(pin_o)
        t_call += b - a
        t_ts += time.perf_counter() - b
    dt = time.perf_counter() - t0
    assert np.all(np.isfinite(ts.reward))
    return {
        "api": "GoalEnvironment.step(np.float32[%d, %d]) -> host TimeStep" % (B, nu),
        "env_steps_per_s": round(B * steps / dt, 1),
        "ms_per_step": round(dt / steps * 1e3, 4),
        "ms_per_step_upload_step_download": round(t_call / steps * 1e3, 4),
        "ms_per_step_timestep_dict": round(t_ts / steps * 1e3, 4),
        "bytes_per_step": {"upload": B * nu * 4, "download": B * (env.obs_dim + 3) * 4},
        "steps": steps,
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world == 1 and args.gpus > 1:
        raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one rank per GPU)")
    from dexterity_amd import _lib, distributed, manipulation

    L = _lib.load()
    comm = distributed.Comm.from_env(device=local) if world > 1 else None
    B = args.envs_per_gpu
    # rank r steps envs [env0, env0 + B) of the job; env i draws from seed 12345 + i
    env0, _ = distributed.env_shard(world * B, rank, world)
    env = manipulation.load("reorient", "state_dense", seed=12345, num_envs=B, device=local, env_offset=env0)
    collator = distributed.OutputCollator(env, comm) if comm else None

    def one_step(i):
        # the random agent (manipulation_test.py:44-45), its actions drawn inside the step
        # kernel: a control step is the step kernel, the mid contact tier beside it on a
        # side stream, and the overflow tier / order launch after it
        env.step_random(i)
        if collator:
            collator.gather()  # enqueued on the env stream behind the step: no host sync

    env.reset()
    for i in range(args.warmup):
        one_step(i)
    env.physics.sync()
    if comm:
        comm.barrier()
    env.physics.health_clear()  # the timed region's own health counters
    # the step kernel's mean launch time: HIP events around every 4th launch of the timed
    # region (each bracket's two event packets cost ~5 us of the step they sit in)
    _lib.check(L.dx_timing_enable(env.physics.ptr, 4))
    _lib.check(L.dx_timing_read(env.physics.ptr, ctypes.byref(ctypes.c_double()), ctypes.byref(ctypes.c_int32())))
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_step(args.warmup + i)
    env.physics.sync()
    if comm:
        comm.barrier()
    elapsed = time.perf_counter() - t0
    kt, kn = ctypes.c_double(), ctypes.c_int32()
    _lib.check(L.dx_timing_read(env.physics.ptr, ctypes.byref(kt), ctypes.byref(kn)))
    _lib.check(L.dx_timing_enable(env.physics.ptr, 0))
    # a substep-queue timeout would mean corrupted hand-offs: no number is reported then
    qerr = env.physics.debug_get("queue_timeouts")
    refuse = "substep queue timed out during the timed region" if int(qerr[0]) != 0 else ""
    # health of the timed region (include/dx.h dx_health): a diverged env, or a capacity
    # overflow that truncates work (contact pool, candidate lists, Jacobian dofs,
    # constraint rows), voids the number.  Physics steps with more than the 32 contacts
    # the step kernel keeps in LDS (~3.4e-6 of env-substeps on this workload,
    # profiles/r3a_ncon_hist.json) are not truncated: the overflow tier runs them with
    # the 256-contact pool, inside the timed region ("contact_deferred").
    nsub = env.task.config.n_sub_steps
    health = env.physics.health()
    health.pop("ncon_hist")
    env_substeps = B * args.steps * nsub
    bad = {k: v for k, v in health.items() if k in ("diverged", "contact_overflow", "candidate_overflow",
                                                    "jacobian_dof_overflow", "row_overflow") and v}
    if bad:
        refuse = refuse or f"health counters of the timed region {health}"
    # every rank learns whether any rank refuses (no rank is left waiting in a collective)
    if (comm.max(1.0 if refuse else 0.0) if comm else (1.0 if refuse else 0.0)) > 0:
        raise SystemExit(f"rank {rank}: {refuse or 'another rank refused'}; refusing to report")
    health["env_substeps"] = env_substeps
    health["contact_deferred_rate"] = health["contact_deferred"] / env_substeps
    if comm:
        elapsed = comm.max(elapsed)
    total_env_steps = world * B * args.steps
    value = total_env_steps / elapsed
    kernel_ms = kt.value / max(1, kn.value)
    if rank == 0:
        import numpy as np

        ph = env.physics
        idx = np.linspace(0, B - 1, min(FLOP_SAMPLE_ENVS, B)).astype(int)
        sample = [ph.get(f)[idx] for f in (_lib.QPOS, _lib.QVEL, _lib.QACC_WARMSTART, _lib.CTRL)]
        by_stage = oracle_flops_per_env_step(sample, nsub)
        flops = sum(v for k, v in by_stage.items() if k != "scan")
        achieved_tf = flops * B / (kernel_ms * 1e-3) / 1e12
        achieved_gbs = ALGO_BYTES_PER_ENV_STEP * B / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_step_kernel.json")
        if os.path.exists(pmc):
            with open(pmc) as f:
                p = json.load(f)
            # only the build the PMC passes measured (profiles/pmc_step_kernel.json
            # build_key = this library's dx_build_key); otherwise unmeasured
            lib = _lib.load()
            key = lib.dx_build_key().decode() if hasattr(lib, "dx_build_key") else None
            if p.get("envs") == B and p.get("build_key") and p.get("build_key") == key:
                traffic = p.get("hbm_bytes_per_launch")
        host_api = host_api_line(env, args.host_api_steps, 5) if world == 1 and args.host_api_steps > 0 else None
        cpu, extra = None, []
        if world == 1 and not args.no_cpu_baseline:
            gpu_states = [ph.get(f) for f in (_lib.QPOS, _lib.QVEL, _lib.QACC_WARMSTART)]
            threads = host_threads()
            cpu = cpu_baseline(args.cpu_seconds, threads, gpu_states, nsub)
            one = [s[: max(8, B // 256)] for s in gpu_states]
            extra.append(cpu_baseline(args.cpu_seconds / 3, 1, one, nsub))
            extra.append(cpu_baseline_reach_1env(args.cpu_seconds / 3))
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
                # MuJoCo's default and the only solver the reference's scenes run (no
                # solver= anywhere in their MJCF); CG and PGS (config 3' / 3'') are
                # tools/bench_configs.py lines, each with its own kernel specialization
                "solver": "Newton",
                "envs_per_gpu": B,
                "global_envs": world * B,
                "substeps_per_env_step": nsub,
                "physics_dt": 0.005,
                "parallelism": f"env-sharded x{world}" + (", RCCL obs all-gather (libdx)" if world > 1 else ""),
            },
            # the path is FP32-VALU / latency bound: the headline
            # roofline is the oracle-counted FLOPs per env-step over the step kernel's
            # mean launch time against the FP32 vector peak; HBM is the secondary block
            "roofline": {
                "bound": "valu_fp32",
                "achieved": round(achieved_tf, 4),
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 5),
                "traffic": traffic,
                "kernel": "dx_step_kernel",
                "kernel_ms_avg": round(kernel_ms, 4),
                "flops_per_env_step": round(flops),
                "flops_by_stage": {k: round(v) for k, v in by_stage.items() if k != "scan"},
                # the oracle's exhaustive hull scans, were they counted as work
                "flops_per_env_step_full_hull_scan": round(flops + by_stage["scan"]),
                "flops_sample": f"oracle stage counters over {len(idx)} env states of the GPU batch, {nsub} substeps; "
                                "a mesh support is charged 16 vertices (an efficient support), not the full hull",
                "hbm": {
                    "achieved": round(achieved_gbs, 3),
                    "peak": HBM_PEAK_GBS,
                    "unit": "GB/s",
                    "frac": round(achieved_gbs / HBM_PEAK_GBS, 6),
                    "algo_bytes_per_env_step": ALGO_BYTES_PER_ENV_STEP,
                    "traffic": traffic,
                },
            },
            "health": health,
            # the reference's call shape (host action in, host TimeStep out), beside the
            # device-resident headline
            "host_api": host_api,
            "cpu_baseline": cpu,
            "cpu_baseline_extra": extra,
        }
        print(json.dumps(out), flush=True)
    if collator:
        collator.close()
    env.close()
    if comm:
        comm.close()


if __name__ == "__main__":
    main()
