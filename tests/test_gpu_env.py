"""Environment-level GPU tests through the C ABI: the RCCL collation path, the
observation vector against the fp64 restatement, termination paths, and the
reference's closed-loop known-answer tests."""

import os

import numpy as np
import pytest

from dexterity_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def built():
    from dexterity_amd import build

    build.build()


@pytest.mark.parametrize("n", [64, 4096])
def test_allgather_world1(built, n):
    """dx_allgather_obs over a one-rank RCCL communicator returns exactly the packed
    [obs | reward | discount | step_type] rows of the env (the in-place gather puts
    rank 0's rows at offset 0) -- also at BASELINE config 4's shard size, 4096 x 126."""
    from dexterity_amd import distributed, manipulation

    env = manipulation.load("reorient", "state_dense", seed=3, num_envs=n, device=0)
    comm = distributed.Comm(0, 1, 0, key=f"gputest_{os.getpid()}")
    col = distributed.OutputCollator(env, comm)
    env.reset()
    for i in range(3):
        env.step(env.sample_actions(i), device_action=True)
        col.gather()
    got = col.read()
    ts = env.timestep()
    obs = np.concatenate([ts.observation[k] for k in ts.observation], axis=1).astype(np.float32)
    assert got.shape == (n, env.obs_dim + 3)
    np.testing.assert_array_equal(got[:, : env.obs_dim], obs)
    np.testing.assert_array_equal(got[:, env.obs_dim], ts.reward.astype(np.float32))
    np.testing.assert_array_equal(got[:, env.obs_dim + 1], ts.discount.astype(np.float32))
    np.testing.assert_array_equal(got[:, env.obs_dim + 2], ts.step_type.astype(np.float32))
    assert comm.max(2.5) == 2.5
    comm.barrier()
    col.close()
    comm.close()
    env.close()


def _oracle_for(env, oracle_mod):
    return oracle_mod.OracleModel(env.model.blob)


def _check_observation(env, oracle_mod, builder):
    """Every float of the env's observation vs the fp64 restatement on the env's own
    post-step state (qpos / qvel / goal read back from the device)."""
    from dexterity_amd import _lib

    ts = env.timestep()
    ph = env.physics
    qpos, qvel = ph.get(_lib.QPOS), ph.get(_lib.QVEL)
    goals = env.goals()
    om = _oracle_for(env, oracle_mod)
    worst = {}
    for e in range(env.num_envs):
        d = oracle_mod.OracleData(om)
        d.qpos[:], d.qvel[:] = qpos[e], qvel[e]
        d.observe()
        ref = builder(d, goals[e])
        assert list(ref) == list(ts.observation), (list(ref), list(ts.observation))
        for k, r in ref.items():
            g = ts.observation[k][e]
            assert g.shape == r.shape, k
            err = np.abs(g - r).max() / max(1.0, np.abs(r).max())
            worst[k] = max(worst.get(k, 0.0), err)
    for k, err in worst.items():
        assert err <= 1e-5, (k, err, worst)
    return worst


def test_observation_matches_oracle_reorient(built, oracle_mod):
    """All 123 floats of reorient.state_dense (dexterous_hand.py:250-310, reorient.py:
    81-86, task.py:207-216) within 1e-5 of each field's scale, over 256 envs after 12
    random-action control steps (episodes in every phase, freshly reset ones included)."""
    from dexterity_amd import manipulation
    from oracle import task_ref

    env = manipulation.load("reorient", "state_dense", seed=21, num_envs=256)
    t = env.task
    env.reset()
    for i in range(12):
        env.step(env.sample_actions(i), device_action=True)
    assert env.obs_dim == 123
    sites = list(range(t.tip_site0, t.tip_site0 + t.ntips))
    worst = _check_observation(
        env, oracle_mod,
        lambda d, g: task_ref.reorient_observation(d, t.compiled, t.hand_name, t.hand_nq, t.hand_nv, sites,
                                                   t.prop_body, g))
    assert set(worst) >= {"prop/angular_velocity", "shadow_hand_e/fingertip_linear_velocities"}
    env.close()


@pytest.mark.parametrize("domain", ["reach", "reach_shadow"])
def test_observation_matches_oracle_reach(built, oracle_mod, domain):
    """All 117 floats of reach.state_dense (Adroit) and of the Shadow variant."""
    from dexterity_amd import manipulation
    from oracle import task_ref

    env = manipulation.load(domain, "state_dense", seed=5, num_envs=128)
    t = env.task
    env.reset()
    for i in range(6):
        env.step(env.sample_actions(i), device_action=True)
    assert env.obs_dim == 117
    _check_observation(env, oracle_mod,
                       lambda d, g: task_ref.reach_observation(d, t.hand_name, t.hand_nq, t.hand_nv, t.tip_sites, g))
    env.close()


def _run(env, steps, actions=None):
    from dexterity_amd import _lib

    out = []
    for i in range(steps):
        if actions is None:
            env.step(env.sample_actions(i), device_action=True)
        else:
            env.step(actions)
        ts = env.timestep()
        out.append(dict(st=ts.step_type.copy(), disc=ts.discount.copy(), rew=ts.reward.copy(),
                        succ=env.successes().copy(), goal=env.goals().copy(),
                        watch=env.physics.get(_lib.GROUND_CONTACT)[:, 0].copy(),
                        time=env.physics.get(_lib.TIME)[:, 0].copy()))
    return out


def test_fall_terminates_with_discount_one(built):
    """ReOrient.after_step / get_discount (reorient.py:201-213, 222-225): a prop-ground
    contact ends the episode (LAST) with discount 1.0; the next step returns FIRST."""
    from dexterity_amd import manipulation

    env = manipulation.load("reorient", "state_dense", seed=9, num_envs=512)
    env.reset()
    rec = _run(env, 60)
    falls = 0
    for k in range(1, len(rec)):
        r, prev = rec[k], rec[k - 1]
        mid = prev["st"] != 2  # this step was not an auto-reset
        fell = mid & (r["watch"] == 1)
        assert np.all(r["st"][fell] == 2)
        assert np.all(r["disc"][fell & (r["succ"] == 0)] == 1.0)
        last = mid & (r["st"] == 2)
        # every LAST is a fall, a success or a per-goal timeout (300 steps: not reached here)
        assert np.all(fell[last] | (r["succ"][last] >= 1))
        assert np.all(r["disc"][last & (r["succ"] == 0)] == 1.0)
        assert np.all(r["disc"][last & (r["succ"] >= 1)] == 0.0)
        assert np.all(r["st"][prev["st"] == 2] == 0)  # auto-reset returns FIRST
        falls += int(fell.sum())
    assert falls >= 50
    env.close()


def test_per_goal_timeout(built):
    """GoalTask.after_step / should_terminate_episode (task.py:180-193): time since the
    goal was set > max_time_per_goal without success ends the episode, discount 1.0."""
    from dexterity_amd import manipulation

    cfg = manipulation.ReOrientConfig(max_steps_single_solve=4.5, fall_termination=False,
                                      orientation_threshold=0.0)  # 0.1125 s, never a success
    env = manipulation.GoalEnvironment(manipulation.ReOrient(cfg), num_envs=64, seed=2)
    env.reset()
    rec = _run(env, 7)
    st = np.stack([r["st"] for r in rec])
    for k in range(4):
        assert np.all(st[k] == 1), k
    assert np.all(st[4] == 2)  # t = 0.125 > 0.1125
    assert np.all(rec[4]["disc"] == 1.0)
    assert np.all(st[5] == 0)  # auto-reset
    env.close()


def test_time_limit(built):
    """composer.Environment(time_limit=...) (manipulation/__init__.py:61,83): LAST once
    the physics time reaches the limit, with the task's discount (1.0 here)."""
    from dexterity_amd import manipulation

    env = manipulation.GoalEnvironment(manipulation.ReOrient(manipulation.ReOrientConfig(fall_termination=False)),
                                       num_envs=64, seed=4, time_limit=0.11)
    env.reset()
    rec = _run(env, 6)
    assert all(np.all(rec[k]["st"] == 1) for k in range(4))
    assert np.all(rec[4]["st"] == 2) and np.all(rec[4]["disc"] == 1.0)
    assert np.all(rec[5]["st"] == 0)
    env.close()


def _fp64_time_steps(limit, h, nsub, strict=False):
    """Control step (1-based) at which MuJoCo's fp64 time (time += h per physics step)
    first reaches `limit` (composer's time >= time_limit) or exceeds it (strict: the
    per-goal test time - start > max_time_per_goal)."""
    t, k = 0.0, 0
    while True:
        k += 1
        for _ in range(nsub):
            t += h
        if (t > limit) if strict else (t >= limit):
            return k


@pytest.mark.parametrize("limit", [0.05, 0.25, 1.05])
def test_time_limit_on_control_step_boundary(built, limit):
    """A time limit that is an exact multiple of the control step ends the episode at the
    step fp64 time accumulation gives (MuJoCo's d->time, compared by composer as
    time >= time_limit): 0.05 is reached only after the 3rd control step (the fp64 sum of
    ten 0.005 steps is 0.049999...), 0.25 after the 10th.  An fp32 running time would end
    the 0.25 episode one step late."""
    from dexterity_amd import manipulation

    cfg = manipulation.ReOrientConfig(fall_termination=False)
    env = manipulation.GoalEnvironment(manipulation.ReOrient(cfg), num_envs=8, seed=4, time_limit=limit)
    k = _fp64_time_steps(limit, cfg.physics_timestep, cfg.n_sub_steps)
    env.reset()
    rec = _run(env, k + 1)
    for i in range(k - 1):
        assert np.all(rec[i]["st"] == 1), (limit, i, k)
    assert np.all(rec[k - 1]["st"] == 2), (limit, k)
    assert np.all(rec[k]["st"] == 0)
    env.close()


def test_time_limit_past_fp32_time_resolution(built):
    """A 60 s time limit (12,000 physics steps): the episode ends at the control step
    MuJoCo's fp64 time reaches it.  The env's fp64 time is the sum of exactly as many
    additions of h as physics steps were taken (an integer count that travels with the
    state); recovering that count from the fp32 batch time (rint(t / h)) goes wrong after
    ~11,000 physics steps at h = 0.005."""
    from dexterity_amd import _lib, manipulation

    cfg = manipulation.ReOrientConfig(fall_termination=False)
    env = manipulation.GoalEnvironment(manipulation.ReOrient(cfg), num_envs=8, seed=4, time_limit=60.0)
    _lib.check(_lib.load().dx_env_set_goal_time_limit(env.ptr, 1e9))
    k = _fp64_time_steps(60.0, cfg.physics_timestep, cfg.n_sub_steps)
    assert k == 2400
    env.reset()
    ended = np.zeros(8, dtype=bool)  # envs that ended early (a success): not checked
    for i in range(k + 1):
        env.step_random(i)
        st = env._read(_lib.OUT_STEP_TYPE, np.int32, 1)[:, 0]
        if i < k - 1:
            ended |= st == 2
        elif i == k - 1:
            assert np.all(st[~ended] == 2), (st, ended)
        else:
            assert np.all(st[~ended] == 0)
    assert (~ended).sum() >= 4
    env.close()


def test_fused_task_logic_matches_task_kernels(built, monkeypatch):
    """The reorient task logic fused into the step kernel (task_pre in an env's first
    physics-step task, task_post in its last; dx_task.h) equals the task kernels around
    the step kernel (DX_NO_FUSE=1) bit for bit -- resets, goal changes, rewards,
    observations and the physics state -- over 1024 envs x 30 control steps of random
    actions; and dx_env_step_random (actions drawn in the kernel) equals stepping with
    dx_env_sample_actions' buffer."""
    from dexterity_amd import _lib, manipulation

    outs = []
    for variant in ("kernels", "fused", "random"):
        if variant == "kernels":
            monkeypatch.setenv("DX_NO_FUSE", "1")
        else:
            monkeypatch.delenv("DX_NO_FUSE", raising=False)
        env = manipulation.load("reorient", "state_dense", seed=9, num_envs=1024)
        env.reset()
        sts = []
        for i in range(30):
            if variant == "random":
                env.step_random(i)
            else:
                env.step(env.sample_actions(i), device_action=True)
            sts.append(env._read(_lib.OUT_STEP_TYPE, np.int32, 1)[:, 0])
        ts = env.timestep()
        outs.append((np.stack(sts), ts.reward, ts.discount,
                     np.concatenate([v.reshape(1024, -1) for v in ts.observation.values()], axis=1),
                     env.physics.qpos, env.physics.qvel, env.goals(), env.successes()))
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        env.close()
    assert (outs[0][0] == 2).any() and (outs[0][0] == 0).any()  # episodes ended and restarted
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("domain", ["reach_shadow", "reach"])
def test_fused_reach_matches_task_kernels(built, domain, monkeypatch):
    """Reach with its task logic and sampling pass fused into the step kernel (task_pre,
    goal rollouts / joint sampling in an env's first physics-step task, task_post in its
    last: dx_step.hip fused_reach_prep) equals the task kernels around a separate sampling
    launch (DX_NO_FUSE=1) bit for bit -- resets with their goal and initial-joint draws,
    goal changes, rewards, observations and the physics state -- over 512 envs x 40
    control steps, for the contact-free Shadow reach (BASELINE config 2: the step kernel
    and the order kernel, 2 launches per control step) and the Adroit reach (contacts,
    the overflow tier).  A 0.3 s time limit ends every episode after 12 control steps, so
    the sampling pass also runs inside later control steps (auto-resets), not only at
    the first."""
    from dexterity_amd import _lib, manipulation

    n = 512
    outs = []
    for variant in ("kernels", "fused"):
        if variant == "kernels":
            monkeypatch.setenv("DX_NO_FUSE", "1")
        else:
            monkeypatch.delenv("DX_NO_FUSE", raising=False)
        env = manipulation.load(domain, "state_dense", seed=17, num_envs=n, time_limit=0.3)
        env.reset()
        sts = []
        for i in range(40):
            env.step_random(i)
            sts.append(env._read(_lib.OUT_STEP_TYPE, np.int32, 1)[:, 0])
        ts = env.timestep()
        outs.append((np.stack(sts), ts.reward, ts.discount,
                     np.concatenate([v.reshape(n, -1) for v in ts.observation.values()], axis=1),
                     env.physics.qpos, env.physics.qvel, env.physics.get(_lib.TIME), env.goals(), env.successes(),
                     env.goal_failures()))
        assert env.physics.debug_get("queue_timeouts")[0] == 0
        env.close()
    assert (outs[0][0] == 2).sum() >= n and (outs[0][0] == 0).sum() >= n  # episodes ended and restarted
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("domain", ["reorient", "reach"])
def test_checkpoint_resume_is_bit_exact(built, domain, tmp_path):
    """Checkpoint / resume: a run saved after control step 10 and resumed
    in a fresh env (another seed, so nothing but the checkpoint carries the state) equals
    the uninterrupted run bit for bit at step 25 -- physics, task counters, goals,
    observations, and the MT19937 streams that later resets draw from (episodes end and
    restart within the window)."""
    from dexterity_amd import _lib, manipulation

    task = "state_dense"
    n = 512

    def run(env, steps):
        st = []
        for i in steps:
            env.step_random(i)
            st.append(env._read(_lib.OUT_STEP_TYPE, np.int32, 1)[:, 0])
        return np.stack(st)

    def outputs(env):
        ts = env.timestep()
        return (ts.reward, ts.discount, ts.step_type,
                np.concatenate([v.reshape(n, -1) for v in ts.observation.values()], axis=1),
                env.physics.qpos, env.physics.qvel, env.physics.get(_lib.QACC_WARMSTART), env.goals(),
                env.successes())

    a = manipulation.load(domain, task, seed=21, num_envs=n)
    a.reset()
    run(a, range(10))
    path = str(tmp_path / "ckpt.npz")
    a.save(path)
    sa = run(a, range(10, 25))
    ref = outputs(a)
    a.close()
    b = manipulation.load(domain, task, seed=99, num_envs=n)
    b.reset()
    b.load(path)  # restores the random agent's key (seed 21) too
    assert b._seed == 21
    sb = run(b, range(10, 25))
    got = outputs(b)
    b.close()
    if domain == "reorient":
        assert (sa == 2).any() and (sa == 0).any()  # episodes ended and restarted in the window
    np.testing.assert_array_equal(sa, sb)
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)
    with np.load(path) as z:
        assert z["qpos"].shape[0] == n and z["time_d"].dtype == np.float64


def test_goal_time_limit_on_control_step_boundary(built):
    """max_time_per_goal = 2 control steps (0.05 s): GoalTask's time - start > max_time
    in fp64 is first true after the 3rd step (task.py:180-183)."""
    from dexterity_amd import manipulation

    cfg = manipulation.ReOrientConfig(max_steps_single_solve=2, fall_termination=False, orientation_threshold=0.0)
    env = manipulation.GoalEnvironment(manipulation.ReOrient(cfg), num_envs=8, seed=5)
    k = _fp64_time_steps(cfg.max_time_per_goal, cfg.physics_timestep, cfg.n_sub_steps, strict=True)
    assert k == 3
    env.reset()
    rec = _run(env, k + 1)
    assert all(np.all(rec[i]["st"] == 1) for i in range(k - 1))
    assert np.all(rec[k - 1]["st"] == 2) and np.all(rec[k - 1]["disc"] == 1.0)
    env.close()


def test_goal_change_after_successes(built):
    """GoalTask.before_step / after_step (task.py:154-185): with every step a success
    (threshold above any orientation distance), the success counter passes
    steps_before_changing_goal = 5, the next before_step draws a new goal, and the
    success is registered again once per goal -- compared step by step with a host
    restatement of the bookkeeping."""
    from dexterity_amd import manipulation

    cfg = manipulation.ReOrientConfig(orientation_threshold=4.0, successes_needed=1000, fall_termination=False)
    env = manipulation.GoalEnvironment(manipulation.ReOrient(cfg), num_envs=32, seed=8)
    env.reset()
    g0 = env.goals().copy()
    rec = _run(env, 20)
    counter, successes, registered = 0, 0, False
    prev_goal = g0
    for k, r in enumerate(rec):
        changed = counter > cfg.steps_before_moving_target
        if changed:
            counter, registered = 0, False
        counter += 1
        if not registered:
            successes += 1
            registered = True
        assert np.all(r["succ"] == successes), (k, r["succ"][:4], successes)
        moved = np.any(r["goal"] != prev_goal, axis=1)
        assert np.all(moved == changed), k
        np.testing.assert_allclose(np.linalg.norm(r["goal"], axis=1), 1.0, atol=1e-6)
        assert np.all(r["st"] == 1)
        prev_goal = r["goal"]
    env.close()


def test_reach_sparse_closed_loop_kat(built):
    """reach_test.py:12-35: sparse reward -1 after a zero action; then the control that
    holds the goal's joint configuration (hand.joint_positions_to_control(goal qpos))
    drives every fingertip within the threshold, and the step that registers the first
    success has reward exactly 0."""
    from dexterity_amd import manipulation

    n = 32
    env = manipulation.load("reach", "state_sparse", seed=12345, num_envs=n)
    env.reset()
    ts = env.step(np.zeros((n, env.model.nu), np.float32))
    # -1 per fingertip farther than 1 cm from its goal, averaged (reach.py:196-210); the
    # reference's single seed starts with every fingertip far (reward -1); here each
    # env has its own draw, so a fingertip may start within reach
    tips = ts.observation["adroit_hand/fingertip_positions"].reshape(n, 5, 3)
    far = np.linalg.norm(tips - env.goals().reshape(n, 5, 3), axis=2) > 0.01
    np.testing.assert_allclose(ts.reward, -far.mean(axis=1), atol=1e-6)  # fp32 mean
    assert np.mean(ts.reward == -1.0) >= 0.75
    qsol = env.goal_qpos().astype(np.float64)
    ctrl = (qsol @ np.asarray(env.task.position_to_control, dtype=np.float64).T).astype(np.float32)
    first = np.full(n, -1)
    reward_at = np.zeros(n)
    for k in range(150):
        ts = env.step(ctrl)
        succ = env.successes()
        new = (first < 0) & (succ > 0)
        first[new] = k
        reward_at[new] = ts.reward[new]
        assert np.all(ts.step_type[first < 0] == 1)  # no episode ends before its first success
        if np.all(first >= 0):
            break
    assert np.all(first >= 0), first
    np.testing.assert_array_equal(reward_at, 0.0)
    env.close()


def test_reset_zeroes_ctrl(built):
    """dx_env_reset = mj_resetData + initialize_episode: ctrl is zero afterwards."""
    from dexterity_amd import _lib, manipulation

    env = manipulation.load("reorient", "state_dense", seed=1, num_envs=16)
    env.reset()
    env.step(env.sample_actions(0), device_action=True)
    assert np.abs(env.physics.get(_lib.CTRL)).max() > 0
    env.reset()
    np.testing.assert_array_equal(env.physics.get(_lib.CTRL), 0.0)
    env.close()


def test_unstripped_observation_buffer_dim(built):
    from dexterity_amd import manipulation

    env = manipulation.load("reorient", "state_dense", seed=1, num_envs=4, strip_singleton_obs_buffer_dim=False)
    ts = env.reset()
    for k, spec in env.observation_spec().items():
        assert ts.observation[k].shape == (4,) + spec.shape and spec.shape[0] == 1
    env.close()


def _uniform_quaternion(rs):
    """[3P] dm_control rotations.UniformQuaternion.__call__ with a RandomState."""
    u1, u2, u3 = rs.uniform([0.0] * 3, [1.0, 2 * np.pi, 2 * np.pi])
    return np.array([np.sqrt(1 - u1) * np.sin(u2), np.sqrt(1 - u1) * np.cos(u2), np.sqrt(u1) * np.sin(u3),
                     np.sqrt(u1) * np.cos(u3)])


def test_reorient_resets_replay_numpy_random_state(built):
    """Seed-level reset parity: env e of a batch seeded s is the
    reference env `load("reorient", "state_dense", seed=s + e)` with numpy's global
    stream seeded s + e.  Replaying numpy in the reference's order -- the goal from the
    global stream (task.py:137-152, prop_orientation.py:34-38), then PropPlacer's
    position (3 uniform draws in the bbox) and quaternion from the env's RandomState
    (reorient.py:143-151, 182-188) -- gives the device's initial goal and prop pose bit
    for bit after the fp32 cast, for the first episode and for every auto-reset
    episode that follows."""
    from dexterity_amd import _lib, manipulation

    seed, n = 777, 128
    env = manipulation.load("reorient", "state_dense", seed=seed, num_envs=n)
    cfg = env.task.config
    lo, hi = np.array(cfg.prop_bbox_lower), np.array(cfg.prop_bbox_upper)
    env_rs = [np.random.RandomState(seed + e) for e in range(n)]
    glob_rs = [np.random.RandomState(seed + e) for e in range(n)]
    qa = env.task.prop_qadr

    def expect(e):
        g = _uniform_quaternion(glob_rs[e])
        pos = env_rs[e].uniform(lo, hi)
        q = _uniform_quaternion(env_rs[e])
        return g.astype(np.float32), pos.astype(np.float32), q.astype(np.float32)

    def check(envs):
        qpos = env.physics.get(_lib.QPOS)
        goals = env.goals()
        for e in envs:
            g, pos, q = expect(e)
            np.testing.assert_array_equal(goals[e], g)
            np.testing.assert_array_equal(qpos[e, qa:qa + 3], pos)
            np.testing.assert_array_equal(qpos[e, qa + 3:qa + 7], q)

    ts = env.reset()
    assert np.all(ts.step_type == 0)
    check(range(n))
    resets = 0
    for i in range(80):
        env.step(env.sample_actions(i), device_action=True)
        first = np.nonzero(env.timestep().step_type == 0)[0]
        check(first)
        resets += len(first)
    assert resets >= 40
    env.close()


def test_collision_free_joint_sampling_kat(built, oracle_mod):
    """hands_test.py:100-110: joint angles drawn by sample_collision_free_joint_angles
    (dexterous_hand.py:144-168, here over the full joint range) put the Adroit hand in
    no self-contact -- checked by the fp64 oracle's collision pass at every env's
    sampled configuration (has_self_collision: any hand-hand contact with dist <= 1e-8,
    utils/mujoco_collisions.py:95-127)."""
    from dexterity_amd import _lib, manipulation

    cfg = manipulation.ReachConfig(init_joint_range_fraction=1.0)
    env = manipulation.GoalEnvironment(manipulation.Reach(cfg, hand="adroit"), num_envs=64, seed=12345)
    ts = env.reset()
    assert np.all(ts.step_type == 0)
    qpos = env.physics.get(_lib.QPOS).astype(np.float64)
    cm = env.task.compiled
    lo, hi = np.asarray(cm.jnt_range, dtype=np.float64)[: cm.nq].T
    assert np.all(qpos >= lo - 1e-6) and np.all(qpos <= hi + 1e-6)
    om = oracle_mod.OracleModel(env.model.blob)
    spread = qpos.std(axis=0)
    assert np.all(spread[hi > lo] > 0.05 * (hi - lo)[hi > lo])  # really spread over the range
    touching = 0
    for e in range(env.num_envs):
        d = oracle_mod.OracleData(om)
        d.qpos[:] = qpos[e]
        d.kinematics()
        c = d.contacts()
        dist = c[:, 12] if len(c) else np.zeros(0)
        assert np.all(dist > -1e-6), (e, dist.min())  # fp32 sampling vs fp64 check
        touching += int(np.any(dist <= 1e-8))
    assert touching == 0
    env.close()


@pytest.mark.parametrize("domain,max_reject", [("reach", 100), ("reach_shadow", 100), ("reach", 1), ("reach", 2)])
def test_reach_resets_replay_numpy_random_state(built, domain, max_reject):
    """Seed-level reset parity for reach: env e's RandomState(seed + e)
    feeds, in the reference's order, the goal sampler -- random_state.normal(midrange,
    0.1 range) per rejection attempt (fingertip_position.py:79-86, numpy's polar
    gaussians with the cached second value) -- and then the initial joints --
    random_state.uniform(0.5 lo, 0.5 hi) per attempt (dexterous_hand.py:137-168), with
    the Shadow hand's coupled joints equalised.  Replaying numpy, the device's initial
    joints equal one of the first uniform draws after one of the first goal attempts,
    bit for bit after the fp32 cast."""
    from dexterity_amd import _lib, hands, manipulation

    seed, n = 4321, 64
    if max_reject == 100:
        env = manipulation.load(domain, "state_dense", seed=seed, num_envs=n)
    else:
        # forced GoalInitializationErrors: with 1 or 2 rejection samples per next_goal
        # call most resets raise and are retried (environment.py:14-34); the retries
        # continue the env's RandomState, so the replay below is unchanged
        cfg = manipulation.ReachConfig(max_rejection_samples=max_reject)
        env = manipulation.GoalEnvironment(manipulation.Reach(cfg, hand="adroit"), num_envs=n, seed=seed)
    t = env.task
    lo, hi = t.joint_range[:, 0], t.joint_range[:, 1]
    mid = t.joint_range.mean(axis=1)
    frac = t.config.init_joint_range_fraction
    env.reset()
    qpos = env.physics.get(_lib.QPOS)
    fails = env.goal_failures()
    attempts = []
    for e in range(n):
        found = None
        # goal attempts: the accepted draw follows fails[e] exhausted batches of max_reject
        # (one GoalInitializationError each), so it is draw fails * max_reject + 1 .. + max_reject
        kgs = range(1, 101) if max_reject == 100 else range(fails[e] * max_reject + 1, (fails[e] + 1) * max_reject + 1)
        for kg in kgs:
            rs = np.random.RandomState(seed + e)
            for _ in range(kg):
                rs.normal(loc=mid, scale=t.config.goal_scale * (hi - lo))
            # the next 400 joint attempts at once (uniform over [400, nq] consumes the
            # stream exactly as 400 successive uniform(lo, hi) calls)
            q = rs.uniform(frac * lo, frac * hi, size=(400, len(lo)))
            if domain == "reach_shadow":
                for ids in hands.COUPLED_JOINT_IDS:
                    q[:, ids] = q[:, [ids[-1]]]
            hit = np.nonzero(np.all(q.astype(np.float32) == qpos[e], axis=1))[0]
            if len(hit):
                found = (kg, int(hit[0]) + 1)
                break
        assert found is not None, (e, fails[e])
        attempts.append(found)
        if max_reject == 100:
            assert fails[e] == 0
    assert max(a[0] for a in attempts) >= 1
    if max_reject < 100:
        assert max(a[0] for a in attempts) > max_reject and fails.sum() > 0  # the retry path ran
    if domain == "reach_shadow":  # contacts disabled: every first draw is accepted
        assert all(a == (1, 1) for a in attempts)
    env.close()


@pytest.mark.parametrize("name", ["reach.state_dense", "reach.state_sparse", "reach_shadow.state_dense",
                                  "reorient.state_dense"])
def test_task_runs(built, name):
    """manipulation_test.py:23-46 for every registered task: 5 episodes x 10 steps from
    seed 12345 with uniform random actions within the action spec; every observation
    matches its spec (shape, finite) and every discount lies in [0, 1].  Batched: 16
    envs; a FIRST step reports reward 0 and discount 1 where dm_env has None."""
    from dexterity_amd import manipulation

    domain, task = name.split(".")
    n = 16
    env = manipulation.load(domain, task, seed=12345, num_envs=n)
    rs = np.random.RandomState(12345)
    obs_spec, act_spec = env.observation_spec(), env.action_spec()
    assert np.all(np.isfinite(act_spec.minimum)) and np.all(np.isfinite(act_spec.maximum))
    for _ in range(5):
        ts = env.reset()
        for _ in range(10):
            assert list(ts.observation) == list(obs_spec)
            for k, spec in obs_spec.items():
                v = ts.observation[k]
                assert v.shape == (n,) + spec.shape and np.all(np.isfinite(v)), k
            first = ts.step_type == 0
            assert np.all(ts.reward[first] == 0) and np.all(ts.discount[first] == 1)
            assert np.all((ts.discount >= 0) & (ts.discount <= 1))
            action = rs.uniform(act_spec.minimum, act_spec.maximum, size=(n,) + act_spec.shape)
            ts = env.step(action.astype(act_spec.dtype))
    env.close()


def _snapshot(env):
    from dexterity_amd import _lib

    ts = env.timestep()
    obs = np.concatenate([ts.observation[k] for k in ts.observation], axis=1).astype(np.float32)
    return {"qpos": env.physics.get(_lib.QPOS), "qvel": env.physics.get(_lib.QVEL), "goal": env.goals(),
            "obs": obs, "reward": ts.reward, "step_type": ts.step_type}


@pytest.mark.parametrize("domain", ["reorient", "reach"])
def test_shard_matches_unsharded_batch(built, domain):
    """A dx_env created for rank 1 of a two-rank job (env_offset = B) is envs B..2B-1 of
    one 2B-env batch with the same seed: resets (goals, prop pose, reach joints), the
    device-sampled actions and every output over 12 control steps agree bit for bit."""
    from dexterity_amd import manipulation

    seed, n = 4242, 48
    whole = manipulation.load(domain, "state_dense", seed=seed, num_envs=2 * n)
    shard = manipulation.load(domain, "state_dense", seed=seed, num_envs=n, env_offset=n)
    whole.reset()
    shard.reset()
    for i in range(13):
        a, b = _snapshot(whole), _snapshot(shard)
        for k in a:
            np.testing.assert_array_equal(a[k][n:], b[k], err_msg=f"{k} at step {i}")
        if i == 12:
            break
        pa, pb = whole.sample_actions(i), shard.sample_actions(i)
        ha = np.empty((2 * n, whole.model.nu), np.float32)
        hb = np.empty((n, shard.model.nu), np.float32)
        whole.physics.sync()
        shard.physics.sync()
        manipulation._copy_d2h(ha, pa)
        manipulation._copy_d2h(hb, pb)
        np.testing.assert_array_equal(ha[n:], hb)
        whole.step(pa, device_action=True)
        shard.step(pb, device_action=True)
    whole.close()
    shard.close()


def _shard_worker(rank, world, n, seed, steps, q):
    from dexterity_amd import distributed, manipulation

    env0, cnt = distributed.env_shard(world * n, rank, world)
    env = manipulation.load("reorient", "state_dense", seed=seed, num_envs=cnt, env_offset=env0)
    env.reset()
    for i in range(steps):
        env.step(env.sample_actions(i), device_action=True)
    q.put((rank, _snapshot(env)))
    env.close()


@pytest.mark.parametrize("n", [64, 4096])
def test_sharded_job_two_processes(built, n, monkeypatch):
    """The sharded job of bench.py on one GPU: two processes step their own shards
    (env_offset from distributed.env_shard); their rows, placed at
    distributed.gathered_rows, equal one process stepping the whole job.  At BASELINE
    config 4's shard size (4096 envs per rank, an 8192-env job, env_offset 4096) with
    physics steps past 20 contacts deferred to the mid tier and past 24 to the overflow
    tier (DX_DEFER_AT / DX_MID_DEFER_AT), so both tiers run in every rank."""
    import multiprocessing as mp

    from dexterity_amd import distributed, manipulation

    world, seed, steps = 2, 12345, 8
    if n >= 4096:
        monkeypatch.setenv("DX_DEFER_AT", "20")
        monkeypatch.setenv("DX_MID_DEFER_AT", "24")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, n, seed, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = manipulation.load("reorient", "state_dense", seed=seed, num_envs=world * n)
    whole.reset()
    for i in range(steps):
        whole.step(whole.sample_actions(i), device_action=True)
    ref = _snapshot(whole)
    for r in range(world):
        sl = distributed.gathered_rows(r, n)
        for k in ref:
            np.testing.assert_array_equal(ref[k][sl], got[r][k], err_msg=f"rank {r} {k}")
    if n >= 4096:
        h = whole.physics.health()
        assert h["contact_deferred"] > 0 and h["contact_overflow"] == 0, h
    whole.close()


def test_effector_set_control_round_trip(built):
    """hand_effector_test.py:12-20 / mujoco_actuation.py:30-33: set_control writes the
    command into ctrl -- the hand effector over every actuator straight to the device, a
    subset effector leaving the other actuators' ctrl as they were."""
    from dexterity_amd import effectors, manipulation

    env = manipulation.load("reorient", "state_dense", seed=1, num_envs=4)
    ph, nu = env.physics, env.physics.model.nu
    cmd = np.random.RandomState(0).uniform(-1, 1, size=(4, nu)).astype(np.float32)
    env.task.hand_effector.set_control(ph, cmd)
    np.testing.assert_array_equal(ph.get(_lib.CTRL), cmd)
    effectors.MujocoEffector([1, 3, 5]).set_control(ph, np.full((4, 3), 0.5, np.float32))
    expect = cmd.copy()
    expect[:, [1, 3, 5]] = 0.5
    np.testing.assert_array_equal(ph.get(_lib.CTRL), expect)
    env.close()


def test_handover_observation_and_reward(built, oracle_mod):
    """BASELINE config 5 as a task (manipulation.load("bimanual", "state_dense"): two
    Shadow hands hand the cube over, dexterity_amd.manipulation.Handover): every float of
    the 221-float observation against task_ref.handover_observation on the env's own
    post-step state (within 1e-5 of each field's scale), and every MID step's reward
    against task_ref.handover_reward on the same step's cube position, goal and ctrl
    (rel 2e-4), over 256 envs after 8 random-action control steps."""
    from dexterity_amd import _lib, manipulation
    from oracle import task_ref

    env = manipulation.load("bimanual", "state_dense", seed=4, num_envs=256)
    t = env.task
    ts = env.reset()
    assert env.obs_dim == 221 and env.goal_dim == 4
    np.testing.assert_allclose(env.goals()[:, :3], np.tile(t.config.hand_targets[1], (256, 1)), atol=1e-7)
    assert np.all(env.goals()[:, 3] == 1.0) and np.all(ts.step_type == 0)
    # the cube spawns in the left hand's box (uniform position, uniform quaternion)
    q = env.physics.qpos
    lo, hi = np.array(t.config.prop_bbox_lower), np.array(t.config.prop_bbox_upper)
    assert np.all(q[:, t.prop_qadr:t.prop_qadr + 3] >= lo - 1e-6) and np.all(q[:, t.prop_qadr:t.prop_qadr + 3] <= hi + 1e-6)
    for i in range(8):
        env.step(env.sample_actions(i), device_action=True)
    sites = list(range(t.tip_site0, t.tip_site0 + t.ntips))
    worst = _check_observation(
        env, oracle_mod,
        lambda d, g: task_ref.handover_observation(d, t.compiled, t.hand_names, t.hand_nq, sites, t.prop_body, g))
    assert set(worst) >= {"prop/angular_velocity", "shadow_hand_right/fingertip_linear_velocities"}
    ts = env.timestep()
    qpos, ctrl, goals = env.physics.qpos, env.physics.get(_lib.CTRL), env.goals()
    mid = ts.step_type == 1
    assert mid.sum() > 128
    for e in np.flatnonzero(mid):
        dist = float(np.linalg.norm(qpos[e, t.prop_qadr:t.prop_qadr + 3].astype(np.float64) - goals[e, :3]))
        ref = task_ref.handover_reward(dist, ctrl[e].astype(np.float64), t.config)
        assert abs(ts.reward[e] - ref) <= 2e-4 * max(1.0, abs(ref)), (e, ts.reward[e], ref)
    env.close()


def test_handover_goal_switches_hands(built):
    """GoalTask.before_step (task.py:154-165) on the handover: with every step a success
    (threshold above any distance), after steps_before_changing_goal successes the goal
    moves to the other hand's target and back, registered once per goal -- step by step
    against a host restatement; the host action path (dx_env_step_host) steps the env."""
    from dexterity_amd import manipulation

    cfg = manipulation.HandoverConfig(success_threshold=10.0, successes_needed=1000, fall_termination=False)
    env = manipulation.GoalEnvironment(manipulation.Handover(cfg), num_envs=32, seed=5)
    env.reset()
    targets = np.array(cfg.hand_targets)
    counter, successes, registered, hand = 0, 0, False, 1
    for k in range(20):
        ts = env.step(np.zeros((32, env.model.nu), dtype=np.float32))
        if counter > cfg.steps_before_moving_target:
            counter, registered, hand = 0, False, 1 - hand
        counter += 1
        if not registered:
            successes, registered = successes + 1, True
        g = env.goals()
        assert np.all(env.successes() == successes), (k, successes)
        np.testing.assert_allclose(g[:, :3], np.tile(targets[hand], (32, 1)), atol=1e-7)
        assert np.all(g[:, 3] == hand) and np.all(ts.step_type == 1)
        np.testing.assert_array_equal(ts.observation["goal_state"], g.astype(np.float64))
    assert successes >= 3
    env.close()


def test_handover_fall_terminates(built):
    """The handover's fall rule (reorient.py:229-235 on the two-hand scene): a cube-ground
    contact ends the episode (LAST) with discount 1.0 and the next step returns FIRST; the
    random agent drops the cube from the left palm within 60 control steps in most envs."""
    from dexterity_amd import manipulation

    env = manipulation.load("bimanual", "state_dense", seed=11, num_envs=256)
    env.reset()
    rec = _run(env, 60)
    falls = 0
    for k in range(1, len(rec)):
        r, prev = rec[k], rec[k - 1]
        mid = prev["st"] != 2
        fell = mid & (r["watch"] == 1)
        assert np.all(r["st"][fell] == 2)
        assert np.all(r["disc"][fell & (r["succ"] < 3)] == 1.0)
        assert np.all(r["st"][prev["st"] == 2] == 0)
        falls += int(fell.sum())
    assert falls >= 20
    env.close()
