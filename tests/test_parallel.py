"""Parallel environment rollouts feeding one planner service (mbrl_amd.parallel, restating
/root/reference/src/mbrl/parallel.py:14-52). Spawned worker processes step
stand-in environments (tests/standin_env.py; dm_control is absent, §8c); the parent serves their
action requests, batched through plan_batch when the planner has one."""
import functools

import numpy as np
import pytest
import torch

import standin_env as se
from mbrl_amd import MPCPolicy, parallel


def _sequential(task, n, policy=None, num_steps=4):
    out = []
    for i in range(n):
        env = se.make_env("linear", task, index=i)
        ga = None
        if policy is not None:
            import copy
            ga = copy.copy(policy).get_action
        out.append(env.get_rollout(num_steps=num_steps, get_action=ga) if ga else None)
    return out


def _same(r1, r2):
    assert len(r1) == len(r2)
    for f in ("states", "observations", "actions", "rewards"):
        for x, y in zip(getattr(r1, f), getattr(r2, f)):
            if x is None or y is None:
                assert x is None and y is None, f
                continue
            assert torch.equal(torch.as_tensor(x).float(), torch.as_tensor(y).float()), f


@pytest.mark.parametrize("planner", [se.BatchFeedbackPlanner, se.FeedbackPlanner], ids=["plan_batch", "plan"])
@pytest.mark.parametrize("workers", [1, 2, 3])
def test_served_policy_matches_in_process_rollouts(planner, workers):
    pol = MPCPolicy(None, None, planner, se.sample_action_1d, 6)
    batches = []
    rs = parallel.get_rollouts_parallel("linear", "run", True, 4, dict(num_steps=5, get_action=pol.get_action),
                                        num_workers=workers, env_factory=se.make_env,
                                        on_batch=lambda i, o, a: batches.append((list(i), o, a)))
    ref = _sequential("run", 4, pol, num_steps=5)
    assert len(rs) == 4
    for r, q in zip(rs, ref):
        _same(r, q)
    # lockstep batches: one request per running worker, ordered by rollout index
    assert len(batches) == 5 * -(-4 // workers)   # rounds = steps x rollouts on the busiest worker
    for idx, o, a in batches:
        assert idx == sorted(idx) and len(idx) <= workers
        assert o.shape == (len(idx), 5) and a.shape == (len(idx), 1)


def test_episodes_that_end_early_leave_the_lockstep():
    pol = MPCPolicy(None, None, se.BatchFeedbackPlanner, se.sample_action_1d, 6)
    rs = parallel.get_rollouts_parallel("linear", "short", True, 3, dict(num_steps=10, get_action=pol.get_action),
                                        num_workers=2, env_factory=se.make_env)
    assert [len(r) for r in rs] == [3, 3, 3]
    for r, q in zip(rs, _sequential("short", 3, pol, num_steps=10)):
        _same(r, q)


def test_unserved_get_action_runs_in_the_workers():
    """A plain callable is pickled into the workers, as the reference does with every policy."""
    rs = parallel.get_rollouts_parallel("linear", "run", True, 3, dict(num_steps=4, get_action=se.zero_action),
                                        num_workers=2, env_factory=se.make_env)
    assert [len(r) for r in rs] == [4, 4, 4]
    assert all(torch.equal(torch.as_tensor(a), torch.zeros(1)) for r in rs for a in r.actions[:-1])


def test_record_rollout_and_mp4path_index():
    rs = parallel.get_rollouts_parallel("linear", "run", True, 2, dict(num_steps=3, mp4path="/nonexistent/m"),
                                        num_workers=2, env_factory=se.make_env)
    assert [len(r.frames) for r in rs] == [3, 3]


def test_worker_errors_reach_the_caller():
    with pytest.raises(RuntimeError, match="no such environment"):
        parallel.get_rollouts_parallel("nope", "run", True, 2, dict(num_steps=3), num_workers=2,
                                       env_factory=se.broken_env)


def test_default_loader_needs_dm_control():
    try:
        import dm_control  # noqa: F401
        pytest.skip("dm_control present")
    except ImportError:
        pass
    with pytest.raises(RuntimeError, match="dm_control"):
        parallel.get_rollouts_parallel("cartpole", "swingup", True, 1, dict(num_steps=3), num_workers=1)


@pytest.mark.gpu
def test_gpu_planner_service_serves_cem_batches():
    """Workers step environments; the parent plans every lockstep round with one
    CEMPlanner.plan_batch (mbrl_cem_plan_batch) on the GPU."""
    from mbrl_amd import CEMPlanner, data, fused, models
    from mbrl_amd import env as menv
    from mbrl_amd import env_wrappers as ew
    torch.manual_seed(0)
    m = models.Model(5, 1, hidden_units=256, n_hidden=2)
    ds = data.TransitionsDataset.from_statistics({"observations": {"mean": torch.zeros(5), "std": torch.ones(5)},
                                                  "actions": {"mean": torch.zeros(1), "std": torch.ones(1)}})
    cost = models.goal_state_cost(models.SmoothAbsLoss(torch.ones(5), torch.zeros(5)), models.CoshLoss())
    sample_action = functools.partial(ew.EnvWrapper._sample_action, action_spec=menv.BoundedActionSpec(1))
    model_fn = functools.partial(m, **ds.normalizers())
    assert fused.describe_model(model_fn) is not None
    pol = MPCPolicy(model_fn, cost, CEMPlanner, sample_action, 10, num_candidates=256, seed=11)
    batches = []
    rs = parallel.get_rollouts_parallel("linear", "run", True, 3, dict(num_steps=4, get_action=pol.get_action),
                                        num_workers=2, env_factory=se.make_env,
                                        on_batch=lambda i, o, a: batches.append((list(i), o, a)))
    answers = {i: [] for i in range(3)}
    for idx, obs, acts in batches:
        _, ref = CEMPlanner.plan_batch(obs, model_fn, cost, sample_action, 10, num_candidates=256, seed=11)
        assert torch.equal(ref[:, 0].reshape(len(idx), -1), acts)
        for b, i in enumerate(idx):
            answers[i].append(acts[b])
    for i, r in enumerate(rs):
        assert len(r) == 4
        assert all(torch.equal(torch.as_tensor(x).reshape(-1), y) for x, y in zip(r.actions[:-1], answers[i]))


def test_a_dead_worker_is_reported():
    with pytest.raises(RuntimeError, match="died"):
        parallel.get_rollouts_parallel("linear", "run", True, 2, dict(num_steps=3), num_workers=2,
                                       env_factory=se.dying_env)


@pytest.mark.gpu
def test_gpu_planner_service_serves_gradient_descent_batches_with_warm_starts():
    """GradientDescentPlanner through the service: one plan_batch (mbrl_gd_plan_batch) per lockstep
    round, each row warm-started from its own rollout's previous plan exactly as its MPCPolicy would
    (agents.py:40-55) -- the rollouts equal in-process rollouts with per-rollout MPCPolicy copies."""
    from mbrl_amd import GradientDescentPlanner, data, fused, models
    torch.manual_seed(0)
    m = models.Model(5, 1, hidden_units=64, n_hidden=2)
    ds = data.TransitionsDataset.from_statistics({"observations": {"mean": torch.zeros(5), "std": torch.ones(5)},
                                                  "actions": {"mean": torch.zeros(1), "std": torch.ones(1)}})
    cost = models.goal_state_cost(models.SmoothAbsLoss(torch.ones(5), torch.zeros(5)), models.CoshLoss())
    model_fn = functools.partial(m, **ds.normalizers())
    assert fused.describe_model(model_fn) is not None

    def sample_action(batch_size):           # deterministic: the worker processes and the parent agree
        return torch.linspace(-0.5, 0.5, batch_size).reshape(batch_size, 1)
    pol = MPCPolicy(model_fn, cost, GradientDescentPlanner, sample_action, 6, num_iterations=15, device="cuda:0")
    rs = parallel.get_rollouts_parallel("linear", "run", True, 3, dict(num_steps=4, get_action=pol.get_action),
                                        num_workers=3, env_factory=se.make_env)
    ref = _sequential("run", 3, pol, num_steps=4)
    for r, q in zip(rs, ref):
        _same(r, q)
