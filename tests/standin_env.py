"""Stand-in environments and planners for tests/test_parallel.py.

A module of its own (not a test file) so that "spawn" worker processes can import what they
unpickle: the factory below replaces EnvWrapper.load, which needs dm_control.
"""
import contextlib

import numpy as np
import torch

from mbrl_amd import env as menv
from mbrl_amd import env_wrappers as ew


class _Step:
    def __init__(self, obs, reward, last):
        self.observation = {"observations": obs}
        self.reward = reward
        self._last = last

    def last(self):
        return self._last


class _Physics:
    def __init__(self, env):
        self._env = env

    def state(self):
        return self._env.x.copy()

    def set_state(self, s):
        self._env.x = np.asarray(s, dtype=np.float64).copy()

    @contextlib.contextmanager
    def reset_context(self):
        yield

    def render(self, camera_id=0):
        return np.zeros((2, 2, 3), np.uint8)


class LinearEnv:
    """dm_env-like linear system: x' = 0.9 x + 0.1 B a, observation = x, reward = -|x|_1; the start
    state is a function of the rollout index; the episode ends after `length` steps."""

    def __init__(self, index, nobs=5, adim=1, length=1000):
        self._spec = menv.BoundedActionSpec(adim, -1.0, 1.0)
        self._B = np.cos(np.arange(nobs * adim, dtype=np.float64)).reshape(nobs, adim)
        self._x0 = np.sin(np.arange(nobs, dtype=np.float64) + 1.7 * index)
        self.x = self._x0.copy()
        self._length, self._t = length, 0
        self.physics = _Physics(self)

    def action_spec(self):
        return self._spec

    def observation_spec(self):
        return {"observations": (self.x.shape[0],)}

    def reset(self):
        self._t = 0
        self.x = self._x0.copy()
        return _Step(self.x.copy(), None, False)

    def step(self, action):
        a = np.asarray(action, dtype=np.float64).reshape(-1)
        self.x = 0.9 * self.x + 0.1 * self._B @ a
        self._t += 1
        return _Step(self.x.copy(), float(-np.abs(self.x).sum()), self._t >= self._length)


class _Wrapper(ew.EnvWrapper):
    state_dim = 5
    observation_dim = 5


def make_env(env_name, task_name, flat_obs=True, index=0):
    """env_factory for get_rollouts_parallel: task_name "short" ends episodes after 3 steps."""
    length = 3 if task_name == "short" else 1000
    return _Wrapper(LinearEnv(index, length=length), flat_obs=flat_obs, env_name=env_name, task_name=task_name)


def broken_env(env_name, task_name, flat_obs=True, index=0):
    raise ValueError("no such environment: {}/{}".format(env_name, task_name))


class FeedbackPlanner:
    """A deterministic stand-in planner: actions = tanh(-obs[:a]) repeated over the horizon."""

    @staticmethod
    def plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kwargs):
        a = sample_action(batch_size=1).shape[1]
        act = torch.tanh(-initial_state.reshape(-1)[:a].float())
        return torch.zeros((horizon, initial_state.shape[-1])), act.reshape(1, a).repeat(horizon, 1)


class BatchFeedbackPlanner(FeedbackPlanner):
    @staticmethod
    def plan_batch(initial_states, model, cost, sample_action, horizon, **kwargs):
        outs = [FeedbackPlanner.plan(s, model, cost, sample_action, horizon) for s in initial_states]
        return torch.stack([o[0] for o in outs]), torch.stack([o[1] for o in outs])


def sample_action_1d(batch_size=None):
    return menv._sample_action(menv.BoundedActionSpec(1), batch_size)


def zero_action(state_and_obs):
    return torch.zeros(1)


def dying_env(env_name, task_name, flat_obs=True, index=0):
    import os
    os._exit(3)
