"""Candidate action sampling with the reference's semantics (/root/reference/src/mbrl/env_wrappers.py:50-62).

The reference's EnvWrapper needs dm_control + MuJoCo (absent here, and not on the planning hot
path); `_sample_action` is the one piece the planner receives (agents.py:233), bound as
functools.partial(_sample_action, action_spec=env.action_spec()).
"""
import functools

import numpy as np
import torch


class BoundedActionSpec:
    """Stand-in for dm_env.specs.BoundedArray: .shape, .minimum, .maximum."""

    def __init__(self, dim, minimum=-1.0, maximum=1.0):
        self.shape = (dim,)
        self.minimum = np.broadcast_to(np.asarray(minimum, dtype=np.float64), (dim,)).copy()
        self.maximum = np.broadcast_to(np.asarray(maximum, dtype=np.float64), (dim,)).copy()


def action_bounds(action_spec):
    """env_wrappers.py:52-55: dim-0 bounds, clipped to [-3, 3] (LQR has infinite bounds)."""
    return max(action_spec.minimum[0], -3), min(action_spec.maximum[0], 3)


def _sample_action(action_spec, batch_size=None):
    """env_wrappers.py:50-62: uniform over the dim-0 bounds from the global NumPy RNG, row-major
    [batch, a], float64 -> float32."""
    minimum, maximum = action_bounds(action_spec)
    if batch_size is None:
        action = np.random.uniform(minimum, maximum, action_spec.shape[0])
    else:
        action = np.random.uniform(minimum, maximum, size=action_spec.shape[0] * batch_size).reshape((batch_size, -1))
    return torch.tensor(action, dtype=torch.float32)


def sample_action_fn(action_spec):
    """The sample_action callable the agents hand the planner (agents.py:233)."""
    return functools.partial(_sample_action, action_spec=action_spec)
