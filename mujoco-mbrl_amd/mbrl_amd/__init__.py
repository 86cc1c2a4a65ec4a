"""mbrl_amd -- MI355X-native MPC/CEM planning hot path of Khodeir/mujoco-mbrl.

Drop-in for the reference's planner API (src/mbrl/planners.py) and DynamicsModel.forward
(src/mbrl/models.py); the compute runs in the in-tree HIP extension libmbrl_cem.so (C ABI:
include/mbrl_cem.h). See DESIGN.md and INTEGRATION.md at the repository root.
"""
from . import agents, data, env, env_wrappers, gd, models, parallel, planners  # noqa: F401
from .agents import MPCPolicy  # noqa: F401
from .env_wrappers import EnvWrapper  # noqa: F401
from .models import (CoshLoss, CostModel, DynamicsModel, EnsembleModel, LinearModel, Model,  # noqa: F401
                     ModelWithReward, QuadraticCost, SmoothAbsLoss, compose, goal_state_cost, state_action_cost)
from .planners import CEMPlanner, GradientDescentPlanner, ModelPlanner, RandomShootingPlanner  # noqa: F401


def load_extension():
    """Load the HIP extension now (raises ImportError if it is not built)."""
    from . import _lib
    return _lib.load()
