"""The MPC policy that calls the planner once per environment step.

MPCPolicy restates /root/reference/src/mbrl/agents.py:29-56 so that the hot path can be driven
the way the reference's agents drive it, without agents.py's training-loop dependencies
(tensorboardX, dm_control): the policy forgets its last plan at timestep 0, passes the previous
plan's tail as `initial_trajectory`, plans with keyword arguments only, and acts with the first
planned action. `plan_kwargs` (an addition) are forwarded to the planner, e.g. CEMPlanner's
num_candidates or distributed=True.
"""
from typing import Dict

import torch


class MPCPolicy:
    def __init__(self, model, cost, planner, sample_action, horizon, **plan_kwargs):
        self.model = model
        self.planner = planner
        self.horizon = horizon
        self.sample_action = sample_action
        self.last_trajectory = None
        self.cost = cost
        self.plan_kwargs = plan_kwargs

    def get_action(self, state_and_obs: Dict[str, torch.Tensor]) -> torch.Tensor:
        """agents.py:37-56."""
        if state_and_obs["timestep"] == 0:
            self.last_trajectory = None
        if self.last_trajectory is not None:
            initial_trajectory = (self.last_trajectory[0][1:], self.last_trajectory[1][0:])
        else:
            initial_trajectory = None
        self.last_trajectory = self.planner.plan(
            initial_state=state_and_obs["observation"],
            model=self.model,
            cost=self.cost,
            sample_action=self.sample_action,
            horizon=self.horizon,
            initial_trajectory=initial_trajectory,
            **self.plan_kwargs,
        )
        return self.last_trajectory[1][0].flatten()
