"""Normalisation statistics with the reference's API (/root/reference/src/mbrl/data.py:229-269).

Only the part of TransitionsDataset the planner touches: the statistics dict and the static
normalize_field / unnormalize_field the agents bind with functools.partial (agents.py:219-221).
"""
import functools

import torch


class TransitionsDataset:
    def __init__(self, statistics=None):
        self.statistics = statistics if statistics is not None else {}

    @staticmethod
    def unnormalize_field(field_value, field_name, stats):
        """data.py:255-257."""
        return (field_value * stats[field_name]["std"]) + stats[field_name]["mean"]

    @staticmethod
    def normalize_field(field_value, field_name, stats):
        """data.py:258-260."""
        return (field_value - stats[field_name]["mean"]) / stats[field_name]["std"]

    @staticmethod
    def _get_stats(array):
        """data.py:262-269 (torch.std is the unbiased estimator)."""
        return {
            "mean": torch.mean(array, dim=0),
            "std": torch.std(array, dim=0),
            "min": torch.min(array, dim=0).values,
            "max": torch.max(array, dim=0).values,
        }

    def set_statistics(self, observations, actions, rewards=None):
        self.statistics["observations"] = self._get_stats(observations)
        self.statistics["actions"] = self._get_stats(actions)
        if rewards is not None:
            self.statistics["rewards"] = self._get_stats(rewards)

    def normalizers(self, reward=False):
        """The three partials GoalStateAgent builds (agents.py:219-221); with reward=True also
        RewardAgent's unnormalize_reward (agents.py:340)."""
        st = self.statistics
        out = dict(
            normalize_state=functools.partial(self.normalize_field, field_name="observations", stats=st),
            unnormalize_state=functools.partial(self.unnormalize_field, field_name="observations", stats=st),
            normalize_action=functools.partial(self.normalize_field, field_name="actions", stats=st),
        )
        if reward:
            out["unnormalize_reward"] = functools.partial(self.unnormalize_field, field_name="rewards", stats=st)
        return out
