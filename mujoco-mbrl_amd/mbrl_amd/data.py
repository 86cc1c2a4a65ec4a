"""Transition data with the reference's API (/root/reference/src/mbrl/data.py).

Rollout (data.py:8-120), TransitionsDatasetDataMode (:121-124), TransitionsDataset (:125-269) and
TransitionsSampler (:271-285) keep the reference's constructors, indexing, normalisation and
sampling order, so the model-training loop (models.train_model) sees the
same batches in the same order as the reference for the same NumPy seed.

Additions for the device path: `TransitionsDataset.from_statistics` (a stats-only dataset for
binding normalisers, as the planners need), `normalizers()` (the partials the agents build,
agents.py:219-221 / 336-340) and `stacked(device)` (every transition as a few device tensors, so a
training epoch gathers batches with one index_select instead of per-sample Python collation).
"""
import functools
from collections import defaultdict
from enum import Enum
from typing import List, Optional

import numpy as np
import torch
from torch.utils.data import Dataset, Sampler


class Rollout:
    """data.py:8-120: states s_0..s_K, observations o_0..o_K, actions a_0..a_{K-1}, rewards
    r_1..r_K; len = K transitions."""

    def __init__(self, states, observations, actions, rewards):
        assert len(states) > 0
        assert len(states) == len(observations)
        assert len(actions) == len(rewards)
        assert len(states) == len(actions) + 1
        self._length = len(rewards)
        self._states = states
        self._flat_obs = isinstance(observations[0], torch.Tensor)
        self._observations = observations
        self._actions = list(actions) + [None]
        self._rewards = [None] + list(rewards)

    states = property(lambda self: self._states)
    observations = property(lambda self: self._observations)
    actions = property(lambda self: self._actions)
    rewards = property(lambda self: self._rewards)
    flat_observations = property(lambda self: self._flat_obs)

    @property
    def sum_of_rewards(self):
        return sum(self.rewards[1:])

    def __len__(self):
        return self._length

    def __getitem__(self, key):
        return Rollout(states=self.states[key], observations=self.observations[key],
                       actions=self.actions[key][:-1], rewards=self.rewards[key][1:])

    @staticmethod
    def _norm(x, stats, name):
        return (x - stats[name]["mean"]) / stats[name]["std"]

    def _norm_obs(self, o, stats):
        if self.flat_observations:
            return self._norm(o, stats, "observations")
        return {k: (v - stats["observations"][k]["mean"]) / stats["observations"][k]["std"] for k, v in o.items()}

    def get_transition(self, idx, stats=None):
        """((s_i, o_i, a_i), (r_{i+1}, s_{i+1}, o_{i+1})), normalised with `stats` when given."""
        assert idx < len(self)
        s, o, a = self._states[idx], self._observations[idx], self._actions[idx]
        r, s1, o1 = self._rewards[idx + 1], self._states[idx + 1], self._observations[idx + 1]
        if stats is not None:
            s, o, a = self._norm(s, stats, "states"), self._norm_obs(o, stats), self._norm(a, stats, "actions")
            r, s1, o1 = self._norm(r, stats, "rewards"), self._norm(s1, stats, "states"), self._norm_obs(o1, stats)
        return (s, o, a), (r, s1, o1)

    def get_multistep_transitions(self, start_idx, horizon, stats=None):
        assert start_idx + horizon < len(self) + 1
        pairs = [self.get_transition(i, stats=stats) for i in range(start_idx, start_idx + horizon)]
        return tuple(p[0] for p in pairs), tuple(p[1] for p in pairs)


class TransitionsDatasetDataMode(Enum):
    state_only = "state_only"
    obs_only = "obs_only"
    both = "both"


class TransitionsDataset(Dataset):
    """data.py:125-269. Items are (inputs, outputs): per horizon step (s, o, a) / (r, s', o'),
    reduced by the data mode to (s, a) / (r, s') (state_only) or (o, a) / (r, o') (obs_only)."""

    def __init__(self, rollouts: Optional[List[Rollout]] = None, transitions_capacity: int = int(1e6),
                 horizon: int = 1, normalise=True, data_mode=TransitionsDatasetDataMode.both):
        super().__init__()
        self.capacity = transitions_capacity
        self.horizon = horizon
        self._rollouts = []
        self._occupied_capacity = 0
        self._flat_obs = None
        self._stats = {"state": None, "observation": None, "action": None, "reward": None}
        self._normalise = normalise
        self._data_mode = TransitionsDatasetDataMode(data_mode)
        self._stacked = None
        if rollouts is not None:
            self.add_rollouts(rollouts)

    @classmethod
    def from_statistics(cls, statistics):
        """A dataset holding only normalisation statistics ({"observations": {"mean", "std"}, ...})."""
        ds = cls()
        ds._stats = statistics
        return ds

    def set_data_mode(self, data_mode):
        self._data_mode = TransitionsDatasetDataMode(data_mode)
        self._stacked = None

    def add_rollouts(self, rollouts):
        if self._flat_obs is None:
            self._flat_obs = rollouts[0].flat_observations
        for roll in rollouts:
            assert roll.flat_observations == self._flat_obs
            self._occupied_capacity += max(len(roll) - self.horizon + 1, 0)
            self._rollouts.append(roll)
        over = self._occupied_capacity - self.capacity
        if over > 0:      # drop the oldest transitions (data.py:178-194)
            print("Exceeded max_capacity of {} transitions".format(self.capacity))
            print("Removing oldest {} transitions from dataset".format(over))
            while over > 0:
                oldest = len(self._rollouts[0])
                if oldest > over:
                    self._rollouts[0] = self._rollouts[0][over:]
                    self._occupied_capacity = self.capacity
                    break
                self._rollouts.pop(0)
                self._occupied_capacity -= oldest
                over = self._occupied_capacity - self.capacity
        self._update_stats()
        self._stacked = None

    occupied_capacity = property(lambda self: sum(len(r) - self.horizon + 1 for r in self._rollouts))
    num_rollouts = property(lambda self: len(self._rollouts))
    statistics = property(lambda self: self._stats)
    rollouts = property(lambda self: self._rollouts)

    def __len__(self):
        return self._occupied_capacity

    def __getitem__(self, trans):
        return self.get_transition(roll_idx=trans[0], start_idx=trans[1])

    def get_transition(self, roll_idx=None, start_idx=None):
        if roll_idx is None:
            roll_idx = np.random.randint(0, self.num_rollouts)
        rollout = self._rollouts[roll_idx]
        if start_idx is None:
            start_idx = np.random.randint(0, len(rollout) - self.horizon)
        inputs, outputs = rollout.get_multistep_transitions(start_idx, self.horizon,
                                                            stats=self._stats if self._normalise else None)
        return self._select(inputs, outputs)

    def _select(self, inputs, outputs):
        mode = self._data_mode
        if mode == TransitionsDatasetDataMode.state_only:
            return [inp[::2] for inp in inputs], [out[:-1] for out in outputs]
        if mode == TransitionsDatasetDataMode.obs_only:
            return [inp[1:] for inp in inputs], [out[::2] for out in outputs]
        return inputs, outputs

    def _update_stats(self):
        """data.py:229-253 (first action of the padding and first reward are excluded)."""
        st = self._stats
        states, actions, rewards = [], [], []
        obs = [] if self._flat_obs else defaultdict(list)
        for r in self._rollouts:
            states.append(torch.stack(r.states))
            actions.append(torch.stack(r.actions[:-1]))
            rewards.append(torch.stack(r.rewards[1:]))
            if self._flat_obs:
                obs.append(torch.stack(r.observations))
            else:
                for o in r.observations:
                    for k, v in o.items():
                        obs[k].append(v)
        st["states"] = self._get_stats(torch.cat(states))
        st["actions"] = self._get_stats(torch.cat(actions))
        st["rewards"] = self._get_stats(torch.cat(rewards))
        st["observations"] = (self._get_stats(torch.cat(obs)) if self._flat_obs
                              else {k: self._get_stats(torch.stack(v)) for k, v in obs.items()})

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
        return {"mean": torch.mean(array, dim=0), "std": torch.std(array, dim=0),
                "min": torch.min(array, dim=0).values, "max": torch.max(array, dim=0).values}

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

    # -------------------------------------------------------------------------------- device path
    def transition_index(self):
        """Every (roll_idx, start_idx) the sampler can draw, in the sampler's pre-shuffle order."""
        return [(ri, si) for ri, roll in enumerate(self._rollouts) for si in range(len(roll) - self.horizon)]

    def num_transitions(self):
        """len(transition_index()) without building the list."""
        return sum(max(0, len(roll) - self.horizon) for roll in self._rollouts)

    def stacked(self, device):
        """(index, inputs, outputs) with inputs/outputs tuples of [T, horizon, dim] tensors on `device`,
        T = len(transition_index()), field order as __getitem__ yields them (flat observations only)."""
        key = str(device)
        if self._stacked is not None and self._stacked[0] == key:
            return self._stacked[1:]
        if not self._flat_obs:
            raise ValueError("stacked() needs flat (tensor) observations")
        index = self.transition_index()
        items = [self[t] for t in index]
        n_in, n_out = len(items[0][0][0]), len(items[0][1][0])

        def field(part, j):
            return torch.stack([torch.stack([torch.as_tensor(step[j]).reshape(-1) for step in it[part]])
                                for it in items]).to(device=device, dtype=torch.float32)
        ins = tuple(field(0, j) for j in range(n_in))
        outs = tuple(field(1, j) for j in range(n_out))
        self._stacked = (key, index, ins, outs)
        return index, ins, outs


class TransitionsSampler(Sampler):
    """data.py:271-285: every (rollout, start) pair once per epoch, order by np.random.shuffle."""

    def __init__(self, data_source: TransitionsDataset):
        self.data_source = data_source

    def __iter__(self):
        possible = self.data_source.transition_index()
        np.random.shuffle(possible)
        yield from possible

    def __len__(self):
        return len(self.data_source.transition_index())
