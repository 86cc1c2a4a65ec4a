"""Synthetic random-weight dynamics problems at BASELINE.json's named shapes.

There are no checkpoints or datasets offline, so the bench and the smoke test plan on random
weights drawn with nn.Linear's init law (U(-1/sqrt(fan_in), 1/sqrt(fan_in))) from NumPy PCG64,
seed = 1000 + config id; normalisation mean ~ U(-0.5, 0.5), std ~ U(0.5, 2) (seed + 1);
s0, goal ~ N(0, 1) (seed + 2); CEM proposal seed = seed + 3. The CPU oracle draws the identical
arrays independently (oracle/cem.py:synth_problem; tests/test_host.py checks the two agree).
"""
import functools
import operator

import numpy as np
import torch

from . import data, env, models

# id: (name, obs dim, action dim, hidden width, hidden layers, candidates, horizon, ensemble)
CONFIGS = {
    1: dict(name="cartpole-swingup-rs", s=5, a=1, W=256, L=2, N=128, H=12, E=1),
    2: dict(name="cartpole-swingup-cem", s=5, a=1, W=256, L=2, N=1024, H=20, E=1),
    3: dict(name="cheetah-run-cem", s=17, a=6, W=512, L=3, N=4096, H=30, E=1),
    4: dict(name="walker-walk-cem", s=24, a=6, W=512, L=3, N=16384, H=30, E=1),
    5: dict(name="humanoid-stand-cem-ens5", s=67, a=21, W=512, L=3, N=32768, H=50, E=5),
    # reward-head variant: ModelWithReward 2x512 trunk, RewardAgent cost
    6: dict(name="cheetah-run-reward-cem", s=17, a=6, W=512, L=2, N=4096, H=30, E=1, reward=True),
}


def flop_per_candidate_step(cfg):
    """Algorithmic MLP FLOP per candidate per step, times the ensemble size.
    Reward-head models run the trunk twice per step (the model call, then the reward cost call on
    (s_{t+1}, a_t): planners.py:207,210 with RewardAgent's closures), each pass with its own head."""
    s, a, W, L, E = cfg["s"], cfg["a"], cfg["W"], cfg["L"], cfg["E"]
    trunk = W * (s + a) + (L - 1) * W * W
    if cfg.get("reward"):
        return 2 * (2 * trunk + W * s + W) * E
    return 2 * (trunk + W * s) * E


def split_stream_bytes_per_step(cfg, pieces):
    """Weight bytes one split-rollout workgroup streams from L2 per step (csrc/mbrl_internal.h
    make_geometry): CS chunks of 32 K rows, 8 waves x T/2 tiles x `pieces` fragments of 1 KiB."""
    s, a, W, L = cfg["s"], cfg["a"], cfg["W"], cfg["L"]
    T = 1
    while 64 * T < W:
        T *= 2
    k0s = (s + a + 31) // 32
    nout = -(-(s + int(bool(cfg.get("reward")))) // 16)
    nout += nout & 1
    nos = nout // 2
    if (k0s + nos) & 1:
        k0s += 1
    cs = k0s + (L - 1) * 2 * T + nos
    return cs * 8 * (T // 2) * pieces * 1024


def make_problem(config_id, **overrides):
    cfg = dict(CONFIGS[config_id])
    cfg.update(overrides)
    seed = 1000 + config_id
    s, a, W, L, E = cfg["s"], cfg["a"], cfg["W"], cfg["L"], cfg["E"]
    rng = np.random.Generator(np.random.PCG64(seed))
    reward = bool(cfg.get("reward"))

    def draw(lin, fi, fo):
        bound = 1.0 / np.sqrt(fi)
        with torch.no_grad():
            lin.weight.copy_(torch.from_numpy(rng.uniform(-bound, bound, size=(fo, fi)).astype(np.float32)))
            lin.bias.copy_(torch.from_numpy(rng.uniform(-bound, bound, size=(fo,)).astype(np.float32)))

    members = []
    for _ in range(E):
        if reward:   # trunk, state head, reward head (oracle/cem.py:synth_reward_model order)
            m = models.ModelWithReward(s, a, hidden_units=W, n_hidden=L)
            dims = [s + a] + [W] * L
            shapes = list(zip(dims[:-1], dims[1:])) + [(W, s), (W, 1)]
        else:
            m = models.Model(s, a, hidden_units=W, n_hidden=L)
            dims = [s + a] + [W] * L + [s]
            shapes = list(zip(dims[:-1], dims[1:]))
        for lin, (fi, fo) in zip(m.linears(), shapes):
            draw(lin, fi, fo)
        members.append(m)
    if reward and E > 1:
        raise ValueError("reward-head ensembles are not a BASELINE configuration")
    module = members[0] if E == 1 else models.EnsembleModel(members)
    rn = np.random.Generator(np.random.PCG64(seed + 1))
    stats = {"observations": {"mean": torch.from_numpy(rn.uniform(-0.5, 0.5, size=s).astype(np.float32)),
                              "std": torch.from_numpy(rn.uniform(0.5, 2.0, size=s).astype(np.float32))},
             "actions": {"mean": torch.from_numpy(rn.uniform(-0.5, 0.5, size=a).astype(np.float32)),
                         "std": torch.from_numpy(rn.uniform(0.5, 2.0, size=a).astype(np.float32))}}
    rs = np.random.Generator(np.random.PCG64(seed + 2))
    s0 = torch.from_numpy(rs.standard_normal(s).astype(np.float32))
    goal = torch.from_numpy(rs.standard_normal(s).astype(np.float32))
    if reward:
        rr = np.random.Generator(np.random.PCG64(seed + 4))
        stats["rewards"] = {"mean": torch.from_numpy(rr.uniform(-0.5, 0.5, size=1).astype(np.float32)),
                            "std": torch.from_numpy(rr.uniform(0.5, 2.0, size=1).astype(np.float32))}
    ds = data.TransitionsDataset.from_statistics(stats)
    if reward:                                                                         # agents.py:342-362
        model_fn = models.compose(functools.partial(module, **ds.normalizers(reward=True)), operator.itemgetter(0))
        cost_fn = models.compose(functools.partial(module, **ds.normalizers(reward=True)), operator.itemgetter(1))
    else:
        model_fn = functools.partial(module, **ds.normalizers())                       # agents.py:224-230
        cost_fn = models.goal_state_cost(models.SmoothAbsLoss(torch.ones(s), goal, 0.4), models.CoshLoss(0.25))
    sample_action = env.sample_action_fn(env.BoundedActionSpec(a, -1.0, 1.0))          # agents.py:233
    return dict(cfg=cfg, module=module, model=model_fn, cost=cost_fn, sample_action=sample_action, s0=s0,
                goal=goal, stats=stats, rng_seed=seed + 3)
