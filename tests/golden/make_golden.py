"""Generate the golden parity fixtures by running the REFERENCE's own planner/model/cost code.

Run in the build container only (the GPU box has no /root/reference):

    python tests/golden/make_golden.py

What runs from the reference (imported read-only from /root/reference, no bytecode written):
  * planners.RandomShootingPlanner.plan / _generate_trajectories  (src/mbrl/planners.py:140-216)
  * models.Model (L = 2) and models.DynamicsModel.forward          (src/mbrl/models.py:8-29, 96-110)
    -- for L = 3 a DynamicsModel subclass whose _forward follows Model._forward's pattern
  * models.SmoothAbsLoss / models.CoshLoss                          (src/mbrl/models.py:244-272)
  * data.TransitionsDataset.normalize_field / unnormalize_field     (src/mbrl/data.py:255-260)
  * models.ModelWithReward (config 6)                                (src/mbrl/models.py:125-163)
Wired exactly as GoalStateAgent does (src/mbrl/agents.py:219-233), or, for config 6, as RewardAgent
does (agents.py:336-362; compose, agents.py:300-304, restated). Two small pieces that live in
modules that cannot import here (dm_control / tensorboardX missing) are restated verbatim in
behaviour: state_action_cost (agents.py:182-183) and EnvWrapper._sample_action
(env_wrappers.py:50-62).

CEM is not in the reference: per iteration the reference's
_generate_trajectories does rollout + cost on the oracle's Philox actions, and the oracle's NumPy
refit (oracle/cem.py) closes the iteration -- the SURVEY.md §8c oracle construction.

Outputs: tests/golden/*.npz (inputs regenerate from seeds; weights are pinned by SHA-256).
"""
import functools
import os
import sys

import numpy as np

sys.dont_write_bytecode = True            # never write into the read-only reference tree
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from oracle import cem as ocem  # noqa: E402
from oracle.philox import cem_actions  # noqa: E402


def _import_reference():
    sys.path.insert(0, REF)
    from src.mbrl import data, models, planners  # noqa: F401
    return data, models, planners


def state_action_cost(state, action, state_cost, action_cost):
    # agents.py:182-183 (agents.py itself does not import here: tensorboardX / dm_control absent)
    return state_cost(state) + action_cost(action)


class _Spec:
    def __init__(self, a, lo=-1.0, hi=1.0):
        self.shape = (a,)
        self.minimum = np.full(a, lo)
        self.maximum = np.full(a, hi)


def sample_action_ref(action_spec, batch_size=None):
    # env_wrappers.py:50-62, behaviour restated (module needs dm_control)
    minimum = max(action_spec.minimum[0], -3)
    maximum = min(action_spec.maximum[0], 3)
    if batch_size is None:
        action = np.random.uniform(minimum, maximum, action_spec.shape[0])
    else:
        action = np.random.uniform(minimum, maximum, size=action_spec.shape[0] * batch_size).reshape(
            (batch_size, -1))
    return torch.tensor(action, dtype=torch.float32)


def build_reference_model(models, layers, s, a, W):
    L = len(layers) - 1
    if L == 2:
        m = models.Model(s, a, hidden_units=W)
        lin = [m.linear1, m.linear2, m.linear3]
    else:
        class ModelL(models.DynamicsModel):
            # models.Model._forward's Linear/ReLU pattern with L hidden layers
            def __init__(self):
                super().__init__()
                dims = [s + a] + [W] * L + [s]
                self.lins = torch.nn.ModuleList(
                    [torch.nn.Linear(i, o) for i, o in zip(dims[:-1], dims[1:])])
                self.activation_fn = torch.nn.ReLU()

            def _forward(self, x):
                for lin in self.lins[:-1]:
                    x = self.activation_fn(lin(x))
                return self.lins[-1](x)
        m = ModelL()
        lin = list(m.lins)
    with torch.no_grad():
        for l, (w, b) in zip(lin, layers):
            l.weight.copy_(torch.from_numpy(w))
            l.bias.copy_(torch.from_numpy(b))
    return m


def compose(a, b):
    # agents.py:300-304 (agents.py does not import here)
    def ab(*args, **kwargs):
        return b(a(*args, **kwargs))
    return ab


def wire_reward(data, models, problem, layers):
    """RewardAgent's model / cost closures (agents.py:336-362) around the reference ModelWithReward."""
    import operator
    cfg = problem["cfg"]
    norm = problem["norm"]
    s, a, W = cfg["s"], cfg["a"], cfg["W"]
    assert cfg["L"] == 2, "the reference ModelWithReward has a 2-layer trunk"
    stats = {"observations": {"mean": torch.from_numpy(norm["obs_mean"]), "std": torch.from_numpy(norm["obs_std"])},
             "actions": {"mean": torch.from_numpy(norm["act_mean"]), "std": torch.from_numpy(norm["act_std"])},
             "rewards": {"mean": torch.from_numpy(norm["rew_mean"]), "std": torch.from_numpy(norm["rew_std"])}}
    TD = data.TransitionsDataset
    m = models.ModelWithReward(s, a, hidden_units=W)
    head_w, head_b = layers[-1]
    with torch.no_grad():
        for lin, (w, b) in zip([m.linear1, m.linear2, m.linear3, m.linear4],
                               list(layers[:-1]) + [(head_w[:s], head_b[:s]), (head_w[s:], head_b[s:])]):
            lin.weight.copy_(torch.from_numpy(np.ascontiguousarray(w)))
            lin.bias.copy_(torch.from_numpy(np.ascontiguousarray(b)))
    kw = dict(normalize_state=functools.partial(TD.normalize_field, field_name="observations", stats=stats),
              normalize_action=functools.partial(TD.normalize_field, field_name="actions", stats=stats),
              unnormalize_state=functools.partial(TD.unnormalize_field, field_name="observations", stats=stats),
              unnormalize_reward=functools.partial(TD.unnormalize_field, field_name="rewards", stats=stats))
    return compose(functools.partial(m, **kw), operator.itemgetter(0)), \
        compose(functools.partial(m, **kw), operator.itemgetter(1))


def wire(data, models, problem, layers):
    cfg = problem["cfg"]
    if cfg.get("reward"):
        return wire_reward(data, models, problem, layers)
    norm = problem["norm"]
    stats = {"observations": {"mean": torch.from_numpy(norm["obs_mean"]),
                              "std": torch.from_numpy(norm["obs_std"])},
             "actions": {"mean": torch.from_numpy(norm["act_mean"]),
                         "std": torch.from_numpy(norm["act_std"])}}
    TD = data.TransitionsDataset
    model = build_reference_model(models, layers, cfg["s"], cfg["a"], cfg["W"])
    # agents.py:219-230
    model_fn = functools.partial(
        model,
        normalize_state=functools.partial(TD.normalize_field, field_name="observations", stats=stats),
        normalize_action=functools.partial(TD.normalize_field, field_name="actions", stats=stats),
        unnormalize_state=functools.partial(TD.unnormalize_field, field_name="observations", stats=stats),
    )
    c = problem["cost"]
    cost_fn = functools.partial(
        state_action_cost,
        state_cost=models.SmoothAbsLoss(weights=torch.from_numpy(c["weights"]),
                                        goal_state=torch.from_numpy(c["goal"]), alpha=c["alpha_state"]),
        action_cost=models.CoshLoss(alpha=c["alpha_action"]))
    return model_fn, cost_fn


def ref_rollout_costs(planners, model_fns, cost_fns, s0, A):
    """Reference _generate_trajectories per ensemble member on fixed time-major actions A [H,N,a]."""
    H, N, a = A.shape
    flat = torch.from_numpy(np.ascontiguousarray(A.reshape(H * N, a)))

    def sample_action(batch_size):
        assert batch_size == H * N
        return flat.clone()

    costs, trajs = [], []
    for mf, cf in zip(model_fns, cost_fns):
        tr, c = planners.RandomShootingPlanner._generate_trajectories(
            initial_state=torch.from_numpy(s0), model=mf, cost=cf, sample_action=sample_action,
            horizon=H, num_trajectories=N)
        costs.append(np.asarray(c, dtype=np.float32))
        trajs.append(tr)
    return np.stack(costs), trajs


def make_rs(data, models, planners, out_dir):
    """Config 1: the reference's RandomShootingPlanner.plan end to end (numpy global RNG)."""
    p = ocem.synth_problem(1)
    cfg = p["cfg"]
    model_fn, cost_fn = wire(data, models, p, p["model"][0])
    spec = _Spec(cfg["a"])
    sample_action = functools.partial(sample_action_ref, action_spec=spec)
    np_seed = 12345
    np.random.seed(np_seed)
    states, actions = planners.RandomShootingPlanner.plan(
        torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, cfg["H"], None,
        num_trajectories=cfg["N"])
    # same draw again to record the inputs and every candidate's return
    np.random.seed(np_seed)
    flat = sample_action(batch_size=cfg["N"] * cfg["H"]).numpy()
    costs, _ = ref_rollout_costs(planners, [model_fn], [cost_fn], p["s0"],
                                 flat.reshape(cfg["H"], cfg["N"], cfg["a"]))
    np.savez_compressed(
        os.path.join(out_dir, "config1_rs.npz"), np_seed=np_seed, weights_sha256=ocem.weights_sha256(p["model"]),
        actions_flat=flat, costs=costs[0], idx=np.int64(np.argmin(costs[0])),
        plan_states=states.detach().numpy(), plan_actions=actions.detach().numpy())
    print("config1: idx", int(np.argmin(costs[0])), "cost", float(costs[0].min()))


def make_cem(data, models, planners, out_dir, config_id, full=False, **over):
    """One CEM plan (I iterations) with the reference's _generate_trajectories as rollout + cost.

    full=True is the BASELINE full-size mode (walker N=16384 H=30; humanoid N=32768 H=50 E=5). It
    runs the reference rollout under torch.no_grad(): the reference builds an autograd graph it never
    uses (planners.py:199-210 without no_grad), which at humanoid size would hold ~10 GB of saved
    activations per member; the forward arithmetic is the same with or without the graph. The
    fixture then keeps the member-mean returns (not the per-member costs) to stay small."""
    p = ocem.synth_problem(config_id, **over)
    cfg = p["cfg"]
    N, H, a = cfg["N"], cfg["H"], cfg["a"]
    K = max(1, int(N * ocem.CEM_DEFAULTS["elite_frac"]))
    I = ocem.CEM_DEFAULTS["num_iterations"]
    alpha, lo, hi = ocem.CEM_DEFAULTS["alpha"], ocem.CEM_DEFAULTS["lo"], ocem.CEM_DEFAULTS["hi"]
    wired = [wire(data, models, p, layers) for layers in p["model"]]
    model_fns = [w[0] for w in wired]
    cost_fns = [w[1] for w in wired]
    mu = np.zeros((H, a), np.float32)
    sigma = np.full((H, a), np.float32((hi - lo) / 4.0), np.float32)
    rec = dict(costs=[], returns=[], elites=[], mu=[], sigma=[], gap=[])
    grad_ctx = torch.no_grad if full else torch.enable_grad
    for it in range(I):
        A = cem_actions(mu, sigma, lo, hi, p["rng_seed"], it, np.arange(N))
        with grad_ctx():
            costs, _ = ref_rollout_costs(planners, model_fns, cost_fns, p["s0"], A)
        ret = ocem.ensemble_returns(costs)
        order = np.argsort(ret, kind="stable")
        elites = np.sort(order[:K])
        gap = (ret[order[K]] - ret[order[K - 1]]) / max(abs(float(ret[order[K - 1]])), 1.0) if K < N else 1.0
        mu, sigma = ocem.refit(mu, sigma, np.ascontiguousarray(A[:, elites, :].transpose(1, 0, 2)), alpha)
        for k, v in zip(("costs", "returns", "elites", "mu", "sigma", "gap"),
                        (costs, ret, elites, mu, sigma, gap)):
            rec[k].append(v)
    final_actions = np.clip(mu, np.float32(lo), np.float32(hi)).astype(np.float32)
    st = []
    for mf, cf in zip(model_fns, cost_fns):
        with grad_ctx():
            _, tr = ref_rollout_costs(planners, [mf], [cf], p["s0"], final_actions[:, None, :])
        st.append(tr[0][0][0].detach().numpy())
    final_states = np.mean(np.stack(st), axis=0, dtype=np.float32) if len(st) > 1 else st[0]
    name = f"config{config_id}_cem" + ("" if not over else "_" + "_".join(f"{k}{v}" for k, v in over.items()))
    if full:
        name += "_full"
    extra = {} if full else dict(costs=np.stack(rec["costs"]))
    np.savez_compressed(
        os.path.join(out_dir, name + ".npz"), weights_sha256=ocem.weights_sha256(p["model"]),
        N=N, H=H, K=K, I=I, alpha=alpha, lo=lo, hi=hi, gap=np.array(rec["gap"], np.float64), **extra,
        returns=np.stack(rec["returns"]),
        elites=np.stack(rec["elites"]).astype(np.int32), mu=np.stack(rec["mu"]),
        sigma=np.stack(rec["sigma"]), final_actions=final_actions, final_states=final_states)
    print(name, "min K-boundary gap (rel)", float(np.min(rec["gap"])),
          "returns[0][:3]", rec["returns"][0][:3])


def make_toy(planners, out_dir):
    """Known answer from test_random_shooting.py:5-25 (1-D ring world, integer costs)."""
    world_size = 10
    goal = torch.tensor(9, dtype=torch.float)

    def model(states, actions):
        next_states = states + actions
        return torch.fmod((torch.fmod(next_states, world_size) + world_size), world_size)

    def sample_action(batch_size):
        return torch.randint(low=-1, high=2, size=(batch_size, 1), dtype=torch.float)

    def cost(states, actions):
        return torch.abs(states - goal)

    torch.manual_seed(0)
    flat = sample_action(1000 * 5).numpy()
    torch.manual_seed(0)
    states, actions = planners.RandomShootingPlanner.plan(
        torch.tensor([2], dtype=torch.float), model, cost, sample_action, 5, None, num_trajectories=1000)
    states = states.numpy()
    total = float(np.abs(states - 9).sum())
    np.savez_compressed(os.path.join(out_dir, "toy_ring_rs.npz"), actions_flat=flat,
                        plan_states=states, plan_actions=actions.numpy(), plan_cost=total)
    print("toy ring: states", states.ravel(), "cost", total)


def main():
    out_dir = HERE
    data, models, planners = _import_reference()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    if len(sys.argv) > 1 and sys.argv[1] == "6":           # regenerate only the reward-head fixture
        make_cem(data, models, planners, out_dir, 6, N=512, H=10)
        return
    if len(sys.argv) > 1 and sys.argv[1] == "full":        # BASELINE configs 4 and 5 at full size
        for cid in sys.argv[2:] or ("4", "5"):
            make_cem(data, models, planners, out_dir, int(cid), full=True)
        return
    make_toy(planners, out_dir)
    make_rs(data, models, planners, out_dir)
    make_cem(data, models, planners, out_dir, 2)
    make_cem(data, models, planners, out_dir, 3)
    make_cem(data, models, planners, out_dir, 4, N=2048)
    make_cem(data, models, planners, out_dir, 5, N=256, H=20)
    make_cem(data, models, planners, out_dir, 6, N=512, H=10)


if __name__ == "__main__":
    main()
