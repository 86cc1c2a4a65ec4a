"""CPU: host-side logic -- synthetic inputs, closure recognition, model semantics, sharding layout."""
import functools

import numpy as np
import pytest
import torch

from oracle import cem as ocem


def test_synthetic_matches_oracle_generator():
    from mbrl_amd import synthetic
    for cid, over in [(1, {}), (3, {}), (5, dict(N=64, H=4))]:
        prob = synthetic.make_problem(cid, **over)
        p = ocem.synth_problem(cid, **over)
        members = prob["module"].members if prob["cfg"]["E"] > 1 else [prob["module"]]
        model = [[(l.weight.detach().numpy(), l.bias.detach().numpy()) for l in m.linears()] for m in members]
        assert ocem.weights_sha256(model) == ocem.weights_sha256(p["model"])
        assert np.array_equal(prob["s0"].numpy(), p["s0"])
        assert np.array_equal(prob["goal"].numpy(), p["cost"]["goal"])
        assert np.array_equal(prob["stats"]["actions"]["std"].numpy(), p["norm"]["act_std"])
        assert prob["rng_seed"] == p["rng_seed"]


def test_flop_per_candidate_step_matches_survey():
    from mbrl_amd import synthetic
    assert synthetic.flop_per_candidate_step(synthetic.CONFIGS[2]) == 136_704
    assert synthetic.flop_per_candidate_step(synthetic.CONFIGS[3]) == 1_089_536
    assert synthetic.flop_per_candidate_step(synthetic.CONFIGS[4]) == 1_103_872
    assert synthetic.flop_per_candidate_step(synthetic.CONFIGS[5]) == 5 * 1_207_296


def test_closure_recognition():
    from mbrl_amd import fused, synthetic
    prob = synthetic.make_problem(3)
    md = fused.describe_model(prob["model"])
    assert md is not None and (md["s"], md["a"], md["W"], md["L"], md["E"]) == (17, 6, 512, 3, 1)
    assert md["norm"]["normalize_state"] and md["norm"]["unnormalize_state"] and md["norm"]["normalize_action"]
    cd = fused.describe_cost(prob["cost"], 17)
    assert cd is not None and cd["alpha_state"] == 0.4 and cd["alpha_action"] == 0.25
    assert fused.describe_sampler(prob["sample_action"]) == (-1.0, 1.0, 6)
    # anything opaque -> generic path
    assert fused.describe_model(lambda s, a: s) is None
    assert fused.describe_cost(lambda s, a: s, 17) is None
    # a noisy model is not deterministic -> generic path
    from mbrl_amd import models
    noisy = models.Model(3, 1, 8, noise=0.1)
    assert fused.describe_model(noisy) is None
    ens = synthetic.make_problem(5, N=8, H=2)
    assert fused.describe_model(ens["model"])["E"] == 5


def test_reference_style_model_duck_typed():
    """The reference's models.Model (linear1..3, ReLU, noise=None) is recognised by duck typing."""
    from mbrl_amd import fused

    class Model(torch.nn.Module):  # same attribute layout as /root/reference/src/mbrl/models.py:96-110
        def __init__(self):
            super().__init__()
            self.linear1 = torch.nn.Linear(7, 50)
            self.linear2 = torch.nn.Linear(50, 50)
            self.linear3 = torch.nn.Linear(50, 5)
            self.activation_fn = torch.nn.ReLU()
            self.noise = None
    md = fused.describe_model(Model())
    assert (md["s"], md["a"], md["W"], md["L"]) == (5, 2, 50, 2)


def test_model_cpu_forward_is_reference_arithmetic():
    from mbrl_amd import synthetic
    prob = synthetic.make_problem(4, N=8)
    p = ocem.synth_problem(4, N=8)
    rng = np.random.default_rng(2)
    s = rng.standard_normal((64, 24)).astype(np.float32)
    a = rng.uniform(-1, 1, (64, 6)).astype(np.float32)
    with torch.no_grad():
        out = prob["model"](torch.from_numpy(s), torch.from_numpy(a)).numpy()
    assert np.allclose(out, ocem.dynamics_step(p["model"][0], p["norm"], s, a), rtol=1e-5, atol=1e-5)
    c = prob["cost"](torch.from_numpy(s), torch.from_numpy(a)).numpy()
    assert np.allclose(c, ocem.goal_state_cost(s, a, p["cost"]), rtol=1e-6)


def test_sample_action_reference_semantics():
    from mbrl_amd import env
    spec = env.BoundedActionSpec(3, -5.0, 0.5)
    np.random.seed(4)
    x = env._sample_action(spec, batch_size=7)
    np.random.seed(4)
    ref = np.random.uniform(-3, 0.5, size=21).reshape(7, 3)
    assert x.dtype == torch.float32 and x.shape == (7, 3)
    assert np.array_equal(x.numpy(), ref.astype(np.float32))


def test_model_state_dict_compatible_with_reference_layout():
    from mbrl_amd import models
    m = models.Model(5, 1, hidden_units=256)
    assert sorted(m.state_dict()) == sorted(
        [f"linear{i}.{p}" for i in (1, 2, 3) for p in ("weight", "bias")])
    assert isinstance(functools.partial(m), functools.partial)


def _reward_layers_combined(m):
    lay = [(l.weight.detach().numpy(), l.bias.detach().numpy()) for l in m.linears()]
    (ws, bs), (wr, br) = lay[-2], lay[-1]
    return lay[:-2] + [(np.vstack([ws, wr]), np.concatenate([bs, br]))]


def test_reward_problem_matches_oracle_and_reference_semantics():
    """Config 6: synthetic ModelWithReward == oracle draw; the RewardAgent
    closures (compose + itemgetter, agents.py:342-362) compute the oracle's next state and reward."""
    from mbrl_amd import synthetic
    prob = synthetic.make_problem(6, N=16, H=3)
    p = ocem.synth_problem(6, N=16, H=3)
    assert ocem.weights_sha256([_reward_layers_combined(prob["module"])]) == ocem.weights_sha256(p["model"])
    assert np.array_equal(prob["stats"]["rewards"]["mean"].numpy(), p["norm"]["rew_mean"])
    rng = np.random.default_rng(6)
    s = rng.standard_normal((32, 17)).astype(np.float32)
    a = rng.uniform(-1, 1, (32, 6)).astype(np.float32)
    with torch.no_grad():
        ns = prob["model"](torch.from_numpy(s), torch.from_numpy(a))
        r = prob["cost"](ns, torch.from_numpy(a))
    ref_ns = ocem.dynamics_step(p["model"][0], p["norm"], s, a)
    assert np.allclose(ns.numpy(), ref_ns, rtol=1e-5, atol=1e-5)
    assert r.shape == (32, 1)
    assert np.allclose(r.numpy()[:, 0], ocem.reward_cost(p["model"][0], p["norm"], ref_ns, a), rtol=1e-5, atol=1e-5)


def test_reward_closure_recognition():
    import operator
    from mbrl_amd import _lib, fused, models, synthetic
    prob = synthetic.make_problem(6, N=16, H=3)
    md = fused.describe_model(prob["model"])
    assert md is not None and md["reward"] and (md["s"], md["a"], md["W"], md["L"]) == (17, 6, 512, 2)
    assert md["norm"]["unnormalize_reward"] and md["norm"]["rew_std"].numel() == 1
    assert fused.mlp_shape(md).reward_head == 1
    cd = fused.describe_cost(prob["cost"], 17, md)
    assert cd is not None and cd["kind"] == _lib.MBRL_COST_MODEL_REWARD
    # the reward cost needs the model description of the same module
    assert fused.describe_cost(prob["cost"], 17) is None
    other = synthetic.make_problem(6, N=16, H=3)
    assert fused.describe_cost(other["cost"], 17, md) is None
    # itemgetter(1) as the model, or a goal-state model with a reward cost -> generic path
    f = prob["cost"].__closure__
    swapped = models.compose(functools.partial(prob["module"]), operator.itemgetter(1))
    assert fused.describe_model(swapped) is None
    assert f is not None
    plain = synthetic.make_problem(3, N=8, H=2)
    assert fused.describe_cost(prob["cost"], 17, fused.describe_model(plain["model"])) is None


def test_reference_style_reward_model_duck_typed():
    """The reference's ModelWithReward (linear1..4, models.py:125-141) is recognised by duck typing."""
    import operator
    from mbrl_amd import fused, models

    class ModelWithReward(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.linear1 = torch.nn.Linear(9, 40)
            self.linear2 = torch.nn.Linear(40, 40)
            self.linear3 = torch.nn.Linear(40, 6)
            self.linear4 = torch.nn.Linear(40, 1)
            self.activation_fn = torch.nn.ReLU()
    md = fused.describe_model(models.compose(functools.partial(ModelWithReward()), operator.itemgetter(0)))
    assert md is not None and md["reward"] and (md["s"], md["a"], md["W"], md["L"]) == (6, 3, 40, 2)


def test_mpc_policy_host_logic():
    """agents.py:37-56: reset at timestep 0, (states[1:], actions[0:]) as initial_trajectory, act with
    actions[0]; kwargs are forwarded to the planner."""
    from mbrl_amd import MPCPolicy
    calls = []

    class FakePlanner:
        @staticmethod
        def plan(initial_state, model, cost, sample_action, horizon, initial_trajectory=None, **kw):
            calls.append((initial_trajectory, kw))
            k = len(calls)
            return torch.full((horizon, 2), float(k)), torch.full((horizon, 1), 10.0 * k)

    pol = MPCPolicy(None, None, FakePlanner, None, 4, num_candidates=64)
    a = pol.get_action({"timestep": 0, "observation": torch.zeros(2)})
    assert a.tolist() == [10.0] and calls[0][0] is None and calls[0][1] == {"num_candidates": 64}
    pol.get_action({"timestep": 1, "observation": torch.zeros(2)})
    it = calls[1][0]
    assert it[0].shape == (3, 2) and it[1].shape == (4, 1) and float(it[1][0, 0]) == 10.0
    pol.get_action({"timestep": 0, "observation": torch.zeros(2)})
    assert calls[2][0] is None


def test_policy_and_closures_pickle_like_the_reference_agent():
    """agents.save pickles the whole agent, planner and model included (agents.py:22-27), and
    parallel.py pickles policies into workers: the planner class, the model closures (partials
    over normalize_field) and the cost closure must round-trip, with no device handles in them."""
    import pickle

    from mbrl_amd import CEMPlanner, MPCPolicy, fused, synthetic
    prob = synthetic.make_problem(3, N=64, H=4)
    pol = MPCPolicy(prob["model"], prob["cost"], CEMPlanner, prob["sample_action"], 4, num_candidates=64, seed=3)
    back = pickle.loads(pickle.dumps(pol))
    assert back.planner is CEMPlanner and back.plan_kwargs == pol.plan_kwargs
    md0, md1 = fused.describe_model(pol.model), fused.describe_model(back.model)
    assert md1 is not None and (md0["s"], md0["a"], md0["W"], md0["L"]) == (md1["s"], md1["a"], md1["W"], md1["L"])
    for l0, l1 in zip(md0["members"][0], md1["members"][0]):
        assert torch.equal(l0.weight, l1.weight) and torch.equal(l0.bias, l1.bias)
    assert fused.describe_cost(back.cost, md1["s"], md1) is not None
    s = torch.randn(5, 17)
    a = torch.rand(5, 6) * 2 - 1
    assert torch.equal(pol.model(s, a), back.model(s, a))


def test_random_shooting_on_a_gpu_less_host_matches_reference_golden(golden):
    """BASELINE configs[0] (the reference's random-shooting planner on CPU) through the public API on
    a host without a GPU: the reference's a2 loop on the closures, np.argmin -- the chosen candidate,
    its actions bit-exact and its states / every candidate's cost as the reference computed them
    (tests/golden/config1_rs.npz, generated by the reference's own planners.py)."""
    import numpy as np
    import torch
    from mbrl_amd import RandomShootingPlanner, planners
    from oracle import cem as ocem
    from test_gpu_parity import build
    if torch.cuda.is_available():
        pytest.skip("the GPU path runs when a GPU is present (tests/test_gpu_parity.py)")
    g = golden("config1_rs")
    p = ocem.synth_problem(1)
    _, model_fn, cost_fn, sample_action = build(p)
    np.random.seed(int(g["np_seed"]))
    states, actions = RandomShootingPlanner.plan(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action,
                                                 p["cfg"]["H"], None, num_trajectories=p["cfg"]["N"])
    assert np.array_equal(actions.numpy(), g["plan_actions"])
    assert np.allclose(states.numpy(), g["plan_states"], rtol=1e-5, atol=1e-5)
    # the costs of every candidate, through the same loop
    N, H = p["cfg"]["N"], p["cfg"]["H"]
    flat = torch.from_numpy(g["actions_flat"])
    it = iter([flat])
    st, ac = planners._rs_host(torch.from_numpy(p["s0"]), model_fn, cost_fn, lambda batch_size: next(it), H, N)
    assert torch.equal(ac, flat.view(H, N, -1)[:, int(g["idx"])])


def test_random_shooting_on_a_gpu_less_host_toy_known_answer():
    """The reference's own known answer (src/mbrl/test_random_shooting.py:5-25: ring world, seed 0 ->
    cost 18, states [1, 0, 9, 9, 8]) on the host path."""
    import torch
    from mbrl_amd import RandomShootingPlanner
    if torch.cuda.is_available():
        pytest.skip("the GPU path runs when a GPU is present (tests/test_gpu_parity.py)")
    world_size, goal = 10, torch.tensor(9, dtype=torch.float)

    def model(states, actions):
        return torch.fmod((torch.fmod(states + actions, world_size) + world_size), world_size)

    def sample_action(batch_size):
        return torch.randint(low=-1, high=2, size=(batch_size, 1), dtype=torch.float)

    def cost(states, actions):
        return torch.abs(states - goal)

    torch.manual_seed(0)
    states, actions = RandomShootingPlanner.plan(torch.tensor([2], dtype=torch.float), model, cost, sample_action, 5,
                                                 None, num_trajectories=1000)
    assert states.numpy().ravel().tolist() == [1.0, 0.0, 9.0, 9.0, 8.0]
    assert float(torch.abs(states - 9).sum()) == 18.0


def test_cem_planner_on_a_gpu_less_host_raises():
    """Only the random-shooting planner (configs[0]) has a host path: CEM needs the HIP extension."""
    import torch
    from mbrl_amd import CEMPlanner
    from oracle import cem as ocem
    from test_gpu_parity import build
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = ocem.synth_problem(2, N=64, H=4)
    _, model_fn, cost_fn, sample_action = build(p)
    with pytest.raises(RuntimeError, match="GPU"):
        CEMPlanner.plan(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 4, num_candidates=64)


def test_cem_settings_cache_semantics():
    """CEMPlanner._settings builds the settings once per (sampler, horizon, kwargs) when the seed is
    explicit: equal kwargs give the same dict, any changed value a new one, the per-plan timing hooks
    are set on a copy, unhashable values and seed=None are never cached (seed=None draws from the
    global NumPy RNG on every call, as the reference's sampler does)."""
    from mbrl_amd import synthetic
    from mbrl_amd.planners import CEMPlanner
    p = synthetic.make_problem(3, N=64, H=4)
    sa = p["sample_action"]
    kw = dict(num_candidates=64, num_iterations=2, seed=5)
    a, b = CEMPlanner._settings(sa, 4, dict(kw)), CEMPlanner._settings(sa, 4, dict(kw))
    assert a is b and a["N"] == 64 and a["seed"] == 5
    c = CEMPlanner._settings(sa, 4, dict(kw, num_candidates=128))
    assert c is not a and c["N"] == 128 and a["N"] == 64
    assert CEMPlanner._settings(sa, 5, dict(kw))["H"] == 5
    hooks = [None, None]
    d = CEMPlanner._settings(sa, 4, dict(kw, rollout_events=hooks))
    assert d["events"] is hooks and a["events"] is None and d["N"] == 64
    e = CEMPlanner._settings(sa, 4, dict(kw, action_bounds=[-2.0, 2.0]))   # unhashable: built afresh
    assert (e["lo"], e["hi"]) == (-2.0, 2.0)
    np.random.seed(0)
    s1 = CEMPlanner._settings(sa, 4, dict(num_candidates=64))["seed"]
    s2 = CEMPlanner._settings(sa, 4, dict(num_candidates=64))["seed"]
    np.random.seed(0)
    assert s1 != s2 and s1 == int(np.random.randint(0, 2 ** 62, dtype=np.int64))
