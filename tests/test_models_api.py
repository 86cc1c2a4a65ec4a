"""The rest of the reference's models.py API (/root/reference/src/mbrl/models.py): LinearModel
(experiment.py:41's "lin" dynamics model), CostModel and QuadraticCost -- constructors, parameter
names (state_dicts load both ways), forward arithmetic, and LinearModel's training and planning
through the generic paths."""
import functools

import numpy as np
import pytest
import torch


def _dataset(s, a, T=300, seed=0):
    from mbrl_amd import data
    rng = np.random.Generator(np.random.PCG64(seed))
    st = rng.standard_normal((T + 1, s)).astype(np.float32)
    acts = rng.uniform(-1, 1, (T, a)).astype(np.float32)
    for t in range(T):                                   # a linear system to learn
        st[t + 1] = 0.9 * st[t] + 0.1 * np.resize(acts[t], s)
    roll = data.Rollout(states=list(torch.from_numpy(st)), observations=list(torch.from_numpy(st)),
                        actions=list(torch.from_numpy(acts)), rewards=list(torch.zeros(T)))
    ds = data.TransitionsDataset(rollouts=[roll])
    ds.set_data_mode("state_only")
    return ds


def test_linear_model_matches_the_reference_layout_and_arithmetic():
    from mbrl_amd import LinearModel
    torch.manual_seed(0)
    m = LinearModel(5, 2)
    assert sorted(m.state_dict()) == ["linear1.bias", "linear1.weight"]
    assert m.linear1.in_features == 7 and m.linear1.out_features == 5
    s, a = torch.randn(4, 5), torch.randn(4, 2)
    assert torch.equal(m(s, a), m.linear1(torch.cat([s, a], 1)))
    torch.manual_seed(1)
    noisy = LinearModel(5, 2, noise=0.5)
    noisy.load_state_dict(m.state_dict())
    assert not torch.equal(noisy(s, a), m(s, a))


def test_linear_model_trains_on_cpu():
    from mbrl_amd import LinearModel
    ds = _dataset(4, 2)
    torch.manual_seed(0)
    m = LinearModel(4, 2)
    opt = torch.optim.Adam(m.parameters(), lr=1e-2)
    np.random.seed(0)
    before = float(np.mean(m.evaluate_model(ds, batch_size=64)))
    np.random.seed(1)
    m.train_model(ds, opt, batch_size=64, num_epochs=20)
    np.random.seed(0)
    after = float(np.mean(m.evaluate_model(ds, batch_size=64)))
    assert after < 0.1 * before and m.train_iterations == 1


def test_cost_model_and_quadratic_cost():
    from mbrl_amd import CostModel, QuadraticCost
    torch.manual_seed(0)
    c = CostModel(5, 2)
    assert sorted(c.state_dict()) == ["linear1.bias", "linear1.weight", "linear2.bias", "linear2.weight",
                                      "linear3.bias", "linear3.weight"]
    s, a = torch.randn(3, 5), torch.randn(3, 2)
    x = torch.relu(c.linear2(torch.relu(c.linear1(torch.cat([s, a], -1)))))
    assert torch.equal(c(s, a), c.linear3(x)) and c(s, a).shape == (3, 1)
    g = torch.randn(4)
    q = QuadraticCost(4, g)
    v = torch.randn(4)
    assert torch.allclose(q(v), torch.dot(v - g, q.linear(v - g)))
    q.set_goal_state(torch.zeros(4))
    assert torch.allclose(q(v), torch.dot(v, q.linear(v)))


@pytest.mark.gpu
def test_linear_model_on_the_gpu_paths():
    """LinearModel trains through autograd on the GPU (within 1e-4 of CPU training) and plans through
    the planners' callable path (the fused kernels need a hidden layer)."""
    from mbrl_amd import CEMPlanner, LinearModel, fused, models
    ds = _dataset(4, 2)
    out = {}
    for dev in ("cpu", "cuda:0"):
        torch.manual_seed(0)
        m = LinearModel(4, 2).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-2)
        np.random.seed(1)
        m.train_model(ds, opt, batch_size=64, num_epochs=3)
        out[dev] = [p.detach().cpu() for p in m.parameters()]
    for x, y in zip(out["cpu"], out["cuda:0"]):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-5)
    model_fn = functools.partial(m)
    assert fused.describe_model(model_fn) is None
    cost = models.goal_state_cost(models.SmoothAbsLoss(torch.ones(4), torch.zeros(4)), models.CoshLoss())
    def sample_action(batch_size):
        return torch.rand((batch_size, 2)) * 2 - 1
    st, ac = CEMPlanner.plan(torch.ones(4), model_fn, cost, sample_action, 5, num_candidates=64, num_iterations=2,
                             seed=3, device="cuda:0")
    assert len(st) == 5 and len(ac) == 5
