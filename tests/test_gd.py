"""GradientDescentPlanner against the reference's own planner (golden fixtures
from tests/golden/make_golden_gd.py): the device restatement on the GPU, and the host loop on the
callables on CPU."""
import os
import sys

import numpy as np
import pytest
import torch

from oracle import cem as ocem

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden_gd as mgd  # noqa: E402


def closures(cid, over):
    import test_gpu_parity as tg
    p = ocem.synth_problem(cid, **over)
    _, model_fn, cost_fn, sample_action = tg.build(p)
    return p, model_fn, cost_fn


def plan(name, golden, device=None):
    from mbrl_amd import GradientDescentPlanner
    cid, over, H, iters, stop = mgd.CASES[name]
    g = golden(name)
    p, model_fn, cost_fn = closures(cid, over)
    assert ocem.weights_sha256(p["model"]) == str(g["weights_sha256"])
    A0 = g["init_actions"]
    init = ([], [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)])
    kw = dict(num_iterations=iters, stop_condition=stop)
    if device is not None:
        kw["device"] = device
    states, actions = GradientDescentPlanner.plan(torch.from_numpy(p["s0"]), model_fn, cost_fn, None, H, init, **kw)
    assert len(states) == H + 1 and len(actions) == H and states[0].shape == (1, p["cfg"]["s"])
    return torch.cat(states).numpy(), torch.cat(actions).numpy(), g


@pytest.mark.parametrize("name", list(mgd.CASES))
def test_gd_host_loop_matches_reference(golden, name, monkeypatch):
    """Unrecognised closures (forced here) run the reference's loop on the given callables."""
    from mbrl_amd import gd
    monkeypatch.setattr(gd, "describe", lambda model, cost, dev: (None, None))
    st, ac, g = plan(name, golden)
    assert np.allclose(ac, g["actions"], rtol=1e-5, atol=1e-6)
    assert np.allclose(st, g["states"], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(mgd.CASES))
def test_gd_device_matches_reference(golden, name):
    st, ac, g = plan(name, golden, device="cuda:0")
    assert np.allclose(ac, g["actions"], rtol=1e-4, atol=1e-5), np.max(np.abs(ac - g["actions"]))
    assert np.allclose(st, g["states"], rtol=1e-4, atol=1e-4), np.max(np.abs(st - g["states"]))


@pytest.mark.gpu
def test_gd_graph_replay_equals_eager():
    from mbrl_amd import gd
    p, model_fn, cost_fn = closures(3, dict(W=50, L=2))
    mdesc, cdesc = gd.describe(model_fn, cost_fn, torch.device("cuda:0"))
    A0 = mgd.initial_actions(10, 6)
    acts = [torch.from_numpy(A0[i:i + 1].copy()) for i in range(10)]
    dev = torch.device("cuda:0")
    s1, a1 = gd.plan_device(torch.from_numpy(p["s0"]), mdesc, cdesc, acts, 10, 20, 0.0, dev, use_graph=True)
    s2, a2 = gd.plan_device(torch.from_numpy(p["s0"]), mdesc, cdesc, acts, 10, 20, 0.0, dev, use_graph=False)
    assert torch.equal(a1, a2) and torch.equal(s1, s2)


@pytest.mark.gpu
@pytest.mark.parametrize("cid,over,H,iters,stop", [(3, dict(W=50, L=2), 10, 25, 0.0), (2, {}, 12, 40, 0.002),
                                                  (3, {}, 30, 15, 0.0), (3, dict(W=200, L=3), 8, 40, 0.01),
                                                  (2, {}, 5, 0, 0.0), (6, dict(W=64, L=2), 8, 30, 0.002),
                                                  (6, {}, 10, 20, 0.0), (6, dict(W=100, L=3), 6, 25, 0.001)])
def test_gd_fused_kernel_matches_graph_path(cid, over, H, iters, stop):
    """mbrl_gd_plan (forward, backward, Adam, stop test on the device in one launch) against the
    graph-replayed torch restatement of the same loop, including early stops and zero iterations, and
    reward-head models (config 6: RewardAgent's reward cost, two trunk passes per step)."""
    from mbrl_amd import gd
    p, model_fn, cost_fn = closures(cid, over)
    mdesc, cdesc = gd.describe(model_fn, cost_fn, torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    assert gd.fused_supported(mdesc, cdesc, dev)
    a = p["cfg"]["a"]
    A0 = mgd.initial_actions(H, a)
    acts = [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)]
    s0 = torch.from_numpy(p["s0"])
    s1, a1, n = gd.plan_fused(s0, mdesc, cdesc, acts, H, iters, stop, dev)
    s2, a2 = gd.plan_device(s0, mdesc, cdesc, acts, H, iters, stop, dev, use_fused=False)
    torch.cuda.synchronize()
    assert int(n.item()) <= iters
    assert torch.allclose(a1, a2, rtol=1e-4, atol=1e-5), float((a1 - a2).abs().max())
    assert torch.allclose(s1, s2, rtol=1e-4, atol=1e-4), float((s1 - s2).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("mode,cid", [("single", 3), ("abort", 3), ("single", 6), ("abort", 6)])
def test_gd_cooperative_kernel_and_its_fallback(mode, cid):
    """mbrl_gd_plan runs the cooperative kernel for W in {64..512} (goal-state and reward-head models):
    it must agree with the one-workgroup kernel (MBRL_OPT_GD_SINGLE), and when a hand-off gives up
    (MBRL_OPT_DEBUG_GD_ABORT) the gated one-workgroup kernel must produce the plan instead."""
    from mbrl_amd import _lib, gd
    p, model_fn, cost_fn = closures(cid, dict(W=256, L=3))
    mdesc, cdesc = gd.describe(model_fn, cost_fn, torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    H, a = 12, p["cfg"]["a"]
    A0 = mgd.initial_actions(H, a)
    acts = [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)]
    s0 = torch.from_numpy(p["s0"])
    s1, a1, n1 = gd.plan_fused(s0, mdesc, cdesc, acts, H, 30, 0.001, dev)
    with _lib.option("gd_single" if mode == "single" else "debug_gd_abort", 1):
        s2, a2, n2 = gd.plan_fused(s0, mdesc, cdesc, acts, H, 30, 0.001, dev)
    torch.cuda.synchronize()
    assert int(n1.item()) == int(n2.item())
    assert torch.allclose(a1, a2, rtol=1e-4, atol=1e-5), float((a1 - a2).abs().max())
    assert torch.allclose(s1, s2, rtol=1e-4, atol=1e-4), float((s1 - s2).abs().max())


def test_gd_reference_toy_known_answer(golden):
    """The reference's own gradient-planner script (src/mbrl/test_gradient_planner.py:5-27): s' = s + a,
    cost |s - 9|, s0 = [2], horizon 5, 40 Adam steps from a torch.randn draw. Plain callables take the
    generic path; states, actions and the printed total cost match the reference run
    (tests/golden/make_golden_gd.py main_toy, which stores the draw)."""
    from mbrl_amd import GradientDescentPlanner
    g = golden("gd_toy_abs_H5")
    drawn = torch.from_numpy(g["sampled"])

    def sample_action(batch_size):
        assert batch_size == 5
        return drawn.clone()

    states, actions = GradientDescentPlanner.plan(torch.tensor([2.0]), mgd.toy_model, mgd.toy_cost, sample_action, 5,
                                                  None, num_iterations=40)
    assert len(states) == 6 and len(actions) == 5
    st, ac = torch.cat(states).numpy(), torch.cat(actions).numpy()
    assert np.allclose(st, g["states"], rtol=1e-6, atol=1e-6), (st.ravel(), g["states"].ravel())
    assert np.allclose(ac, g["actions"], rtol=1e-6, atol=1e-6)
    total = float(mgd.toy_cost(torch.stack(states), torch.cat(actions)).sum())
    assert abs(total - float(g["total_cost"])) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("cid,over,H,B,mode", [(3, {}, 12, 11, None), (3, dict(W=64, L=2), 8, 5, None),
                                                (6, dict(W=256, L=3), 8, 9, None), (2, {}, 6, 3, "gd_single"),
                                                (3, dict(W=128, L=3), 6, 4, "debug_gd_abort")])
def test_gd_plan_batch_equals_single_plans(cid, over, H, B, mode):
    """mbrl_gd_plan_batch: B plans from different start states and initial sequences, in groups of
    co-resident cooperative grids (B = 11 at Wpad 512 needs two groups), are bit for bit the B plans
    mbrl_gd_plan makes one at a time -- through the cooperative kernel, the one-workgroup kernel, and
    the gated fallback after a forced hand-off timeout. Each plan keeps its own stop test."""
    from mbrl_amd import _lib, gd
    p, model_fn, cost_fn = closures(cid, over)
    mdesc, cdesc = gd.describe(model_fn, cost_fn, torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    s, a = p["cfg"]["s"], p["cfg"]["a"]
    rng = np.random.default_rng(cid * 10 + B)
    S0 = torch.from_numpy(np.stack([p["s0"]] + [rng.standard_normal(s).astype(np.float32) for _ in range(B - 1)]))
    A0 = torch.from_numpy(rng.uniform(-1, 1, (B, H, a)).astype(np.float32))
    iters, stop = 25, 0.002
    ctx = _lib.option(mode, 1) if mode else _lib.option("gd_single", 0)
    with ctx:
        sb, ab, nb = gd.plan_fused_batch(S0, mdesc, cdesc, A0, H, iters, stop, dev)
        singles = [gd.plan_fused(S0[b], mdesc, cdesc, list(A0[b].split(1, 0)), H, iters, stop, dev) for b in range(B)]
    torch.cuda.synchronize()
    for b, (s1, a1, n1) in enumerate(singles):
        assert torch.equal(sb[b], s1) and torch.equal(ab[b], a1), b
        assert int(nb[b]) == int(n1.item()), b
    assert len({int(x) for x in nb.tolist()}) >= 1


@pytest.mark.gpu
def test_gd_planner_plan_batch_api():
    """GradientDescentPlanner.plan_batch returns what B plan() calls return for the same start
    states and the same sampler draws (the sampler is called in row order)."""
    from mbrl_amd import GradientDescentPlanner
    p, model_fn, cost_fn = closures(3, dict(W=64, L=2))
    s, a, H, B = p["cfg"]["s"], p["cfg"]["a"], 6, 4
    S0 = torch.from_numpy(np.random.default_rng(0).standard_normal((B, s)).astype(np.float32))

    def sampler(batch_size):
        return torch.rand((batch_size, a)) * 2 - 1
    torch.manual_seed(7)
    st, ac = GradientDescentPlanner.plan_batch(S0, model_fn, cost_fn, sampler, H, num_iterations=20, device="cuda:0")
    torch.manual_seed(7)
    for b in range(B):
        s1, a1 = GradientDescentPlanner.plan(S0[b], model_fn, cost_fn, sampler, H, num_iterations=20, device="cuda:0")
        assert torch.equal(st[b], torch.cat(s1, 0)) and torch.equal(ac[b], torch.cat(a1, 0)), b
    assert st.shape == (B, H + 1, s) and ac.shape == (B, H, a)



@pytest.mark.gpu
@pytest.mark.parametrize("case", range(12))
def test_gd_fused_random_shapes_match_graph_path(case):
    """mbrl_gd_plan at random shapes (the cooperative kernel where it applies, the one-workgroup kernel
    elsewhere) against the graph-replayed torch restatement, within the float tolerance."""
    from mbrl_amd import gd
    rng = np.random.default_rng(9000 + case)
    reward = case % 3 == 2
    over = dict(s=int(rng.integers(1, 24)), a=int(rng.integers(1, 8)),
                W=int(rng.choice([16, 50, 64, 100, 128, 256, 512])), L=int(rng.integers(1, 4)))
    p = ocem.synth_problem(6 if reward else 3, **over)
    import test_gpu_parity as tg
    _, model_fn, cost_fn, _ = tg.build(p)
    mdesc, cdesc = gd.describe(model_fn, cost_fn, torch.device("cuda:0"))
    dev = torch.device("cuda:0")
    assert gd.fused_supported(mdesc, cdesc, dev)
    H, iters = int(rng.integers(1, 16)), int(rng.integers(0, 30))
    A0 = rng.uniform(-0.5, 0.5, (H, over["a"])).astype(np.float32)
    acts = [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)]
    s0 = torch.from_numpy(p["s0"])
    s1, a1, _ = gd.plan_fused(s0, mdesc, cdesc, acts, H, iters, 0.0, dev)
    s2, a2 = gd.plan_device(s0, mdesc, cdesc, acts, H, iters, 0.0, dev, use_fused=False)
    torch.cuda.synchronize()
    assert torch.allclose(a1, a2, rtol=1e-4, atol=1e-5), (over, H, iters, float((a1 - a2).abs().max()))
    assert torch.allclose(s1, s2, rtol=1e-4, atol=1e-4), (over, H, iters, float((s1 - s2).abs().max()))
