"""Whole CEM plans at random model shapes against the oracle (oracle/cem.py, pinned by the
reference's own goldens): state / action dims, widths off the 16/64 grid, 1-4 hidden layers,
ensembles, reward-head models, candidate counts off every tile grid, short and long horizons,
elite counts from 1 to N and smoothing factors from 0 to 0.9.
Bars as test_gpu_parity.py's: returns within RTOL, every elite set, mu and sigma bit-exact, the
final actions bit-exact and the returned states within 1e-4."""
import numpy as np
import pytest
import torch

from oracle import cem as ocem

from test_gpu_parity import RTOL, build, rel_err

pytestmark = pytest.mark.gpu


def _shape(case):
    rng = np.random.default_rng(7000 + case)
    reward = case % 5 == 4
    cid = 6 if reward else 3
    over = dict(s=int(rng.integers(1, 41)), a=int(rng.integers(1, 13)),
                W=int(rng.choice([8, 16, 33, 50, 64, 100, 128, 200, 256, 300, 512])),
                L=int(rng.integers(1, 5)) if not reward else int(rng.integers(1, 4)),
                E=1 if reward else int(rng.choice([1, 1, 2, 3])))
    N = int(rng.choice([1, 5, 16, 31, 100, 257, 600]))
    H = int(rng.integers(1, 13))
    I = int(rng.integers(1, 4))
    if over["W"] >= 300 and N > 257:          # keep the NumPy oracle to seconds
        N = 257
    K = int(rng.integers(1, N + 1)) if case % 3 == 0 else max(1, N // 10)
    alpha = float(rng.choice([0.0, 0.1, 0.5, 0.9]))
    return cid, over, N, H, I, K, alpha


@pytest.mark.parametrize("case", range(48))
def test_cem_plan_random_shapes_against_the_oracle(case):
    from mbrl_amd import CEMPlanner, fused
    cid, over, N, H, I, K, alpha = _shape(case)
    p = ocem.synth_problem(cid, N=N, H=H, **over)
    module, model_fn, cost_fn, sample_action = build(p)
    md = fused.describe_model(model_fn)
    assert md is not None and fused.describe_cost(cost_fn, md["s"], md) is not None, "fused path not taken"
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H,
                                   num_candidates=N, num_elites=K, alpha=alpha, num_iterations=I,
                                   seed=p["rng_seed"], record=True)
    ref = ocem.cem_plan(p, N=N, H=H, K=K, alpha=alpha, num_iterations=I)
    for it in range(I):
        assert rel_err(res["returns"][it], ref["returns"][it]) < RTOL, (over, N, H, it)
        assert np.array_equal(res["elites"][it].cpu().numpy(), ref["elites"][it]), (over, N, H, it)
    assert np.array_equal(res["mu"].cpu().numpy(), ref["mu"][-1])
    assert np.array_equal(res["sigma"].cpu().numpy(), ref["sigma"][-1])
    assert np.array_equal(res["actions"].numpy(), ref["final_actions"])
    assert np.allclose(res["states"].numpy(), ref["final_states"], rtol=1e-4, atol=1e-4)
