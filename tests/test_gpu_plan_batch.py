"""RandomShootingPlanner.plan_batch (the reference's planners.py:140-216 for B start states at once,
the planner service's batched call for that planner) against B single plans."""
import numpy as np
import pytest
import torch

from test_gd import closures


@pytest.mark.gpu
@pytest.mark.parametrize("cid,N,H,B", [(2, 128, 12, 5), (3, 300, 6, 3), (6, 64, 5, 4)])
def test_random_shooting_plan_batch_equals_single_plans(cid, N, H, B):
    """RandomShootingPlanner.plan_batch (all B*N candidates in one rollout, per-candidate start states,
    per-row np.argmin) returns bit for bit what B plan() calls return for the same sampler draws."""
    from mbrl_amd import RandomShootingPlanner
    p, model_fn, cost_fn = closures(cid, {})
    s, a = p["cfg"]["s"], p["cfg"]["a"]
    S0 = torch.from_numpy(np.random.default_rng(cid).standard_normal((B, s)).astype(np.float32))

    def sampler(batch_size):
        return torch.rand((batch_size, a)) * 2 - 1
    torch.manual_seed(3)
    st, ac = RandomShootingPlanner.plan_batch(S0, model_fn, cost_fn, sampler, H, num_trajectories=N,
                                              device="cuda:0")
    torch.manual_seed(3)
    for b in range(B):
        s1, a1 = RandomShootingPlanner.plan(S0[b], model_fn, cost_fn, sampler, H, num_trajectories=N,
                                            device="cuda:0")
        assert torch.equal(st[b], s1) and torch.equal(ac[b], a1), b
    assert st.shape == (B, H, s) and ac.shape == (B, H, a)
