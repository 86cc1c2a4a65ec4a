"""The fused per-iteration update (cem.hip cem_update_kernel + cem_init_kernel; DESIGN.md §3 "update"):
one launch per CEM iteration selects the elites, refits every row and draws the next iteration's
proposals. It runs the same select / refit / draw bodies as the separate launches, so a plan must
come out BIT FOR BIT the same with mbrl_set_option(MBRL_OPT_UNFUSED_UPDATE, 1) (the separate
select_reg_kernel, refit_fused_kernel and sample_kernel launches): returns, elites, mu, sigma, the
final actions and the predicted states. The oracle bars themselves are test_gpu_parity.py's, which
run through the fused path by default."""
import numpy as np
import pytest
import torch

from oracle import cem as ocem

from test_gpu_parity import build

pytestmark = pytest.mark.gpu


def _plans(p, H, **kw):
    from mbrl_amd import CEMPlanner, _lib
    _, model_fn, cost_fn, sample_action = build(p)
    out = {}
    for unfused in (0, 1):
        with _lib.option("unfused_update", unfused):
            out[unfused] = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H,
                                                    seed=p["rng_seed"], record=True, **kw)
    return out


# cartpole (N * a small: the draw is fused), cheetah, walker at full N (KPT 16), an ensemble, the
# reward-head model, degenerate sizes (one candidate, every candidate an elite, off the tile grid)
@pytest.mark.parametrize("cid,N,H,K,I", [(2, 1024, 20, None, 5), (3, 4096, 30, None, 3), (4, 16384, 6, None, 2),
                                          (5, 300, 5, None, 3), (6, 512, 8, None, 3), (3, 1, 2, 1, 2),
                                          (3, 17, 3, 17, 2), (2, 33, 4, 5, 3), (4, 5000, 3, 7, 2)])
def test_fused_update_plan_equals_separate_launches(cid, N, H, K, I):
    p = ocem.synth_problem(cid, N=N, H=H)
    kw = dict(num_candidates=N, num_iterations=I)
    if K is not None:
        kw["num_elites"] = K
    out = _plans(p, H, **kw)
    for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
        a, b = out[0][k], out[1][k]
        if isinstance(a, (list, tuple)):
            for it, (x, y) in enumerate(zip(a, b)):
                assert torch.equal(torch.as_tensor(x), torch.as_tensor(y)), (k, it)
        else:
            assert torch.equal(torch.as_tensor(a), torch.as_tensor(b)), k


@pytest.mark.parametrize("cid,N,H,B", [(2, 1024, 20, 4), (3, 512, 6, 3), (5, 128, 4, 2)])
def test_fused_update_batched_plans_equal_separate_launches(cid, N, H, B):
    from mbrl_amd import CEMPlanner, _lib
    p = ocem.synth_problem(cid, N=N, H=H)
    _, model_fn, cost_fn, sample_action = build(p)
    rng = np.random.default_rng(cid)
    S0 = np.stack([p["s0"]] + [rng.standard_normal(p["cfg"]["s"]).astype(np.float32) for _ in range(B - 1)])
    out = {}
    for unfused in (0, 1):
        with _lib.option("unfused_update", unfused):
            out[unfused] = CEMPlanner.plan_batch(torch.from_numpy(S0), model_fn, cost_fn, sample_action, H,
                                                 num_candidates=N, num_iterations=3, seed=p["rng_seed"])
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
