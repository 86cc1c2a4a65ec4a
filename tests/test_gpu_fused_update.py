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


def _fused_k_cap(N, a):
    """Largest K whose selection + refit working set fits cem_update_kernel's LDS (cem.hip update_kpt)."""
    kpt = 1
    while N > 1024 * kpt:
        kpt *= 2
    a4 = (a + 3) & ~3
    sel = max(33 * 32 * kpt, 2 * 16 * 257)
    K = N
    while K > 1:
        nch = (K + 31) // 32
        ref = ((K * a + 3) & ~3) + ((nch * a + 3) & ~3) + 3 * a4
        if (((K + 3) & ~3) + 2 * a4 + max(sel, ref)) * 4 + 1024 <= 160 * 1024:
            break
        K = max(1, K * 3 // 4)
    return K


@pytest.mark.parametrize("case", range(24))
def test_cem_update_abi_against_the_oracle_random_shapes(case):
    """mbrl_cem_update at random shapes against the oracle: E-member costs with ties, NaN, -0/+0 and
    repeated values; the elite set (stable top-K of the member mean), the refit's mu / sigma, and the
    next iteration's proposals for a random global candidate range -- all bit for bit."""
    from mbrl_amd import fused
    from oracle.philox import cem_actions
    rng = np.random.default_rng(1000 + case)
    E = int(rng.choice([1, 1, 2, 5]))
    N = int(rng.choice([1, 3, 17, 64, 255, 1024, 1500, 4096, 9000, 16384, 32768]))
    H = int(rng.integers(1, 12))
    a = int(rng.integers(1, 22))
    K = int(rng.integers(1, N + 1)) if case % 3 else max(1, N // 10)
    K = min(K, _fused_k_cap(N, a))           # keep the shape inside the fused kernel's LDS
    seed, it = int(rng.integers(0, 2 ** 62)), int(rng.integers(0, 4))
    c = rng.uniform(100, 140, (E, N)).astype(np.float32)
    if N > 4:
        c[:, rng.integers(0, N, N // 4)] = np.float32(120.0)          # exact ties
        c[0, rng.integers(0, N)] = np.float32(-0.0)
        c[-1, rng.integers(0, N)] = np.float32(0.0)
        if case % 4 == 0:
            c[0, rng.integers(0, N)] = np.nan
    mu = rng.uniform(-0.3, 0.3, (H, a)).astype(np.float32)
    sg = rng.uniform(0.05, 0.6, (H, a)).astype(np.float32)
    off = int(rng.integers(0, N))
    cnt = int(rng.integers(1, N - off + 1))
    dev = torch.device("cuda", 0)
    costs = torch.from_numpy(c).to(dev)
    mu_d, sg_d = torch.from_numpy(mu).to(dev), torch.from_numpy(sg).to(dev)
    mu_o, sg_o = torch.empty_like(mu_d), torch.empty_like(sg_d)
    nxt = torch.empty((H, cnt, a), dtype=torch.float32, device=dev)
    rets = torch.empty(N, dtype=torch.float32, device=dev)
    sp = fused.make_sampler(seed, it, mu_d, sg_d, -1.0, 1.0)
    el = fused.cem_update(costs, K, sp, H, a, 0.1, mu_o, sg_o, returns_out=rets, next_actions=nxt, draw_offset=off)
    torch.cuda.synchronize()
    assert el is not None
    ret = ocem.ensemble_returns(c)
    assert np.array_equal(rets.cpu().numpy(), ret, equal_nan=True)
    ref_el = ocem.select_elites(ret, K)
    assert np.array_equal(el.cpu().numpy(), ref_el)
    A = cem_actions(mu, sg, -1.0, 1.0, seed, it, ref_el)
    m2, s2 = ocem.refit(mu, sg, np.ascontiguousarray(A.transpose(1, 0, 2)), 0.1)
    assert np.array_equal(mu_o.cpu().numpy(), m2) and np.array_equal(sg_o.cpu().numpy(), s2)
    nref = cem_actions(m2, s2, -1.0, 1.0, seed, it + 1, np.arange(off, off + cnt))
    assert np.array_equal(nxt.cpu().numpy(), nref)


# the split update (cem_select_regen_kernel + cem_refit_draw_kernel: the elites' regeneration shared
# out over the row's workgroups) forced on and off: walker at full N (where auto takes it), cheetah,
# cartpole, the reward head, degenerate sizes (one candidate; every candidate an elite; K < S)
@pytest.mark.parametrize("cid,N,H,K,I", [(4, 16384, 6, None, 3), (3, 4096, 30, None, 3), (2, 1024, 20, None, 3),
                                          (6, 512, 8, None, 2), (3, 1, 2, 1, 2), (3, 17, 3, 17, 2), (2, 33, 4, 5, 3)])
def test_split_update_plan_equals_one_launch_update(cid, N, H, K, I):
    from mbrl_amd import CEMPlanner, _lib
    p = ocem.synth_problem(cid, N=N, H=H)
    _, model_fn, cost_fn, sample_action = build(p)
    kw = dict(num_candidates=N, num_iterations=I)
    if K is not None:
        kw["num_elites"] = K
    out = {}
    for split in (0, 1, 2):
        with _lib.option("update_split", split):
            out[split] = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H,
                                                  seed=p["rng_seed"], record=True, **kw)
    for split in (0, 2):
        for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
            a, b = out[split][k], out[1][k]
            if isinstance(a, (list, tuple)):
                for it, (x, y) in enumerate(zip(a, b)):
                    assert torch.equal(torch.as_tensor(x), torch.as_tensor(y)), (split, k, it)
            else:
                assert torch.equal(torch.as_tensor(a), torch.as_tensor(b)), (split, k)
