"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the reference's golden
vectors. Bars: bit-exact for the RNG draw, elite index sets, argmin and the refit's mu / sigma;
returns within 1e-5 relative (BASELINE.json north_star) against max(|ref|, 1)."""
import functools
import os

import numpy as np
import pytest
import torch

from oracle import cem as ocem
from oracle.philox import cem_actions

pytestmark = pytest.mark.gpu
RTOL = 1e-5
DEV = "cuda:0"


def rel_err(x, ref):
    x = x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)
    return float(np.max(np.abs(x.astype(np.float64) - ref) / np.maximum(np.abs(ref), 1.0)))


def build(problem):
    """mbrl_amd model / cost / sampler closures wired exactly as GoalStateAgent (agents.py:219-233),
    or as RewardAgent (agents.py:336-362) for a reward-head problem."""
    from mbrl_amd import data, env, models
    cfg = problem["cfg"]
    s, a, W, L = cfg["s"], cfg["a"], cfg["W"], cfg["L"]
    if cfg.get("reward"):
        import operator
        m = models.ModelWithReward(s, a, hidden_units=W, n_hidden=L)
        (*trunk, (hw, hb)) = problem["model"][0]
        with torch.no_grad():
            for lin, (w, b) in zip(m.linears(), trunk + [(hw[:s], hb[:s]), (hw[s:], hb[s:])]):
                lin.weight.copy_(torch.from_numpy(np.ascontiguousarray(w)))
                lin.bias.copy_(torch.from_numpy(np.ascontiguousarray(b)))
        nm = problem["norm"]
        ds = data.TransitionsDataset.from_statistics({k: {"mean": torch.from_numpy(nm[p + "_mean"]), "std": torch.from_numpy(nm[p + "_std"])}
                                      for k, p in (("observations", "obs"), ("actions", "act"), ("rewards", "rew"))})
        kw = ds.normalizers(reward=True)
        model_fn = models.compose(functools.partial(m, **kw), operator.itemgetter(0))
        cost_fn = models.compose(functools.partial(m, **kw), operator.itemgetter(1))
        return m, model_fn, cost_fn, env.sample_action_fn(env.BoundedActionSpec(a, -1.0, 1.0))
    members = []
    for layers in problem["model"]:
        m = models.Model(s, a, hidden_units=W, n_hidden=L)
        with torch.no_grad():
            for lin, (w, b) in zip(m.linears(), layers):
                lin.weight.copy_(torch.from_numpy(w))
                lin.bias.copy_(torch.from_numpy(b))
        members.append(m)
    module = members[0] if len(members) == 1 else models.EnsembleModel(members)
    nm = problem["norm"]
    ds = data.TransitionsDataset.from_statistics({"observations": {"mean": torch.from_numpy(nm["obs_mean"]),
                                                   "std": torch.from_numpy(nm["obs_std"])},
                                  "actions": {"mean": torch.from_numpy(nm["act_mean"]),
                                              "std": torch.from_numpy(nm["act_std"])}})
    model_fn = functools.partial(module, **ds.normalizers())
    c = problem["cost"]
    cost_fn = models.goal_state_cost(models.SmoothAbsLoss(torch.from_numpy(c["weights"]), torch.from_numpy(c["goal"]),
                                                          c["alpha_state"]), models.CoshLoss(c["alpha_action"]))
    sample_action = env.sample_action_fn(env.BoundedActionSpec(a, -1.0, 1.0))
    return module, model_fn, cost_fn, sample_action


def device_problem(problem):
    from mbrl_amd import fused
    _, model_fn, cost_fn, _ = build(problem)
    md = fused.describe_model(model_fn)
    cd = fused.describe_cost(cost_fn, md["s"], md)
    assert md is not None and cd is not None, "closures not recognised by the fused path"
    return fused.device_problem(md, cd, torch.device(DEV))


# ------------------------------------------------------------------------------------------------ RNG
@pytest.mark.parametrize("a,N,H,it,offset", [(1, 1000, 12, 0, 0), (6, 4096, 30, 3, 0), (21, 257, 5, 4, 4096),
                                             (5, 33, 3, 1, 7)])
def test_proposal_draw_bit_exact(a, N, H, it, offset):
    from mbrl_amd import fused
    rng = np.random.default_rng(a * 131 + N)
    mu = rng.uniform(-0.5, 0.5, size=(H, a)).astype(np.float32)
    sg = rng.uniform(0.1, 0.9, size=(H, a)).astype(np.float32)
    mu_d, sg_d = torch.from_numpy(mu).to(DEV), torch.from_numpy(sg).to(DEV)
    out = torch.empty((H, N, a), dtype=torch.float32, device=DEV)
    seed = 0x1234_5678_9ABC + a
    fused.sample_actions(fused.make_sampler(seed, it, mu_d, sg_d, -1.0, 1.0), H, a, N, offset, out)
    ref = cem_actions(mu, sg, -1.0, 1.0, seed, it, np.arange(offset, offset + N))
    assert np.array_equal(out.cpu().numpy(), ref)


# ------------------------------------------------------------------------------------------------ rollout
@pytest.mark.parametrize("cid,over", [(2, dict(N=1000, H=20)), (3, dict(N=300, H=30)), (4, dict(N=200, H=7)),
                                      (5, dict(N=40, H=6)), (2, dict(N=1, H=3)), (3, dict(N=17, H=2)),
                                      (6, dict(N=300, H=12)), (6, dict(N=5000, H=4)), (6, dict(N=9000, H=3))])
def test_rollout_costs_and_states_given_actions(cid, over):
    from mbrl_amd import fused
    p = ocem.synth_problem(cid, **over)
    N, H, a, s, E = over["N"], over["H"], p["cfg"]["a"], p["cfg"]["s"], p["cfg"]["E"]
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 11, 0, np.arange(N))
    ref_costs, ref_states = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A, store_states=True)
    prob = device_problem(p)
    states = torch.empty((E, H, N, s), dtype=torch.float32, device=DEV)
    costs = fused.rollout(prob, torch.from_numpy(p["s0"]).to(DEV), N, H, actions=torch.from_numpy(A).to(DEV),
                          states_out=states)
    torch.cuda.synchronize()
    assert rel_err(costs, ref_costs) < RTOL
    assert np.allclose(states.cpu().numpy(), ref_states, rtol=1e-4, atol=1e-4)


def test_rollout_sampled_matches_given():
    """In-kernel Philox draw == the standalone draw: same costs and the same recorded actions."""
    from mbrl_amd import _lib, fused
    p = ocem.synth_problem(3, N=500, H=9)
    prob = device_problem(p)
    N, H, a = 500, 9, 6
    mu = torch.full((H, a), 0.1, device=DEV)
    sg = torch.full((H, a), 0.4, device=DEV)
    sp = fused.make_sampler(77, 2, mu, sg, -1.0, 1.0)
    acts = torch.empty((H, N, a), device=DEV)
    s0 = torch.from_numpy(p["s0"]).to(DEV)
    c1 = fused.rollout(prob, s0, N, H, sampler=sp, actions_out=acts)
    c2 = fused.rollout(prob, s0, N, H, actions=acts.clone())
    torch.cuda.synchronize()
    ref = cem_actions(mu.cpu().numpy(), sg.cpu().numpy(), -1, 1, 77, 2, np.arange(N))
    assert np.array_equal(acts.cpu().numpy(), ref)
    assert torch.equal(c1, c2)
    assert _lib is not None


def test_dynamics_forward_matches_oracle_step():
    p = ocem.synth_problem(4)
    module, model_fn, _, _ = build(p)
    rng = np.random.default_rng(5)
    B = 333
    s = rng.standard_normal((B, 24)).astype(np.float32)
    a = rng.uniform(-1, 1, (B, 6)).astype(np.float32)
    with torch.no_grad():
        out = model_fn(torch.from_numpy(s).to(DEV), torch.from_numpy(a).to(DEV))
    ref = ocem.dynamics_step(p["model"][0], p["norm"], s, a)
    assert np.allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    from mbrl_amd import fused
    assert fused._PACKED.get(module) is not None, "forward did not take the HIP path"


# ------------------------------------------------------------------------------------------------ select / refit
def test_select_matches_stable_argsort_with_ties_nan_and_signed_zero():
    from mbrl_amd import _lib, fused
    rng = np.random.default_rng(0)
    for N, K in [(1, 1), (10, 3), (1000, 100), (4096, 409), (32768, 3276), (5000, 5000), (70001, 7000),
                 (250000, 25000)]:
        r = rng.integers(0, 50, size=N).astype(np.float32)      # heavy ties
        if N >= 10:
            r[rng.integers(0, N, size=N // 10 + 1)] = np.nan
            r[rng.integers(0, N, size=3)] = -0.0
            r[rng.integers(0, N, size=3)] = 0.0
            r[rng.integers(0, N, size=2)] = -np.inf
        el = fused.select(torch.from_numpy(r).to(DEV).view(1, N), K)
        assert np.array_equal(el.cpu().numpy(), ocem.select_elites(r, K)), (N, K)
        am = fused.select(torch.from_numpy(r).to(DEV).view(1, N), 1, nan_policy=_lib.MBRL_NAN_FIRST)
        assert int(am[0]) == ocem.rs_argmin(r), N


@pytest.mark.parametrize("N", [1024, 4096, 16384, 32768, 4094, 16381])
def test_select_fuzz_distributions(N):
    """The register-resident selection (wide 11-bit first pass, the bucket's keys listed in LDS, 8-bit
    passes over the list or over every key when the bucket is too large; the bitmap compaction when
    every key equal to the K-th is an elite, the packed-count compaction when ties are cut) against
    NumPy's stable order on distributions that exercise each branch: plan-like returns in one binade
    (wide, and a few % of it as walker's late iterations), a narrow cluster (the K-th bucket large), heavy ties, NaN- and signed-zero-heavy sets, a wide spread
    over binades, all-equal keys; K from 1 to N; N not a multiple of 4 for the single-key layout."""
    from mbrl_amd import fused
    rng = np.random.default_rng(N)
    dists = [lambda: rng.uniform(130, 250, N), lambda: rng.uniform(189.3, 192.9, N), lambda: rng.uniform(120, 120.01, N),
             lambda: rng.integers(0, 7, N), lambda: np.where(rng.random(N) < .4, np.nan, rng.standard_normal(N)),
             lambda: np.where(rng.random(N) < .5, -0.0, 0.0), lambda: np.exp(rng.uniform(-30, 30, N)),
             lambda: np.full(N, 3.5)]
    for i, d in enumerate(dists):
        r = np.asarray(d(), dtype=np.float32)
        for K in (1, max(1, N // 10), N // 2 + 1, N):
            el = fused.select(torch.from_numpy(r).to(DEV).view(1, N), K)
            assert np.array_equal(el.cpu().numpy(), ocem.select_elites(r, K)), (N, i, K)


def test_select_ensemble_mean():
    from mbrl_amd import fused
    rng = np.random.default_rng(1)
    c = rng.uniform(100, 200, size=(5, 3000)).astype(np.float32)
    ret = torch.empty(3000, device=DEV)
    el = fused.select(torch.from_numpy(c).to(DEV), 300, returns_out=ret)
    r = ocem.ensemble_returns(c)
    assert np.array_equal(ret.cpu().numpy(), r)
    assert np.array_equal(el.cpu().numpy(), ocem.select_elites(r, 300))


@pytest.mark.parametrize("H,a,N,K", [(30, 6, 4096, 409), (50, 21, 2000, 200), (12, 1, 128, 1), (7, 5, 100, 100)])
def test_refit_bit_exact(H, a, N, K):
    from mbrl_amd import fused
    rng = np.random.default_rng(H + a)
    mu = rng.uniform(-0.3, 0.3, size=(H, a)).astype(np.float32)
    sg = rng.uniform(0.2, 0.6, size=(H, a)).astype(np.float32)
    elites = np.sort(rng.choice(N, size=K, replace=False)).astype(np.int64)
    mu_d, sg_d = torch.from_numpy(mu).to(DEV), torch.from_numpy(sg).to(DEV)
    mo, so = torch.empty_like(mu_d), torch.empty_like(sg_d)
    sp = fused.make_sampler(4242, 1, mu_d, sg_d, -1.0, 1.0)
    fused.refit(sp, H, a, torch.from_numpy(elites).to(DEV), 0.1, mo, so)
    A = cem_actions(mu, sg, -1, 1, 4242, 1, elites)                # [H, K, a]
    rm, rs = ocem.refit(mu, sg, np.ascontiguousarray(A.transpose(1, 0, 2)), 0.1)
    assert np.array_equal(mo.cpu().numpy(), rm)
    assert np.array_equal(so.cpu().numpy(), rs)


# ------------------------------------------------------------------------------------------------ whole planners
CEM_CASES = [("config2_cem", 2, {}), ("config3_cem", 3, {}), ("config4_cem_N2048", 4, dict(N=2048)),
             ("config5_cem_N256_H20", 5, dict(N=256, H=20)), ("config6_cem_N512_H10", 6, dict(N=512, H=10))]


@pytest.mark.parametrize("name,cid,over", CEM_CASES, ids=[c[0] for c in CEM_CASES])
def test_cem_plan_against_reference_golden(golden, name, cid, over):
    from mbrl_amd import CEMPlanner
    g = golden(name)
    p = ocem.synth_problem(cid, **over)
    _, model_fn, cost_fn, sample_action = build(p)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, int(g["H"]),
                                   num_candidates=int(g["N"]), num_elites=int(g["K"]),
                                   num_iterations=int(g["I"]), alpha=float(g["alpha"]), seed=p["rng_seed"],
                                   record=True)
    for it in range(int(g["I"])):
        assert rel_err(res["returns"][it], g["returns"][it]) < RTOL, f"iteration {it}"
        assert np.array_equal(res["elites"][it].cpu().numpy(), g["elites"][it]), f"iteration {it}"
    assert np.array_equal(res["mu"].cpu().numpy(), g["mu"][-1])
    assert np.array_equal(res["sigma"].cpu().numpy(), g["sigma"][-1])
    assert np.array_equal(res["actions"].numpy(), g["final_actions"])
    assert np.allclose(res["states"].numpy(), g["final_states"], rtol=1e-4, atol=1e-4)


def test_random_shooting_planner_against_reference_golden(golden):
    """Config 1 through the public API with the reference's sampler semantics and global NumPy RNG."""
    from mbrl_amd import RandomShootingPlanner
    g = golden("config1_rs")
    p = ocem.synth_problem(1)
    _, model_fn, cost_fn, sample_action = build(p)
    np.random.seed(int(g["np_seed"]))
    states, actions = RandomShootingPlanner.plan(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action,
                                                 p["cfg"]["H"], None, num_trajectories=p["cfg"]["N"])
    assert np.array_equal(actions.numpy(), g["plan_actions"])
    assert np.allclose(states.numpy(), g["plan_states"], rtol=1e-5, atol=1e-5)


def test_random_shooting_toy_known_answer(golden):
    """test_random_shooting.py:5-25 through the generic callable path (HIP argmin)."""
    from mbrl_amd import RandomShootingPlanner
    world_size, goal = 10, torch.tensor(9, dtype=torch.float)

    def model(states, actions):
        return torch.fmod((torch.fmod(states + actions, world_size) + world_size), world_size)

    def sample_action(batch_size):
        return torch.randint(low=-1, high=2, size=(batch_size, 1), dtype=torch.float)

    def cost(states, actions):
        return torch.abs(states - goal.to(states.device))

    torch.manual_seed(0)
    states, actions = RandomShootingPlanner.plan(torch.tensor([2], dtype=torch.float), model, cost, sample_action, 5,
                                                 None, num_trajectories=1000)
    assert states.numpy().ravel().tolist() == [1.0, 0.0, 9.0, 9.0, 8.0]
    assert float(torch.abs(states - 9).sum()) == 18.0


def _impostors():
    """Functions that carry the names closure recognition goes by (fused._field_stats,
    describe_cost) but compute something else."""
    def normalize_field(field_value, field_name, stats):
        return (field_value - stats[field_name]["mean"]) / stats[field_name]["std"] * 0.5

    def state_action_cost(state, action, state_cost, action_cost):
        return state_cost(state) + 2.0 * action_cost(action)
    return normalize_field, state_action_cost


def test_semantic_check_sends_impostor_closures_to_the_generic_path():
    """A one-time probe (fused.semantic_check) compares the fused arithmetic with the callables; a
    same-named impostor normaliser or cost is caught and the planner runs the callables as given
    (the reference's semantics), with a warning. Genuine closures keep the fused path."""
    from mbrl_amd import CEMPlanner, fused
    p = ocem.synth_problem(2, N=256, H=6)
    module, model_fn, cost_fn, sample_action = build(p)
    assert fused.describe(model_fn, cost_fn, torch.device(DEV))[0] is not None
    imp_norm, imp_cost = _impostors()
    kw = dict(model_fn.keywords)
    kw["normalize_state"] = functools.partial(imp_norm, **kw["normalize_state"].keywords)
    bad_model = functools.partial(model_fn.func, **kw)
    bad_cost = functools.partial(imp_cost, **cost_fn.keywords)
    for m, c in ((bad_model, cost_fn), (model_fn, bad_cost)):
        assert fused.describe_model(m) is not None and fused.describe_cost(c, 5, fused.describe_model(m)) is not None
        with pytest.warns(UserWarning, match="generic path"):
            md, cd = fused.describe(m, c, torch.device(DEV))
        assert md is None and cd is None
        opts = dict(num_candidates=256, num_iterations=2, seed=9, record=True)
        got = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), m, c, sample_action, 6, **opts)
        opaque = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), lambda s, a: m(s, a), lambda s, a: c(s, a),
                                          sample_action, 6, **opts)
        assert torch.equal(got["returns"], opaque["returns"]) and torch.equal(got["elites"], opaque["elites"])
    # the verdict is cached per closure identity and weights version: no second probe
    assert fused.describe(bad_model, cost_fn, torch.device(DEV))[0] is None
    assert fused.describe(model_fn, cost_fn, torch.device(DEV))[0] is not None


def test_semantic_check_guards_dynamics_forward():
    """DynamicsModel.forward's fused path runs only after its normalisers pass the probe."""
    from mbrl_amd import fused
    p = ocem.synth_problem(4)
    module, model_fn, _, _ = build(p)
    module.to(DEV)                      # the module's own forward runs once the probe fails
    imp_norm, _ = _impostors()
    # every normaliser on device statistics (the module's own forward runs once the probe fails)
    kw = {}
    for k, f in model_fn.keywords.items():
        st = f.keywords["stats"]
        dev_stats = {n: {q: torch.as_tensor(v[q]).to(DEV) for q in ("mean", "std")} for n, v in st.items()}
        kw[k] = functools.partial(imp_norm if k == "normalize_action" else f.func, field_name=f.keywords["field_name"],
                                  stats=dev_stats)
    rng = np.random.default_rng(3)
    s = torch.from_numpy(rng.standard_normal((64, 24)).astype(np.float32)).to(DEV)
    a = torch.from_numpy(rng.uniform(-1, 1, (64, 6)).astype(np.float32)).to(DEV)
    with pytest.warns(UserWarning, match="normalisers"):
        with torch.no_grad():
            got = module(s, a, **kw)
    with torch.enable_grad():
        want = module(s, a, **kw).detach()
    assert torch.equal(got, want)
    with torch.no_grad():
        ok = model_fn(s, a)
    assert fused._PACKED.get(module) is not None
    assert np.allclose(ok.cpu().numpy(), ocem.dynamics_step(p["model"][0], p["norm"], s.cpu().numpy(), a.cpu().numpy()),
                       rtol=1e-5, atol=1e-5)


def test_cem_generic_path_matches_fused():
    """Opaque callables (generic path) and recognised closures (fused path) agree on the elite sets."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(2, N=512, H=10)
    _, model_fn, cost_fn, sample_action = build(p)
    kw = dict(num_candidates=512, num_iterations=3, seed=5, record=True)
    fused_res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 10, **kw)
    opaque_model = lambda s, a: model_fn(s, a)        # noqa: E731  (not introspectable)
    opaque_cost = lambda s, a: cost_fn(s, a)          # noqa: E731
    gen = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), opaque_model, opaque_cost, sample_action, 10, **kw)
    for it in range(3):
        assert rel_err(gen["returns"][it], fused_res["returns"][it].cpu().numpy()) < RTOL
        assert torch.equal(gen["elites"][it], fused_res["elites"][it])


# ------------------------------------------------------------------------------------------------ full sizes
@pytest.mark.parametrize("cid", [3, 4, 5, 6])
def test_full_size_plan_sampled_candidates(cid):
    """BASELINE configs at full N/H/E: every iteration's returns for 48 random candidates are
    recomputed by the oracle from the counter RNG (size-independent check), elites are exactly the
    stable top-K of the device returns, and the plan is deterministic across calls."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(cid)
    cfg = p["cfg"]
    N, H, a = cfg["N"], cfg["H"], cfg["a"]
    _, model_fn, cost_fn, sample_action = build(p)
    kw = dict(num_candidates=N, num_iterations=3, seed=p["rng_seed"], record=True)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H, **kw)
    res2 = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H, **kw)
    assert torch.equal(res["returns"], res2["returns"]) and torch.equal(res["mu"], res2["mu"])
    rng = np.random.default_rng(cid)
    mu = np.zeros((H, a), np.float32)
    sg = np.full((H, a), 0.5, np.float32)
    K = N // 10
    for it in range(3):
        rets = res["returns"][it].cpu().numpy()
        elites = res["elites"][it].cpu().numpy()
        assert np.array_equal(elites, ocem.select_elites(rets, K))
        idx = np.sort(rng.choice(N, size=48, replace=False))
        A = cem_actions(mu, sg, -1, 1, p["rng_seed"], it, idx)
        ref = ocem.ensemble_returns(ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A))
        assert rel_err(rets[idx], ref) < RTOL, f"iteration {it}"
        Ael = cem_actions(mu, sg, -1, 1, p["rng_seed"], it, elites)
        mu, sg = ocem.refit(mu, sg, np.ascontiguousarray(Ael.transpose(1, 0, 2)), 0.1)
    assert np.array_equal(res["mu"].cpu().numpy(), mu)
    assert np.array_equal(res["sigma"].cpu().numpy(), sg)


# ------------------------------------------------------------------------------------------------ full sizes vs the reference
FULL_CASES = [("config4_cem_full", 4), ("config5_cem_full", 5), ("config6_cem_full", 6)]


def elite_diff_at_ties(got, ref_elites, ref_returns, K, tie_rel):
    """Candidates in exactly one of the two elite sets, and whether every one of them has a reference
    return within tie_rel (relative to max(|r|, 1)) of the reference K-th order value -- i.e. a
    candidate the reference itself ranks inside fp32 rounding of the elite boundary."""
    diff = np.setxor1d(got, ref_elites)
    order = np.argsort(ref_returns, kind="stable")
    kth = float(ref_returns[order[K - 1]])
    near = np.abs(ref_returns[diff].astype(np.float64) - kth) <= tie_rel * max(abs(kth), 1.0)
    return diff, bool(np.all(near))


@pytest.mark.parametrize("name,cid", FULL_CASES, ids=[c[0] for c in FULL_CASES])
def test_full_size_iterations_against_reference_golden(golden, name, cid, capsys):
    """BASELINE configs 4 (walker N=16384 H=30) and 5 (humanoid N=32768 H=50 E=5) at full size against
    the reference's own _generate_trajectories (tests/golden/make_golden.py full), every iteration,
    teacher-forced on the reference's mu / sigma so that one boundary swap cannot cascade:
      * all N returns within 1e-5 relative (north_star);
      * the refit of the reference's elite set reproduces the reference's mu / sigma bit for bit;
      * the GPU elite set equals the reference's, except for candidates whose reference return lies
        within 4 ulp-scale units (5e-7 relative) of the reference's K-th value. At these sizes the
        reference's own K-boundary gaps are 0 (exact fp32 ties) to 1 ulp (the fixture's `gap`), so
        any two fp32 implementations with different GEMM summation orders can rank those candidates
        differently; the count of such swaps is printed.
    The free-running plan (no teacher forcing) is compared last, and its elite agreement is printed."""
    from mbrl_amd import CEMPlanner, fused
    g = golden(name)
    p = ocem.synth_problem(cid)
    assert ocem.weights_sha256(p["model"]) == str(g["weights_sha256"])
    N, H, K, I = int(g["N"]), int(g["H"]), int(g["K"]), int(g["I"])
    a = p["cfg"]["a"]
    prob = device_problem(p)
    s0 = torch.from_numpy(p["s0"]).to(DEV)
    mu = np.zeros((H, a), np.float32)
    sg = np.full((H, a), 0.5, np.float32)
    acts = torch.empty((H, N, a), dtype=torch.float32, device=DEV)
    lines = []
    for it in range(I):
        mu_d, sg_d = torch.from_numpy(mu).to(DEV), torch.from_numpy(sg).to(DEV)
        sp = fused.make_sampler(p["rng_seed"], it, mu_d, sg_d, -1.0, 1.0)
        costs = fused.rollout(prob, s0, N, H, sampler=sp, actions_out=acts)
        ret = torch.empty(N, dtype=torch.float32, device=DEV)
        el = fused.select(costs, K, returns_out=ret).cpu().numpy()
        err = rel_err(ret, g["returns"][it])
        assert err < RTOL, f"iteration {it}: max rel err {err}"
        diff, near = elite_diff_at_ties(el, g["elites"][it], g["returns"][it], K, 5e-7)
        assert near, f"iteration {it}: elites differ away from the K boundary: {diff[:10]}"
        mo, so = torch.empty_like(mu_d), torch.empty_like(sg_d)
        fused.refit(sp, H, a, torch.from_numpy(g["elites"][it].astype(np.int64)).to(DEV), 0.1, mo, so)
        assert np.array_equal(mo.cpu().numpy(), g["mu"][it]) and np.array_equal(so.cpu().numpy(), g["sigma"][it])
        lines.append(f"it {it}: max rel err {err:.2e}, ref K-gap {float(g['gap'][it]):.2e}, "
                     f"boundary swaps {len(diff) // 2}")
        mu, sg = g["mu"][it], g["sigma"][it]
    _, model_fn, cost_fn, sample_action = build(p)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H,
                                   num_candidates=N, num_iterations=I, seed=p["rng_seed"], record=True)
    fr = free_running_against_reference(prob, s0, p, g, res, acts)
    with capsys.disabled():
        print(f"\n{name}: " + "; ".join(lines))
        for ln in fr["lines"]:
            print(f"  free-running {ln}")
    if cid in (4, 6):
        # walker, and the cheetah reward head: the reference's K-boundary gaps exceed the GEMM-order
        # error at every iteration, so the free-running plan is the reference's plan bit for bit
        assert fr["swaps"] == [0] * I
        assert np.array_equal(res["mu"].cpu().numpy(), g["mu"][-1])
        assert np.array_equal(res["sigma"].cpu().numpy(), g["sigma"][-1])
        assert np.array_equal(res["actions"].numpy(), g["final_actions"])


def free_running_against_reference(prob, s0, p, g, res, acts):
    """The free-running plan (no teacher forcing) against the reference's, with the drift that
    boundary swaps can cause derived and ASSERTED (the one relaxation of bit-exact
    elites). Iteration i starts from the plan's own mu^G, sigma^G and the reference's mu^R, sigma^R,
    with measured drifts Dmu = |mu^G - mu^R| and Dsigma (per element [t, j]):
      * proposals share their normal draws eps (same Philox counters), and clip is 1-Lipschitz, so
        |a^G_n - a^R_n| <= Dmu + Dsigma |eps_n|;
      * elites: both sets are exact stable top-K, so with delta = max_n |r^G_n - r^R_n| every
        candidate in exactly one set has a reference return within 2 delta (+ 5e-7 relative ties)
        of the reference's K-th return -- asserted; s = |G xor R| / 2 swaps;
      * elite mean over K: |Dmean| <= Dmu + Dsigma e + s w / K, e = the mean |eps| over the
        candidates in both sets, w = the spread (max - min) of the swapped candidates' actions (a^G for
        those only in the GPU set, a^R for those only in the reference's: s ins and s outs pair up,
        each pair's difference is at most w; w <= hi - lo); mu' = alpha mu + (1 - alpha) mean, so
        |Dmu'| <= alpha Dmu + (1 - alpha) Dmean;
      * population variance (E a^2 - mean^2, |a| <= M = max(|lo|, |hi|)):
        |Dvar| <= 2 M (Dmu + Dsigma e) + s w2 / K + 2 M Dmean (w2: the spread of the swapped candidates'
        a^2, <= M^2); sigma'^2 = alpha sigma^2 + (1 - alpha) var, so
        X := |D sigma'^2| <= alpha |D sigma^2| + (1 - alpha) Dvar, and |Dsigma'| <= min(sqrt(X), X / (sigma'^G + sigma'^R));
      * fp32 rounding: nothing when every input is bit-identical (then so are the outputs), else
        2 (32 + K / 32 + 8) ulp(M) for the chunked refit sums (and 1e-6 on w for the fp64 recompute
        of the reference's proposals).
    Each iteration's measured drift is asserted against the bound from its measured inputs, and the
    final actions clip(mu_I) against the last iteration's (|Daction| <= |Dmu_I|, clip is 1-Lipschitz).
    The same recurrences fed with the swap counts alone (w = hi - lo, w2 = M^2) give the a-priori bound
    compounded over the I iterations, printed beside it."""
    from mbrl_amd import fused
    N, H, K, I = int(g["N"]), int(g["H"]), int(g["K"]), int(g["I"])
    a = p["cfg"]["a"]
    alpha, lo, hi = 0.1, -1.0, 1.0
    M = max(abs(lo), abs(hi))
    ulp = float(np.finfo(np.float32).eps) * M
    zero = torch.zeros((H, a), dtype=torch.float32, device=DEV)
    one = torch.ones((H, a), dtype=torch.float32, device=DEV)
    mu = np.zeros((H, a), np.float32)
    sg = np.full((H, a), 0.5, np.float32)
    mu_r, sg_r = mu.astype(np.float64), sg.astype(np.float64)     # the reference's, entering iteration it
    c_mu, c_sq, c_sg = np.zeros((H, a)), np.zeros((H, a)), np.zeros((H, a))   # a-priori (swaps only)
    swaps, lines = [], []

    def step_bound(dmu, dsg, dsq, e, s, any_diff, sg_new_sum, w=hi - lo, w2=M * M):
        rnd = 2 * (32 + K / 32 + 8) * ulp if any_diff else 0.0
        dmean = dmu + dsg * e + s * w / K
        dvar = 2 * M * (dmu + dsg * e) + s * w2 / K + 2 * M * dmean
        b_mu = alpha * dmu + (1 - alpha) * dmean + rnd
        x = alpha * dsq + (1 - alpha) * dvar + rnd
        b_sg = np.minimum(np.sqrt(x), x / sg_new_sum) + rnd
        return b_mu, x, b_sg

    for it in range(I):
        mu_d, sg_d = torch.from_numpy(mu).to(DEV), torch.from_numpy(sg).to(DEV)   # the sampler holds their pointers
        sp = fused.make_sampler(p["rng_seed"], it, mu_d, sg_d, lo, hi)
        costs = fused.rollout(prob, s0, N, H, sampler=sp, actions_out=acts)
        ret = torch.empty(N, dtype=torch.float32, device=DEV)
        el = fused.select(costs, K, returns_out=ret).cpu().numpy()
        assert np.array_equal(el, res["elites"][it].cpu().numpy()), "step-by-step plan != CEMPlanner plan"
        mo = torch.empty((H, a), dtype=torch.float32, device=DEV)
        so = torch.empty((H, a), dtype=torch.float32, device=DEV)
        fused.refit(sp, H, a, torch.from_numpy(el).to(DEV), alpha, mo, so)
        ref_el = g["elites"][it].astype(np.int64)
        rG, rR = ret.cpu().numpy().astype(np.float64), g["returns"][it].astype(np.float64)
        delta = float(np.max(np.abs(rG - rR)))
        kth = float(rR[np.argsort(g["returns"][it], kind="stable")[K - 1]])
        diff = np.setxor1d(el, ref_el)
        assert np.all(np.abs(rR[diff] - kth) <= 2 * delta + 5e-7 * max(abs(kth), 1.0)), \
            f"iteration {it}: elite swaps away from the K boundary"
        s = len(diff) // 2
        swaps.append(s)
        only_g = torch.from_numpy(np.setdiff1d(el, ref_el)).to(DEV)
        only_r = torch.from_numpy(np.setdiff1d(ref_el, el)).to(DEV)
        a_swap = [acts.index_select(1, only_g).double().cpu().numpy()]          # a^G of the GPU-only elites
        common = torch.from_numpy(np.intersect1d(el, ref_el)).to(DEV)
        fused.sample_actions(fused.make_sampler(p["rng_seed"], it, zero, one, -3.0e38, 3.0e38), H, a, N, 0, acts)
        e = acts.index_select(1, common).abs().double().mean(dim=1).cpu().numpy()      # [H, a]
        eps_r = acts.index_select(1, only_r).double().cpu().numpy()
        a_swap.append(np.clip(mu_r[:, None, :] + sg_r[:, None, :] * eps_r, lo, hi))  # a^R of the reference-only
        if s:
            sw = np.concatenate(a_swap, axis=1)                                       # [H, 2s, a]
            w = sw.max(1) - sw.min(1) + 1e-6
            w2 = (sw ** 2).max(1) - (sw ** 2).min(1) + 1e-6
        else:
            w, w2 = np.zeros((H, a)), np.zeros((H, a))
        mu_g, sg_g = mu.astype(np.float64), sg.astype(np.float64)
        dmu, dsg, dsq = np.abs(mu_g - mu_r), np.abs(sg_g - sg_r), np.abs(sg_g ** 2 - sg_r ** 2)
        mu, sg = mo.cpu().numpy(), so.cpu().numpy()
        mu_r, sg_r = g["mu"][it].astype(np.float64), g["sigma"][it].astype(np.float64)
        sg_sum = sg.astype(np.float64) + sg_r
        b_mu, _, b_sg = step_bound(dmu, dsg, dsq, e, s, bool(dmu.any() or dsg.any() or s), sg_sum, w, w2)
        got_mu, got_sg = np.abs(mu - mu_r), np.abs(sg - sg_r)
        assert np.all(got_mu <= b_mu), f"iteration {it}: |Dmu| {got_mu.max():.3e} above its bound"
        assert np.all(got_sg <= b_sg), f"iteration {it}: |Dsigma| {got_sg.max():.3e} above its bound"
        c_mu, c_sq, c_sg = step_bound(c_mu, c_sg, c_sq, e, s, bool(c_mu.any() or c_sg.any() or s), sg_sum)
        lines.append(f"it {it}: swaps {s}, max|r^G - r^R| {delta:.2e}, |Dmu| {got_mu.max():.2e} "
                     f"(bound {b_mu.max():.2e}), |Dsigma| {got_sg.max():.2e} (bound {b_sg.max():.2e})")
    assert np.array_equal(mu, res["mu"].cpu().numpy()) and np.array_equal(sg, res["sigma"].cpu().numpy())
    d_act = np.abs(res["actions"].numpy().astype(np.float64) - g["final_actions"])
    assert np.all(d_act <= b_mu), f"final actions drift {d_act.max():.3e} beyond the last iteration's bound"
    assert np.all(d_act <= c_mu), f"final actions drift {d_act.max():.3e} beyond the a-priori bound"
    lines.append(f"final: max|Daction| {d_act.max():.3e} <= bound {b_mu.max():.3e} (last iteration, measured "
                 f"inputs; {b_mu.max() / max(d_act.max(), 1e-30):.1f}x the drift); a-priori from swaps {swaps} "
                 f"alone {c_mu.max():.3e}")
    return dict(swaps=swaps, lines=lines, final_bound=float(b_mu.max()), final_drift=float(d_act.max()))


# ------------------------------------------------------------------------------------------------ trajectory / sharding
@pytest.mark.parametrize("cid,H,over", [(2, 20, {}), (3, 30, {}), (4, 7, {}), (5, 50, {}), (3, 9, dict(W=50, L=2)),
                                        (3, 6, dict(W=50, L=4)), (2, 11, dict(W=100, L=3)), (6, 8, dict(W=200, L=2)),
                                        (5, 5, dict(W=128, L=4)), (2, 4, dict(W=64, L=1))])
def test_trajectory_states_match_oracle(cid, H, over):
    """mbrl_trajectory vs the oracle's N=1 rollout, per member and member mean: the register-resident
    kernel (Wpad <= 256: cartpole, the reference's default widths 50 / 200, ensembles) and the
    cooperative kernel (Wpad 512)."""
    from mbrl_amd import fused
    p = ocem.synth_problem(cid, N=1, H=H, **over)
    a, s, E = p["cfg"]["a"], p["cfg"]["s"], p["cfg"]["E"]
    acts = np.random.default_rng(cid).uniform(-1, 1, size=(H, a)).astype(np.float32)
    prob = device_problem(p)
    members = torch.empty((E, H, s), dtype=torch.float32, device=DEV)
    st = fused.trajectory(prob, torch.from_numpy(p["s0"]).to(DEV), torch.from_numpy(acts).to(DEV), H,
                          member_states=members)
    torch.cuda.synchronize()
    _, ref = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], acts[:, None, :], store_states=True)
    assert np.allclose(members.cpu().numpy(), ref[:, :, 0, :], rtol=1e-4, atol=1e-4)
    assert np.allclose(st.cpu().numpy(), np.mean(ref[:, :, 0, :], axis=0, dtype=np.float32), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cid,H", [(3, 12), (5, 7)])
def test_trajectory_fallback_when_the_cooperative_kernel_gives_up(cid, H):
    """MBRL_OPT_DEBUG_TRAJ_ABORT makes the cooperative kernel behave as a timed-out hand-off (it sets
    the status word and exits); the gated single-workgroup kernel behind it must then produce the states."""
    from mbrl_amd import _lib, fused
    with _lib.option("debug_traj_abort", 1):
        _trajectory_fallback(fused, cid, H)


def _trajectory_fallback(fused, cid, H):
    p = ocem.synth_problem(cid, N=1, H=H)
    a, s, E = p["cfg"]["a"], p["cfg"]["s"], p["cfg"]["E"]
    acts = np.random.default_rng(7 + cid).uniform(-1, 1, size=(H, a)).astype(np.float32)
    prob = device_problem(p)
    members = torch.full((E, H, s), float("nan"), dtype=torch.float32, device=DEV)
    fused.trajectory(prob, torch.from_numpy(p["s0"]).to(DEV), torch.from_numpy(acts).to(DEV), H,
                     member_states=members)
    torch.cuda.synchronize()
    _, ref = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], acts[:, None, :], store_states=True)
    assert np.allclose(members.cpu().numpy(), ref[:, :, 0, :], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cid,N,H,world", [(3, 2048, 10, 2), (5, 512, 6, 4), (4, 16384, 30, 4), (4, 16384, 30, 8),
                                           (2, 40000, 4, 2)])
def test_sharded_protocol_with_fused_ops_matches_single_gpu_plan(cid, N, H, world):
    """The multi-GPU protocol with its math on the HIP extension: every rank's shard computed here on
    one GPU (the all-gather stitches the shards' rollouts), against the single-call mbrl_cem_plan.
    Elites, mu and sigma must be bit-identical (no floating-point reduction crosses ranks). Walker
    N=16384 (BASELINE configs[3]) is the case where the tile heights differ: one GPU runs 32-candidate
    tiles, a 4-way shard 16-candidate tiles, an 8-way shard 8-candidate tiles; all three close the
    output layer in the same canonical order (rollout.hip mma_out). N=40000 is past the fused update
    (mbrl_cem_update returns MBRL_EUNSUPPORTED): the ranks fall back to select + refit + draw."""
    from mbrl_amd import CEMPlanner, fused, planners
    p = ocem.synth_problem(cid, N=N, H=H)
    _, model_fn, cost_fn, sample_action = build(p)
    I, K = 3, N // 10
    single = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H,
                                      num_candidates=N, num_elites=K, num_iterations=I, seed=p["rng_seed"],
                                      record=True, return_device=True)
    prob = device_problem(p)
    s0 = torch.from_numpy(p["s0"]).to(DEV)
    st = dict(N=N, K=K, H=H, I=I, E=p["cfg"]["E"], a=p["cfg"]["a"], alpha=0.1, lo=-1.0, hi=1.0, init_std=0.5,
              seed=p["rng_seed"], record=True, events=None)

    class AllShardsOps(planners._FusedShardOps):
        def rollout(self, it, mu, sigma, n_offset, n_local, costs_out, events=None):
            self._it_args = (it, mu, sigma)
            super().rollout(it, mu, sigma, n_offset, n_local, costs_out, events)

        def all_gather(self, out_flat, local):
            it, mu, sigma = self._it_args
            E, Nl = local.shape
            view = out_flat.view(world, E, Nl)
            for r in range(world):
                super().rollout(it, mu, sigma, r * Nl, Nl, view[r])

    res = planners.cem_sharded_protocol(AllShardsOps(prob, s0, st), st, world, 0)
    assert torch.equal(res["elites"], single["elites"])
    assert torch.equal(res["returns"], single["returns"])
    assert torch.equal(res["mu"], single["mu"]) and torch.equal(res["sigma"], single["sigma"])
    assert torch.allclose(res["states"], single["states"], rtol=1e-5, atol=1e-5)
    assert fused is not None


def test_random_shooting_with_reward_model():
    """RewardAgent wiring through RandomShootingPlanner (agents.py:336-362 + planners.py:140-187): the
    fused path rolls out with the reward head as the cost and takes the first argmin."""
    from mbrl_amd import RandomShootingPlanner
    p = ocem.synth_problem(6, N=700, H=8)
    _, model_fn, cost_fn, sample_action = build(p)
    np.random.seed(3)
    states, actions = RandomShootingPlanner.plan(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 8,
                                                 num_trajectories=700)
    np.random.seed(3)
    flat = sample_action(batch_size=700 * 8).numpy()
    A = flat.reshape(8, 700, 6)
    costs, st = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A, store_states=True)
    idx = ocem.rs_argmin(costs[0])
    assert np.array_equal(actions.numpy(), A[:, idx])
    assert np.allclose(states.numpy(), st[0, :, idx], rtol=1e-4, atol=1e-4)


def test_mpc_policy_drives_the_planner_like_the_reference_agent():
    """agents.py:29-56: plan per step, act with actions[0], reset at timestep 0."""
    from mbrl_amd import CEMPlanner, MPCPolicy
    p = ocem.synth_problem(3, N=512, H=6)
    _, model_fn, cost_fn, sample_action = build(p)
    pol = MPCPolicy(model_fn, cost_fn, CEMPlanner, sample_action, 6, num_candidates=512, seed=p["rng_seed"])
    obs = torch.from_numpy(p["s0"])
    a0 = pol.get_action({"timestep": 0, "observation": obs})
    ref = ocem.cem_plan(p, N=512, H=6)
    assert a0.shape == (6,) and np.array_equal(a0.numpy(), ref["final_actions"][0])
    assert pol.last_trajectory[0].shape == (6, 17)
    a1 = pol.get_action({"timestep": 1, "observation": pol.last_trajectory[0][0]})
    assert a1.shape == (6,) and torch.isfinite(a1).all()


@pytest.mark.parametrize("cid,W,L", [(3, 50, 2), (6, 200, 2), (2, 100, 1), (3, 200, 3)])
def test_reference_default_widths(cid, W, L):
    """The reference's default widths (Model hidden_units=50, ModelWithReward 200; models.py:97,126)
    are not multiples of 64: the packed stream zero-pads them. CEM plan vs the oracle, elites exact."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(cid, N=640, H=7, W=W, L=L)
    _, model_fn, cost_fn, sample_action = build(p)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 7,
                                   num_candidates=640, num_iterations=3, seed=p["rng_seed"], record=True)
    ref = ocem.cem_plan(p, N=640, H=7, num_iterations=3)
    for it in range(3):
        assert rel_err(res["returns"][it], ref["returns"][it]) < RTOL, it
        assert np.array_equal(res["elites"][it].cpu().numpy(), ref["elites"][it]), it
    assert np.array_equal(res["mu"].cpu().numpy(), ref["mu"][-1])
    assert np.allclose(res["states"].numpy(), ref["final_states"], rtol=1e-4, atol=1e-4)


def _sharded_worker(rank, world, init_file, out_dir):
    import os
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "mujoco-mbrl_amd")]
    import torch.distributed as dist
    from mbrl_amd import CEMPlanner
    from oracle import cem as oc
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        p = oc.synth_problem(3, N=1024, H=8)
        _, model_fn, cost_fn, sample_action = build(p)
        res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 8,
                                       num_candidates=1024, num_iterations=3, seed=p["rng_seed"], record=True,
                                       distributed=True, device="cuda:0")
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), mu=res["mu"].cpu().numpy(), sigma=res["sigma"].cpu().numpy(),
                 elites=res["elites"].cpu().numpy(), states=res["states"].numpy(), actions=res["actions"].numpy())
    finally:
        dist.destroy_process_group()


def test_sharded_plan_two_processes_on_one_gpu():
    """The real multi-process sharded path (CEMPlanner(distributed=True), fused ops, a process group)
    with two ranks sharing this GPU over gloo: bit-identical to the single-process plan."""
    import tempfile
    import torch.multiprocessing as mp
    from mbrl_amd import CEMPlanner
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_sharded_worker, args=(2, os.path.join(d, "pg"), d), nprocs=2, join=True,
                           start_method="spawn")
        got = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(2)]
    p = ocem.synth_problem(3, N=1024, H=8)
    _, model_fn, cost_fn, sample_action = build(p)
    ref = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 8,
                                   num_candidates=1024, num_iterations=3, seed=p["rng_seed"], record=True)
    for g in got:
        assert np.array_equal(g["elites"], ref["elites"].cpu().numpy())
        assert np.array_equal(g["mu"], ref["mu"].cpu().numpy()) and np.array_equal(g["sigma"], ref["sigma"].cpu().numpy())
        assert np.array_equal(g["actions"], ref["actions"].numpy())
        assert np.allclose(g["states"], ref["states"].numpy(), rtol=1e-5, atol=1e-5)


RCCL_CASES = [(3, dict(N=1024, H=8)), (5, dict(N=256, H=6))]


def _rccl_worker(rank, world, init_file, out_dir):
    import os
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "mujoco-mbrl_amd")]
    import torch.distributed as dist
    from mbrl_amd import CEMPlanner, fused, planners
    from oracle import cem as oc
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        assert dist.get_backend() == "nccl"
        dev = torch.device("cuda", 0)
        for cid, over in RCCL_CASES:
            p = oc.synth_problem(cid, **over)
            _, model_fn, cost_fn, sample_action = build(p)
            md = fused.describe_model(model_fn)
            prob = fused.device_problem(md, fused.describe_cost(cost_fn, md["s"], md), dev)
            st = CEMPlanner._settings(sample_action, over["H"], dict(num_candidates=over["N"], num_iterations=3,
                                                                     seed=p["rng_seed"], record=True))
            s0 = torch.from_numpy(p["s0"]).to(dev)
            for native in (True, False):
                # native: mbrl_cem_plan_sharded (ncclAllGather on the plan's stream, the library's own
                # communicator); else cem_sharded_protocol (torch.distributed all_gather_into_tensor)
                planners.SHARDED_NATIVE = native
                res = planners._cem_fused_sharded(prob, s0, st, world)
                np.savez(os.path.join(out_dir, f"c{cid}_n{int(native)}_r{rank}.npz"), mu=res["mu"].cpu().numpy(),
                         sigma=res["sigma"].cpu().numpy(), elites=torch.stack(list(res["elites"])).cpu().numpy(),
                         returns=torch.stack(list(res["returns"])).cpu().numpy(),
                         costs=torch.stack(list(res["costs"])).cpu().numpy(),
                         actions=res["actions"].cpu().numpy(), states=res["states"].cpu().numpy())
        # a launch failure after the first collective (injected at iteration 1): the rank keeps joining
        # the remaining all-gathers and reports the error at the end, so the communicator stays in step
        # -- the next plan over the same communicator runs and equals the first one
        cid, over = RCCL_CASES[0]
        p = oc.synth_problem(cid, **over)
        _, model_fn, cost_fn, sample_action = build(p)
        md = fused.describe_model(model_fn)
        prob = fused.device_problem(md, fused.describe_cost(cost_fn, md["s"], md), dev)
        st = CEMPlanner._settings(sample_action, over["H"], dict(num_candidates=over["N"], num_iterations=3,
                                                                 seed=p["rng_seed"], record=True))
        s0 = torch.from_numpy(p["s0"]).to(dev)
        planners.SHARDED_NATIVE = True
        with planners._lib.option("debug_shard_fail", 2):
            try:
                planners._cem_fused_sharded(prob, s0, st, world)
                raised = ""
            except RuntimeError as e:
                raised = str(e)
        torch.cuda.synchronize()
        again = planners._cem_fused_sharded(prob, s0, st, world)
        np.savez(os.path.join(out_dir, f"c{cid}_nagain_r{rank}.npz"), mu=again["mu"].cpu().numpy(),
                 elites=torch.stack(list(again["elites"])).cpu().numpy(), raised=np.array(raised))
        # a communicator that cannot be created (simulated: mbrl_comm_init fails) sends every rank to
        # the protocol, with a warning, instead of failing the plan
        real_load = planners._lib.load

        class _NoComm:
            def __init__(self, lib):
                self._lib = lib

            def __getattr__(self, name):
                return getattr(self._lib, name)

            def mbrl_comm_init(self, *args):
                return -3

            def mbrl_last_error(self):
                return b"simulated"

        planners._COMMS.clear()
        planners.SHARDED_NATIVE = True
        planners._lib.load = lambda: _NoComm(real_load())
        try:
            import warnings
            cid, over = RCCL_CASES[0]
            p = oc.synth_problem(cid, **over)
            _, model_fn, cost_fn, sample_action = build(p)
            md = fused.describe_model(model_fn)
            prob = fused.device_problem(md, fused.describe_cost(cost_fn, md["s"], md), dev)
            st = CEMPlanner._settings(sample_action, over["H"], dict(num_candidates=over["N"], num_iterations=3,
                                                                     seed=p["rng_seed"], record=True))
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                res = planners._cem_fused_sharded(prob, torch.from_numpy(p["s0"]).to(dev), st, world)
            assert any("RCCL communicator unavailable" in str(x.message) for x in w)
            np.savez(os.path.join(out_dir, f"c{cid}_nfail_r{rank}.npz"), mu=res["mu"].cpu().numpy(),
                     elites=torch.stack(list(res["elites"])).cpu().numpy())
        finally:
            planners._lib.load = real_load
            planners._COMMS.clear()
    finally:
        planners.SHARDED_NATIVE = True
        dist.destroy_process_group()


def test_sharded_plan_over_rccl():
    """The multi-GPU plan over RCCL (torch.distributed backend "nccl") with a one-rank process group
    on this GPU -- RCCL refuses two ranks on one device, so the 2-8 rank runs are the driver's 8-GPU
    node's: both the one-call C path (mbrl_cem_plan_sharded: the library's RCCL communicator, the
    all-gather a step on the plan's stream, the ensemble's rank-major cost permutation) and the
    per-iteration protocol (cem_sharded_protocol over all_gather_into_tensor) are bit-identical to the
    single-process plan, for a single model and a 5-member ensemble."""
    import tempfile
    import torch.multiprocessing as mp
    from mbrl_amd import CEMPlanner
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_rccl_worker, args=(1, os.path.join(d, "pg"), d), nprocs=1, join=True,
                           start_method="spawn")
        got = {(cid, n): dict(np.load(os.path.join(d, f"c{cid}_n{n}_r0.npz"))) for cid, _ in RCCL_CASES for n in (0, 1)}
        fail = dict(np.load(os.path.join(d, f"c{RCCL_CASES[0][0]}_nfail_r0.npz")))
        again = dict(np.load(os.path.join(d, f"c{RCCL_CASES[0][0]}_nagain_r0.npz")))
    assert np.array_equal(fail["mu"], got[(RCCL_CASES[0][0], 0)]["mu"])
    assert np.array_equal(fail["elites"], got[(RCCL_CASES[0][0], 0)]["elites"])
    # the injected in-loop failure was reported, and the same communicator then ran the next plan exactly
    assert "injected launch failure at iteration 1" in str(again["raised"]), str(again["raised"])
    assert "still joined every all-gather" in str(again["raised"])
    assert np.array_equal(again["mu"], got[(RCCL_CASES[0][0], 1)]["mu"])
    assert np.array_equal(again["elites"], got[(RCCL_CASES[0][0], 1)]["elites"])
    for cid, over in RCCL_CASES:
        p = ocem.synth_problem(cid, **over)
        _, model_fn, cost_fn, sample_action = build(p)
        ref = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, over["H"],
                                       num_candidates=over["N"], num_iterations=3, seed=p["rng_seed"], record=True)
        for n in (0, 1):
            g = got[(cid, n)]
            assert np.array_equal(g["elites"], ref["elites"].cpu().numpy()), (cid, n)
            assert np.array_equal(g["returns"], ref["returns"].cpu().numpy()), (cid, n)
            assert np.array_equal(g["costs"], ref["costs"].cpu().numpy()), (cid, n)
            assert np.array_equal(g["mu"], ref["mu"].cpu().numpy()) and np.array_equal(g["sigma"], ref["sigma"].cpu().numpy())
            assert np.array_equal(g["actions"], ref["actions"].numpy()) and np.array_equal(g["states"], ref["states"].numpy())


@pytest.mark.parametrize("cid,N,H,B", [(2, 1024, 20, 4), (3, 512, 6, 3), (6, 256, 5, 2), (5, 128, 4, 2)])
def test_batched_plans_match_per_problem_oracle(cid, N, H, B):
    """mbrl_cem_plan_batch: problem b == a single CEM plan whose proposals are candidates
    [b*N, (b+1)*N) of the Philox stream; elites, mu and the final actions bit-exact per problem."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(cid, N=N, H=H)
    _, model_fn, cost_fn, sample_action = build(p)
    s = p["cfg"]["s"]
    rng = np.random.default_rng(cid)
    S0 = np.stack([p["s0"]] + [rng.standard_normal(s).astype(np.float32) for _ in range(B - 1)])
    states, actions = CEMPlanner.plan_batch(torch.from_numpy(S0), model_fn, cost_fn, sample_action, H,
                                            num_candidates=N, num_iterations=3, seed=p["rng_seed"])
    assert states.shape == (B, H, s) and actions.shape == (B, H, p["cfg"]["a"])
    a, K = p["cfg"]["a"], N // 10
    for b in range(B):
        mu = np.zeros((H, a), np.float32)
        sg = np.full((H, a), 0.5, np.float32)
        idx = np.arange(b * N, (b + 1) * N)
        for it in range(3):
            A = cem_actions(mu, sg, -1.0, 1.0, p["rng_seed"], it, idx)
            r = ocem.ensemble_returns(ocem.rollout(p["model"], p["norm"], p["cost"], S0[b], A))
            el = ocem.select_elites(r, K)
            mu, sg = ocem.refit(mu, sg, np.ascontiguousarray(A[:, el].transpose(1, 0, 2)), 0.1)
        fa = np.clip(mu, -1.0, 1.0).astype(np.float32)
        assert np.array_equal(actions[b].numpy(), fa), b
        _, st = ocem.rollout(p["model"], p["norm"], p["cost"], S0[b], fa[:, None, :], store_states=True)
        assert np.allclose(states[b].numpy(), np.mean(st[:, :, 0, :], axis=0), rtol=1e-4, atol=1e-4), b


@pytest.mark.parametrize("cid,N,H,K,I", [(3, 1, 1, 1, 1), (3, 17, 3, 17, 2), (2, 33, 4, 5, 3), (5, 9, 2, 2, 2)])
def test_cem_plan_edge_sizes_against_oracle(cid, N, H, K, I):
    """Degenerate plans: one candidate, every candidate an elite, sizes off the 8/16 tile grid,
    ensembles with a handful of candidates -- elites, mu, sigma and the final actions exactly as
    the oracle's, returns within 1e-5."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(cid, N=N, H=H)
    _, model_fn, cost_fn, sample_action = build(p)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H, num_candidates=N,
                                   num_elites=K, num_iterations=I, seed=p["rng_seed"], record=True)
    ref = ocem.cem_plan(p, N=N, H=H, K=K, num_iterations=I)
    for it in range(I):
        assert rel_err(res["returns"][it], ref["returns"][it]) < RTOL
        assert np.array_equal(res["elites"][it].cpu().numpy(), ref["elites"][it])
    assert np.array_equal(res["mu"].cpu().numpy(), ref["mu"][-1])
    assert np.array_equal(res["sigma"].cpu().numpy(), ref["sigma"][-1])
    assert np.array_equal(res["actions"].numpy(), ref["final_actions"])


@pytest.mark.parametrize("cid,over", [(2, {}), (3, dict(N=512, H=8)), (5, dict(N=256, H=6)), (6, dict(N=256, H=5))])
def test_staged_host_plan_equals_device_plan(cid, over):
    """plan() with a host initial state and host results runs mbrl_cem_plan on mapped pinned staging
    (planners._cem_plan_host: the first launch reads s0 from host memory, the last ones write the
    results there): bit-identical to the device-buffer path (record=True / return_device=True / a
    device initial state), for single models, ensembles (member-mean states) and reward heads."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(cid, **over)
    _, model_fn, cost_fn, sample_action = build(p)
    H, N = p["cfg"]["H"], p["cfg"]["N"]
    kw = dict(num_candidates=N, num_iterations=3, seed=p["rng_seed"])
    s0 = torch.from_numpy(p["s0"])
    st_h, act_h = CEMPlanner.plan(s0, model_fn, cost_fn, sample_action, H, **kw)
    assert not st_h.is_cuda and not act_h.is_cuda
    ref = CEMPlanner.plan_detailed(s0, model_fn, cost_fn, sample_action, H, record=True, **kw)
    st_d, act_d = CEMPlanner.plan(s0.to(DEV), model_fn, cost_fn, sample_action, H, return_device=True, **kw)
    for st, act in ((ref["states"], ref["actions"]), (st_d.cpu(), act_d.cpu())):
        assert torch.equal(st_h, st) and torch.equal(act_h, act)
    st2, act2 = CEMPlanner.plan(s0.double(), model_fn, cost_fn, sample_action, H, **kw)   # dtype conversion
    assert torch.equal(st2, st_h) and torch.equal(act2, act_h)
