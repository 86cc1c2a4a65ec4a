"""GPU parity of the split-operand rollouts F16X3 and F16X6 (fp32 emulated on the f16 matrix cores;
include/mbrl_cem.h, MBRL_PRECISION_F16X3 / _F16X6) against the CPU oracle and the reference's golden vectors, with the same
bars as the exact-fp32 path: elite index sets, mu and sigma bit-exact; returns within 1e-5
relative (BASELINE.json north_star) to max(|ref|, 1). Also the fp32 redo of operands outside the
split range, which must reproduce the F32 kernel bit for bit."""
import numpy as np
import pytest
import torch

from oracle import cem as ocem
from oracle.philox import cem_actions

from test_gpu_parity import CEM_CASES, DEV, RTOL, build, rel_err

pytestmark = pytest.mark.gpu


SPLITS = ["f16x3", "f16x6"]


def problems(p, precision="f16x3"):
    from mbrl_amd import _lib, fused
    _, model_fn, cost_fn, _ = build(p)
    md = fused.describe_model(model_fn)
    cd = fused.describe_cost(cost_fn, md["s"], md)
    dev = torch.device(DEV)
    return (fused.device_problem(md, cd, dev, _lib.MBRL_PRECISION_F32),
            fused.device_problem(md, cd, dev, _lib.precision_code(precision)))


@pytest.mark.parametrize("cid,over", [(2, dict(N=1000, H=20)), (3, dict(N=300, H=30)), (4, dict(N=200, H=7)),
                                      (5, dict(N=40, H=6)), (3, dict(N=17, H=2)), (3, dict(N=4096, H=30)),
                                      (4, dict(N=8200, H=5))])
@pytest.mark.parametrize("precision", SPLITS)
def test_f16x3_rollout_costs_and_states(cid, over, precision):
    from mbrl_amd import fused
    p = ocem.synth_problem(cid, **over)
    N, H, a, s, E = over["N"], over["H"], p["cfg"]["a"], p["cfg"]["s"], p["cfg"]["E"]
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 11, 0, np.arange(N))
    ref_costs, ref_states = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A, store_states=True)
    _, prob = problems(p, precision)
    states = torch.empty((E, H, N, s), dtype=torch.float32, device=DEV)
    costs = fused.rollout(prob, torch.from_numpy(p["s0"]).to(DEV), N, H, actions=torch.from_numpy(A).to(DEV),
                          states_out=states)
    torch.cuda.synchronize()
    err = rel_err(costs, ref_costs)
    print(f"config {cid} N={N} H={H}: {precision} return max rel err {err:.3e}")
    assert err < RTOL
    assert np.allclose(states.cpu().numpy(), ref_states, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("name,cid,over", CEM_CASES, ids=[c[0] for c in CEM_CASES])
@pytest.mark.parametrize("precision", SPLITS)
def test_f16x3_cem_plan_against_reference_golden(golden, name, cid, over, precision):
    """The fixtures of test_cem_plan_against_reference_golden through precision='f16x3' (config 6,
    the reward-head model, runs the F32 kernel and must match as well)."""
    from mbrl_amd import CEMPlanner
    g = golden(name)
    p = ocem.synth_problem(cid, **over)
    _, model_fn, cost_fn, sample_action = build(p)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, int(g["H"]),
                                   num_candidates=int(g["N"]), num_elites=int(g["K"]),
                                   num_iterations=int(g["I"]), alpha=float(g["alpha"]), seed=p["rng_seed"],
                                   record=True, precision=precision)
    for it in range(int(g["I"])):
        assert rel_err(res["returns"][it], g["returns"][it]) < RTOL, f"iteration {it}"
        assert np.array_equal(res["elites"][it].cpu().numpy(), g["elites"][it]), f"iteration {it}"
    assert np.array_equal(res["mu"].cpu().numpy(), g["mu"][-1])
    assert np.array_equal(res["sigma"].cpu().numpy(), g["sigma"][-1])
    assert np.array_equal(res["actions"].numpy(), g["final_actions"])
    assert np.allclose(res["states"].numpy(), g["final_states"], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("cid", [3, 4])
@pytest.mark.parametrize("precision", SPLITS)
def test_f16x3_full_size_plan_sampled_candidates(cid, precision):
    """Full BASELINE sizes: sampled candidates' returns against the oracle, exact stable top-K of the
    device returns, exact refit, determinism."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(cid)
    cfg = p["cfg"]
    N, H, a = cfg["N"], cfg["H"], cfg["a"]
    _, model_fn, cost_fn, sample_action = build(p)
    kw = dict(num_candidates=N, num_iterations=3, seed=p["rng_seed"], record=True, precision=precision)
    res = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H, **kw)
    res2 = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H, **kw)
    assert torch.equal(res["returns"], res2["returns"]) and torch.equal(res["mu"], res2["mu"])
    rng = np.random.default_rng(100 + cid)
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


@pytest.mark.parametrize("N,tile", [(256, 16), (8192, 32)])
@pytest.mark.parametrize("precision", SPLITS)
def test_f16x3_activation_overflow_redone_in_f32(N, tile, precision):
    """Candidates whose start state normalises past the split range (|x| >= 2048) are redone by the
    F32 kernel: their workgroups (16 candidates, or 32 once N >= 8192) carry fp32 results (equal to
    the F32 path's up to its summation order: the redo runs at the split kernel's tile height), the
    rest of the batch stays F16X3 (within the return bar of the F32 path)."""
    from mbrl_amd import fused
    p = ocem.synth_problem(3, N=N, H=6)
    H, a, s = 6, p["cfg"]["a"], p["cfg"]["s"]
    f32, f16 = problems(p, precision)
    s0 = np.tile(p["s0"], (N, 1)).astype(np.float32)
    hot = [5, 40, 41, 200]
    s0[hot, 3] = 1.0e6
    A = torch.from_numpy(cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 3, 0,
                                     np.arange(N))).to(DEV)
    s0d = torch.from_numpy(s0).to(DEV)
    st32 = torch.empty((1, H, N, s), device=DEV)
    st16 = torch.empty((1, H, N, s), device=DEV)
    c32 = fused.rollout(f32, s0d, N, H, actions=A, s0_per_candidate=True, states_out=st32)
    c16 = fused.rollout(f16, s0d, N, H, actions=A, s0_per_candidate=True, states_out=st16)
    torch.cuda.synchronize()
    redone = np.zeros(N, bool)
    for n in hot:
        redone[tile * (n // tile):tile * (n // tile) + tile] = True
    c32n, c16n = c32.cpu().numpy()[0], c16.cpu().numpy()[0]
    # no redo mark survives, and the redone workgroups hold fp32 results
    assert not np.any(c16n.view(np.uint32) == 0x7FC0DEAD)
    assert np.allclose(c16n[redone], c32n[redone], rtol=1e-6, atol=0, equal_nan=True)
    m = torch.from_numpy(redone).to(DEV)
    assert torch.allclose(st16[:, :, m], st32[:, :, m], rtol=1e-4, atol=1e-4, equal_nan=True)
    if tile == 16:   # same tile height and waves as the F32 path at this N: bit for bit
        assert np.array_equal(c16n[redone].view(np.int32), c32n[redone].view(np.int32))
    assert rel_err(c16n[~redone], c32n[~redone].astype(np.float64)) < RTOL


@pytest.mark.parametrize("precision", SPLITS)
def test_f16x3_weight_out_of_range_falls_back_to_f32(precision):
    """A weight with |w| >= 128 cannot be split: the pack flags it and every workgroup is redone in
    F32, so the F16X3 call returns the F32 costs exactly."""
    from mbrl_amd import fused
    p = ocem.synth_problem(2, N=300, H=5)
    p["model"][0][1][0][7, 11] = 40000.0            # hidden layer weight
    N, H, a = 300, 5, p["cfg"]["a"]
    f32, f16 = problems(p, precision)
    A = torch.from_numpy(cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 9, 0,
                                     np.arange(N))).to(DEV)
    s0 = torch.from_numpy(p["s0"]).to(DEV)
    c32 = fused.rollout(f32, s0, N, H, actions=A)
    c16 = fused.rollout(f16, s0, N, H, actions=A)
    torch.cuda.synchronize()
    assert torch.equal(c16.view(torch.int32), c32.view(torch.int32))


@pytest.mark.parametrize("precision", SPLITS)
def test_f16x3_batched_and_sharded_paths_accept_precision(precision):
    """plan_batch with precision='f16x3' equals B single plans of the same precision."""
    from mbrl_amd import CEMPlanner
    p = ocem.synth_problem(3, N=512, H=8)
    _, model_fn, cost_fn, sample_action = build(p)
    B = 3
    s0 = torch.from_numpy(np.stack([p["s0"] + 0.1 * b for b in range(B)]).astype(np.float32))
    kw = dict(num_candidates=512, num_iterations=2, seed=21, precision=precision)
    states, actions = CEMPlanner.plan_batch(s0, model_fn, cost_fn, sample_action, 8, **kw)
    assert actions.shape == (B, 8, p["cfg"]["a"]) and torch.isfinite(states).all()
