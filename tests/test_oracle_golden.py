"""CPU: the oracle restatement (oracle/cem.py) against golden vectors produced by the reference's own
planner / model / cost code (tests/golden/make_golden.py). Pins the oracle before it is trusted as
the checker for the HIP path."""
import numpy as np
import pytest

from oracle import cem as ocem
from oracle.philox import cem_actions

RTOL = 1e-5  # BASELINE.json north_star: returns within 1e-5 relative


def rel_err(x, ref):
    return float(np.max(np.abs(np.asarray(x, np.float64) - ref) / np.maximum(np.abs(ref), 1.0)))


def test_toy_ring_known_answer(golden):
    """test_random_shooting.py:5-25: torch.manual_seed(0) -> states [1, 0, 9, 9, 8], cost 18."""
    g = golden("toy_ring_rs")
    H, N = 5, 1000
    A = g["actions_flat"].reshape(H, N, 1)
    st = np.full((N, 1), 2.0, np.float32)
    states, costs = [], np.zeros(N, np.float32)
    for t in range(H):
        st = np.fmod(np.fmod(st + A[t], 10.0) + 10.0, 10.0).astype(np.float32)
        states.append(st)
        costs += np.abs(st[:, 0] - 9.0)
    idx = ocem.rs_argmin(costs)
    assert costs[idx] == 18.0 == float(g["plan_cost"])
    assert np.array_equal(np.stack(states)[:, idx, 0], g["plan_states"].ravel())
    assert np.array_equal(A[:, idx], g["plan_actions"])


def test_config1_random_shooting(golden):
    g = golden("config1_rs")
    p = ocem.synth_problem(1)
    assert ocem.weights_sha256(p["model"]) == str(g["weights_sha256"])
    N, H = p["cfg"]["N"], p["cfg"]["H"]
    states, actions, ret, idx = ocem.rs_plan(p, g["actions_flat"], N, H)
    assert rel_err(ret, g["costs"]) < RTOL
    assert idx == int(g["idx"])
    assert np.array_equal(actions, g["plan_actions"])
    assert np.allclose(states, g["plan_states"], rtol=1e-5, atol=1e-5)


CEM_CASES = [("config2_cem", 2, {}), ("config3_cem", 3, {}), ("config4_cem_N2048", 4, dict(N=2048)),
             ("config5_cem_N256_H20", 5, dict(N=256, H=20)),
             ("config6_cem_N512_H10", 6, dict(N=512, H=10))]   # reward head: ModelWithReward + RewardAgent cost


@pytest.mark.parametrize("name,cid,over", CEM_CASES, ids=[c[0] for c in CEM_CASES])
def test_cem_against_reference(golden, name, cid, over):
    g = golden(name)
    p = ocem.synth_problem(cid, **over)
    assert ocem.weights_sha256(p["model"]) == str(g["weights_sha256"])
    out = ocem.cem_plan(p)
    for it in range(int(g["I"])):
        assert rel_err(out["returns"][it], g["returns"][it]) < RTOL, f"iteration {it}"
        assert np.array_equal(out["elites"][it], g["elites"][it]), f"iteration {it}"
        assert np.array_equal(out["mu"][it], g["mu"][it])
        assert np.array_equal(out["sigma"][it], g["sigma"][it])
    assert np.array_equal(out["final_actions"], g["final_actions"])
    assert np.allclose(out["final_states"], g["final_states"], rtol=1e-5, atol=1e-5)


def test_refit_chunk_order_is_canonical():
    """mu/sigma depend only on the elite SET: permuting which rank holds which elite cannot matter
    because the refit always sums in ascending candidate order, chunk by chunk."""
    rng = np.random.default_rng(3)
    H, a, K = 4, 3, 77
    A = rng.uniform(-1, 1, size=(K, H, a)).astype(np.float32)
    mu = np.zeros((H, a), np.float32)
    sg = np.full((H, a), 0.5, np.float32)
    m1, s1 = ocem.refit(mu, sg, A, 0.1)
    m2, s2 = ocem.refit(mu, sg, A.copy(), 0.1)
    assert np.array_equal(m1, m2) and np.array_equal(s1, s2)
    ref_mean = A.astype(np.float64).mean(0)
    assert np.allclose(m1, 0.9 * ref_mean, atol=1e-6)
    assert np.all(s1 > 0)


def test_select_elites_semantics():
    r = np.array([3.0, 1.0, np.nan, 1.0, -0.0, 0.0, 2.0, np.nan], np.float32)
    assert list(ocem.select_elites(r, 4)) == [1, 3, 4, 5]      # stable: -0.0 (idx 4) before 0.0 (idx 5)
    assert list(ocem.select_elites(r, 7)) == [0, 1, 2, 3, 4, 5, 6]  # NaN last, first NaN first
    assert ocem.rs_argmin(r) == 2                                # np.argmin: first NaN wins


def test_cem_actions_are_the_ones_rolled_out():
    p = ocem.synth_problem(2, N=64, H=6)
    H, a = 6, 1
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, p["rng_seed"], 0,
                    np.arange(64))
    c1 = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A)
    c2 = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A[:, ::-1].copy())
    assert np.allclose(c1[0], c2[0][::-1], rtol=1e-6)


FULL_CASES = [("config4_cem_full", 4), ("config5_cem_full", 5), ("config6_cem_full", 6)]


@pytest.mark.parametrize("name,cid", FULL_CASES, ids=[c[0] for c in FULL_CASES])
def test_full_size_fixture_sampled(golden, name, cid):
    """The full-size reference fixtures (walker N=16384; humanoid N=32768 H=50 E=5): for 24 sampled
    candidates per iteration the oracle, teacher-forced on the fixture's mu / sigma, reproduces the
    reference returns within 1e-5; the oracle refit of the fixture's elite set reproduces its mu /
    sigma bit for bit; the fixture's elites are the stable top-K of its returns."""
    g = golden(name)
    p = ocem.synth_problem(cid)
    assert ocem.weights_sha256(p["model"]) == str(g["weights_sha256"])
    N, H, K = int(g["N"]), int(g["H"]), int(g["K"])
    a = p["cfg"]["a"]
    mu = np.zeros((H, a), np.float32)
    sg = np.full((H, a), 0.5, np.float32)
    rng = np.random.default_rng(cid)
    for it in range(int(g["I"])):
        assert np.array_equal(g["elites"][it], ocem.select_elites(g["returns"][it], K))
        idx = np.sort(rng.choice(N, size=24, replace=False))
        A = cem_actions(mu, sg, -1.0, 1.0, p["rng_seed"], it, idx)
        ref = ocem.ensemble_returns(ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A))
        assert rel_err(ref, g["returns"][it][idx]) < RTOL, f"iteration {it}"
        Ael = cem_actions(mu, sg, -1.0, 1.0, p["rng_seed"], it, g["elites"][it])
        mu, sg = ocem.refit(mu, sg, np.ascontiguousarray(Ael.transpose(1, 0, 2)), 0.1)
        assert np.array_equal(mu, g["mu"][it]) and np.array_equal(sg, g["sigma"][it]), f"iteration {it}"
    assert np.array_equal(np.clip(mu, -1.0, 1.0), g["final_actions"])
