"""The 8-candidate rollout tile (rollout_m8_kernel, v_mfma_f32_4x4x1_16b_f32) against
the 16-candidate kernel and the CPU oracle. The two kernels consume every accumulator's k in the
same order, so their costs and states must agree BIT FOR BIT (that keeps a sharded plan independent
of the tile height its shard size picks); both stay within the oracle bars of test_gpu_parity.py.
mbrl_set_option(MBRL_OPT_ROLLOUT_TILE, 8 / 16) forces the tile height (cem.hip rollout_impl)."""
import numpy as np
import pytest
import torch

from oracle import cem as ocem
from oracle.philox import cem_actions

from test_gpu_parity import DEV, RTOL, build, device_problem, rel_err

pytestmark = pytest.mark.gpu


def _rollout(prob, p, N, H, m, A):
    from mbrl_amd import _lib, fused
    E, s = p["cfg"]["E"], p["cfg"]["s"]
    states = torch.empty((E, H, N, s), dtype=torch.float32, device=DEV)
    with _lib.option("rollout_tile", m):
        costs = fused.rollout(prob, torch.from_numpy(p["s0"]).to(DEV), N, H, actions=torch.from_numpy(A).to(DEV),
                              states_out=states)
    torch.cuda.synchronize()
    return costs, states


@pytest.mark.parametrize("cid,N,H,over", [(2, 1000, 20, {}), (2, 9, 5, {}), (3, 2048, 6, {}), (3, 300, 30, {}),
                                          (3, 1, 3, {}), (4, 517, 7, {}), (5, 40, 6, {}), (5, 250, 3, {}),
                                          (3, 33, 1, {}), (2, 300, 5, dict(L=1)), (3, 100, 4, dict(W=200)),
                                          (4, 64, 3, dict(W=256, L=4))])
def test_m8_matches_m16_bitwise_and_the_oracle(cid, N, H, over):
    p = ocem.synth_problem(cid, N=N, H=H, **over)
    a = p["cfg"]["a"]
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 5, 0, np.arange(N))
    prob = device_problem(p)
    c8, s8 = _rollout(prob, p, N, H, 8, A)
    c16, s16 = _rollout(prob, p, N, H, 16, A)
    assert torch.equal(c8, c16), float((c8 - c16).abs().max())
    assert torch.equal(s8, s16)
    ref_costs, ref_states = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A, store_states=True)
    assert rel_err(c8, ref_costs) < RTOL
    assert np.allclose(s8.cpu().numpy(), ref_states, rtol=1e-4, atol=1e-4)


def test_m8_plan_equals_m16_plan():
    """A whole CEM plan at a strong-scaling shard size (walker, 2048 candidates): identical
    returns, elites, mu and sigma with either tile height."""
    from mbrl_amd import CEMPlanner, _lib
    p = ocem.synth_problem(4, N=2048, H=10)
    _, model_fn, cost_fn, sample_action = build(p)
    out = {}
    for m in (8, 16):
        with _lib.option("rollout_tile", m):
            out[m] = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 10,
                                              num_candidates=2048, num_iterations=3, seed=p["rng_seed"],
                                              record=True)
    for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
        assert torch.equal(out[8][k], out[16][k]), k


@pytest.mark.parametrize("cid,N,H", [(5, 8192, 4), (4, 8200, 3), (3, 8192, 5)])
def test_32_candidate_tiles_match_smaller_shards_bitwise(cid, N, H):
    """N >= 8192 runs 32-candidate tiles (R = 2, 4 waves); humanoid's wide state fits them only with the
    output partials aliased onto the activation buffer the last hidden layer does not read
    (RolloutArgs.part_alias). Costs must equal, bit for bit, the same candidates rolled out as shards
    of <= 2048 (8- and 16-candidate tiles): the canonical output-layer sum of every tile height."""
    p = ocem.synth_problem(cid, N=N, H=H)
    a = p["cfg"]["a"]
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 5, 0, np.arange(N))
    prob = device_problem(p)
    full, _ = _rollout(prob, p, N, H, 16, A)
    parts = []
    for lo in range(0, N, 2048):
        hi = min(N, lo + 2048)
        c, _ = _rollout(prob, p, hi - lo, H, 8 if (hi - lo) % 2 == 0 else 16, np.ascontiguousarray(A[:, lo:hi]))
        parts.append(c)
    assert torch.equal(full, torch.cat(parts, dim=1))
    ref = ocem.ensemble_returns(ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A[:, :64]))
    assert rel_err(full.mean(0)[:64] if p["cfg"]["E"] > 1 else full[0, :64], ref) < RTOL


@pytest.mark.parametrize("cid,N,H,m", [(5, 8192, 3, 16), (5, 1000, 4, 16), (5, 1000, 4, 8), (5, 33, 2, 16),
                                       (3, 600, 3, 16)])
def test_ensemble_xcd_order_is_bitwise_neutral(cid, N, H, m):
    """MBRL_OPT_XCD_MAP: ensembles launch a 1-D grid whose workgroups map member-major onto the XCDs
    (xcd_unit): every (tile, member) is still computed exactly once, so costs and states
    equal the plain (tile, member) grid bit for bit -- including grids whose size is not a multiple of
    8 and single-member models (which never remap)."""
    from mbrl_amd import _lib
    p = ocem.synth_problem(cid, N=N, H=H)
    a = p["cfg"]["a"]
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 7, 0, np.arange(N))
    prob = device_problem(p)
    c_plain, s_plain = _rollout(prob, p, N, H, m, A)
    with _lib.option("xcd_map", 1):
        c_map, s_map = _rollout(prob, p, N, H, m, A)
    assert torch.equal(c_map, c_plain) and torch.equal(s_map, s_plain)
    ref = ocem.ensemble_returns(ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A[:, :48]))
    assert rel_err(c_map.mean(0)[:48] if p["cfg"]["E"] > 1 else c_map[0, :48], ref) < RTOL


@pytest.mark.parametrize("cid,N,H,over", [(2, 1000, 20, {}), (2, 9, 5, {}), (3, 1024, 6, {}), (3, 300, 30, {}),
                                          (3, 1, 3, {}), (4, 517, 7, {}), (5, 40, 6, {}), (3, 33, 1, {}),
                                          (2, 300, 5, dict(L=1)), (3, 100, 4, dict(W=200)),
                                          (4, 64, 3, dict(W=256, L=4)), (2, 64, 4, dict(W=512)),
                                          (4, 90, 3, dict(W=200, L=1))])
def test_m4_matches_m16_bitwise_and_the_oracle(cid, N, H, over):
    """The 4-candidate tile (rollout_m4_kernel: one 64-row chain per wave, the output layer's
    canonical chains as 4x4x1 blocks closed by lane swaps) against the 16-candidate kernel: the same
    bits, costs and states, and the oracle bars. Humanoid (s = 67 > 64) has no 4-candidate stream and
    falls back to 8-candidate tiles -- also bit-identical."""
    p = ocem.synth_problem(cid, N=N, H=H, **over)
    a = p["cfg"]["a"]
    A = cem_actions(np.zeros((H, a), np.float32), np.full((H, a), 0.5, np.float32), -1, 1, 5, 0, np.arange(N))
    prob = device_problem(p)
    c4, s4 = _rollout(prob, p, N, H, 4, A)
    c16, s16 = _rollout(prob, p, N, H, 16, A)
    assert torch.equal(c4, c16), float((c4 - c16).abs().max())
    assert torch.equal(s4, s16)
    ref_costs, ref_states = ocem.rollout(p["model"], p["norm"], p["cost"], p["s0"], A, store_states=True)
    assert rel_err(c4, ref_costs) < RTOL
    assert np.allclose(s4.cpu().numpy(), ref_states, rtol=1e-4, atol=1e-4)


def test_cartpole_plan_equal_for_every_tile_height():
    """BASELINE config 2 (cartpole N=1024, H=20): the whole plan is the same with 4, 8 and 16
    candidates per workgroup."""
    from mbrl_amd import CEMPlanner, _lib
    p = ocem.synth_problem(2)
    _, model_fn, cost_fn, sample_action = build(p)
    out = {}
    for m in (4, 8, 16):
        with _lib.option("rollout_tile", m):
            out[m] = CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, 20,
                                              num_candidates=1024, num_iterations=5, seed=p["rng_seed"], record=True)
    for m in (8, 16):
        for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
            assert torch.equal(out[4][k], out[m][k]), (m, k)
