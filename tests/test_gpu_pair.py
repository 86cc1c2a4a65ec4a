"""GPU: column-split pairs (rollout.hip rollout_kernel PAIR: two workgroups per 16-candidate tile, each
computing half of every hidden layer's columns, halves crossing through L2) give the same plans as
8- and 16-candidate tiles, bit for bit: every accumulator keeps the canonical K order and the output
sum is the canonical ((p0 + p1) + (p2 + p3)) + ((p4 + p5) + (p6 + p7)). MBRL_OPT_ROLLOUT_PAIR = 1
forces the pair kernel (a plan fails instead of falling back), and MBRL_OPT_DEBUG_PAIR_ABORT = 2 drops
the gated redo launch behind it (which recomputes a launch whose hand-off timed out), so these tests
compare the pair kernel's own results."""
from contextlib import ExitStack

import numpy as np
import pytest
import torch

from oracle import cem as ocem
from test_gpu_parity import build

pytestmark = pytest.mark.gpu

# (config, N, H): walker / cheetah at the 8- and 2-GPU shard sizes, ragged and tiny N, the ensemble
# (humanoid E = 5: K0C = NOT = 6) and a 2x512 model (L = 2: one layer hand-off per step)
CASES = [(4, 2048, 30), (3, 2048, 30), (3, 1024, 12), (4, 300, 7), (3, 17, 5), (3, 1, 3), (5, 200, 4)]
PAIR_ONLY = {"rollout_pair": 1, "debug_pair_abort": 2}


def _plan(p, N, H, opts):
    from mbrl_amd import CEMPlanner, _lib
    _, model_fn, cost_fn, sample_action = build(p)
    with ExitStack() as stack:
        for name, value in opts.items():
            stack.enter_context(_lib.option(name, value))
        return CEMPlanner.plan_detailed(torch.from_numpy(p["s0"]), model_fn, cost_fn, sample_action, H,
                                        num_candidates=N, num_iterations=3, seed=p["rng_seed"], record=True)


@pytest.mark.parametrize("cid,N,H", CASES)
def test_pair_plan_equals_every_tile_height(cid, N, H):
    p = ocem.synth_problem(cid, N=N, H=H)
    pair = _plan(p, N, H, PAIR_ONLY)
    m16 = _plan(p, N, H, {"rollout_tile": 16, "rollout_pair": 2})
    m8 = _plan(p, N, H, {"rollout_tile": 8, "rollout_pair": 2})
    for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
        assert torch.equal(pair[k], m16[k]), (k, "pair vs 16")
        assert torch.equal(pair[k], m8[k]), (k, "pair vs 8")
    assert np.isfinite(pair["returns"].cpu().numpy()).all()


def test_pair_plan_two_hidden_layers():
    """L = 2 (one layer hand-off per step) at the shard size."""
    p = ocem.synth_problem(3, N=512, H=6, L=2)
    pair = _plan(p, 512, 6, PAIR_ONLY)
    m16 = _plan(p, 512, 6, {"rollout_tile": 16, "rollout_pair": 2})
    for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
        assert torch.equal(pair[k], m16[k]), k


def test_forced_pair_fails_loudly_where_it_cannot_run():
    """Cartpole (Wpad 256) has no pair kernel: forcing it is an error, not a silent fallback."""
    from mbrl_amd import _lib
    p = ocem.synth_problem(2, N=256, H=4)
    with pytest.raises(RuntimeError, match="rollout_pair"):
        _plan(p, 256, 4, {"rollout_pair": 1})
    assert _lib is not None


def _fuzz_shape(case):
    rng = np.random.default_rng(9100 + case)
    over = dict(s=int(rng.integers(1, 41)), a=int(rng.integers(1, 13)), W=int(rng.choice([300, 400, 512])),
                L=int(rng.integers(2, 5)), E=int(rng.choice([1, 1, 2, 3])))
    N = int(rng.choice([3, 16, 47, 200, 513]))
    H = int(rng.integers(1, 9))
    return over, N, H


@pytest.mark.parametrize("case", range(8))
def test_pair_plan_fuzz_equals_16_candidate_tiles(case):
    """Random Wpad-512 shapes (state / action dims, widths below 512, 2-4 hidden layers, ensembles,
    ragged N): column-split pairs and 16-candidate tiles give the same plan bit for bit, or the pair
    kernel declines the shape loudly (no instance for its chunk counts)."""
    over, N, H = _fuzz_shape(case)
    p = ocem.synth_problem(3, N=N, H=H, **over)
    try:
        pair = _plan(p, N, H, PAIR_ONLY)
    except RuntimeError as exc:
        assert "rollout_pair" in str(exc)
        return
    m16 = _plan(p, N, H, {"rollout_tile": 16, "rollout_pair": 2})
    for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
        assert torch.equal(pair[k], m16[k]), (case, over, N, H, k)


@pytest.mark.parametrize("cid,N,H", [(4, 2048, 8), (5, 200, 4)])
def test_pair_hand_off_timeout_is_recomputed(cid, N, H):
    """a plain launch does not promise that both halves of a pair are resident, so a
    hand-off wait can time out. Every pair workgroup then sets bit 0 of the status word and the gated
    launch behind it recomputes the candidates: MBRL_OPT_DEBUG_PAIR_ABORT = 1 makes every workgroup give
    up at once, and the plan still equals the 16-candidate plan bit for bit (with the redo the default,
    a normal pair plan is the same too)."""
    p = ocem.synth_problem(cid, N=N, H=H)
    aborted = _plan(p, N, H, {"rollout_pair": 1, "debug_pair_abort": 1})
    gated = _plan(p, N, H, {"rollout_pair": 1})
    m16 = _plan(p, N, H, {"rollout_tile": 16, "rollout_pair": 2})
    for k in ("returns", "elites", "mu", "sigma", "actions", "states"):
        assert torch.equal(aborted[k], m16[k]), (k, "aborted pair + redo vs 16")
        assert torch.equal(gated[k], m16[k]), (k, "pair + idle redo vs 16")
