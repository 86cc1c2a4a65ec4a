"""The one-call sharded plan (mbrl_cem_plan_sharded, the default path of an RCCL process group) run
at G = 2, 4 and 8 ranks on ONE GPU, through the C entry, rank by rank.

RCCL will not put two ranks on one device, so under MBRL_OPT_SHARD_EMULATE a call with comm == NULL
computes every other rank's shard itself (its proposals drawn at that rank's global offset, rolled out
by the same kernels) and writes the rank-major buffer the all-gather would deliver. Everything else is
the multi-rank code path: this rank's offset r * N / G, its own proposal draws (initial and fused into
each update), the rank-major -> member-major cost permutation of ensembles, the selection over all N.
Each rank's costs, returns, elites, mu, sigma, actions and states must equal mbrl_cem_plan's bit for
bit (per-iteration semantics: /root/reference/src/mbrl/planners.py:189-216)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import cem as ocem
from test_gpu_parity import DEV, build

pytestmark = pytest.mark.gpu

KEYS = ("costs", "returns", "elites", "mu", "sigma", "actions", "states")


def _problem(cid, N, H, **over):
    from mbrl_amd import CEMPlanner, fused
    p = ocem.synth_problem(cid, N=N, H=H, **over)
    _, model_fn, cost_fn, sample_action = build(p)
    dev = torch.device(DEV)
    md = fused.describe_model(model_fn)
    prob = fused.device_problem(md, fused.describe_cost(cost_fn, md["s"], md), dev)
    st = CEMPlanner._settings(sample_action, H, dict(num_candidates=N, num_iterations=5, seed=p["rng_seed"],
                                                     record=True))
    s0 = torch.from_numpy(p["s0"]).to(dev)
    return prob, st, s0


def _single(prob, st, s0):
    from mbrl_amd import planners
    with torch.cuda.device(prob.device):
        res = planners._cem_fused_single(prob, s0, st)
    torch.cuda.synchronize()
    return {k: res[k].cpu() for k in KEYS}


def _emulated(prob, st, s0, world, rank):
    from mbrl_amd import _lib, planners
    with _lib.option("shard_emulate", 1), torch.cuda.device(prob.device):
        res = planners._cem_sharded_native(prob, s0, st, world, rank, comm=None)
        torch.cuda.synchronize()
    return {k: res[k].cpu() for k in KEYS}


def _assert_same(got, ref, tag):
    for k in KEYS:
        assert got[k].shape == ref[k].shape, (tag, k)
        assert torch.equal(got[k], ref[k]), (tag, k, float((got[k].double() - ref[k].double()).abs().max()))


# (cid, N, H, over, worlds): walker configs[3] at full size over 2/4/8 ranks (8-candidate tiles at
# 2048 per rank); humanoid configs[4] (E = 5, N = 32768, H = 50) over 8 ranks: 4096 per rank, the
# ensemble permutation and the unfused select / refit / draw path (K a exceeds the fused update);
# cheetah configs[2] over 8 ranks (512 per rank); the reward head and cartpole at smaller sizes
CASES = [
    (4, 16384, 30, {}, (2, 4, 8)),
    (5, 32768, 50, {}, (8,)),
    (3, 4096, 30, {}, (8,)),
    (6, 2048, 12, {}, (4,)),
    (2, 1024, 20, {}, (8,)),
]


@pytest.mark.parametrize("cid,N,H,over,worlds", CASES, ids=[f"c{c[0]}_N{c[1]}_G{'-'.join(map(str, c[4]))}"
                                                           for c in CASES])
def test_sharded_plan_every_rank_equals_single_gpu_plan(cid, N, H, over, worlds):
    prob, st, s0 = _problem(cid, N, H, **over)
    ref = _single(prob, st, s0)
    for world in worlds:
        for rank in range(world):
            _assert_same(_emulated(prob, st, s0, world, rank), ref, (cid, world, rank))
    print(f"c{cid} N={N} H={H} E={prob.mdesc['E']}: ranks of G={worlds} bit-identical to mbrl_cem_plan "
          f"(elites {tuple(ref['elites'].shape)}, mu[0,0] {float(ref['mu'][0, 0]):.6g})")


def test_sharded_plan_through_the_c_entry_rejects_bad_calls():
    """The C entry's refusals: N % nranks != 0 (workspace query 0, plan MBRL_EINVAL), comm == NULL
    without the emulation switch, bad communicator arguments -- all before any collective."""
    from mbrl_amd import _lib, fused
    lib = _lib.load()
    prob, st, s0 = _problem(3, 1000, 6)
    params = _lib.CemParams(1000, 6, 100, 2, 0.1, -1.0, 1.0, 0.0, 0.5, 0, 1)
    shape = fused.ctypes_ref(prob.shape)
    assert lib.mbrl_cem_plan_sharded_workspace_bytes(shape, ctypes.byref(params), 3) == 0
    assert lib.mbrl_cem_plan_sharded_workspace_bytes(shape, ctypes.byref(params), 8) > 0
    need = lib.mbrl_cem_plan_sharded_workspace_bytes(shape, ctypes.byref(params), 8)
    ws = torch.empty(need, dtype=torch.uint8, device=DEV)
    out = torch.empty(6 * (17 + 3 * 6), dtype=torch.float32, device=DEV)

    def call(nranks, rank, comm=None):
        return lib.mbrl_cem_plan_sharded(shape, _lib.ptr(prob.packed), fused.ctypes_ref(prob.norm),
                                         fused.ctypes_ref(prob.cost), _lib.ptr(s0), ctypes.byref(params), comm,
                                         nranks, rank, _lib.ptr(out), _lib.ptr(out), _lib.ptr(out), _lib.ptr(out),
                                         None, None, None, None, _lib.ptr(ws), ws.numel(), _lib.stream_handle(DEV))

    assert call(8, 0) == _lib.MBRL_EINVAL                    # comm NULL, no emulation
    assert b"comm" in lib.mbrl_last_error()
    with _lib.option("shard_emulate", 1):
        assert call(3, 0) == _lib.MBRL_EINVAL                 # 1000 % 3
        assert b"1000 over 3 ranks" in lib.mbrl_last_error()
        assert call(8, 8) == _lib.MBRL_EINVAL                 # rank out of range
        emu_need = lib.mbrl_cem_plan_sharded_workspace_bytes(shape, ctypes.byref(params), 8)
        assert emu_need > need                               # + one shard of emulated proposals
        assert call(8, 0) == _lib.MBRL_EWORKSPACE             # the emulation's buffer is not in `ws`
    torch.cuda.synchronize()
    comm = ctypes.c_void_p()
    ident = ctypes.create_string_buffer(_lib.MBRL_COMM_ID_BYTES)
    assert lib.mbrl_comm_init(ident, 0, 0, ctypes.byref(comm)) == _lib.MBRL_EINVAL
    assert lib.mbrl_comm_init(ident, 2, 2, ctypes.byref(comm)) == _lib.MBRL_EINVAL
    assert lib.mbrl_comm_init(None, 2, 0, ctypes.byref(comm)) == _lib.MBRL_EINVAL
    assert lib.mbrl_comm_destroy(None) == _lib.MBRL_OK


def _emulated_mode(prob, st, s0, world, rank, mode, **opts):
    from mbrl_amd import _lib, planners
    import contextlib
    with contextlib.ExitStack() as stack:
        stack.enter_context(_lib.option("shard_emulate", mode))
        for k, v in opts.items():
            stack.enter_context(_lib.option(k, v))
        stack.enter_context(torch.cuda.device(prob.device))
        res = planners._cem_sharded_native(prob, s0, st, world, rank, comm=None)
        torch.cuda.synchronize()
    return {k: res[k].cpu() for k in KEYS}


@pytest.mark.parametrize("cid,N,H,world", [(4, 16384, 30, 8), (5, 32768, 50, 8), (3, 4096, 30, 4)],
                         ids=["c4_G8", "c5_G8", "c3_G4"])
def test_timing_emulation_runs_one_ranks_work_bit_identically(cid, N, H, world):
    """MBRL_OPT_SHARD_EMULATE = 2 (the per-rank timing mode, tools/rank_split.py): the other ranks'
    slots come from the costs a mode-1 plan kept, in one launch per iteration, so the call runs one
    rank's own work only -- and, kept costs being the same problem's, every output equals the single-GPU
    plan's bit for bit (the selection still runs over all N with K = N / 10)."""
    prob, st, s0 = _problem(cid, N, H)
    ref = _single(prob, st, s0)
    _assert_same(_emulated_mode(prob, st, s0, world, 0, 1), ref, (cid, world, "mode 1"))
    for rank in (0, world // 2, world - 1):
        _assert_same(_emulated_mode(prob, st, s0, world, rank, 2), ref, (cid, world, rank, "mode 2"))


@pytest.mark.parametrize("cid,N,H,world", [(4, 16384, 30, 8), (5, 32768, 50, 8), (2, 1024, 20, 4)],
                         ids=["c4_G8", "c5_G8", "c2_G4"])
def test_a_failed_peer_is_reported_on_every_rank(cid, N, H, world):
    """A launch failure on one rank (injected at iteration 1 in an emulated peer's slot: its costs
    poisoned and its status word set, as the failing rank itself does) makes every other rank id return
    MBRL_EPEER -- not a plan over N - N/G candidates (planners.py:184 chooses over all N) -- and the
    failing rank id its own error. The next plan is the single-GPU plan again, bit for bit."""
    from mbrl_amd import _lib
    prob, st, s0 = _problem(cid, N, H)
    ref = _single(prob, st, s0)
    bad = 1
    for rank in range(world):
        with pytest.raises(RuntimeError) as ei:
            _emulated_mode(prob, st, s0, world, rank, 1, debug_shard_fail=2, debug_shard_fail_rank=bad + 1)
        msg = str(ei.value)
        if rank == bad:
            assert f"({_lib.MBRL_EHIP})" in msg and "injected launch failure at iteration 1" in msg, msg
        else:
            assert f"({_lib.MBRL_EPEER})" in msg and f"rank(s) {bad} failed during this plan" in msg, msg
    _assert_same(_emulated_mode(prob, st, s0, world, 0, 1), ref, (cid, world, "after"))


def test_sharded_plan_with_the_split_update_forced_both_ways():
    """The sharded plan's update over all N (walker N = 16384 at G = 8: K = 1638, where auto splits it)
    with the split update forced off and on: every rank id equal to the single-GPU plan."""
    prob, st, s0 = _problem(4, 16384, 30)
    ref = _single(prob, st, s0)
    for split in (1, 2):
        for rank in (0, 7):
            _assert_same(_emulated_mode(prob, st, s0, 8, rank, 1, update_split=split), ref, ("split", split, rank))


@pytest.mark.parametrize("mode", [1, 2])
def test_a_timed_out_pair_handoff_redoes_the_plan_without_pairs(mode):
    """With peers the sharded plan checks its column-split pair launches once, after the plan (the pair
    status word gathered with the last iteration's costs) instead of a gated redo launch behind every
    pair launch. A hand-off that times out (MBRL_OPT_DEBUG_PAIR_ABORT = 1: the pair kernel gives up at
    once) sends every rank through the plan again on 8-candidate tiles: the result is still the
    single-GPU plan, bit for bit (walker N = 16384 at G = 8: 2048 candidates per rank, pairs)."""
    prob, st, s0 = _problem(4, 16384, 30)
    ref = _single(prob, st, s0)
    _emulated_mode(prob, st, s0, 8, 0, 1)   # keeps the gathered costs for mode 2
    for rank in (0, 5):
        got = _emulated_mode(prob, st, s0, 8, rank, mode, debug_pair_abort=1)
        _assert_same(got, ref, ("pair abort", mode, rank))
