"""The sharded plan over a real multi-rank RCCL group: one process per GPU, G = the largest power of
two <= min(8, torch.cuda.device_count()) ranks, mbrl_cem_plan_sharded with the library's own
communicator (ncclAllGather over xGMI on the plan's stream).

On a one-GPU box this file skips (RCCL refuses two ranks on one device; the G > 1 code path is
covered there by tests/test_gpu_sharded_emul.py). On a node with 2-8 GPUs it is the multi-rank parity
evidence of SURVEY.md §8e: every rank's elites (per iteration), mu, sigma, actions and states must equal
the single-GPU plan's bit for bit, for walker configs[3] (N = 16384, H = 30) and the humanoid E = 5
ensemble of configs[4] (N = 32768, H = 50); then a launch failure injected on the last rank makes that
rank raise its own error and every other rank raise MBRL_EPEER, and the same communicator plans again
exactly (reference semantics: the argmin / elite choice over ALL N candidates,
/root/reference/src/mbrl/planners.py:184,189-216)."""
import os

import numpy as np
import pytest
import torch

from oracle import cem as ocem
from test_gpu_parity import build

pytestmark = pytest.mark.gpu

CASES = [(4, dict(N=16384, H=30)), (5, dict(N=32768, H=50))]


def _world():
    n = min(8, torch.cuda.device_count())
    g = 1
    while g * 2 <= n:
        g *= 2
    return g


def _problem(cid, over, dev, record=True):
    from mbrl_amd import CEMPlanner, fused
    p = ocem.synth_problem(cid, **over)
    _, model_fn, cost_fn, sample_action = build(p)
    md = fused.describe_model(model_fn)
    prob = fused.device_problem(md, fused.describe_cost(cost_fn, md["s"], md), dev)
    st = CEMPlanner._settings(sample_action, over["H"], dict(num_candidates=over["N"], num_iterations=5,
                                                             seed=p["rng_seed"], record=record))
    return prob, st, torch.from_numpy(p["s0"]).to(dev)


def _save(res, path, **extra):
    np.savez(path, mu=res["mu"].cpu().numpy(), sigma=res["sigma"].cpu().numpy(),
             elites=torch.stack(list(res["elites"])).cpu().numpy(), actions=res["actions"].cpu().numpy(),
             states=res["states"].cpu().numpy(), **extra)


def _worker(rank, world, init_file, out_dir):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "mujoco-mbrl_amd")]
    import torch.distributed as dist
    from mbrl_amd import _lib, planners
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"file://{init_file}", rank=rank, world_size=world, device_id=dev)
    try:
        planners.SHARDED_NATIVE = True
        for cid, over in CASES:
            prob, st, s0 = _problem(cid, over, dev)
            res = planners._cem_fused_sharded(prob, s0, st, world)
            _save(res, os.path.join(out_dir, f"c{cid}_r{rank}.npz"))
            if rank == 0:   # the single-GPU plan on this rank's device, after the sharded one
                _save(planners._cem_fused_single(prob, s0, st), os.path.join(out_dir, f"c{cid}_single.npz"))
            dist.barrier()
        # one rank's launch fails at iteration 1: it raises its own error, every peer MBRL_EPEER
        cid, over = CASES[0]
        prob, st, s0 = _problem(cid, over, dev)
        with _lib.option("debug_shard_fail", 2), _lib.option("debug_shard_fail_rank", world):
            try:
                planners._cem_fused_sharded(prob, s0, st, world)
                raised = ""
            except RuntimeError as e:
                raised = str(e)
        torch.cuda.synchronize()
        again = planners._cem_fused_sharded(prob, s0, st, world)   # the same communicator
        _save(again, os.path.join(out_dir, f"again_r{rank}.npz"), raised=np.array(raised))
    finally:
        dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (one rank per GPU over RCCL)")
def test_sharded_plan_over_multi_rank_rccl():
    import tempfile
    import torch.multiprocessing as mp
    from mbrl_amd import _lib
    world = _world()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, os.path.join(d, "pg"), d), nprocs=world, join=True,
                           start_method="spawn")
        for cid, _ in CASES:
            ref = dict(np.load(os.path.join(d, f"c{cid}_single.npz")))
            for r in range(world):
                got = dict(np.load(os.path.join(d, f"c{cid}_r{r}.npz")))
                for k in ("elites", "mu", "sigma", "actions", "states"):
                    assert np.array_equal(got[k], ref[k]), (cid, world, r, k)
        ref = dict(np.load(os.path.join(d, f"c{CASES[0][0]}_single.npz")))
        for r in range(world):
            again = dict(np.load(os.path.join(d, f"again_r{r}.npz"), allow_pickle=False))
            msg = str(again["raised"])
            if r == world - 1:
                assert "injected launch failure at iteration 1" in msg, (r, msg)
            else:
                assert f"({_lib.MBRL_EPEER})" in msg and f"rank(s) {world - 1} failed" in msg, (r, msg)
            for k in ("elites", "mu", "sigma", "actions", "states"):
                assert np.array_equal(again[k], ref[k]), ("again", r, k)
    print(f"RCCL over {world} GPUs: walker N=16384 and humanoid E=5 N=32768 bit-identical on every rank; "
          f"a failure on rank {world - 1} raised MBRL_EPEER on the other {world - 1}")
