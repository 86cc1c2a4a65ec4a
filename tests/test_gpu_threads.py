"""GPU: plans in flight at the same time never share scratch. The CEM workspace (proposals, costs,
the pair flags and per-plan epochs, the trajectory granules) belongs to one thread and one stream
(planners._workspace), so plans from several threads -- on the default stream or on streams of their
own -- and one thread's plans left in flight on two streams (return_device=True) each equal the same
plan made alone, bit for bit. The reference's caller is single-threaded; this is what
a caller with threads may rely on."""
import threading
from contextlib import nullcontext

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _plan(prob, N, **kw):
    from mbrl_amd import CEMPlanner
    return CEMPlanner.plan(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], prob["cfg"]["H"],
                           num_candidates=N, num_iterations=3, seed=prob["rng_seed"], device=DEV, **kw)


def _same(x, y):
    return torch.equal(x[0].cpu(), y[0].cpu()) and torch.equal(x[1].cpu(), y[1].cpu())


def test_threads_plan_concurrently_like_one_thread():
    from mbrl_amd import synthetic
    # cartpole (8-candidate tiles, register trajectory) and cheetah at the pair size (column-split
    # pairs, cooperative trajectory: cross-workgroup flags in the workspace)
    cases = {2: 1024, 3: 2048}
    probs = {c: synthetic.make_problem(c) for c in cases}
    ref = {c: _plan(probs[c], n) for c, n in cases.items()}
    results, errors = {}, []

    def worker(c, own_stream):
        try:
            stream = torch.cuda.Stream(DEV) if own_stream else None
            with torch.cuda.stream(stream) if stream is not None else nullcontext():
                out = [_plan(probs[c], cases[c]) for _ in range(12)]
            results[(c, own_stream)] = out
        except Exception as e:          # pragma: no cover - reported below
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(c, own)) for c in cases for own in (False, True)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert len(results) == 4
    for (c, _), outs in results.items():
        assert all(_same(o, ref[c]) for o in outs), c


def test_one_thread_two_streams_in_flight():
    from mbrl_amd import synthetic
    prob = synthetic.make_problem(3)
    ref = _plan(prob, 2048, return_device=True)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    outs = []
    for _ in range(4):                  # nothing waits between the plans: both streams hold plans in flight
        with torch.cuda.stream(s1):
            outs.append(_plan(prob, 2048, return_device=True))
        with torch.cuda.stream(s2):
            outs.append(_plan(prob, 2048, return_device=True))
    torch.cuda.synchronize()
    assert all(_same(o, ref) for o in outs)


def test_training_beside_plans_on_another_stream():
    """the fused training step's bounded in-launch waits assume its workgroups are
    co-resident; plans with cross-workgroup kernels (column-split pairs, the cooperative trajectory) on
    another stream can hold CUs. Training on one thread and stream while another thread plans: the
    plans equal the plan made alone, and training either equals training alone bit for bit or raises
    the status word's RuntimeError -- it never returns wrong parameters silently."""
    import numpy as np
    from mbrl_amd import data, models, synthetic
    prob = synthetic.make_problem(3)
    ref_plan = _plan(prob, 2048)

    def make():
        rng = np.random.Generator(np.random.PCG64(5))
        rolls = []
        for _ in range(6):
            st = rng.standard_normal((201, 17)).astype(np.float32)
            rolls.append(data.Rollout(states=list(torch.from_numpy(st)), observations=list(torch.from_numpy(st)),
                                      actions=list(torch.from_numpy(rng.uniform(-1, 1, (200, 6)).astype(np.float32))),
                                      rewards=list(torch.from_numpy(rng.standard_normal(200).astype(np.float32)))))
        ds = data.TransitionsDataset(rollouts=rolls)
        ds.set_data_mode("state_only")
        torch.manual_seed(0)
        m = models.Model(17, 6, hidden_units=512).to(DEV)
        return m, ds, torch.optim.Adam(m.parameters(), lr=1e-3)

    def train(m, ds, opt):
        np.random.seed(3)
        m.train_model(ds, opt, batch_size=512, num_epochs=10)
        torch.cuda.synchronize()
        return [p.detach().cpu().clone() for p in m.parameters()]

    alone = train(*make())
    out, errors, plans = {}, [], []

    def trainer():
        try:
            with torch.cuda.stream(torch.cuda.Stream(DEV)):
                out["params"] = train(*make())
        except RuntimeError as e:
            out["raised"] = str(e)
        except Exception as e:          # pragma: no cover
            errors.append(repr(e))

    def planner():
        try:
            with torch.cuda.stream(torch.cuda.Stream(DEV)):
                for _ in range(20):
                    plans.append(_plan(prob, 2048))
        except Exception as e:          # pragma: no cover
            errors.append(repr(e))

    threads = [threading.Thread(target=trainer), threading.Thread(target=planner)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not errors, errors
    assert plans and all(_same(p, ref_plan) for p in plans)
    if "raised" in out:
        assert "bounded wait timed out" in out["raised"], out["raised"]
    else:
        assert all(torch.equal(a, b) for a, b in zip(out["params"], alone))
