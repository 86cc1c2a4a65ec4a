"""A/B of one mbrl_set_option switch on a BASELINE config: plan wall time and the rollout kernel's
HIP-event time for each value, interleaved over three rounds.
Usage: python tools/opt_ab.py <option> <config_id> [reps] [values, default "1,0"]
<option> "staging" toggles planners.HOST_STAGING (the plan's mapped pinned host staging) instead."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402

import contextlib  # noqa: E402

from mbrl_amd import CEMPlanner, _lib, fused, planners, synthetic  # noqa: E402


@contextlib.contextmanager
def setting(opt, val):
    if opt == "staging":
        prev = planners.HOST_STAGING
        planners.HOST_STAGING = bool(val)
        try:
            yield
        finally:
            planners.HOST_STAGING = prev
    else:
        with _lib.option(opt, val):
            yield


def main():
    opt, cid = sys.argv[1], int(sys.argv[2])
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    values = [int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "1,0").split(",")]
    p = synthetic.make_problem(cid)
    cfg = p["cfg"]
    kw = dict(num_candidates=cfg["N"], num_iterations=5, seed=p["rng_seed"], device="cuda:0")
    md = fused.describe_model(p["model"])
    cd = fused.describe_cost(p["cost"], md["s"], md)
    prob = fused.device_problem(md, cd, torch.device("cuda:0"))
    s0 = torch.as_tensor(p["s0"], dtype=torch.float32, device="cuda:0")
    out = {}
    for rnd in range(3):
        for val in values:
            with setting(opt, val):
                for _ in range(3):
                    CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], cfg["H"], **kw)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], cfg["H"], **kw)
                torch.cuda.synchronize()
                plan_ms = (time.perf_counter() - t0) / reps * 1e3
                acts = torch.rand((cfg["H"], cfg["N"], cfg["a"]), device="cuda:0") * 2 - 1
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                fused.rollout(prob, s0, cfg["N"], cfg["H"], actions=acts)
                e0.record()
                for _ in range(reps):
                    fused.rollout(prob, s0, cfg["N"], cfg["H"], actions=acts)
                e1.record()
                torch.cuda.synchronize()
                roll_ms = e0.elapsed_time(e1) / reps
                out.setdefault(f"{opt}={val}", []).append(dict(plan_ms=round(plan_ms, 4), rollout_ms=round(roll_ms, 4)))
    print(json.dumps(dict(config=cfg["name"], **out)))


if __name__ == "__main__":
    main()
