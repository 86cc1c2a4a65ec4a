"""Where the host's turn between two small plans goes: wall time per synchronous CEMPlanner.plan()
split into the Python/host pieces of planners.plan_detailed (wrapped with perf_counter timers) and
the rest (the GPU's own time, the result copy's wait). Usage: python tools/host_turn.py [config_id]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402

from mbrl_amd import CEMPlanner, _lib, fused, planners, synthetic  # noqa: E402

ACC = {}


def timed(mod, name, label=None):
    fn = getattr(mod, name)

    def wrap(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label or name] = ACC.get(label or name, 0.0) + time.perf_counter() - t
    setattr(mod, name, wrap)


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    p = synthetic.make_problem(cid)
    cfg = p["cfg"]
    kw = dict(num_candidates=cfg["N"], num_iterations=5, seed=p["rng_seed"], device="cuda:0")
    for _ in range(10):
        CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], cfg["H"], **kw)
    torch.cuda.synchronize()
    for mod, name in ((fused, "describe"), (fused, "semantic_check"), (fused, "describe_model"),
                      (fused, "describe_cost"), (fused, "device_problem"),
                      (fused, "describe_sampler"), (planners, "_cem_fused_single")):
        timed(mod, name)
    lib = _lib.load()
    real = lib.mbrl_cem_plan

    def c_call(*a):
        t = time.perf_counter()
        rc = real(*a)
        ACC["mbrl_cem_plan (C enqueue)"] = ACC.get("mbrl_cem_plan (C enqueue)", 0.0) + time.perf_counter() - t
        return rc
    lib.mbrl_cem_plan = c_call
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], cfg["H"], **kw)
    wall = (time.perf_counter() - t0) / n
    lib.mbrl_cem_plan = real
    out = dict(config=cfg["name"], wall_us=wall * 1e6, **{k + "_us": v / n * 1e6 for k, v in ACC.items()})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
