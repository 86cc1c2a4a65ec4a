"""Where a bench plan's host time goes (bench.py's timed loop, same kwargs and events): per plan the
Python before the C call, the C call (enqueue), the sync + copy-out, the rest of plan_detailed, the
bench loop between plans, the garbage collector's pauses, and the device span from the plan events.
Usage: python tools/host_split.py [config_id] [plans] [candidates]"""
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mbrl_amd import CEMPlanner, _lib, planners, synthetic  # noqa: E402


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    prob = synthetic.make_problem(cid)
    cfg = prob["cfg"]
    N = int(sys.argv[3]) if len(sys.argv) > 3 else cfg["N"]
    dev = torch.device("cuda:0")
    kw = dict(num_candidates=N, num_elites=N // 10, num_iterations=5, alpha=0.1,
              seed=prob["rng_seed"], distributed=False, device=dev, precision="f32")
    stamps = {}
    lib = _lib.load()
    real_c = lib.mbrl_cem_plan

    def c_call(*a):
        stamps.setdefault("c_in", []).append(time.perf_counter())
        rc = real_c(*a)
        stamps.setdefault("c_out", []).append(time.perf_counter())
        return rc
    lib.mbrl_cem_plan = c_call
    real_host = planners._cem_plan_host

    def host(*a, **k):
        r = real_host(*a, **k)
        stamps.setdefault("host_out", []).append(time.perf_counter())
        return r
    planners._cem_plan_host = host
    from mbrl_amd import fused
    real_dp = fused.describe_problem

    def dp(*a, **k):
        t = time.perf_counter()
        r = real_dp(*a, **k)
        stamps.setdefault("describe", []).append(time.perf_counter() - t)
        return r
    fused.describe_problem = dp
    real_settings = planners.CEMPlanner._settings

    def settings(*a, **k):
        t = time.perf_counter()
        r = real_settings(*a, **k)
        stamps.setdefault("settings", []).append(time.perf_counter() - t)
        return r
    planners.CEMPlanner._settings = staticmethod(settings)
    gc_time = [0.0, 0, None]

    def gc_cb(phase, info):
        if phase == "start":
            gc_time[2] = time.perf_counter()
        elif gc_time[2] is not None:
            gc_time[0] += time.perf_counter() - gc_time[2]
            gc_time[1] += 1
    gc.callbacks.append(gc_cb)

    def plan(**extra):
        return CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], cfg["H"],
                                        **kw, **extra)
    for _ in range(5):
        plan()
    ev = [[(bench.TimingEvent(), bench.TimingEvent()) if it == 2 else None for it in range(5)] for _ in range(n)]
    spans = [(bench.TimingEvent(), bench.TimingEvent()) for _ in range(n)]
    for e in ev:
        e[2][0].record(); e[2][1].record()
    for sp in spans:
        sp[0].record(); sp[1].record()
    torch.cuda.synchronize()
    stamps.clear()
    gc_time[:2] = [0.0, 0]
    t_in, t_out = [], []
    t0 = time.perf_counter()
    for k in range(n):
        t_in.append(time.perf_counter())
        plan(rollout_events=ev[k], plan_events=spans[k])
        t_out.append(time.perf_counter())
    wall = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    span = float(np.mean([a.elapsed_time(b) for a, b in spans])) * 1e3
    ci, co, ho = map(np.array, (stamps["c_in"], stamps["c_out"], stamps["host_out"]))
    ti, to = np.array(t_in), np.array(t_out)
    us = lambda x: float(np.mean(x) * 1e6)  # noqa: E731
    out = dict(config=cfg["name"], plans=n, wall_us=wall * 1e6, plan_gpu_span_us=span,
               host_us=wall * 1e6 - span, python_before_c_us=us(ci - ti), c_enqueue_us=us(co - ci),
               sync_and_copy_us=us(ho - co), after_host_us=us(to - ho), between_plans_us=us(ti[1:] - to[:-1]),
               gc_us_per_plan=gc_time[0] / n * 1e6, gc_runs=gc_time[1],
               python_before_c_max_us=float(np.max(ci - ti) * 1e6),
               describe_problem_us=us(stamps["describe"]), settings_us=us(stamps["settings"]), candidates=N)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
