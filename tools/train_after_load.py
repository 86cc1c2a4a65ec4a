"""Diagnostic: bench.py's `train` line measured on a GPU that has been idle and again right after
~20 s of CEM planning (the bench's order), to tell the GPU's state after a sustained MFMA load from the
training step itself. Usage: python tools/train_after_load.py [seconds]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from mbrl_amd import CEMPlanner, synthetic  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    dev = torch.device("cuda:0")
    out = {"idle": [bench.train_line(dev) for _ in range(2)]}
    p = synthetic.make_problem(4)
    kw = dict(num_candidates=p["cfg"]["N"], num_elites=p["cfg"]["N"] // 10, num_iterations=5, alpha=0.1,
              seed=p["rng_seed"], device=dev)
    t0, plans = time.perf_counter(), 0
    while time.perf_counter() - t0 < secs:
        CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], p["cfg"]["H"], **kw)
        plans += 1
    out["after_load"] = [bench.train_line(dev) for _ in range(2)]
    out["load"] = dict(config=p["cfg"]["name"], seconds=secs, plans=plans)
    for k in ("idle", "after_load"):
        out[k] = [dict(gpu_us_per_step=round(r["gpu_us_per_step"], 2),
                       gpu_us_per_step_10_epochs=round(r["gpu_us_per_step_10_epochs"], 2)) for r in out[k]]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
