"""A/B of the 2048-candidate shard's rollout (walker configs[3] over 8 GPUs, cheetah at 2048):
8-candidate tiles vs column-split pairs with written-through (sc1) or L2-resident hand-offs
(MBRL_OPT_PAIR_L2); per mode the rollout launch (fence-free HIP events around iteration 2's rollout)
and the whole plan's wall time, rounds interleaved; plans must be bit-identical.
Usage: python tools/pair_l2_ab.py [rounds] [plans]"""
import json
import os
import sys
import time
from contextlib import ExitStack

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mbrl_amd import CEMPlanner, _lib, synthetic  # noqa: E402

MODES = {"m8": {"rollout_tile": 8, "rollout_pair": 2},
         "pair_sc1": {"rollout_pair": 1, "pair_l2": 2},
         "pair_l2": {"rollout_pair": 1, "pair_l2": 1}}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    out = {}
    for cid, N in ((4, 2048), (3, 2048), (3, 1024)):
        prob = synthetic.make_problem(cid)
        H = prob["cfg"]["H"]
        kw = dict(num_candidates=N, num_elites=N // 10, num_iterations=5, alpha=0.1, seed=prob["rng_seed"],
                  device=dev)
        ref = None
        for _ in range(rounds):
            for name, opts in MODES.items():
                with ExitStack() as stack:
                    for k, v in opts.items():
                        stack.enter_context(_lib.option(k, v))
                    rec = CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"],
                                                   H, record=True, **kw)
                    for _ in range(3):
                        CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], H, **kw)
                    ev = [[(bench.TimingEvent(), bench.TimingEvent()) if it == 2 else None for it in range(5)]
                          for _ in range(n)]
                    for e in ev:
                        e[2][0].record(); e[2][1].record()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for k in range(n):
                        CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], H,
                                                 rollout_events=ev[k], **kw)
                    torch.cuda.synchronize()
                    wall = (time.perf_counter() - t0) / n * 1e3
                    roll = float(np.mean([e[2][0].elapsed_time(e[2][1]) for e in ev]))
                got = {k: rec[k].cpu() for k in ("returns", "elites", "mu", "sigma", "actions", "states")}
                if ref is None:
                    ref = got
                assert all(torch.equal(got[k], ref[k]) for k in got), (cid, N, name)
                d = out.setdefault(f"{prob['cfg']['name']} N={N}", {}).setdefault(name, {"rollout_ms": [], "plan_ms": []})
                d["rollout_ms"].append(round(roll, 4))
                d["plan_ms"].append(round(wall, 3))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
