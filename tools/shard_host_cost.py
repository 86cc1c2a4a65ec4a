"""What the sharded plan costs over the one-call single-GPU plan (mbrl_cem_plan): the one-call C path
(mbrl_cem_plan_sharded, the all-gather a step on the plan's stream) and the per-iteration protocol
(planners.cem_sharded_protocol: rollout, RCCL all-gather, update, issued from Python each iteration),
on one GPU with a one-rank RCCL process group (the collective really runs; RCCL refuses two ranks on
one device). Per plan: wall time with a stream sync, and the host time spent issuing it.
Usage: python tools/shard_host_cost.py [config_id] [candidates] [plans]"""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mbrl_amd import CEMPlanner, fused, planners, synthetic  # noqa: E402


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n_cand = int(sys.argv[2]) if len(sys.argv) > 2 else None
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with tempfile.TemporaryDirectory() as d:
        dist.init_process_group("nccl", init_method=f"file://{os.path.join(d, 'pg')}", rank=0, world_size=1)
        try:
            p = synthetic.make_problem(cid)
            cfg = p["cfg"]
            N = n_cand or cfg["N"]
            H = cfg["H"]
            kw = dict(num_candidates=N, num_iterations=5, seed=p["rng_seed"], device=dev)
            md, cd = fused.describe(p["model"], p["cost"], dev)
            prob = fused.device_problem(md, cd, dev)
            st = CEMPlanner._settings(p["sample_action"], H, dict(kw, return_device=True))
            s0 = p["s0"].to(dev)
            stream = torch.cuda.current_stream(dev)

            def single():
                return planners._cem_fused_single(prob, s0, st)

            def native():
                planners.SHARDED_NATIVE = True
                return planners._cem_fused_sharded(prob, s0, st, 1)

            def protocol():
                planners.SHARDED_NATIVE = False
                return planners._cem_fused_sharded(prob, s0, st, 1)

            out = dict(config=cfg["name"], candidates=N)
            for label, fn in (("single", single), ("sharded_native", native), ("sharded_protocol", protocol)) * 2:
                for _ in range(5):
                    fn()
                stream.synchronize()
                host = 0.0
                t0 = time.perf_counter()
                for _ in range(n):
                    h0 = time.perf_counter()
                    fn()
                    host += time.perf_counter() - h0
                    stream.synchronize()
                out.setdefault(label + "_ms", []).append(round((time.perf_counter() - t0) / n * 1e3, 4))
                out.setdefault(label + "_host_issue_us", []).append(round(host / n * 1e6, 1))
            print(json.dumps(out))
        finally:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
