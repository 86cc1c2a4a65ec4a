"""Batched planning throughput (mbrl_cem_plan_batch): B environments' CEM plans per call on one GPU.

    python tools/batch_bench.py [config] [B ...]    -> one JSON line per B

Small-N configurations fill few CUs per plan (cartpole N=1024: 64 workgroups); batching B plans
into shared launches multiplies the work per launch. Reports plans/s and candidate-timesteps/s."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402

from mbrl_amd import CEMPlanner, synthetic  # noqa: E402


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    Bs = [int(x) for x in sys.argv[2:]] or [1, 4, 16]
    prob = synthetic.make_problem(cid)
    cfg = prob["cfg"]
    N, H = cfg["N"], cfg["H"]
    dev = torch.device("cuda", 0)
    for B in Bs:
        S0 = prob["s0"].unsqueeze(0).repeat(B, 1) + 0.01 * torch.arange(B, dtype=torch.float32).unsqueeze(1)
        kw = dict(num_candidates=N, num_iterations=5, seed=prob["rng_seed"], device=dev, return_device=True)
        for _ in range(3):
            CEMPlanner.plan_batch(S0, prob["model"], prob["cost"], prob["sample_action"], H, **kw)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            CEMPlanner.plan_batch(S0, prob["model"], prob["cost"], prob["sample_action"], H, **kw)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        print(json.dumps(dict(workload=f"{cfg['name']} N={N} H={H} I=5", B=B, ms_per_call=dt * 1e3,
                              plans_per_s=B / dt, cand_steps_per_s=5 * B * N * H / dt)))


if __name__ == "__main__":
    main()
