"""Planner service vs per-worker planning for parallel rollouts.

B workers each run one cartpole-shaped stand-in environment for S steps with an MPC policy
(CEMPlanner, N=1024, H=20, 2x256 model):
  served      the workers step environments, the parent plans each lockstep round with one
              CEMPlanner.plan_batch (mbrl_amd.parallel's service);
  per-worker  the policy is pickled into the workers and each plans on the GPU itself (the
              reference's parallel.py arrangement): B GPU contexts, B single plans per round.
Each mode runs S/10 and S steps; the difference gives the steady-state time per round (worker
start-up cancels). Prints one JSON line per mode.
Usage: python tools/service_bench.py [--workers 8] [--steps 300]
"""
import argparse
import functools
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tests")]

import torch  # noqa: E402

import standin_env as se  # noqa: E402
from mbrl_amd import CEMPlanner, MPCPolicy, data, models, parallel  # noqa: E402
from mbrl_amd import env as menv  # noqa: E402
from mbrl_amd import env_wrappers as ew  # noqa: E402


class PolicyAction:
    """A picklable get_action that is not a bound policy method: the service does not take it, so
    every worker plans for itself."""

    def __init__(self, policy):
        self.policy = policy

    def __call__(self, state_and_obs):
        return self.policy.get_action(state_and_obs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--candidates", type=int, default=1024)
    args = ap.parse_args()
    torch.manual_seed(0)
    m = models.Model(5, 1, hidden_units=256, n_hidden=2)
    ds = data.TransitionsDataset.from_statistics({"observations": {"mean": torch.zeros(5), "std": torch.ones(5)},
                                                  "actions": {"mean": torch.zeros(1), "std": torch.ones(1)}})
    cost = models.goal_state_cost(models.SmoothAbsLoss(torch.ones(5), torch.zeros(5)), models.CoshLoss())
    sample_action = functools.partial(ew.EnvWrapper._sample_action, action_spec=menv.BoundedActionSpec(1))
    model_fn = functools.partial(m, **ds.normalizers())
    pol = MPCPolicy(model_fn, cost, CEMPlanner, sample_action, 20, num_candidates=args.candidates, seed=5,
                    device="cuda")
    B, S = args.workers, args.steps
    # warm the parent's GPU path once (extension load, weight upload, workspaces)
    CEMPlanner.plan_batch(torch.zeros(B, 5), model_fn, cost, sample_action, 20, num_candidates=args.candidates,
                          seed=5, device="cuda")
    torch.cuda.synchronize()
    for mode in ("served", "per-worker"):
        ga = pol.get_action if mode == "served" else PolicyAction(pol)
        times = {}
        for steps in (S // 10, S):
            rounds = []
            t0 = time.perf_counter()
            rs = parallel.get_rollouts_parallel("linear", "run", True, B, dict(num_steps=steps, get_action=ga),
                                                num_workers=B, env_factory=se.make_env,
                                                on_batch=lambda i, o, a: rounds.append(len(i)))
            times[steps] = time.perf_counter() - t0
            assert len(rs) == B and all(len(r) == steps for r in rs)
        # steady state: the extra steps of the long run over the short one (worker start-up cancels)
        per_round = (times[S] - times[S // 10]) / (S - S // 10)
        print(json.dumps(dict(mode=mode, workers=B, steps=S, candidates=args.candidates, horizon=20,
                              seconds=times[S], steady_ms_per_round=per_round * 1e3,
                              steady_env_steps_per_s=B / per_round,
                              steady_candidate_timesteps_per_s=B * 5 * args.candidates * 20 / per_round,
                              startup_s=times[S] - S * per_round,
                              gpu_contexts=1 if mode == "served" else B + 1)), flush=True)


if __name__ == "__main__":
    main()
