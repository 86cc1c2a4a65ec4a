"""Diagnostic: cProfile of the host side of bench plans (cheetah, the bench's kwargs without events):
which Python calls make up the ~66 us before the C call. Usage: python tools/host_cprofile.py [plans]"""
import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402

from mbrl_amd import CEMPlanner, synthetic  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    prob = synthetic.make_problem(3)
    cfg = prob["cfg"]
    dev = torch.device("cuda:0")
    kw = dict(num_candidates=cfg["N"], num_elites=cfg["N"] // 10, num_iterations=5, alpha=0.1,
              seed=prob["rng_seed"], distributed=False, device=dev, precision="f32")

    def plan():
        return CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], cfg["H"], **kw)
    for _ in range(10):
        plan()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        plan()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
