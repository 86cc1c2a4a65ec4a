"""Golden fixtures for the gradient-descent planner: the REFERENCE's own
GradientDescentPlanner.plan (src/mbrl/planners.py:28-137) on synthetic problems, wired as
GoalStateAgent wires model and cost (agents.py:219-233).

    python tests/golden/make_golden_gd.py          (build container only; writes gd_*.npz)

Problems come from oracle.cem.synth_problem (weights pinned by SHA-256). The initial action
sequence is given explicitly (PCG64 seed 99), so no RNG is involved in the plan itself.

gd_toy_abs_H5 is the reference's own known-answer script, src/mbrl/test_gradient_planner.py:5-27
(s' = s + a, cost |s - 9|, s0 = [2], horizon 5, 40 Adam iterations, the initial sequence drawn by
sample_action = torch.randn((batch, 1)) under torch.manual_seed(0)); the draw is stored with it.
"""
import functools
import os
import sys

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from oracle import cem as ocem  # noqa: E402

CASES = {
    # name: (config id, overrides, horizon, num_iterations, stop_condition)
    "gd_config3_W50_H10": (3, dict(W=50, L=2), 10, 40, 0.002),
    "gd_config2_H12": (2, dict(), 12, 25, 0.0),
    "gd_config6_reward_W64_H8": (6, dict(W=64, L=2), 8, 30, 0.002),
}


def initial_actions(H, a):
    return np.random.Generator(np.random.PCG64(99)).uniform(-0.5, 0.5, (H, a)).astype(np.float32)


def main():
    sys.path.insert(0, REF)
    sys.path.insert(0, HERE)
    from src.mbrl import data, models, planners
    import make_golden as mg
    torch.set_num_threads(1)
    for name, (cid, over, H, iters, stop) in CASES.items():
        p = ocem.synth_problem(cid, **over)
        model_fn, cost_fn = mg.wire(data, models, p, p["model"][0])
        a = p["cfg"]["a"]
        A0 = initial_actions(H, a)
        init = ([], [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)])
        states, actions = planners.GradientDescentPlanner.plan(
            torch.from_numpy(p["s0"]), model_fn, cost_fn, None, H, init, num_iterations=iters,
            stop_condition=stop)
        st = torch.cat(states).numpy()
        ac = torch.cat(actions).numpy()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), weights_sha256=ocem.weights_sha256(p["model"]),
                            init_actions=A0, states=st, actions=ac)
        print(name, "states", st.shape, "actions[0]", ac[0])


TOY = dict(s0=2.0, goal=9.0, H=5, iterations=40, seed=0)


def toy_model(states, actions):
    """test_gradient_planner.py:13-14"""
    return states + actions


def toy_cost(states, actions, goal=torch.tensor(TOY["goal"], dtype=torch.float)):
    """test_gradient_planner.py:19-20"""
    return torch.abs(states - goal)


def main_toy():
    sys.path.insert(0, REF)
    from src.mbrl import planners
    torch.manual_seed(TOY["seed"])
    drawn = []

    def sample_action(batch_size):   # test_gradient_planner.py:16-17, recording the draw
        x = torch.randn((batch_size, 1))
        drawn.append(x.clone())
        return x

    states, actions = planners.GradientDescentPlanner.plan(
        torch.tensor([TOY["s0"]], dtype=torch.float), toy_model, toy_cost, sample_action, TOY["H"], None,
        num_iterations=TOY["iterations"])
    st = torch.cat(states).numpy()
    ac = torch.cat(actions).numpy()
    total = float(toy_cost(torch.stack(states), torch.cat(actions)).sum())
    np.savez_compressed(os.path.join(HERE, "gd_toy_abs_H5.npz"), sampled=drawn[0].numpy(), states=st, actions=ac,
                        total_cost=np.float32(total))
    print("gd_toy_abs_H5 states", st.ravel(), "actions", ac.ravel(), "cost", total)


if __name__ == "__main__":
    main()
    main_toy()
