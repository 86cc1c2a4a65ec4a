"""Soak of the cross-workgroup hand-offs: many repetitions of each path whose result depends on
one workgroup reading what another wrote during the same launch, each compared bit for bit with
the path's first result (and, for the pairs, with the 8-candidate tiles that need no hand-off):
* column-split pair rollouts (the same-XCD L2 hand-offs and the tagged output granules) in whole
  walker / cheetah plans at the 2048-candidate shard size, with the gated redo launch dropped
  (MBRL_OPT_DEBUG_PAIR_ABORT = 2), so a timed-out or stale hand-off shows as a different plan;
* the cooperative trajectory kernel (its L2 granule gathers) inside the same plans (states);
* the cooperative gradient-descent planner (hop hand-offs every layer of every Adam step); its
  one-workgroup fallback sums in another order, so a timeout also shows as a different plan;
* the training step's band waits (F -> O inside one launch) and arrival waits (dH_0 -> dW_1), over
  a long train_model call: the sticky status word is read at its end and must be clear, and the
  weights must equal a run of the three-launch layout (MBRL_OPT_TRAIN_FO = 1).
Usage: python tools/soak.py [seconds_per_part] [parts: any of cem,gd,train; default all]. Prints one
JSON line per part and a summary."""
import json
import os
import sys
import time
from contextlib import ExitStack

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import CEMPlanner, _lib, gd, models, synthetic  # noqa: E402

DEV = torch.device("cuda:0")
KEYS = ("states", "actions", "mu", "sigma")


def _options(opts):
    stack = ExitStack()
    for name, value in opts.items():
        stack.enter_context(_lib.option(name, value))
    return stack


def cem_part(cfg_id, N, seconds, opts, ref_opts):
    prob = synthetic.make_problem(cfg_id)
    H = prob["cfg"]["H"]
    kw = dict(num_candidates=N, num_elites=N // 10, num_iterations=5, alpha=0.1, seed=prob["rng_seed"],
              device=DEV, return_device=True)

    def plan(o):
        with _options(o):
            res = CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], H, **kw)
        return [res[k].clone() for k in KEYS]

    ref = plan(ref_opts)
    first = plan(opts)
    same_as_ref = all(torch.equal(x, y) for x, y in zip(first, ref))
    bad, n, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        got = plan(opts)
        n += 1
        if not all(torch.equal(x, y) for x, y in zip(got, first)):
            bad += 1
    torch.cuda.synchronize()
    return dict(part=f"cem config {cfg_id} N={N} {opts}", plans=n, mismatches=bad, first_equals_reference=same_as_ref)


def gd_part(seconds):
    prob = synthetic.make_problem(3)
    mdesc, cdesc = gd.describe(prob["model"], prob["cost"], DEV)
    H, a = 30, prob["cfg"]["a"]
    rng = np.random.default_rng(5)
    acts = [torch.from_numpy(rng.uniform(-1, 1, (1, a)).astype(np.float32)) for _ in range(H)]
    s0 = prob["s0"]

    def plan():
        s, ac, it = gd.plan_fused(s0, mdesc, cdesc, acts, H, 40, 0.0, DEV)
        return s.clone(), ac.clone(), int(it.item())

    first = plan()
    bad, n, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        got = plan()
        n += 1
        if not (torch.equal(got[0], first[0]) and torch.equal(got[1], first[1]) and got[2] == first[2]):
            bad += 1
    return dict(part="gd cooperative cheetah 3x512 H=30, 40 Adam iterations", plans=n, mismatches=bad)


def train_part(seconds):
    import train_bench
    ds = train_bench.dataset()

    def run(epochs, fo_split):
        torch.manual_seed(0)
        m = models.Model(17, 6, hidden_units=512).to(DEV)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        np.random.seed(1)
        with _lib.option("train_fo", fo_split):
            m.train_model(ds, opt, batch_size=512, num_epochs=epochs)   # raises if the status word is set
        torch.cuda.synchronize()
        return [p.detach().clone() for p in m.parameters()]

    run(5, 0)                                   # first call: bindings, ring, clocks
    t0 = time.perf_counter()
    run(20, 0)
    per_epoch = (time.perf_counter() - t0) / 20
    epochs = max(10, int(seconds / max(per_epoch, 1e-4) / 2))
    fused = run(epochs, 0)
    split = run(epochs, 1)
    same = all(torch.equal(x, y) for x, y in zip(fused, split))
    steps = epochs * ((ds.num_transitions() + 511) // 512)
    return dict(part="train_model 2x512 batch 512, FO launch vs F and O apart", epochs=epochs, steps=steps,
                status="clear", mismatches=0 if same else 1)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    which = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else {"cem", "gd", "train"}
    parts = []
    pair = {"rollout_pair": 1, "debug_pair_abort": 2}
    m8 = {"rollout_tile": 8, "rollout_pair": 2}
    if "cem" in which:
        for cfg_id, N in ((4, 2048), (3, 2048)):
            parts.append(cem_part(cfg_id, N, seconds, pair, m8))
            print(json.dumps(parts[-1]), flush=True)
        parts.append(cem_part(3, 4096, seconds, {}, {"traj_hop": 1}))     # the bench plan; trajectory hop modes
        print(json.dumps(parts[-1]), flush=True)
    if "gd" in which:
        parts.append(gd_part(seconds))
        print(json.dumps(parts[-1]), flush=True)
    if "train" in which:
        parts.append(train_part(seconds))
        print(json.dumps(parts[-1]), flush=True)
    bad = sum(p["mismatches"] for p in parts) + sum(1 for p in parts if p.get("first_equals_reference") is False)
    print(json.dumps(dict(summary=True, parts=len(parts), failures=bad, seconds_per_part=seconds)))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
