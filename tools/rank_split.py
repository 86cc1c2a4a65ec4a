"""Per-rank-faithful multi-GPU projection on ONE GPU.

A G-rank sharded plan on rank r runs: its shard's rollout (N/G candidates), the all-gather, the update
over ALL N candidates with K = N/10 (selection + refit + its own shard's next draw), and the trajectory.
This tool times exactly that with mbrl_cem_plan_sharded under MBRL_OPT_SHARD_EMULATE = 2: one mode-1
plan first keeps every iteration's gathered costs in the workspace, then each timed call fills the other
ranks' slots from them in one launch per iteration (a stand-in for the all-gather, counted in the time)
and does nothing else beyond the rank's own work. The result is checked bit-identical to the
single-GPU plan before timing.

Per row: the rank's wall time per plan (host s0 in, host results out, as bench.py's plans) and its device
span; the single-GPU plan of the full N timed the same way beside it; projected speed-up =
T1 / (T_rank + I * allgather_us), both timed without timing events (ms_per_plan; the evented loop that
gives the device span and the rollout launch is ms_per_plan_with_events). The all-gather itself cannot
run on one GPU: its allowance is an ASSUMPTION, reported at 10 / 25 / 40 us per iteration (RCCL
all-gather of 8 x 16-64 KB over xGMI).

  strong rows (--mode strong): config N split over G ranks (walker N=16384: 2048 per rank at G=8).
  weak rows   (--mode weak):   n_local per rank fixed (cheetah 4096), N = G * n_local, K = N/10.

Usage: python tools/rank_split.py [--mode strong|weak] [--configs 3 4 5] [--gpus 2 4 8] [--plans 30]
One JSON line per row on stdout (and --out FILE)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import ITERATIONS, MEASURED_IT, TimingEvent  # noqa: E402
from mbrl_amd import CEMPlanner, _lib, fused, planners, synthetic  # noqa: E402

ALLGATHER_US = (10.0, 25.0, 40.0)
T1_MS = None   # --t1-ms: the single-GPU plan's time given (profiling runs time the rank's plan only)


def _time(fn, plans, warmup):
    """fn(plan_events, rollout_events): warm-up, then `plans` timed calls; the plan's device span and
    iteration MEASURED_IT's rollout launch from fence-free events (as bench.py)."""
    for _ in range(warmup):
        fn(None, None)
    torch.cuda.synchronize()
    pev = [(TimingEvent(), TimingEvent()) for _ in range(plans)]
    rev = [[(TimingEvent(), TimingEvent()) if it == MEASURED_IT else None for it in range(ITERATIONS)]
           for _ in range(plans)]
    for pair in pev + [r[MEASURED_IT] for r in rev]:
        pair[0].record()
        pair[1].record()
    torch.cuda.synchronize()
    walls = []
    t0 = time.perf_counter()
    for k in range(plans):
        t = time.perf_counter()
        fn(pev[k], rev[k])
        walls.append(time.perf_counter() - t)
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()
    span = float(np.mean([a.elapsed_time(b) for a, b in pev]))
    roll = float(np.mean([r[MEASURED_IT][0].elapsed_time(r[MEASURED_IT][1]) for r in rev]))
    # the same plans again with no timing events (each record leaves the GPU idle a few us, 4 per plan
    # above): the production-like figure the projection uses, for T1 and the rank alike
    t0 = time.perf_counter()
    for k in range(plans):
        fn(None, None)
    torch.cuda.synchronize()
    plain = (time.perf_counter() - t0) / plans * 1e3
    return dict(ms_per_plan=plain, ms_per_plan_with_events=elapsed / plans * 1e3, plan_gpu_ms=span,
                wall_median_ms=float(np.median(walls)) * 1e3, rollout_ms=roll)


def row(cid, world, n_total, plans, warmup, dev, mode):
    p = synthetic.make_problem(cid)
    cfg = p["cfg"]
    H, E = cfg["H"], cfg["E"]
    K = n_total // 10
    md, cd = fused.describe(p["model"], p["cost"], dev)
    prob = fused.device_problem(md, cd, dev)
    kw = dict(num_candidates=n_total, num_elites=K, num_iterations=ITERATIONS, seed=p["rng_seed"], device=dev)
    st = CEMPlanner._settings(p["sample_action"], H, kw)
    st_rec = CEMPlanner._settings(p["sample_action"], H, dict(kw, record=True))
    s0_host = p["s0"].cpu().float()
    s0_dev = s0_host.to(dev)

    def single(pev, rev):
        return planners._cem_fused_single(prob, s0_host, dict(st, plan_events=pev, events=rev))

    rank = world - 1   # every rank does the same work; the last one's shard is the last candidates

    def sharded(pev, rev):
        return planners._cem_sharded_native(prob, s0_host, dict(st, plan_events=pev, events=rev), world, rank,
                                            comm=None)

    # bit-identity first: mode 1 (keeps the gathered costs), then mode 2, against the single-GPU plan
    ref = planners._cem_fused_single(prob, s0_dev, st_rec)
    with _lib.option("shard_emulate", 1):
        planners._cem_sharded_native(prob, s0_dev, st_rec, world, 0, comm=None)
    with _lib.option("shard_emulate", 2):
        got = planners._cem_sharded_native(prob, s0_dev, st_rec, world, rank, comm=None)
        for k in ("elites", "mu", "sigma", "actions", "states"):
            assert torch.equal(torch.as_tensor(got[k]).cpu(), torch.as_tensor(ref[k]).cpu()), (cid, world, k)
        t_rank = _time(sharded, plans, warmup)
    t_one = _time(single, plans, warmup) if T1_MS is None else dict(ms_per_plan=T1_MS, given=True)
    out = dict(config=cid, workload=cfg["name"], mode=mode, gpus=world, rank=rank, N=n_total,
               candidates_per_rank=n_total // world, K=K, H=H, E=E, rank_plan=t_rank, single_gpu_plan=t_one,
               bit_identical=True, allgather_us_assumed=list(ALLGATHER_US))
    if mode == "strong":
        base = out["t1_ms"] = t_one["ms_per_plan"]   # the full-N plan on one GPU
        out["projected_speedup"] = {f"{a:g}us": base / (t_rank["ms_per_plan"] + ITERATIONS * a / 1e3)
                                    for a in ALLGATHER_US}
        if "ms_per_plan_with_events" in t_one:
            out["projected_speedup_with_events"] = {
                f"{a:g}us": t_one["ms_per_plan_with_events"] / (t_rank["ms_per_plan_with_events"] + ITERATIONS * a / 1e3)
                for a in ALLGATHER_US}
    else:
        # weak: per-GPU work fixed; efficiency = (single GPU at n_local) / (rank's plan at N = G n_local)
        out["projected_weak_efficiency"] = {}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="strong", choices=["strong", "weak"])
    ap.add_argument("--configs", type=int, nargs="+", default=[3, 4, 5])
    ap.add_argument("--gpus", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--plans", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n-local", type=int, default=None, help="weak mode: candidates per rank (default config N)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--t1-ms", type=float, default=None, help="strong mode: the single-GPU plan's ms (not timed)")
    ap.add_argument("--option", action="append", default=[], help="NAME=VALUE: an mbrl_set_option for the run (A/B)")
    args = ap.parse_args()
    for o in args.option:
        name, val = o.split("=")
        _lib.load().mbrl_set_option(_lib.OPTIONS[name], int(val))
    global T1_MS
    T1_MS = args.t1_ms
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    f = open(args.out, "a") if args.out else None
    for cid in args.configs:
        cfg = synthetic.CONFIGS[cid]
        plans = max(3, args.plans // (20 if cfg["E"] > 1 else 1))
        base_one = None
        for world in args.gpus:
            if args.mode == "strong":
                r = row(cid, world, cfg["N"], plans, min(args.warmup, plans), dev, "strong")
            else:
                n_local = args.n_local or cfg["N"]
                r = row(cid, world, n_local * world, plans, min(args.warmup, plans), dev, "weak")
                if base_one is None:   # the 1-GPU plan at n_local candidates, timed the same way
                    p = synthetic.make_problem(cid)
                    md, cd = fused.describe(p["model"], p["cost"], dev)
                    prob = fused.device_problem(md, cd, dev)
                    st = CEMPlanner._settings(p["sample_action"], cfg["H"], dict(
                        num_candidates=n_local, num_elites=n_local // 10, num_iterations=ITERATIONS,
                        seed=p["rng_seed"], device=dev))
                    s0 = p["s0"].cpu().float()
                    base_one = _time(lambda pev, rev: planners._cem_fused_single(prob, s0, dict(st, plan_events=pev,
                                                                                                 events=rev)),
                                     plans, min(args.warmup, plans))
                r["one_gpu_n_local_plan"] = base_one
                r["projected_weak_efficiency"] = {
                    f"{a:g}us": base_one["ms_per_plan"] / (r["rank_plan"]["ms_per_plan"] + ITERATIONS * a / 1e3)
                    for a in ALLGATHER_US}
            if args.option:
                r["options"] = args.option
            line = json.dumps(r)
            print(line, flush=True)
            # a bench.py-shaped line for tools/plan_timeline.py (rocprofv3 runs of this tool)
            rp = r["rank_plan"]
            flop = r["candidates_per_rank"] * r["H"] * synthetic.flop_per_candidate_step(cfg)
            print(json.dumps({"metric": "rank plan", "ms_per_step": rp["ms_per_plan"],
                              "config": {"workload": f"{cfg['name']} N={r['N']} G={world} rank {r['rank']}",
                                         "candidates_per_gpu": r["candidates_per_rank"]},
                              "roofline": {"avg_launch_ms": rp["rollout_ms"],
                                           "frac": flop / (rp["rollout_ms"] * 1e-3) / 1e12 / 157.3}}), flush=True)
            if f:
                f.write(line + "\n")
                f.flush()
    if f:
        f.close()


if __name__ == "__main__":
    main()
