"""Per-plan GPU timeline from a rocprofv3 kernel trace of `bench.py` (profiles/ summaries).

    python tools/plan_timeline.py <prof dir> <bench json log> <steps> <out json>

A plan starts at its fill2_kernel or cem_init_kernel (mbrl_cem_plan's first launch). Over the last `steps` plans (the
timed ones) it reports: the rollout kernel's mean dispatch duration next to bench.py's HIP-event
figure (they must agree: the roofline's `achieved` divides by the latter), GPU busy time per kernel
family per plan, the idle gaps inside a plan (launch-to-launch), and the idle time between plans
(the host's turn: result copy, Python, the next C call)."""
import csv
import glob
import json
import os
import re
import sys

FAMILIES = [("rollout", r"rollout(_m8|_split)?_kernel<"), ("update", r"cem_update_kernel"), ("sample", r"sample_kernel"),
            ("select", r"select(_reg)?_kernel|select_regen"), ("allgather_emulated", r"emu_gather_kernel"),
            ("refit", r"refit|gather_elites|finalize_kernel"),
            ("trajectory", r"traj(_coop|_reg)?_kernel|member_mean"), ("fill", r"fill2_kernel|cem_init_kernel"),
            ("memset", r"fillBuffer|[Mm]emset")]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def main():
    d, bench_log, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(trace)))
    starts = [i for i, r in enumerate(rows) if "fill2_kernel" in r[2] or "cem_init_kernel" in r[2]]
    plans = [rows[a:b] for a, b in zip(starts, starts[1:] + [len(rows)])][-steps:]
    fams = sorted({family(r[2]) for p in plans for r in p})
    busy = {f: 0.0 for f in fams}
    count = {f: 0 for f in fams}
    span = gaps = 0.0
    for p in plans:
        span += (p[-1][1] - p[0][0]) / 1e3
        gaps += ((p[-1][1] - p[0][0]) - sum(e - s for s, e, _ in p)) / 1e3
        for s, e, n in p:
            busy[family(n)] += (e - s) / 1e3
            count[family(n)] += 1
    between = [(b[0][0] - a[-1][1]) / 1e3 for a, b in zip(plans, plans[1:])]
    # the dominant rollout kernel by total time (a column-split pair launch is followed by its gated
    # redo launch, whose workgroups exit at once: that one is reported apart)
    tot = {}
    for p in plans:
        for s, e, n in p:
            if family(n) == "rollout" and "split" not in n:
                tot[n] = tot.get(n, 0) + (e - s)
    roll_name = max(tot, key=tot.get) if tot else ""
    roll = [(e - s) / 1e6 for p in plans for s, e, n in p if n == roll_name]
    other_roll = {n: dict(dispatches=sum(1 for p in plans for s, e, m in p if m == n),
                          mean_us=v / 1e3 / max(1, sum(1 for p in plans for s, e, m in p if m == n)))
                  for n, v in tot.items() if n != roll_name}
    bench = [json.loads(l) for l in open(bench_log) if l.startswith('{"metric"')][-1]
    P = len(plans)
    res = dict(
        workload=bench["config"]["workload"], candidates_per_gpu=bench["config"]["candidates_per_gpu"],
        plans=P, rollout_kernel=roll_name, rollout_dispatches=len(roll), other_rollout_kernels=other_roll,
        rollout_mean_ms=sum(roll) / max(1, len(roll)), bench_events_mean_ms=bench["roofline"]["avg_launch_ms"],
        bench_frac=bench["roofline"]["frac"], bench_ms_per_plan=bench["ms_per_step"],
        plan_span_us=span / P, plan_gaps_us=gaps / P,
        between_plans_us=sum(between) / max(1, len(between)),
        between_plans_median_us=(sorted(between)[len(between) // 2] if between else 0.0),   # (one slow host turn moves the mean)
        busy_us_per_plan={f: busy[f] / P for f in fams}, launches_per_plan={f: count[f] / P for f in fams},
        note=f"rocprofv3 --kernel-trace --stats of bench.py ({steps} timed plans); under the profiler, "
             "so ms_per_plan is a little above the unprofiled bench line")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
