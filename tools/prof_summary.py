"""Summarise a rocprofv3 kernel trace of `bench.py` for profiles/: the rollout kernel's mean duration
over the TIMED dispatches (the last steps x 5 rollout launches, as bench.py's HIP events see them)
next to the all-dispatch mean rocprof's --stats reports, and bench.py's own figure.

    python tools/prof_summary.py <prof dir> <bench json log> <steps> <out json> [kernel substring]

The kernel substring defaults to "rollout_kernel<" (the F32 rollout); "rollout_split_kernel" selects
the F16X3 kernel (its fp32 redo pass is a separate, near-empty rollout_kernel launch)."""
import csv
import glob
import json
import os
import sys


def main():
    d, bench_log, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    pat = sys.argv[5] if len(sys.argv) > 5 else "rollout_kernel<"
    trace = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    roll = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace))
            if pat in r["Kernel_Name"]]
    roll.sort()
    dur = [(e - s) / 1e6 for s, e in roll]
    timed = dur[-steps * 5:]
    # the bench line is the last line that parses as a JSON object (rocprofv3 logs to the same file)
    bench = [json.loads(l) for l in open(bench_log) if l.startswith('{"metric"')][-1]
    res = dict(kernel=pat, dispatches=len(dur), all_mean_ms=sum(dur) / len(dur),
               timed_dispatches=len(timed), timed_mean_ms=sum(timed) / len(timed),
               bench_events_mean_ms=bench["roofline"]["avg_launch_ms"],
               note="rocprofv3 --kernel-trace --stats of `python3 bench.py --steps %d --warmup 3 "
                    "--no-cpu-baseline`; timed = the last steps*5 rollout dispatches" % steps)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
