"""Where the split update's time goes at a walker rank (N = 16384 selected, 2048 drawn, G = 8): per
workgroup s_memrealtime stamps (-DMBRL_STAMPS library) of cem_select_regen_kernel (start, selection
done, end) and cem_refit_draw_kernel (start, sums done, end), from rank 7's emulated plan
(MBRL_OPT_SHARD_EMULATE = 2, as tools/rank_split.py). Per iteration and kernel: the workgroups' start
spread, median / max of each phase, and the span (first start to last end); the gap from the emulated
gather's end to the selection's first start (the launch of cem_select_regen_kernel, last iteration) and
from the selection's last end to the sums' first start (the kernel boundary between the two). Times in us
(100 MHz clock). (profiles/r06/split_stamps_j_s*.jsonl came from a diagnostic build whose S -- the
workgroups per row -- an environment variable overrode; that override is gone.)
Usage: python tools/split_stamps.py [config] [gpus]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so")
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import ITERATIONS  # noqa: E402
from mbrl_amd import CEMPlanner, _lib, fused, planners, synthetic  # noqa: E402


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    buf = torch.zeros(8 * 2 * 1024 * 4, dtype=torch.int64, device=dev)
    sel = torch.zeros(16, dtype=torch.int64, device=dev)   # workgroup 0: selection (CSTAMP 0-5), sums (8-12)
    lib.mbrl_diag_set_cem_wg_stamps.argtypes = [ctypes.c_void_p]
    lib.mbrl_diag_set_cem_stamps.argtypes = [ctypes.c_void_p]
    p = synthetic.make_problem(cid)
    cfg = p["cfg"]
    N = cfg["N"]
    md, cd = fused.describe(p["model"], p["cost"], dev)
    prob = fused.device_problem(md, cd, dev)
    kw = dict(num_candidates=N, num_elites=N // 10, num_iterations=ITERATIONS, seed=p["rng_seed"], device=dev)
    st = CEMPlanner._settings(p["sample_action"], cfg["H"], kw)
    s0 = p["s0"].cpu().float()
    with _lib.option("shard_emulate", 1):
        planners._cem_sharded_native(prob, s0.to(dev), st, world, 0, comm=None)
    rows, sels = [], []
    with _lib.option("shard_emulate", 2):
        for k in range(12):
            assert lib.mbrl_diag_set_cem_wg_stamps(buf.data_ptr() if k >= 2 else None) == 0
            assert lib.mbrl_diag_set_cem_stamps(sel.data_ptr() if k >= 2 else None) == 0
            buf.zero_()
            sel.zero_()
            torch.cuda.synchronize()
            planners._cem_sharded_native(prob, s0, st, world, world - 1, comm=None)
            torch.cuda.synchronize()
            if k >= 2:
                rows.append(buf.view(8, 2, 1024, 4).cpu().numpy().copy())
                sels.append(sel.cpu().numpy().copy())
    assert lib.mbrl_diag_set_cem_wg_stamps(None) == 0
    assert lib.mbrl_diag_set_cem_stamps(None) == 0
    d = np.diff(np.array(sels, dtype=np.float64)[:, :6], axis=1).mean(0) / 100.0
    sel_phases = dict(zip(["load+minmax", "wide", "list", "passes", "compaction"], [round(float(x), 2) for x in d]))
    sm = np.array(sels, dtype=np.float64)[:, 8:13]
    d = np.diff(sm, axis=1).mean(0) / 100.0
    sums_phases = dict(zip(["pass0 chunk sums", "pass0 sequential", "pass1 chunk sums", "pass1 sequential"],
                           [round(float(x), 2) for x in d]))
    print(json.dumps({"last_iteration_selection_phases_us": sel_phases,
                      "last_iteration_sums_phases_us (refit_draw workgroup 0)": sums_phases}), flush=True)
    out = dict(config=cid, workload=cfg["name"], N=N, gpus=world, rank=world - 1, plans=len(rows), iterations={},
               last_iteration_selection_phases_us=sel_phases)
    names = (("select_regen", "select", "regen", None), ("refit_draw", "sums", "draw", "staged"))
    for it in range(ITERATIONS):
        per = {}
        for q, (kern, p1, p2, p3) in enumerate(names):
            acc = []
            for r in rows:
                st_ = r[it, q]
                used = st_[:, 0] > 0
                if not used.any():
                    continue
                s = st_[used].astype(np.float64) / 100.0
                t0 = s[:, 0].min()
                acc.append(dict(wgs=int(used.sum()), start_spread=s[:, 0].max() - t0,
                                p1_med=np.median(s[:, 1] - s[:, 0]), p1_max=(s[:, 1] - s[:, 0]).max(),
                                p2_med=np.median(s[:, 2] - s[:, 1]) if (s[:, 2] > 0).all() else None,
                                p3_med=np.median(s[:, 3] - s[:, 0]) if (s[:, 3] > 0).all() else None,
                                span=(s[:, 2].max() if (s[:, 2] > 0).all() else s[:, 1].max()) - t0))
            if acc:
                per[kern] = {"wgs": acc[0]["wgs"]}
                for key, label in (("start_spread", "start_spread"), ("p1_med", p1 + "_median"),
                                   ("p1_max", p1 + "_max"), ("p2_med", p2 + "_median"), ("span", "span"),
                                   ("p3_med", (p3 or "") + "_from_start_median")):
                    if key == "p3_med" and p3 is None:
                        continue
                    vals = [a[key] for a in acc if a[key] is not None]
                    per[kern][label] = round(float(np.mean(vals)), 2) if vals else None
        gaps = []
        for r in rows:
            a, b = r[it, 0], r[it, 1]
            ua, ub = a[:, 0] > 0, b[:, 0] > 0
            if ua.any() and ub.any() and (a[ua, 2] > 0).all():
                gaps.append((b[ub, 0].min() - a[ua, 2].max()) / 100.0)
        per["gap_select_end_to_sums_start"] = round(float(np.mean(gaps)), 2) if gaps else None
        if it == ITERATIONS - 1:
            lead = [(r[it, 0][r[it, 0][:, 0] > 0, 0].min() - r.reshape(-1)[-1]) / 100.0 for r in rows
                    if r.reshape(-1)[-1] > 0]
            per["gap_gather_end_to_select_start"] = round(float(np.mean(lead)), 2) if lead else None
        out["iterations"][it] = per
        print(json.dumps({"iteration": it, **per}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
