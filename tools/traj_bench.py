"""Duration of the final-mean trajectory kernel (mbrl_trajectory: traj_reg_kernel for Wpad <= 256,
traj_coop_kernel for Wpad 512) against the horizon: the slope is the per-step cost, the intercept the
prologue (weights into registers / LDS). Run under rocprofv3 --kernel-trace, then parse the trace:
  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/traj -o run -- python3 tools/traj_bench.py
  python3 tools/traj_bench.py --parse gpurun_out/traj"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

CIDS = (2, 3)
WARM, REPS = 5, 50


def horizons(H):
    return sorted({1, 2, 5, 10, H})


def run():
    import torch
    from mbrl_amd import fused, synthetic
    dev = torch.device("cuda", 0)
    for cid in CIDS:
        p = synthetic.make_problem(cid)
        cfg = p["cfg"]
        md, cd = fused.describe(p["model"], p["cost"], dev)
        prob = fused.device_problem(md, cd, dev)
        s0 = torch.as_tensor(p["s0"], dtype=torch.float32, device=dev)
        for H in horizons(cfg["H"]):
            acts = torch.rand((H, cfg["a"]), device=dev) * 2 - 1
            for _ in range(WARM + REPS):
                fused.trajectory(prob, s0, acts, H)
            torch.cuda.synchronize()


def parse(d):
    import numpy as np
    from mbrl_amd import synthetic
    path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    # the working kernel of each launch: traj_reg / traj_coop (traj_coop's gated fallback traj_kernel
    # launch follows it and returns at once)
    rows = [r for r in csv.DictReader(open(path)) if "traj_reg" in r["Kernel_Name"] or "traj_coop" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    i = 0
    for cid in CIDS:
        cfg = synthetic.CONFIGS[cid]
        hs, us, name = horizons(cfg["H"]), [], None
        for H in hs:
            blk = rows[i + WARM:i + WARM + REPS]
            i += WARM + REPS
            name = blk[0]["Kernel_Name"].split("(")[0]
            us.append(float(np.mean([int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in blk])) / 1e3)
        slope, icpt = np.polyfit(np.array(hs, float), np.array(us), 1)
        print(json.dumps(dict(config=cfg["name"], kernel=name, H=hs, us_per_launch=[round(u, 2) for u in us],
                              us_per_step=round(float(slope), 3), intercept_us=round(float(icpt), 2))))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run()
