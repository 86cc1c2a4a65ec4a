"""Counter-derived MFMA utilisation of the rollout kernel per config, from tools/mfma_pmc.sh output:
per dispatch (averaged over the timed launches), FLOP issued = SQ_INSTS_VALU_MFMA_MOPS_F32 x 512, the
clock = GRBM_GUI_ACTIVE / 8 XCDs / duration, util_issue = FLOP issued / (active cycles x 65536 FLOP per
chip cycle: 256 CUs x 4 SIMDs x 64 fp32 MFMA FLOP/clk, 157.3 TF at 2.4 GHz), and the busy-cycle form
SQ_VALU_MFMA_BUSY_CYCLES / (active cycles x 1024 SIMDs) (rocprofv3's MfmaUtil); beside the
FLOP-derived frac = algorithmic FLOP / (duration x 157.3 TF) that bench.py reports.
Usage: python tools/mfma_util.py <out dir> [label ...]"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

from mbrl_amd import synthetic  # noqa: E402

CFG = {"c2": (2, None), "c3": (3, None), "c4": (4, None), "c4s2048": (4, 2048), "c5": (5, None), "c6": (6, None)}


def summarise(d, label):
    cid, n = CFG[label]
    cfg = synthetic.make_problem(cid)["cfg"]
    N = n or cfg["N"]
    flop_alg = N * cfg["H"] * synthetic.flop_per_candidate_step(cfg)
    rows = {}
    for f in glob.glob(os.path.join(d, label, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Dispatch_Id"]
            rows.setdefault(k, dict(kernel=r["Kernel_Name"], t=(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9))
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
    # the dominant kernel (most total time; a column-split pair launch is followed by its gated redo
    # launch, whose workgroups exit at once), its last 15 dispatches: the bench's 3 timed plans x 5
    by = {}
    for x in rows.values():
        by.setdefault(x["kernel"], []).append(x)
    kern = max(by, key=lambda k: sum(x["t"] for x in by[k]))
    disp = by[kern][-15:]
    avg = lambda k: sum(x[k] for x in disp) / len(disp)  # noqa: E731
    t = avg("t")
    grbm = avg("GRBM_GUI_ACTIVE") / 8
    flop_issued = avg("SQ_INSTS_VALU_MFMA_MOPS_F32") * 512
    out = dict(label=label, kernel=disp[0]["kernel"], dispatches=len(disp), duration_ms=t * 1e3,
               clock_ghz=grbm / t / 1e9, flop_alg=flop_alg, flop_issued=flop_issued,
               padding=flop_issued / flop_alg - 1, frac_flop=flop_alg / t / 157.3e12,
               util_issue=flop_issued / (grbm * 65536), frac_issued_at_2p4=flop_issued / t / 157.3e12,
               sq_valu_mfma_busy_cycles=avg("SQ_VALU_MFMA_BUSY_CYCLES"), sq_busy_cu_cycles=avg("SQ_BUSY_CU_CYCLES"))
    # SQ_VALU_MFMA_BUSY_CYCLES summed over the SIMDs: its MfmaUtil form (rocprofv3's derived counter)
    # is busy / (GRBM_GUI_ACTIVE max over XCDs x 1024 SIMDs); it reads 2139095040 (0x7F800000, the
    # bits of +inf) on some dispatches -- a saturated value, reported as null
    busy = out["sq_valu_mfma_busy_cycles"]
    sat = any(x["SQ_VALU_MFMA_BUSY_CYCLES"] == 2139095040.0 for x in disp)
    out["mfma_util_busy"] = None if sat else busy / (grbm * 1024)
    out["mfma_busy_saturated"] = sat
    out["other_kernels"] = {k: dict(dispatches=len(v), mean_ms=sum(x["t"] for x in v) / len(v) * 1e3)
                            for k, v in by.items() if k != kern}
    del out["sq_valu_mfma_busy_cycles"], out["sq_busy_cu_cycles"]
    return out


def main():
    d = sys.argv[1]
    for label in sys.argv[2:] or CFG:
        if os.path.isdir(os.path.join(d, label)):
            print(json.dumps(summarise(d, label)))


if __name__ == "__main__":
    main()
