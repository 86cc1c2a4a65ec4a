"""Diagnostic: per-segment cycle shares of the rollout kernel from the -DMBRL_STAMPS build.

    make -C mujoco-mbrl_amd diag && python tools/stamps.py [config_id]

Only shares are meaningful (the stamps' own waits perturb the schedule); never quote its time."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd",
                                         os.environ.get("MBRL_DIAG_LIB", "libmbrl_cem_diag.so"))
sys.path.insert(0, os.path.join(REPO, "mujoco-mbrl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, fused, synthetic  # noqa: E402

SEGS = ["layer0 mma", "layer0 store+bar", "hidden mma", "hidden store+bar", "output mma", "output bar",
        "epilogue+bar"]
NSEG = 8   # slot 7: s_memrealtime ticks (100 MHz) over the same loop -> the shader clock


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    over = {"N": int(sys.argv[2])} if len(sys.argv) > 2 else {}
    prob = synthetic.make_problem(cid, **over)
    cfg = prob["cfg"]
    N, H, a, E = cfg["N"], cfg["H"], cfg["a"], cfg["E"]
    lib = _lib.load()
    lib.mbrl_diag_set_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    md = fused.describe_model(prob["model"])
    cd = fused.describe_cost(prob["cost"], md["s"], md)
    p = fused.device_problem(md, cd, dev)
    R = 2 if (N >= 2 * 16 * 256 and md["W"] <= 512) else 1
    tiles = (N + 16 * R - 1) // (16 * R)
    if os.environ.get("MBRL_ROLLOUT_M") == "8":     # rollout_m8_kernel: 8 candidates per workgroup
        R, tiles = 0.5, (N + 7) // 8
        lib.mbrl_set_option(_lib.OPTIONS["rollout_tile"], 8)   # the library reads no environment
    NWMAX = 8   # waves per workgroup (4 or 8); unused slots stay zero and are dropped below
    buf = torch.zeros(E * tiles * NWMAX * NSEG, dtype=torch.int64, device=dev)
    assert lib.mbrl_diag_set_stamps(buf.data_ptr()) == 0
    mu = torch.zeros((H, a), device=dev)
    sg = torch.full((H, a), 0.5, device=dev)
    acts = torch.empty((H, N, a), device=dev)
    s0 = prob["s0"].to(dev)
    for _ in range(3):
        fused.rollout(p, s0, N, H, sampler=fused.make_sampler(1, 0, mu, sg, -1, 1), actions_out=acts)
    torch.cuda.synchronize()
    st = buf.view(E * tiles * NWMAX, NSEG).cpu().numpy().astype(np.float64)
    if os.environ.get("MBRL_STAMPS_BY_WAVE"):      # per wave slot: waves 0-3 state epilogue, 4-7 actions
        byw = st.reshape(-1, NWMAX, NSEG)
        for w in range(NWMAX):
            sw = byw[:, w, :]
            sw = sw[sw.sum(1) > 0]
            if len(sw):
                print(f"  wave {w}: " + " ".join(f"{v / H:8.0f}" for v in sw[:, :7].mean(0)))
    st = st[st.sum(1) > 0]
    ghz = st[:, :7].sum(1).mean() / (st[:, 7].mean() * 10.0)
    per_step = st[:, :7].mean(0) / H
    tot = per_step.sum()
    print(f"  shader clock over the step loop: {ghz:.2f} GHz (s_memtime / s_memrealtime)")
    print(f"config {cid} N={N} R={R} tiles={tiles}: mean cycles per step per wave {tot:.0f} (diag build; shares only)")
    for name, v in zip(SEGS, per_step):
        print(f"  {name:18s} {v:9.0f}  {100 * v / tot:5.1f}%")
    mfma = int(2176 * R) if cid in (3, 4) and R >= 1 else None
    if mfma:
        print(f"  ideal MFMA issue per step per wave: {mfma * 32} cycles; hidden-loop efficiency "
              f"{2048 * R * 32 / per_step[2]:.3f}")


if __name__ == "__main__":
    main()
