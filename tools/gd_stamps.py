"""Diagnostic: segment times of the cooperative gradient-descent kernel (gd.hip) from the -DMBRL_STAMPS
build, per step (forward + backward of one horizon step) in microseconds.

    make -C mujoco-mbrl_amd diag && python tools/gd_stamps.py [config_id]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so")
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, gd, synthetic  # noqa: E402

SEGS = ["fwd layer 0", "fwd hidden (hand-offs)", "fwd output + x0", "bwd output layer", "bwd hidden (hand-offs)",
        "bwd layer 0", "adam + stop (per iteration)"]


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    iters = 40
    prob = synthetic.make_problem(cid)
    cfg = prob["cfg"]
    H, a, W = cfg["H"], cfg["a"], cfg["W"]
    lib = _lib.load()
    lib.mbrl_diag_set_gd_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    P = ((W + 63) // 64 * 64) // 16
    buf = torch.zeros(P * len(SEGS), dtype=torch.int64, device=dev)
    assert lib.mbrl_diag_set_gd_stamps(buf.data_ptr()) == 0
    A0 = np.random.Generator(np.random.PCG64(99)).uniform(-0.5, 0.5, (H, a)).astype(np.float32)
    acts = [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)]
    md, cd = gd.describe(prob["model"], prob["cost"], dev)
    for _ in range(2):
        gd.plan_device(prob["s0"], md, cd, acts, H, iters, 0.0, dev, use_fused=True)
    torch.cuda.synchronize()
    st = buf.view(P, len(SEGS)).cpu().numpy().astype(np.float64) / 100.0   # us per launch
    per = np.array([iters * H] * 6 + [iters], dtype=np.float64)
    print(f"config {cid}: cooperative gd kernel, {P} workgroups, {iters} iterations x H={H}; us per step "
          f"(mean / max over workgroups)")
    for k, name in enumerate(SEGS):
        print(f"  {name:30s} {st[:, k].mean() / per[k]:7.3f} {st[:, k].max() / per[k]:7.3f}")
    tot = st[:, :6].sum(1).mean() / (iters * H) + st[:, 6].mean() / (iters * H)
    print(f"  {'total per step':30s} {tot:7.3f}")


if __name__ == "__main__":
    main()
