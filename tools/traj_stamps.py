"""Diagnostic: segment times of the cooperative trajectory kernel (traj.hip) from the -DMBRL_STAMPS build.

    make -C mujoco-mbrl_amd diag && python tools/traj_stamps.py [config_id] [traj_hop option]

s_memrealtime ticks (100 MHz) summed per workgroup over the horizon; printed per step in microseconds."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so")
sys.path.insert(0, os.path.join(REPO, "mujoco-mbrl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import CEMPlanner, _lib, synthetic  # noqa: E402

SEGS = ["actions+layer0", "hidden dot+publish", "gather wait", "output+state"]


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    hop = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    prob = synthetic.make_problem(cid)
    cfg = prob["cfg"]
    N, H, E, W = cfg["N"], cfg["H"], cfg["E"], cfg["W"]
    lib = _lib.load()
    lib.mbrl_diag_set_traj_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    P = ((W + 63) // 64 * 64) // 16
    buf = torch.zeros(E * P * len(SEGS), dtype=torch.int64, device=dev)
    assert lib.mbrl_diag_set_traj_stamps(buf.data_ptr()) == 0
    lib.mbrl_set_option(_lib.OPTIONS["traj_hop"], hop)
    for _ in range(3):
        CEMPlanner.plan_detailed(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], H,
                                 num_candidates=N, num_elites=N // 10, num_iterations=5, alpha=0.1,
                                 seed=prob["rng_seed"], device=dev)
    torch.cuda.synchronize()
    st = buf.view(E * P, len(SEGS)).cpu().numpy().astype(np.float64) / 100.0 / H   # us per step
    print(f"config {cid}: coop trajectory kernel (traj_hop option {hop}), {E * P} workgroups, us per step "
          f"(mean / max over WGs)")
    for k, name in enumerate(SEGS):
        print(f"  {name:20s} {st[:, k].mean():7.2f} {st[:, k].max():7.2f}")
    print(f"  {'total':20s} {st.sum(1).mean():7.2f}  -> {st.sum(1).mean() * H:.0f} us per launch")


if __name__ == "__main__":
    main()
