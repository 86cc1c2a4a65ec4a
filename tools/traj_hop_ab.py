"""A/B of the cooperative trajectory kernel's hand-off placement (MBRL_OPT_TRAJ_HOP 1 / 2 / 3: (P, E)
grid with sc1 granules, per-member XCD grid with sc1 granules, XCD grid with L2-resident granules
after the XCC_ID roll call): mbrl_trajectory (memset + coop kernel + gated fallback launch) timed with
fence-free HIP events, rounds interleaved; states must be bit-identical across modes.
Usage: python tools/traj_hop_ab.py [rounds]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from mbrl_amd import _lib, fused, synthetic  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda", 0)
    res = {}
    for cid in (3, 4, 5, 6):
        p = synthetic.make_problem(cid)
        cfg = p["cfg"]
        md, cd = fused.describe(p["model"], p["cost"], dev)
        prob = fused.device_problem(md, cd, dev)
        s0 = torch.as_tensor(p["s0"], dtype=torch.float32, device=dev)
        H = cfg["H"]
        acts = (torch.rand((H, cfg["a"]), device=dev, generator=torch.Generator(device=dev).manual_seed(cid)) * 2 - 1)
        ref = None
        for r in range(rounds):
            for mode in (1, 2, 3):
                with _lib.option("traj_hop", mode):
                    for _ in range(5):
                        st = fused.trajectory(prob, s0, acts, H)
                    ev = [(bench.TimingEvent(), bench.TimingEvent()) for _ in range(50)]
                    torch.cuda.synchronize()
                    for a, b in ev:
                        a.record()
                        st = fused.trajectory(prob, s0, acts, H)
                        b.record()
                    torch.cuda.synchronize()
                    us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
                if ref is None:
                    ref = st.clone()
                assert torch.equal(st, ref), (cid, mode)
                res.setdefault(f"{cfg['name']} H={H} E={cfg['E']}", {}).setdefault(f"hop{mode}", []).append(round(us, 1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
