"""A/B of the cooperative gradient-descent kernel's hand-off placement (MBRL_OPT_GD_HOP 1 / 2 / 3, as
tools/traj_hop_ab.py): cheetah 3x512 (and the reward head), H = 30, 40 Adam iterations (no early stop),
one plan and a batch of 8; per-step time = plan time / (40 * H). Results must be bit-identical.
Usage: python tools/gd_hop_ab.py [rounds]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, gd, synthetic  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    iters = 40
    dev = torch.device("cuda:0")
    out = {}
    for cid in (3, 6):
        prob = synthetic.make_problem(cid)
        H, a = prob["cfg"]["H"], prob["cfg"]["a"]
        A0 = np.random.Generator(np.random.PCG64(99)).uniform(-0.5, 0.5, (H, a)).astype(np.float32)
        acts = [torch.from_numpy(A0[i:i + 1].copy()) for i in range(H)]
        md, cd = gd.describe(prob["model"], prob["cost"], dev)
        s0 = torch.as_tensor(np.asarray(prob["s0"], np.float32))
        S0 = torch.stack([s0 + 0.01 * k for k in range(8)])
        AB = torch.from_numpy(np.stack([A0] * 8))
        ref = None
        for _ in range(rounds):
            for mode in (1, 2, 3):
                with _lib.option("gd_hop", mode):
                    r = gd.plan_device(prob["s0"], md, cd, acts, H, iters, 0.0, dev, use_fused=True)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(5):
                        r = gd.plan_device(prob["s0"], md, cd, acts, H, iters, 0.0, dev, use_fused=True)
                    torch.cuda.synchronize()
                    ms1 = (time.perf_counter() - t0) * 1e3 / 5
                    rb = gd.plan_fused_batch(S0, md, cd, AB, H, iters, 0.0, dev)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(3):
                        rb = gd.plan_fused_batch(S0, md, cd, AB, H, iters, 0.0, dev)
                    torch.cuda.synchronize()
                    ms8 = (time.perf_counter() - t0) * 1e3 / 3
                flat = [r[0].reshape(-1).cpu(), r[1].reshape(-1).cpu()] + [x.reshape(-1).cpu() for x in rb]
                if ref is None:
                    ref = flat
                assert all(torch.equal(x, y) for x, y in zip(flat, ref)), (cid, mode)
                d = out.setdefault(f"{prob['cfg']['name']} H={H}", {}).setdefault(f"hop{mode}", {"plan_ms": [],
                                                                                                  "us_per_step": [],
                                                                                                  "batch8_ms": []})
                d["plan_ms"].append(round(ms1, 2))
                d["us_per_step"].append(round(ms1 * 1e3 / (iters * H), 2))
                d["batch8_ms"].append(round(ms8, 2))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
