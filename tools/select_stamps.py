"""Diagnostic: phase times of select_reg_kernel from the -DMBRL_STAMPS build (thread 0's
s_memrealtime, 100 MHz). make -C mujoco-mbrl_amd diag && python tools/select_stamps.py [N [lo hi]]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["MBRL_AMD_LIB"] = os.path.join(REPO, "mujoco-mbrl_amd", "mbrl_amd", "libmbrl_cem_diag.so")
sys.path.insert(0, os.path.join(REPO, "mujoco-mbrl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mbrl_amd import _lib, fused  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    lib = _lib.load()
    lib.mbrl_diag_set_cem_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    buf = torch.zeros(16, dtype=torch.int64, device=dev)
    assert lib.mbrl_diag_set_cem_stamps(buf.data_ptr()) == 0
    lo, hi = (float(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (120.0, 123.0)
    costs = torch.from_numpy(np.random.default_rng(0).uniform(lo, hi, N).astype(np.float32)).to(dev).view(1, N)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    rows = []
    for _ in range(20):
        fused.select(costs, N // 10, workspace=ws)
        torch.cuda.synchronize()
        rows.append(buf.cpu().numpy().copy())
    st = np.array(rows[5:], dtype=np.float64)
    d = np.diff(st[:, :6], axis=1).mean(0) / 100.0
    names = ["load+keys+minmax", "wide pass", "list", "8-bit passes", "compaction"]
    print(f"select_reg N={N}: us per phase (thread 0, mean of 15)")
    for n, v in zip(names, d):
        print(f"  {n:12s} {v:7.2f}")
    print(f"  {'total':12s} {d.sum():7.2f}")


if __name__ == "__main__":
    main()
