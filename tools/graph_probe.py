"""Does a HIP graph of one whole mbrl_cem_plan shorten a small plan? Times, per plan, on one GPU:
  direct  -- mbrl_cem_plan enqueued from the host, then a stream sync;
  graph   -- the same call captured once (torch.cuda.CUDAGraph around the C call, fixed s0 / seed /
             outputs), replayed, then a stream sync;
  plan()  -- the public CEMPlanner.plan (host tensors back).
Usage: python tools/graph_probe.py [config_id] [plans]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd")]

import torch  # noqa: E402

from mbrl_amd import CEMPlanner, _lib, fused, synthetic  # noqa: E402


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    dev = torch.device("cuda:0")
    p = synthetic.make_problem(cid)
    cfg = p["cfg"]
    N, H = cfg["N"], cfg["H"]
    kw = dict(num_candidates=N, num_iterations=5, seed=p["rng_seed"], device=dev)
    for _ in range(5):
        CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], H, **kw)
    md, cd = fused.describe(p["model"], p["cost"], dev)
    prob = fused.device_problem(md, cd, dev)
    lib = _lib.load()
    a, s = md["a"], md["s"]
    params = _lib.CemParams(N, H, N // 10, 5, 0.1, -1.0, 1.0, 0.0, 0.5, 0, p["rng_seed"])
    need = lib.mbrl_cem_workspace_bytes(fused.ctypes_ref(prob.shape), fused.ctypes_ref(params))
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    s0 = p["s0"].to(dev)
    buf = torch.empty(H * (s + 3 * a), dtype=torch.float32, device=dev)
    states, actions = buf[:H * s], buf[H * s:H * (s + a)]
    mu, sigma = buf[H * (s + a):H * (s + 2 * a)], buf[H * (s + 2 * a):]

    def call():
        _lib.check(lib.mbrl_cem_plan(fused.ctypes_ref(prob.shape), _lib.ptr(prob.packed), fused.ctypes_ref(prob.norm),
                                     fused.ctypes_ref(prob.cost), _lib.ptr(s0), fused.ctypes_ref(params), _lib.ptr(mu),
                                     _lib.ptr(sigma), _lib.ptr(actions), _lib.ptr(states), None, None, None, None,
                                     _lib.ptr(ws), ws.numel(), _lib.stream_handle(dev)), "mbrl_cem_plan")
    stream = torch.cuda.current_stream(dev)
    out = dict(config=cfg["name"])

    def bench(fn, label):
        for _ in range(10):
            fn()
        stream.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
            stream.synchronize()
        out[label + "_us"] = (time.perf_counter() - t0) / n * 1e6
    bench(call, "direct")
    ref = buf.clone()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream(dev)
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        call()
    stream.wait_stream(side)
    with torch.cuda.graph(g):
        call()
    g.replay()
    stream.synchronize()
    out["graph_equals_direct"] = bool(torch.equal(buf, ref))
    bench(g.replay, "graph")
    bench(lambda: CEMPlanner.plan(p["s0"], p["model"], p["cost"], p["sample_action"], H, **kw), "plan")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
