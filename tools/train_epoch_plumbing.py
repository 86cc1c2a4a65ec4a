"""Diagnostic: what train_model's per-epoch plumbing costs the GPU. 50 epochs issued back to back from
one order (bare), then the same with one piece of the epoch loop's plumbing added per epoch: a
fence-free event recorded on the training stream; the training stream waiting on an event recorded
(and complete) on the side stream; a side-stream copy of a ring row plus that wait; the full ring
(draw, copy, waits, records); device us per step between two events. Usage:
python tools/train_epoch_plumbing.py [epochs] [reps]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "mujoco-mbrl_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import train_bench  # noqa: E402
from mbrl_amd import _lib, models  # noqa: E402
from mbrl_amd.optim import AdamStep  # noqa: E402


def main():
    epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda:0")
    ds = train_bench.dataset()
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=512).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    np.random.seed(1)
    for n in (10, 50, 50):
        m.train_model(ds, opt, batch_size=512, num_epochs=n)
    torch.cuda.synchronize()
    n = ds.num_transitions()
    steps = epochs * ((n + 511) // 512)
    native = models._NATIVE_CACHE[m][1]
    fast = AdamStep.maybe(opt)
    ring = models._order_ring(dev, n)
    main_s = torch.cuda.current_stream(dev)
    order = ring.rows(0)[1]
    ev = _lib.StreamEvent()
    ev.record(ring.side)
    ring.draw(0)
    ring.copy(0, main_s)
    torch.cuda.synchronize()

    def span(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / steps

    def bare():
        for _ in range(epochs):
            native.epoch(order, 512, fast)

    def record():
        for e in range(epochs):
            native.epoch(order, 512, fast)
            ring.consumed[e % ring.K].record(main_s)

    def wait():
        for _ in range(epochs):
            ev.wait(main_s)
            native.epoch(order, 512, fast)

    def copy_wait():
        for e in range(epochs):
            if e:
                ring.copied[e % ring.K].wait(main_s)
            native.epoch(ring.rows(e)[1], 512, fast)
            ring.draw(e + 1)                    # (valid row indices in every row the copy reads)
            ring.copy(e + 1, ring.side)

    def ring_exact():
        # train_model's epoch loop, statement for statement, around the cached objects
        ring.draw(0)
        ring.copy(0, main_s)
        losses = []
        for e in range(epochs):
            if e:
                ring.copied[e % ring.K].wait(main_s)
            losses.append(native.epoch(ring.rows(e)[1], 512, fast))
            if e + 1 < epochs:
                ring.draw(e + 1)
                ring.copy(e + 1, ring.side)
            ring.consumed[e % ring.K].record(main_s)
        native.check_status()

    def ring_nosync():
        # the same loop without the host's wait on `consumed` (rows are reused while an epoch may still
        # read them: a timing probe only -- every index stays valid)
        ring.draw(0)
        ring.copy(0, main_s)
        for e in range(epochs):
            if e:
                ring.copied[e % ring.K].wait(main_s)
            native.epoch(ring.rows(e)[1], 512, fast)
            if e + 1 < epochs:
                r = (e + 1) % ring.K
                ring.draw(e + 1)
                with torch.cuda.stream(ring.side):
                    ring.dev[r, :ring.n].copy_(ring.pinned[r, :ring.n], non_blocking=True)
                    ring.copied[r].record(ring.side)
            ring.consumed[e % ring.K].record(main_s)
        native.check_status()

    def full():
        m.train_model(ds, opt, batch_size=512, num_epochs=epochs)

    out = {}
    for _ in range(reps):
        for name, fn in (("bare", bare), ("record", record), ("wait", wait), ("copy_wait", copy_wait),
                         ("ring_exact", ring_exact), ("ring_nosync", ring_nosync), ("train_model", full)):
            out.setdefault(name, []).append(round(span(fn), 2))
    out["epochs"], out["steps"] = epochs, steps
    print(json.dumps(out))


if __name__ == "__main__":
    main()
