"""Model training on the GPU: mbrl_train_grads (csrc/train.hip) -- the
batch loss gradient of Model / ModelWithReward under train_model's MSELoss -- against autograd on
the same batch, in fp32 on the same device.

The native kernels sum in a different order from autograd's GEMMs and reductions, so the bar is
rounding-level agreement: every gradient within 1e-4 relative of the tensor's largest autograd
entry (plus 1e-4 elementwise relative), losses within 1e-5 relative. End-to-end training parity
against the reference's own train_model is tests/test_train.py (1e-4 on the weights after
training), which runs this path by default."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _dataset(s, a, horizon, T, seed):
    from mbrl_amd import data
    rng = np.random.Generator(np.random.PCG64(seed))
    rolls = []
    per = T // 3 + horizon
    for _ in range(3):
        st = rng.standard_normal((per + 1, s)).astype(np.float32)
        rolls.append(data.Rollout(states=list(torch.from_numpy(st)), observations=list(torch.from_numpy(st)),
                                  actions=list(torch.from_numpy(rng.uniform(-1, 1, (per, a)).astype(np.float32))),
                                  rewards=list(torch.from_numpy(rng.standard_normal(per).astype(np.float32)))))
    ds = data.TransitionsDataset(rollouts=rolls, horizon=horizon)
    ds.set_data_mode("state_only")
    return ds


def _model(kind, s, a, W, L, seed):
    from mbrl_amd import models
    torch.manual_seed(seed)
    if kind == "model":
        return models.Model(s, a, hidden_units=W, n_hidden=L).to(DEV)
    return models.ModelWithReward(s, a, hidden_units=W, n_hidden=L).to(DEV)


def _autograd(m, ds, ins, outs, idx, reward):
    from mbrl_amd import models
    crit = torch.nn.MSELoss()
    for p in m.parameters():
        p.grad = None

    def step_loss(inp, out):
        (st, ac), (rw, ns) = inp, out
        if reward:
            sh, rh = m.forward(st, ac)
            return [crit(sh, ns), crit(rh, rw.reshape(-1, 1))]
        return [crit(m.forward(st, ac), ns)]
    loss, parts = models._batch_loss(ds, ins, outs, idx, step_loss, 2 if reward else 1)
    loss.backward()
    return loss.detach(), [p.grad.clone() for p in m.parameters()], [x.detach() for x in parts]


CASES = [("model", 17, 6, 512, 2, 1, 512), ("model", 17, 6, 50, 2, 1, 512), ("model", 5, 1, 64, 1, 2, 37),
         ("model", 24, 8, 200, 3, 3, 300), ("model", 3, 2, 33, 2, 1, 1), ("reward", 17, 6, 200, 2, 1, 512),
         ("reward", 11, 3, 96, 2, 2, 129), ("model", 67, 21, 128, 2, 1, 256), ("model", 17, 6, 512, 2, 1, 200)]


@pytest.mark.parametrize("kind,s,a,W,L,H,B", CASES)
def test_native_gradients_match_autograd(kind, s, a, W, L, H, B):
    from mbrl_amd import models
    ds = _dataset(s, a, H, max(3 * B, 60), seed=s * 7 + W)
    m = _model(kind, s, a, W, L, seed=W)
    _, ins, outs = ds.stacked(DEV)
    reward = kind == "reward"
    assert models._NativeGrads.supported(m, ds, ins, outs, torch.nn.MSELoss()) == reward
    g = torch.Generator().manual_seed(B)
    idx = torch.randperm(ds.num_transitions(), generator=g)[:B].to(DEV)
    ref_loss, ref_grads, ref_parts = _autograd(m, ds, ins, outs, idx, reward)
    nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
    loss, parts = nat.run(idx)
    torch.cuda.synchronize()
    got = [p.grad for p in m.parameters()]
    for i, (x, y) in enumerate(zip(got, ref_grads)):
        scale = float(y.abs().max())
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-4 * scale + 1e-12), (i, float((x - y).abs().max()), scale)
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * abs(float(ref_loss))
    for k, rp in enumerate(ref_parts):
        assert abs(float(parts[k]) - float(rp)) <= 1e-5 * abs(float(rp))


def test_native_training_tracks_autograd_training():
    """Ten epochs of train_model (Adam) through the native gradients and through autograd end within
    1e-4 of each other (fp32 summation-order differences, amplified by Adam's normalisation)."""
    from mbrl_amd import models
    ds = _dataset(17, 6, 2, 900, seed=3)
    out = {}
    for native in (True, False):
        m = _model("model", 17, 6, 64, 2, seed=0)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        saved = models.NATIVE_TRAINING
        models.NATIVE_TRAINING = native
        try:
            np.random.seed(4)
            m.train_model(ds, opt, batch_size=128, num_epochs=10)
        finally:
            models.NATIVE_TRAINING = saved
        out[native] = [p.detach().cpu() for p in m.parameters()]
    for x, y in zip(out[True], out[False]):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-5), float((x - y).abs().max())


def test_native_training_declines_other_criteria_and_models():
    from mbrl_amd import models
    ds = _dataset(4, 2, 1, 60, seed=1)
    _, ins, outs = ds.stacked(DEV)
    m = _model("model", 4, 2, 16, 2, seed=0)
    assert models._NativeGrads.supported(m, ds, ins, outs, torch.nn.L1Loss()) is None
    assert models._NativeGrads.supported(m, ds, ins, outs, torch.nn.MSELoss(reduction="sum")) is None
    noisy = models.Model(4, 2, hidden_units=16, noise=0.1).to(DEV)
    assert models._NativeGrads.supported(noisy, ds, ins, outs, torch.nn.MSELoss()) is None
    assert models._NativeGrads.supported(m, ds, ins, outs, torch.nn.MSELoss()) is False


class _Writer:
    def __init__(self):
        self.rows = []

    def add_scalar(self, tag, value, step):
        self.rows.append((tag, float(value), int(step)))


@pytest.mark.parametrize("kind", ["model", "reward"])
def test_epoch_call_equals_per_batch_calls(kind, monkeypatch):
    """mbrl_train_epoch (every batch's gradient and Adam step from one host call) trains to the same
    bits as one mbrl_train_grads + mbrl_adam_step per batch, leaves the same optimizer state and
    step counters, and hands the writer the same per-batch losses."""
    from mbrl_amd import models
    ds = _dataset(17, 6, 2, 700, seed=9)
    out = {}
    for epoch_call in (True, False):
        m = _model(kind, 17, 6, 96, 2, seed=1)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4)
        w = _Writer()
        with monkeypatch.context() as mp:
            if not epoch_call:
                mp.setattr(models._NativeGrads, "epoch", lambda self, *a: None)
            np.random.seed(2)
            m.train_model(ds, opt, batch_size=128, num_epochs=3, writer=w)
        torch.cuda.synchronize()
        out[epoch_call] = ([p.detach().cpu() for p in m.parameters()],
                           [(float(s["step"]), s["exp_avg"].cpu(), s["exp_avg_sq"].cpu()) for s in opt.state.values()],
                           w.rows)
    (wa, sa, ra), (wb, sb, rb) = out[True], out[False]
    assert all(torch.equal(x, y) for x, y in zip(wa, wb))
    for (ka, ma, va), (kb, mb, vb) in zip(sa, sb):
        assert ka == kb and torch.equal(ma, mb) and torch.equal(va, vb)
    assert ra == rb and len(ra) > 0


def test_native_training_leaves_the_last_batch_gradient():
    """After train_model, every .grad holds the last batch's gradient, as after the reference's loop
    (zero_grad, backward, step per batch)."""
    from mbrl_amd import models
    ds = _dataset(7, 2, 1, 300, seed=4)
    m = _model("model", 7, 2, 32, 2, seed=2)
    opt = torch.optim.SGD(m.parameters(), lr=0.0)          # lr 0: the weights stay put
    np.random.seed(6)
    m.train_model(ds, opt, batch_size=64, num_epochs=1)
    got = [p.grad.clone() for p in m.parameters()]
    np.random.seed(6)
    order = models._epoch_order(ds)
    last = torch.from_numpy(order[(len(order) - 1) // 64 * 64:]).to(DEV)
    _, ins, outs = ds.stacked(DEV)
    _, ref, _ = _autograd(m, ds, ins, outs, last, False)
    for x, y in zip(got, ref):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-4 * float(y.abs().max()) + 1e-12)


def test_cached_native_object_trains_like_a_fresh_one():
    """train_model reuses the model's _NativeGrads (gradients, workspace) across calls while nothing it
    binds changed. Three calls with the cache equal three calls that each start from a fresh object,
    bit for bit; growing the dataset (new stacked tensors) or the batch size rebuilds it. The order
    ring is kept across the grown dataset (same power-of-two capacity), and a fresh ring per call
    trains to the same bits."""
    from mbrl_amd import models
    out = {}
    for cached in (True, False):
        ds = _dataset(17, 6, 1, 700, seed=11)
        m = _model("model", 17, 6, 512, 2, seed=3)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        np.random.seed(8)
        objs, rings = [], []
        for call, bs in enumerate((512, 512, 256, 512)):
            if not cached:
                models._NativeGrads.forget(m)
                models._ORDER_RINGS.clear()
            if call == 3:   # a grown dataset: new stacked tensors
                extra = _dataset(17, 6, 1, 90, seed=12)
                ds.add_rollouts(extra.rollouts)
            m.train_model(ds, opt, batch_size=bs, num_epochs=2)
            objs.append(models._NATIVE_CACHE.get(m, (None, None))[1])
            rings.append(models._order_ring(DEV, ds.num_transitions()))
        out[cached] = [p.detach().cpu() for p in m.parameters()]
        if cached:
            assert objs[0] is objs[1]            # same binding: reused
            assert objs[2] is not objs[1]        # batch size changed
            assert objs[3] is not objs[2]        # dataset grew
            assert rings[3] is rings[0] and rings[3].n == ds.num_transitions() < rings[3].cap
    assert all(torch.equal(x, y) for x, y in zip(out[True], out[False]))


@pytest.mark.parametrize("case", range(24))
def test_native_gradients_random_shapes(case):
    """mbrl_train_grads at random shapes (dims, widths off the tile grid, depth, horizon, batch sizes
    that leave partial row tiles, both model kinds) against autograd on the same batch."""
    from mbrl_amd import models
    rng = np.random.default_rng(5000 + case)
    kind = "reward" if case % 4 == 3 else "model"
    s, a = int(rng.integers(1, 40)), int(rng.integers(1, 12))
    W = int(rng.choice([1, 7, 16, 31, 64, 97, 128, 200, 256, 333]))
    L = int(rng.integers(1, 5))
    H = int(rng.integers(1, 4))
    B = int(rng.choice([1, 3, 32, 33, 100, 257]))
    ds = _dataset(s, a, H, max(3 * B, 40), seed=case)
    m = _model(kind, s, a, W, L, seed=case)
    _, ins, outs = ds.stacked(DEV)
    reward = kind == "reward"
    g = torch.Generator().manual_seed(case)
    idx = torch.randperm(ds.num_transitions(), generator=g)[:B].to(DEV)
    ref_loss, ref_grads, _ = _autograd(m, ds, ins, outs, idx, reward)
    nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
    loss, _ = nat.run(idx)
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip([p.grad for p in m.parameters()], ref_grads)):
        scale = float(y.abs().max())
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-4 * scale + 1e-12), (i, s, a, W, L, H, B)
    assert abs(float(loss) - float(ref_loss)) <= 1e-5 * abs(float(ref_loss)) + 1e-12


@pytest.mark.parametrize("kind,s,a,W,L,H,B", [("model", 17, 6, 512, 2, 1, 512), ("model", 24, 8, 512, 3, 2, 300),
                                             ("reward", 17, 6, 512, 2, 1, 512), ("model", 5, 1, 256, 2, 1, 1000)])
def test_backward_tile_height_is_bitwise_neutral(kind, s, a, W, L, H, B):
    """The W x W backward products run on 64 x 32 C tiles when 32 x 32 tiles would need a second round
    of the CUs (2 x 512 at batch 512: dH_0 and dW_1 are 256 tiles each). Every element keeps its K
    order (the K split over the 16 waves does not depend on the tile), so gradients and losses equal
    the 32-row path (MBRL_OPT_TRAIN_TILE = 32) bit for bit, as do the epoch's fused Adam steps."""
    from mbrl_amd import _lib, models
    ds = _dataset(s, a, H, max(3 * B, 60), seed=s * 7 + W)
    m = _model(kind, s, a, W, L, seed=W)
    _, ins, outs = ds.stacked(DEV)
    reward = kind == "reward"
    idx = torch.randperm(ds.num_transitions(), generator=torch.Generator().manual_seed(B))[:B].to(DEV)
    res = {}
    for tile in (32, 64, 0):
        with _lib.option("train_tile", tile):
            nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
            loss, parts = nat.run(idx)
            torch.cuda.synchronize()
            res[tile] = [loss.clone()] + [p.grad.clone() for p in m.parameters()]
    for tile in (64, 0):
        for x, y in zip(res[tile], res[32]):
            assert torch.equal(x, y), tile


@pytest.mark.parametrize("kind,W,L,H,B", [("model", 512, 2, 1, 512), ("model", 96, 2, 1, 300), ("model", 64, 3, 2, 50),
                                         ("reward", 200, 2, 1, 400), ("reward", 64, 1, 1, 500),
                                         ("model", 128, 1, 2, 60)])
def test_layer0_gradient_fold_is_bitwise_neutral(kind, W, L, H, B):
    """The layer-0 weight gradient folded into the dH_0 launch (per-32-row partials of each dH_0 tile,
    summed in wave order by the last tile of a column block; layer 0's Adam step there, layer 1's in the
    next batch's first launch) against its own launch (MBRL_OPT_TRAIN_NO_FOLD): the same gradients and
    losses from mbrl_train_grads, and the same parameters, optimizer state and losses after three epochs
    of mbrl_train_epoch with the last batch partial."""
    from mbrl_amd import _lib, models
    ds = _dataset(17, 6, H, 3 * B + 37, seed=W + L)
    _, ins, outs = ds.stacked(DEV)
    reward = kind == "reward"
    idx = torch.randperm(ds.num_transitions(), generator=torch.Generator().manual_seed(B))[:B].to(DEV)
    grads, trained = {}, {}
    for no_fold in (1, 0):
        with _lib.option("train_no_fold", no_fold):
            m = _model(kind, 17, 6, W, L, seed=W)
            nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
            loss, parts = nat.run(idx)
            torch.cuda.synchronize()
            grads[no_fold] = [loss.clone()] + [p.grad.clone() for p in m.parameters()]
            m = _model(kind, 17, 6, W, L, seed=W)
            opt = torch.optim.Adam(m.parameters(), lr=1e-3)
            w = _Writer()
            np.random.seed(3)
            m.train_model(ds, opt, batch_size=B, num_epochs=3, writer=w)
            torch.cuda.synchronize()
            trained[no_fold] = ([p.detach().clone() for p in m.parameters()],
                                [(float(s["step"]), s["exp_avg"].clone(), s["exp_avg_sq"].clone())
                                 for s in opt.state.values()], w.rows)
    assert all(torch.equal(x, y) for x, y in zip(grads[0], grads[1]))
    (pa, sa, ra), (pb, sb, rb) = trained[0], trained[1]
    assert all(torch.equal(x, y) for x, y in zip(pa, pb))
    for (ka, ma, va), (kb, mb, vb) in zip(sa, sb):
        assert ka == kb and torch.equal(ma, mb) and torch.equal(va, vb)
    assert ra == rb and len(ra) > 0


@pytest.mark.parametrize("kind,s,a,W,H,B", [("model", 17, 6, 512, 1, 512), ("reward", 17, 6, 512, 1, 512),
                                           ("reward", 17, 6, 200, 1, 400), ("model", 17, 6, 50, 1, 512),
                                           ("model", 24, 8, 333, 2, 150), ("model", 5, 1, 96, 1, 100),
                                           ("reward", 31, 33, 256, 1, 300), ("model", 11, 2, 512, 3, 171),
                                           ("model", 17, 6, 512, 1, 252), ("reward", 17, 6, 200, 1, 200)])
def test_fused_step_is_bitwise_neutral(kind, s, a, W, H, B):
    """Two hidden layers train in three launches (H_0 recomputed per H_1 tile, dY per dH_1 tile, the
    output layer's weight gradient folded; W_1's Adam step in the dH_0 launch after the tiles that
    read it) instead of five (MBRL_OPT_TRAIN_SPLIT = 1). The same chains in the same order: equal
    gradients and losses from mbrl_train_grads, and equal parameters, optimizer state and losses
    after three epochs of mbrl_train_epoch whose last batch is short (and takes the five-launch
    path); the status word of the bounded in-launch waits stays clear. The fused step is checked both
    as the default single F+O launch (band waits) and with F and O as two launches
    (MBRL_OPT_TRAIN_FO = 1), and with the backward tiles in XCD order (MBRL_OPT_TRAIN_XCD = 1, where
    the dW_1 tiles, not the last dH_0 row tiles, finish the dW_0 fold)."""
    import contextlib
    from mbrl_amd import _lib, models
    ds = _dataset(s, a, H, 3 * B + 37, seed=W + s)
    _, ins, outs = ds.stacked(DEV)
    reward = kind == "reward"
    idx = torch.randperm(ds.num_transitions(), generator=torch.Generator().manual_seed(B))[:B].to(DEV)
    grads, trained = {}, {}
    for split in (1, 0, "fo_split", "xcd"):
        with contextlib.ExitStack() as opts:
            opts.enter_context(_lib.option("train_split", 1 if split == 1 else 0))
            opts.enter_context(_lib.option("train_fo", 1 if split == "fo_split" else 0))
            opts.enter_context(_lib.option("train_xcd", 1 if split == "xcd" else 0))
            m = _model(kind, s, a, W, 2, seed=W)
            nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
            loss, parts = nat.run(idx)
            torch.cuda.synchronize()
            grads[split] = [loss.clone(), parts[0].clone(), parts[1].clone()] + [p.grad.clone() for p in m.parameters()]
            nat.check_status()
            m = _model(kind, s, a, W, 2, seed=W)
            opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4 if reward else 0.0)
            w = _Writer()
            np.random.seed(3)
            m.train_model(ds, opt, batch_size=B, num_epochs=3, writer=w)
            torch.cuda.synchronize()
            trained[split] = ([p.detach().clone() for p in m.parameters()],
                              [(float(st["step"]), st["exp_avg"].clone(), st["exp_avg_sq"].clone())
                               for st in opt.state.values()], w.rows)
    for mode in (0, "fo_split", "xcd"):
        for i, (x, y) in enumerate(zip(grads[mode], grads[1])):
            assert torch.equal(x, y), (mode, i, float((x - y).abs().max()))
        (pa, sa, ra), (pb, sb, rb) = trained[mode], trained[1]
        for i, (x, y) in enumerate(zip(pa, pb)):
            assert torch.equal(x, y), (mode, i, float((x - y).abs().max()))
        for (ka, ma, va), (kb, mb, vb) in zip(sa, sb):
            assert ka == kb and torch.equal(ma, mb) and torch.equal(va, vb)
        assert ra == rb and len(ra) > 0


@pytest.mark.parametrize("case", range(12))
def test_fused_step_random_shapes_bitwise(case):
    """The fused three-launch step against the five-launch layout at random shapes it accepts (two
    hidden layers, s + a <= 64, J <= 32, W <= 512, batch rows in the dW_0 fold's ranges): gradients and
    losses bit for bit, and the status word clear."""
    from mbrl_amd import _lib, models
    rng = np.random.default_rng(7000 + case)
    kind = "reward" if case % 3 == 2 else "model"
    s = int(rng.integers(1, 31 if kind == "reward" else 32))
    a = int(rng.integers(1, 64 - s + 1))
    W = int(rng.choice([33, 50, 64, 97, 128, 200, 255, 256, 333, 400, 512]))
    H = int(rng.integers(1, 3))
    lo, hi = [(64, 128), (128, 255), (256, 512)][int(rng.integers(0, 3))]
    B = int(rng.integers(lo // H + 1, hi // H + 1))
    R = B * H
    nw = 16 if R >= 256 else 8 if R > 128 else 4   # train.hip fold_waves: the fused step needs per == 2
    assert lo < R <= hi and (((R + 15) // 16 + nw - 1) // nw) == 2
    ds = _dataset(s, a, H, 3 * B + 5, seed=case)
    _, ins, outs = ds.stacked(DEV)
    reward = kind == "reward"
    idx = torch.randperm(ds.num_transitions(), generator=torch.Generator().manual_seed(case))[:B].to(DEV)
    got = {}
    for split in (1, 0):
        with _lib.option("train_split", split):
            m = _model(kind, s, a, W, 2, seed=case)
            nat = models._NativeGrads(m, ins, outs, ds.horizon, B, reward)
            loss, parts = nat.run(idx)
            torch.cuda.synchronize()
            nat.check_status()
            got[split] = [loss.clone(), parts[0].clone(), parts[1].clone()] + [p.grad.clone() for p in m.parameters()]
    for i, (x, y) in enumerate(zip(got[0], got[1])):
        assert torch.equal(x, y), (case, kind, s, a, W, H, B, i, float((x - y).abs().max()))
