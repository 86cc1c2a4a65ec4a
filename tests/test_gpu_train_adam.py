"""Model training on the GPU: mbrl_adam_step (csrc/train.hip) against
torch.optim.Adam itself, and train_model's device paths against each other.

mbrl_adam_step promises torch's Adam step bit for bit (parameters, exp_avg, exp_avg_sq, the CPU step
counters), so these tests compare with torch.equal: torch.optim.Adam (foreach path, the one torch
takes for HIP tensors) is the oracle here -- it is the optimizer the reference's training loop
steps (models.py:53-93, experiment.py:55-62)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
SHAPES = [(512, 23), (512,), (512, 512), (17, 512), (17,), (5, 3), (1,), (1027,)]


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g).to(DEV).requires_grad_(True) for s in SHAPES]


def _grads(seed, step):
    g = torch.Generator().manual_seed(seed * 1000 + step)
    out = []
    for i, s in enumerate(SHAPES):
        x = torch.randn(s, generator=g) * (10.0 ** (i % 5 - 3))
        if i == 2:
            x.view(-1)[:7] = 0.0                      # zero gradients (exp_avg_sq stays tiny)
            x.view(-1)[7] = -0.0
        out.append(x.to(DEV))
    return out


def _state(opt, params):
    return [(p.detach().clone(), opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone(),
             float(opt.state[p]["step"])) for p in params]


def _run(kw, steps, fused, seed=3, skip=None):
    from mbrl_amd.optim import AdamStep
    params = _params(seed)
    opt = torch.optim.Adam(params, **kw)
    fast = AdamStep.maybe(opt) if fused else None
    assert (fast is not None) == fused
    for k in range(steps):
        for i, (p, g) in enumerate(zip(params, _grads(seed, k))):
            p.grad = None if (skip is not None and i == skip and k % 2) else g.clone()
        if fast is not None:
            assert fast.step()
        else:
            opt.step()
    torch.cuda.synchronize()
    return opt, params


CONFIGS = [dict(lr=1e-3), dict(lr=3e-2, betas=(0.8, 0.99), eps=1e-6), dict(lr=1e-3, weight_decay=1e-2),
           dict(lr=0.5, betas=(0.3, 0.5), eps=1e-3, weight_decay=0.1), dict(lr=1e-4, foreach=True)]


@pytest.mark.parametrize("kw", CONFIGS)
def test_adam_step_equals_torch_adam_bit_for_bit(kw):
    ref_opt, ref_p = _run(kw, 12, fused=False)
    got_opt, got_p = _run(kw, 12, fused=True)
    for (a, ma, va, sa), (b, mb, vb, sb) in zip(_state(ref_opt, ref_p), _state(got_opt, got_p)):
        assert torch.equal(a, b) and torch.equal(ma, mb) and torch.equal(va, vb) and sa == sb


def test_adam_step_params_without_grad_keep_their_step_count():
    """A parameter without a gradient is skipped (no state change, its step counter lags), as torch's
    _init_group skips it."""
    ref_opt, ref_p = _run(dict(lr=1e-2), 7, fused=False, skip=3)
    got_opt, got_p = _run(dict(lr=1e-2), 7, fused=True, skip=3)
    for (a, ma, va, sa), (b, mb, vb, sb) in zip(_state(ref_opt, ref_p), _state(got_opt, got_p)):
        assert torch.equal(a, b) and torch.equal(ma, mb) and torch.equal(va, vb) and sa == sb


def test_adam_arith_pattern_is_pinned():
    """The contraction pattern matters: every other pattern of mbrl_adam_step's four fused
    multiply-add sites differs from torch somewhere in the same run (so the equality above is not
    vacuous), and the built-in one is the only one that matches. (With weight decay all four sites
    round differently; with beta2 = 0.5 the addcmul site could not tell, 0.5 * x being exact.)"""
    from mbrl_amd import _lib
    kw = dict(lr=1e-3, weight_decay=1e-2)
    ref_opt, ref_p = _run(kw, 6, fused=False)
    ref = _state(ref_opt, ref_p)
    matches = []
    for bits in range(16):
        with _lib.option("adam_arith", bits + 1):
            got_opt, got_p = _run(kw, 6, fused=True)
        same = all(torch.equal(a, b) and torch.equal(ma, mb) and torch.equal(va, vb)
                   for (a, ma, va, _), (b, mb, vb, _) in zip(ref, _state(got_opt, got_p)))
        if same:
            matches.append(bits)
    assert len(matches) == 1, matches
    got_opt, got_p = _run(kw, 6, fused=True)          # default pattern
    assert all(torch.equal(a, b) for (a, *_), (b, *_) in zip(ref, _state(got_opt, got_p)))


def test_adam_step_bumps_version_counters():
    """The kernel writes through raw pointers; the parameters' version counters must still move (the
    fused planners cache packed weights by them: fused.device_problem)."""
    from mbrl_amd.optim import AdamStep
    p = torch.ones(8, device=DEV, requires_grad=True)
    opt = torch.optim.Adam([p], lr=0.1)
    fast = AdamStep.maybe(opt)
    p.grad = torch.ones_like(p)
    v = p._version
    assert fast.step()
    assert p._version > v and opt.state[p]["exp_avg"]._version > 0


def test_adam_step_declines_what_it_does_not_implement():
    from mbrl_amd.optim import AdamStep
    p = [torch.zeros(4, device=DEV, requires_grad=True)]
    assert AdamStep.maybe(torch.optim.Adam(p, amsgrad=True)) is None
    assert AdamStep.maybe(torch.optim.Adam(p, maximize=True)) is None
    assert AdamStep.maybe(torch.optim.Adam(p, foreach=False)) is None
    assert AdamStep.maybe(torch.optim.AdamW(p)) is None
    assert AdamStep.maybe(torch.optim.SGD(p, lr=0.1)) is None
    assert AdamStep.maybe(torch.optim.Adam([torch.zeros(4, requires_grad=True)])) is None   # CPU
    sch_opt = torch.optim.Adam(p)
    torch.optim.lr_scheduler.StepLR(sch_opt, 1)       # wraps step() on the instance
    assert AdamStep.maybe(sch_opt) is None
    hooked = torch.optim.Adam(p)
    hooked.register_step_post_hook(lambda *a: None)
    assert AdamStep.maybe(hooked) is None
    assert AdamStep.maybe(torch.optim.Adam(p)) is not None


def _train(fast, graph, epochs=3, continue_with_torch=0):
    """train_model on cheetah-shaped synthetic data; returns weights and optimizer state."""
    import mbrl_amd.models as models
    from mbrl_amd import data
    rng = np.random.Generator(np.random.PCG64(11))
    rolls = []
    for _ in range(3):
        K = 400
        st = rng.standard_normal((K + 1, 17)).astype(np.float32)
        rolls.append(data.Rollout(states=list(torch.from_numpy(st)), observations=list(torch.from_numpy(st)),
                                  actions=list(torch.from_numpy(rng.uniform(-1, 1, (K, 6)).astype(np.float32))),
                                  rewards=list(torch.from_numpy(rng.standard_normal(K).astype(np.float32)))))
    ds = data.TransitionsDataset(rollouts=rolls, horizon=2)
    ds.set_data_mode("state_only")
    torch.manual_seed(0)
    m = models.Model(17, 6, hidden_units=64).to(DEV)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    saved = models.AdamStep, models._GraphStep, models.NATIVE_TRAINING
    models.NATIVE_TRAINING = False            # autograd's gradients (bit-comparable with torch's)
    try:
        if not fast:
            models.AdamStep = type("NoFast", (), {"maybe": staticmethod(lambda o: None)})
        if not graph:
            def no_graph(*a, **k):
                raise RuntimeError("eager")
            models._GraphStep = no_graph
        np.random.seed(5)
        m.train_model(ds, opt, batch_size=256, num_epochs=epochs)
    finally:
        models.AdamStep, models._GraphStep, models.NATIVE_TRAINING = saved
    for _ in range(continue_with_torch):
        for p in m.parameters():
            p.grad = torch.full_like(p, 1e-3)
        opt.step()
    torch.cuda.synchronize()
    return [t.detach().cpu() for t in m.parameters()], [(float(s["step"]), s["exp_avg"].cpu(), s["exp_avg_sq"].cpu())
                                                        for s in opt.state.values()]


def test_train_model_device_paths_agree_bit_for_bit():
    """Graph replay + mbrl_adam_step, graph replay + torch's step, and the eager loop + torch's step
    train to the same bits (1200 transitions, horizon 2, batch 256: full batches replay the graph,
    the short last batch of every epoch runs eagerly) -- and the optimizer stays a working torch
    optimizer afterwards."""
    ref_w, ref_s = _train(fast=False, graph=False, continue_with_torch=2)
    for fast, graph in ((False, True), (True, True), (True, False)):
        w, s = _train(fast=fast, graph=graph, continue_with_torch=2)
        assert all(torch.equal(a, b) for a, b in zip(ref_w, w)), (fast, graph)
        for (sa, ma, va), (sb, mb, vb) in zip(ref_s, s):
            assert sa == sb and torch.equal(ma, mb) and torch.equal(va, vb), (fast, graph)
