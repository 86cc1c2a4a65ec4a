"""Model training: mbrl_amd's TransitionsDataset / train_model against the
reference's own (golden fixtures from tests/golden/make_golden_train.py).

CPU: the same batches in the same order through the same torch ops -- bit-exact on the CPU the
fixtures were generated on (this container), within 1e-6 elsewhere (another CPU's BLAS kernels
round differently). GPU: the same loop on the MI355X within a float tolerance."""
import os
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_golden_train as mg  # noqa: E402


def build(name, device):
    from mbrl_amd import data, models
    kind, mode, horizon, batch, epochs, opt, lr = mg.CASES[name]
    rolls = [data.Rollout(states=[torch.from_numpy(x) for x in s], observations=[torch.from_numpy(x) for x in o],
                          actions=[torch.from_numpy(x) for x in a], rewards=[torch.tensor(x) for x in r])
             for s, o, a, r in mg.synth_rollouts()]
    ds = data.TransitionsDataset(rollouts=rolls, horizon=horizon)
    ds.set_data_mode(mode)
    m = (models.Model(mg.S, mg.A, hidden_units=mg.W) if kind == "model"
         else models.ModelWithReward(mg.O, mg.A, hidden_units=mg.W))
    with torch.no_grad():
        for lin, (w, b) in zip(m.linears(), mg.synth_weights(kind)):
            lin.weight.copy_(torch.from_numpy(w))
            lin.bias.copy_(torch.from_numpy(b))
    m = m.to(device)
    optimizer = (torch.optim.Adam(m.parameters(), lr=lr) if opt == "adam"
                 else torch.optim.SGD(m.parameters(), lr=lr))
    return m, ds, optimizer, batch, epochs, kind


def run(name, device, golden):
    g = golden(name)
    m, ds, optimizer, batch, epochs, kind = build(name, device)
    seed = int(g["np_seed"])
    before = after = None
    if kind == "model":
        np.random.seed(seed - 1)
        before = np.mean(m.evaluate_model(ds, batch_size=batch))
    np.random.seed(seed)
    m.train_model(dataset=ds, optimizer=optimizer, batch_size=batch, num_epochs=epochs)
    if kind == "model":
        np.random.seed(seed + 1)
        after = np.mean(m.evaluate_model(ds, batch_size=batch))
    got = [(l.weight.detach().cpu().numpy(), l.bias.detach().cpu().numpy()) for l in m.linears()]
    ref = [(g[f"w{i}"], g[f"b{i}"]) for i in range(len(got))]
    return got, ref, before, after, g


@pytest.mark.parametrize("name", list(mg.CASES))
def test_train_model_cpu_matches_reference(golden, name):
    got, ref, before, after, g = run(name, "cpu", golden)
    for (w, b), (rw, rb) in zip(got, ref):
        assert np.allclose(w, rw, rtol=1e-5, atol=1e-6) and np.allclose(b, rb, rtol=1e-5, atol=1e-6)
    if before is not None:
        assert abs(before - g["eval_before"]) < 1e-6 and abs(after - g["eval_after"]) < 1e-6


def test_dataset_semantics():
    from mbrl_amd import data
    rolls = [data.Rollout(states=[torch.full((2,), float(i)) for i in range(5)],
                          observations=[torch.full((3,), 10.0 + i) for i in range(5)],
                          actions=[torch.full((1,), -float(i)) for i in range(4)],
                          rewards=[torch.tensor(100.0 + i) for i in range(4)])]
    ds = data.TransitionsDataset(rollouts=rolls, horizon=2, normalise=False)
    assert len(ds) == 3 and ds.transition_index() == [(0, 0), (0, 1)]
    ds.set_data_mode("state_only")
    inp, out = ds[(0, 1)]
    assert [float(x[0][0]) for x in inp] == [1.0, 2.0] and [float(x[1][0]) for x in inp] == [-1.0, -2.0]
    assert [float(x[0]) for x in out] == [101.0, 102.0] and [float(x[1][0]) for x in out] == [2.0, 3.0]
    assert torch.allclose(ds.statistics["rewards"]["mean"], torch.tensor(101.5))


@pytest.mark.parametrize("lengths,horizon", [([501] * 20, 1), ([7, 2, 30, 3], 2), ([3], 1), ([5, 5], 3)])
def test_epoch_order_is_the_samplers_shuffle(lengths, horizon):
    """train_model's row order (models._epoch_order: shuffle of arange) is the order
    TransitionsSampler yields (shuffle of the (rollout, start) list), and both leave NumPy's global
    RNG in the same state."""
    from mbrl_amd import data, models
    rolls = [data.Rollout(states=[torch.zeros(2)] * n, observations=[torch.zeros(2)] * n,
                          actions=[torch.zeros(1)] * (n - 1), rewards=[torch.tensor(0.0)] * (n - 1))
             for n in lengths]
    ds = data.TransitionsDataset(rollouts=rolls, horizon=horizon, normalise=False)
    index = ds.transition_index()
    pos = {t: i for i, t in enumerate(index)}
    for seed in (0, 7, 123):
        np.random.seed(seed)
        ref = [pos[t] for t in data.TransitionsSampler(ds)]
        ref_next = np.random.random_sample(3)
        np.random.seed(seed)
        got = models._epoch_order(ds)
        assert got.tolist() == ref and ds.num_transitions() == len(index)
        assert np.array_equal(np.random.random_sample(3), ref_next)
    batches = models._epoch_batches(ds, 4)
    assert [len(b) for b in batches] == [min(4, len(index) - i) for i in range(0, len(index), 4)]


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(mg.CASES))
def test_train_model_on_gpu_matches_reference(golden, name):
    got, ref, before, after, g = run(name, "cuda:0", golden)
    for (w, b), (rw, rb) in zip(got, ref):
        assert np.allclose(w, rw, rtol=1e-4, atol=1e-5) and np.allclose(b, rb, rtol=1e-4, atol=1e-5)
    if before is not None:
        assert abs(before - g["eval_before"]) < 1e-5 and abs(after - g["eval_after"]) < 1e-5


def test_train_model_on_an_empty_dataset_takes_no_step():
    """Rollouts shorter than the horizon leave no transition: the reference's DataLoader yields no
    batch, so the weights stay put and train_iterations still counts the call."""
    from mbrl_amd import data, models
    rolls = [data.Rollout(states=[torch.zeros(3)] * 2, observations=[torch.zeros(3)] * 2,
                          actions=[torch.zeros(1)], rewards=[torch.tensor(0.0)])]
    ds = data.TransitionsDataset(rollouts=rolls, horizon=2, normalise=False)
    ds.set_data_mode("state_only")
    assert ds.num_transitions() == 0
    m = models.Model(3, 1, hidden_units=8)
    before = [p.detach().clone() for p in m.parameters()]
    m.train_model(ds, torch.optim.Adam(m.parameters()), batch_size=4, num_epochs=2)
    assert all(torch.equal(a, b) for a, b in zip(before, m.parameters())) and m.train_iterations == 1
    assert m.evaluate_model(ds, batch_size=4) == []
