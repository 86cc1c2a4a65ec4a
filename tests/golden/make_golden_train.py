"""Golden fixtures for model training: the REFERENCE's own
TransitionsDataset / Rollout / TransitionsSampler (src/mbrl/data.py) and Model.train_model /
ModelWithReward.train_model (src/mbrl/models.py:53-93, 165-217) on small synthetic rollouts.

    python tests/golden/make_golden_train.py        (build container only; writes train_*.npz)

Inputs are regenerated from seeds by tests/test_train.py (rollouts: PCG64 seed 77; initial weights:
PCG64 seed 78); the fixture stores the reference's trained weights, its evaluate_model losses before
and after, and the NumPy seed used for the sampler's shuffles.
"""
import os
import sys

import numpy as np

sys.dont_write_bytecode = True            # never write into the read-only reference tree
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import torch  # noqa: E402

CASES = {
    # name: (model kind, data mode, horizon, batch, epochs, optimizer, lr)
    "train_model_state_h1": ("model", "state_only", 1, 16, 2, "adam", 1e-3),
    "train_model_state_h2": ("model", "state_only", 2, 8, 1, "sgd", 0.05),
    "train_reward_obs_h1": ("reward", "obs_only", 1, 16, 2, "adam", 1e-3),
}
S, O, A, W = 5, 4, 2, 32
LENGTHS = (40, 25, 33)


def synth_rollouts():
    """[(states [K+1, S], observations [K+1, O], actions [K, A], rewards [K])] from PCG64(77)."""
    rng = np.random.Generator(np.random.PCG64(77))
    out = []
    for K in LENGTHS:
        out.append((rng.standard_normal((K + 1, S)).astype(np.float32) * 2 + 1,
                    rng.standard_normal((K + 1, O)).astype(np.float32) - 0.5,
                    rng.uniform(-1, 1, (K, A)).astype(np.float32),
                    rng.standard_normal(K).astype(np.float32) * 3))
    return out


def synth_weights(kind):
    """nn.Linear-law weights for linear1.. in order, PCG64(78)."""
    rng = np.random.Generator(np.random.PCG64(78))
    if kind == "model":
        dims = [(S + A, W), (W, W), (W, S)]
    else:
        dims = [(O + A, W), (W, W), (W, O), (W, 1)]
    out = []
    for fi, fo in dims:
        b = 1.0 / np.sqrt(fi)
        out.append((rng.uniform(-b, b, (fo, fi)).astype(np.float32), rng.uniform(-b, b, fo).astype(np.float32)))
    return out


def main():
    sys.path.insert(0, REF)
    from src.mbrl import data, models
    torch.set_num_threads(1)
    for name, (kind, mode, horizon, batch, epochs, opt, lr) in CASES.items():
        rolls = [data.Rollout(states=[torch.from_numpy(x) for x in s], observations=[torch.from_numpy(x) for x in o],
                              actions=[torch.from_numpy(x) for x in a], rewards=[torch.tensor(x) for x in r])
                 for s, o, a, r in synth_rollouts()]
        ds = data.TransitionsDataset(rollouts=rolls, horizon=horizon)
        ds.set_data_mode(mode)
        m = models.Model(S, A, hidden_units=W) if kind == "model" else models.ModelWithReward(O, A, hidden_units=W)
        lins = [m.linear1, m.linear2, m.linear3] + ([m.linear4] if kind == "reward" else [])
        with torch.no_grad():
            for lin, (w, b) in zip(lins, synth_weights(kind)):
                lin.weight.copy_(torch.from_numpy(w))
                lin.bias.copy_(torch.from_numpy(b))
        optimizer = (torch.optim.Adam(m.parameters(), lr=lr) if opt == "adam"
                     else torch.optim.SGD(m.parameters(), lr=lr))
        np_seed = 4242
        before = None
        if kind == "model":
            np.random.seed(np_seed - 1)
            before = np.mean(m.evaluate_model(ds, batch_size=batch))
        np.random.seed(np_seed)
        m.train_model(dataset=ds, optimizer=optimizer, batch_size=batch, num_epochs=epochs)
        after = None
        if kind == "model":
            np.random.seed(np_seed + 1)
            after = np.mean(m.evaluate_model(ds, batch_size=batch))
        out = {f"w{i}": l.weight.detach().numpy() for i, l in enumerate(lins)}
        out.update({f"b{i}": l.bias.detach().numpy() for i, l in enumerate(lins)})
        np.savez_compressed(os.path.join(HERE, name + ".npz"), np_seed=np_seed,
                            eval_before=np.float64(before if before is not None else np.nan),
                            eval_after=np.float64(after if after is not None else np.nan), **out)
        print(name, "eval", before, "->", after)


if __name__ == "__main__":
    main()
