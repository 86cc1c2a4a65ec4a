"""GPU: the plan-to-plan cache of recognised closures (fused.describe_problem's fast path: the same
closure objects, their stamp unchanged) never serves a stale device problem. After each change a
caller can make between two plans -- weights updated in place (what train_model's optimizer does),
normaliser statistics replaced or updated in place (a dataset's new statistics), the goal moved, the
cost weight reassigned, the activation module swapped, a forward hook added -- the next plan equals
the plan of freshly built closures with the same change (new objects: nothing cached), bit for bit,
and differs from the plan before the change. Fresh closures come from synthetic.make_problem, which
builds identical weights from its seed."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
N, ITERS = 512, 2


def _plan(prob):
    from mbrl_amd import CEMPlanner
    st, ac = CEMPlanner.plan(prob["s0"], prob["model"], prob["cost"], prob["sample_action"], 8,
                             num_candidates=N, num_iterations=ITERS, seed=prob["rng_seed"], device=DEV)
    return torch.cat([st.reshape(-1), ac.reshape(-1)])


def _stats(prob):
    return prob["model"].keywords["normalize_state"].keywords["stats"]


def _state_cost(prob):
    return prob["cost"].keywords["state_cost"]


def _to_dev(prob):
    """Every tensor the closures hold on the GPU, so that the generic path (taken once a change makes
    the closures unrecognisable: another activation, a hook) can call them with device tensors."""
    prob["module"].to(DEV)
    for field in _stats(prob).values():
        for k in ("mean", "std"):
            field[k] = field[k].to(DEV)
    c = _state_cost(prob)
    c.weights, c.goal_state = c.weights.to(DEV), c.goal_state.to(DEV)
    return prob


def _bump_weight(prob):
    with torch.no_grad():
        prob["module"].linear2.weight.mul_(1.01)


def _replace_mean(prob):
    st = _stats(prob)["observations"]
    st["mean"] = st["mean"] + 0.25


def _update_std_in_place(prob):
    _stats(prob)["observations"]["std"].mul_(1.5)


def _move_goal(prob):
    _state_cost(prob).goal_state.add_(0.5)


def _reassign_weights(prob):
    c = _state_cost(prob)
    c.weights = torch.full_like(c.weights, 2.0)


def _swap_activation(prob):
    prob["module"].activation_fn = torch.nn.Tanh()


def _add_hook(prob):
    prob["module"].register_forward_hook(lambda mod, inp, out: out * 0.5)


CHANGES = [_bump_weight, _replace_mean, _update_std_in_place, _move_goal, _reassign_weights, _swap_activation,
           _add_hook]


@pytest.mark.parametrize("change", CHANGES, ids=[c.__name__.strip("_") for c in CHANGES])
def test_cached_closures_see_the_change(change):
    from mbrl_amd import synthetic
    prob = _to_dev(synthetic.make_problem(3))
    before = _plan(prob)
    assert torch.equal(_plan(prob), before)          # the cache hit: same plan
    change(prob)
    after = _plan(prob)
    fresh = _to_dev(synthetic.make_problem(3))
    change(fresh)
    assert torch.equal(after, _plan(fresh)), change.__name__
    assert not torch.equal(after, before), change.__name__

