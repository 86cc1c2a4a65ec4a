"""Recognise the reference's model / cost / sampler closures and drive the HIP extension.

The planners receive opaque callables: the model is
functools.partial(model, normalize_state=partial(normalize_field, field_name="observations",
stats=S), normalize_action=..., unnormalize_state=...) (agents.py:219-230), the cost is
functools.partial(state_action_cost, state_cost=SmoothAbsLoss, action_cost=CoshLoss)
(agents.py:231) and sample_action is functools.partial(_sample_action, action_spec=spec)
(agents.py:233). This module unpacks those closures (partial.func / .keywords) into the POD
descriptors of include/mbrl_cem.h. Anything it does not recognise returns None and the planner
takes its generic path (the callables run on device tensors; selection and refit still run in
the HIP extension).

Device state is cached per module: packed weights are re-packed only when a parameter changes
(torch's in-place version counter moves on every optimizer.step()).
"""
import functools
import operator
import weakref

import numpy as np
import torch

from . import _lib
from .models import CoshLoss, EnsembleModel, Model, ModelWithReward, SmoothAbsLoss


# ------------------------------------------------------------------------------------------------
# introspection
# ------------------------------------------------------------------------------------------------
def _unpartial(f):
    kw = {}
    while isinstance(f, functools.partial):
        kw = {**f.keywords, **kw}
        f = f.func
    return f, kw


def _uncompose(f):
    """compose(a, b) closure (agents.py:300-304, models.compose) -> (a, b), else None."""
    code, cells = getattr(f, "__code__", None), getattr(f, "__closure__", None)
    if code is None or cells is None or set(code.co_freevars) != {"a", "b"}:
        return None
    env = dict(zip(code.co_freevars, (c.cell_contents for c in cells)))
    return env["a"], env["b"]


def _getter_index(g):
    """operator.itemgetter(i) -> i for a single int index, else None."""
    if not isinstance(g, operator.itemgetter):
        return None
    try:
        _, args = g.__reduce__()
    except Exception:  # pragma: no cover
        return None
    return args[0] if len(args) == 1 and isinstance(args[0], int) else None


def _reward_layers(module):
    """(members, L, W, s, a) for a reward-head model: this package's ModelWithReward, or the
    reference's (duck-typed: linear1..linear4, ReLU, linear3 -> s, linear4 -> 1)."""
    if isinstance(module, ModelWithReward):
        return [module.linears()], module.n_hidden, module.hidden_units, module.state_dim, module.action_dim
    lins = [getattr(module, f"linear{i}", None) for i in range(1, 5)]
    if (type(module).__name__ == "ModelWithReward" and all(isinstance(l, torch.nn.Linear) for l in lins)
            and isinstance(getattr(module, "activation_fn", None), torch.nn.ReLU) and not hasattr(module, "linear5")):
        W = lins[0].out_features
        s = lins[2].out_features
        a = lins[0].in_features - s
        if (lins[1].in_features == W and lins[1].out_features == W and lins[2].in_features == W
                and lins[3].in_features == W and lins[3].out_features == 1 and a >= 1):
            return [lins], 2, W, s, a
    return None


def _linear_layers(module):
    """(members, L, W, s, a) for a recognised dynamics module, else None. members = list of lists of
    nn.Linear. Accepts this package's Model / EnsembleModel and the reference's models.Model
    (duck-typed: linear1..linear3 + ReLU activation_fn + noise None)."""
    if isinstance(module, EnsembleModel):
        members = [m.linears() for m in module.members]
        m0 = module.members[0]
        return members, m0.n_hidden, m0.hidden_units, m0.state_dim, m0.action_dim
    if isinstance(module, Model):
        if module.noise is not None or module.n_hidden < 1:
            return None
        return [module.linears()], module.n_hidden, module.hidden_units, module.state_dim, module.action_dim
    names = [n for n in ("linear1", "linear2", "linear3") if isinstance(getattr(module, n, None), torch.nn.Linear)]
    if (type(module).__name__ == "Model" and len(names) == 3 and not hasattr(module, "linear4")
            and isinstance(getattr(module, "activation_fn", None), torch.nn.ReLU)
            and getattr(module, "noise", None) is None):
        lins = [module.linear1, module.linear2, module.linear3]
        W = lins[0].out_features
        s = lins[2].out_features
        a = lins[0].in_features - s
        if lins[1].in_features == W and lins[1].out_features == W and lins[2].in_features == W and a >= 1:
            return [lins], 2, W, s, a
    return None


def _field_stats(norm_fn, expect_name):
    """(field_name, mean, std) of partial(normalize_field|unnormalize_field, field_name=, stats=)."""
    if norm_fn is None:
        return None
    f, kw = _unpartial(norm_fn)
    if getattr(f, "__name__", "") != expect_name or "field_name" not in kw or "stats" not in kw:
        return False
    try:
        st = kw["stats"][kw["field_name"]]
        return kw["field_name"], torch.as_tensor(st["mean"]), torch.as_tensor(st["std"])
    except (KeyError, TypeError):
        return False


def describe_norm(normalize_state, normalize_action, unnormalize_state, s, a):
    ns = _field_stats(normalize_state, "normalize_field")
    us = _field_stats(unnormalize_state, "unnormalize_field")
    na = _field_stats(normalize_action, "normalize_field")
    if ns is False or us is False or na is False:
        return None
    obs = ns or us
    if ns and us and not ((ns[1] is us[1] or torch.equal(ns[1].float(), us[1].float()))
                          and (ns[2] is us[2] or torch.equal(ns[2].float(), us[2].float()))):
        return None  # one obs-stat pair serves both directions in the kernel
    if obs and (obs[1].numel() != s or obs[2].numel() != s):
        return None
    if na and (na[1].numel() != a or na[2].numel() != a):
        return None
    return dict(obs_mean=obs[1] if obs else None, obs_std=obs[2] if obs else None,
                act_mean=na[1] if na else None, act_std=na[2] if na else None,
                normalize_state=bool(ns), unnormalize_state=bool(us), normalize_action=bool(na),
                rew_mean=None, rew_std=None, unnormalize_reward=False)


def _describe_partial(fn, reward):
    """partial(module, <normaliser keywords>) -> model description, else None."""
    f, kw = _unpartial(fn)
    allowed = {"normalize_state", "normalize_action", "unnormalize_state"} | ({"unnormalize_reward"} if reward else set())
    if set(kw) - allowed or not isinstance(f, torch.nn.Module):
        return None
    layers = _reward_layers(f) if reward else _linear_layers(f)
    if layers is None:
        return None
    members, L, W, s, a = layers
    norm = describe_norm(kw.get("normalize_state"), kw.get("normalize_action"), kw.get("unnormalize_state"), s, a)
    if norm is None:
        return None
    if reward:
        rn = _field_stats(kw.get("unnormalize_reward"), "unnormalize_field")
        if rn is False or (rn and (rn[1].numel() != 1 or rn[2].numel() != 1)):
            return None
        if rn:
            norm.update(rew_mean=rn[1].reshape(1), rew_std=rn[2].reshape(1), unnormalize_reward=True)
    return dict(module=f, members=members, L=L, W=W, s=s, a=a, E=len(members), norm=norm, reward=reward)


def _norms_equal(n1, n2):
    for k in ("obs_mean", "obs_std", "act_mean", "act_std", "rew_mean", "rew_std"):
        x, y = n1[k], n2[k]
        if (x is None) != (y is None) or (x is not None and not torch.equal(x.float(), y.float())):
            return False
    return all(n1[k] == n2[k] for k in ("normalize_state", "unnormalize_state", "normalize_action",
                                         "unnormalize_reward"))


def describe_model(model):
    """Model callable -> dict(module, members, L, W, s, a, E, norm, reward) or None. Accepts
    partial(Model|EnsembleModel, ...) (agents.py:224-230) and RewardAgent's
    compose(partial(ModelWithReward, ...), itemgetter(0)) (agents.py:342-352)."""
    uc = _uncompose(model)
    if uc is not None:
        if _getter_index(uc[1]) != 0:
            return None
        return _describe_partial(uc[0], reward=True)
    return _describe_partial(model, reward=False)


def describe_cost(cost, s, mdesc=None):
    """partial(state_action_cost, state_cost=SmoothAbsLoss, action_cost=CoshLoss) -> goal-state dict;
    compose(partial(<the model's module>, <the same normalisers>), itemgetter(1)) (agents.py:353-362)
    -> reward dict when `mdesc` is that reward model; else None."""
    uc = _uncompose(cost)
    if uc is not None:
        if _getter_index(uc[1]) != 1 or mdesc is None or not mdesc.get("reward"):
            return None
        cd = _describe_partial(uc[0], reward=True)
        if cd is None or cd["module"] is not mdesc["module"] or not _norms_equal(cd["norm"], mdesc["norm"]):
            return None
        return dict(kind=_lib.MBRL_COST_MODEL_REWARD, key=("reward", id(mdesc["module"])))
    f, kw = _unpartial(cost)
    if getattr(f, "__name__", "") != "state_action_cost" or set(kw) != {"state_cost", "action_cost"}:
        return None
    sc, ac = kw["state_cost"], kw["action_cost"]
    if not (isinstance(sc, SmoothAbsLoss) or type(sc).__name__ == "SmoothAbsLoss"):
        return None
    if not (isinstance(ac, CoshLoss) or type(ac).__name__ == "CoshLoss"):
        return None
    if sc.goal_state is None:
        return None
    goal = torch.as_tensor(sc.goal_state, dtype=torch.float32).flatten()
    w = torch.as_tensor(sc.weights, dtype=torch.float32).flatten()
    if goal.numel() == 1:
        goal = goal.expand(s)
    if w.numel() == 1:
        w = w.expand(s)
    if goal.numel() != s or w.numel() != s:
        return None
    def raw_key(x):
        return _tensor_key(x) if torch.is_tensor(x) else ("v", float(np.asarray(x).ravel()[0]), np.size(x))
    return dict(kind=_lib.MBRL_COST_GOAL_STATE, weights=w.contiguous(), goal=goal.contiguous(),
                alpha_state=float(sc.alpha),
                alpha_action=float(ac.alpha), key=(raw_key(sc.weights), raw_key(sc.goal_state),
                                                   float(sc.alpha), float(ac.alpha)))


def describe(model, cost, device):
    """(mdesc, cdesc) for closures the fused path may run, else (None, None): recognised by
    describe_model / describe_cost AND confirmed once by semantic_check (recognition goes by names
    and types; the check makes sure the arithmetic behind those names is the reference's)."""
    mdesc, cdesc, _ = describe_problem(model, cost, device)
    return mdesc, cdesc


_PLAIN = frozenset((dict, str, int, bool, type(None), functools.partial))


def _value_stamp(v, out):
    """Identity of a value recognition reads, plus a tensor's storage and version (in-place updates)."""
    t = type(v)
    if t in _PLAIN:                       # (the common cases first: this runs on every plan's host turn)
        out.append(id(v))
    elif t is float:
        out.append(v)
    elif isinstance(v, torch.Tensor):
        out.append((id(v), v.data_ptr(), v._version))
    elif isinstance(v, np.ndarray):       # mutable in place with no version: stamped by content
        out.append((id(v), v.dtype.str, v.shape, v.tobytes()))
    elif t is list or t is tuple:         # (goal / weights / statistics given as Python sequences)
        out.append((id(v), len(v)))
        for x in v:
            _value_stamp(x, out)
    else:
        out.append(id(v))


def _callable_stamp(fn, out):
    """Everything describe_model / describe_cost read from a closure, as identities and versions: the
    compose cells, every partial level and its keyword values, the normalisers' statistics
    (stats[field_name]["mean" / "std"]) and the cost modules' goal, weights and alpha."""
    uc = _uncompose(fn)
    if uc is not None:
        out.append(("compose", id(fn), id(uc[1])))
        fn = uc[0]
    while isinstance(fn, functools.partial):
        out.append(("partial", id(fn), id(fn.func), len(fn.keywords)))
        for k, v in fn.keywords.items():
            out.append(k)
            _value_stamp(v, out)
            if isinstance(v, functools.partial):
                f2, kw2 = _unpartial(v)
                out.append(id(f2))
                st, name = kw2.get("stats"), kw2.get("field_name")
                _value_stamp(st, out)
                out.append(name)
                if isinstance(st, dict) and name in st:
                    fld = st[name]
                    _value_stamp(fld, out)
                    if isinstance(fld, dict):
                        _value_stamp(fld.get("mean"), out)
                        _value_stamp(fld.get("std"), out)
            elif isinstance(v, torch.nn.Module):
                for a in ("goal_state", "weights", "alpha"):
                    _value_stamp(getattr(v, a, None), out)
        fn = fn.func
    out.append(id(fn))
    if isinstance(fn, torch.nn.Module):   # the module tree: a replaced submodule changes the layers read
        stack = [fn]
        while stack:
            mod = stack.pop()
            subs = mod._modules
            out.append((id(mod), len(subs), len(mod._forward_hooks), len(mod._forward_pre_hooks)))
            stack.extend(x for x in subs.values() if x is not None)


_FAST = {}   # (id(model), id(cost), device, precision) -> (model, cost, stamp, (mdesc, cdesc, prob))


def describe_problem(model, cost, device, precision=_lib.MBRL_PRECISION_F32):
    """describe() plus the recognised closures' DeviceProblem at `precision`: (mdesc, cdesc, prob),
    or (None, None, None). The problem's cache key (every weight and statistic's version) is
    computed once per call, for the semantic check and the plan alike.

    Fast path (the host turn of every plan): the same closure objects as a previous call whose stamp
    -- the identities and tensor versions of everything the recognition read (_callable_stamp), and
    the weights' storage and versions (_param_key) -- is unchanged get that call's result back
    without re-walking and re-describing them (~25 us -> a few)."""
    key = (id(model), id(cost), str(device), int(precision))
    hit = _FAST.get(key)
    if hit is not None and hit[0] is model and hit[1] is cost:
        stamp = []
        _callable_stamp(model, stamp)
        _callable_stamp(cost, stamp)
        stamp.append(_param_key(hit[3][0]["members"], ""))
        if tuple(stamp) == hit[2]:
            return hit[3]
    device = torch.device(device)
    mdesc = describe_model(model)
    cdesc = describe_cost(cost, mdesc["s"], mdesc) if mdesc is not None else None
    if mdesc is None or cdesc is None:
        return None, None, None
    prob = device_problem(mdesc, cdesc, device)
    if not semantic_check(model, cost, mdesc, cdesc, device, prob):
        return None, None, None
    if int(precision) != _lib.MBRL_PRECISION_F32:
        prob = device_problem(mdesc, cdesc, device, precision)
    stamp = []
    _callable_stamp(model, stamp)
    _callable_stamp(cost, stamp)
    stamp.append(_param_key(mdesc["members"], ""))
    if len(_FAST) > 16:
        _FAST.clear()
    _FAST[key] = (model, cost, tuple(stamp), (mdesc, cdesc, prob))
    return mdesc, cdesc, prob


def _fn_sig(fn):
    """Identity of what a recognised closure resolves to: the functions behind the partials, the
    module's class and hooks, the cost modules' classes."""
    uc = _uncompose(fn)
    if uc is not None:
        fn = uc[0]
    f, kw = _unpartial(fn)
    if isinstance(f, torch.nn.Module):
        head = (id(type(f)), id(f), len(f._forward_hooks), len(f._forward_pre_hooks),
                id(type(getattr(f, "activation_fn", None))))
    else:
        head = (id(f),)
    return head + tuple((k, id(_unpartial(kw[k])[0]), id(type(kw[k]))) for k in sorted(kw))


def _rebind(fn, module, new):
    """fn (module | partial(module, ...) | compose(partial(module, ...), getter)) with module -> new."""
    from .models import compose
    if fn is module:
        return new
    uc = _uncompose(fn)
    if uc is not None:
        return compose(_rebind(uc[0], module, new), uc[1])
    f, kw = _unpartial(fn)
    return functools.partial(new, **kw) if f is module else fn


def _probe_call(fn, module, *args):
    """The user's callable on the probe batch, on the device; if its tensors live elsewhere (e.g.
    normaliser statistics on the host while the module is on the GPU -- the fused path moves them),
    on the host with a host copy of the module."""
    try:
        return fn(*args)
    except RuntimeError as e:
        if "device" not in str(e):
            raise
    import copy
    return _rebind(fn, module, copy.deepcopy(module).cpu())(*[x.cpu() for x in args])


PROBE_ROWS = 8
PROBE_RTOL = 1e-4   # fp32 summation-order differences here are ~1e-6; any change of arithmetic is far above


def _close(x, ref):
    x = x.detach().to("cpu", torch.float64).reshape(-1)
    ref = ref.detach().to("cpu", torch.float64).reshape(-1)
    return x.shape == ref.shape and bool(torch.all(torch.abs(x - ref) <= PROBE_RTOL * torch.clamp(ref.abs(), min=1.0)))


def semantic_check(model, cost, mdesc, cdesc, device, prob=None):
    """One-time check (per closure identity and weights version) that the fused arithmetic equals
    the caller's callables: a one-step fused rollout of PROBE_ROWS random (state, action) rows
    against model(s, a) and cost(s', a) evaluated through the callables themselves (torch autograd
    mode, so a DynamicsModel does not take its own fused forward). A mismatch -- e.g. a function
    that is named normalize_field / state_action_cost but computes something else -- disables the
    fused path for these closures with a warning; the planner then runs them on the generic path
    (the reference's semantics: planners.py:199-210 on the callables as given)."""
    import warnings
    device = torch.device(device)
    if prob is None:
        prob = device_problem(mdesc, cdesc, device)
    sig = (_fn_sig(model), _fn_sig(cost))
    ok = prob.verified.get(sig)
    if ok is not None:
        return ok
    s, a, E, P = mdesc["s"], mdesc["a"], mdesc["E"], PROBE_ROWS
    n = mdesc["norm"]
    gen = torch.Generator().manual_seed(0x5eed)
    om = n["obs_mean"].float().cpu() if n["obs_mean"] is not None else torch.zeros(s)
    osd = n["obs_std"].float().cpu() if n["obs_std"] is not None else torch.ones(s)
    states = (om + osd * torch.randn((P, s), generator=gen)).to(device).contiguous()
    acts = (torch.rand((P, a), generator=gen) * 2 - 1).to(device).contiguous()
    out = torch.empty((E, 1, P, s), dtype=torch.float32, device=device)
    with torch.cuda.device(device):
        costs = rollout(prob, states, P, 1, actions=acts.view(1, P, a), s0_per_candidate=True, states_out=out)
    try:
        with torch.enable_grad():
            nxt = _probe_call(model, mdesc["module"], states, acts)
            ok = _close(out[:, 0].mean(0) if E > 1 else out[0, 0], nxt)
            for e in range(E):
                ok = ok and _close(costs[e], _probe_call(cost, mdesc["module"], out[e, 0], acts))
    except Exception as exc:   # the callables cannot run the probe: not the arithmetic the kernels assume
        ok = False
        warnings.warn(f"mbrl_amd: probing the model / cost closures raised {exc!r}")
    if not ok:
        warnings.warn("mbrl_amd: the model / cost closures are recognised by name but do not compute what the "
                      "fused kernels compute on a probe batch; these closures run on the generic path")
    prob.verified[sig] = ok
    return ok


def describe_sampler(sample_action):
    """partial(_sample_action, action_spec=spec) -> (lo, hi, a) or None."""
    f, kw = _unpartial(sample_action)
    spec = kw.get("action_spec")
    if spec is None or getattr(f, "__name__", "") not in ("_sample_action", "sample_action"):
        return None
    lo = max(float(spec.minimum[0]), -3.0)
    hi = min(float(spec.maximum[0]), 3.0)
    return lo, hi, int(spec.shape[0])


# ------------------------------------------------------------------------------------------------
# device caches
# ------------------------------------------------------------------------------------------------
_PACKED = weakref.WeakKeyDictionary()   # module -> (key, packed tensor)


def _param_key(members, device):
    # Linear._parameters directly (a replaced Parameter shows up; Module.__getattr__ and a nested
    # generator cost ~8x as much per plan)
    key = [str(device)]
    for lins in members:
        for lin in lins:
            prm = lin._parameters
            w, b = prm["weight"], prm["bias"]
            key.append((w.data_ptr(), w._version, b.data_ptr(), b._version))
    return tuple(key)


def mlp_shape(desc, precision=_lib.MBRL_PRECISION_F32):
    return _lib.MlpShape(desc["s"], desc["a"], desc["W"], desc["L"], desc["E"], int(desc.get("reward", False)),
                         int(precision))


def packed_weights(desc, device):
    """Packed fragment stream of desc's module on `device` (cached until a parameter changes)."""
    module, members = desc["module"], desc["members"]
    key = _param_key(members, device)
    hit = _PACKED.get(module)
    if hit is not None and hit[0] == key:
        return hit[1]
    lib = _lib.load()
    shape = mlp_shape(desc)
    nbytes = lib.mbrl_mlp_packed_bytes(ctypes_ref(shape))
    if nbytes == 0:
        raise RuntimeError(f"unsupported MLP shape for the HIP path: {desc['s']}/{desc['a']} W={desc['W']} L={desc['L']}")
    packed = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
    keep, wp, bp = [], [], []
    for lins in members:
        for lin in lins:
            w = lin.weight.detach().to(device=device, dtype=torch.float32).contiguous()
            b = lin.bias.detach().to(device=device, dtype=torch.float32).contiguous()
            keep += [w, b]
            wp.append(w.data_ptr())
            bp.append(b.data_ptr())
    n = len(wp)
    warr = (_lib.c_void_p * n)(*wp)
    barr = (_lib.c_void_p * n)(*bp)
    with torch.cuda.device(device):
        _lib.check(lib.mbrl_mlp_pack(ctypes_ref(shape), warr, barr, _lib.ptr(packed), _lib.stream_handle(device)),
                   "mbrl_mlp_pack")
        # the temporaries in `keep` must outlive the pack kernels
        torch.cuda.current_stream(device).synchronize()
    _PACKED[module] = (key, packed)
    return packed


def ctypes_ref(x):
    import ctypes
    return ctypes.byref(x)


def _dev(t, device):
    return None if t is None else t.detach().to(device=device, dtype=torch.float32).contiguous()


class DeviceProblem:
    """Device-resident descriptors for one (model, cost) pair; holds the tensors the POD structs point at."""

    def __init__(self, mdesc, cdesc, device, precision=_lib.MBRL_PRECISION_F32):
        self.mdesc, self.cdesc, self.device = mdesc, cdesc, device
        self.verified = {}                          # semantic_check results per closure identity
        self.shape = mlp_shape(mdesc, precision)   # the packed buffer serves both precisions
        self.packed = packed_weights(mdesc, device)
        n = mdesc["norm"]
        self._norm_t = [_dev(n[k], device) for k in ("obs_mean", "obs_std", "act_mean", "act_std", "rew_mean",
                                                     "rew_std")]
        self.norm = _lib.Norm(*[_lib.ptr(t) for t in self._norm_t], int(n["normalize_state"]),
                              int(n["unnormalize_state"]), int(n["normalize_action"]), int(n["unnormalize_reward"]))
        if cdesc is not None and cdesc["kind"] == _lib.MBRL_COST_MODEL_REWARD:
            self._cost_t = []
            self.cost = _lib.Cost(_lib.MBRL_COST_MODEL_REWARD, 0, 0, 0, None, None, 0.0, 0.0)
        elif cdesc is not None:
            self._cost_t = [_dev(cdesc["weights"], device), _dev(cdesc["goal"], device)]
            self.cost = _lib.Cost(_lib.MBRL_COST_GOAL_STATE, 1, 1, 0, _lib.ptr(self._cost_t[0]),
                                  _lib.ptr(self._cost_t[1]), cdesc["alpha_state"], cdesc["alpha_action"])
        else:
            self._cost_t = []
            self.cost = _lib.Cost(_lib.MBRL_COST_GOAL_STATE, 0, 0, 0, None, None, 0.0, 0.0)
        # the C-call arguments that never change for this problem (built once, not per plan)
        self.refs = (ctypes_ref(self.shape), _lib.ptr(self.packed), ctypes_ref(self.norm), ctypes_ref(self.cost))
        self.plan_cache = {}   # planners: per (CEM settings) the params struct and workspace size


def _tensor_key(t):
    return None if t is None else (t.data_ptr(), t._version, t.device.type, tuple(t.shape))


_PROBLEMS = {}


def device_problem(mdesc, cdesc, device, precision=_lib.MBRL_PRECISION_F32):
    """Cached DeviceProblem: rebuilt only when weights, statistics or cost parameters change."""
    n = mdesc["norm"]
    key = (id(mdesc["module"]), _param_key(mdesc["members"], device),
           tuple(_tensor_key(n[k]) for k in ("obs_mean", "obs_std", "act_mean", "act_std", "rew_mean", "rew_std")),
           (n["normalize_state"], n["unnormalize_state"], n["normalize_action"], n["unnormalize_reward"]),
           None if cdesc is None else cdesc["key"], int(precision))
    hit = _PROBLEMS.get(key)
    if hit is not None and hit[0]() is mdesc["module"]:
        return hit[1]
    prob = DeviceProblem(mdesc, cdesc, device, precision)
    if len(_PROBLEMS) > 64:
        _PROBLEMS.clear()
    _PROBLEMS[key] = (weakref.ref(mdesc["module"]), prob)
    return prob


# ------------------------------------------------------------------------------------------------
# thin wrappers over the C ABI (all on the current stream of `device`)
# ------------------------------------------------------------------------------------------------
def rollout(prob, s0, N, H, *, actions=None, sampler=None, n_offset=0, s0_per_candidate=False,
            costs=None, actions_out=None, states_out=None):
    lib = _lib.load()
    dev = prob.device
    E = prob.mdesc["E"]
    if costs is None:
        costs = torch.empty((E, N), dtype=torch.float32, device=dev)
    _lib.check(lib.mbrl_rollout_cost(ctypes_ref(prob.shape), _lib.ptr(prob.packed), ctypes_ref(prob.norm),
                                     ctypes_ref(prob.cost), _lib.ptr(s0), int(s0_per_candidate), _lib.ptr(actions),
                                     ctypes_ref(sampler) if sampler is not None else None, N, H, n_offset,
                                     _lib.ptr(costs), _lib.ptr(actions_out), _lib.ptr(states_out),
                                     _lib.stream_handle(dev)), "mbrl_rollout_cost")
    return costs


def select(costs, K, nan_policy=_lib.MBRL_NAN_LAST, returns_out=None, workspace=None):
    """costs: [E, N] device tensor -> elite indices [K] (int64, ascending)."""
    lib = _lib.load()
    E, N = costs.shape
    dev = costs.device
    elites = torch.empty(K, dtype=torch.int64, device=dev)
    need = lib.mbrl_select_workspace_bytes(N)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.mbrl_select_elites(_lib.ptr(costs), E, N, K, nan_policy, _lib.ptr(elites), _lib.ptr(returns_out),
                                      _lib.ptr(workspace), workspace.numel(), _lib.stream_handle(dev)),
               "mbrl_select_elites")
    return elites


def refit(sampler, H, a, elites, alpha, mu_out, sigma_out, workspace=None):
    lib = _lib.load()
    dev = mu_out.device
    K = elites.numel()
    need = lib.mbrl_refit_workspace_bytes(H, a, K)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.mbrl_cem_refit(ctypes_ref(sampler), H, a, _lib.ptr(elites), K, float(alpha), _lib.ptr(mu_out),
                                  _lib.ptr(sigma_out), _lib.ptr(workspace), workspace.numel(),
                                  _lib.stream_handle(dev)), "mbrl_cem_refit")


def trajectory(prob, s0, actions, H, member_states=None, workspace=None):
    """States [H, s] (ensemble mean) of ONE action sequence actions [H, a]; member_states [E, H, s] optional."""
    lib = _lib.load()
    dev = prob.device
    states = torch.empty((H, prob.mdesc["s"]), dtype=torch.float32, device=dev)
    need = lib.mbrl_trajectory_workspace_bytes(ctypes_ref(prob.shape), H)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=dev)
    _lib.check(lib.mbrl_trajectory(ctypes_ref(prob.shape), _lib.ptr(prob.packed), ctypes_ref(prob.norm), _lib.ptr(s0),
                                   _lib.ptr(actions), H, _lib.ptr(states), _lib.ptr(member_states),
                                   _lib.ptr(workspace), workspace.numel(), _lib.stream_handle(dev)),
               "mbrl_trajectory")
    return states


def sample_actions(sampler, H, a, N, n_offset, out):
    lib = _lib.load()
    _lib.check(lib.mbrl_sample_actions(ctypes_ref(sampler), H, a, N, n_offset, _lib.ptr(out),
                                       _lib.stream_handle(out.device)), "mbrl_sample_actions")
    return out


def cem_update(costs, K, sampler, H, a, alpha, mu_out, sigma_out, elites=None, returns_out=None, next_actions=None,
               draw_offset=0):
    """mbrl_cem_update: select + refit + (optionally) the next iteration's proposals for global
    candidates [draw_offset, draw_offset + next_actions.shape[1]) in one launch. costs: [E, N].
    Returns the elites [K] (int64), or None when the shape exceeds the fused kernel
    (MBRL_EUNSUPPORTED: the caller runs select + refit + sample_actions instead)."""
    lib = _lib.load()
    E, N = costs.shape
    dev = costs.device
    if elites is None:
        elites = torch.empty(K, dtype=torch.int64, device=dev)
    dn = 0 if next_actions is None else int(next_actions.shape[1])
    rc = lib.mbrl_cem_update(_lib.ptr(costs), E, N, K, ctypes_ref(sampler), H, a, float(alpha), _lib.ptr(elites),
                             _lib.ptr(returns_out), _lib.ptr(mu_out), _lib.ptr(sigma_out), _lib.ptr(next_actions),
                             int(draw_offset), dn, _lib.stream_handle(dev))
    if rc == _lib.MBRL_EUNSUPPORTED:
        return None
    _lib.check(rc, "mbrl_cem_update")
    return elites


def make_sampler(seed, iteration, mu, sigma, lo, hi):
    return _lib.Sampler(int(seed) & 0xFFFFFFFFFFFFFFFF, int(iteration), 0, _lib.ptr(mu), _lib.ptr(sigma),
                        float(lo), float(hi))


# ------------------------------------------------------------------------------------------------
# DynamicsModel.forward on device (one step, per-row start states)
# ------------------------------------------------------------------------------------------------
def _forward_checked(prob, module, normalize_action, normalize_state, unnormalize_state):
    """semantic_check for DynamicsModel.forward's fused path: the module's own forward (autograd
    mode) with the given normalisers on a probe batch, against the fused one-step rollout."""
    import warnings
    norms = dict(normalize_action=normalize_action, normalize_state=normalize_state,
                 unnormalize_state=unnormalize_state)
    sig = ("forward", _fn_sig(functools.partial(module, **{k: v for k, v in norms.items() if v is not None})))
    ok = prob.verified.get(sig)
    if ok is not None:
        return ok
    s, a, P, dev = prob.mdesc["s"], prob.mdesc["a"], PROBE_ROWS, prob.device
    gen = torch.Generator().manual_seed(0x5eed)
    st = torch.randn((P, s), generator=gen).to(dev)
    ac = (torch.rand((P, a), generator=gen) * 2 - 1).to(dev)
    out = torch.empty((1, 1, P, s), dtype=torch.float32, device=dev)
    rollout(prob, st, P, 1, actions=ac.view(1, P, a), s0_per_candidate=True, states_out=out)
    try:
        with torch.enable_grad():
            ok = _close(out[0, 0], _probe_call(functools.partial(module, **norms), module, st, ac))
    except Exception:
        ok = False
    if not ok:
        warnings.warn("mbrl_amd: DynamicsModel.forward's normalisers are recognised by name but compute "
                      "something else on a probe batch; forward runs the module as written")
    prob.verified[sig] = ok
    return ok


def try_forward(module, state, action, normalize_action, normalize_state, unnormalize_state):
    layers = _linear_layers(module)
    if layers is None or isinstance(module, EnsembleModel):
        return None
    members, L, W, s, a = layers
    if state.dim() != 2 or action.dim() != 2 or state.shape[1] != s or action.shape[1] != a \
            or state.shape[0] != action.shape[0] or state.dtype != torch.float32 or action.dtype != torch.float32:
        return None
    norm = describe_norm(normalize_state, normalize_action, unnormalize_state, s, a)
    if norm is None:
        return None
    desc = dict(module=module, members=members, L=L, W=W, s=s, a=a, E=1, norm=norm, reward=False)
    dev = state.device
    prob = device_problem(desc, None, dev)
    if not _forward_checked(prob, module, normalize_action, normalize_state, unnormalize_state):
        return None
    B = state.shape[0]
    st = state.contiguous()
    act = action.contiguous().view(1, B, a)
    out = torch.empty((1, 1, B, s), dtype=torch.float32, device=dev)
    rollout(prob, st, B, 1, actions=act, s0_per_candidate=True, states_out=out)
    return out.view(B, s)
