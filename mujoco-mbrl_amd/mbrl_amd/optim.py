"""torch.optim.Adam.step() as one launch per parameter group (csrc/train.hip, mbrl_adam_step).

The reference's training loop (models.py:53-93, 165-217) ends every batch with optimizer.step();
the optimizer is torch.optim.Adam(model.parameters(), lr, weight_decay) or SGD (experiment.py:55-62).
torch's Adam on HIP tensors runs its foreach implementation (adam.py _multi_tensor_adam): seven or
eight multi-tensor kernels and a few dozen Python-level list operations per step, which at the
reference's model sizes cost more than the forward and backward passes together.

AdamStep.maybe(optimizer) accepts a plain torch.optim.Adam whose step torch would run on that
foreach path with default semantics (no amsgrad / maximize / capturable / differentiable / fused,
float hyper-parameters, fp32 contiguous HIP parameters, no step hooks, step() not wrapped on the
instance, e.g. by an LR scheduler). Its step() keeps torch's own bookkeeping -- the lazily created
state tensors, the per-parameter CPU step counters, the bias corrections computed in double -- and
hands the element-wise chain to mbrl_adam_step, which leaves parameters, exp_avg and exp_avg_sq
bit-identical to torch's step (tests/test_gpu_train_adam.py). The optimizer object stays a normal
torch optimizer: its state can be saved, loaded or stepped by torch afterwards.
For anything else maybe() returns None and the caller steps the optimizer itself."""
import ctypes

import torch
from torch.autograd.graph import increment_version
from torch.optim import optimizer as _optimizer_module

from . import _lib

_ONE = torch.tensor(1.0)


def _plain_float(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool)


class AdamStep:
    """Fused replacement for optimizer.step() on a supported torch.optim.Adam (module docstring)."""

    def __init__(self, optimizer, device):
        self.opt = optimizer
        self.device = device
        self._tables = {}
        self._pending = None     # (step counters, steps) of the epoch_plan awaiting epoch_done

    @classmethod
    def maybe(cls, optimizer):
        if type(optimizer) is not torch.optim.Adam or "step" in vars(optimizer):
            return None
        if optimizer._optimizer_step_pre_hooks or optimizer._optimizer_step_post_hooks:
            return None
        if _optimizer_module._global_optimizer_pre_hooks or _optimizer_module._global_optimizer_post_hooks:
            return None
        device = None
        for g in optimizer.param_groups:
            if (g.get("amsgrad") or g.get("maximize") or g.get("capturable") or g.get("differentiable")
                    or g.get("fused") or g.get("foreach") is False or g.get("decoupled_weight_decay")):
                return None
            b1, b2 = g["betas"]
            if not all(_plain_float(x) for x in (g["lr"], b1, b2, g["eps"], g["weight_decay"])):
                return None
            # torch adds weight decay when weight_decay != 0; a value that rounds to float 0 would still
            # add 0 * param (NaN for infinite parameters) -- leave such a group to torch
            if g["weight_decay"] != 0 and ctypes.c_float(g["weight_decay"]).value == 0:
                return None
            for p in g["params"]:
                if type(p) not in (torch.Tensor, torch.nn.Parameter) or not p.is_cuda or p.dtype != torch.float32:
                    return None
                if not p.is_contiguous() or (device is not None and p.device != device):
                    return None
                device = p.device
                st = optimizer.state.get(p)
                if st and not cls._state_ok(p, st):
                    return None
        return cls(optimizer, device) if device is not None else None

    @staticmethod
    def _state_ok(p, st):
        step, m, v = st.get("step"), st.get("exp_avg"), st.get("exp_avg_sq")
        if not (isinstance(step, torch.Tensor) and not step.is_cuda and step.numel() == 1):
            return False
        return all(isinstance(t, torch.Tensor) and t.device == p.device and t.dtype == torch.float32
                   and t.shape == p.shape and t.is_contiguous() for t in (m, v))

    def step(self):
        """One optimizer.step(). Returns False (nothing done) if a gradient is not a contiguous fp32
        tensor of its parameter's shape; the caller then runs torch's step."""
        work = []
        for gi, g in enumerate(self.opt.param_groups):
            params = [p for p in g["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                gr = p.grad
                if gr.is_sparse or gr.dtype != torch.float32 or gr.shape != p.shape or not gr.is_contiguous():
                    return False
            work.append((gi, g, params))
        lib = _lib.load()
        stream = _lib.stream_handle(self.device)
        scalar_dtype = _optimizer_module._get_scalar_dtype()
        for gi, g, params in work:
            state = self.opt.state
            for p in params:                      # adam.py Adam._init_group: lazy state initialisation
                st = state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=scalar_dtype)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            steps = [state[p]["step"] for p in params]
            torch._foreach_add_(steps, _ONE, alpha=1.0)
            lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
            table = self._table(gi, params)
            for i, s in enumerate(steps):         # adam.py _multi_tensor_adam, capturable = False
                k = s.item()
                table[i].step_size = (lr / (1 - b1 ** k)) * -1
                table[i].bc2_sqrt = (1 - b2 ** k) ** 0.5
            hp = _lib.AdamHparams(1 - b1, b2, 1 - b2, eps, wd)
            _lib.check(lib.mbrl_adam_step(table, len(params), ctypes.byref(hp), stream), "mbrl_adam_step")
            # the kernel wrote through raw pointers: bump the version counters as torch's in-place
            # ops would, so that caches keyed on them (fused.device_problem's packed weights) and
            # autograd's saved-tensor checks see the change
            increment_version(params + [state[p][k] for p in params for k in ("exp_avg", "exp_avg_sq")])
        return True

    def epoch_plan(self, params, steps):
        """Inputs of mbrl_train_epoch for `steps` Adam steps over `params` (the optimizer's only
        group, every parameter with a gradient each step): (table, hparams, step_sizes, bc2_sqrt),
        with the state created as torch would and the step counters advanced by `steps` -- what
        `steps` calls of step() leave once epoch_done() confirms the launch -- or None when the group
        does not have that shape."""
        groups = self.opt.param_groups
        if len(groups) != 1 or len(groups[0]["params"]) != len(params) or \
                {id(p) for p in groups[0]["params"]} != {id(p) for p in params}:
            return None
        for p in params:
            gr = p.grad
            if gr is None or gr.dtype != torch.float32 or gr.shape != p.shape or not gr.is_contiguous():
                return None
        g = groups[0]
        state = self.opt.state
        scalar_dtype = _optimizer_module._get_scalar_dtype()
        for p in params:                          # adam.py Adam._init_group: lazy state initialisation
            st = state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0, dtype=scalar_dtype)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        counters = [state[p]["step"] for p in params]
        k0 = counters[0].item()
        if any(c.item() != k0 for c in counters) or k0 + steps >= 2 ** 24:
            return None
        lr, (b1, b2), eps, wd = g["lr"], g["betas"], g["eps"], g["weight_decay"]
        n = len(params)
        va, vb = [], []
        for s in range(steps):                    # adam.py _multi_tensor_adam, capturable = False
            k = k0 + s + 1                        # (Python floats, as torch computes them; c_float rounds)
            va += [(lr / (1 - b1 ** k)) * -1] * n
            vb += [(1 - b2 ** k) ** 0.5] * n
        ss, bc = (ctypes.c_float * (steps * n))(*va), (ctypes.c_float * (steps * n))(*vb)
        table = self._table(0, params)            # (rebuilt only when a tensor moved)
        self._pending = (counters, steps)
        return table, _lib.AdamHparams(1 - b1, b2, 1 - b2, eps, wd), ss, bc

    def epoch_done(self, params):
        """After a successful mbrl_train_epoch: advance the step counters by the epoch's steps (the
        float32 counters, as `steps` increments by one) -- only then, so that a failed launch leaves
        the optimizer as it was -- and bump the version counters of what the kernels wrote."""
        counters, steps = self._pending
        self._pending = None
        for c in counters:
            c.add_(float(steps))
        state = self.opt.state
        increment_version(list(params) + [state[p][k] for p in params for k in ("exp_avg", "exp_avg_sq")])

    def _table(self, gi, params):
        """The group's mbrl_adam_tensor array, rebuilt when any tensor moved."""
        state = self.opt.state
        key = tuple((p.data_ptr(), p.grad.data_ptr(), state[p]["exp_avg"].data_ptr(),
                     state[p]["exp_avg_sq"].data_ptr(), p.numel()) for p in params)
        hit = self._tables.get(gi)
        if hit is not None and hit[0] == key:
            return hit[1]
        table = (_lib.AdamTensor * len(params))()
        for i, (pp, gp, mp, vp, n) in enumerate(key):
            table[i].param, table[i].grad, table[i].exp_avg, table[i].exp_avg_sq = pp, gp, mp, vp
            table[i].numel = n
        self._tables[gi] = (key, table)
        return table
