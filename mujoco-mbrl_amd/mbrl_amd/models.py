"""Dynamics models and costs with the reference's API (/root/reference/src/mbrl/models.py).

`DynamicsModel.forward(state, action, normalize_action=None, normalize_state=None,
unnormalize_state=None)` keeps the reference contract (models.py:13-29). On CUDA tensors with
autograd off it runs the one-step batch through the same HIP rollout kernel the planners use
(H = 1, per-row start states); otherwise (training, CPU tensors) it is plain PyTorch, exactly the
reference's arithmetic.
"""
import ctypes
import functools
import threading
import weakref

import numpy as np
import torch
import torch.nn as nn

from .optim import AdamStep


def _epoch_order(dataset):
    """The row order DataLoader(dataset, batch_size, sampler=TransitionsSampler(dataset)) visits
    (models.py:61-63), as an int64 array of row indices into dataset.stacked().

    TransitionsSampler (data.py:271-285) np.random.shuffle()s the list of (rollout, start) pairs.
    NumPy's legacy shuffle draws j = random_interval(i) for i = n-1 .. 1 and swaps x[i], x[j] on
    every path (the list path and the 1-D array path alike), so shuffling arange(n) in place yields
    the same permutation of positions and leaves the global RNG in the same state -- without
    building and hashing n tuples per epoch (16 ms for 10k transitions, more than the GPU's
    20 training steps of that epoch)."""
    order = np.arange(dataset.num_transitions(), dtype=np.int64)
    np.random.shuffle(order)
    return order


def _epoch_batches(dataset, batch_size):
    """_epoch_order split into the DataLoader's batches (the last one may be short)."""
    order = _epoch_order(dataset)
    return [order[i:i + batch_size] for i in range(0, len(order), batch_size)]


def _device_of(module):
    return next(module.parameters()).device


def _batch_loss(dataset, ins, outs, idx, step_loss, n_parts):
    bi = [x.index_select(0, idx) for x in ins]
    bo = [x.index_select(0, idx) for x in outs]
    loss, parts = 0, [0] * n_parts
    for h in range(dataset.horizon):
        for k, term in enumerate(step_loss([x[:, h] for x in bi], [x[:, h] for x in bo])):
            parts[k] = parts[k] + term
            loss = loss + term
    return loss, parts


class _GraphStep:
    """A full-size batch's zero_grad + gather + forward + loss + backward captured once in a HIP
    graph (through torch.cuda.CUDAGraph) and replayed per batch; optimizer.step() stays outside the
    graph so any optimizer works unchanged. The warm-up before capture only touches .grad (zeroed
    after), never the parameters, so training follows exactly the eager sequence of updates."""

    def __init__(self, model, dataset, ins, outs, batch_size, step_loss, n_parts):
        dev = _device_of(model)
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.idx = torch.zeros(batch_size, dtype=torch.long, device=dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                loss, _ = _batch_loss(dataset, ins, outs, self.idx, step_loss, n_parts)
                loss.backward()
            del loss                      # drop the warm-up autograd graph before capturing
        torch.cuda.current_stream(dev).wait_stream(side)
        grads = [p.grad for p in self.params if p.grad is not None]
        if grads:
            torch._foreach_zero_(grads)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            if grads:                     # zero_grad() as the graph's first node: backward accumulates
                torch._foreach_zero_(grads)
            self.loss, self.parts = _batch_loss(dataset, ins, outs, self.idx, step_loss, n_parts)
            self.loss.backward()
        # the replay accumulates into exactly these tensors; an eager step in between (the last,
        # partial batch: optimizer.zero_grad() sets .grad to None) must not orphan them
        self.grads = [p.grad for p in self.params]

    def run(self, rows):
        self.idx.copy_(rows)
        for p, g in zip(self.params, self.grads):
            p.grad = g
        self.graph.replay()
        return self.loss, self.parts


# train_model's device path for the reference's MLP models under the default MSELoss: the batch
# gradient from mbrl_train_grads (csrc/train.hip) instead of autograd. False: autograd in a HIP graph.
NATIVE_TRAINING = True

# model -> (binding key, _NativeGrads) of its last native train_model call (_NativeGrads.cached)
_NATIVE_CACHE = weakref.WeakKeyDictionary()


class _NativeGrads:
    """mbrl_train_grads for Model (noise None) / ModelWithReward with MSELoss(reduction='mean'):
    per batch, one C call that gathers the batch, runs the forward pass and the loss gradient, and
    overwrites every Linear's .grad (what zero_grad + backward leave). The loss values come back
    as device scalars (total, state, reward) for the writer."""

    def __init__(self, model, ins, outs, horizon, batch_size, reward):
        from . import _lib
        self.lib = _lib.load()
        dev = _device_of(model)
        lins = model.linears()
        self.params = [t for lin in lins for t in (lin.weight, lin.bias)]
        self.grads = [torch.zeros_like(t) for t in self.params]
        m = _lib.TrainModel()
        m.state_dim, m.action_dim, m.hidden = model.state_dim, model.action_dim, model.hidden_units
        m.n_hidden, m.reward_head, m.horizon = model.n_hidden, int(reward), int(horizon)
        for i, lin in enumerate(lins):
            m.weight[i], m.bias[i] = lin.weight.data_ptr(), lin.bias.data_ptr()
            m.weight_grad[i], m.bias_grad[i] = self.grads[2 * i].data_ptr(), self.grads[2 * i + 1].data_ptr()
        (states, actions), (rewards, next_states) = ins, outs
        self.keep = [x.contiguous() for x in (states, actions, next_states, rewards)]
        d = _lib.TrainData()
        d.states, d.actions, d.next_states, d.rewards = [x.data_ptr() for x in self.keep]
        d.transitions = states.shape[0]
        self.model, self.data = m, d
        need = self.lib.mbrl_train_workspace_bytes(ctypes.byref(m), int(batch_size))
        if need == 0:
            _lib.check(-1, "mbrl_train_workspace_bytes")
        # zeroed once: the fused step's sticky status word lives in it (mbrl_train_status_offset)
        self.ws = torch.zeros(need, dtype=torch.uint8, device=dev)
        self.status_at = int(self.lib.mbrl_train_status_offset(ctypes.byref(m), int(batch_size)))
        self.loss = torch.zeros(3, dtype=torch.float32, device=dev)
        self.ptrs = [t.data_ptr() for t in self.params]
        self.dev = dev
        self._lib = _lib

    @classmethod
    def cached(cls, model, ins, outs, horizon, batch_size, reward):
        """The object of the model's previous train_model call when nothing it binds has changed (the
        parameter and gradient storage, the stacked transitions, the batch size), else a new one. A
        call then starts its first launch without allocating and zeroing the gradients and the
        workspace (host time the GPU idles through at the start of every call,
        tools/train_startup.py). Rebuilt when a non-contiguous input would need a fresh contiguous
        copy."""
        key = (str(_device_of(model)), int(horizon), int(batch_size), bool(reward),
               tuple(t.data_ptr() for lin in model.linears() for t in (lin.weight, lin.bias)),
               tuple((x.data_ptr(), tuple(x.shape), x.is_contiguous()) for x in (*ins, *outs)))
        hit = _NATIVE_CACHE.get(model)
        if hit is not None and hit[0] == key:
            return hit[1]
        obj = cls(model, ins, outs, horizon, batch_size, reward)
        if all(x.is_contiguous() for x in (*ins, *outs)):
            _NATIVE_CACHE[model] = (key, obj)
        else:
            _NATIVE_CACHE.pop(model, None)
        return obj

    @staticmethod
    def forget(model):
        """Drop the model's cached object (after a failed status check: its sticky word is set)."""
        _NATIVE_CACHE.pop(model, None)

    @staticmethod
    def supported(model, dataset, ins, outs, criterion):
        if not NATIVE_TRAINING or type(criterion) is not torch.nn.MSELoss or criterion.reduction != "mean":
            return None
        if type(model) is Model:
            if model.noise is not None:
                return None
            reward = False
        elif type(model) is ModelWithReward:
            reward = True
        else:
            return None
        if model.n_hidden < 1 or model.n_hidden + 2 > 10 or len(ins) != 2 or len(outs) != 2:
            return None
        # train.hip computes Linear-ReLU chains and never calls the module: a replaced activation or
        # a hook would make it train a different function than the model computes
        if type(model.activation_fn) is not nn.ReLU or any(
                m._forward_hooks or m._forward_pre_hooks or m._backward_hooks for m in model.modules()):
            return None
        params = list(model.parameters())
        if len(params) != 2 * len(model.linears()):
            return None
        if not all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.requires_grad for p in params):
            return None
        (states, actions), (rewards, next_states) = ins, outs
        T, H = states.shape[0], dataset.horizon
        want = [(states, model.state_dim), (actions, model.action_dim), (next_states, model.state_dim)]
        if any(tuple(x.shape) != (T, H, w) or x.dtype != torch.float32 for x, w in want):
            return None
        if rewards.numel() != T * H:
            return None
        return reward

    def epoch(self, order, batch_size, adam):
        """One epoch over the device row order `order`: every batch's gradient and Adam step from one
        mbrl_train_epoch call. Returns the per-batch losses [batches, 3] (device), or None when the
        optimizer's state does not allow it (the caller then steps per batch)."""
        for p, g in zip(self.params, self.grads):
            if p.grad is not g:
                p.grad = g
        if [p.data_ptr() for p in self.params] != self.ptrs:
            raise RuntimeError("model parameters moved during training")
        rows = int(order.shape[0])
        steps = (rows + batch_size - 1) // batch_size
        plan = adam.epoch_plan(self.params, steps)
        if plan is None:
            return None
        table, hp, ss, bc = plan
        losses = torch.empty((steps, 3), dtype=torch.float32, device=self.dev)
        self._lib.check(self.lib.mbrl_train_epoch(ctypes.byref(self.model), ctypes.byref(self.data),
                                                  ctypes.c_void_p(order.data_ptr()), rows, int(batch_size), table,
                                                  len(self.params), ctypes.byref(hp), ss, bc,
                                                  ctypes.c_void_p(losses.data_ptr()),
                                                  ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(),
                                                  self._lib.stream_handle(self.dev)), "mbrl_train_epoch")
        adam.epoch_done(self.params)
        return losses

    def check_status(self):
        """Raise if an in-launch wait of the fused step timed out (the workgroup dispatch order its
        Adam placement relies on was not kept): the parameters may then be off. Never expected. The
        word is sticky (set by any launch since the workspace was zeroed), so one read after the last
        epoch of a train_model call covers every epoch of it: no per-epoch copy or kernel."""
        word = int(self.ws[self.status_at:self.status_at + 4].view(torch.int32).item())
        if word & 1:
            raise RuntimeError("mbrl_amd: a fused training step's bounded wait timed out (status word "
                               f"{word:#x}); the parameters of that step may be wrong")

    def run(self, idx):
        """The batch gradient for the rows `idx` (int64, on the device) into p.grad."""
        for p, g in zip(self.params, self.grads):
            if p.grad is not g:
                p.grad = g
        if [p.data_ptr() for p in self.params] != self.ptrs:
            raise RuntimeError("model parameters moved during training")
        self._lib.check(self.lib.mbrl_train_grads(ctypes.byref(self.model), ctypes.byref(self.data),
                                                  ctypes.c_void_p(idx.data_ptr()), int(idx.shape[0]),
                                                  ctypes.c_void_p(self.loss.data_ptr()),
                                                  ctypes.c_void_p(self.ws.data_ptr()), self.ws.numel(),
                                                  self._lib.stream_handle(self.dev)), "mbrl_train_grads")
        loss = self.loss.clone()          # the buffer is reused by the next batch; the writer keeps these
        return loss[0], [loss[1], loss[2]]


def _train_loop(model, dataset, optimizer, batch_size, num_epochs, step_loss, writer, tags, criterion=None):
    """models.py:53-93 / 165-217 on the model's device: per batch, the loss summed over the horizon
    steps, zero_grad, backward, step -- the reference's order of operations. Batches are gathered
    from device-resident transitions (TransitionsDataset.stacked) instead of per-sample collation;
    on a GPU the full-size batches replay one captured graph (_GraphStep), and a plain Adam steps
    through mbrl_adam_step (optim.AdamStep: one launch, torch's arithmetic bit for bit)."""
    dev = _device_of(model)
    if dev.type == "cuda":
        with torch.cuda.device(dev):       # launches and workspaces on the model's GPU
            return _train_loop_on(dev, model, dataset, optimizer, batch_size, num_epochs, step_loss, writer, tags,
                                  criterion)
    return _train_loop_on(dev, model, dataset, optimizer, batch_size, num_epochs, step_loss, writer, tags, criterion)


def _train_loop_on(dev, model, dataset, optimizer, batch_size, num_epochs, step_loss, writer, tags, criterion):
    if dataset.num_transitions() == 0:    # the reference's DataLoader yields no batch
        model.train_iterations += 1
        return
    _, ins, outs = dataset.stacked(dev)
    n_parts = len(tags)
    graph = native = None
    if dev.type == "cuda":
        reward = _NativeGrads.supported(model, dataset, ins, outs, criterion)
        if reward is not None:
            native = _NativeGrads.cached(model, ins, outs, dataset.horizon, batch_size, reward)
    if native is None and dev.type == "cuda" and dataset.num_transitions() >= batch_size:
        try:
            graph = _GraphStep(model, dataset, ins, outs, batch_size, step_loss, n_parts)
        except RuntimeError:           # capture unsupported for this model / criterion: stay eager
            graph = None
            for p in model.parameters():
                p.grad = None
    fast = AdamStep.maybe(optimizer) if dev.type == "cuda" else None
    # parameters the optimizer steps that the native gradient call does not overwrite each batch
    own = set() if native is None else {id(p) for p in native.params}
    extra = [p for g in optimizer.param_groups for p in g["params"] if id(p) not in own] if native is not None else []
    num_iters = 0
    whole = native is not None and fast is not None
    if whole and num_epochs > 0:
        # The device path issues the epochs back to back with no host round trip between them (a
        # per-epoch copy of the row order from pageable memory waited for the previous epoch to drain).
        # Epoch k + 1's order is drawn while epoch k runs -- the same np.random draws in the same order
        # (nothing else in this loop draws from the global RNG) -- into a ring of pinned rows and copied
        # on a side stream that the training stream waits on before epoch k + 1 (the copy lands while
        # epoch k computes). The sticky status word is read once, after the last epoch.
        ring = _order_ring(dev, dataset.num_transitions())
        main = torch.cuda.current_stream(dev)
        ring.draw(0)
        ring.copy(0, main)
    epoch_losses = []
    for ep in range(num_epochs):
        if whole:
            host, order = ring.rows(ep)
            if ep >= 1:
                ring.copied[ep % ring.K].wait(main)   # epoch ep's order has landed
        else:
            host = _epoch_order(dataset)
            order = torch.from_numpy(host).to(dev)
        losses = native.epoch(order, batch_size, fast) if whole else None
        if whole and ep + 1 < num_epochs:
            ring.draw(ep + 1)
            ring.copy(ep + 1, ring.side)
        if losses is not None:            # the whole epoch in one call; the writer gets its values after
            ring.consumed[ep % ring.K].record(main)   # the ring row is free once this epoch has run
            epoch_losses.append(losses)
            continue
        num_iters = _write_epoch_losses(epoch_losses, writer, tags, n_parts, model, num_iters)
        epoch_losses = []
        for i in range(0, len(host), batch_size):
            idx = order[i:i + batch_size]
            if native is not None:
                for p in extra:               # optimizer.zero_grad() for what the native call does not write
                    p.grad = None
                loss, parts = native.run(idx)
                parts = parts[:n_parts]
            elif graph is not None and idx.shape[0] == batch_size:
                loss, parts = graph.run(idx)
            else:
                optimizer.zero_grad()
                loss, parts = _batch_loss(dataset, ins, outs, idx, step_loss, n_parts)
                loss.backward(retain_graph=True)
            if fast is None or not fast.step():
                optimizer.step()
            num_iters += 1
            if writer is not None:
                for tag, val in zip(tags, parts if n_parts > 1 else [loss]):
                    writer.add_scalar(tag.format(model.train_iterations), val, num_iters)
                if n_parts > 1:
                    writer.add_scalar("loss/total/{}".format(model.train_iterations), loss, num_iters)
        if whole:
            ring.consumed[ep % ring.K].record(torch.cuda.current_stream(dev))
    num_iters = _write_epoch_losses(epoch_losses, writer, tags, n_parts, model, num_iters)
    if graph is not None:
        for p in model.parameters():      # release the graph-pool grads; the eager path re-allocates
            p.grad = None
    # (the native path leaves the last batch's gradients in .grad, as the reference's loop does)
    try:
        if native is not None:
            native.check_status()
    except RuntimeError:
        _NativeGrads.forget(model)        # the workspace's sticky status word is set: start afresh
        raise
    model.train_iterations += 1


class _OrderRing:
    """K pinned host rows and K device rows of n row indices, a copy stream and per-row events, reused
    by every train_model call on datasets of n transitions: epoch e's order lives in row e % K. The
    host draws into a pinned row only once the copy that last read it has finished (`copied`), and
    enqueues the copy into a device row only once the epoch that last read it has run (`consumed`),
    so the host may run up to ~K epochs ahead -- ~17 ms of 2x512 training at K = 16,
    room for a garbage-collector pause of the host thread -- and no call allocates (a pinned
    allocation costs milliseconds, a new stream's first use ~6 ms of queue set-up). Rows hold
    `cap` indices, n rounded up to a power of two, and an epoch uses the first n: the dataset of an
    MBRL loop grows every episode, and it reuses one ring until it doubles. K shrinks with the
    capacity (16 rows up to 131k, 4 from 524k on: a longer epoch is a longer lead), so the ring
    holds at most 16 MB of pinned memory up to 524k indices and 4 rows beyond."""

    def __init__(self, dev, cap):
        self.cap = cap
        self.n = cap
        self.K = max(4, min(16, (1 << 21) // max(cap, 1)))
        self.pinned = torch.empty((self.K, cap), dtype=torch.int64, pin_memory=True)
        self.host = self.pinned.numpy()
        self.arange = np.arange(cap, dtype=np.int64)
        self.dev = torch.empty((self.K, cap), dtype=torch.int64, device=dev)
        self.side = torch.cuda.Stream(dev)
        with torch.cuda.stream(self.side):          # set up the side stream's queue here, once
            self.dev[:1].copy_(self.pinned[:1], non_blocking=True)
        self.side.synchronize()
        from . import _lib
        self.copied = [_lib.StreamEvent() for _ in range(self.K)]      # fence-free: a torch.cuda.Event
        self.consumed = [_lib.StreamEvent() for _ in range(self.K)]    # record idles the GPU ~5.5 us
        # a host wait on an event that is still pending takes a slow first-use path (~2 ms, measured
        # on the first long train_model call of a process, tools/train_after_load.py): take it here
        for r in range(self.K):
            with torch.cuda.stream(self.side):
                self.dev[r].copy_(self.pinned[r], non_blocking=True)
                self.copied[r].record(self.side)
            self.copied[r].synchronize()

    def draw(self, e):
        """Epoch e's order (models._epoch_order's draws: NumPy's shuffle of arange(n), in place)."""
        r = e % self.K
        self.copied[r].synchronize()                # the copy that last read this pinned row is done
        row = self.host[r, :self.n]
        np.copyto(row, self.arange[:self.n])
        np.random.shuffle(row)                      # (in place on the view: the draws of a fresh arange(n))

    def copy(self, e, stream):
        r = e % self.K
        # the epoch that last read this device row must have run: the host checks (it is K epochs
        # back, so this rarely waits) -- a wait of the side stream on the training stream's event cost
        # the training stream 20-45 us per epoch (tools/train_epoch_plumbing.py)
        self.consumed[r].synchronize()              # (an event never recorded is complete)
        with torch.cuda.stream(stream):
            self.dev[r, :self.n].copy_(self.pinned[r, :self.n], non_blocking=True)
            self.copied[r].record(stream)

    def rows(self, e):
        r = e % self.K
        return self.host[r, :self.n], self.dev[r, :self.n]


_ORDER_RINGS = {}


def _order_ring(dev, n):
    # one ring per thread: two threads training at once must not share pinned rows
    cap = 1 << max(10, (max(n, 1) - 1).bit_length())
    key = (str(dev), cap, threading.get_ident())
    ring = _ORDER_RINGS.get(key)
    if ring is None:
        if len(_ORDER_RINGS) > 8:
            _ORDER_RINGS.clear()
        ring = _ORDER_RINGS[key] = _OrderRing(dev, cap)
    ring.n = n                  # (the previous call's epochs were all enqueued before this one draws)
    return ring


def _write_epoch_losses(epoch_losses, writer, tags, n_parts, model, num_iters):
    """The writer's per-batch values of whole-epoch device calls (in batch order), after the epochs ran."""
    for losses in epoch_losses:
        if writer is None:
            num_iters += losses.shape[0]
            continue
        for row in losses.cpu().tolist():
            num_iters += 1
            parts = [row[1], row[2]][:n_parts]
            for tag, val in zip(tags, parts if n_parts > 1 else [row[0]]):
                writer.add_scalar(tag.format(model.train_iterations), val, num_iters)
            if n_parts > 1:
                writer.add_scalar("loss/total/{}".format(model.train_iterations), row[0], num_iters)
    return num_iters


class DynamicsModel(nn.Module):
    """models.py:8-93."""

    def __init__(self):
        super().__init__()
        self.train_iterations = 0

    def train_model(self, dataset, optimizer, batch_size=512, num_epochs=50, criterion=None, writer=None):
        """models.py:53-93 (state_only / obs_only data modes: inputs (s, a), outputs (r, s'))."""
        criterion = criterion or torch.nn.MSELoss()

        def step_loss(inp, out):
            (states, actions), (_, next_states) = inp, out
            return [criterion(self.forward(states, actions, normalize_action=None, normalize_state=None,
                                           unnormalize_state=None), next_states)]
        _train_loop(self, dataset, optimizer, batch_size, num_epochs, step_loss, writer, ["loss/state/{}"],
                    criterion)

    def evaluate_model(self, dataset, batch_size, criterion=None):
        """models.py:30-51: one criterion value per batch and horizon step."""
        criterion = criterion or torch.nn.MSELoss()
        dev = _device_of(self)
        if dataset.num_transitions() == 0:
            return []
        _, ins, outs = dataset.stacked(dev)
        evals = []
        with torch.no_grad():
            for rows in _epoch_batches(dataset, batch_size):
                idx = torch.from_numpy(rows).to(dev)
                bi = [x.index_select(0, idx) for x in ins]
                bo = [x.index_select(0, idx) for x in outs]
                for h in range(dataset.horizon):
                    hat = self.forward(bi[0][:, h], bi[1][:, h], normalize_action=None, normalize_state=None,
                                       unnormalize_state=None)
                    evals.append(np.asarray(criterion(hat, bo[1][:, h]).cpu()))
        return evals

    def forward(self, state, action, normalize_action=None, normalize_state=None, unnormalize_state=None):
        if state.is_cuda and not torch.is_grad_enabled() and getattr(self, "noise", None) is None:
            from . import fused
            out = fused.try_forward(self, state, action, normalize_action, normalize_state, unnormalize_state)
            if out is not None:
                return out
        if normalize_action:
            action = normalize_action(action)
        if normalize_state:
            state = normalize_state(state)
        x = torch.cat([state, action], dim=1)
        out = self._forward(x)
        if unnormalize_state:
            out = unnormalize_state(out)
        return out


class Model(DynamicsModel):
    """models.py:96-110 generalised to `n_hidden` Linear-ReLU layers (default 2 = the reference).

    Layers are named linear1 .. linear{n_hidden+1} so an n_hidden=2 state_dict loads into the
    reference's Model and vice versa."""

    def __init__(self, state_dim, action_dim, hidden_units=50, noise=None, n_hidden=2):
        super().__init__()
        self.state_dim, self.action_dim = state_dim, action_dim
        self.hidden_units, self.n_hidden = hidden_units, n_hidden
        dims = [state_dim + action_dim] + [hidden_units] * n_hidden + [state_dim]
        for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
            setattr(self, f"linear{i + 1}", nn.Linear(fi, fo))
        self.activation_fn = nn.ReLU()
        self.noise = noise

    def linears(self):
        m = self._modules   # the registered submodules (what getattr resolves to), without its overhead
        return [m[f"linear{i + 1}"] for i in range(self.n_hidden + 1)]

    def _forward(self, x):
        lins = self.linears()
        for lin in lins[:-1]:
            x = self.activation_fn(lin(x))
        x = lins[-1](x)
        return x if self.noise is None else x + torch.randn_like(x) * self.noise


class LinearModel(DynamicsModel):
    """models.py:113-122: one Linear from (s, a) to s, plus optional Gaussian noise (experiment.py:41's
    "lin" model). The fused kernels need a hidden layer, so the planners run this model through its
    callable and train_model through autograd."""

    def __init__(self, state_dim, action_dim, noise=None):
        super().__init__()
        self.state_dim, self.action_dim = state_dim, action_dim
        self.linear1 = nn.Linear(state_dim + action_dim, state_dim)
        self.noise = noise

    def _forward(self, x):
        x = self.linear1(x)
        return x if self.noise is None else x + torch.randn_like(x) * self.noise


class EnsembleModel(DynamicsModel):
    """PETS-style ensemble of E `Model`s (not in the reference; BASELINE.json config 5).

    The CEM planner rolls every member out on the same actions and scores a candidate by the mean
    of the members' returns. Called directly, forward() returns the member-mean next state."""

    def __init__(self, members):
        super().__init__()
        self.members = nn.ModuleList(members)
        m0 = self.members[0]
        for m in self.members:
            if not isinstance(m, Model) or (m.state_dim, m.action_dim, m.hidden_units, m.n_hidden) != \
                    (m0.state_dim, m0.action_dim, m0.hidden_units, m0.n_hidden):
                raise ValueError("EnsembleModel members must be Models of one shape")
        self.state_dim, self.action_dim = m0.state_dim, m0.action_dim
        self.hidden_units, self.n_hidden = m0.hidden_units, m0.n_hidden
        self.noise = None

    def _forward(self, x):
        return torch.stack([m._forward(x) for m in self.members]).mean(0)


class ModelWithReward(nn.Module):
    """models.py:125-163: a shared Linear-ReLU trunk, state head and reward head. `n_hidden`
    generalises the reference's 2-layer trunk. Layers are linear1..linear{n_hidden} (trunk),
    linear{n_hidden+1} (state head) and linear{n_hidden+2} (reward head). n_hidden=2 gives the
    reference's names, so state_dicts load both ways.

    The planners take RewardAgent's wiring (agents.py:342-362) on the fused path: the model closure
    compose(partial(model, ...), itemgetter(0)) and the cost closure compose(partial(model, ...),
    itemgetter(1)). The cost is the unnormalised reward head at (s_{t+1}, a_t)."""

    def __init__(self, state_dim, action_dim, hidden_units=200, n_hidden=2):
        super().__init__()
        self.train_iterations = 0
        self.state_dim, self.action_dim = state_dim, action_dim
        self.hidden_units, self.n_hidden = hidden_units, n_hidden
        dims = [state_dim + action_dim] + [hidden_units] * n_hidden
        for i, (fi, fo) in enumerate(zip(dims[:-1], dims[1:])):
            setattr(self, f"linear{i + 1}", nn.Linear(fi, fo))
        setattr(self, f"linear{n_hidden + 1}", nn.Linear(hidden_units, state_dim))
        setattr(self, f"linear{n_hidden + 2}", nn.Linear(hidden_units, 1))
        self.activation_fn = nn.ReLU()

    def linears(self):
        """Trunk layers, state head, reward head (the packing order of mbrl_mlp_pack)."""
        m = self._modules
        return [m[f"linear{i + 1}"] for i in range(self.n_hidden + 2)]

    def _forward(self, x):
        lins = self.linears()
        for lin in lins[:self.n_hidden]:
            x = self.activation_fn(lin(x))
        return lins[-2](x), lins[-1](x)

    def train_model(self, dataset, optimizer, batch_size=512, num_epochs=50, criterion=None, writer=None):
        """models.py:165-217: state loss + reward loss per horizon step."""
        criterion = criterion or torch.nn.MSELoss()

        def step_loss(inp, out):
            (states, actions), (rewards, next_states) = inp, out
            s_hat, r_hat = self.forward(states, actions, normalize_action=None, normalize_state=None,
                                        unnormalize_state=None, unnormalize_reward=None)
            return [criterion(s_hat, next_states), criterion(r_hat, rewards.reshape(-1, 1))]
        _train_loop(self, dataset, optimizer, batch_size, num_epochs, step_loss, writer,
                    ["loss/state/{}", "loss/reward/{}"], criterion)

    def forward(self, state, action, normalize_state=None, unnormalize_state=None, normalize_action=None,
                unnormalize_reward=None):
        if normalize_action:
            action = normalize_action(action)
        if normalize_state:
            state = normalize_state(state)
        x = torch.cat([state, action], dim=1)
        state, reward = self._forward(x)
        if unnormalize_reward:
            reward = unnormalize_reward(reward)
        if unnormalize_state:
            state = unnormalize_state(state)
        return state, reward


class CostModel(nn.Module):
    """models.py:220-234: a learned cost of (state, action), two ReLU layers and a scalar head."""

    def __init__(self, state_dim, action_dim, hidden_units=70):
        super().__init__()
        self.linear1 = nn.Linear(state_dim + action_dim, hidden_units)
        self.linear2 = nn.Linear(hidden_units, hidden_units)
        self.linear3 = nn.Linear(hidden_units, 1)
        self.activation_fn = nn.ReLU()

    def forward(self, state, action):
        x = torch.cat((state, action), -1)
        x = self.activation_fn(self.linear1(x))
        x = self.activation_fn(self.linear2(x))
        return self.linear3(x)


class StateCost(nn.Module):
    goal_state = None

    def set_goal_state(self, goal_state):
        self.goal_state = goal_state


class SmoothAbsLoss(StateCost):
    """models.py:244-259: sum_d sqrt((w_d (x_d - g_d))^2 + alpha^2) - alpha."""

    def __init__(self, weights, goal_state, alpha=0.4):
        super().__init__()
        self.alpha = alpha
        self.weights = weights
        self.goal_state = goal_state

    def forward(self, x):
        x = x - self.goal_state
        return torch.sum(torch.sqrt((x * self.weights) ** 2 + self.alpha ** 2) - self.alpha, dim=-1)


class QuadraticCost(StateCost):
    """models.py:275-288: (x - g) . L(x - g) with a learned Linear L on the state. The reference's
    forward reads `self.goalState`, an attribute it never sets, so it raises AttributeError; this
    restatement computes what the code spells out with the goal it stores (`goal_state`)."""

    def __init__(self, dim, goal_state):
        super().__init__()
        self.linear = nn.Linear(dim, dim)
        self.goal_state = goal_state

    def forward(self, x):
        d = x - self.goal_state
        return torch.dot(d, self.linear(d))


class CoshLoss(nn.Module):
    """models.py:262-272: alpha^2 * mean_d(cosh(a_d / alpha) - 1)."""

    def __init__(self, alpha=0.25):
        super().__init__()
        self.alpha = alpha

    def forward(self, x):
        return (self.alpha ** 2) * torch.mean(torch.cosh(x / self.alpha) - 1, dim=-1)


def state_action_cost(state, action, state_cost, action_cost):
    """agents.py:182-183."""
    return state_cost(state) + action_cost(action)


def compose(a, b):
    """agents.py:300-304."""
    def ab(*args, **kwargs):
        return b(a(*args, **kwargs))
    return ab


def goal_state_cost(state_cost, action_cost):
    """The cost GoalStateAgent hands the planner (agents.py:231)."""
    return functools.partial(state_action_cost, state_cost=state_cost, action_cost=action_cost)
