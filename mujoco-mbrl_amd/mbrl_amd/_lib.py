"""ctypes binding of the HIP extension's C ABI (include/mbrl_cem.h).

The library is built in-tree (`make -C mujoco-mbrl_amd`, or `__graft_entry__.build()`) and loaded
from this directory. There is no fallback: if the library is missing every fused entry point
raises, so a GPU run can never silently take a CPU path.

torch is imported first on purpose: torch's bundled libamdhip64 and /opt/rocm's share the soname
libamdhip64.so.7, so the extension binds to the runtime torch already loaded and the stream handles
it receives (torch.cuda.current_stream().cuda_stream) are valid for it.
"""
import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_size_t, c_uint64, c_void_p

import numpy as np
import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_PATH = os.environ.get("MBRL_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                          "libmbrl_cem.so")

MBRL_OK = 0
MBRL_COMM_ID_BYTES = 128
MBRL_EINVAL = -1
MBRL_EUNSUPPORTED = -2
MBRL_EHIP = -3
MBRL_EWORKSPACE = -4
MBRL_EPEER = -5          # mbrl_cem_plan_sharded: another rank failed during the plan (ABI v13)
MBRL_COST_GOAL_STATE = 0
MBRL_COST_MODEL_REWARD = 1
ABI_VERSION = 13
MBRL_NAN_LAST = 0
MBRL_NAN_FIRST = 1
MBRL_PRECISION_F32 = 0
MBRL_PRECISION_F16X3 = 1
MBRL_PRECISION_F16X6 = 2
PRECISIONS = {"f32": MBRL_PRECISION_F32, "f16x3": MBRL_PRECISION_F16X3, "f16x6": MBRL_PRECISION_F16X6}
# mbrl_set_option switches (include/mbrl_cem.h MBRL_OPT_*): A/B runs and forced fallbacks in tests
OPTIONS = {"rollout_tile": 0, "split_tile": 1, "debug_traj_abort": 2, "gd_single": 3, "debug_gd_abort": 4,
           "unfused_update": 5, "adam_arith": 6, "xcd_map": 7, "train_tile": 8, "train_no_fold": 9,
           "rollout_pair": 10, "shard_emulate": 11, "debug_pair_abort": 12,
           "traj_hop": 13, "gd_hop": 14, "pair_l2": 15,
           "train_xcd": 16, "train_split": 17, "debug_shard_fail": 18, "train_fo": 19,
           "debug_shard_fail_rank": 20, "update_split": 21}


def precision_code(name):
    """'f32' (exact fp32 MFMA), 'f16x3' or 'f16x6' (fp32 emulated on the f16 matrix cores with 2 or 3
    operand pieces; include/mbrl_cem.h)."""
    try:
        return PRECISIONS[str(name).lower()]
    except KeyError:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {name!r}") from None

# Every symbol include/mbrl_cem.h declares (tests/test_abi.py checks the two lists agree).
EXPORTED = (
    "mbrl_abi_version", "mbrl_last_error", "mbrl_set_option", "mbrl_get_option", "mbrl_mlp_packed_bytes",
    "mbrl_mlp_pack",
    "mbrl_rollout_cost", "mbrl_select_workspace_bytes", "mbrl_select_elites",
    "mbrl_refit_workspace_bytes", "mbrl_cem_refit", "mbrl_sample_actions",
    "mbrl_trajectory_workspace_bytes", "mbrl_trajectory", "mbrl_cem_workspace_bytes", "mbrl_cem_plan",
    "mbrl_cem_plan_batch_workspace_bytes", "mbrl_cem_plan_batch", "mbrl_gd_workspace_bytes", "mbrl_gd_plan",
    "mbrl_cem_update", "mbrl_adam_step", "mbrl_train_workspace_bytes", "mbrl_train_status_offset",
    "mbrl_train_grads",
    "mbrl_train_epoch", "mbrl_gd_batch_workspace_bytes", "mbrl_gd_plan_batch", "mbrl_host_alloc",
    "mbrl_host_free", "mbrl_comm_unique_id", "mbrl_comm_init", "mbrl_comm_destroy",
    "mbrl_cem_plan_sharded_workspace_bytes", "mbrl_cem_plan_sharded",
    "mbrl_build_info", "mbrl_event_create", "mbrl_event_record", "mbrl_stream_wait_event", "mbrl_event_synchronize",
    "mbrl_event_destroy",
)


class MlpShape(ctypes.Structure):
    _fields_ = [("state_dim", c_int32), ("action_dim", c_int32), ("hidden", c_int32),
                ("n_hidden", c_int32), ("ensemble", c_int32), ("reward_head", c_int32), ("precision", c_int32)]


class Norm(ctypes.Structure):
    _fields_ = [("obs_mean", c_void_p), ("obs_std", c_void_p), ("act_mean", c_void_p),
                ("act_std", c_void_p), ("rew_mean", c_void_p), ("rew_std", c_void_p),
                ("normalize_state", c_int32), ("unnormalize_state", c_int32),
                ("normalize_action", c_int32), ("unnormalize_reward", c_int32)]


class Cost(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("has_state_cost", c_int32), ("has_action_cost", c_int32),
                ("_pad", c_int32), ("weights", c_void_p), ("goal", c_void_p),
                ("alpha_state", c_float), ("alpha_action", c_float)]


class Sampler(ctypes.Structure):
    _fields_ = [("seed", c_uint64), ("iteration", c_int32), ("_pad", c_int32), ("mu", c_void_p),
                ("sigma", c_void_p), ("lo", c_float), ("hi", c_float)]


class CemParams(ctypes.Structure):
    _fields_ = [("N", c_int32), ("H", c_int32), ("K", c_int32), ("iterations", c_int32),
                ("alpha", c_float), ("lo", c_float), ("hi", c_float), ("init_mu", c_float),
                ("init_sigma", c_float), ("_pad", c_int32), ("seed", c_uint64)]


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("numel", c_int64), ("step_size", c_float), ("bc2_sqrt", c_float)]


class AdamHparams(ctypes.Structure):
    _fields_ = [("lerp_weight", c_float), ("beta2", c_float), ("one_minus_beta2", c_float), ("eps", c_float),
                ("weight_decay", c_float)]


TRAIN_MAX_LAYERS = 10


class TrainModel(ctypes.Structure):
    _fields_ = [("state_dim", c_int32), ("action_dim", c_int32), ("hidden", c_int32), ("n_hidden", c_int32),
                ("reward_head", c_int32), ("horizon", c_int32), ("weight", c_void_p * TRAIN_MAX_LAYERS),
                ("bias", c_void_p * TRAIN_MAX_LAYERS), ("weight_grad", c_void_p * TRAIN_MAX_LAYERS),
                ("bias_grad", c_void_p * TRAIN_MAX_LAYERS)]


class TrainData(ctypes.Structure):
    _fields_ = [("states", c_void_p), ("actions", c_void_p), ("next_states", c_void_p), ("rewards", c_void_p),
                ("transitions", c_int64)]


_lib = None


def load():
    """Load (once) and type the extension. Raises ImportError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"mbrl_amd HIP extension not found at {LIB_PATH}; build it with "
            "`make -C mujoco-mbrl_amd` or `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    P = c_void_p
    sig = {
        "mbrl_abi_version": (c_int32, []),
        "mbrl_build_info": (ctypes.c_char_p, []),
        "mbrl_last_error": (ctypes.c_char_p, []),
        "mbrl_set_option": (c_int32, [c_int32, c_int32]),
        "mbrl_get_option": (c_int32, [c_int32]),
        "mbrl_host_alloc": (c_int32, [c_size_t, POINTER(c_void_p), POINTER(c_void_p)]),
        "mbrl_host_free": (c_int32, [c_void_p]),
        "mbrl_event_create": (c_int32, [POINTER(c_void_p)]),
        "mbrl_event_record": (c_int32, [c_void_p, c_void_p]),
        "mbrl_stream_wait_event": (c_int32, [c_void_p, c_void_p]),
        "mbrl_event_synchronize": (c_int32, [c_void_p]),
        "mbrl_event_destroy": (c_int32, [c_void_p]),
        "mbrl_mlp_packed_bytes": (c_size_t, [POINTER(MlpShape)]),
        "mbrl_mlp_pack": (c_int32, [POINTER(MlpShape), POINTER(c_void_p), POINTER(c_void_p), P, P]),
        "mbrl_rollout_cost": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), POINTER(Cost), P, c_int32, P,
                                        POINTER(Sampler), c_int32, c_int32, c_int32, P, P, P, P]),
        "mbrl_select_workspace_bytes": (c_size_t, [c_int32]),
        "mbrl_select_elites": (c_int32, [P, c_int32, c_int32, c_int32, c_int32, P, P, P, c_size_t, P]),
        "mbrl_refit_workspace_bytes": (c_size_t, [c_int32, c_int32, c_int32]),
        "mbrl_cem_refit": (c_int32, [POINTER(Sampler), c_int32, c_int32, P, c_int32, c_float, P, P, P,
                                     c_size_t, P]),
        "mbrl_sample_actions": (c_int32, [POINTER(Sampler), c_int32, c_int32, c_int32, c_int32, P, P]),
        "mbrl_cem_update": (c_int32, [P, c_int32, c_int32, c_int32, POINTER(Sampler), c_int32, c_int32, c_float, P, P,
                                      P, P, P, c_int32, c_int32, P]),
        "mbrl_trajectory_workspace_bytes": (c_size_t, [POINTER(MlpShape), c_int32]),
        "mbrl_trajectory": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), P, P, c_int32, P, P, P, c_size_t, P]),
        "mbrl_cem_plan_batch_workspace_bytes": (c_size_t, [POINTER(MlpShape), POINTER(CemParams), c_int32]),
        "mbrl_cem_plan_batch": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), POINTER(Cost), P, c_int32,
                                          POINTER(CemParams), P, P, P, P, P, c_size_t, P]),
        "mbrl_cem_workspace_bytes": (c_size_t, [POINTER(MlpShape), POINTER(CemParams)]),
        "mbrl_gd_workspace_bytes": (c_size_t, [POINTER(MlpShape), c_int32]),
        "mbrl_gd_batch_workspace_bytes": (c_size_t, [POINTER(MlpShape), c_int32, c_int32]),
        "mbrl_gd_plan_batch": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), POINTER(Cost), P, P, c_int32, c_int32,
                                         c_int32, c_float, c_float, P, P, P, c_size_t, P]),
        "mbrl_gd_plan": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), POINTER(Cost), P, P, c_int32, c_int32,
                                   c_float, c_float, P, P, P, c_size_t, P]),
        "mbrl_adam_step": (c_int32, [POINTER(AdamTensor), c_int32, POINTER(AdamHparams), P]),
        "mbrl_train_workspace_bytes": (c_size_t, [POINTER(TrainModel), c_int32]),
        "mbrl_train_status_offset": (c_size_t, [POINTER(TrainModel), c_int32]),
        "mbrl_train_grads": (c_int32, [POINTER(TrainModel), POINTER(TrainData), P, c_int32, P, P, c_size_t, P]),
        "mbrl_train_epoch": (c_int32, [POINTER(TrainModel), POINTER(TrainData), P, c_int64, c_int32, POINTER(AdamTensor),
                                       c_int32, POINTER(AdamHparams), P, P, P, P, c_size_t, P]),
        "mbrl_cem_plan": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), POINTER(Cost), P, POINTER(CemParams),
                                    P, P, P, P, P, P, P, P, P, c_size_t, P]),
        "mbrl_comm_unique_id": (c_int32, [P]),
        "mbrl_comm_init": (c_int32, [P, c_int32, c_int32, POINTER(c_void_p)]),
        "mbrl_comm_destroy": (c_int32, [P]),
        "mbrl_cem_plan_sharded_workspace_bytes": (c_size_t, [POINTER(MlpShape), POINTER(CemParams), c_int32]),
        "mbrl_cem_plan_sharded": (c_int32, [POINTER(MlpShape), P, POINTER(Norm), POINTER(Cost), P,
                                            POINTER(CemParams), P, c_int32, c_int32, P, P, P, P, P, P, P, P, P,
                                            c_size_t, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mbrl_abi_version() != ABI_VERSION:
        raise ImportError(f"mbrl_amd ABI version mismatch: {lib.mbrl_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def source_digest():
    """The digest mujoco-mbrl_amd/Makefile compiles into mbrl_build_info(), recomputed from the tree's
    sources (None where they are absent)."""
    import glob
    import hashlib
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(pkg, "csrc", "*.hip")) + glob.glob(os.path.join(pkg, "csrc", "*.h")),
                   key=lambda f: os.path.relpath(f, pkg))
    if not any(f.endswith(".hip") for f in files):
        return None
    files.append(os.path.join(os.path.dirname(pkg), "include", "mbrl_cem.h"))
    if not all(os.path.exists(f) for f in files):
        return None
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info():
    """(the loaded library's source digest, whether it equals the tree's: None when the tree has no
    sources to compare with, e.g. an installed or prebuilt library)."""
    info = load().mbrl_build_info().decode()
    built = dict(kv.split("=", 1) for kv in info.split())["src"]
    tree = source_digest()
    return built, (None if tree is None else built == tree)


def check(rc, what):
    if rc != MBRL_OK:
        msg = load().mbrl_last_error()
        raise RuntimeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


class option:
    """Context manager around mbrl_set_option: `with option("rollout_tile", 8): ...` sets a
    process-wide switch and restores its previous value on exit (include/mbrl_cem.h MBRL_OPT_*)."""

    def __init__(self, name, value):
        self.code, self.value = OPTIONS[name], int(value)

    def __enter__(self):
        lib = load()
        prev = lib.mbrl_set_option(self.code, self.value)
        if prev < 0:
            check(prev, "mbrl_set_option")
        self.prev = prev
        return self

    def __exit__(self, *exc):
        load().mbrl_set_option(self.code, self.prev)
        return False


class HostStaging:
    """Mapped, coherent pinned host memory (mbrl_host_alloc) as `n` float32s: `.array` is the host's
    NumPy view, `.device` the address kernels read and write. Freed with the object."""

    def __init__(self, n):
        lib = load()
        h, d = c_void_p(), c_void_p()
        check(lib.mbrl_host_alloc(4 * int(n), ctypes.byref(h), ctypes.byref(d)), "mbrl_host_alloc")
        self._lib, self.host, self.n = lib, h.value, int(n)
        self.device = c_void_p(d.value)
        self.array = np.ctypeslib.as_array((ctypes.c_float * self.n).from_address(self.host))

    def at(self, offset):
        """Device address of element `offset`."""
        return c_void_p(self.device.value + 4 * int(offset))

    def cached_at(self, key, offsets):
        """at() of each offset, built once per `key` (a plan's fixed layout of this buffer)."""
        cache = self.__dict__.setdefault("_at", {})
        hit = cache.get(key)
        if hit is None:
            hit = cache[key] = tuple(self.at(o) for o in offsets)
        return hit

    def __del__(self):
        if getattr(self, "host", None):
            self._lib.mbrl_host_free(c_void_p(self.host))
            self.host = None


class StreamEvent:
    """A fence-free HIP event (mbrl_event_create: no timing, no system-scope fence at its record) for
    ordering one stream after another or letting the host wait: torch.cuda.Event's record idles the
    GPU ~5.5 us behind its system-scope fence. `record(stream)`, `wait(stream)` and `synchronize()` take
    torch streams; a never-recorded event is complete."""

    def __init__(self):
        lib = load()
        h = c_void_p()
        check(lib.mbrl_event_create(ctypes.byref(h)), "mbrl_event_create")
        self._lib, self.handle, self.recorded = lib, h, False

    def record(self, stream):
        check(self._lib.mbrl_event_record(self.handle, c_void_p(stream.cuda_stream)), "mbrl_event_record")
        self.recorded = True

    def wait(self, stream):
        if self.recorded:
            check(self._lib.mbrl_stream_wait_event(c_void_p(stream.cuda_stream), self.handle),
                  "mbrl_stream_wait_event")

    def synchronize(self):
        if self.recorded:
            check(self._lib.mbrl_event_synchronize(self.handle), "mbrl_event_synchronize")

    def __del__(self):
        if getattr(self, "handle", None):
            self._lib.mbrl_event_destroy(self.handle)
            self.handle = None


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else c_void_p(t.data_ptr())


def stream_handle(device=None):
    """The current HIP stream of `device` (a torch.device, an index or None: the current device) as
    the hipStream_t every entry point takes (the raw-pointer query: no Stream object per call)."""
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        if not isinstance(device, torch.device):
            device = torch.device(device)
        idx = device.index if device.index is not None else torch.cuda.current_device()
    return c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def require_gpu(t):
    if not t.is_cuda:
        raise RuntimeError("mbrl_amd fused path needs CUDA (HIP) tensors; got a CPU tensor")


__all__ = ["load", "check", "ptr", "stream_handle", "MlpShape", "Norm", "Cost", "Sampler", "CemParams",
           "EXPORTED", "MBRL_NAN_LAST", "MBRL_NAN_FIRST", "MBRL_COST_GOAL_STATE", "MBRL_COST_MODEL_REWARD",
           "ABI_VERSION", "c_int64", "MBRL_PRECISION_F32", "MBRL_PRECISION_F16X3", "MBRL_PRECISION_F16X6",
           "precision_code", "option", "OPTIONS", "AdamTensor", "AdamHparams",
           "TrainModel", "TrainData", "TRAIN_MAX_LAYERS", "HostStaging"]
