"""Oracle (TEST INFRASTRUCTURE ONLY): counter-based RNG for the CEM sampler, restated in NumPy.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline / parity leg may import
this module. The shipped planner never does: its sampler is the HIP device function in
`mujoco-mbrl_amd/csrc/mbrl_rng.h`, and this file is the checker for it.

Why a counter RNG at all: the reference samples candidate actions with the global
`np.random.uniform` (`/root/reference/src/mbrl/env_wrappers.py:50-62`). That stream cannot be
reproduced on a GPU or split across ranks, so the CEM path (which the reference does not have,
SURVEY.md fact 1 / §8a a11) draws its Gaussian perturbations from Philox4x32-10 keyed by
(seed) with counter (global candidate n, timestep t, CEM iteration i, action group d>>2).
The same draw is therefore identical on the host, on one GPU and on any number of GPUs.

Philox4x32-10 follows Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11), the
Random123 reference constants; it is pinned by the published known-answer vectors in
`tests/test_oracle_rng.py`.

The normal transform is a Box-Muller pair built only from IEEE-754 float32 operations that are
correctly rounded everywhere (+, -, *, /, sqrt, exact int->float conversion) in a fixed order
with no fused multiply-add, so the device sampler reproduces it bit for bit. log and sin/cos
are short fixed polynomials (|rel err| < 3e-7 against libm), which is ample for a CEM proposal.
"""
import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint32(0x9E3779B9)
PHILOX_W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def _f32(bits):
    return np.uint32(bits).view(np.float32)


# float32 constants, fixed by bit pattern so host and device agree exactly
LN2 = _f32(0x3F317218)
SQRT2 = _f32(0x3FB504F3)
INV3 = _f32(0x3EAAAAAB)
INV5 = _f32(0x3E4CCCCD)
INV7 = _f32(0x3E124925)
INV9 = _f32(0x3DE38E39)
INV11 = _f32(0x3DBA2E8C)
HALF_PI = _f32(0x3FC90FDB)
S3 = _f32(0x3E2AAAAB)
S5 = _f32(0x3C088889)
S7 = _f32(0x39500D01)
S9 = _f32(0x3638EF1D)
C2 = _f32(0x3F000000)
C4 = _f32(0x3D2AAAAB)
C6 = _f32(0x3AB60B61)
C8 = _f32(0x37D00D01)
C10 = _f32(0x3493F27E)
TWO_M24 = np.float32(2.0 ** -24)
ONE = np.float32(1.0)
TWO = np.float32(2.0)
HALF = np.float32(0.5)
MINUS_TWO = np.float32(-2.0)


def philox4x32_10(ctr, key):
    """Philox4x32 with 10 rounds.

    ctr: uint32 array [..., 4]; key: uint32 array [..., 2] (broadcastable). Returns uint32 [..., 4].
    """
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    c0, c1, c2, c3 = (ctr[..., i].astype(np.uint64) for i in range(4))
    k0 = np.broadcast_to(key[..., 0], ctr.shape[:-1]).astype(np.uint64)
    k1 = np.broadcast_to(key[..., 1], ctr.shape[:-1]).astype(np.uint64)
    for r in range(10):
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        n0 = hi1 ^ c1 ^ k0
        n2 = hi0 ^ c3 ^ k1
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        if r != 9:
            k0 = (k0 + np.uint64(PHILOX_W0)) & _MASK32  # uint32 wrap-around
            k1 = (k1 + np.uint64(PHILOX_W1)) & _MASK32
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def _log_f32(u):
    """ln(u) for float32 u in (0, 1], fixed-order float32 arithmetic (no FMA)."""
    bits = u.view(np.uint32)
    e = (bits >> np.uint32(23)).astype(np.int32) - np.int32(127)
    m = ((bits & np.uint32(0x007FFFFF)) | np.uint32(0x3F800000)).view(np.float32)
    big = m > SQRT2
    m = np.where(big, m * HALF, m).astype(np.float32)
    e = np.where(big, e + np.int32(1), e)
    f = (m - ONE).astype(np.float32)                 # exact (Sterbenz)
    s = (f / (TWO + f)).astype(np.float32)
    z = (s * s).astype(np.float32)
    p = (INV9 + (z * INV11).astype(np.float32)).astype(np.float32)
    p = (INV7 + (z * p).astype(np.float32)).astype(np.float32)
    p = (INV5 + (z * p).astype(np.float32)).astype(np.float32)
    p = (INV3 + (z * p).astype(np.float32)).astype(np.float32)
    p = (z * p).astype(np.float32)
    lnm = ((s + s).astype(np.float32) + ((s + s).astype(np.float32) * p).astype(np.float32)).astype(np.float32)
    return ((e.astype(np.float32) * LN2).astype(np.float32) + lnm).astype(np.float32)


def _sincos_turn_f32(v):
    """(sin, cos) of 2*pi*v for float32 v in [0, 1), fixed-order float32 arithmetic (no FMA)."""
    v4 = (v * np.float32(4.0)).astype(np.float32)      # exact
    q = np.floor(v4).astype(np.int32)
    f = (v4 - q.astype(np.float32)).astype(np.float32)  # exact, in [0, 1)
    hi = f >= HALF
    f = np.where(hi, (f - ONE).astype(np.float32), f).astype(np.float32)   # exact, in [-0.5, 0.5)
    q = np.where(hi, q + np.int32(1), q) & np.int32(3)
    x = (f * HALF_PI).astype(np.float32)
    x2 = (x * x).astype(np.float32)
    ps = (S7 - (x2 * S9).astype(np.float32)).astype(np.float32)
    ps = (S5 - (x2 * ps).astype(np.float32)).astype(np.float32)
    ps = (S3 - (x2 * ps).astype(np.float32)).astype(np.float32)
    sn = (x - ((x * x2).astype(np.float32) * ps).astype(np.float32)).astype(np.float32)
    pc = (C8 - (x2 * C10).astype(np.float32)).astype(np.float32)
    pc = (C6 - (x2 * pc).astype(np.float32)).astype(np.float32)
    pc = (C4 - (x2 * pc).astype(np.float32)).astype(np.float32)
    pc = (C2 - (x2 * pc).astype(np.float32)).astype(np.float32)
    cs = (ONE - (x2 * pc).astype(np.float32)).astype(np.float32)
    # rotate by the quadrant: theta = x + q*pi/2
    s_out = np.select([q == 0, q == 1, q == 2], [sn, cs, -sn], -cs).astype(np.float32)
    c_out = np.select([q == 0, q == 1, q == 2], [cs, -sn, -cs], sn).astype(np.float32)
    return s_out, c_out


def box_muller_f32(x0, x1):
    """Two standard normals from two uint32 words (exactly reproducible float32 Box-Muller)."""
    u1 = (((x0 >> np.uint32(8)) + np.uint32(1)).astype(np.float32) * TWO_M24).astype(np.float32)  # (0,1]
    u2 = ((x1 >> np.uint32(8)).astype(np.float32) * TWO_M24).astype(np.float32)                   # [0,1)
    r = np.sqrt((MINUS_TWO * _log_f32(u1)).astype(np.float32)).astype(np.float32)
    sn, cs = _sincos_turn_f32(u2)
    return (r * cs).astype(np.float32), (r * sn).astype(np.float32)


def seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)


def cem_normals(seed, iteration, n_idx, horizon, action_dim):
    """eps[t, j, d] ~ N(0,1) for global candidates n_idx[j]; float32 [H, len(n_idx), a].

    Counter = (n, t, iteration, d >> 2); the 4 Philox words give two Box-Muller pairs:
    d&3 = 0,1 <- (w0, w1) as (r cos, r sin); d&3 = 2,3 <- (w2, w3).
    Same layout as `mbrl_cem_normal` in mujoco-mbrl_amd/csrc/mbrl_rng.h.
    """
    n_idx = np.asarray(n_idx, dtype=np.uint32)
    groups = (action_dim + 3) // 4
    t = np.arange(horizon, dtype=np.uint32)
    g = np.arange(groups, dtype=np.uint32)
    T, Nn, G = np.meshgrid(t, n_idx, g, indexing="ij")
    ctr = np.stack([Nn, T, np.full_like(T, np.uint32(iteration)), G], axis=-1)
    w = philox4x32_10(ctr, seed_key(seed))
    z0, z1 = box_muller_f32(w[..., 0], w[..., 1])
    z2, z3 = box_muller_f32(w[..., 2], w[..., 3])
    z = np.stack([z0, z1, z2, z3], axis=-1).reshape(horizon, len(n_idx), groups * 4)
    return np.ascontiguousarray(z[..., :action_dim])


def cem_actions(mu, sigma, lo, hi, seed, iteration, n_idx):
    """a[t, j, d] = clip(mu[t,d] + sigma[t,d] * eps[t,j,d], lo, hi), float32, no FMA.

    Restates `mbrl_cem_action` (csrc/mbrl_rng.h). The clip bounds are the reference's dim-0 action
    bounds `[max(min[0], -3), min(max[0], 3)]` (`/root/reference/src/mbrl/env_wrappers.py:52-55`).
    """
    mu = np.asarray(mu, dtype=np.float32)
    sigma = np.asarray(sigma, dtype=np.float32)
    H, a = mu.shape
    eps = cem_normals(seed, iteration, n_idx, H, a)
    x = (mu[:, None, :] + (sigma[:, None, :] * eps).astype(np.float32)).astype(np.float32)
    return np.minimum(np.maximum(x, np.float32(lo)), np.float32(hi)).astype(np.float32)
