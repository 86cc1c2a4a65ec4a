"""CPU: the oracle's counter RNG (oracle/philox.py) against published known answers and basic laws."""
import numpy as np
import pytest

from oracle import philox

# Random123 known-answer vectors for philox4x32 with 10 rounds (Salmon et al., SC'11; kat_vectors).
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_known_answers(ctr, key, expect):
    out = philox.philox4x32_10(np.array(ctr, np.uint32), np.array(key, np.uint32))
    assert [int(x) for x in out] == list(expect)


def test_philox_vectorised_matches_scalar():
    ctr = np.random.default_rng(0).integers(0, 2 ** 32, size=(37, 4), dtype=np.uint64).astype(np.uint32)
    key = np.array([0xDEADBEEF, 0x12345678], np.uint32)
    batch = philox.philox4x32_10(ctr, key)
    for i in range(len(ctr)):
        assert np.array_equal(batch[i], philox.philox4x32_10(ctr[i], key))


def test_log_and_sincos_accuracy():
    u = (np.arange(1, 2 ** 24 + 1, 4093).astype(np.float32) * philox.TWO_M24).astype(np.float32)
    ref = np.log(u.astype(np.float64))
    assert np.max(np.abs(philox._log_f32(u) - ref)) < 5e-7
    v = (np.arange(0, 2 ** 24, 4091).astype(np.float32) * philox.TWO_M24).astype(np.float32)
    s, c = philox._sincos_turn_f32(v)
    th = 2 * np.pi * v.astype(np.float64)
    assert np.max(np.abs(s - np.sin(th))) < 2e-7
    assert np.max(np.abs(c - np.cos(th))) < 2e-7


def test_normals_moments():
    z = philox.cem_normals(7, 0, np.arange(8192), 8, 6)
    assert z.dtype == np.float32 and z.shape == (8, 8192, 6)
    assert abs(float(z.mean())) < 0.01
    assert abs(float(z.std()) - 1.0) < 0.01
    # independent streams for different iterations / seeds
    assert not np.array_equal(z, philox.cem_normals(7, 1, np.arange(8192), 8, 6))
    assert not np.array_equal(z, philox.cem_normals(8, 0, np.arange(8192), 8, 6))


def test_actions_clip_and_shard_invariance():
    H, a = 5, 7
    mu = np.linspace(-1.5, 1.5, H * a, dtype=np.float32).reshape(H, a)
    sigma = np.full((H, a), 0.8, np.float32)
    full = philox.cem_actions(mu, sigma, -1.0, 1.0, 99, 3, np.arange(100))
    assert full.min() >= -1.0 and full.max() <= 1.0
    # drawing a shard of candidate indices reproduces the same rows: sharding cannot change samples
    part = philox.cem_actions(mu, sigma, -1.0, 1.0, 99, 3, np.arange(40, 75))
    assert np.array_equal(full[:, 40:75], part)
