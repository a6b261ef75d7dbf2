"""Shared test setup: paths, the `gpu` marker, cached oracle keys."""
import os
import sys

import numpy as np
import pytest

try:  # load torch's HIP runtime before libtfhe_gpu.so so both share one runtime
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "zig-tfhe_amd"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import Oracle
    return Oracle()


class Keys:
    def __init__(self, o, name, sk_seed=42, ck_seed=43):
        from oracle import params
        self.name = name
        self.p = params(name)
        self.k0, self.k1 = o.secret_key(self.p, sk_seed)
        self.ck = o.cloud_key(self.p, ck_seed, self.k0, self.k1)


_KEYS = {}


def get_keys(o, name):
    if name not in _KEYS:
        _KEYS[name] = Keys(o, name)
    return _KEYS[name]


@pytest.fixture(scope="session")
def keys128(oracle):
    return get_keys(oracle, "128")


@pytest.fixture(scope="session")
def keys80(oracle):
    return get_keys(oracle, "80")


@pytest.fixture(scope="session")
def keys_uint4(oracle):
    return get_keys(oracle, "uint4")


def rng(seed=0):
    return np.random.default_rng(seed)


def crafted_near_tie_case(oracle, p, seed=3):
    """(testvec, reference-layout BK, TLWELv0) of a blind rotation whose fused
    arithmetic rounds near a tie and parts from the reference:
    constant test vector offset/2 (so tmp = -offset and every digit is -32 at
    step 0 with a~_0 = N, b~ = 2N), BK[0]'s rows all FFT(2^31 - 1), the other
    steps zero (their external products are exactly 0)."""
    off = oracle.decomposition_offset(p)
    tv = np.full(2 * p.N, off // 2, np.uint32)
    bk = np.zeros((p.n, 2 * p.L, 2, p.N))
    spec = oracle.ifft(np.full(p.N, (1 << 31) - 1, np.uint32))
    bk[0, :, :, :] = spec
    ct = rng(seed).integers(0, 1 << 32, p.n + 1, dtype=np.uint64).astype(np.uint32)
    ct[0], ct[p.n] = 1 << 31, 0  # a~_0 = N, b~ = 2N (identity)
    return tv, bk, ct
