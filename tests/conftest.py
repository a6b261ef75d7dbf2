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
