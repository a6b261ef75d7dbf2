"""The reference's examples, restated in examples/, run end to end on the GPU; and the
bit_utils.zig tests (:56-200) restated on the host mirror."""
import importlib.util
import os

import numpy as np
import pytest

import tfhe_amd
from conftest import ROOT


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "examples", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bit_utils_convert():  # bit_utils.zig "convert bits to number"
    bits = [True, False, True] + [False] * 29
    assert tfhe_amd.bit_utils.convert(bits[:8]) == 5
    assert tfhe_amd.bit_utils.convert(bits[:16]) == 5
    assert tfhe_amd.bit_utils.convert(bits) == 5


def test_bit_utils_to_bits():  # bit_utils.zig "to bits conversion", "as bits trait for u8/u16"
    b8 = tfhe_amd.bit_utils.to_bits(0b10101010, 8)
    assert list(b8) == [False, True] * 4  # LSB first
    b16 = tfhe_amd.bit_utils.to_bits(0b1010101010101010, 16)
    assert len(b16) == 16 and not b16[0] and b16[15]
    for v in (0, 1, 402, 65535):
        assert tfhe_amd.bit_utils.convert(tfhe_amd.bit_utils.to_bits(v, 16)) == v


def test_bit_utils_encrypt_roundtrip(oracle):
    from oracle import params
    p = params("128")
    k0, k1 = oracle.secret_key(p, 42)
    sk = tfhe_amd.SecretKey(tfhe_amd.make_params("128"), k0, k1)
    cts = tfhe_amd.bit_utils.encrypt(402, 16, sk, seed0=9)
    assert cts.shape == (16, 701)
    assert tfhe_amd.bit_utils.convert(sk.decrypt_bool(cts)) == 402


@pytest.mark.gpu
def test_add_two_numbers_example():
    assert _load("add_two_numbers").main(["--mode", "both"]) == 0


@pytest.mark.gpu
def test_proxy_reencryption_demo():
    assert _load("proxy_reencryption_demo").main(["--batch", "1024"]) == 0
