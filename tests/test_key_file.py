"""Cloud-key files (include/tfhe_gpu.h 'Cloud-key files'; SURVEY §5 checkpoint row,
§8f N3).  The reference has no key serialization (every process runs CloudKey.new,
key.zig:70-77), so there is no reference fixture: the CPU tests pin the format
(header fields, checksum, parameter check, error codes) and the round trip; the
GPU tests check that a saved key reloads bit-exact and drives the same gates."""
import struct

import numpy as np
import pytest

import tfhe_amd
from conftest import rng

P80 = tfhe_amd.make_params("80")


def _random_key(p, seed=5):
    g = rng(seed)
    tv = g.integers(0, 1 << 32, 2 * p.N, dtype=np.uint64).astype(np.uint32)
    bk = g.standard_normal((p.n, 2 * p.L, 2, p.N)) * 1e9
    ksk = g.integers(0, 1 << 32, (p.N * p.iks_t * (1 << p.basebit), p.n + 1), dtype=np.uint64).astype(np.uint32)
    return 0x82080000, tv, bk, ksk


@pytest.fixture(scope="module")
def key80():
    return _random_key(P80)


@pytest.fixture
def written(tmp_path, key80):
    path = str(tmp_path / "ck80.key")
    off, tv, bk, ksk = key80
    tfhe_amd.cloud_key_write(path, P80, off, tv, bk, ksk)
    return path


def test_round_trip_bit_exact(written, key80):
    off, tv, bk, ksk = tfhe_amd.cloud_key_read(written, P80)
    assert off == key80[0]
    assert np.array_equal(tv, key80[1])
    assert np.array_equal(bk.view(np.uint64), key80[2].view(np.uint64))  # bit patterns, incl. signed zeros
    assert np.array_equal(ksk, key80[3])


def test_header_layout(written, key80):
    raw = open(written, "rb").read(64)
    magic, ver, n, N, L, bgbit, basebit, t, off, bl, kl, _ = struct.unpack("<8s8I3Q", raw)
    assert magic == b"ZTFHECK1" and ver == 1
    assert (n, N, L, bgbit, basebit, t) == (550, 1024, 3, 6, 2, 7)
    assert off == key80[0] and bl == key80[2].size and kl == key80[3].size
    import os
    assert os.path.getsize(written) == 64 + 2 * 1024 * 4 + bl * 8 + kl * 4


def test_checksum_detects_a_flipped_bit(written):
    with open(written, "r+b") as f:
        f.seek(64 + 8192 + 12345 * 8 + 3)
        b = f.read(1)
        f.seek(-1, 1)
        f.write(bytes([b[0] ^ 0x10]))
    with pytest.raises(tfhe_amd.TfheError, match="status -1"):
        tfhe_amd.cloud_key_read(written, P80)


def test_truncated_file_is_an_io_error(written):
    import os
    os.truncate(written, os.path.getsize(written) - 4)
    with pytest.raises(tfhe_amd.TfheError, match="status -5"):
        tfhe_amd.cloud_key_read(written, P80)


def test_other_parameter_set_is_rejected(written):
    with pytest.raises(tfhe_amd.TfheError, match="status -1"):
        tfhe_amd.cloud_key_read(written, tfhe_amd.make_params("128"))


def test_missing_file_and_bad_magic(tmp_path):
    with pytest.raises(tfhe_amd.TfheError, match="status -5"):
        tfhe_amd.cloud_key_read(str(tmp_path / "nope.key"), P80)
    junk = tmp_path / "junk.key"
    junk.write_bytes(b"\0" * 4096)
    with pytest.raises(tfhe_amd.TfheError, match="status -1"):
        tfhe_amd.cloud_key_read(str(junk), P80)


def test_write_rejects_wrong_lengths(tmp_path, key80):
    off, tv, bk, ksk = key80
    with pytest.raises(tfhe_amd.TfheError, match="status -1"):
        tfhe_amd.cloud_key_write(str(tmp_path / "x.key"), P80, off, tv, bk[:-1], ksk)


@pytest.mark.gpu
def test_gpu_save_load_drives_identical_gates(tmp_path):
    """keygen -> save -> a second context loads the file: same key bits
    (export_cloud_key vs keygen's host copy), same gate outputs."""
    c1 = tfhe_amd.Context("128", 0)
    sk, (bk, ksk) = c1.keygen(42, 43, want_host_copy=True)
    off, tv, bk_x, ksk_x = c1.export_cloud_key()
    assert np.array_equal(bk_x.view(np.uint64), bk.view(np.uint64))  # device layout round trip is exact
    nz = np.ones(ksk.shape[0], bool)
    nz[::1 << c1.params.basebit] = False  # k = 0 rows: never read, zero on the device
    assert np.array_equal(ksk_x[nz], ksk[nz])
    assert not ksk_x[~nz].any()
    path = str(tmp_path / "ck128.key")
    c1.save_cloud_key(path)
    c2 = tfhe_amd.Context("128", 0)
    c2.load_cloud_key_file(path)
    off2, tv2, bk2, ksk2 = c2.export_cloud_key()
    assert off2 == off and np.array_equal(tv2, tv)
    assert np.array_equal(bk2.view(np.uint64), bk_x.view(np.uint64)) and np.array_equal(ksk2, ksk_x)
    g = rng(9)
    ops = g.integers(0, 10, 64).astype(np.uint8)
    a = sk.encrypt_bool(g.integers(0, 2, 64).astype(np.uint8), seed0=100)
    b = sk.encrypt_bool(g.integers(0, 2, 64).astype(np.uint8), seed0=200)
    assert np.array_equal(c1.gate_batch(ops, a, b), c2.gate_batch(ops, a, b))
    c1.close()
    c2.close()
