"""ctypes binding of the CPU parity oracle (oracle/tfhe_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package (zig-tfhe_amd/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libtfhe_oracle.so")
FAST_LIB_PATH = os.path.join(HERE, "build", "libtfhe_oracle_fast.so")


class OracleParams(C.Structure):
    _fields_ = [("n", C.c_uint32), ("N", C.c_uint32), ("nbit", C.c_uint32), ("L", C.c_uint32),
                ("bgbit", C.c_uint32), ("basebit", C.c_uint32), ("iks_t", C.c_uint32),
                ("_pad", C.c_uint32), ("alpha_lv0", C.c_double), ("alpha_lv1", C.c_double),
                ("alpha_ksk", C.c_double), ("alpha_bsk", C.c_double)]


# Parameter sets, params.zig.  KSK/BSK alphas: the reference hard-wires the
# 128-bit constants (params.zig:419-422) for every set; UINT4 keeps its own
# lv0/KSK noise and a zero BSK noise (its 2^-52 alpha is below the torus
# resolution).
PARAM_SETS = {
    "128": dict(n=700, N=1024, nbit=10, L=3, bgbit=6, basebit=2, iks_t=9,
                alpha_lv0=2.0e-5, alpha_lv1=2.0e-8, alpha_ksk=2.0e-5, alpha_bsk=2.0e-8),   # :350-375
    "80": dict(n=550, N=1024, nbit=10, L=3, bgbit=6, basebit=2, iks_t=7,
               alpha_lv0=5.0e-5, alpha_lv1=3.73e-8, alpha_ksk=2.0e-5, alpha_bsk=2.0e-8),   # :70-95
    "uint4": dict(n=820, N=1024, nbit=10, L=1, bgbit=22, basebit=5, iks_t=3,
                  alpha_lv0=0.00000251676160959795544987084234,
                  alpha_lv1=0.00000000000000022204460492503131,
                  alpha_ksk=0.00000251676160959795544987084234,
                  alpha_bsk=0.0),  # :210-235; BSK noise below torus resolution, see DESIGN.md
}


def params(name: str) -> OracleParams:
    return OracleParams(**PARAM_SETS[name])


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_P = C.POINTER
u32p, f64p, u8p = _P(C.c_uint32), _P(C.c_double), _P(C.c_uint8)


def _ptr(a: np.ndarray, t):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


class Oracle:
    """Thin numpy wrapper; every method maps 1:1 to a tfhe_oracle.c function."""

    def __init__(self, fast: bool = False):
        path = FAST_LIB_PATH if fast else LIB_PATH
        if not os.path.exists(path):
            build()
        self.lib = C.CDLL(path)
        L = self.lib
        L.oracle_f64_to_torus.restype = C.c_uint32
        L.oracle_f64_to_torus.argtypes = [C.c_double]
        L.oracle_decomposition_offset.restype = C.c_uint32
        L.oracle_tlwe_decrypt_bool.restype = C.c_int
        L.oracle_tlwe_phase.restype = C.c_uint32
        L.oracle_tlwe_decrypt_lwe_message.restype = C.c_uint32
        L.oracle_tlwe_encrypt_f64.argtypes = [C.c_uint32, C.c_double, C.c_double, u32p, C.c_uint64, u32p]
        L.oracle_tlwe_encrypt_lwe_message.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_double,
                                                       u32p, C.c_uint64, u32p]
        L.oracle_trlwe_encrypt_f64.argtypes = [C.c_void_p, f64p, C.c_double, u32p, C.c_uint64, u32p]
        L.oracle_secret_key_new.argtypes = [C.c_void_p, C.c_uint64, u32p, u32p]
        L.oracle_cloud_key_new.argtypes = [C.c_void_p, C.c_uint64, u32p, u32p, u32p, f64p]
        L.oracle_gate_batch.argtypes = [C.c_void_p, C.c_int, C.c_size_t, u8p, u32p, u32p, u32p, f64p,
                                        u32p, C.c_uint32, u32p]
        L.oracle_reencrypt.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, u32p, u32p, u32p]
        L.oracle_public_key_gen.argtypes = [C.c_uint32, u32p, C.c_size_t, C.c_double, C.c_uint64, u32p]
        L.oracle_public_key_encrypt_f64.argtypes = [C.c_uint32, u32p, C.c_size_t, C.c_double, C.c_double,
                                                    C.c_uint64, u32p]
        L.oracle_reenc_key_gen.argtypes = [C.c_uint32, u32p, u32p, u32p, C.c_size_t, C.c_double, C.c_uint32,
                                           C.c_uint32, C.c_uint64, u32p]
        L.oracle_set_trig_source.argtypes = [C.c_int]
        L.oracle_get_trig_source.restype = C.c_int
        L.oracle_take_round_error.restype = C.c_double
        L.oracle_capture_rounded.restype = C.c_size_t
        L.oracle_capture_rounded.argtypes = [C.c_void_p, C.c_size_t]
        L.oracle_set_fused.argtypes = [C.c_int]
        L.oracle_set_regroup.argtypes = [C.c_int]
        L.oracle_set_fold.argtypes = [C.c_int]
        L.oracle_folded_twiddles.argtypes = [C.c_uint32, C.c_void_p, C.c_void_p]
        L.oracle_get_fused.restype = C.c_int

    # ---- cos/sin source of the twiddles (0 glibc, 1 fdlibm/musl; tfhe_oracle.c)
    def set_trig_source(self, source: int):
        self.lib.oracle_set_trig_source(int(source))

    def trig_source(self) -> int:
        return self.lib.oracle_get_trig_source()

    def set_fused(self, fused):
        """Arithmetic of the transforms / MAC: reference expression trees (False / 0),
        fused multiply-adds (True / 1), or "guarded" (2): fused with the kernels'
        margin guard, a blind rotation that rounds near a tie redone in the
        reference's trees (the MI355X default at the 128/80-bit sets)."""
        self.lib.oracle_set_fused(2 if fused == 2 else int(bool(fused)))

    def set_regroup(self, mode):
        """Fused mode only: 1 / True = each output's MAC as (rows of a) + (rows of b),
        two fma chains from 0.0 added once (the pair and duo kernel forms); 2 = each
        row's product from 0.0, the six added in row order (the latency forms)."""
        self.lib.oracle_set_regroup(int(mode))

    def set_fold(self, fold):
        """Fused mode only: forward transforms with the twist folded into the stage
        twiddles (evidence only: no kernel uses it)."""
        self.lib.oracle_set_fold(int(bool(fold)))

    def folded_twiddles(self, N=1024):
        """The folded stage twiddles exp(i*pi*(1/2 - 2j)/len) at len/2 - 1 + j."""
        re, im = np.zeros(N // 2 - 1), np.zeros(N // 2 - 1)
        self.lib.oracle_folded_twiddles(N, re.ctypes.data, im.ctypes.data)
        return re + 1j * im

    def rounded_values(self, fn, cap=1 << 16):
        """Run fn() and return the pre-rounding values its inverse transforms
        rounded, in output order (coefficient i, then i + N/2 of each transform)."""
        buf = np.zeros(cap, np.float64)
        self.lib.oracle_capture_rounded(buf.ctypes.data, cap)
        try:
            fn()
        finally:
            n = self.lib.oracle_capture_rounded(None, 0)
        v = buf[:n].reshape(-1, 512, 2)  # [transform][i][re, im] -> coefficient order i ++ i + 512
        return np.concatenate([v[:, :, 0], v[:, :, 1]], axis=1).ravel()

    def take_round_error(self) -> float:
        """max |x - round(x)| of the inverse transforms run on this thread since the last call."""
        return self.lib.oracle_take_round_error()

    # ---- utils / fft
    def f64_to_torus(self, d: float) -> int:
        return self.lib.oracle_f64_to_torus(C.c_double(d))

    def twist_table(self, N=1024):
        re, im = np.zeros(N // 2), np.zeros(N // 2)
        self.lib.oracle_twist_table(C.c_uint32(N), _ptr(re, f64p), _ptr(im, f64p))
        return re, im

    def stage_twiddles(self, N=1024, inverse=False):
        re, im = np.zeros(N // 2 - 1), np.zeros(N // 2 - 1)
        self.lib.oracle_stage_twiddles(C.c_uint32(N), C.c_int(int(inverse)), _ptr(re, f64p), _ptr(im, f64p))
        return re, im

    def ifft(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.uint32)
        out = np.zeros(x.shape[-1], dtype=np.float64)
        self.lib.oracle_ifft(C.c_uint32(x.shape[-1]), _ptr(x, u32p), _ptr(out, f64p))
        return out

    def fft(self, f: np.ndarray) -> np.ndarray:
        f = np.ascontiguousarray(f, dtype=np.float64)
        out = np.zeros(f.shape[-1], dtype=np.uint32)
        self.lib.oracle_fft(C.c_uint32(f.shape[-1]), _ptr(f, f64p), _ptr(out, u32p))
        return out

    def poly_mul(self, a, b, naive=False):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros_like(a)
        fn = self.lib.oracle_poly_mul_naive if naive else self.lib.oracle_poly_mul
        fn(C.c_uint32(a.size), _ptr(a, u32p), _ptr(b, u32p), _ptr(out, u32p))
        return out

    # ---- trgsw / trlwe
    def decomposition_offset(self, p) -> int:
        return self.lib.oracle_decomposition_offset(C.byref(p))

    def decomposition(self, p, trlwe, offset):
        trlwe = np.ascontiguousarray(trlwe, dtype=np.uint32)
        out = np.zeros((2 * p.L, p.N), dtype=np.uint32)
        self.lib.oracle_decomposition(C.byref(p), _ptr(trlwe, u32p), C.c_uint32(offset), _ptr(out, u32p))
        return out

    def poly_mul_with_xk(self, a, k):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        out = np.zeros_like(a)
        self.lib.oracle_poly_mul_with_xk(C.c_uint32(a.size), _ptr(a, u32p), C.c_uint32(k), _ptr(out, u32p))
        return out

    def external_product(self, p, trgsw_fft, trlwe, offset):
        trgsw_fft = np.ascontiguousarray(trgsw_fft, dtype=np.float64)
        trlwe = np.ascontiguousarray(trlwe, dtype=np.uint32)
        out = np.zeros(2 * p.N, dtype=np.uint32)
        self.lib.oracle_external_product(C.byref(p), _ptr(trgsw_fft, f64p), _ptr(trlwe, u32p),
                                         C.c_uint32(offset), _ptr(out, u32p))
        return out

    def cmux(self, p, in1, in2, trgsw_fft, offset):
        in1 = np.ascontiguousarray(in1, dtype=np.uint32)
        in2 = np.ascontiguousarray(in2, dtype=np.uint32)
        trgsw_fft = np.ascontiguousarray(trgsw_fft, dtype=np.float64)
        out = np.zeros(2 * p.N, dtype=np.uint32)
        self.lib.oracle_cmux(C.byref(p), _ptr(in1, u32p), _ptr(in2, u32p), _ptr(trgsw_fft, f64p),
                             C.c_uint32(offset), _ptr(out, u32p))
        return out

    def blind_rotate(self, p, tlwe, testvec, bk, offset):
        tlwe = np.ascontiguousarray(tlwe, dtype=np.uint32)
        out = np.zeros(2 * p.N, dtype=np.uint32)
        self.lib.oracle_blind_rotate(C.byref(p), _ptr(tlwe, u32p), _ptr(testvec, u32p), _ptr(bk, f64p),
                                     C.c_uint32(offset), _ptr(out, u32p))
        return out

    def sample_extract_index(self, trlwe, k, N=1024):
        trlwe = np.ascontiguousarray(trlwe, dtype=np.uint32)
        out = np.zeros(N + 1, dtype=np.uint32)
        self.lib.oracle_sample_extract_index(C.c_uint32(N), _ptr(trlwe, u32p), C.c_uint32(k), _ptr(out, u32p))
        return out

    def sample_extract_index2(self, p, trlwe, k):
        trlwe = np.ascontiguousarray(trlwe, dtype=np.uint32)
        out = np.zeros(p.n + 1, dtype=np.uint32)
        self.lib.oracle_sample_extract_index2(C.c_uint32(p.n), C.c_uint32(p.N), _ptr(trlwe, u32p), C.c_uint32(k),
                                              _ptr(out, u32p))
        return out

    def bootstrap_without_key_switch(self, p, tlwe, keys):
        tlwe = np.ascontiguousarray(tlwe, dtype=np.uint32)
        out = np.zeros(p.n + 1, dtype=np.uint32)
        self.lib.oracle_bootstrap_without_key_switch(C.byref(p), _ptr(tlwe, u32p), _ptr(keys.testvec, u32p),
                                                     _ptr(keys.bk, f64p), C.c_uint32(keys.offset), _ptr(out, u32p))
        return out

    def identity_key_switch(self, p, lv1, ksk):
        lv1 = np.ascontiguousarray(lv1, dtype=np.uint32)
        out = np.zeros(p.n + 1, dtype=np.uint32)
        self.lib.oracle_identity_key_switch(C.byref(p), _ptr(lv1, u32p), _ptr(ksk, u32p), _ptr(out, u32p))
        return out

    def bootstrap(self, p, tlwe, keys):
        tlwe = np.ascontiguousarray(tlwe, dtype=np.uint32)
        out = np.zeros(p.n + 1, dtype=np.uint32)
        self.lib.oracle_bootstrap(C.byref(p), _ptr(tlwe, u32p), _ptr(keys.testvec, u32p),
                                  _ptr(keys.bk, f64p), _ptr(keys.ksk, u32p), C.c_uint32(keys.offset),
                                  _ptr(out, u32p))
        return out

    def gate_combine(self, p, op, a, b):
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros(p.n + 1, dtype=np.uint32)
        self.lib.oracle_gate_combine(C.byref(p), C.c_int(op), _ptr(a, u32p), _ptr(b, u32p), _ptr(out, u32p))
        return out

    def gate_batch(self, p, ops, a, b, keys, threads=1, testvec=None):
        ops = np.ascontiguousarray(ops, dtype=np.uint8)
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.zeros_like(a)
        tv = keys.testvec if testvec is None else np.ascontiguousarray(testvec, dtype=np.uint32)
        self.lib.oracle_gate_batch(C.byref(p), threads, ops.size, _ptr(ops, u8p), _ptr(a, u32p),
                                   _ptr(b, u32p), _ptr(tv, u32p), _ptr(keys.bk, f64p),
                                   _ptr(keys.ksk, u32p), keys.offset, _ptr(out, u32p))
        return out

    # ---- keys / encryption
    def secret_key(self, p, seed):
        k0 = np.zeros(p.n, dtype=np.uint32)
        k1 = np.zeros(p.N, dtype=np.uint32)
        self.lib.oracle_secret_key_new(C.byref(p), seed, _ptr(k0, u32p), _ptr(k1, u32p))
        return k0, k1

    def testvec(self, p):
        tv = np.zeros(2 * p.N, dtype=np.uint32)
        self.lib.oracle_testvec(C.byref(p), _ptr(tv, u32p))
        return tv

    def cloud_key(self, p, seed, k0, k1):
        base = 1 << p.basebit
        ksk = np.zeros((p.N * p.iks_t * base, p.n + 1), dtype=np.uint32)
        bk = np.zeros((p.n, 2 * p.L, 2, p.N), dtype=np.float64)
        self.lib.oracle_cloud_key_new(C.byref(p), seed, _ptr(k0, u32p), _ptr(k1, u32p),
                                      _ptr(ksk, u32p), _ptr(bk, f64p))
        return CloudKeyArrays(self.decomposition_offset(p), self.testvec(p), ksk, bk)

    def tlwe_encrypt_f64(self, n, mu, alpha, key, seed):
        out = np.zeros(n + 1, dtype=np.uint32)
        self.lib.oracle_tlwe_encrypt_f64(n, mu, alpha, _ptr(key, u32p), seed, _ptr(out, u32p))
        return out

    def tlwe_encrypt_bool(self, n, bit, alpha, key, seed):
        return self.tlwe_encrypt_f64(n, 0.125 if bit else -0.125, alpha, key, seed)

    def tlwe_decrypt_bool(self, n, ct, key) -> bool:
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        return bool(self.lib.oracle_tlwe_decrypt_bool(C.c_uint32(n), _ptr(ct, u32p), _ptr(key, u32p)))

    def tlwe_phase(self, n, ct, key) -> int:
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        return self.lib.oracle_tlwe_phase(C.c_uint32(n), _ptr(ct, u32p), _ptr(key, u32p))

    def trlwe_encrypt_f64(self, p, mu, alpha, key1, seed):
        mu = np.ascontiguousarray(mu, dtype=np.float64)
        out = np.zeros(2 * p.N, dtype=np.uint32)
        self.lib.oracle_trlwe_encrypt_f64(C.byref(p), _ptr(mu, f64p), alpha, _ptr(key1, u32p), seed,
                                          _ptr(out, u32p))
        return out

    def trlwe_decrypt_bool(self, p, ct, key1):
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        out = np.zeros(p.N, dtype=np.uint8)
        self.lib.oracle_trlwe_decrypt_bool(C.byref(p), _ptr(ct, u32p), _ptr(key1, u32p), _ptr(out, u8p))
        return out.astype(bool)

    def trgsw_encrypt_torus_fft(self, p, mu, alpha, key1, seed):
        rng = (C.c_uint64 * 4)()
        self.lib.oracle_rng_init(C.byref(rng), C.c_uint64(seed))
        out = np.zeros((2 * p.L, 2, p.N), dtype=np.float64)
        self.lib.oracle_trgsw_encrypt_torus_fft(C.byref(p), C.c_uint32(mu), C.c_double(alpha),
                                                _ptr(key1, u32p), C.byref(rng), _ptr(out, f64p))
        return out

    def lut_generate(self, N, m, f_table):
        f = np.ascontiguousarray(f_table, dtype=np.uint32)
        tv = np.zeros(2 * N, dtype=np.uint32)
        self.lib.oracle_lut_generate(C.c_uint32(N), C.c_uint32(m), _ptr(f, u32p), _ptr(tv, u32p))
        return tv

    def lut_generate_scaled(self, N, m, scale, f_table):
        f = np.ascontiguousarray(f_table, dtype=np.uint32)
        tv = np.zeros(2 * N, dtype=np.uint32)
        self.lib.oracle_lut_generate_scaled(C.c_uint32(N), C.c_uint32(m), C.c_double(scale), _ptr(f, u32p),
                                            _ptr(tv, u32p))
        return tv

    def lut_generate_full(self, N, m, values):
        v = np.ascontiguousarray(values, dtype=np.uint32)
        tv = np.zeros(2 * N, dtype=np.uint32)
        self.lib.oracle_lut_generate_full(C.c_uint32(N), C.c_uint32(m), _ptr(v, u32p), _ptr(tv, u32p))
        return tv

    def div_round(self, a, b):
        """divRound (lut/generator.zig:253-255)."""
        self.lib.oracle_div_round.restype = C.c_size_t
        return int(self.lib.oracle_div_round(C.c_size_t(a), C.c_size_t(b)))

    def lut_mod_switch(self, x, size):
        """Generator.modSwitch (lut/generator.zig:223-227)."""
        self.lib.oracle_lut_mod_switch.restype = C.c_size_t
        return int(self.lib.oracle_lut_mod_switch(C.c_uint32(x), C.c_size_t(size)))

    def encrypt_lwe_message(self, n, msg, m, alpha, key, seed):
        out = np.zeros(n + 1, dtype=np.uint32)
        self.lib.oracle_tlwe_encrypt_lwe_message(n, msg, m, alpha, _ptr(key, u32p), seed, _ptr(out, u32p))
        return out

    def decrypt_lwe_message(self, n, ct, m, key) -> int:
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        return self.lib.oracle_tlwe_decrypt_lwe_message(C.c_uint32(n), _ptr(ct, u32p), C.c_uint32(m),
                                                        _ptr(key, u32p))

    # ---- proxy re-encryption (proxy_reenc.zig)
    def reencrypt(self, n, basebit, t, ct, key):
        ct = np.ascontiguousarray(ct, dtype=np.uint32)
        out = np.zeros(n + 1, dtype=np.uint32)
        self.lib.oracle_reencrypt(n, basebit, t, _ptr(ct, u32p), _ptr(key, u32p), _ptr(out, u32p))
        return out

    def public_key_gen(self, n, key, size, alpha, seed0):
        pk = np.zeros((size, n + 1), dtype=np.uint32)
        self.lib.oracle_public_key_gen(n, _ptr(key, u32p), size, alpha, seed0, _ptr(pk, u32p))
        return pk

    def public_key_encrypt_f64(self, n, pk, plaintext, alpha, seed):
        out = np.zeros(n + 1, dtype=np.uint32)
        self.lib.oracle_public_key_encrypt_f64(n, _ptr(pk, u32p), pk.shape[0], plaintext, alpha, seed,
                                               _ptr(out, u32p))
        return out

    def reenc_key_gen(self, n, key_from, alpha, basebit, t, seed0, key_to=None, pk=None):
        """symmetric when key_to is given, asymmetric (public key) when pk is given"""
        assert (key_to is None) != (pk is None)
        out = np.zeros(((1 << basebit) * t * n, n + 1), dtype=np.uint32)
        self.lib.oracle_reenc_key_gen(n, _ptr(key_from, u32p), None if key_to is None else _ptr(key_to, u32p),
                                      None if pk is None else _ptr(pk, u32p),
                                      0 if pk is None else pk.shape[0], alpha, basebit, t, seed0,
                                      _ptr(out, u32p))
        return out


class CloudKeyArrays:
    """CloudKey fields (key.zig:61-66) as numpy arrays in the reference layout."""

    def __init__(self, offset, testvec, ksk, bk):
        self.offset, self.testvec, self.ksk, self.bk = int(offset), testvec, ksk, bk
