"""Host-side mirror of zig-tfhe's public surface over the MI355X C ABI.

Names follow the reference (src/gates.zig `Gates.nandGate` ..., src/key.zig
`SecretKey` / `CloudKey`, src/tlwe.zig `TLWELv0`, src/params.zig parameter
sets); every method is a thin call into lib/libtfhe_gpu.so (include/tfhe_gpu.h).
There is no CPU fallback: without the built HIP library every entry point
raises.

Batches of ciphertexts are numpy uint32 arrays of shape (B, n+1) — B
TLWELv0 values laid out exactly as `TLWELv0.p` (tlwe.zig:11-12).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TFHE_GPU_LIB") or os.path.join(HERE, "lib", "libtfhe_gpu.so")  # env: A/B builds

# tfhe_gpu_set_option keys / values (include/tfhe_gpu.h TFHE_OPT_*, TFHE_TWIDDLES_*)
OPTIONS = {"br_form": 1, "br_loader": 2, "ks_form": 3, "ks_narrow": 4, "ks_item_groups": 5, "ks_sel_items": 6,
           "circuit_pack": 7, "twiddles": 8, "arith": 9, "br_sync": 10, "br_spin_cap": 11, "host_pipeline": 12,
           "circuit_split": 13, "host_staging": 17}
READONLY_OPTIONS = {"fused_admitted": 14, "level_issue_us": 15, "key_row_rms_ppm": 16}  # tfhe_gpu_get_option only
OPTION_DEFAULTS = {"br_form": 0, "br_loader": 1, "ks_form": 3, "ks_narrow": 0, "ks_item_groups": 0,
                   "ks_sel_items": 8, "circuit_pack": 1, "twiddles": 0, "arith": 0, "br_sync": 1, "br_spin_cap": 0,
                   "host_pipeline": 0, "circuit_split": 0, "host_staging": 0}
# status codes (include/tfhe_gpu.h TFHE_ERR_*)
ERR_INVALID, ERR_HIP, ERR_NO_KEY, ERR_OOM, ERR_IO, ERR_DEVICE = -1, -2, -3, -4, -5, -6
# 2 split, 4 pair: removed (round 4); 6 duo, 7 wide2: A/B libraries only (tools/ab/, round 5); 5 octo: L = 1
BR_FORMS = {"auto": 0, "whole": 1, "wide": 3, "octo": 5, "duo": 6, "wide2": 7, "plain": 8}
BUILD_PRODUCT, BUILD_AB = 0, 1  # tfhe_gpu_build_kind
TWIDDLES_GLIBC, TWIDDLES_FDLIBM = 0, 1
ARITH_AUTO, ARITH_REFERENCE, ARITH_FUSED_FORCED = 0, 1, 2
STAGING_PAGEABLE, STAGING_PINNED = 0, 1  # TFHE_OPT_HOST_STAGING

# gate op codes, include/tfhe_gpu.h TFHE_GATE_* (gates.zig:48-121)
NAND, OR, AND, XOR, XNOR, NOR, ANDNY, ANDYN, ORNY, ORYN = range(10)
NOT = 254  # circuits only: negation, no bootstrap
COPY = 255
GATE_NAMES = {"nand": NAND, "or": OR, "and": AND, "xor": XOR, "xnor": XNOR, "nor": NOR,
              "andny": ANDNY, "andyn": ANDYN, "orny": ORNY, "oryn": ORYN}


class TfheParams(C.Structure):
    _fields_ = [("n", C.c_uint32), ("N", C.c_uint32), ("nbit", C.c_uint32), ("L", C.c_uint32),
                ("bgbit", C.c_uint32), ("basebit", C.c_uint32), ("iks_t", C.c_uint32),
                ("_pad", C.c_uint32), ("alpha_lv0", C.c_double), ("alpha_lv1", C.c_double),
                ("alpha_ksk", C.c_double), ("alpha_bsk", C.c_double)]

    def __repr__(self):
        return (f"TfheParams(n={self.n}, N={self.N}, L={self.L}, bgbit={self.bgbit}, "
                f"basebit={self.basebit}, iks_t={self.iks_t})")


# params.zig parameter sets (runtime form).  KSK/BSK noise: the reference's
# KSK_ALPHA/BSK_ALPHA (params.zig:419-422) are the 128-bit constants; UINT4
# keeps its own set's alphas.
SECURITY_128_BIT = dict(n=700, N=1024, nbit=10, L=3, bgbit=6, basebit=2, iks_t=9,
                        alpha_lv0=2.0e-5, alpha_lv1=2.0e-8, alpha_ksk=2.0e-5, alpha_bsk=2.0e-8)
SECURITY_80_BIT = dict(n=550, N=1024, nbit=10, L=3, bgbit=6, basebit=2, iks_t=7,
                       alpha_lv0=5.0e-5, alpha_lv1=3.73e-8, alpha_ksk=2.0e-5, alpha_bsk=2.0e-8)
SECURITY_UINT4 = dict(n=820, N=1024, nbit=10, L=1, bgbit=22, basebit=5, iks_t=3,
                      alpha_lv0=0.00000251676160959795544987084234,
                      alpha_lv1=0.00000000000000022204460492503131,
                      alpha_ksk=0.00000251676160959795544987084234,
                      # 2^-52 is below the 32-bit torus resolution; the reference's
                      # f64ToTorus would turn it into a {0,-1} bias that the
                      # L=1/Bg=2^22 gadget amplifies 2^21x
                      alpha_bsk=0.0)
PARAM_SETS = {"128": SECURITY_128_BIT, "80": SECURITY_80_BIT, "uint4": SECURITY_UINT4}


def make_params(name_or_dict="128") -> TfheParams:
    d = PARAM_SETS[name_or_dict] if isinstance(name_or_dict, str) else name_or_dict
    return TfheParams(**d)


_lib = None
u32p, f64p, u8p, vp = C.POINTER(C.c_uint32), C.POINTER(C.c_double), C.POINTER(C.c_uint8), C.c_void_p

_SIGS = {
    "tfhe_gpu_abi_version": (C.c_int, []),
    "tfhe_gpu_build_id": (C.c_char_p, []),
    "tfhe_gpu_build_kind": (C.c_int, []),
    "tfhe_gpu_create": (C.c_int, [C.POINTER(TfheParams), C.c_int, C.POINTER(vp)]),
    "tfhe_gpu_create_on_device": (C.c_int, [C.POINTER(TfheParams), C.c_int, C.POINTER(vp)]),
    "tfhe_gpu_destroy": (None, [vp]),
    "tfhe_gpu_last_error": (C.c_char_p, [vp]),
    "tfhe_gpu_sync": (C.c_int, [vp]),
    "tfhe_gpu_set_stream": (C.c_int, [vp, vp]),
    "tfhe_gpu_reset_stream": (C.c_int, [vp]),
    "tfhe_gpu_create_multi": (C.c_int, [C.POINTER(TfheParams), C.c_int, C.POINTER(C.c_int), C.POINTER(vp)]),
    "tfhe_gpu_num_devices": (C.c_int, [vp]),
    "tfhe_gpu_device_bootstraps": (C.c_int, [vp, C.POINTER(C.c_uint64), C.c_int]),
    "tfhe_gpu_near_tie_items": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    "tfhe_gpu_set_option": (C.c_int, [vp, C.c_int, C.c_int64]),
    "tfhe_gpu_get_option": (C.c_int, [vp, C.c_int, C.POINTER(C.c_int64)]),
    "tfhe_gpu_last_kernels": (C.c_char_p, [vp]),
    "tfhe_fft_tables": (C.c_int, [C.c_uint32, C.c_int, f64p, f64p, f64p, f64p]),
    "tfhe_gpu_load_cloud_key": (C.c_int, [vp, C.c_uint32, u32p, u32p, f64p, C.c_size_t, u32p, C.c_size_t]),
    "tfhe_gpu_keygen": (C.c_int, [vp, C.c_uint64, C.c_uint64, u32p, u32p, f64p, u32p]),
    "tfhe_gpu_key_blob_bytes": (C.c_int, [vp, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]),
    "tfhe_gpu_key_fingerprint": (C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "tfhe_gpu_export_key_device": (C.c_int, [vp, vp, vp, u32p, u32p]),
    "tfhe_gpu_import_key_device": (C.c_int, [vp, vp, vp, C.c_uint32, u32p]),
    "tfhe_gpu_export_cloud_key": (C.c_int, [vp, C.POINTER(C.c_uint32), u32p, u32p, f64p, u32p]),
    "tfhe_cloud_key_write": (C.c_int, [C.c_char_p, C.POINTER(TfheParams), C.c_uint32, u32p, u32p, f64p, C.c_size_t,
                                       u32p, C.c_size_t]),
    "tfhe_cloud_key_read": (C.c_int, [C.c_char_p, C.POINTER(TfheParams), C.POINTER(C.c_uint32), u32p, u32p, f64p,
                                      C.c_size_t, u32p, C.c_size_t]),
    "tfhe_gpu_save_cloud_key": (C.c_int, [vp, C.c_char_p]),
    "tfhe_gpu_load_cloud_key_file": (C.c_int, [vp, C.c_char_p]),
    "tfhe_gpu_bootstrap_batch": (C.c_int, [vp, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_bootstrap_without_key_switch_batch": (C.c_int, [vp, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_gate_batch": (C.c_int, [vp, u8p, u32p, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_circuit_eval": (C.c_int, [vp, C.c_size_t, u32p, C.c_size_t, u8p, u32p, u32p, C.c_size_t, u32p, u32p,
                                        C.POINTER(C.c_uint32)]),
    "tfhe_gpu_circuit_eval_dev": (C.c_int, [vp, C.c_size_t, vp, C.c_size_t, u8p, u32p, u32p, C.c_size_t, u32p, vp,
                                        C.POINTER(C.c_uint32)]),
    "tfhe_circuit_schedule": (C.c_int, [C.c_size_t, C.c_size_t, u8p, u32p, u32p, C.c_uint32, C.c_int, u32p,
                                        C.POINTER(C.c_uint32)]),
    "tfhe_circuit_partition": (C.c_int, [C.c_size_t, C.c_size_t, u8p, u32p, u32p, C.c_int, u32p]),
    "tfhe_gpu_blind_rotate_batch": (C.c_int, [vp, u32p, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_bootstrap_lut_batch": (C.c_int, [vp, u32p, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_gate_batch_dev": (C.c_int, [vp, vp, vp, vp, vp, C.c_size_t]),
    "tfhe_gpu_bootstrap_batch_dev": (C.c_int, [vp, vp, vp, C.c_size_t]),
    "tfhe_gpu_profile_begin": (C.c_int, [vp]),
    "tfhe_gpu_profile_end": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "tfhe_gpu_fft_forward_batch": (C.c_int, [vp, u32p, f64p, C.c_size_t]),
    "tfhe_gpu_fft_inverse_batch": (C.c_int, [vp, f64p, u32p, C.c_size_t]),
    "tfhe_gpu_poly_mul_batch": (C.c_int, [vp, u32p, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_external_product_batch": (C.c_int, [vp, f64p, C.c_uint32, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_key_switch_batch": (C.c_int, [vp, u32p, u32p, C.c_size_t]),
    "tfhe_encrypt_bool_batch": (C.c_int, [C.POINTER(TfheParams), u32p, u8p, C.c_uint64, u32p, C.c_size_t]),
    "tfhe_decrypt_bool_batch": (C.c_int, [C.POINTER(TfheParams), u32p, u32p, u8p, C.c_size_t]),
    "tfhe_encrypt_lwe_message_batch": (C.c_int, [C.POINTER(TfheParams), u32p, u32p, C.c_uint32, C.c_uint64,
                                                 u32p, C.c_size_t]),
    "tfhe_decrypt_lwe_message_batch": (C.c_int, [C.POINTER(TfheParams), u32p, u32p, C.c_uint32, u32p,
                                                 C.c_size_t]),
    "tfhe_lut_generate": (C.c_int, [C.POINTER(TfheParams), C.c_uint32, u32p, u32p]),
    "tfhe_lut_generate_scaled": (C.c_int, [C.POINTER(TfheParams), C.c_uint32, C.c_double, u32p, u32p]),
    "tfhe_lut_generate_full": (C.c_int, [C.POINTER(TfheParams), C.c_uint32, u32p, u32p]),
    "tfhe_secret_key_new": (C.c_int, [C.POINTER(TfheParams), C.c_uint64, u32p, u32p]),
    "tfhe_gpu_reenc_key_load": (C.c_int, [vp, u32p, C.c_size_t, C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "tfhe_gpu_reenc_key_destroy": (None, [vp]),
    "tfhe_gpu_reencrypt_batch": (C.c_int, [vp, vp, u32p, u32p, C.c_size_t]),
    "tfhe_gpu_reencrypt_batch_dev": (C.c_int, [vp, vp, vp, vp, C.c_size_t]),
    "tfhe_gpu_bootstrap_lut_batch_dev": (C.c_int, [vp, vp, vp, vp, C.c_size_t]),
    "tfhe_public_key_gen": (C.c_int, [C.POINTER(TfheParams), u32p, C.c_size_t, C.c_double, C.c_uint64, u32p]),
    "tfhe_public_key_encrypt_bool_batch": (C.c_int, [C.POINTER(TfheParams), u32p, C.c_size_t, u8p, C.c_double,
                                                     C.c_uint64, u32p, C.c_size_t]),
    "tfhe_reenc_key_gen_symmetric": (C.c_int, [C.POINTER(TfheParams), u32p, u32p, C.c_double, C.c_uint32,
                                               C.c_uint32, C.c_uint64, u32p]),
    "tfhe_reenc_key_gen_asymmetric": (C.c_int, [C.POINTER(TfheParams), u32p, u32p, C.c_size_t, C.c_double,
                                                C.c_uint32, C.c_uint32, C.c_uint64, u32p]),
}
EXPORTED_SYMBOLS = tuple(_SIGS)


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Load the HIP library; raises (no fallback) if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libtfhe_gpu.so not built ({path}); run __graft_entry__.build() "
                           "or `make -C zig-tfhe_amd`")
    # If PyTorch is present, load its HIP runtime first: its libamdhip64 has
    # the same SONAME, so this library then binds to it and device pointers /
    # streams from torch are valid here (one runtime per process).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a, a.ctypes.data_as(u32p)


def _f64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(f64p)


def build_id() -> str:
    """tfhe_gpu_build_id: hash of the gfx950 kernels object the loaded library carries."""
    return load_library().tfhe_gpu_build_id().decode()


def build_kind() -> int:
    """tfhe_gpu_build_kind: BUILD_PRODUCT, or BUILD_AB for a development build
    (knock-out / timing / losing-form variants), which contexts refuse unless
    TFHE_ALLOW_AB_BUILD=1."""
    return load_library().tfhe_gpu_build_kind()


class TfheError(RuntimeError):
    """A nonzero C-ABI status; `status` is the TFHE_ERR_* code."""

    def __init__(self, msg: str, status: int = 0):
        super().__init__(msg)
        self.status = status


def fft_tables(N: int = 1024, source: int = TWIDDLES_GLIBC):
    """tfhe_fft_tables: (twist_re, twist_im, stage_re, stage_im) as the context builds them."""
    lib = load_library()
    t = [np.zeros(N // 2, np.float64), np.zeros(N // 2, np.float64), np.zeros(N // 2 - 1, np.float64),
         np.zeros(N // 2 - 1, np.float64)]
    rc = lib.tfhe_fft_tables(N, source, *[a.ctypes.data_as(f64p) for a in t])
    if rc != 0:
        raise TfheError(f"tfhe_fft_tables: status {rc}")
    return tuple(t)


class Context:
    """One HIP device + its resident CloudKey (tfhe_gpu_ctx), or with
    `devices` a multi-device context (tfhe_gpu_create_multi): batches are
    sharded over the devices, the key is broadcast once over RCCL."""

    def __init__(self, params="128", device: int = 0, devices=None):
        self.lib = load_library()
        self.params = make_params(params) if not isinstance(params, TfheParams) else params
        h = vp()
        if devices is None:
            rc = self.lib.tfhe_gpu_create_on_device(C.byref(self.params), device, C.byref(h))
            what = "tfhe_gpu_create_on_device"
        else:
            devs = (C.c_int * len(devices))(*devices)
            rc = self.lib.tfhe_gpu_create_multi(C.byref(self.params), len(devices), devs, C.byref(h))
            what = "tfhe_gpu_create_multi"
            device = devices[0]
        if rc != 0:  # tfhe_gpu_last_error(NULL): this thread's last failed create
            raise TfheError(f"{what} failed ({rc}): {self.lib.tfhe_gpu_last_error(None).decode()}", rc)
        self.h = h
        self.device = device

    @classmethod
    def multi(cls, params="128", num_devices: int = 1, devices=None):
        return cls(params, devices=list(devices) if devices is not None else list(range(num_devices)))

    @property
    def num_devices(self) -> int:
        return self.lib.tfhe_gpu_num_devices(self.h)

    def near_tie_items(self) -> int:
        """Items the margin guard recomputed in the reference's expression trees
        (tfhe_gpu_near_tie_items), as of the last synchronisation."""
        v = C.c_uint64()
        self.check(self.lib.tfhe_gpu_near_tie_items(self.h, C.byref(v)), "near_tie_items")
        return v.value

    def device_bootstraps(self) -> np.ndarray:
        """Blind rotations launched per device since creation (tfhe_gpu_device_bootstraps)."""
        n = self.num_devices
        out = np.zeros(n, np.uint64)
        rc = self.lib.tfhe_gpu_device_bootstraps(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        if rc < 0:
            self.check(rc, "device_bootstraps")
        return out

    def set_option(self, name: str, value: int):
        """tfhe_gpu_set_option (kernel forms, twiddle source; OPTIONS)."""
        if name == "br_form" and isinstance(value, str):
            value = int(value) if value.isdigit() else BR_FORMS[value]
        key = READONLY_OPTIONS[name] if name in READONLY_OPTIONS else OPTIONS[name]  # read-only: the library refuses
        self.check(self.lib.tfhe_gpu_set_option(self.h, key, int(value)), f"set_option({name})")

    def get_option(self, name: str) -> int:
        v = C.c_int64()
        key = READONLY_OPTIONS[name] if name in READONLY_OPTIONS else OPTIONS[name]
        self.check(self.lib.tfhe_gpu_get_option(self.h, key, C.byref(v)), f"get_option({name})")
        return v.value

    def reset_options(self):
        for k, v in OPTION_DEFAULTS.items():
            if self.get_option(k) != v:
                self.set_option(k, v)

    @contextlib.contextmanager
    def options(self, **kw):
        """Temporarily set options (A/B runs, tests).  On exit each option named
        in `kw` goes back to the value it had on entry (not to its default:
        a `twiddles` choice made before the block survives it)."""
        before = {k: self.get_option(k) for k in kw}
        try:
            for k, v in kw.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in before.items():
                if self.get_option(k) != v:
                    self.set_option(k, v)

    def last_kernels(self) -> str:
        """Kernel names of this context's last bootstrap launch (tfhe_gpu_last_kernels)."""
        return self.lib.tfhe_gpu_last_kernels(self.h).decode()

    def close(self):
        if getattr(self, "h", None):
            self.lib.tfhe_gpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, what: str):
        if rc != 0:
            raise TfheError(f"{what}: status {rc}: {self.lib.tfhe_gpu_last_error(self.h).decode()}", rc)

    @property
    def n1(self) -> int:
        return self.params.n + 1

    # ---- keys
    def load_cloud_key(self, offset, testvec, bk, ksk):
        tv, _ = _u32(testvec)
        bk, bkp = _f64(bk)
        ksk, kp = _u32(ksk)
        N = self.params.N
        self.check(self.lib.tfhe_gpu_load_cloud_key(self.h, offset, tv[:N].ctypes.data_as(u32p),
                                                    tv[N:].ctypes.data_as(u32p), bkp, bk.size, kp, ksk.size),
                   "load_cloud_key")

    def keygen(self, secret_seed: int, cloud_seed: int, want_host_copy: bool = False):
        p = self.params
        k0 = np.zeros(p.n, np.uint32)
        k1 = np.zeros(p.N, np.uint32)
        bk = ksk = None
        bkp = kp = None
        if want_host_copy:
            bk = np.zeros((p.n, 2 * p.L, 2, p.N), np.float64)
            ksk = np.zeros((p.N * p.iks_t * (1 << p.basebit), p.n + 1), np.uint32)
            bkp, kp = bk.ctypes.data_as(f64p), ksk.ctypes.data_as(u32p)
        self.check(self.lib.tfhe_gpu_keygen(self.h, secret_seed, cloud_seed, k0.ctypes.data_as(u32p),
                                            k1.ctypes.data_as(u32p), bkp, kp), "keygen")
        return SecretKey(p, k0, k1), (bk, ksk)

    def export_cloud_key(self):
        """The loaded CloudKey in the reference layout: (offset, testvec 2N, bk (n,2L,2,N) f64,
        ksk (N*t*2^basebit, n+1) u32; k = 0 rows zero)."""
        p = self.params
        off = C.c_uint32()
        tv = np.zeros(2 * p.N, np.uint32)
        bk = np.zeros((p.n, 2 * p.L, 2, p.N), np.float64)
        ksk = np.zeros((p.N * p.iks_t * (1 << p.basebit), p.n + 1), np.uint32)
        self.check(self.lib.tfhe_gpu_export_cloud_key(self.h, C.byref(off), tv[:p.N].ctypes.data_as(u32p),
                                                      tv[p.N:].ctypes.data_as(u32p), bk.ctypes.data_as(f64p),
                                                      ksk.ctypes.data_as(u32p)), "export_cloud_key")
        return off.value, tv, bk, ksk

    def save_cloud_key(self, path: str):
        """Key file (include/tfhe_gpu.h 'Cloud-key files'): the reference has no serialization."""
        self.check(self.lib.tfhe_gpu_save_cloud_key(self.h, os.fsencode(path)), "save_cloud_key")

    def load_cloud_key_file(self, path: str):
        self.check(self.lib.tfhe_gpu_load_cloud_key_file(self.h, os.fsencode(path)), "load_cloud_key_file")

    def key_blob_bytes(self):
        a, b = C.c_size_t(), C.c_size_t()
        self.check(self.lib.tfhe_gpu_key_blob_bytes(self.h, C.byref(a), C.byref(b)), "key_blob_bytes")
        return a.value, b.value

    def key_fingerprint(self):
        """tfhe_gpu_key_fingerprint: (bk, ksk) 64-bit sums of the resident device key."""
        a, b = C.c_uint64(), C.c_uint64()
        self.check(self.lib.tfhe_gpu_key_fingerprint(self.h, C.byref(a), C.byref(b)), "key_fingerprint")
        return a.value, b.value

    def export_key_device(self, bk_dev_ptr: int, ksk_dev_ptr: int):
        off = C.c_uint32()
        tv = np.zeros(2 * self.params.N, np.uint32)
        self.check(self.lib.tfhe_gpu_export_key_device(self.h, vp(bk_dev_ptr), vp(ksk_dev_ptr), C.byref(off),
                                                       tv.ctypes.data_as(u32p)), "export_key_device")
        return off.value, tv

    def import_key_device(self, bk_dev_ptr: int, ksk_dev_ptr: int, offset: int, testvec):
        tv, tvp = _u32(testvec)
        self.check(self.lib.tfhe_gpu_import_key_device(self.h, vp(bk_dev_ptr), vp(ksk_dev_ptr), offset, tvp),
                   "import_key_device")

    def set_stream(self, stream_ptr: int | None):
        """Run on a HIP stream handle (e.g. torch.cuda.current_stream().cuda_stream; 0 is the
        device's null stream, torch's default stream); None: back to the context's own stream."""
        if stream_ptr is None:
            self.check(self.lib.tfhe_gpu_reset_stream(self.h), "reset_stream")
        else:
            self.check(self.lib.tfhe_gpu_set_stream(self.h, vp(stream_ptr)), "set_stream")

    def sync(self):
        self.check(self.lib.tfhe_gpu_sync(self.h), "sync")

    def profile_begin(self):
        self.check(self.lib.tfhe_gpu_profile_begin(self.h), "profile_begin")

    def profile_end(self):
        """-> (blind_rotate_ms_total, key_switch_ms_total, launches), HIP events on the ctx stream."""
        br, ks, n = C.c_double(), C.c_double(), C.c_int()
        self.check(self.lib.tfhe_gpu_profile_end(self.h, C.byref(br), C.byref(ks), C.byref(n)), "profile_end")
        return br.value, ks.value, n.value

    # ---- batch bootstrap API
    def bootstrap_batch(self, cts):
        cts, cp = _u32(cts)
        out = np.zeros_like(cts)
        self.check(self.lib.tfhe_gpu_bootstrap_batch(self.h, cp, out.ctypes.data_as(u32p), cts.shape[0]),
                   "bootstrap_batch")
        return out

    def bootstrap_without_key_switch_batch(self, cts):
        """VanillaBootstrap.bootstrapWithoutKeySwitch (vanilla.zig:58-69): the
        reference's hybrid sampleExtractIndex2 form, n+1 words per item."""
        cts, cp = _u32(cts)
        out = np.zeros_like(cts)
        self.check(self.lib.tfhe_gpu_bootstrap_without_key_switch_batch(self.h, cp, out.ctypes.data_as(u32p),
                                                                        cts.shape[0]),
                   "bootstrap_without_key_switch_batch")
        return out

    def circuit_eval(self, inputs, ops, in_a, in_b, out_wires):
        """Level-scheduled gate DAG (tfhe_gpu_circuit_eval).  -> (outputs, bootstrap depth)."""
        inputs, ip = _u32(np.asarray(inputs, np.uint32).reshape(-1, self.params.n + 1))
        ops = np.ascontiguousarray(ops, np.uint8)
        in_a, ap = _u32(in_a)
        in_b, bp = _u32(in_b)
        out_wires, op_ = _u32(out_wires)
        out = np.zeros((out_wires.size, self.params.n + 1), np.uint32)
        lv = C.c_uint32()
        self.check(self.lib.tfhe_gpu_circuit_eval(self.h, inputs.shape[0], ip, ops.size, ops.ctypes.data_as(u8p), ap,
                                                  bp, out_wires.size, op_, out.ctypes.data_as(u32p), C.byref(lv)),
                   "circuit_eval")
        return out, lv.value

    def circuit_eval_dev(self, inputs_ptr, n_inputs, ops, in_a, in_b, out_wires, outputs_ptr):
        """tfhe_gpu_circuit_eval_dev: inputs / outputs in HBM (async on the context stream). -> depth."""
        ops = np.ascontiguousarray(ops, np.uint8)
        in_a, ap = _u32(in_a)
        in_b, bp = _u32(in_b)
        out_wires, op_ = _u32(out_wires)
        lv = C.c_uint32()
        self.check(self.lib.tfhe_gpu_circuit_eval_dev(self.h, n_inputs, vp(inputs_ptr), ops.size, ops.ctypes.data_as(u8p),
                                                      ap, bp, out_wires.size, op_, vp(outputs_ptr), C.byref(lv)),
                   "circuit_eval_dev")
        return lv.value

    def gate_batch(self, ops, a, b):
        ops = np.ascontiguousarray(ops, dtype=np.uint8)
        a, ap = _u32(a)
        b, bp = _u32(b)
        out = np.zeros_like(a)
        self.check(self.lib.tfhe_gpu_gate_batch(self.h, ops.ctypes.data_as(u8p), ap, bp,
                                                out.ctypes.data_as(u32p), ops.size), "gate_batch")
        return out

    def blind_rotate_batch(self, cts, testvec=None):
        cts, cp = _u32(cts)
        out = np.zeros((cts.shape[0], 2 * self.params.N), np.uint32)
        tvp = None
        if testvec is not None:
            tv, tvp = _u32(testvec)
        self.check(self.lib.tfhe_gpu_blind_rotate_batch(self.h, cp, tvp, out.ctypes.data_as(u32p),
                                                        cts.shape[0]), "blind_rotate_batch")
        return out

    def bootstrap_lut_batch(self, cts, testvec):
        cts, cp = _u32(cts)
        tv, tvp = _u32(testvec)
        out = np.zeros_like(cts)
        self.check(self.lib.tfhe_gpu_bootstrap_lut_batch(self.h, cp, tvp, out.ctypes.data_as(u32p),
                                                         cts.shape[0]), "bootstrap_lut_batch")
        return out

    def gate_batch_dev(self, ops_ptr, a_ptr, b_ptr, out_ptr, B):
        self.check(self.lib.tfhe_gpu_gate_batch_dev(self.h, vp(ops_ptr), vp(a_ptr), vp(b_ptr), vp(out_ptr), B),
                   "gate_batch_dev")

    def bootstrap_batch_dev(self, in_ptr, out_ptr, B):
        self.check(self.lib.tfhe_gpu_bootstrap_batch_dev(self.h, vp(in_ptr), vp(out_ptr), B), "bootstrap_batch_dev")

    def bootstrap_lut_batch_dev(self, in_ptr, tv_ptr, out_ptr, B):
        self.check(self.lib.tfhe_gpu_bootstrap_lut_batch_dev(self.h, vp(in_ptr), vp(tv_ptr), vp(out_ptr), B),
                   "bootstrap_lut_batch_dev")

    # ---- stage entry points
    def fft_forward(self, polys):
        x, xp = _u32(np.atleast_2d(polys))
        out = np.zeros(x.shape, np.float64)
        self.check(self.lib.tfhe_gpu_fft_forward_batch(self.h, xp, out.ctypes.data_as(f64p), x.shape[0]),
                   "fft_forward")
        return out

    def fft_inverse(self, freqs):
        f, fp = _f64(np.atleast_2d(freqs))
        out = np.zeros(f.shape, np.uint32)
        self.check(self.lib.tfhe_gpu_fft_inverse_batch(self.h, fp, out.ctypes.data_as(u32p), f.shape[0]),
                   "fft_inverse")
        return out

    def poly_mul(self, a, b):
        a, ap = _u32(np.atleast_2d(a))
        b, bp = _u32(np.atleast_2d(b))
        out = np.zeros(a.shape, np.uint32)
        self.check(self.lib.tfhe_gpu_poly_mul_batch(self.h, ap, bp, out.ctypes.data_as(u32p), a.shape[0]),
                   "poly_mul")
        return out

    def external_product(self, trlwes, trgsw_fft=None, bk_index=0):
        x, xp = _u32(np.atleast_2d(trlwes))
        out = np.zeros(x.shape, np.uint32)
        tp = None
        if trgsw_fft is not None:
            tg, tp = _f64(trgsw_fft)
        self.check(self.lib.tfhe_gpu_external_product_batch(self.h, tp, bk_index, xp, out.ctypes.data_as(u32p),
                                                            x.shape[0]), "external_product")
        return out

    def key_switch(self, lv1):
        x, xp = _u32(np.atleast_2d(lv1))
        out = np.zeros((x.shape[0], self.n1), np.uint32)
        self.check(self.lib.tfhe_gpu_key_switch_batch(self.h, xp, out.ctypes.data_as(u32p), x.shape[0]),
                   "key_switch")
        return out


@dataclass
class SecretKey:
    """key.SecretKey (key.zig:34-58): binary lv0 / lv1 keys."""
    params: TfheParams
    key_lv0: np.ndarray
    key_lv1: np.ndarray

    def encrypt_bool(self, bits, seed0: int = 1):
        """TLWELv0.encryptBool per bit, DefaultPrng(seed0 + i) in place of getUniqueSeed()."""
        lib = load_library()
        bits = np.ascontiguousarray(np.atleast_1d(bits), dtype=np.uint8)
        out = np.zeros((bits.size, self.params.n + 1), np.uint32)
        rc = lib.tfhe_encrypt_bool_batch(C.byref(self.params), _u32(self.key_lv0)[1], bits.ctypes.data_as(u8p),
                                         seed0, out.ctypes.data_as(u32p), bits.size)
        if rc:
            raise TfheError(f"encrypt_bool: {rc}")
        return out

    def decrypt_bool(self, cts):
        lib = load_library()
        cts, cp = _u32(np.atleast_2d(cts))
        out = np.zeros(cts.shape[0], np.uint8)
        rc = lib.tfhe_decrypt_bool_batch(C.byref(self.params), _u32(self.key_lv0)[1], cp,
                                         out.ctypes.data_as(u8p), cts.shape[0])
        if rc:
            raise TfheError(f"decrypt_bool: {rc}")
        return out.astype(bool)

    def encrypt_lwe_message(self, msgs, m: int, seed0: int = 1):
        lib = load_library()
        msgs, mp = _u32(np.atleast_1d(msgs))
        out = np.zeros((msgs.size, self.params.n + 1), np.uint32)
        rc = lib.tfhe_encrypt_lwe_message_batch(C.byref(self.params), _u32(self.key_lv0)[1], mp, m, seed0,
                                                out.ctypes.data_as(u32p), msgs.size)
        if rc:
            raise TfheError(f"encrypt_lwe_message: {rc}")
        return out

    def decrypt_lwe_message(self, cts, m: int):
        lib = load_library()
        cts, cp = _u32(np.atleast_2d(cts))
        out = np.zeros(cts.shape[0], np.uint32)
        rc = lib.tfhe_decrypt_lwe_message_batch(C.byref(self.params), _u32(self.key_lv0)[1], cp, m,
                                                out.ctypes.data_as(u32p), cts.shape[0])
        if rc:
            raise TfheError(f"decrypt_lwe_message: {rc}")
        return out


def secret_key_new(params: TfheParams, seed: int) -> SecretKey:
    """key.SecretKey.new (key.zig:41-57) with DefaultPrng(seed) in place of getUniqueSeed()."""
    lib = load_library()
    k0, k1 = np.zeros(params.n, np.uint32), np.zeros(params.N, np.uint32)
    rc = lib.tfhe_secret_key_new(C.byref(params), seed, k0.ctypes.data_as(u32p), k1.ctypes.data_as(u32p))
    if rc:
        raise TfheError(f"secret_key_new: {rc}")
    return SecretKey(params, k0, k1)


class PublicKeyLv0:
    """proxy_reenc.PublicKeyLv0 (proxy_reenc.zig:35-121): `size` encryptions of zero under key_lv0.
    Encryption e uses DefaultPrng(seed0 + e); size defaults to 2n (:44-54)."""

    def __init__(self, sk: SecretKey, seed0: int, size: int | None = None, alpha: float | None = None):
        p = self.params = sk.params
        size = 2 * p.n if size is None else size
        alpha = p.alpha_lv0 if alpha is None else alpha
        self.encryptions = np.zeros((size, p.n + 1), np.uint32)
        rc = load_library().tfhe_public_key_gen(C.byref(p), _u32(sk.key_lv0)[1], size, alpha, seed0,
                                                self.encryptions.ctypes.data_as(u32p))
        if rc:
            raise TfheError(f"public_key_gen: {rc}")

    def encrypt_bool(self, bits, seed0: int = 1, alpha: float | None = None):
        """encryptBool (:116-120); item i uses DefaultPrng(seed0 + i)."""
        p = self.params
        alpha = p.alpha_lv0 if alpha is None else alpha
        bits = np.ascontiguousarray(np.atleast_1d(bits), dtype=np.uint8)
        out = np.zeros((bits.size, p.n + 1), np.uint32)
        rc = load_library().tfhe_public_key_encrypt_bool_batch(
            C.byref(p), self.encryptions.ctypes.data_as(u32p), self.encryptions.shape[0],
            bits.ctypes.data_as(u8p), alpha, seed0, out.ctypes.data_as(u32p), bits.size)
        if rc:
            raise TfheError(f"public_key_encrypt_bool: {rc}")
        return out


class ProxyReencryptionKey:
    """proxy_reenc.ProxyReencryptionKey (proxy_reenc.zig:124-257): key_encryptions[(base*t*i)+(base*j)+k]
    = Enc_to(k * key_from[i] / 2^((j+1)*basebit)), k = 0 entries zero. Defaults: KSK_ALPHA and the
    parameter set's BASEBIT / IKS_T (:131-147). The c-th encryption uses DefaultPrng(seed0 + c)."""

    def __init__(self, key_encryptions: np.ndarray, basebit: int, t: int):
        self.key_encryptions, self.basebit, self.t = key_encryptions, basebit, t
        self.base = 1 << basebit

    @classmethod
    def _gen(cls, params, fn, extra, key_from, alpha, basebit, t, seed0):
        alpha = params.alpha_ksk if alpha is None else alpha
        basebit = params.basebit if basebit is None else basebit
        t = params.iks_t if t is None else t
        out = np.zeros(((1 << basebit) * t * params.n, params.n + 1), np.uint32)
        rc = fn(C.byref(params), _u32(key_from)[1], *extra, alpha, basebit, t, seed0, out.ctypes.data_as(u32p))
        if rc:
            raise TfheError(f"reenc_key_gen: {rc}")
        return cls(out, basebit, t)

    @classmethod
    def new_symmetric(cls, key_from: SecretKey, key_to: SecretKey, seed0: int, alpha=None, basebit=None, t=None):
        """newSymmetricWithParams (:214-256)."""
        return cls._gen(key_from.params, load_library().tfhe_reenc_key_gen_symmetric, [_u32(key_to.key_lv0)[1]],
                        key_from.key_lv0, alpha, basebit, t, seed0)

    @classmethod
    def new_asymmetric(cls, key_from: SecretKey, pk_to: PublicKeyLv0, seed0: int, alpha=None, basebit=None,
                       t=None):
        """newAsymmetricWithParams (:150-196)."""
        pk = pk_to.encryptions
        return cls._gen(key_from.params, load_library().tfhe_reenc_key_gen_asymmetric,
                        [pk.ctypes.data_as(u32p), pk.shape[0]], key_from.key_lv0, alpha, basebit, t, seed0)


class HipReencryptor:
    """reencryptTLWELv0 (proxy_reenc.zig:267-306) for a batch of TLWELv0, on the GPU: the re-encryption
    key lives in HBM (padded rows, like the KSK) and each ciphertext is one lane of the key-switch kernel."""

    def __init__(self, ctx: Context, key: ProxyReencryptionKey):
        self.ctx, self.h = ctx, vp()
        ke, kp = _u32(key.key_encryptions)
        ctx.check(ctx.lib.tfhe_gpu_reenc_key_load(ctx.h, kp, ke.size, key.basebit, key.t, C.byref(self.h)),
                  "reenc_key_load")

    def close(self):
        if self.h:
            self.ctx.lib.tfhe_gpu_reenc_key_destroy(self.h)
            self.h = vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reencrypt(self, cts):
        x, xp = _u32(np.atleast_2d(cts))
        out = np.zeros_like(x)
        self.ctx.check(self.ctx.lib.tfhe_gpu_reencrypt_batch(self.ctx.h, self.h, xp, out.ctypes.data_as(u32p),
                                                             x.shape[0]), "reencrypt")
        return out

    def reencrypt_dev(self, in_ptr, out_ptr, B):
        """Device-resident batch (async on the context stream): B TLWELv0 at in_ptr -> out_ptr."""
        self.ctx.check(self.ctx.lib.tfhe_gpu_reencrypt_batch_dev(self.ctx.h, self.h, vp(in_ptr), vp(out_ptr), B),
                       "reencrypt_dev")


class bit_utils:
    """bit_utils.zig (host-side plaintext plumbing of the examples): `convert` (:9-16) packs
    bits LSB first into an unsigned integer; `AsBits(T).toBits` (:24-27, :42-50) unpacks the
    width of T; `AsBits(T).encrypt` (:29-39) encrypts every bit (DefaultPrng(seed0 + i) per bit
    in place of getUniqueSeed())."""

    @staticmethod
    def convert(bits, width: int | None = None) -> int:
        bits = list(bits)
        width = len(bits) if width is None else width
        v = 0
        for i, b in enumerate(bits[:width]):
            v |= (1 if b else 0) << i
        return v

    @staticmethod
    def to_bits(value: int, width: int) -> np.ndarray:
        return np.array([(int(value) >> i) & 1 for i in range(width)], dtype=bool)

    @staticmethod
    def encrypt(value: int, width: int, sk: SecretKey, seed0: int = 1) -> np.ndarray:
        return sk.encrypt_bool(bit_utils.to_bits(value, width).astype(np.uint8), seed0=seed0)


def lut_generate(params: TfheParams, m: int, f) -> np.ndarray:
    """Generator.generateLookupTable (lut/generator.zig:85-135) for f: x -> f(x), x < m."""
    lib = load_library()
    table = np.array([f(x) for x in range(m)], dtype=np.uint32)
    tv = np.zeros(2 * params.N, np.uint32)
    rc = lib.tfhe_lut_generate(C.byref(params), m, table.ctypes.data_as(u32p), tv.ctypes.data_as(u32p))
    if rc:
        raise TfheError(f"lut_generate: {rc}")
    return tv


class Encoder:
    """lut/encoder.zig Encoder: message x -> f64ToTorus((x mod m) * scale);
    new(m) uses scale 1/(2m) (encoder.zig:29-42), with_scale a custom one (:49-54)."""

    def __init__(self, message_modulus: int, scale: float | None = None):
        self.message_modulus = int(message_modulus)
        self.scale = 1.0 / (2.0 * float(message_modulus)) if scale is None else float(scale)

    @classmethod
    def new(cls, message_modulus: int) -> "Encoder":
        return cls(message_modulus)

    @classmethod
    def with_scale(cls, message_modulus: int, scale: float) -> "Encoder":
        return cls(message_modulus, scale)


class LookupTable:
    """lut/lookup_table.zig LookupTable: a TRLWELv1 (a ++ b, 2N words) that the
    blind rotation uses as its test vector (tfhe_gpu_bootstrap_lut_batch)."""

    def __init__(self, poly=None, N: int = 1024):
        self.poly = np.zeros(2 * N, np.uint32) if poly is None else np.array(poly, np.uint32).reshape(-1)
        if self.poly.size != 2 * int(N):
            raise ValueError(f"LookupTable: a TRLWELv1 has 2N = {2 * int(N)} words (a ++ b), got {self.poly.size}")

    @classmethod
    def new(cls, N: int = 1024) -> "LookupTable":  # :23-27
        return cls(N=N)

    @classmethod
    def from_poly(cls, poly, N: int = 1024) -> "LookupTable":  # :33-35 (a copy of the TRLWELv1's words)
        return cls(poly, N)

    @property
    def a(self):
        return self.poly[: self.poly.size // 2]

    @property
    def b(self):
        return self.poly[self.poly.size // 2:]

    def get_poly(self) -> np.ndarray:  # :38-45
        return self.poly

    def copy_from(self, other: "LookupTable"):  # :51-54
        self.poly[:] = other.poly

    def clear(self):  # :57-61
        self.poly[:] = 0

    def is_empty(self) -> bool:  # :64-77
        return not self.poly.any()


class Generator:
    """lut/generator.zig Generator over the C ABI's table generation
    (tfhe_lut_generate_scaled / _full): poly_degree = lookup_table_size = N
    (the reference's poly_extend_factor 1)."""

    def __init__(self, encoder: Encoder, params: TfheParams | None = None):
        self.encoder = encoder
        self.params = params if params is not None else make_params("128")
        self.poly_degree_ = self.lookup_table_size_ = int(self.params.N)

    @classmethod
    def new(cls, message_modulus: int, params: TfheParams | None = None) -> "Generator":  # :29-41
        return cls(Encoder.new(message_modulus), params)

    @classmethod
    def with_scale(cls, message_modulus: int, scale: float, params: TfheParams | None = None) -> "Generator":  # :47-56
        return cls(Encoder.with_scale(message_modulus, scale), params)

    def message_modulus(self) -> int:  # :230-232
        return self.encoder.message_modulus

    def poly_degree(self) -> int:  # :235-237
        return self.poly_degree_

    def lookup_table_size(self) -> int:  # :240-242
        return self.lookup_table_size_

    def _check_lut(self, lut: LookupTable):
        """The C side writes 2N words into lut.poly: refuse anything else before the call."""
        p = lut.poly
        if not (isinstance(p, np.ndarray) and p.dtype == np.uint32 and p.flags.c_contiguous
                and p.size == 2 * int(self.params.N)):
            raise ValueError(f"LookupTable.poly must be a C-contiguous uint32 array of 2N = {2 * int(self.params.N)} "
                             f"words for these params, got {getattr(p, 'dtype', type(p))} of size {getattr(p, 'size', '?')}")

    def generate_lookup_table_assign(self, f, lut: LookupTable):  # :85-135
        self._check_lut(lut)
        m = self.encoder.message_modulus
        # Encoder.encode reduces f(x) (a usize) mod m in 64 bits (encoder.zig:66-74): reduce in
        # Python first, so f(x) >= 2^32 neither overflows the uint32 table nor wraps before the mod
        table = np.array([int(f(x)) % m for x in range(m)], dtype=np.uint32)
        rc = load_library().tfhe_lut_generate_scaled(C.byref(self.params), m, self.encoder.scale,
                                                     table.ctypes.data_as(u32p), lut.poly.ctypes.data_as(u32p))
        if rc:
            raise TfheError(f"lut_generate_scaled: {rc}", rc)

    def generate_lookup_table(self, f) -> LookupTable:  # :65-69
        lut = LookupTable.new(self.params.N)
        self.generate_lookup_table_assign(f, lut)
        return lut

    def generate_lookup_table_full_assign(self, f, lut: LookupTable):  # :155-191: f(x) is a Torus value
        self._check_lut(lut)
        m = self.encoder.message_modulus
        vals = np.array([int(f(x)) & 0xFFFFFFFF for x in range(m)], dtype=np.uint32)
        rc = load_library().tfhe_lut_generate_full(C.byref(self.params), m, vals.ctypes.data_as(u32p),
                                                   lut.poly.ctypes.data_as(u32p))
        if rc:
            raise TfheError(f"lut_generate_full: {rc}", rc)

    def generate_lookup_table_full(self, f) -> LookupTable:  # :144-148
        lut = LookupTable.new(self.params.N)
        self.generate_lookup_table_full_assign(f, lut)
        return lut

    def generate_lookup_table_custom(self, f, message_modulus: int, scale: float) -> LookupTable:  # :202-213
        return Generator(Encoder.with_scale(message_modulus, scale), self.params).generate_lookup_table(f)

    def mod_switch(self, x: int) -> int:  # :223-227, the reference's f64 expression
        scaled = (float(int(x) & 0xFFFFFFFF) / 4294967295.0) * float(self.lookup_table_size_)
        return int(scaled + 0.5) % self.lookup_table_size_


def cloud_key_write(path: str, params: TfheParams, offset: int, testvec, bk, ksk):
    """Write a CloudKey (reference layout) as a key file; host only (tfhe_cloud_key_write)."""
    lib = load_library()
    tv, _ = _u32(testvec)
    bk, bkp = _f64(bk)
    ksk, kp = _u32(ksk)
    N = params.N
    rc = lib.tfhe_cloud_key_write(os.fsencode(path), C.byref(params), offset, tv[:N].ctypes.data_as(u32p),
                                  tv[N:].ctypes.data_as(u32p), bkp, bk.size, kp, ksk.size)
    if rc:
        raise TfheError(f"cloud_key_write: status {rc}")


def cloud_key_read(path: str, params: TfheParams):
    """-> (offset, testvec 2N, bk (n,2L,2,N), ksk (N*t*2^basebit, n+1)); raises TfheError
    (status -5: I/O, -1: not a key file of this parameter set or checksum mismatch)."""
    lib = load_library()
    p = params
    off = C.c_uint32()
    tv = np.zeros(2 * p.N, np.uint32)
    bk = np.zeros((p.n, 2 * p.L, 2, p.N), np.float64)
    ksk = np.zeros((p.N * p.iks_t * (1 << p.basebit), p.n + 1), np.uint32)
    rc = lib.tfhe_cloud_key_read(os.fsencode(path), C.byref(p), C.byref(off), tv[:p.N].ctypes.data_as(u32p),
                                 tv[p.N:].ctypes.data_as(u32p), bk.ctypes.data_as(f64p), bk.size,
                                 ksk.ctypes.data_as(u32p), ksk.size)
    if rc:
        raise TfheError(f"cloud_key_read: status {rc}")
    return off.value, tv, bk, ksk


class HipBootstrap:
    """The bootstrap strategy object (bootstrap.zig:30-47, vanilla.zig:24-76)
    on the MI355X: bootstrap / bootstrap_without_key_switch / name, each over a
    single TLWELv0 (n+1,) or a batch (B, n+1).  The cloud key is the one the
    Context holds (the reference passes it per call)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    @staticmethod
    def _run(fn, ct):
        ct = np.asarray(ct, np.uint32)
        out = fn(np.atleast_2d(ct))
        return out[0] if ct.ndim == 1 else out

    def bootstrap(self, ct):  # vanilla.zig:38-52
        return self._run(self.ctx.bootstrap_batch, ct)

    def bootstrap_without_key_switch(self, ct):  # vanilla.zig:58-69
        return self._run(self.ctx.bootstrap_without_key_switch_batch, ct)

    def name(self) -> str:  # vanilla.zig:72-75
        return "mi355x"


class Gates:
    """gates.Gates (gates.zig:25-152) on the MI355X bootstrap strategy.

    Each *_gate accepts single ciphertexts (n+1,) or batches (B, n+1); NOT /
    COPY / CONSTANT need no bootstrap and stay on the host like the reference.
    """

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def bootstrap_strategy(self) -> str:  # gates.zig:43-45
        return "mi355x"

    def _gate(self, op, a, b):
        a = np.atleast_2d(np.asarray(a, np.uint32))
        b = np.atleast_2d(np.asarray(b, np.uint32))
        single = np.asarray(a).ndim == 2 and a.shape[0] == 1
        out = self.ctx.gate_batch(np.full(a.shape[0], op, np.uint8), a, b)
        return out[0] if single else out

    def nand_gate(self, a, b): return self._gate(NAND, a, b)
    def or_gate(self, a, b): return self._gate(OR, a, b)
    def and_gate(self, a, b): return self._gate(AND, a, b)
    def xor_gate(self, a, b): return self._gate(XOR, a, b)
    def xnor_gate(self, a, b): return self._gate(XNOR, a, b)
    def nor_gate(self, a, b): return self._gate(NOR, a, b)
    def and_ny_gate(self, a, b): return self._gate(ANDNY, a, b)
    def and_yn_gate(self, a, b): return self._gate(ANDYN, a, b)
    def or_ny_gate(self, a, b): return self._gate(ORNY, a, b)
    def or_yn_gate(self, a, b): return self._gate(ORYN, a, b)

    def mux_naive(self, a, b, c):
        """muxNaive (gates.zig:124-129): AND(a,b) || AND(NOT a, c), then OR — 2 levels."""
        a = np.atleast_2d(np.asarray(a, np.uint32))
        b = np.atleast_2d(np.asarray(b, np.uint32))
        c = np.atleast_2d(np.asarray(c, np.uint32))
        B = a.shape[0]
        lvl1 = self.ctx.gate_batch(np.full(2 * B, AND, np.uint8), np.concatenate([a, self.not_gate(a)]),
                                   np.concatenate([b, c]))
        return self.ctx.gate_batch(np.full(B, OR, np.uint8), lvl1[:B], lvl1[B:])

    @staticmethod
    def not_gate(a):  # gates.zig:132-135 (TLWELv0.neg)
        return (np.uint32(0) - np.asarray(a, np.uint32)).astype(np.uint32)

    @staticmethod
    def copy(a):  # gates.zig:138-141
        return np.array(a, np.uint32, copy=True)

    def constant(self, value: bool):  # gates.zig:144-151
        res = np.zeros(self.ctx.n1, np.uint32)
        mu = 0x20000000  # f64ToTorus(0.125)
        res[-1] = mu if value else (1 - mu) & 0xFFFFFFFF
        return res


class Circuit:
    """Gate DAG builder for Context.circuit_eval: the
    reference's circuits are sequences of Gates calls (gates.zig:48-151,
    examples/add_two_numbers.zig:24-73); here they are recorded as wires and
    evaluated level by level, one batched bootstrap launch per level.

        c = Circuit(); a, b = c.input(), c.input(); s = c.xor(a, b); c.output(s)
        outs, depth = c.run(ctx, [ct_a, ct_b])
    """

    def __init__(self):
        self.n_inputs = 0
        self.ops, self.ia, self.ib = [], [], []
        self.outputs = []

    def input(self) -> int:
        if self.ops:
            raise ValueError("declare every input before the first gate")
        self.n_inputs += 1
        return self.n_inputs - 1

    def gate(self, op: int, a: int, b: int | None = None) -> int:
        w = self.n_inputs + len(self.ops)
        if not (0 <= a < w) or (b is not None and not (0 <= b < w)):
            raise ValueError("gate inputs must be existing wires")
        self.ops.append(op)
        self.ia.append(a)
        self.ib.append(a if b is None else b)
        return w

    # gates.zig:48-151
    def nand(self, a, b): return self.gate(NAND, a, b)
    def or_(self, a, b): return self.gate(OR, a, b)
    def and_(self, a, b): return self.gate(AND, a, b)
    def xor(self, a, b): return self.gate(XOR, a, b)
    def xnor(self, a, b): return self.gate(XNOR, a, b)
    def nor(self, a, b): return self.gate(NOR, a, b)
    def and_ny(self, a, b): return self.gate(ANDNY, a, b)
    def and_yn(self, a, b): return self.gate(ANDYN, a, b)
    def or_ny(self, a, b): return self.gate(ORNY, a, b)
    def or_yn(self, a, b): return self.gate(ORYN, a, b)
    def not_(self, a): return self.gate(NOT, a)
    def copy(self, a): return self.gate(COPY, a)

    def mux(self, a, b, c):
        """muxNaive (gates.zig:124-129): OR(AND(a, b), AND(NOT a, c)) — 2 bootstrap levels."""
        return self.or_(self.and_(a, b), self.and_(self.not_(a), c))

    def full_adder(self, a, b, cin):
        """examples/add_two_numbers.zig:24-47: (sum, carry)."""
        x = self.xor(a, b)
        ab = self.and_(a, b)
        xc = self.and_(x, cin)
        return self.xor(x, cin), self.or_(ab, xc)

    def ripple_add(self, a_bits, b_bits, cin):
        """examples/add_two_numbers.zig:50-73: LSB-first bit wires -> (sum wires, carry)."""
        out, carry = [], cin
        for a, b in zip(a_bits, b_bits):
            s, carry = self.full_adder(a, b, carry)
            out.append(s)
        return out, carry

    def output(self, *wires):
        self.outputs.extend(wires)

    def schedule(self, cus: int = 256, pack: bool = True):
        """The level of every gate as tfhe_gpu_circuit_eval runs it on a device
        with `cus` CUs (host only, tfhe_circuit_schedule) -> (levels, depth)."""
        lib = load_library()
        ops = np.array(self.ops, np.uint8)
        ia, iap = _u32(np.array(self.ia, np.uint32))
        ib, ibp = _u32(np.array(self.ib, np.uint32))
        levels = np.zeros(max(len(self.ops), 1), np.uint32)
        depth = C.c_uint32(0)
        rc = lib.tfhe_circuit_schedule(self.n_inputs, ops.size, ops.ctypes.data_as(u8p), iap, ibp, cus, int(pack),
                                       levels.ctypes.data_as(u32p), C.byref(depth))
        if rc:
            raise TfheError(f"circuit_schedule: status {rc}")
        return levels[:ops.size], depth.value

    def partition(self, num_devices: int):
        """The device of every gate a multi-device context's circuit_eval uses
        (host only, tfhe_circuit_partition)."""
        lib = load_library()
        ops = np.array(self.ops, np.uint8)
        ia, iap = _u32(np.array(self.ia, np.uint32))
        ib, ibp = _u32(np.array(self.ib, np.uint32))
        dev = np.zeros(max(len(self.ops), 1), np.uint32)
        rc = lib.tfhe_circuit_partition(self.n_inputs, ops.size, ops.ctypes.data_as(u8p), iap, ibp, num_devices,
                                        dev.ctypes.data_as(u32p))
        if rc:
            raise TfheError(f"circuit_partition: status {rc}")
        return dev[:ops.size]

    def run(self, ctx: "Context", inputs):
        inputs = np.asarray(inputs, np.uint32).reshape(-1, ctx.params.n + 1)
        if inputs.shape[0] != self.n_inputs:
            raise ValueError(f"circuit has {self.n_inputs} inputs, got {inputs.shape[0]}")
        return ctx.circuit_eval(inputs, np.array(self.ops, np.uint8), np.array(self.ia, np.uint32),
                                np.array(self.ib, np.uint32), np.array(self.outputs, np.uint32))

    def run_dev(self, ctx: "Context", inputs_ptr, outputs_ptr):
        """Inputs (n_inputs TLWELv0) and outputs in HBM; returns the bootstrap depth."""
        return ctx.circuit_eval_dev(inputs_ptr, self.n_inputs, np.array(self.ops, np.uint8),
                                    np.array(self.ia, np.uint32), np.array(self.ib, np.uint32),
                                    np.array(self.outputs, np.uint32), outputs_ptr)
