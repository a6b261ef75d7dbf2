"""The programmable-bootstrap table generator: the reference's
own known answers of src/lut/ restated on the product's host mirror
(tfhe_amd.Generator / LookupTable over tfhe_lut_generate*) and on the oracle,
and the product's tables bit-identical to the oracle's over message moduli
that hit divRound's rounding and the m > N edge.  Host only: no kernel runs."""
import numpy as np
import pytest

import tfhe_amd
from conftest import rng

N = 1024
MAX_U32 = 0xFFFFFFFF


# ---- lut/generator.zig tests (:259-356) --------------------------------------
def test_div_round_known_answers(oracle):  # generator.zig:350-356
    assert [oracle.div_round(a, 2) for a in (5, 4, 3, 1, 0)] == [3, 2, 2, 1, 0]


def test_generator_creation():  # generator.zig:259-264
    g = tfhe_amd.Generator.new(2)
    assert g.message_modulus() == 2
    assert g.poly_degree() == N
    assert g.lookup_table_size() == N


@pytest.mark.parametrize("m,f", [(2, lambda x: x), (2, lambda x: 1 - x), (2, lambda x: 1),
                                 (4, lambda x: (x + 1) % 4)])
def test_functions_give_nonempty_tables(oracle, m, f):  # generator.zig:266-321 (identity, not, constant, 4bit)
    lut = tfhe_amd.Generator.new(m).generate_lookup_table(f)
    assert not lut.is_empty()
    assert np.array_equal(lut.poly, oracle.lut_generate(N, m, np.array([f(x) for x in range(m)], np.uint32)))


def test_custom_scale(oracle):  # generator.zig:323-335
    lut = tfhe_amd.Generator.with_scale(2, 0.5).generate_lookup_table(lambda x: x)
    assert not lut.is_empty()
    assert np.array_equal(lut.poly, oracle.lut_generate_scaled(N, 2, 0.5, np.array([0, 1], np.uint32)))


def test_mod_switch(oracle):  # generator.zig:337-348, and the values themselves against the oracle
    g = tfhe_amd.Generator.new(2)
    for x in (0, MAX_U32 // 2, MAX_U32):
        assert g.mod_switch(x) < g.lookup_table_size()
    assert [g.mod_switch(x) for x in (0, MAX_U32 // 2, MAX_U32)] == [0, 512, 0]
    xs = rng(60).integers(0, 1 << 32, 2000, dtype=np.uint64)
    xs = np.concatenate([xs, [1, 2, 2 ** 21, 2 ** 22 - 1, 2 ** 22, 2 ** 31, 2 ** 32 - 2 ** 21]])
    assert [g.mod_switch(int(x)) for x in xs] == [oracle.lut_mod_switch(int(x), N) for x in xs]


# ---- lut/lookup_table.zig tests (:81-128) ------------------------------------
def test_lookup_table_creation():  # :81-84
    assert tfhe_amd.LookupTable.new().is_empty()


def test_lookup_table_from_poly():  # :86-92
    poly = np.zeros(2 * N, np.uint32)
    poly[N + 0] = 1  # poly.b[0]
    assert not tfhe_amd.LookupTable.from_poly(poly).is_empty()


def test_lookup_table_copy():  # :94-107
    lut1, lut2 = tfhe_amd.LookupTable.new(), tfhe_amd.LookupTable.new()
    lut1.b[0], lut1.b[1] = 42, 24
    lut2.copy_from(lut1)
    assert (int(lut2.b[0]), int(lut2.b[1])) == (42, 24)
    assert np.array_equal(lut2.poly, lut1.poly)


def test_lookup_table_clear():  # :109-120
    lut = tfhe_amd.LookupTable.new()
    lut.b[0], lut.b[1] = 42, 24
    assert not lut.is_empty()
    lut.clear()
    assert lut.is_empty()


def test_lookup_table_conversions():  # :122-128
    poly = np.zeros(2 * N, np.uint32)
    poly[N + 0] = 123
    assert int(tfhe_amd.LookupTable.from_poly(poly).b[0]) == 123


# ---- the product's tables against the oracle's ---------------------------------
@pytest.mark.parametrize("m", [1, 2, 3, 4, 5, 7, 16, 100, 683, 1023, 1024, 2048, 3000])
def test_tables_equal_the_oracle(oracle, m):
    """Every message modulus from 1 to past N (divRound ties at m = 2048, empty
    ranges and a zero rotation past N): default encoding, a custom scale and
    full Torus values, word for word."""
    g = rng(61 + m)
    f = g.integers(0, 1 << 20, m).astype(np.uint32)
    gen = tfhe_amd.Generator.new(m)
    assert np.array_equal(gen.generate_lookup_table(lambda x: int(f[x])).poly, oracle.lut_generate(N, m, f))
    assert np.array_equal(gen.generate_lookup_table_custom(lambda x: int(f[x]), m, 0.3).poly,
                          oracle.lut_generate_scaled(N, m, 0.3, f))
    vals = g.integers(0, 1 << 32, m, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(gen.generate_lookup_table_full(lambda x: int(vals[x])).poly,
                          oracle.lut_generate_full(N, m, vals))
    # the function-style entry used by the bootstrap tests is the same table
    assert np.array_equal(tfhe_amd.lut_generate(tfhe_amd.make_params("uint4"), m, lambda x: int(f[x])),
                          oracle.lut_generate(N, m, f))


def test_table_ranges_follow_div_round(oracle):
    """m = 2048 over N = 1024: message x's range is [divRound(1024x, 2048),
    divRound(1024(x+1), 2048)) = [floor((x+1)/2), floor((x+2)/2)), i.e. even x
    own one slot and odd x none (x/2 ties round up), and the rotation
    divRound(1024, 4096) is 0: no entry is negated."""
    m = 2048
    vals = np.arange(1, m + 1, dtype=np.uint32)  # value x + 1 for message x: nonzero, distinct
    tv = tfhe_amd.Generator.new(m).generate_lookup_table_full(lambda x: int(vals[x])).b
    assert oracle.div_round(1024, 2 * m) == 0
    owner = [x for x in range(m) if oracle.div_round(x * N, m) < oracle.div_round((x + 1) * N, m)]
    assert owner == list(range(0, m, 2))
    assert np.array_equal(tv, vals[owner])


# ---- argument checks at the boundary --------------------------------
def test_short_table_is_refused_before_the_c_call():
    """The C side writes 2N words: a LookupTable of any other size never reaches it."""
    with pytest.raises(ValueError):
        tfhe_amd.LookupTable.from_poly(np.zeros(16, np.uint32))
    small = tfhe_amd.LookupTable.new(N=8)  # a valid 16-word table, but the generator's params have N = 1024
    with pytest.raises(ValueError):
        tfhe_amd.Generator.new(4).generate_lookup_table_assign(lambda x: x, small)
    lut = tfhe_amd.LookupTable.new()
    lut.poly = np.zeros(2 * N, np.uint64)  # right size, wrong word type
    with pytest.raises(ValueError):
        tfhe_amd.Generator.new(4).generate_lookup_table_full_assign(lambda x: x, lut)
    lut.poly = np.zeros(4 * N, np.uint32)[::2]  # right size and type, not contiguous
    with pytest.raises(ValueError):
        tfhe_amd.Generator.new(4).generate_lookup_table_assign(lambda x: x, lut)


def test_function_values_past_32_bits_reduce_mod_m_first(oracle):
    """Encoder.encode reduces the usize f(x) mod m (encoder.zig:66-74): f(x) >= 2^32
    with m not a power of two gives (f(x) mod m), not (f(x) mod 2^32) mod m."""
    m = 7
    f = [(1 << 40) + 3 * x for x in range(m)]
    got = tfhe_amd.Generator.new(m).generate_lookup_table(lambda x: f[x]).poly
    want = oracle.lut_generate(N, m, np.array([v % m for v in f], np.uint32))
    assert np.array_equal(got, want)
    assert not np.array_equal(got, oracle.lut_generate(N, m, np.array([v & MAX_U32 for v in f], np.uint32)))


def test_huge_message_modulus_is_an_error_not_an_abort():
    """m is bounded (TFHE_LUT_MAX_M); m = 2^32 - 1 returns TFHE_ERR_INVALID from every entry."""
    import ctypes as C
    lib = tfhe_amd.load_library()
    p = tfhe_amd.make_params("128")
    tab = np.zeros(4, np.uint32)
    out = np.zeros(2 * N, np.uint32)
    u32p = C.POINTER(C.c_uint32)
    for call in (lambda m: lib.tfhe_lut_generate(C.byref(p), m, tab.ctypes.data_as(u32p), out.ctypes.data_as(u32p)),
                 lambda m: lib.tfhe_lut_generate_scaled(C.byref(p), m, 0.5, tab.ctypes.data_as(u32p),
                                                        out.ctypes.data_as(u32p)),
                 lambda m: lib.tfhe_lut_generate_full(C.byref(p), m, tab.ctypes.data_as(u32p),
                                                      out.ctypes.data_as(u32p))):
        assert call(0xFFFFFFFF) == -1
        assert call((1 << 24) + 1) == -1
