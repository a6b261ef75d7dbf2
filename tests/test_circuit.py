"""Level-scheduled circuits: tfhe_gpu_circuit_eval vs a
gate-by-gate oracle evaluation, as the reference evaluates circuits
(examples/add_two_numbers.zig:24-73, gates.zig:124-129 muxNaive)."""
import numpy as np
import pytest

import tfhe_amd
from tfhe_amd import Circuit


def oracle_eval(oracle, keys, circ, inputs):
    """Reference semantics: each gate is one Gates.*Gate call (bootstrap) or a
    negation, evaluated in wire order."""
    p = keys.p
    wires = [np.asarray(x, np.uint32) for x in inputs]
    for op, a, b in zip(circ.ops, circ.ia, circ.ib):
        if op == tfhe_amd.NOT:
            wires.append((0 - wires[a].astype(np.int64)).astype(np.uint32))
        else:
            wires.append(oracle.gate_batch(p, np.array([op], np.uint8), wires[a][None], wires[b][None], keys.ck)[0])
    return np.array([wires[w] for w in circ.outputs])


def test_circuit_builder_wires():
    c = Circuit()
    a, b, cin = c.input(), c.input(), c.input()
    s, carry = c.full_adder(a, b, cin)
    c.output(s, carry)
    assert (a, b, cin) == (0, 1, 2)
    assert c.ops == [tfhe_amd.XOR, tfhe_amd.AND, tfhe_amd.AND, tfhe_amd.XOR, tfhe_amd.OR]
    assert c.outputs == [6, 7]
    m = c.mux(a, b, cin)
    assert c.ops[-4:] == [tfhe_amd.AND, tfhe_amd.NOT, tfhe_amd.AND, tfhe_amd.OR] and m == c.n_inputs + len(c.ops) - 1
    with pytest.raises(ValueError):
        c.input()  # inputs come first
    with pytest.raises(ValueError):
        c.and_(0, 999)


@pytest.mark.gpu
@pytest.mark.parametrize("pname", ["80", "128"])
def test_circuit_adder_16bit_bit_exact(oracle, pname):
    """402 + 304 = 706 through one circuit launch sequence; every one of the 17
    output words equals the reference's gate-by-gate evaluation.  "128" is
    BASELINE config 3 at its stated parameter set (examples/add_two_numbers.zig:
    24-73, 102-105): 80 oracle bootstraps, a few seconds of CPU."""
    from conftest import get_keys
    k = get_keys(oracle, pname)
    ctx = tfhe_amd.Context(pname, 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    c = Circuit()
    A = [c.input() for _ in range(16)]
    Bw = [c.input() for _ in range(16)]
    cin = c.input()
    s, carry = c.ripple_add(A, Bw, cin)
    c.output(*s, carry)
    bits = [(402 >> i) & 1 for i in range(16)] + [(304 >> i) & 1 for i in range(16)] + [0]
    inputs = sk.encrypt_bool(bits, seed0=77)
    got, depth = c.run(ctx, inputs)
    assert depth == 33  # carry chain: XOR then 2 levels per bit (AND, OR)
    val = sum(int(x) << i for i, x in enumerate(sk.decrypt_bool(got[:16])))
    assert val == 706 and not sk.decrypt_bool(got[16:])[0]
    assert np.array_equal(got, oracle_eval(oracle, k, c, inputs))
    ctx.close()


@pytest.mark.gpu
def test_circuit_mixed_gates_with_mux(oracle):
    """Config-4-shaped workload: independent AND/OR/XOR/MUX gates (MUX = 3
    bootstraps in 2 levels) over shared inputs, outputs bit-exact."""
    from conftest import get_keys
    k = get_keys(oracle, "80")
    ctx = tfhe_amd.Context("80", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    g = np.random.default_rng(5)
    c = Circuit()
    ins = [c.input() for _ in range(12)]
    want_bits = []
    bits = g.integers(0, 2, 12)
    for _ in range(24):
        kind = int(g.integers(0, 4))
        x, y, z = (int(v) for v in g.choice(12, 3, replace=False))
        if kind == 0: w = c.and_(ins[x], ins[y]); want_bits.append(bits[x] & bits[y])
        elif kind == 1: w = c.or_(ins[x], ins[y]); want_bits.append(bits[x] | bits[y])
        elif kind == 2: w = c.xor(ins[x], ins[y]); want_bits.append(bits[x] ^ bits[y])
        else: w = c.mux(ins[x], ins[y], ins[z]); want_bits.append(bits[y] if bits[x] else bits[z])
        c.output(w)
    inputs = sk.encrypt_bool(bits.astype(np.uint8), seed0=500)
    got, depth = c.run(ctx, inputs)
    assert depth == 2
    assert np.array_equal(sk.decrypt_bool(got), np.array(want_bits, bool))
    assert np.array_equal(got, oracle_eval(oracle, k, c, inputs))
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["adder128", "wide80"])
def test_circuit_device_resident(oracle, shape):
    """tfhe_gpu_circuit_eval_dev (inputs and outputs in HBM, async on the context
    stream) returns the host-buffer call's words and depth: the 16-bit adder at
    128-bit (33 levels), and a 2-level 80-bit circuit of 1,030 gates per level
    (a whole-form round plus a tail round)."""
    import torch
    from conftest import get_keys
    pname = "128" if shape == "adder128" else "80"
    k = get_keys(oracle, pname)
    ctx = tfhe_amd.Context(pname, 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    c = Circuit()
    if shape == "adder128":
        A = [c.input() for _ in range(16)]
        Bw = [c.input() for _ in range(16)]
        cin = c.input()
        s, carry = c.ripple_add(A, Bw, cin)
        c.output(*s, carry)
        bits = [(402 >> i) & 1 for i in range(16)] + [(304 >> i) & 1 for i in range(16)] + [0]
    else:
        ins = [c.input() for _ in range(40)]
        g = np.random.default_rng(11)
        first = [c.nand(ins[int(x)], ins[int(y)]) for x, y in g.integers(0, 40, (1030, 2))]
        for i in range(1030):
            c.output(c.xor(first[i], first[(i * 7 + 3) % 1030]))
        bits = g.integers(0, 2, 40).tolist()
    inputs = sk.encrypt_bool(bits, seed0=91)
    want, depth = c.run(ctx, inputs)
    t_in = torch.from_numpy(np.ascontiguousarray(inputs).view(np.int32)).to("cuda:0")
    t_out = torch.full((len(c.outputs), inputs.shape[1]), -1, dtype=torch.int32, device="cuda:0")
    try:
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)
        d2 = c.run_dev(ctx, t_in.data_ptr(), t_out.data_ptr())
        ctx.sync()
    finally:
        ctx.set_stream(None)
    assert d2 == depth
    assert np.array_equal(t_out.cpu().numpy().view(np.uint32), want)
    if shape == "adder128":
        assert sum(int(x) << i for i, x in enumerate(sk.decrypt_bool(want[:16]))) == 706
    ctx.close()


@pytest.mark.gpu
def test_circuit_device_resident_edges(oracle):
    """tfhe_gpu_circuit_eval_dev edge cases: no gates (the outputs are the inputs,
    reordered), no outputs (depth only), a bad graph rejected before any copy."""
    import torch
    from conftest import get_keys
    k = get_keys(oracle, "80")
    ctx = tfhe_amd.Context("80", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    w = ctx.params.n + 1
    x = np.random.default_rng(3).integers(0, 2**32, (3, w), dtype=np.uint32)
    t_in = torch.from_numpy(x.view(np.int32)).to("cuda:0")
    t_out = torch.zeros((3, w), dtype=torch.int32, device="cuda:0")
    none8, none32 = np.zeros(0, np.uint8), np.zeros(0, np.uint32)
    assert ctx.circuit_eval_dev(t_in.data_ptr(), 3, none8, none32, none32, np.array([2, 0, 1], np.uint32),
                                t_out.data_ptr()) == 0
    ctx.sync()
    assert np.array_equal(t_out.cpu().numpy().view(np.uint32), x[[2, 0, 1]])
    assert ctx.circuit_eval_dev(t_in.data_ptr(), 3, np.array([tfhe_amd.NAND], np.uint8), np.array([0], np.uint32),
                                np.array([1], np.uint32), none32, 0) == 1
    with pytest.raises(RuntimeError):  # forward reference
        ctx.circuit_eval_dev(t_in.data_ptr(), 3, np.array([tfhe_amd.AND], np.uint8), np.array([0], np.uint32),
                             np.array([3], np.uint32), np.array([3], np.uint32), t_out.data_ptr())
    ctx.sync()
    ctx.close()


@pytest.mark.gpu
def test_circuit_rejects_bad_graphs(oracle):
    from conftest import get_keys
    k = get_keys(oracle, "80")
    ctx = tfhe_amd.Context("80", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    x = np.zeros((2, ctx.params.n + 1), np.uint32)
    with pytest.raises(RuntimeError):  # forward reference
        ctx.circuit_eval(x, np.array([tfhe_amd.AND], np.uint8), np.array([0], np.uint32), np.array([2], np.uint32),
                         np.array([2], np.uint32))
    with pytest.raises(RuntimeError):  # unknown op
        ctx.circuit_eval(x, np.array([77], np.uint8), np.array([0], np.uint32), np.array([1], np.uint32),
                         np.array([2], np.uint32))
    out, depth = ctx.circuit_eval(x, np.zeros(0, np.uint8), np.zeros(0, np.uint32), np.zeros(0, np.uint32),
                                  np.array([1, 0], np.uint32))  # no gates: outputs are inputs
    assert depth == 0 and np.array_equal(out, x[[1, 0]])
    ctx.close()


@pytest.mark.gpu
def test_circuit_ragged_levels_tail_form(oracle):
    """Levels of 1,030 gates: a 1,024-gate whole-form round plus a 6-gate tail that
    launch_blind_rotate hands to the latency form (inputs gathered by index in both).
    Bit-identical to forcing the whole form for the full level, and level-1
    samples (tail included) bit-exact vs the oracle."""
    from conftest import get_keys
    k = get_keys(oracle, "80")
    ctx = tfhe_amd.Context("80", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    g = np.random.default_rng(11)
    c = Circuit()
    ins = [c.input() for _ in range(40)]
    pairs = g.integers(0, 40, (1030, 2))
    lvl1 = [c.and_(ins[x], ins[y]) if i % 2 else c.xor(ins[x], ins[y]) for i, (x, y) in enumerate(pairs)]
    lvl2 = [c.or_(lvl1[i], lvl1[(i * 7 + 3) % 1030]) for i in range(1030)]
    c.output(*lvl1, *lvl2)
    bits = g.integers(0, 2, 40)
    inputs = sk.encrypt_bool(bits.astype(np.uint8), seed0=900)
    got, depth = c.run(ctx, inputs)
    assert depth == 2
    l1 = np.array([(bits[x] & bits[y]) if i % 2 else (bits[x] ^ bits[y]) for i, (x, y) in enumerate(pairs)], bool)
    l2 = np.array([l1[i] | l1[(i * 7 + 3) % 1030] for i in range(1030)], bool)
    assert np.array_equal(sk.decrypt_bool(got), np.concatenate([l1, l2]))
    with ctx.options(br_form="whole"):
        forced, _ = c.run(ctx, inputs)
    assert np.array_equal(got, forced)
    for i in (0, 511, 1023, 1024, 1027, 1029):  # level-1 gates; 1024.. are the tail
        op = tfhe_amd.AND if i % 2 else tfhe_amd.XOR
        want = oracle.gate_batch(k.p, np.array([op], np.uint8), inputs[pairs[i][0]][None], inputs[pairs[i][1]][None], k.ck)
        assert np.array_equal(got[i], want[0])
    ctx.close()


@pytest.mark.gpu
def test_circuit_round_packing(oracle):
    """Round packing: level 1 has 1,064 gates, 40 of which only drive outputs.
    The scheduler moves those 40 to level 2 (one 1,024-gate round + a 140-gate
    level) instead of running a 40-gate tail after the round.  Outputs are
    bit-identical to the unpacked schedule (TFHE_OPT_CIRCUIT_PACK = 0), decrypt to
    the truth table and sample bit-exact vs the oracle.  (The packed/unpacked
    timing is a bench line, `bench.py --workload mixed [--no-pack]`, not an
    assertion here.)"""
    from conftest import get_keys
    k = get_keys(oracle, "80")
    ctx = tfhe_amd.Context("80", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    g = np.random.default_rng(12)
    c = Circuit()
    ins = [c.input() for _ in range(40)]
    pairs = g.integers(0, 40, (1064, 2))
    lvl1 = [c.and_(ins[x], ins[y]) if i % 2 else c.xor(ins[x], ins[y]) for i, (x, y) in enumerate(pairs)]
    lvl2 = [c.or_(lvl1[i], lvl1[i + 1]) for i in range(0, 200, 2)]  # uses gates 0..199 only
    c.output(*lvl1, *lvl2)
    bits = g.integers(0, 2, 40)
    inputs = sk.encrypt_bool(bits.astype(np.uint8), seed0=901)

    got, depth = c.run(ctx, inputs)
    assert depth == 2
    l1 = np.array([(bits[x] & bits[y]) if i % 2 else (bits[x] ^ bits[y]) for i, (x, y) in enumerate(pairs)], bool)
    l2 = np.array([l1[i] | l1[i + 1] for i in range(0, 200, 2)], bool)
    assert np.array_equal(sk.decrypt_bool(got), np.concatenate([l1, l2]))
    with ctx.options(circuit_pack=0):
        plain, _ = c.run(ctx, inputs)
    assert np.array_equal(got, plain)
    for i in (0, 1023, 1024, 1063):  # 1024.. are the moved gates
        op = tfhe_amd.AND if i % 2 else tfhe_amd.XOR
        want = oracle.gate_batch(k.p, np.array([op], np.uint8), inputs[pairs[i][0]][None], inputs[pairs[i][1]][None], k.ck)
        assert np.array_equal(got[i], want[0])
    ctx.close()


def oracle_cone(oracle, keys, circ, inputs, wire, memo):
    """The reference's gate-by-gate value of one wire (only its input cone)."""
    if wire < circ.n_inputs:
        return np.asarray(inputs[wire], np.uint32)
    if wire not in memo:
        g = wire - circ.n_inputs
        op, a, b = circ.ops[g], circ.ia[g], circ.ib[g]
        x = oracle_cone(oracle, keys, circ, inputs, a, memo)
        if op == tfhe_amd.NOT:
            memo[wire] = (0 - x.astype(np.int64)).astype(np.uint32)
        else:
            y = oracle_cone(oracle, keys, circ, inputs, b, memo)
            memo[wire] = oracle.gate_batch(keys.p, np.array([op], np.uint8), x[None], y[None], keys.ck)[0]
    return memo[wire]


def mixed_circuit(n_gates, n_inputs, seed):
    """BASELINE config 4's workload shape: independent gates, op uniform over
    AND/OR/XOR/MUX (MUX = Gates.muxNaive, gates.zig:124-129: 3 bootstraps in 2 levels)."""
    g = np.random.default_rng(seed)
    c = Circuit()
    ins = [c.input() for _ in range(n_inputs)]
    bits = g.integers(0, 2, n_inputs)
    want = []
    for _ in range(n_gates):
        kind = int(g.integers(0, 4))
        x, y, z = (int(v) for v in g.choice(n_inputs, 3, replace=False))
        if kind == 0: c.output(c.and_(ins[x], ins[y])); want.append(bits[x] & bits[y])
        elif kind == 1: c.output(c.or_(ins[x], ins[y])); want.append(bits[x] | bits[y])
        elif kind == 2: c.output(c.xor(ins[x], ins[y])); want.append(bits[x] ^ bits[y])
        else: c.output(c.mux(ins[x], ins[y], ins[z])); want.append(bits[y] if bits[x] else bits[z])
    return c, bits.astype(np.uint8), np.array(want, bool)


@pytest.mark.gpu
def test_circuit_mixed_config4_128bit(oracle):
    """BASELINE config 4 at 128-bit params: 1,200 independent AND/OR/XOR/MUX gates
    (~1,500 level-1 bootstraps: one whole-form round of 1,024 plus the rest), every
    gate's truth table, a sample (MUX outputs and gates of both rounds) bit-exact
    vs the reference's gate-by-gate evaluation, and the same circuit on a
    two-shard multi-device context (one GPU listed twice) bit-identical."""
    from conftest import get_keys
    k = get_keys(oracle, "128")
    ctx = tfhe_amd.Context("128", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    c, bits, want = mixed_circuit(1200, 96, 44)
    inputs = sk.encrypt_bool(bits, seed0=4400)
    got, depth = c.run(ctx, inputs)
    assert depth == 2
    assert sum(op != tfhe_amd.NOT for op in c.ops) > 1100
    assert np.array_equal(sk.decrypt_bool(got), want)
    mux_out = [i for i, w in enumerate(c.outputs) if c.ops[w - c.n_inputs] == tfhe_amd.OR]
    sample = sorted(set([0, 1, 600, 1199] + mux_out[:3] + mux_out[-2:]))
    memo = {}
    for i in sample:
        assert np.array_equal(got[i], oracle_cone(oracle, k, c, inputs, c.outputs[i], memo)), i
    ctx.close()
    # two shards (one GPU listed twice): the 96 shared inputs are replicated, so the
    # gates split evenly; both shards run, the words are the single device's
    multi = tfhe_amd.Context.multi("128", devices=[0, 0])
    multi.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    before = multi.device_bootstraps()
    got2, depth2 = c.run(multi, inputs)
    ran = multi.device_bootstraps() - before
    assert depth2 == 2 and np.array_equal(got2, got)
    n_boot = sum(op != tfhe_amd.NOT for op in c.ops)
    assert int(ran.sum()) == n_boot and ran.min() > 0
    assert abs(int(ran[0]) - int(ran[1])) <= 3  # components of at most 3 bootstraps (a MUX)
    multi.close()


def _check_schedule(c, levels):
    """Every gate after its inputs (NOT: with its input), in wire terms."""
    wl = [0] * c.n_inputs + [int(x) for x in levels]
    for g, (op, a, b) in enumerate(zip(c.ops, c.ia, c.ib)):
        w = c.n_inputs + g
        if op == tfhe_amd.NOT:
            assert wl[w] == wl[a]
        else:
            assert wl[w] >= wl[a] + 1
            if op != tfhe_amd.COPY:
                assert wl[w] >= wl[b] + 1


def test_circuit_schedule_round_packing_host():
    """tfhe_circuit_schedule (host only): the 1,064-gate level of
    test_circuit_round_packing hands its 40 output-only gates to level 2 on a
    256-CU device (one 1,024-gate round), keeps them without packing, and the
    depth stays 2."""
    g = np.random.default_rng(12)
    c = Circuit()
    ins = [c.input() for _ in range(40)]
    pairs = g.integers(0, 40, (1064, 2))
    lvl1 = [c.and_(ins[x], ins[y]) if i % 2 else c.xor(ins[x], ins[y]) for i, (x, y) in enumerate(pairs)]
    for i in range(0, 200, 2):
        c.or_(lvl1[i], lvl1[i + 1])
    plain, d0 = c.schedule(256, pack=False)
    packed, d1 = c.schedule(256, pack=True)
    assert d0 == d1 == 2
    assert np.bincount(plain, minlength=3)[1:].tolist() == [1064, 100]
    assert np.bincount(packed, minlength=3)[1:].tolist() == [1024, 140]
    assert (packed[1024:1064] == 2).all() and (packed[:1024] == 1).all()
    _check_schedule(c, packed)
    # a 64-CU device: rounds of 256 gates, 1,064 = 4 rounds + a 40-gate tail
    # (one latency-form pass, 0.43 round); level 2's 100 gates take two passes
    # (0.86).  Moved, level 2's 140 gates run as one whole-form round (1.0, cheaper
    # than three passes at 1.29; blind_rotate_plan): 5.0 < 5.29, so the 40 move
    p64, _ = c.schedule(64)
    assert np.array_equal(p64, packed)


def test_circuit_schedule_mixed_config4_host():
    """BASELINE config 4 (ops uniform over AND/OR/XOR/MUX, MUX = 3 bootstraps in
    2 levels): packing leaves level 1 a whole number of 1,024-gate rounds."""
    g = np.random.default_rng(4)
    c = Circuit()
    ins = [c.input() for _ in range(64)]
    for k in g.integers(0, 4, 8192):
        a, b, s = (ins[int(x)] for x in g.integers(0, 64, 3))
        c.output([c.and_, c.or_, c.xor][k](a, b) if k < 3 else c.mux(s, a, b))
    plain, d0 = c.schedule(256, pack=False)
    packed, d1 = c.schedule(256, pack=True)
    assert d0 == d1 == 2
    boot = np.array([op != tfhe_amd.NOT for op in c.ops])
    assert int((packed[boot] == 1).sum()) % 1024 == 0
    assert int((plain[boot] == 1).sum()) % 1024 != 0
    _check_schedule(c, packed)


def test_circuit_schedule_random_dags_host():
    """Random DAGs with NOT and COPY: packing keeps every dependency and the depth."""
    g = np.random.default_rng(7)
    for _ in range(20):
        c = Circuit()
        wires = [c.input() for _ in range(8)]
        for _ in range(int(g.integers(50, 3000))):
            a, b = (wires[int(x)] for x in g.integers(0, len(wires), 2))
            r = g.random()
            wires.append(c.not_(a) if r < 0.1 else c.copy(a) if r < 0.15 else c.nand(a, b))
        c.output(*wires[-5:])
        for cus in (4, 64, 256):
            _, d0 = c.schedule(cus, pack=False)
            packed, d1 = c.schedule(cus, pack=True)
            assert d0 == d1
            assert packed.max(initial=0) <= d0
            _check_schedule(c, packed)


def test_circuit_schedule_rejects_bad_graphs_host():
    c = Circuit()
    a = c.input()
    c.ops.append(77)  # unknown op
    c.ia.append(a)
    c.ib.append(a)
    with pytest.raises(tfhe_amd.TfheError):
        c.schedule()
    with pytest.raises(tfhe_amd.TfheError):
        Circuit().schedule(cus=0)


def config4_circuit(n_gates, n_inputs, seed):
    """Config 4 as bench.py --workload mixed builds it, with shared inputs: op
    uniform over AND/OR/XOR/MUX, operands drawn from n_inputs input wires."""
    g = np.random.default_rng(seed)
    c = Circuit()
    ins = [c.input() for _ in range(n_inputs)]
    bits = g.integers(0, 2, n_inputs).astype(np.uint8)
    kinds = g.integers(0, 4, n_gates)
    xyz = g.integers(0, n_inputs, (n_gates, 3))
    want = np.empty(n_gates, bool)
    for i, (kd, (x, y, z)) in enumerate(zip(kinds, xyz)):
        if kd == 0: c.output(c.and_(ins[x], ins[y])); want[i] = bits[x] & bits[y]
        elif kd == 1: c.output(c.or_(ins[x], ins[y])); want[i] = bits[x] | bits[y]
        elif kd == 2: c.output(c.xor(ins[x], ins[y])); want[i] = bits[x] ^ bits[y]
        else: c.output(c.mux(ins[x], ins[y], ins[z])); want[i] = bits[y] if bits[x] else bits[z]
    return c, bits, want, kinds


def test_circuit_partition_config4_host():
    """tfhe_circuit_partition (host only): an 8,192-gate config-4 circuit over 64
    shared inputs splits within 1 % over 2 and over 8 devices (inputs are
    replicated, so only a MUX's three gates stay together); one 16-bit adder is a
    single component and stays on one device."""
    c, _, _, _ = config4_circuit(8192, 64, 4)
    boot = np.array([op != tfhe_amd.NOT for op in c.ops])
    total = int(boot.sum())
    for D in (2, 8):
        dev = c.partition(D)
        per = np.bincount(dev[boot], minlength=D)
        assert per.sum() == total and (np.abs(per - total / D) <= 0.01 * total / D).all(), per
        # every gate sits with the gates that drive it
        for g, (op, a, b) in enumerate(zip(c.ops, c.ia, c.ib)):
            for w in (a, b) if op != tfhe_amd.NOT else (a,):
                if w >= c.n_inputs:
                    assert dev[w - c.n_inputs] == dev[g]
    a = Circuit()
    A, B = [a.input() for _ in range(16)], [a.input() for _ in range(16)]
    s, _ = a.ripple_add(A, B, a.input())
    a.output(*s)
    assert len(set(a.partition(8).tolist())) == 1


@pytest.mark.gpu
def test_circuit_config4_full_65536_128bit(oracle):
    """BASELINE config 4 at its full size on one GPU: 65,536 gates, op uniform over
    AND/OR/XOR/MUX over 64 shared inputs, 128-bit (~82 k level-1 bootstraps = 80
    whole-form rounds, 16 k level-2 ORs).  Every gate's truth table, and an oracle
    cone sample across level-1 rounds and MUX outputs bit-exact vs the reference's
    gate-by-gate evaluation."""
    from conftest import get_keys
    k = get_keys(oracle, "128")
    ctx = tfhe_amd.Context("128", 0)
    ctx.load_cloud_key(k.ck.offset, k.ck.testvec, k.ck.bk, k.ck.ksk)
    sk = tfhe_amd.SecretKey(ctx.params, k.k0, k.k1)
    c, bits, want, kinds = config4_circuit(65536, 64, 65536)
    inputs = sk.encrypt_bool(bits, seed0=65536)
    before = ctx.device_bootstraps()
    got, depth = c.run(ctx, inputs)
    assert depth == 2
    assert int((ctx.device_bootstraps() - before)[0]) == sum(op != tfhe_amd.NOT for op in c.ops)
    assert np.array_equal(sk.decrypt_bool(got), want)
    mux = np.flatnonzero(kinds == 3)
    single = np.flatnonzero(kinds != 3)
    sample = sorted(set(single[[0, 1, 1500, 20000, 40000, -1]].tolist() + mux[[0, 7000, -1]].tolist()))
    memo = {}
    for i in sample:
        assert np.array_equal(got[i], oracle_cone(oracle, k, c, inputs, c.outputs[i], memo)), i
    ctx.close()
