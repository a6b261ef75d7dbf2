"""examples/add_two_numbers.zig on the MI355X: 402 + 304 with a 16-bit ripple-carry adder
of encrypted bits (5 gates per full adder, 80 gate bootstraps).

Two ways, same results:
  gates   - the reference's program structure: each Gates.*Gate call is one bootstrap
            (one GPU launch of one item; latency-bound)
  circuit - the same adder recorded as a gate DAG and evaluated level by level
            (tfhe_gpu_circuit_eval: 33 levels, one batched launch each)

    python examples/add_two_numbers.py [--mode gates|circuit|both] [--device 0]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zig-tfhe_amd"))
import tfhe_amd  # noqa: E402
from tfhe_amd import bit_utils  # noqa: E402


def full_adder(gates, a, b, c):
    """add_two_numbers.zig:24-47."""
    a_xor_b = gates.xor_gate(a, b)
    a_and_b = gates.and_gate(a, b)
    a_xor_b_and_c = gates.and_gate(a_xor_b, c)
    s = gates.xor_gate(a_xor_b, c)
    carry = gates.or_gate(a_and_b, a_xor_b_and_c)
    return s, carry


def add(gates, a_bits, b_bits, cin):
    """add_two_numbers.zig:50-73: LSB first."""
    out, carry = [], cin
    for a, b in zip(a_bits, b_bits):
        s, carry = full_adder(gates, a, b, carry)
        out.append(s)
    return out, carry


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="both", choices=["gates", "circuit", "both"])
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args(argv)

    print("=== TFHE Add Two Numbers Example (MI355X) ===\n")
    t0 = time.perf_counter()
    ctx = tfhe_amd.Context("128", args.device)
    sk, _ = ctx.keygen(secret_seed=42, cloud_seed=43)
    print(f"Keys generated in {time.perf_counter() - t0:.2f} s\n")

    a, b = 402, 304
    expected = (a + b) & 0xFFFF
    print(f"Plaintext inputs:\n  A = {a}\n  B = {b}\n  Expected sum = {expected}\n")
    ca = bit_utils.encrypt(a, 16, sk, seed0=1000)
    cb = bit_utils.encrypt(b, 16, sk, seed0=2000)
    cin = sk.encrypt_bool([0], seed0=3000)[0]

    ok = True
    if args.mode in ("gates", "both"):
        gates = tfhe_amd.Gates(ctx)
        t0 = time.perf_counter()
        s, carry = add(gates, list(ca), list(cb), cin)
        ms = (time.perf_counter() - t0) * 1e3
        got = bit_utils.convert(sk.decrypt_bool(s))
        print(f"[gates]   {got} (carry {bool(sk.decrypt_bool(carry)[0])}) in {ms:.1f} ms, "
              f"{ms / 80:.2f} ms per gate")
        ok &= got == expected
    if args.mode in ("circuit", "both"):
        c = tfhe_amd.Circuit()
        wa = [c.input() for _ in range(16)]
        wb = [c.input() for _ in range(16)]
        wc = c.input()
        sum_wires, carry_wire = c.ripple_add(wa, wb, wc)
        c.output(*sum_wires, carry_wire)
        inputs = list(ca) + list(cb) + [cin]
        c.run(ctx, inputs)  # warm-up
        t0 = time.perf_counter()
        outs, depth = c.run(ctx, inputs)
        ms = (time.perf_counter() - t0) * 1e3
        dec = sk.decrypt_bool(outs)
        got = bit_utils.convert(dec[:16])
        print(f"[circuit] {got} (carry {bool(dec[16])}) in {ms:.1f} ms, {len(c.ops)} bootstraps in {depth} levels")
        ok &= got == expected
    ctx.close()
    print("\n✓ Success! Homomorphic addition computed correctly." if ok else "\n✗ Error! Result mismatch.")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
