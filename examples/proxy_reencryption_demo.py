"""examples/proxy_reencryption_demo.zig on the MI355X: Alice's ciphertexts re-encrypted for
Bob with an asymmetric key (Bob's public key only), then Bob -> Carol (multi-hop).  Key
material is generated on the host (seeded DefaultPrng restated); re-encryption runs on
the GPU (tfhe_gpu_reencrypt_batch, the key-switch lane kernel).

    python examples/proxy_reencryption_demo.py [--device 0] [--batch 4096]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "zig-tfhe_amd"))
import tfhe_amd  # noqa: E402


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--batch", type=int, default=4096, help="extra batch to time the GPU path")
    args = ap.parse_args(argv)
    p = tfhe_amd.make_params("128")
    ctx = tfhe_amd.Context(p, args.device)

    print("=== LWE Proxy Reencryption Demo (MI355X) ===\n")
    print("1. Setting up keys for Alice and Bob...")
    alice, bob = tfhe_amd.secret_key_new(p, 11), tfhe_amd.secret_key_new(p, 12)
    t0 = time.perf_counter()
    bob_pk = tfhe_amd.PublicKeyLv0(bob, seed0=100_000)
    pk_ms = (time.perf_counter() - t0) * 1e3
    print(f"   Bob's public key generated in {pk_ms:.2f} ms\n")

    print("2. Alice encrypts her data...")
    messages = np.array([1, 0, 1, 1, 0], np.uint8)
    alice_cts = alice.encrypt_bool(messages, seed0=500)
    for i, m in enumerate(messages):
        print(f"   - Message {i + 1}: {bool(m)}")

    print("\n3. Alice generates a proxy reencryption key (Alice -> Bob), asymmetric mode...")
    t0 = time.perf_counter()
    key_ab = tfhe_amd.ProxyReencryptionKey.new_asymmetric(alice, bob_pk, seed0=1_000_000)
    kg_ms = (time.perf_counter() - t0) * 1e3
    print(f"   Reencryption key generated in {kg_ms:.2f} ms")

    print("\n4. Proxy converts Alice's ciphertexts to Bob's ciphertexts (GPU)...")
    prox_ab = tfhe_amd.HipReencryptor(ctx, key_ab)
    t0 = time.perf_counter()
    bob_cts = prox_ab.reencrypt(alice_cts)
    re_ms = (time.perf_counter() - t0) * 1e3
    print(f"   {len(bob_cts)} ciphertexts reencrypted in {re_ms:.2f} ms")

    print("\n5. Bob decrypts the reencrypted data...")
    dec = bob.decrypt_bool(bob_cts)
    correct = int((dec == messages.astype(bool)).sum())
    for i, (d, m) in enumerate(zip(dec, messages)):
        print(f"   {'✓' if d == bool(m) else '✗'} Message {i + 1}: {bool(d)} (original: {bool(m)})")
    print(f"\nAccuracy: {correct}/{len(messages)}")

    print("\n=== Multi-Hop Reencryption Demo (Asymmetric): Alice -> Bob -> Carol ===")
    carol = tfhe_amd.secret_key_new(p, 13)
    key_bc = tfhe_amd.ProxyReencryptionKey.new_asymmetric(bob, tfhe_amd.PublicKeyLv0(carol, seed0=200_000),
                                                          seed0=3_000_000)
    prox_bc = tfhe_amd.HipReencryptor(ctx, key_bc)
    ct = alice.encrypt_bool([1], seed0=77)
    bob_ct = prox_ab.reencrypt(ct)
    carol_ct = prox_bc.reencrypt(bob_ct)
    bob_ok, carol_ok = bool(bob.decrypt_bool(bob_ct)[0]), bool(carol.decrypt_bool(carol_ct)[0])
    print(f"   Bob decrypts: {bob_ok} {'✓' if bob_ok else '✗'}")
    print(f"   Carol decrypts: {carol_ok} {'✓' if carol_ok else '✗'}")

    bits = np.random.default_rng(5).integers(0, 2, args.batch).astype(np.uint8)
    cts = alice.encrypt_bool(bits, seed0=10_000)
    prox_ab.reencrypt(cts)  # warm-up
    t0 = time.perf_counter()
    out = prox_ab.reencrypt(cts)
    batch_ms = (time.perf_counter() - t0) * 1e3
    batch_ok = int((bob.decrypt_bool(out) == bits.astype(bool)).sum())
    print(f"\n=== Performance Summary ===\nBob's public key generation: {pk_ms:.2f} ms\n"
          f"Reencryption key generation: {kg_ms:.2f} ms\n"
          f"Batch of {args.batch} reencryptions on the GPU: {batch_ms:.2f} ms "
          f"({args.batch / batch_ms * 1e3:.0f}/s incl. PCIe), {batch_ok}/{args.batch} decrypt correctly")
    prox_ab.close()
    prox_bc.close()
    ctx.close()
    ok = correct == len(messages) and bob_ok and carol_ok and batch_ok >= 0.99 * args.batch
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
