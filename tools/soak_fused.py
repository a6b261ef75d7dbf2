"""Soak of the default (fused, guarded) blind rotation against the reference's
expression trees on the same device, at a scale the oracle cannot check: BATCHES
batches of B gates with uniformly random ciphertext words (every rotation
uniform) and random gate ops, device-resident; every output word compared.
Development evidence for DESIGN.md §6.1 (profiles/r05_soak_fused.json).

    python tools/soak_fused.py [PARAMS=128] [BATCHES=256] [B=4096] [SEED=2024]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-tfhe_amd"))

import torch  # noqa: E402  (HIP runtime first)

import tfhe_amd  # noqa: E402


def main():
    pname = sys.argv[1] if len(sys.argv) > 1 else "128"
    batches = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 2024
    dev = torch.device("cuda", 0)
    c = tfhe_amd.Context(pname, 0)
    c.keygen(42, 43)
    n1 = c.params.n + 1
    c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    t_a = torch.empty((B, n1), dtype=torch.int32, device=dev)
    t_b = torch.empty_like(t_a)
    o_f = torch.empty_like(t_a)
    o_r = torch.empty_like(t_a)
    ops = torch.empty(B, dtype=torch.uint8, device=dev)
    differ = 0
    kernels = {}
    ties0 = c.near_tie_items()
    t0 = time.time()
    for rep in range(batches):
        t_a.random_(generator=gen)
        t_b.random_(generator=gen)
        ops.random_(0, 10, generator=gen)
        c.set_option("arith", tfhe_amd.ARITH_AUTO)
        c.gate_batch_dev(ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), o_f.data_ptr(), B)
        kernels["fused"] = c.last_kernels()
        c.set_option("arith", tfhe_amd.ARITH_REFERENCE)
        c.gate_batch_dev(ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), o_r.data_ptr(), B)
        kernels["reference"] = c.last_kernels()
        differ += int((o_f != o_r).any(dim=1).sum().item())
        if rep % 32 == 0:
            print(f"batch {rep}: {differ} gates differ so far", flush=True)
    torch.cuda.synchronize(dev)
    c.sync()
    rec = {"params": pname, "gates": batches * B, "batches": batches, "batch": B,
           "inputs": f"uniformly random ciphertext words (torch generator seed {seed}), ops uniform over the ten gates",
           "gates_with_differing_words": differ, "near_tie_items_recomputed": c.near_tie_items() - ties0,
           "kernels": kernels, "build_id": tfhe_amd.build_id(), "seconds": round(time.time() - t0, 1)}
    print(json.dumps(rec))
    c.set_stream(None)
    c.close()
    return 0 if differ == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
