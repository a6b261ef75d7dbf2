"""Gate-bootstrap throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: B NAND gates (128-bit
params) = linear pre-combination + blind rotation (700 CMUX) + sample extract
+ identity key switch, inputs already resident in HBM.  One process per GPU
(torch.distributed.run); per-GPU batch fixed (weak scaling); the cloud key is
generated on rank 0 and broadcast once over RCCL/xGMI; no collective on the
data path.  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--params 128]

Other BASELINE configs (parity cases; these print their own line, never the
default one): --workload adder (config 3: 16-bit ripple-carry adder, one
circuit = 80 gates in 33 levels, and --batch independent adders side by side),
mixed (config 4: --batch gates per GPU, op uniform over AND/OR/XOR/MUX),
lut (config 5: UINT4 programmable bootstrap, --batch 4096), reenc (SURVEY
§8f N4: proxy re-encryption of --batch TLWELv0 ciphertexts).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zig-tfhe_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (loads the HIP runtime before libtfhe_gpu.so)
import torch.distributed as dist  # noqa: E402

import tfhe_dist as tdist  # noqa: E402
import tfhe_amd  # noqa: E402

HBM_PEAK_BPS = 8.0e12  # MI355X_MICROARCH.md chip table (spec)
METRIC = "gate-bootstraps/sec (NAND, 128-bit params) at 1/2/4/8 MI355X; % HBM roofline"


def algorithmic_bytes_per_gate(p) -> int:
    """Streamed-key model: each gate consumes every BK row once
    (n*2L*2*N f64) + its two input TLWELv0 + the TLWELv1 it writes."""
    return p.n * 2 * p.L * 2 * p.N * 8 + 2 * (p.n + 1) * 4 + (p.N + 1) * 4


def f64_ops_per_cmux(L: int) -> int:
    """Algorithmic f64 adds+muls of one CMUX (no FMA: the reference's
    expression trees), excluding torus conversion: 2L forward + 2 inverse
    512-point radix-2 FFTs (1,793 non-trivial butterflies x 4 mul + 2 add,
    2,304 x 4 add), 2L twists + 2 untwists (4 mul + 2 add per point, + the
    1/1024 norm), 2L x 2 x 512 complex MACs (4 mul + 4 add).  L=3: 235,568;
    matches SQ_INSTS_VALU_{ADD,MUL}_F64 x 64 to within the conversion adds
    (profiles/r01_pmc_blind_rotate_whole.txt)."""
    fft_mul, fft_add = 1793 * 4, 1793 * 2 + 2304 * 4
    fwd, inv = 2 * L, 2
    mul = (fwd + inv) * fft_mul + fwd * 2048 + inv * (2048 + 1024) + 2 * L * 2 * 512 * 4
    add = (fwd + inv) * fft_add + fwd * 1024 + inv * 1024 + 2 * L * 2 * 512 * 4
    return mul + add


VALU_F64_PEAK = 256 * 4 * 16 * 2.4e9  # non-FMA f64 ops/s: 256 CUs x 4 SIMD x 16 lanes x 2.4 GHz (78.6 TF FMA spec / 2)
# measured with tools/isa_rate.hip (profiles/r01_isa_rate.txt): independent v_add_f64 / v_mul_f64
# at 4 waves per SIMD issue every 2.01 ns per SIMD -> 1024 SIMDs x 64 lanes / 2.01 ns
VALU_F64_SUSTAINED = 1024 * 64 / 2.01e-9


def cpu_baseline(p, sk, bk, ksk, A, B, gpu_out, seconds: float):
    """Oracle (C restatement of zig-tfhe's CPU path, -O3) on the host cores,
    on a bounded sample of the same workload; also spot-checks GPU bits."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import CloudKeyArrays, Oracle, params
    o = Oracle(fast=True)
    op = params("128")
    ck = CloudKeyArrays(0x82080000, np.concatenate([np.zeros(p.N, np.uint32),
                                                    np.full(p.N, 0x20000000, np.uint32)]), ksk, bk)
    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    # parity spot check of the first gates of the GPU batch
    nchk = min(cores, A.shape[0])
    want = o.gate_batch(op, np.zeros(nchk, np.uint8), A[:nchk], B[:nchk], ck, threads=cores)
    spot_ok = bool(np.array_equal(want, gpu_out[:nchk]))
    # single-thread rate on a few gates, then all cores for ~`seconds`
    t0 = time.perf_counter()
    o.gate_batch(op, np.zeros(2, np.uint8), A[:2], B[:2], ck, threads=1)
    st_rate = 2 / (time.perf_counter() - t0)
    done, t0 = 0, time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < seconds:
        idx = (np.arange(cores) + i) % A.shape[0]
        o.gate_batch(op, np.zeros(cores, np.uint8), A[idx], B[idx], ck, threads=cores)
        done += cores
        i += cores
    rate = done / (time.perf_counter() - t0)
    return {"value": round(rate, 2), "unit": "gate-bootstraps/s", "cores": cores, "kind": "port",
            "sample": (f"{done} NAND gate bootstraps (128-bit) of the same batch, {cores} threads x 1 gate each, "
                       f"~{seconds:.0f}s; single-thread {st_rate:.2f} gates/s; oracle/tfhe_oracle.c -O3"),
            "parity_spot_check": {"gates": nchk, "bit_exact": spot_ok}}


def timed(fn, steps, warmup, world, device):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        st = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        el = float(st[0])
    return el, out


def run_workload(args, rank, world, device):
    """Configs 3-5 of BASELINE.json (host-buffer APIs: PCIe copies included)."""
    pname = "uint4" if args.workload == "lut" else args.params
    ctx = tfhe_amd.Context(pname, device.index)
    p = ctx.params
    if rank == 0:
        sk, _ = ctx.keygen(42, 43)
    if world > 1:
        tdist.broadcast_cloud_key(ctx, device)
        kbuf = torch.zeros(p.n + p.N, dtype=torch.int64, device=device)
        if rank == 0:
            kbuf[:] = torch.from_numpy(np.concatenate([sk.key_lv0, sk.key_lv1]).astype(np.int64))
        dist.broadcast(kbuf, 0)
        kk = kbuf.cpu().numpy().astype(np.uint32)
        sk = tfhe_amd.SecretKey(p, kk[:p.n], kk[p.n:])
    g = np.random.default_rng(2000 + rank)
    extra = {}
    if args.workload == "adder":
        nadd = args.batch
        c = tfhe_amd.Circuit()
        wa = [[c.input() for _ in range(16)] for _ in range(nadd)]
        wb = [[c.input() for _ in range(16)] for _ in range(nadd)]
        wc = [c.input() for _ in range(nadd)]
        for k in range(nadd):
            sm, carry = c.ripple_add(wa[k], wb[k], wc[k])
            c.output(*sm)
        xa, xb = g.integers(0, 1 << 16, nadd), g.integers(0, 1 << 16, nadd)
        xa[0], xb[0] = 402, 304
        bits = np.concatenate([((xa[:, None] >> np.arange(16)) & 1).ravel(), ((xb[:, None] >> np.arange(16)) & 1).ravel(),
                               np.zeros(nadd, np.int64)]).astype(np.uint8)
        inputs = sk.encrypt_bool(bits, seed0=1)
        el, (outs, depth) = timed(lambda: c.run(ctx, inputs), args.steps, args.warmup, world, device)
        dec = sk.decrypt_bool(outs).reshape(nadd, 16)
        vals = (dec.astype(np.int64) << np.arange(16)).sum(1)
        ok = bool(np.array_equal(vals, (xa + xb) & 0xFFFF)) and int(vals[0]) == 706
        units = len(c.ops) * world * args.steps  # every adder gate is a bootstrap
        metric, unit = "gate-bootstraps/sec (16-bit ripple-carry adders, level-scheduled circuit)", "gate-bootstraps/s"
        extra = {"adders_per_step": nadd * world, "gates_per_adder": len(c.ops) // nadd, "levels": depth,
                 "ms_per_adder_circuit": round(el / args.steps * 1e3, 3), "sums_check": ok}
        workload = f"{nadd} independent 16-bit ripple-carry adders per GPU (examples/add_two_numbers.zig), 402+304 first"
    elif args.workload == "mixed":
        B = args.batch
        c = tfhe_amd.Circuit()
        ins = [c.input() for _ in range(3 * B)]
        kinds = g.integers(0, 4, B)
        bits = g.integers(0, 2, 3 * B).astype(np.uint8)
        want = np.empty(B, bool)
        for k in range(B):
            x, y, z = ins[3 * k], ins[3 * k + 1], ins[3 * k + 2]
            bx, by, bz = bits[3 * k], bits[3 * k + 1], bits[3 * k + 2]
            if kinds[k] == 0: c.output(c.and_(x, y)); want[k] = bx & by
            elif kinds[k] == 1: c.output(c.or_(x, y)); want[k] = bx | by
            elif kinds[k] == 2: c.output(c.xor(x, y)); want[k] = bx ^ by
            else: c.output(c.mux(x, y, z)); want[k] = by if bx else bz
        inputs = sk.encrypt_bool(bits, seed0=1)
        el, (outs, depth) = timed(lambda: c.run(ctx, inputs), args.steps, args.warmup, world, device)
        ok = bool(np.array_equal(sk.decrypt_bool(outs), want))
        n_boot = int(sum(1 for op in c.ops if op != tfhe_amd.NOT))
        units = B * world * args.steps
        metric, unit = "gates/sec (mixed AND/OR/XOR/MUX, 128-bit)", "gates/s"
        extra = {"bootstraps_per_sec": round(n_boot * world * args.steps / el, 2), "levels": depth,
                 "decrypt_check": ok}
        workload = f"{B} gates per GPU, op uniform over AND/OR/XOR/MUX (MUX = 3 bootstraps, 2 levels)"
    elif args.workload == "reenc":
        B = args.batch
        alice, bob = tfhe_amd.secret_key_new(p, 11), tfhe_amd.secret_key_new(p, 12)
        key = tfhe_amd.ProxyReencryptionKey.new_symmetric(alice, bob, 1000)  # same seeds on every rank
        hr = tfhe_amd.HipReencryptor(ctx, key)
        bits = g.integers(0, 2, B).astype(np.uint8)
        cts = alice.encrypt_bool(bits, seed0=1)
        el, outs = timed(lambda: hr.reencrypt(cts), args.steps, args.warmup, world, device)
        ok = bool(np.array_equal(bob.decrypt_bool(outs), bits.astype(bool)))
        hr.close()
        units = B * world * args.steps
        metric, unit = "TLWELv0 proxy re-encryptions/sec", "reencryptions/s"
        extra = {"decrypt_check": ok, "dtype": "u32"}
        workload = (f"{B} reencryptTLWELv0 per GPU (proxy_reenc.zig:267-306; n={p.n}, basebit {p.basebit}, "
                    f"t={p.iks_t}; host buffers, PCIe included)")
    else:  # lut
        B = args.batch
        m = 16
        tv = tfhe_amd.lut_generate(p, m, lambda x: (x * x + 3) % m)
        msgs = g.integers(0, m, B).astype(np.uint32)
        cts = sk.encrypt_lwe_message(msgs, m, seed0=1)
        el, outs = timed(lambda: ctx.bootstrap_lut_batch(cts, tv), args.steps, args.warmup, world, device)
        ok = bool(np.array_equal(sk.decrypt_lwe_message(outs, m), (msgs * msgs + 3) % m))
        units = B * world * args.steps
        metric, unit = "programmable bootstraps/sec (UINT4 LUT)", "bootstraps/s"
        extra = {"decrypt_check": ok}
        workload = f"{B} UINT4 LUT bootstraps per GPU (f(x) = x^2+3 mod 16; n=820, L=1, Bg=2^22, t=3, basebit 5)"
    if rank == 0:
        line = {"metric": metric, "value": round(units / el, 2), "unit": unit, "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic (seeded keys and inputs)",
                "config": {"workload": workload, "params": pname, "parallelism": f"dp{world}"}}
        line.update(extra)
        print(json.dumps(line), flush=True)
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="NAND gates per GPU per step")
    ap.add_argument("--params", default="128")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--workload", default="nand", choices=["nand", "adder", "mixed", "lut", "reenc"],
                    help="nand = the headline metric (default); others: BASELINE configs 3-5")
    args = ap.parse_args()

    rank, world, local = tdist.env_rank_world()
    if world > 1:
        dist.init_process_group(args.dist_backend)  # nccl = RCCL over xGMI
    # one rank per GPU; --dist-backend gloo with more ranks than GPUs only
    # rehearses the multi-rank path (ranks then share a device)
    device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(device)
    if args.workload != "nand":
        run_workload(args, rank, world, device)
        if world > 1:
            dist.destroy_process_group()
        return

    ctx = tfhe_amd.Context(args.params, device.index)
    p = ctx.params
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    bk = ksk = None
    if rank == 0:
        sk, (bk, ksk) = ctx.keygen(42, 43, want_host_copy=want_cpu)
    if world > 1:
        tdist.broadcast_cloud_key(ctx, device)
        kbuf = torch.zeros(p.n + p.N, dtype=torch.int64, device=device)
        if rank == 0:
            kbuf[:] = torch.from_numpy(np.concatenate([sk.key_lv0, sk.key_lv1]).astype(np.int64))
        dist.broadcast(kbuf, 0)
        kk = kbuf.cpu().numpy().astype(np.uint32)
        sk = tfhe_amd.SecretKey(p, kk[:p.n], kk[p.n:])

    # synthetic inputs: fresh encryptions of uniform random bits (seed 1000 + rank)
    B = args.batch
    g = np.random.default_rng(1000 + rank)
    a_bits = g.integers(0, 2, B).astype(np.uint8)
    b_bits = g.integers(0, 2, B).astype(np.uint8)
    A = sk.encrypt_bool(a_bits, seed0=1_000_000 + rank * 10 * B)
    Bc = sk.encrypt_bool(b_bits, seed0=5_000_000 + rank * 10 * B)
    t_ops = torch.zeros(B, dtype=torch.uint8, device=device)  # NAND
    t_a = torch.from_numpy(A.view(np.int32)).to(device)
    t_b = torch.from_numpy(Bc.view(np.int32)).to(device)
    t_o = torch.zeros_like(t_a)
    stream = torch.cuda.current_stream(device)
    ctx.set_stream(stream.cuda_stream)

    def step():
        ctx.gate_batch_dev(t_ops.data_ptr(), t_a.data_ptr(), t_b.data_ptr(), t_o.data_ptr(), B)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(device)
    out = t_o.cpu().numpy().view(np.uint32).copy()
    correct = bool(np.array_equal(sk.decrypt_bool(out), ~(a_bits.astype(bool) & b_bits.astype(bool))))

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    ctx.profile_begin()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    br_ms, ks_ms, launches = ctx.profile_end()

    stats = torch.tensor([elapsed, 0.0 if correct else 1.0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed = float(stats[0])
    all_correct = float(stats[1]) == 0.0

    if rank == 0:
        total = B * world * args.steps
        value = total / elapsed
        br_avg_s = br_ms / 1e3 / max(1, launches)
        ks_avg_s = ks_ms / 1e3 / max(1, launches)
        alg = algorithmic_bytes_per_gate(p) * B
        achieved = alg / br_avg_s
        f64_rate = f64_ops_per_cmux(p.L) * p.n * B / br_avg_s
        form = "split" if os.environ.get("TFHE_BR_KERNEL", "").startswith("s") else "whole"
        if form == "whole" and os.environ.get("TFHE_BR_LOADER", "1")[:1] != "0":
            form = "whole, loader waves"
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_blind_rotate_r01.json")
        if os.path.exists(pmc_path):
            pmc = json.load(open(pmc_path))
            if pmc.get("batch") == B and pmc.get("params") == args.params:
                traffic = pmc.get("hbm_bytes_per_launch")
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "gate-bootstraps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: fresh encryptions of uniform random bits under a seeded key (sk 42, ck 43)",
            "config": {"workload": f"{B} NAND gate bootstraps per GPU per step, SECURITY_128_BIT "
                                   f"(n={p.n}, N={p.N}, L={p.L}, Bg=2^{p.bgbit}, t={p.iks_t})",
                       "global_batch": B * world, "params": args.params, "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved / 1e9, 2), "peak": HBM_PEAK_BPS / 1e9,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_BPS, 4), "traffic": traffic,
                         "kernel": f"k_blind_rotate<{p.L}> ({form} form)", "kernel_avg_ms": round(br_avg_s * 1e3, 3),
                         "algorithmic_bytes_per_launch": alg},
            "valu_f64": {"achieved": round(f64_rate / 1e12, 2), "peak": round(VALU_F64_PEAK / 1e12, 1),
                         "unit": "Tops/s (f64 add+mul, no FMA)", "frac": round(f64_rate / VALU_F64_PEAK, 4),
                         "peak_sustained": round(VALU_F64_SUSTAINED / 1e12, 1),
                         "frac_sustained": round(f64_rate / VALU_F64_SUSTAINED, 4)},
            "key_switch_avg_ms": round(ks_avg_s * 1e3, 3),
            "decrypt_check": all_correct,
        }
        if want_cpu:
            line["cpu_baseline"] = cpu_baseline(p, sk, bk, ksk, A, Bc, out, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
