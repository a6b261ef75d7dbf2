"""Gate-bootstrap throughput on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: B NAND gates (128-bit
params) = linear pre-combination + blind rotation (700 CMUX) + sample extract
+ identity key switch, inputs already resident in HBM.  One process per GPU;
per-GPU batch fixed (weak scaling) unless --global-batch splits a fixed total
(strong scaling); the cloud key is generated on rank 0 and broadcast once over
RCCL/xGMI; no collective on the data path.  Rank 0 prints one JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B | --global-batch G] [--params 128]

--gpus N > 1 without RANK in the environment: this process starts
`torch.distributed.run --nproc-per-node N` on itself (a child process; this
one never touches a GPU) and exits with its status, so the plain command and
the torchrun form give the same line.  --single-process instead drives all N
devices from one process through the library's multi-device context
(tfhe_gpu_create_multi: in-library RCCL key broadcast, one host thread per
device; host-buffer API, so PCIe copies are inside the timed region).

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
KERNEL_SRC = os.path.join(ROOT, "zig-tfhe_amd", "csrc", "tfhe_kernels.hip")
PMC_PATH = os.path.join(ROOT, "profiles", "pmc_blind_rotate.json")
# rocprofv3 --kernel-trace --stats average of the blind-rotation kernel for the kernel
# binary it was measured on (tools/rocprof_record.py writes it from a committed stats csv)
ROCPROF_PATH = os.path.join(ROOT, "profiles", "rocprof_blind_rotate.json")
# the blind rotation's core-clock cycles per launch (tools/bin/clock_probe: s_memtime over
# s_memrealtime per wave, no phase marks; tools/clock_probe_record.py), invariant to DVFS
CLOCK_PROBE_PATH = os.path.join(ROOT, "profiles", "clock_probe.json")
REFERENCE_MS_PER_GATE = 37.31  # zig-tfhe's published single-thread gate time (CHANGELOG.md:86)


def kernel_source_hash() -> str:
    """sha256 of the HIP source in the tree (informational)."""
    import hashlib
    return hashlib.sha256(open(KERNEL_SRC, "rb").read()).hexdigest()[:16]


def kernel_build_id() -> str:
    """Tag of the kernel binary actually loaded: tfhe_gpu_build_id() = sha256 of
    the gfx950 kernels object the .so was linked from (a PMC file measured on
    another binary is not reported as this one's)."""
    return tfhe_amd.build_id()


def algorithmic_bytes_per_gate(p) -> int:
    """Streamed-key model: each gate consumes every BK row once
    (n*2L*2*N f64) + its two input TLWELv0 + the TLWELv1 it writes."""
    return p.n * 2 * p.L * 2 * p.N * 8 + 2 * (p.n + 1) * 4 + (p.N + 1) * 4


def f64_ops_per_cmux(L: int, fused: bool = False) -> int:
    """f64 VALU lane-operations (v_add/v_mul/v_fma_f64, one each) of one CMUX,
    the torus conversion's 4 adds per output coefficient (2N of them) included.
    Reference expression trees (fused=False; the reference's adds+muls): 2L
    forward + 2 inverse 512-point radix-2 FFTs (1,793 butterflies with a
    twiddle x 4 mul + 2 add, 2,304 x 4 add), 2L twists + 2 untwists (4 mul + 2 add
    per point, + the 1/1024 norm), 2L x 2 x 512 complex MACs (4 mul + 4 add).
    L=3: 243,760 (PMC: 241,603 per CMUX per item, profiles/r02a_pmc_blind_rotate.json: the
    kernel turns 48 products by an exact -1 into sign flips).
    Fused (the kernels' default at the L=3 / Bg=2^6 sets): a butterfly with a
    twiddle is 6 fma, a j = 0 one 2 add + 2 fma, a twist / untwist point 2 mul +
    2 fma (norm folded), a MAC term 4 fma, a torus conversion 1 add.  L=3: 145,424
    (151,568 with round 2's 4-add conversion; PMC 152,571 per CMUX per item for that
    build, profiles/r02c_pmc_blind_rotate.json)."""
    conversion = 2 * 1024 * 4  # torus_from_f64_small: v - t, 2 frac, t + adj, + 1.5*2^52
    if fused:  # torus_from_f64_near_integer: one add (v + 1.5*2^52) per coefficient
        conversion = 2 * 1024
        per_fft = 511 * 4 + 1793 * 6
        return (2 * L + 2) * per_fft + 2 * L * 512 * 4 + 2 * 512 * 4 + 2 * L * 2 * 512 * 4 + conversion
    fft_mul, fft_add = 1793 * 4, 1793 * 2 + 2304 * 4
    fwd, inv = 2 * L, 2
    mul = (fwd + inv) * fft_mul + fwd * 2048 + inv * (2048 + 1024) + 2 * L * 2 * 512 * 4
    add = (fwd + inv) * fft_add + fwd * 1024 + inv * 1024 + 2 * L * 2 * 512 * 4
    return mul + add + conversion


VALU_F64_PEAK = 256 * 4 * 16 * 2.4e9  # f64 VALU lane-ops/s: 256 CUs x 4 SIMD x 16 lanes x 2.4 GHz (78.6 TF FMA spec / 2)
# measured with tools/isa_rate.hip in core-clock cycles (profiles/r06o_isa_rate_cycles.txt; the
# round-1 ns figures ran at an unknown, ramping clock): independent v_fmac_f64, 8 chains per wave,
# issue every 4.41 cycles per SIMD at 4 waves per SIMD, 4.84 at 2 and 5.99 at 1
ISSUE_CYCLES_F64 = {4: 4.41, 2: 4.84, 1: 5.99}
VALU_F64_SUSTAINED = 1024 * 64 * 2.4e9 / ISSUE_CYCLES_F64[4]  # at 2.4 GHz, as VALU_F64_PEAK


def host_cpu_info() -> dict:
    """What the CPU baseline ran on: nproc, the affinity set, the cgroup CPU quota, lscpu's model."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip().lower().replace("(s)", "s").replace(" ", "_")] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def effective_cpus(info) -> int:
    """CPUs this process may actually use: the affinity set, capped by the
    cgroup CPU quota (256 hardware threads under a 16-CPU quota on the GPU box)."""
    cores = info["affinity"]
    quota = info.get("cgroup_cpu_quota")
    return max(1, min(cores, int(quota))) if quota else cores


def cpu_baseline(p, sk, bk, ksk, A, B, gpu_out, seconds: float):
    """Oracle (C restatement of zig-tfhe's CPU path, -O3 -march=x86-64-v4, no
    FMA contraction) on the host cores, on a bounded sample of the same workload
    (SURVEY §8d(ii)): one gate per thread on every CPU the process may use (the
    affinity set capped by the cgroup quota: `value`, `cores`), the whole
    affinity set beside it when that is larger, the single-thread rate, and a
    spot check of the GPU's bits."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import CloudKeyArrays, Oracle, params
    o = Oracle(fast=True)
    op = params("128")
    ck = CloudKeyArrays(0x82080000, np.concatenate([np.zeros(p.N, np.uint32),
                                                    np.full(p.N, 0x20000000, np.uint32)]), ksk, bk)
    info = host_cpu_info()
    cores = info["affinity"]
    nchk = min(16, A.shape[0])  # parity spot check of the first gates of the GPU batch
    want = o.gate_batch(op, np.zeros(nchk, np.uint8), A[:nchk], B[:nchk], ck, threads=nchk)
    spot_ok = bool(np.array_equal(want, gpu_out[:nchk]))
    t0 = time.perf_counter()
    o.gate_batch(op, np.zeros(2, np.uint8), A[:2], B[:2], ck, threads=1)
    st_rate = 2 / (time.perf_counter() - t0)

    def rate_on(threads, secs):
        done, i = 0, 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < secs:
            idx = (np.arange(threads) + i) % A.shape[0]
            o.gate_batch(op, np.zeros(threads, np.uint8), A[idx], B[idx], ck, threads=threads)
            done += threads
            i += threads
        return done, done / (time.perf_counter() - t0)

    eff = effective_cpus(info)
    done, rate = rate_on(eff, seconds)
    res = {"value": round(rate, 2), "unit": "gate-bootstraps/s", "cores": eff, "kind": "port",
           "sample": (f"{done} NAND gate bootstraps (128-bit) of the same batch, {eff} threads x 1 gate each "
                      f"(every CPU the process may use: affinity {cores} capped by the cgroup quota "
                      f"{info.get('cgroup_cpu_quota')}), ~{seconds:.0f}s; oracle/tfhe_oracle.c -O3 -march=x86-64-v4"),
           "single_thread": {"value": round(st_rate, 2), "ms_per_gate": round(1e3 / st_rate, 2),
                             "reference_published_ms_per_gate": REFERENCE_MS_PER_GATE},
           "host": info, "parity_spot_check": {"gates": nchk, "bit_exact": spot_ok}}
    if cores > eff:  # oversubscribed: one thread per CPU of the affinity set, for comparison
        fd, fr = rate_on(cores, seconds / 2)
        res["full_affinity"] = {"threads": cores, "value": round(fr, 2), "gates": fd}
    return res


def pmc_record(batch: int, params: str):
    """profiles/pmc_blind_rotate.json if it was measured on this kernel source, batch and params."""
    if not os.path.exists(PMC_PATH):
        return None, "no PMC file"
    pmc = json.load(open(PMC_PATH))
    if pmc.get("kernel_build_id") != kernel_build_id():
        return None, "PMC file measured on another kernel binary (build id differs): not reported"
    if pmc.get("batch") != batch or pmc.get("params") != params:
        return None, "PMC file measured on another batch / parameter set"
    return pmc, None


def clock_probe_record(batch: int, params: str):
    """profiles/clock_probe.json if it was measured on this kernel binary's source, batch and params."""
    if not os.path.exists(CLOCK_PROBE_PATH):
        return None
    rec = json.load(open(CLOCK_PROBE_PATH))
    if rec.get("kernel_build_id") != kernel_build_id() or rec.get("batch") != batch or rec.get("params") != params:
        return None
    return rec


def rooflines(p, B, params, br_avg_s, kernel):
    """Primary roofline: f64 VALU issue, the bound the blind rotation is on (its
    HBM traffic is ~60 GB/s): the kernel's f64 VALU lane-operations (model
    f64_ops_per_cmux, checked against the PMC instruction counts) per second vs
    the chip's issue rate; the SURVEY §8d streamed-key figure beside it."""
    fused = "fused" in kernel
    per_cmux = f64_ops_per_cmux(p.L, fused)
    ops = per_cmux * p.n * B
    f64_rate = ops / br_avg_s
    pmc, why = pmc_record(B, params)
    roof = {"bound": "valu_f64", "achieved": round(f64_rate / 1e12, 3), "peak": round(VALU_F64_PEAK / 1e12, 1),
            "unit": "T f64 VALU lane-ops/s (v_add/v_mul/v_fma_f64 count one each)",
            "frac": round(f64_rate / VALU_F64_PEAK, 4),
            "peak_sustained": round(VALU_F64_SUSTAINED / 1e12, 1),
            "frac_sustained": round(f64_rate / VALU_F64_SUSTAINED, 4),
            "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
            "kernel": kernel, "kernel_avg_ms": round(br_avg_s * 1e3, 3),
            "algorithmic_f64_ops_per_launch": ops, "f64_ops_per_cmux": per_cmux,
            # the reference's work (its expression trees' adds + muls) per second: what the
            # fused kernel's fewer instructions deliver, against the same issue peak
            "reference_equivalent": {"achieved": round(f64_ops_per_cmux(p.L) * p.n * B / br_avg_s / 1e12, 3),
                                     "frac": round(f64_ops_per_cmux(p.L) * p.n * B / br_avg_s / VALU_F64_PEAK, 4)},
            "arithmetic": "fused multiply-add (exact-integer regime, DESIGN.md §6)" if fused else "reference expression trees",
            "reference_tree_f64_ops_per_cmux": f64_ops_per_cmux(p.L)}
    # the clock THIS run held: the kernel's core-clock cycles per launch (clock probe; the same at every
    # clock) over this run's kernel time, and the fraction of the f64 issue peak AT that
    # clock: how much of the gap to `frac` is DVFS
    probe = clock_probe_record(B, params)
    if probe:
        clk = probe["cycles_per_launch"] / (br_avg_s * 1e9)
        roof["clock_ghz"] = round(clk, 4)
        roof["clock_provenance"] = (f"{probe['cycles_per_launch']:,} core-clock cycles per launch (+/- "
                                    f"{probe['cycles_per_launch_spread']:,}) from committed record "
                                    f"{os.path.relpath(CLOCK_PROBE_PATH, ROOT)} (kernel build id "
                                    f"{probe['kernel_build_id']}), over this run's kernel time (HIP events)")
        roof["frac_at_clock"] = round(f64_rate / (VALU_F64_PEAK / 2.4 * clk), 4)
    if pmc:
        if pmc.get("clock_ghz"):
            # the PMC pass's own clock (GRBM_GUI_ACTIVE / 8 / duration): profiled passes run slower and clock
            # lower; the line's clock when no clock-probe record matches
            key = "clock_ghz_pmc_pass" if probe else "clock_ghz"
            roof[key] = pmc["clock_ghz"]
            if not probe:
                roof["clock_provenance"] = record_provenance(PMC_PATH, pmc) + "; " + pmc.get("clock_basis", "")
                roof["frac_at_clock"] = round(f64_rate / (VALU_F64_PEAK / 2.4 * pmc["clock_ghz"]), 4)
        roof["pmc"] = {k: pmc[k] for k in ("valu_f64_insts_per_launch", "valu_insts_per_item_per_cmux",
                                           "lds_insts_per_item_per_cmux", "valu_insts_per_gate_wave_per_cmux",
                                           "lds_insts_per_gate_wave_per_cmux", "wait_any_frac_all_waves")
                       if k in pmc}
        roof["pmc"]["provenance"] = record_provenance(PMC_PATH, pmc)
        f64_insts = pmc.get("valu_f64_insts_per_launch", 0) + pmc.get("valu_fma_f64_insts_per_launch", 0)
        if f64_insts:
            roof["pmc"]["valu_f64_frac_from_pmc"] = round(f64_insts * 64 / br_avg_s / VALU_F64_PEAK, 4)
        # what binds the step: the SIMD's VALU issue for the item as a whole (gate
        # and loader waves, f64 and integer), as core-clock cycles per VALU wave-instruction per SIMD
        # (the kernel's cycles per launch / (PMC SQ_INSTS_VALU / 1,024 SIMDs)) against the issue
        # interval tools/isa_rate.hip measures in cycles (ISSUE_CYCLES_F64); both sides in cycles, so
        # the clock the run held cancels
        insts = pmc.get("raw_per_launch", {}).get("SQ_INSTS_VALU")
        if insts:
            per_simd = insts / (256 * 4)
            cyc = probe["cycles_per_launch"] / per_simd if probe else br_avg_s * 2.4e9 / per_simd
            roof["valu_issue"] = {"cycles_per_valu_inst_per_simd": round(cyc, 3),
                                  "peak_cycles_4_waves": ISSUE_CYCLES_F64[4], "peak_cycles_2_waves": ISSUE_CYCLES_F64[2],
                                  "peak_cycles_1_wave": ISSUE_CYCLES_F64[1], "frac": round(ISSUE_CYCLES_F64[4] / cyc, 4),
                                  "frac_2_waves": round(ISSUE_CYCLES_F64[2] / cyc, 4),
                                  "valu_insts_per_item_per_cmux": pmc.get("valu_insts_per_item_per_cmux"),
                                  "note": "cycles per VALU instruction per SIMD achieved vs the measured f64 issue interval "
                                          "(profiles/r06o_isa_rate_cycles.txt); the kernel runs 2 waves per SIMD "
                                          "(gate + loader), and one wave alone issues f64 every 5.99 cycles",
                                  "provenance": "SQ_INSTS_VALU " + record_provenance(PMC_PATH, pmc)
                                                + ("; cycles per launch from the clock-probe record" if probe
                                                   else "; cycles = in-run kernel time x 2.4 GHz (no clock-probe record)")}
        # the DRAM side of the same kernel: measured bytes per launch / kernel time / HBM peak
        roof["dram"] = {"achieved_gbs": round(pmc["hbm_bytes_per_launch"] / br_avg_s / 1e9, 1),
                        "peak_gbs": HBM_PEAK_BPS / 1e9,
                        "frac": round(pmc["hbm_bytes_per_launch"] / br_avg_s / HBM_PEAK_BPS, 4)}
    else:
        roof["traffic_note"] = why
    # the same kernel's rocprofv3 --stats average, beside the HIP-event one above
    rp, rwhy = rocprof_record()
    if rp:
        # rocprof basis: with the run's kernel trace committed, the launches after bench.py's
        # warm-up steps BY POSITION (never by dropping the slowest launch); otherwise the plain
        # average over every recorded launch (the basis of rounds 1-4)
        if "avg_ms_excl_warmup" in rp:
            avg = rp["avg_ms_excl_warmup"]
            basis = (f"the launches after the first {rp['warmup_launches_excluded']} (bench.py's warm-up steps) in "
                     f"dispatch order, from the kernel trace {rp['trace']}")
        else:
            avg, basis = rp["avg_ms"], "AverageNs of the csv row: every recorded launch"
        roof["kernel_avg_ms_rocprof"] = avg
        roof["rocprof"] = {k: rp[k] for k in ("launches", "avg_ms", "avg_ms_excl_warmup", "min_ms", "max_ms", "source")
                           if k in rp}
        roof["rocprof"]["basis"] = basis
        roof["rocprof"]["provenance"] = record_provenance(ROCPROF_PATH, rp)
        roof["frac_rocprof"] = round(ops / (avg / 1e3) / VALU_F64_PEAK, 4)
    else:
        roof["rocprof_note"] = rwhy
    alg = algorithmic_bytes_per_gate(p) * B
    # SURVEY §8d's streamed-key figure is not a DRAM roofline for this kernel: the 4 gates
    # of a workgroup share every BK row through LDS and the XCDs' L2s hold the key, so it
    # counts key bytes CONSUMED per second (no fraction of the HBM peak is claimed for it;
    # roofline.dram is the measured DRAM side)
    key = {"key_bytes_consumed_per_s": round(alg / br_avg_s, 0), "key_bytes_consumed_per_launch": alg,
           "note": "n*2L*2*N*8 + I/O bytes every gate consumes, / kernel time; on-chip reuse, not DRAM traffic"}
    return roof, key


def record_provenance(path, rec) -> str:
    """Which figures of the line are read from a committed record rather than measured in this run."""
    return (f"from committed record {os.path.relpath(path, ROOT)} (source {rec.get('source', rec.get('method', '?'))[:60]}), "
            f"measured in a separate profiled run, possibly on another box; matched to this binary by kernel build id "
            f"{rec.get('kernel_build_id')}")


def rocprof_record():
    """profiles/rocprof_blind_rotate.json if it was measured on this kernel binary."""
    if not os.path.exists(ROCPROF_PATH):
        return None, "no rocprof record"
    rec = json.load(open(ROCPROF_PATH))
    if rec.get("kernel_build_id") != kernel_build_id():
        return None, "rocprof record measured on another kernel binary (build id differs): not reported"
    return rec, None


def timed(fn, steps, warmup, world, device):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
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


def timed_circuit(ctx, circ, inputs, args, world, device):
    """A circuit workload timed both ways: through host buffers (tfhe_gpu_circuit_eval, PCIe
    copies in the timed region) and on HBM-resident inputs and outputs
    (tfhe_gpu_circuit_eval_dev on the torch stream: the line's value).
    -> (elapsed dev, outputs dev, depth, elapsed host, outputs host)."""
    el_host, (outs_host, depth) = timed(lambda: circ.run(ctx, inputs), args.steps, args.warmup, world, device)
    t_in = torch.from_numpy(np.ascontiguousarray(inputs).view(np.int32)).to(device)
    t_out = torch.zeros((len(circ.outputs), inputs.shape[1]), dtype=torch.int32, device=device)
    ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
    el, _ = timed(lambda: circ.run_dev(ctx, t_in.data_ptr(), t_out.data_ptr()), args.steps, args.warmup, world, device)
    outs = t_out.cpu().numpy().view(np.uint32)
    ctx.set_stream(None)
    return el, outs, depth, el_host, outs_host


def apply_opts(ctx, args):
    """--opt NAME=VALUE -> tfhe_gpu_set_option (names: tfhe_amd.OPTIONS)."""
    for kv in args.opt:
        k, _, v = kv.partition("=")
        ctx.set_option(k, v if k == "br_form" and not v.isdigit() else int(v))


def per_rank_batch(args, rank, world):
    """(items on this rank, items over all ranks, scaling): --global-batch G splits
    G contiguously (strong scaling); else --batch per GPU (weak scaling)."""
    if args.global_batch:
        lo, hi = tdist.shard_range(args.global_batch, rank, world)
        return hi - lo, args.global_batch, "strong"
    return args.batch, args.batch * world, "weak"


def shared_secret_key(ctx, p, rank, world, device):
    """Rank 0 generates the keys; the cloud key goes to every rank once over RCCL
    (tfhe_dist.broadcast_cloud_key), the secret key too (test data only: the
    bench encrypts its synthetic inputs and checks its outputs with it)."""
    sk = None
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
    return sk


def mixed_circuit(B, g):
    """Config 4: B independent gates, op uniform over AND/OR/XOR/MUX (a MUX is
    3 bootstraps in 2 levels, gates.zig:124-129), each over its own 3 inputs.
    -> (circuit, input bits, expected output bits)."""
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
    return c, bits, want


def run_workload(args, rank, world, device):
    """Configs 3-5 of BASELINE.json (host-buffer APIs: PCIe copies included)."""
    pname = "uint4" if args.workload == "lut" else args.params
    ctx = tfhe_amd.Context(pname, device.index)
    apply_opts(ctx, args)
    p = ctx.params
    sk = shared_secret_key(ctx, p, rank, world, device)
    if args.no_pack:
        ctx.set_option("circuit_pack", 0)
    g = np.random.default_rng(2000 + rank)
    B, total, scaling = per_rank_batch(args, rank, world)
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
        el, outs, depth, el_host, outs_host = timed_circuit(ctx, c, inputs, args, world, device)
        dec = sk.decrypt_bool(outs).reshape(nadd, 16)
        vals = (dec.astype(np.int64) << np.arange(16)).sum(1)
        ok = bool(np.array_equal(vals, (xa + xb) & 0xFFFF)) and int(vals[0]) == 706 and \
            bool(np.array_equal(outs, outs_host))
        units = len(c.ops) * world * args.steps  # every adder gate is a bootstrap
        metric, unit = "gate-bootstraps/sec (16-bit ripple-carry adders, level-scheduled circuit)", "gate-bootstraps/s"
        extra = {"adders_per_step": nadd * world, "gates_per_adder": len(c.ops) // nadd, "levels": depth,
                 "ms_per_adder_circuit": round(el / args.steps * 1e3, 3), "sums_check": ok,
                 "host_buffers": {"ms_per_step": round(el_host / args.steps * 1e3, 3),
                                  "note": "tfhe_gpu_circuit_eval: input/output PCIe copies in the timed region"}}
        workload = f"{nadd} independent 16-bit ripple-carry adders per GPU (examples/add_two_numbers.zig), 402+304 first"
        scaling = "weak"
    elif args.workload == "mixed":
        c, bits, want = mixed_circuit(B, g)
        inputs = sk.encrypt_bool(bits, seed0=1)
        el, outs, depth, el_host, outs_host = timed_circuit(ctx, c, inputs, args, world, device)
        ok = bool(np.array_equal(sk.decrypt_bool(outs), want)) and bool(np.array_equal(outs, outs_host))
        n_boot = int(sum(1 for op in c.ops if op != tfhe_amd.NOT))
        units = total * args.steps
        metric, unit = "gates/sec (mixed AND/OR/XOR/MUX, 128-bit)", "gates/s"
        extra = {"bootstraps_per_sec": round(n_boot * world * args.steps / el, 2), "levels": depth,
                 "decrypt_check": ok, "round_packing": not args.no_pack,
                 "host_buffers": {"value": round(total * args.steps / el_host, 2),
                                  "ms_per_step": round(el_host / args.steps * 1e3, 3),
                                  "note": "tfhe_gpu_circuit_eval: input/output PCIe copies in the timed region"}}
        workload = (f"{total} gates over {world} GPU(s) ({B} on rank 0), op uniform over AND/OR/XOR/MUX "
                    f"(MUX = 3 bootstraps, 2 levels)")
    elif args.workload == "reenc":
        alice, bob = tfhe_amd.secret_key_new(p, 11), tfhe_amd.secret_key_new(p, 12)
        key = tfhe_amd.ProxyReencryptionKey.new_symmetric(alice, bob, 1000)  # same seeds on every rank
        hr = tfhe_amd.HipReencryptor(ctx, key)
        bits = g.integers(0, 2, B).astype(np.uint8)
        cts = alice.encrypt_bool(bits, seed0=1)
        # value: inputs resident in HBM (tfhe_gpu_reencrypt_batch_dev on the torch stream);
        # the host-buffer API (PCIe copies included, the context's own stream) is timed first, beside it
        el_host, outs_host = timed(lambda: hr.reencrypt(cts), args.steps, args.warmup, world, device)
        t_in = torch.from_numpy(cts.view(np.int32)).to(device)
        t_out = torch.zeros_like(t_in)
        ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
        el, _ = timed(lambda: hr.reencrypt_dev(t_in.data_ptr(), t_out.data_ptr(), B), args.steps, args.warmup,
                      world, device)
        outs = t_out.cpu().numpy().view(np.uint32)
        ctx.set_stream(None)
        ok = bool(np.array_equal(bob.decrypt_bool(outs), bits.astype(bool))) and bool(np.array_equal(outs, outs_host))
        hr.close()
        units = total * args.steps
        metric, unit = "TLWELv0 proxy re-encryptions/sec", "reencryptions/s"
        extra = {"decrypt_check": ok, "dtype": "u32",
                 "host_buffers": {"value": round(total * args.steps / el_host, 2),
                                  "ms_per_step": round(el_host / args.steps * 1e3, 3),
                                  "note": "tfhe_gpu_reencrypt_batch: PCIe copies in the timed region"}}
        workload = (f"{total} reencryptTLWELv0 over {world} GPU(s) (proxy_reenc.zig:267-306; n={p.n}, "
                    f"basebit {p.basebit}, t={p.iks_t}; device-resident, tfhe_gpu_reencrypt_batch_dev)")
    else:  # lut
        m = 16
        tv = tfhe_amd.lut_generate(p, m, lambda x: (x * x + 3) % m)
        msgs = g.integers(0, m, B).astype(np.uint32)
        cts = sk.encrypt_lwe_message(msgs, m, seed0=1)
        # value: inputs resident in HBM (tfhe_gpu_bootstrap_lut_batch_dev on the torch stream);
        # the host-buffer API (PCIe copies included) is timed first, beside it
        el_host, outs_host = timed(lambda: ctx.bootstrap_lut_batch(cts, tv), args.steps, args.warmup, world, device)
        t_in = torch.from_numpy(np.ascontiguousarray(cts).view(np.int32)).to(device)
        t_tv = torch.from_numpy(np.ascontiguousarray(tv, np.uint32).view(np.int32)).to(device)
        t_out = torch.zeros_like(t_in)
        ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
        el, _ = timed(lambda: ctx.bootstrap_lut_batch_dev(t_in.data_ptr(), t_tv.data_ptr(), t_out.data_ptr(), B),
                      args.steps, args.warmup, world, device)
        outs = t_out.cpu().numpy().view(np.uint32)
        ctx.set_stream(None)
        ok = bool(np.array_equal(sk.decrypt_lwe_message(outs, m), (msgs * msgs + 3) % m)) and \
            bool(np.array_equal(outs, outs_host))
        units = total * args.steps
        metric, unit = "programmable bootstraps/sec (UINT4 LUT)", "bootstraps/s"
        extra = {"decrypt_check": ok,
                 "host_buffers": {"value": round(total * args.steps / el_host, 2),
                                  "ms_per_step": round(el_host / args.steps * 1e3, 3),
                                  "note": "tfhe_gpu_bootstrap_lut_batch: PCIe copies in the timed region"}}
        workload = (f"{total} UINT4 LUT bootstraps over {world} GPU(s) (f(x) = x^2+3 mod 16; n=820, L=1, "
                    f"Bg=2^22, t=3, basebit 5; device-resident, tfhe_gpu_bootstrap_lut_batch_dev)")
    ok_all = torch.tensor([0.0 if extra.get("decrypt_check", extra.get("sums_check", True)) else 1.0],
                          dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(ok_all, op=dist.ReduceOp.MAX)
    if rank == 0:
        for k in ("decrypt_check", "sums_check"):
            if k in extra:
                extra[k] = float(ok_all[0]) == 0.0
        line = {"metric": metric, "value": round(units / el, 2), "unit": unit, "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                "scaling": scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic (seeded keys and inputs)",
                "config": {"workload": workload, "params": pname, "parallelism": f"dp{world}"},
                "kernels": ctx.last_kernels()}
        line.update(extra)
        print(json.dumps(line), flush=True)
    ctx.close()


def run_single_process(args):
    """All --gpus devices from this one process through tfhe_gpu_create_multi:
    the library broadcasts the key over RCCL itself (a device listed twice gets
    a device-to-device copy) and runs one host thread per device.  Host-buffer
    entry points (PCIe in the timed region).  --workload nand (gate batches),
    mixed (config 4's circuit: components over the devices, or the level split
    with --opt circuit_split=2) or lut (config 5).  After the timed steps the
    same inputs run once on a single-device context with the same seeded key:
    `words_equal_one_device` says whether every output word matches."""
    n = args.gpus
    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(n))
    if len(devices) != n:
        raise SystemExit(f"bench.py: --devices lists {len(devices)} ids for --gpus {n}")
    pname = "uint4" if args.workload == "lut" else args.params
    ctx = tfhe_amd.Context.multi(pname, devices=devices)
    apply_opts(ctx, args)
    p = ctx.params
    t0 = time.perf_counter()
    sk, _ = ctx.keygen(42, 43)
    keygen_s = time.perf_counter() - t0
    B = args.global_batch or args.batch * n
    g = np.random.default_rng(1000)
    extra = {}
    if args.workload == "nand":
        a_bits = g.integers(0, 2, B).astype(np.uint8)
        b_bits = g.integers(0, 2, B).astype(np.uint8)
        A = sk.encrypt_bool(a_bits, seed0=1_000_000)
        Bc = sk.encrypt_bool(b_bits, seed0=5_000_000)
        ops = np.zeros(B, np.uint8)
        run = lambda c: c.gate_batch(ops, A, Bc)  # noqa: E731
        check = lambda out: bool(np.array_equal(sk.decrypt_bool(out), ~(a_bits.astype(bool) & b_bits.astype(bool))))  # noqa: E731
        metric, unit, units = METRIC + " [single-process multi-device context, host buffers]", "gate-bootstraps/s", B
        workload = f"{B} NAND gate bootstraps per step"
    elif args.workload == "mixed":
        circ, bits, want = mixed_circuit(B, g)
        inputs = sk.encrypt_bool(bits, seed0=1)
        run = lambda c: circ.run(c, inputs)[0]  # noqa: E731
        check = lambda out: bool(np.array_equal(sk.decrypt_bool(out), want))  # noqa: E731
        metric, unit, units = "gates/sec (mixed AND/OR/XOR/MUX, 128-bit) [single-process multi-device context]", "gates/s", B
        workload = f"{B} mixed AND/OR/XOR/MUX gates per step (config 4)"
    elif args.workload == "lut":
        m = 16
        tv = tfhe_amd.lut_generate(p, m, lambda x: (x * x + 3) % m)
        msgs = g.integers(0, m, B).astype(np.uint32)
        cts = sk.encrypt_lwe_message(msgs, m, seed0=1)
        run = lambda c: c.bootstrap_lut_batch(cts, tv)  # noqa: E731
        check = lambda out: bool(np.array_equal(sk.decrypt_lwe_message(out, m), (msgs * msgs + 3) % m))  # noqa: E731
        metric, unit, units = "programmable bootstraps/sec (UINT4 LUT) [single-process multi-device context]", "bootstraps/s", B
        workload = f"{B} UINT4 LUT bootstraps per step (config 5)"
    else:
        raise SystemExit("bench.py --single-process: --workload nand, mixed or lut")
    for _ in range(args.warmup):
        out = run(ctx)
    boots0 = ctx.device_bootstraps()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = run(ctx)
    el = time.perf_counter() - t0
    per_dev = ((ctx.device_bootstraps() - boots0) // max(1, args.steps)).tolist()
    ok = check(out)
    if args.workload == "mixed":
        extra["level_issue_us"] = ctx.get_option("level_issue_us")  # the level split's host issue time
        extra["circuit_split"] = ctx.get_option("circuit_split")
    kernels = ctx.last_kernels()
    ctx.close()
    one = tfhe_amd.Context(pname, devices[0])  # the same seeded key on one device
    apply_opts(one, args)
    one.keygen(42, 43)
    same = bool(np.array_equal(run(one), out))
    one.close()
    line = {"metric": metric, "value": round(units * args.steps / el, 2), "unit": unit, "n_gpus": n, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong" if args.global_batch else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: fresh encryptions of uniform random inputs under a seeded key (sk 42, ck 43)",
            "config": {"workload": f"{workload} over {n} device(s) {devices} of one context "
                                   f"(tfhe_gpu_create_multi; keygen + key broadcast {keygen_s:.1f} s, untimed)",
                       "global_batch": B, "params": pname, "parallelism": f"dp{n} (one process)"},
            "kernels": kernels, "bootstraps_per_device_per_step": per_dev,
            "decrypt_check": ok, "words_equal_one_device": same}
    line.update(extra)
    print(json.dumps(line), flush=True)


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: run `torch.distributed.run` on this script as
    a child process (this process never initialises a GPU) and return its status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # 0.3 s of GPU time at 6.2 ms per step
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024, help="gates per GPU per step (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="gates per step over all GPUs, split ceil(G/N) per GPU (strong scaling)")
    ap.add_argument("--params", default="128")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--prof-steps", type=int, default=50,
                    help="steps of the untimed profiled pass (HIP events per launch) after the timed region")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives --gpus devices through the library's multi-device context")
    ap.add_argument("--devices", default="",
                    help="--single-process: device ids (default 0..N-1); a device listed twice rehearses the "
                         "sharding on one GPU (device-to-device key copy instead of RCCL)")
    ap.add_argument("--no-pack", action="store_true", help="mixed/adder: circuit round packing off")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="tfhe_gpu_set_option before the run (A/B of kernel forms), e.g. br_loader=0, arith=1")
    ap.add_argument("--workload", default="nand", choices=["nand", "adder", "mixed", "lut", "reenc"],
                    help="nand = the headline metric (default); others: BASELINE configs 3-5")
    args = ap.parse_args()

    if args.single_process:
        return run_single_process(args)
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(spawn_ranks(args))
    rank, world, local = tdist.env_rank_world()
    if world != args.gpus:
        raise SystemExit(f"bench.py: {world} rank(s) launched but --gpus {args.gpus}")
    # one rank per GPU; --dist-backend gloo with more ranks than GPUs only
    # rehearses the multi-rank path (ranks then share a device).  The device is set
    # before the process group exists, so RCCL's communicator binds this rank's GPU.
    device = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group(args.dist_backend)  # nccl = RCCL over xGMI
    if args.workload != "nand":
        run_workload(args, rank, world, device)
        if world > 1:
            dist.destroy_process_group()
        return

    ctx = tfhe_amd.Context(args.params, device.index)
    apply_opts(ctx, args)
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
    B, total, scaling = per_rank_batch(args, rank, world)
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
    ctx.sync()
    ties0 = ctx.near_tie_items()
    # the timed region: K steps and nothing else (no per-launch events: they cost 0.5-0.9 ms
    # per step at 2,048-4,096 gates, profiles/r04k_batch_sizes.txt)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    ctx.sync()  # the device error word of the timed launches, and the guard's counter
    recomputed = ctx.near_tie_items() - ties0
    # kernel averages from a separate, untimed pass of the same steps with HIP events
    # recorded around every blind-rotation and key-switch launch on the launch stream
    prof_steps = max(1, min(args.steps, args.prof_steps))
    ctx.profile_begin()
    for _ in range(prof_steps):
        step()
    br_ms, ks_ms, launches = ctx.profile_end()

    stats = torch.tensor([elapsed, 0.0 if correct else 1.0], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
    elapsed = float(stats[0])
    all_correct = float(stats[1]) == 0.0

    if rank == 0:
        value = total * args.steps / elapsed
        br_avg_s = br_ms / 1e3 / max(1, launches)
        ks_avg_s = ks_ms / 1e3 / max(1, launches)
        kernels = ctx.last_kernels()
        roof, hbm = rooflines(p, B, args.params, br_avg_s, kernels.split(" + ")[0])
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "gate-bootstraps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: fresh encryptions of uniform random bits under a seeded key (sk 42, ck 43)",
            "config": {"workload": f"{B} NAND gate bootstraps per GPU per step, SECURITY_128_BIT "
                                   f"(n={p.n}, N={p.N}, L={p.L}, Bg=2^{p.bgbit}, t={p.iks_t})",
                       "global_batch": total, "params": args.params, "parallelism": f"dp{world}"},
            "roofline": roof,
            "key_bytes_consumed": hbm,
            "key_switch": {"kernel": " + ".join(kernels.split(" + ")[1:]), "avg_ms": round(ks_avg_s * 1e3, 3)},
            "kernel_timing": {"profiled_steps": prof_steps, "launches": launches,
                              "note": "kernel averages (roofline.kernel_avg_ms, key_switch.avg_ms) come from an "
                                      "untimed pass of profiled_steps steps after the timed region, HIP events "
                                      "around each launch on its stream; the timed steps carry no events"},
            "margin_guard": {"recomputed_items": recomputed, "items": B * args.steps,
                             "note": ("fused arithmetic; items that round a value 1/4 or more off its integer are "
                                      "redone in the reference's expression trees inside the timed launches "
                                      "(DESIGN.md §6.1)") if "fused" in kernels else
                                     "reference expression trees throughout (no guard, no admission assumption)"},
            "kernel_build_id": kernel_build_id(),
            "kernel_source_sha256": kernel_source_hash(),
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
