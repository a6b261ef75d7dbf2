"""rocprofv3 --pmc passes over tools/br_only.py -> profiles/pmc_blind_rotate.json.

Reads gpurun_out/<dir>/p*/run_counter_collection.csv (one counter group per
pass, tools/pmc_br.sh), keeps the blind-rotation launches, and writes the
per-launch figures bench.py reports as roofline.traffic / roofline.pmc,
tagged with the library's kernel build id (tfhe_gpu_build_id) so a later
kernel binary is not reported with these bytes.  FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 tallies
128-B streaming requests at 64 B); counter KB -> bytes x 1024.

    python tools/pmc_traffic.py gpurun_out/<dir> [batch] [params] [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def clock_from_grbm(d, kernel):
    """{'clock_ghz', 'clock_basis'} from the pass holding GRBM_GUI_ACTIVE and a kernel trace, or None."""
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        rows = [r for r in csv.DictReader(open(f)) if r["Kernel_Name"].split("(")[0] == kernel
                and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
        if not rows:
            continue
        # the dispatch's duration: the kernel trace of the same run if it was collected, else
        # the counter rows' own dispatch timestamps
        tr = glob.glob(os.path.join(os.path.dirname(f), "run_kernel_trace.csv"))
        src = csv.DictReader(open(tr[0])) if tr else rows
        dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
               for r in src if r["Kernel_Name"].split("(")[0] == kernel}
        act = collections.defaultdict(float)
        for r in rows:
            act[r["Dispatch_Id"]] += float(r["Counter_Value"])
        # warm launches only: the pass runs the batch several times, the first is cold
        ids = sorted((k for k in act if k in dur and dur[k] > 0), key=int)
        pairs = [(act[k], dur[k]) for k in (ids[1:] if len(ids) > 1 else ids)]
        if not pairs:
            continue
        a, ns = sum(p[0] for p in pairs), sum(p[1] for p in pairs)
        return {"clock_ghz": round(a / 8 / ns, 4), "grbm_gui_active_per_launch": a / len(pairs),
                "clock_pass_kernel_ns": ns / len(pairs), "clock_pass_launches": len(pairs),
                "clock_basis": "GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's kernel-trace duration, in a profiled "
                               "pass of its own (profiled passes clock lower than unprofiled runs)"}
    return None


def main():
    d = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    params = sys.argv[3] if len(sys.argv) > 3 else "128"
    n = {"128": 700, "80": 550, "uint4": 820}[params]
    # per blind-rotation kernel: the fused launch and the margin guard's
    # recompute launch (workgroups that return at once) are separate kernels;
    # the figures are the main kernel's, the one with the most counts
    by = collections.defaultdict(lambda: (collections.defaultdict(float), collections.defaultdict(set)))
    for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "k_blind_rotate" not in k:
                continue
            t, l = by[k.split("(")[0]]
            c = row["Counter_Name"]
            t[c] += float(row["Counter_Value"])
            l[c].add((f, row.get("Dispatch_Id", row.get("Correlation_Id", ""))))
    if not by:
        raise SystemExit(f"no blind-rotation rows under {d}")
    name = max(by, key=lambda k: sum(v for c, v in by[k][0].items() if c != "SQ_WAVES"))
    tot, launches = by[name]
    others = sorted(k for k in by if k != name)
    per = {c: tot[c] / max(1, len(launches[c])) for c in tot}
    fetch = per.get("FETCH_SIZE", 0.0) * 1024 * 2
    write = per.get("WRITE_SIZE", 0.0) * 1024
    import bench  # noqa: E402  (kernel_source_hash, kernel_build_id)
    rec = {
        "kernel": name, "batch": batch, "params": params,
        "kernel_build_id": bench.kernel_build_id(),
        "kernel_source_sha256": bench.kernel_source_hash(),
        "launches_per_pass": max(len(v) for v in launches.values()),
        "other_blind_rotation_kernels": others,
        "hbm_bytes_per_launch": int(fetch + write) if "FETCH_SIZE" in per and "WRITE_SIZE" in per else None,
        "fetch_bytes_corrected": int(fetch), "write_bytes": int(write),
        "raw_per_launch": {c: per[c] for c in sorted(per)},
        "method": ("rocprofv3 --pmc, one counter group per pass (tools/pmc_br.sh over tools/br_only.py "
                   f"{batch} 1), blind-rotation dispatches only; FETCH_SIZE x2 (gfx950 rule), KB x1024"),
    }
    if "SQ_INSTS_VALU_ADD_F64" in per:
        rec["valu_f64_insts_per_launch"] = per["SQ_INSTS_VALU_ADD_F64"] + per.get("SQ_INSTS_VALU_MUL_F64", 0.0)
        rec["valu_fma_f64_insts_per_launch"] = per.get("SQ_INSTS_VALU_FMA_F64", 0.0)
    # per item (= per gate wave and its loader wave): since round 5 the L = 3 whole form's loader
    # waves run polynomial b's inverse transform, conversion and gather, so the
    # loader's VALU is part of the item's stream; the gate wave's own share is a static count
    # (tools/isa_stats.py, profiles/r05_isa_census.txt).  The *_per_gate_wave_* keys of earlier
    # files are the same ratio (their loader waves issued almost no VALU).
    if "SQ_INSTS_VALU" in per:
        rec["valu_insts_per_item_per_cmux"] = round(per["SQ_INSTS_VALU"] / batch / n, 1)
    if "SQ_INSTS_LDS" in per:
        rec["lds_insts_per_item_per_cmux"] = round(per["SQ_INSTS_LDS"] / batch / n, 1)
    if "SQ_WAIT_ANY" in per and "SQ_WAVE_CYCLES" in per:
        rec["wait_any_frac_all_waves"] = round(per["SQ_WAIT_ANY"] / per["SQ_WAVE_CYCLES"], 4)
    if "SQ_ACTIVE_INST_VALU" in per and "SQ_WAVE_CYCLES" in per:
        rec["valu_active_frac_all_waves"] = round(per["SQ_ACTIVE_INST_VALU"] / per["SQ_WAVE_CYCLES"], 4)
    # effective clock (MI355X_MICROARCH.md, DVFS give-back): GRBM_GUI_ACTIVE is summed over the 8 XCDs;
    # the pass that collected it also ran --kernel-trace, which gives the same dispatch's duration
    clk = clock_from_grbm(d, name)
    if clk:
        rec.update(clk)
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "profiles", "pmc_blind_rotate.json")
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
