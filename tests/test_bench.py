"""The bench line's host-side arithmetic (bench.py), on CPU: the f64 operation
model behind roofline.achieved, the rank split of weak and strong scaling, and
the roofline object built from the committed PMC and rocprof records (the same
numbers the GPU line reports, recomputed here from the files)."""
import csv
import json
import os
import types

import pytest

import bench
import tfhe_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_f64_model():
    # 145,424 fused / 243,760 reference-tree f64 lane-ops per CMUX at L = 3
    assert bench.f64_ops_per_cmux(3, True) == 145424
    assert bench.f64_ops_per_cmux(3) == 243760
    # 8 transforms x (511 j=0 butterflies x 4 + 1,793 twiddled x 6), 6 twists + 2 untwists x 512 x 4,
    # 6 rows x 2 outputs x 512 MAC terms x 4, 2,048 one-add conversions
    fft = 511 * 4 + 1793 * 6
    assert 8 * fft + 8 * 2048 + 12 * 2048 + 2048 == 145424


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_rank_split(world):
    weak = types.SimpleNamespace(global_batch=0, batch=1024)
    strong = types.SimpleNamespace(global_batch=65536 + 5, batch=1024)
    assert [bench.per_rank_batch(weak, r, world) for r in range(world)] == [(1024, 1024 * world, "weak")] * world
    parts = [bench.per_rank_batch(strong, r, world) for r in range(world)]
    assert sum(p[0] for p in parts) == 65541 and max(p[0] for p in parts) - min(p[0] for p in parts) <= 1
    assert all(p[1:] == (65541, "strong") for p in parts)


def test_roofline_from_committed_records(monkeypatch):
    """roofline.frac_rocprof and roofline.valu_issue from profiles/ reproduce by hand
    from the committed csv and PMC file, for the build id those records carry."""
    pmc = json.load(open(bench.PMC_PATH))
    rp = json.load(open(bench.ROCPROF_PATH))
    assert pmc["kernel_build_id"] == rp["kernel_build_id"]
    monkeypatch.setattr(bench, "kernel_build_id", lambda: pmc["kernel_build_id"])  # the records' binary
    p = tfhe_amd.make_params("128")
    kernel_s = 5.97e-3
    roof, key = bench.rooflines(p, 1024, "128", kernel_s, "k_blind_rotate_assist<true> (whole form, fused)")
    ops = 145424 * 700 * 1024
    assert roof["algorithmic_f64_ops_per_launch"] == ops
    assert roof["frac"] == pytest.approx(ops / kernel_s / bench.VALU_F64_PEAK, abs=1e-4)
    # rocprof basis: the launches after the warm-up steps BY POSITION from the committed
    # kernel trace when the record names one, else the csv row's plain average over every launch
    src = os.path.join(ROOT, rp["source"])
    row = next(r for r in csv.DictReader(open(src)) if r["Name"].startswith(rp["kernel"] + "("))
    if "trace" in rp:
        ds = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
                    for x in csv.DictReader(open(os.path.join(ROOT, rp["trace"])))
                    if x["Kernel_Name"].split("(")[0] == rp["kernel"])
        assert len(ds) == int(row["Calls"])
        kept = [d for _, d in ds[rp["warmup_launches_excluded"]:]]
        avg_ms = sum(kept) / len(kept) / 1e6
    else:
        avg_ms = float(row["AverageNs"]) / 1e6
    assert roof["kernel_avg_ms_rocprof"] == pytest.approx(avg_ms, abs=1e-3)
    assert "committed record" in roof["rocprof"]["provenance"] and "committed record" in roof["pmc"]["provenance"]
    assert roof["frac_rocprof"] == pytest.approx(ops / (avg_ms / 1e3) / bench.VALU_F64_PEAK, abs=1e-4)
    # VALU issue in core-clock cycles: the kernel's cycles per launch (clock-probe record) per VALU
    # wave-instruction per SIMD, against the measured f64 issue interval at 4 waves per SIMD
    probe = json.load(open(bench.CLOCK_PROBE_PATH))
    cyc = probe["cycles_per_launch"] / (pmc["raw_per_launch"]["SQ_INSTS_VALU"] / 1024)
    assert roof["valu_issue"]["cycles_per_valu_inst_per_simd"] == pytest.approx(cyc, abs=1e-3)
    assert roof["valu_issue"]["frac"] == pytest.approx(4.41 / cyc, abs=1e-4)
    assert 0.5 < roof["valu_issue"]["frac"] < 1.0
    # DRAM side: measured bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, KB x1024)
    raw = pmc["raw_per_launch"]
    assert roof["traffic"] == int(raw["FETCH_SIZE"] * 1024 * 2 + raw["WRITE_SIZE"] * 1024)
    assert key["key_bytes_consumed_per_launch"] == bench.algorithmic_bytes_per_gate(p) * 1024


def test_clock_and_frac_at_clock_from_committed_records(monkeypatch):
    """roofline.clock_ghz = the clock probe's cycles per launch / this run's kernel time, and
    frac_at_clock = achieved / (1,024 SIMDs x 16 lanes x clock); the PMC pass's own clock
    (GRBM_GUI_ACTIVE / 8 XCDs / its kernel duration) beside it."""
    pmc = json.load(open(bench.PMC_PATH))
    probe = json.load(open(bench.CLOCK_PROBE_PATH))
    assert probe["kernel_build_id"] == pmc["kernel_build_id"]
    monkeypatch.setattr(bench, "kernel_build_id", lambda: pmc["kernel_build_id"])
    # the record's cycle counts reproduce from its launches: event ms x GHz, after the clock ramp
    settled = probe["launches"][3:]
    assert probe["cycles_per_launch"] == pytest.approx(
        sum(r["kernel_ms"] * r["clock_ghz"] for r in settled) / len(settled) * 1e6, rel=1e-4)
    # and the wave span's count is the same at every clock the launches held (1.88-2.35 GHz)
    spans = [r["wave_span_ms"] * r["clock_ghz"] * 1e6 for r in probe["launches"]]
    assert max(spans) / min(spans) < 1.001 and min(r["clock_ghz"] for r in probe["launches"]) < 2.0
    p = tfhe_amd.make_params("128")
    kernel_s = 5.97e-3
    roof, _ = bench.rooflines(p, 1024, "128", kernel_s, "k_blind_rotate_assist<true> (whole form, fused)")
    ops = 145424 * 700 * 1024
    clk = probe["cycles_per_launch"] / (kernel_s * 1e9)
    assert roof["clock_ghz"] == pytest.approx(clk, abs=1e-4)
    assert roof["frac_at_clock"] == pytest.approx(ops / kernel_s / (1024 * 16 * clk * 1e9), abs=1e-4)
    assert roof["frac_at_clock"] >= roof["frac"] - 1e-9 or clk > 2.4
    assert "this run's kernel time" in roof["clock_provenance"]
    # the PMC pass's clock, from its own counters
    pclk = pmc["grbm_gui_active_per_launch"] / 8 / pmc["clock_pass_kernel_ns"]
    assert pmc["clock_ghz"] == pytest.approx(pclk, abs=1e-3)
    assert roof["clock_ghz_pmc_pass"] == pmc["clock_ghz"]


def test_clock_falls_back_to_the_pmc_pass(monkeypatch, tmp_path):
    """Without a matching clock-probe record the line states the PMC pass's clock, as in round 6's
    first records."""
    pmc = json.load(open(bench.PMC_PATH))
    monkeypatch.setattr(bench, "kernel_build_id", lambda: pmc["kernel_build_id"])
    monkeypatch.setattr(bench, "CLOCK_PROBE_PATH", str(tmp_path / "none.json"))
    roof, _ = bench.rooflines(tfhe_amd.make_params("128"), 1024, "128", 5.97e-3, "k_blind_rotate_assist<true> (fused)")
    assert roof["clock_ghz"] == pmc["clock_ghz"] and "clock_ghz_pmc_pass" not in roof


def test_clock_probe_record_from_its_log():
    """tools/clock_probe_record.py turns the committed probe log back into the committed record's
    cycle counts (the numbers bench.py divides by its kernel time)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("cpr", os.path.join(ROOT, "tools", "clock_probe_record.py"))
    cpr = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cpr)
    probe = json.load(open(bench.CLOCK_PROBE_PATH))
    reps = cpr.parse(open(os.path.join(ROOT, probe["source"])).read())
    assert len(reps) == 6 and all(r["batch"] == 1024 and r["waves"] == 2048 for r in reps)
    rec = cpr.record(reps, probe["source"], probe["kernel_build_id"])
    for k in ("cycles_per_launch", "cycles_per_launch_spread", "cycles_per_wave_span", "cycles_per_wave_span_spread"):
        assert rec[k] == probe[k], k
    with pytest.raises(SystemExit):
        cpr.record(reps[:3], "x", "y")
