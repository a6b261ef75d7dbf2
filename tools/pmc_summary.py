"""Summarise rocprofv3 --pmc passes (gpurun_out/<dir>/p*/run_counter_collection.csv) per kernel."""
import collections, csv, glob, sys
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_br"
res = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        k = "BR" if "blind_rotate" in k else "KS" if "key_switch" in k else None
        if k:
            res[k][row["Counter_Name"]] = res[k].get(row["Counter_Name"], 0) + float(row["Counter_Value"])
for k, c in res.items():
    wc = c.get("SQ_WAVE_CYCLES", 1)
    print(k, " ".join("%s=%.4g" % kv for kv in sorted(c.items())))
    if "SQ_WAVES" in c:
        print("   per-wave: WAVE_CYCLES %.3g  active %.1f%%  wait_any %.1f%%  wait_inst %.1f%% (lds %.1f%%)  VALU %.1f%%" % (
            wc / c["SQ_WAVES"], 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 100 * c.get("SQ_WAIT_ANY", 0) / wc,
            100 * c.get("SQ_WAIT_INST_ANY", 0) / wc, 100 * c.get("SQ_WAIT_INST_LDS", 0) / wc,
            100 * c.get("SQ_ACTIVE_INST_VALU", 0) / wc))
