"""Collect the bench lines of an alternating A/B run (gpurun_out/<TAG>_<variant><round>.json)
into one text record for profiles/: python tools/ab_collect.py TAG OUT "header line" ...
"""
import glob
import json
import re
import sys


def main():
    tag, out = sys.argv[1], sys.argv[2]
    head = sys.argv[3:]
    rows = []
    for f in sorted(glob.glob(f"gpurun_out/{tag}_*.json")):
        # variant names may end in digits (w0, md2): the round is the LAST digit run, rounds < 10
        m = re.match(rf"gpurun_out/{re.escape(tag)}_(.+)(\d)\.json$", f)
        try:
            d = json.loads(open(f).read().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        r = d.get("roofline") or {}
        rows.append((int(m.group(2)), m.group(1), d.get("value"), d.get("ms_per_step"), r.get("kernel_avg_ms"),
                     d.get("decrypt_check", d.get("sums_check")), (d.get("kernels") or "").split(" ")[0]))
    rows.sort()
    with open(out, "w") as fh:
        for h in head:
            fh.write(f"# {h}\n")
        fh.write("# round variant value ms_per_step kernel_avg_ms check blind_rotation_kernel\n")
        for rnd, v, val, ms, k, dc, kn in rows:
            fh.write(f"{rnd} {v} {val} {ms} {k} {dc} {kn}\n")
    print(open(out).read())


if __name__ == "__main__":
    main()
