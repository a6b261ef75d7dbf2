"""Kernel stats CSV (the columns of rocprofv3's --stats kernel_stats.csv) from a rocprofv3
run that wrote its default rocpd SQLite database instead of CSV.
usage: python tools/rocpd_stats.py <dir with the .db> <out.csv>"""
import csv
import glob
import sqlite3
import sys

db = glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)[0]
rows = sqlite3.connect(db).execute(
    "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
    "from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, c, s, a, mi, ma in rows:
        w.writerow([n, c, s, round(a, 1), round(100 * s / tot, 3), mi, ma])
