"""Timeline of a rocprofv3 --kernel-trace (+ --memory-copy-trace) CSV run (DEV TOOL): kernels and copies in
start order with their start/end relative to the first, gaps and overlaps.
usage: python scripts/timeline.py <dir with *_kernel_trace.csv> [name filter]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40], r.get("Queue_Id", "")))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "") + " " + r.get("Size", ""), ""))
rows.sort()
rows = [r for r in rows if flt in r[2]] if flt else rows
t0 = rows[0][0]
for s, e, n, q in (rows if os.environ.get("TL_ALL") else rows[-80:]):
    print(f"{(s - t0) / 1e6:10.3f} {(e - t0) / 1e6:10.3f} {(e - s) / 1e6:8.3f} ms  q{q:>3} {n}")
