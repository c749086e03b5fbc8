"""Summarize SQ counter passes (scripts/pmc_sq.sh) for one kernel: usage pmc_report.py <outdir> [kernel]"""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "trace_kernel<double"
vals = defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
v = {k: x[-1] for k, x in vals.items()}   # last dispatch (timed one)
for k in sorted(v):
    print(f"{k:28s} {v[k]:.4g}")
if "SQ_INSTS_VALU" in v and "SQ_WAVES" in v:
    w = v["SQ_WAVES"]
    print(f"VALU insts / wave        {v['SQ_INSTS_VALU'] / w:.4g}")
    print(f"SALU insts / wave        {v.get('SQ_INSTS_SALU', 0) / w:.4g}")
    print(f"SMEM insts / wave        {v.get('SQ_INSTS_SMEM', 0) / w:.4g}")
    print(f"branches / wave          {v.get('SQ_INSTS_BRANCH', 0) / w:.4g}")
if "SQ_THREAD_CYCLES_VALU" in v and "SQ_ACTIVE_INST_VALU" in v:
    print(f"VALU lane utilization    {v['SQ_THREAD_CYCLES_VALU'] / (64 * v['SQ_ACTIVE_INST_VALU']):.3f}")
if "SQ_WAVE_CYCLES" in v:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in v:
            print(f"{k} / WAVE_CYCLES  {v[k] / v['SQ_WAVE_CYCLES']:.3f}")
