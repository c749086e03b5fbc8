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
# memory-pipeline ratios (scripts/pmc_sets.sh passes); *_sum counters add over the 256 CUs' TA/TD/TCP
if "TCP_TOTAL_CACHE_ACCESSES_sum" in v and "TCP_TCC_READ_REQ_sum" in v:
    print(f"L1 hit rate              {1 - v['TCP_TCC_READ_REQ_sum'] / v['TCP_TOTAL_CACHE_ACCESSES_sum']:.3f}")
if "TCC_HIT_sum" in v and "TCC_MISS_sum" in v:
    print(f"L2 hit rate              {v['TCC_HIT_sum'] / (v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.3f}")
# GRBM_GUI_ACTIVE as rocprofv3 reports it is the SUM over the 8 XCDs (MI355X_MICROARCH.md, DVFS note):
# one XCD's busy cycles are GRBM_GUI_ACTIVE / 8, so a per-CU fraction divides by 256 x GRBM / 8
if "GRBM_GUI_ACTIVE" in v:
    for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum",
              "TCP_PENDING_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum",
              "TD_TC_STALL_sum"):
        if k in v:
            print(f"{k} per CU-cycle  {v[k] / (256 * v['GRBM_GUI_ACTIVE'] / 8):.3f}")
