"""SQ counters of the trace step (trace_pool_kernel + accumulate_kernel, one launch each) from one
rocprofv3 --pmc pass -> profiles/r01_final_sq_<workload>_<prec>.json (round 1), read by bench.py for `valu_issue`.
usage: python scripts/pmc_sq_summary.py COUNTERS.csv OUT.json"""
import csv
import json
import sys

KERNELS = ("trace_pool_kernel", "accumulate_kernel")
src, out = sys.argv[1:3]
tot = {}
for r in csv.DictReader(open(src)):
    if any(k in r["Kernel_Name"] for k in KERNELS):
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
f64 = sum(tot.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
res = {"kernels": list(KERNELS), "counters": tot,
       # issue slots: a wave64 VALU instruction holds a SIMD-32 for 2 cycles, a binary64 one for 4
       "valu_issue_slots": tot.get("SQ_INSTS_VALU", 0.0) + f64,
       "valu_lane_utilization": tot["SQ_THREAD_CYCLES_VALU"] / (64.0 * tot["SQ_ACTIVE_INST_VALU"])
       if tot.get("SQ_ACTIVE_INST_VALU") else None,
       "method": "rocprofv3 --pmc (one pass, SQ block) over bench.py --steps 1 --warmup 0; summed over the "
                 "two kernels of the trace step"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
