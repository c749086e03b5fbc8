"""Per-segment event counts of a workload for the instruction-floor model (DEV TOOL): the
kernel's own per-lane code compiled for the CPU with -DRT_HOST_COUNTERS (tests/hostcheck) traces a few
crops of the frame; prints the events per segment and bench.py's floor model on them as JSON.
usage: python scripts/floor_counts.py [config] [crop side] [spp]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "rtow"
side = int(sys.argv[2]) if len(sys.argv) > 2 else 48
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 8
cfg = bench.CONFIGS[cfg_name]
rt = bench.make_tracer(cfg, "f64", 1, 0)
print(json.dumps(bench.instruction_floor(rt, cfg, side=side, spp=spp), indent=1))
