"""Progressive-render cost probe (DEV TOOL): config 3 as one batch and as 16 batches of 32 spp, each
rendered `reps` times; prints the median kernel and wall time.
usage: [PROBE_CONFIG=mesh50k] [PROBE_PROGRESS=1: with a progress callback] [PROBE_PREVIEW=1: running frames]
       python scripts/probe_progressive.py [reps] [batch sizes, comma-separated; 0 = one batch]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = bench.CONFIGS[os.environ.get("PROBE_CONFIG", "rtow")]
rt = bench.make_tracer(cfg, "f64", 1, 0)
rt.render()
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 32]
for b in sizes + sizes:
    ks, ws = [], []
    for _ in range(reps):
        t = time.perf_counter()
        rt.render(batch_samples=b, on_progress=(lambda f: False) if os.environ.get("PROBE_PROGRESS") else None,
                  want=("rgba8", "preview") if os.environ.get("PROBE_PREVIEW") else ("rgba8",))
        ws.append(time.perf_counter() - t)
        ks.append(rt.last_stats.kernel_ms)
    print(f"batch {b}: kernel median {statistics.median(ks):.1f} ms (min {min(ks):.1f}), wall median "
          f"{statistics.median(ws) * 1e3:.1f} ms", flush=True)
