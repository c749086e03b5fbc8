"""Progressive render timeline probe (DEV TOOL): config 3 in 16 batches of 32 spp with a preview frame
and a progress callback after each (the Node drop-in's default), `reps` times after a warm-up; meant to
run under rocprofv3 --kernel-trace (scripts/timeline.py reads the trace).
usage: python scripts/probe_preview_timeline.py [reps] [preview 0|1]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
want = ("rgba8", "preview") if (len(sys.argv) <= 2 or sys.argv[2] == "1") else ("rgba8",)
rt = bench.make_tracer(bench.CONFIGS["rtow"], "f64", 1, 0)
rt.render()
for k in range(reps + 1):
    calls = []
    t = time.perf_counter()
    rt.render(on_progress=lambda f: calls.append(f) and False, want=want, batch_samples=32)
    dt = time.perf_counter() - t
    print(f"rep {k}: wall {dt * 1e3:.1f} ms, kernel_ms {rt.last_stats.kernel_ms:.1f}, progress calls {len(calls)}",
          flush=True)
