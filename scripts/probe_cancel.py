"""Cancel-to-return latency of a progressive render (DEV TOOL): a full-frame render in `batches` batches
is cancelled from another thread (rt_cancel, as the Node drop-in's window.renderCancelled) at `at` of its
frame time; prints the latency per repetition and the checkpointed samples.
usage: python scripts/probe_cancel.py [config rtow|mesh50k] [reps] [batches (default 4; -16: the drop-in's)] [at]"""
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import bench  # noqa: E402
from blenderraytracer_amd import capi  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mesh50k"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 4
at = float(sys.argv[4]) if len(sys.argv) > 4 else 0.4
cfg = bench.CONFIGS[name]
rt = bench.make_tracer(cfg, "f64", 5, 0)
batch = cfg["spp"] // nb if nb > 0 else nb
lib = capi.load_library()
rt.render(batch_samples=batch)
t = time.perf_counter()
rt.render(batch_samples=batch)
frame = time.perf_counter() - t
lat = []
for r in range(reps):
    box = {}

    def run():
        try:
            rt.render(batch_samples=batch)
            box["rc"] = "finished"
        except RuntimeError as e:
            box["rc"] = str(e)[:40]
        box["t"] = time.perf_counter()
    th = threading.Thread(target=run)
    th.start()
    time.sleep(at * frame)
    t0 = time.perf_counter()
    capi.check(lib.rt_cancel(rt.scene_handle()))
    th.join()
    lat.append((box["t"] - t0) * 1e3)
    print(f"{name} batches {batch}: cancel-to-return {lat[-1]:.2f} ms of a {frame * 1e3:.1f}-ms frame "
          f"({box['rc']}, checkpoint {rt.checkpoint()[1]} samples)", flush=True)
print(f"{name}: median {statistics.median(lat):.2f} ms, frame {frame * 1e3:.1f} ms", flush=True)
