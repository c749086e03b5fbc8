"""Cost of progressive sample batches (DEV TOOL): one frame as one batch vs B-sample batches (with and
without preview frames and a progress callback), kernel (GPU) and wall time.
usage: python scripts/probe_batches.py [config] [batch ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
import bench  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "rtow"
batches = [int(b) for b in sys.argv[2:]] or [0, 32]
cfg = bench.CONFIGS[cfg_name]
rt = bench.make_tracer(cfg, "f64", 1, 0)
rt.render()
n = cfg["w"] * cfg["h"] * cfg["spp"]
for b in batches:
    for want, cb in ((("rgba8",), None), (("rgba8", "preview"), None), (("rgba8",), True), (("rgba8", "preview"), True)):
        if b == 0 and (cb is not None or "preview" in want):
            continue
        calls = []
        t = time.perf_counter()
        rt.render(want=want, batch_samples=b, on_progress=(lambda f: calls.append(f) and False) if cb else None)
        wall = time.perf_counter() - t
        st = rt.last_stats
        print(f"{cfg_name} batch {b} {'+'.join(w for w in want if w != 'rgba8') or 'plain'}{' progress' if cb else ''}: kernel {st.kernel_ms:.1f} ms, wall "
              f"{wall * 1e3:.1f} ms, {n / wall / 1e6:.0f} Msamples/s wall, {len(calls)} progress calls", flush=True)
