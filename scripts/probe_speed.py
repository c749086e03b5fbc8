"""Quick throughput probe: renders a workload at reduced spp in both precisions, prints Msamples/s.
usage: python scripts/probe_speed.py [config] [spp] [precisions] [accel: auto|brute|bvh]"""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402
from blenderraytracer_amd import capi  # noqa: E402
import bench  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "rtow"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 8
precs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["f32", "f64"]
accel = sys.argv[4] if len(sys.argv) > 4 else "auto"
cfg = dict(bench.CONFIGS[cfg_name], spp=spp)
for prec in precs:
    rt = bench.make_tracer(cfg, prec, 1, 0, accel)
    rt.render()                                  # warm-up + upload
    t = time.perf_counter()
    img = rt.render()
    dt = time.perf_counter() - t
    st = rt.last_stats
    n = cfg["w"] * cfg["h"] * spp
    print(f"{cfg_name} {cfg['w']}x{cfg['h']}x{spp} {prec} {accel}: wall {dt*1e3:.1f} ms, kernel {st.kernel_ms:.1f} ms, "
          f"{n / (st.kernel_ms * 1e-3) / 1e6:.1f} Msamples/s (kernel), segments/sample {st.segments / n:.3f}, "
          f"image md5 {hashlib.md5(img['rgba8'].tobytes()).hexdigest()[:12]}", flush=True)
    rt.close()
