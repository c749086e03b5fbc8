"""Host experiment (dev tool): BVH walk work per segment on a crop of a workload, computed by the
kernel's own per-lane code compiled for the CPU (tests/hostcheck).  Builder / walk variants are
compared by passing -D defines.
usage: python scripts/bvh_work.py [config] [crop side] [spp] [DEF=1,DEF2=3]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import hostcheck_binding as hb  # noqa: E402
from blenderraytracer_amd import capi  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "rtow"
side = int(sys.argv[2]) if len(sys.argv) > 2 else 64
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 8
defs = tuple(d for d in sys.argv[4].split(",") if d) if len(sys.argv) > 4 else ()
cfg = dict(bench.CONFIGS[cfg_name], spp=spp)
rt = bench.make_tracer(cfg, "f64", 1, 0)
L = hb.lib(defs)
L.ptc_work.argtypes = [C.POINTER(capi.SceneDesc), C.POINTER(capi.Settings), C.POINTER(C.c_double)]
out = (C.c_double * 4)()
tot = [0.0] * 4
# a few crops spread over the frame
for (fx, fy) in ((0.5, 0.5), (0.25, 0.7), (0.75, 0.3), (0.5, 0.9), (0.1, 0.2)):
    x0, y0 = int(fx * (cfg["w"] - side)), int(fy * (cfg["h"] - side))
    st = rt.settings(crop=(x0, y0, side, side))
    assert L.ptc_work(C.byref(rt.packed().desc), C.byref(st), out) == 0
    tot = [a + b for a, b in zip(tot, out)]
seg = tot[0]
print(f"{cfg_name} {defs}: segments {seg:.0f}, nodes/seg {tot[1]/seg:.3f}, spheres/seg {tot[2]/seg:.3f}, "
      f"tris/seg {tot[3]/seg:.3f}")
