"""Band-by-band reduce rehearsal on ONE GPU (DEV TOOL): a rank's share of config 3
(1920x1080, samples [0, S/N) of 512) traced (a) by rt_trace_device, then a 50-MB copy of the sums (the
reduce's stand-in, serialized after the trace as the unbanded step runs it); (b) by
rt_trace_device_bands with a no-op callback; (c) the same with every band's rows copied (device to device,
on the trace's caller stream right behind the band's reduce: what an RCCL reduce of the band waits for) as
soon as the band is delivered.  Prints the median wall time per frame of each, and the trace kernel's.
usage: python scripts/probe_bands.py [ranks N (default 8)] [bands (default 8)] [reps (default 7)]"""
import ctypes as C
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from blenderraytracer_amd import capi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
cfg = bench.CONFIGS["rtow"]
rt = bench.make_tracer(cfg, "f64", 1, 0)
lib = capi.load_library()
sc = rt.scene_handle()
st = rt.settings(sample_range=(0, cfg["spp"] // N))
n = cfg["w"] * cfg["h"]
sums = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
dst = torch.zeros_like(sums)
stream = torch.cuda.current_stream()
stats = capi.Stats()


def plain():
    sums.zero_()
    capi.check(lib.rt_trace_device(sc, C.byref(st), C.c_void_p(sums.data_ptr()), C.c_void_p(stream.cuda_stream), 0, None))
    dst.copy_(sums)


def banded(copy):
    sums.zero_()
    cw = cfg["w"]

    def ready(b, row0, rows, user):
        if copy:
            sl = slice(3 * row0 * cw, 3 * (row0 + rows) * cw)
            dst[sl].copy_(sums[sl])
        return 0
    cb = capi.BAND_FN(ready)
    capi.check(lib.rt_trace_device_bands(sc, C.byref(st), C.c_void_p(sums.data_ptr()), C.c_void_p(stream.cuda_stream),
                                         B, cb, None, C.byref(stats)))


for name, fn in (("plain+copy", plain), ("bands", lambda: banded(False)), ("bands+copies", lambda: banded(True)),
                 ("plain+copy", plain), ("bands", lambda: banded(False)), ("bands+copies", lambda: banded(True))):
    fn()
    torch.cuda.synchronize()
    ts, ks = [], []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
        ks.append(stats.kernel_ms)
    extra = f", trace kernel {statistics.median(ks):.3f} ms" if name != "plain+copy" else ""
    print(f"N={N} share {cfg['spp'] // N} spp, {B} bands, {name}: wall median {statistics.median(ts) * 1e3:.3f} ms "
          f"(min {min(ts) * 1e3:.3f}){extra}", flush=True)
