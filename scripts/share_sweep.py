"""Per-rank share of a multi-GPU frame, timed on ONE GPU (DEV TOOL; DESIGN.md "Multi-GPU projection").

    python scripts/share_sweep.py [--reps 3] > gpurun_out/shares.json

Rank r of N traces samples [r*S/N, (r+1)*S/N) of every pixel (distributed.ShardedRender).  This times
rt_trace_device over the sample range of rank 0 for N = 1, 2, 4, 8 on configs 3 and 4 (the shares the
8-GPU node's ranks run) and prints the projected N-GPU frame time = max share time + the RCCL reduce
(not measurable on one GPU: given as the 3 x 8 bytes/pixel of the sums over one xGMI link, 2 hops).
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from blenderraytracer_amd import capi  # noqa: E402
from blenderraytracer_amd.renderer import GpuRayTracer  # noqa: E402
from blenderraytracer_amd.scene import load_scene_json  # noqa: E402

XGMI_LINK_GBS = 153.0   # one xGMI link per direction (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    lib = capi.load_library()
    out = {}
    for name, w, h, spp in (("config3_rtow", 1920, 1080, 512), ("config4_rtow4k", 3840, 2160, 1024)):
        rt = GpuRayTracer(w, h, seed=1)
        assert rt.load_from_json(load_scene_json("rtow.json"))
        rt.update_render_settings({"maxBounces": 5, "samples": spp})
        scene = rt.scene_handle()
        buf = torch.zeros(w * h * 3, dtype=torch.float64, device="cuda")
        rows = {}
        for n in (1, 2, 4, 8):
            st = rt.settings(sample_range=(0, spp // n))
            stats = capi.Stats()
            ms = []
            for k in range(args.reps + 1):
                buf.zero_()
                torch.cuda.synchronize()
                capi.check(lib.rt_trace_device(scene, C.byref(st), C.c_void_p(buf.data_ptr()), None, 1, C.byref(stats)))
                if k:
                    ms.append(stats.kernel_ms)
            t = min(ms)
            reduce_ms = 2 * w * h * 3 * 8 / (XGMI_LINK_GBS * 1e9) * 1e3 if n > 1 else 0.0
            rows[n] = {"share_spp": spp // n, "share_kernel_ms": round(t, 3),
                       "share_msamples_per_s": round(w * h * (spp // n) / (t * 1e-3) / 1e6, 1),
                       "reduce_ms_estimate": round(reduce_ms, 3)}
            print(f"{name} N={n}: {spp // n} spp share {t:.2f} ms", file=sys.stderr, flush=True)
        t1 = rows[1]["share_kernel_ms"]
        for n, r in rows.items():
            proj = r["share_kernel_ms"] + r["reduce_ms_estimate"]
            r["projected_frame_ms"] = round(proj, 3)
            r["projected_speedup"] = round(t1 / proj, 3)
            r["projected_efficiency"] = round(t1 / proj / n, 3)
        out[name] = rows
        rt.close()
        del buf
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
