"""Benchmark of the path-tracing hot path (BASELINE.json metric) on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config rtow|cornell|rtow4k|mesh50k|sample_scene]
                    [--precision f64|f32] [--no-cpu-baseline] [--no-end-to-end]

A "step" renders one full frame of the workload: every pixel x every sample, traced on the GPU(s)
from a scene already resident in HBM, the per-pixel float64 sums RCCL-reduced to rank 0 (N>1), and
the epilogue (mean, tone map, gamma, RGBA8) run on rank 0's GPU.  Rank r traces samples
[r*S/N, (r+1)*S/N) of every pixel, so the frame is fixed as N grows ("scaling": "strong").

Prints ONE JSON line on rank 0 (driver contract).  `roofline` is computed from HIP events recorded
inside librt_hip.so on the stream the trace kernel runs on; `cpu_baseline` times the CPU oracle
(oracle/pt_oracle.c, 1 thread, the JS semantics in C) on a bounded crop of the same workload.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (load torch's HIP runtime before librt_hip.so)
import torch.distributed as dist  # noqa: E402

from blenderraytracer_amd import capi  # noqa: E402
from blenderraytracer_amd.distributed import ShardedRender  # noqa: E402
from blenderraytracer_amd.renderer import GpuRayTracer  # noqa: E402
from blenderraytracer_amd.scene import load_scene_json  # noqa: E402

METRIC = "Msamples/s (pixels×spp/s) at 1/2/4/8 MI355X; % HBM roofline; RMS vs JS ref"

# BASELINE.json configs; "rtow" (config 3) is the headline single-GPU workload
CONFIGS = {
    "sample_scene": dict(scene="sample_scene.json", w=256, h=256, spp=4, depth=4, cfg=1),
    "cornell": dict(scene="cornell.json", w=512, h=512, spp=64, depth=5, cfg=2),
    "rtow": dict(scene="rtow.json", w=1920, h=1080, spp=512, depth=5, cfg=3),
    "rtow4k": dict(scene="rtow.json", w=3840, h=2160, spp=1024, depth=5, cfg=4),
    "mesh50k": dict(scene="mesh50k", w=1920, h=1080, spp=256, depth=5, cfg=5),
}
# canonical algorithmic flops per primitive test, miss path
FLOPS = {"sphere": 23, "plane": 14, "box": 20, "triangle": 51, "mesh": 51}
HBM_PEAK_GBS = 8000.0                        # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_TFLOPS = {"f64": 78.6, "f32": 157.3}  # vector FP64 / FP32 (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="rtow", choices=sorted(CONFIGS))
    ap.add_argument("--precision", default="f64", choices=["f64", "f32"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--accel", default="auto", choices=["auto", "brute", "bvh"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true", help="skip the PCIe-inclusive rt_render timing")
    ap.add_argument("--cpu-crop", type=int, default=64, help="side of the square crop the CPU oracle renders")
    return ap.parse_args()


ACCEL = {"auto": capi.RT_ACCEL_AUTO, "brute": capi.RT_ACCEL_BRUTE, "bvh": capi.RT_ACCEL_BVH}


def make_tracer(cfg, precision, seed, device, accel="auto"):
    rt = GpuRayTracer(cfg["w"], cfg["h"], seed=seed, device=device,
                      precision=capi.RT_PREC_F64 if precision == "f64" else capi.RT_PREC_F32, accel=ACCEL[accel])
    assert rt.load_from_json(load_scene_json(cfg["scene"]))
    if (rt.width, rt.height) != (cfg["w"], cfg["h"]):
        rt.resize_canvas(cfg["w"], cfg["h"])
    rt.update_render_settings({"maxBounces": cfg["depth"], "samples": cfg["spp"]})
    return rt


def cpu_baseline(rt, cfg, side):
    """Oracle (C restatement of the JS, 1 thread) on a centred side x side crop at full spp/depth."""
    from oracle import binding
    w, h = cfg["w"], cfg["h"]
    side = min(side, w, h)
    x0, y0 = (w - side) // 2, (h - side) // 2
    st = rt.settings(crop=(x0, y0, side, side))
    binding.lib()
    t = time.perf_counter()
    binding.render(rt.packed(), st)
    dt = time.perf_counter() - t
    samples = side * side * st.samples
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"{side}x{side} crop at ({x0},{y0}) of the {w}x{h} frame, {st.samples} spp, "
                      f"maxDepth {cfg['depth']}: {samples} samples in {dt:.1f} s (oracle/pt_oracle.c, 1 thread)"}


def load_traffic(workload, precision):
    """HBM bytes per trace step (trace_pool_kernel + accumulate_kernel) from the rocprofv3 PMC passes
    (profiles/pmc_<workload>_<prec>.json, written by scripts/profile_round.sh)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}_{precision}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    return None


# VALU issue ceiling: 256 CUs x 4 SIMD-32s, a wave64 VALU instruction holds its SIMD for 2 cycles (a
# binary64 one for 4: FP64 vector is half the FP32 rate) at 2.4 GHz (MI355X_MICROARCH.md)
VALU_ISSUE_PEAK_GSLOTS = 256 * 4 * 2.4 / 2


def load_sq(workload, precision):
    """SQ counters of one trace step (profiles/sq_<workload>_<prec>.json, scripts/profile_round.sh)."""
    p = os.path.join(ROOT, "profiles", f"sq_{workload}_{precision}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return None


def main():
    args = parse()
    cfg = CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rt = make_tracer(cfg, args.precision, args.seed, local, args.accel)
    packed = rt.packed()
    flops_per_segment = sum(FLOPS[k] * (o.count if k in ("mesh", "triangle") else 1)
                            for k, o in zip(packed.kinds, packed.objects))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(rt, cfg, args.cpu_crop)

    job = ShardedRender(rt, rank=rank, world=world, device=torch.device("cuda", local))
    for _ in range(args.warmup):
        job.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    kernel_ms, segs, abytes, work = [], [], [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        job.step()
        kernel_ms.append(job.stats.kernel_ms)
        segs.append(job.stats.segments)
        abytes.append(job.stats.algorithmic_bytes)
        work.append((job.stats.node_visits, job.stats.sphere_tests, job.stats.tri_tests))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    e2e = None
    if rank == 0 and world == 1 and not args.no_end_to_end:
        # RayTracer.render as the drop-in boundary runs it (rt_render): sums zeroed on device, the
        # trace, the epilogue, Float32 post-gamma + RGBA8 frames copied back over PCIe
        rt.render()
        t1 = time.perf_counter()
        rt.render()
        wall = time.perf_counter() - t1
        e2e = {"value": round(cfg["w"] * cfg["h"] * rt.settings().samples / wall / 1e6, 3), "unit": "Msamples/s",
               "wall_ms": round(wall * 1e3, 3), "kernel_ms": round(rt.last_stats.kernel_ms, 3),
               "what": "one rt_render call from Python: trace + tone map/gamma/RGBA8 + Float32 and RGBA8 readback"}

    if rank == 0:
        total_samples = cfg["w"] * cfg["h"] * rt.settings().samples * args.steps
        value = total_samples / elapsed / 1e6
        k_ms = sum(kernel_ms) / len(kernel_ms)
        a_bytes = sum(abytes) / len(abytes)
        achieved = a_bytes / (k_ms * 1e-3) / 1e9
        seg_launch = sum(segs) / len(segs)
        nodes, sph, tri = (sum(w[k] for w in work) / len(work) for k in range(3))
        bvh = nodes > 0
        if bvh:   # BVH: slab test 12 flops/node + per-test flops of the leaves + brute planes/boxes
            brute = sum(FLOPS[k] for k in packed.kinds if k in ("plane", "box"))
            flops = 12 * nodes + FLOPS["sphere"] * sph + FLOPS["triangle"] * tri + seg_launch * brute
        else:
            flops = seg_launch * flops_per_segment
        rank_samples = cfg["w"] * cfg["h"] * (job.range[1] - job.range[0])
        traffic = load_traffic(args.config, args.precision)
        sq = load_sq(args.config, args.precision)
        issue = None
        if sq and world == 1:
            slots = sq["valu_issue_slots"]
            gslots = slots / (k_ms * 1e-3) / 1e9
            issue = {"valu_insts_per_launch": sq["counters"]["SQ_INSTS_VALU"], "issue_slots_per_launch": slots,
                     "achieved": round(gslots, 1), "peak": VALU_ISSUE_PEAK_GSLOTS,
                     "unit": "G issue slots/s (wave64 VALU instruction = 1 slot, binary64 = 2)",
                     "frac": round(gslots / VALU_ISSUE_PEAK_GSLOTS, 4),
                     "lane_utilization": round(sq["valu_lane_utilization"], 4),
                     "source": f"profiles/sq_{args.config}_{args.precision}.json (rocprofv3 SQ counters) / this run's kernel_ms"}
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic",
            "config": {"workload": f"config{cfg['cfg']}_{args.config}_{cfg['w']}x{cfg['h']}_{cfg['spp']}spp",
                       "scene": cfg["scene"], "width": cfg["w"], "height": cfg["h"], "spp": cfg["spp"],
                       "max_depth": cfg["depth"], "primitives": packed.primitives_per_segment(), "accel": args.accel,
                       "parallelism": f"sample-split x{world} + RCCL reduce" if world > 1 else "1 GPU"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": "trace_pool_kernel + accumulate_kernel (one launch each per frame)",
                         "kernel_ms": round(k_ms, 3),
                         "algorithmic_bytes_per_launch": a_bytes,
                         "definition": ("BVH: 64 B/node visited + 16 B/sphere + 36 B/triangle tested + segments x "
                                        "24 B/plane|box + 12 B/pixel" if bvh else
                                        "segments x sum(prim record bytes: sphere 16, plane 24, box 24, tri 36) "
                                        "+ 12 B/pixel (SURVEY 8d); served from SGPR/L1, not HBM"),
                         "bvh_nodes_per_segment": round(nodes / seg_launch, 3) if bvh else None,
                         "prim_tests_per_segment": round((sph + tri) / seg_launch, 3) if bvh else None},
            "valu": {"achieved": round(flops / (k_ms * 1e-3) / 1e12, 3), "peak": VALU_PEAK_TFLOPS[args.precision],
                     "unit": "TFLOP/s", "frac": round(flops / (k_ms * 1e-3) / 1e12 / VALU_PEAK_TFLOPS[args.precision], 4),
                     "flops_per_segment": round(flops / seg_launch, 2)},
            "valu_issue": issue,
            "segments_per_sample": round(seg_launch / rank_samples, 4),
            "kernel_msamples_per_s": round(rank_samples / (k_ms * 1e-3) / 1e6, 3),
            "cpu_baseline": cpu,
            "end_to_end": e2e,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
