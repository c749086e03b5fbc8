"""Benchmark of the path-tracing hot path (BASELINE.json metric) on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config rtow|cornell|rtow4k|mesh50k|sample_scene]
                    [--precision f64|f32] [--no-cpu-baseline] [--no-end-to-end] [--no-pmc]
                    [--mp-mode ranks|inproc] [--dist-backend nccl|gloo] [--dump frame.npz]

A "step" renders one full frame of the workload: every pixel x every sample, traced on the GPU(s)
from a scene already resident in HBM, the per-pixel float64 sums RCCL-reduced to rank 0 (N>1), and
the epilogue (mean, tone map, gamma, RGBA8) run on rank 0's GPU.  Rank r traces samples
[r*S/N, (r+1)*S/N) of every pixel, so the frame is fixed as N grows ("scaling": "strong").

N > 1, two ways, both runnable as a plain `python bench.py --gpus N`:
  --mp-mode ranks (default): one process per GPU over torch.distributed (RCCL).  Under
      torch.distributed.run (WORLD_SIZE set) this process is one rank; without it, this process starts
      the N rank processes itself (before touching any GPU) and exits with rank 0's status.
  --mp-mode inproc: one process, rt_settings.devices = [0..N-1] — the split the Node drop-in ships
      (installGpuRender(rt, {devices})): replicas of the scene, whole sample batches round-robin over
      the devices, each batch's chunk partials copied over xGMI to device 0 and reduced there in batch
      order, the epilogue there; a step is one rt_render call delivering RGBA8 to the host.  The line
      also carries `progressive_16`: the same with the Node default of 16 progressive batches.

Prints ONE JSON line on rank 0 (driver contract).  The trace step's duration comes from HIP events
recorded inside librt_hip.so on the stream the kernels run on.  At N=1 (unless --no-pmc) rank 0 then
re-runs one frame of the same workload under rocprofv3 three times — FETCH_SIZE, WRITE_SIZE and eight
SQ counters, each pass in its own process — so `roofline` (measured HBM bytes, bound "hbm") and
`roofline_binding` (VALU issue slots and lane utilization, the resource that binds) are measured by
this run, at this commit.  `cpu_baseline` times the reference's JS CPU path (oracle/js/pt_cpu.mjs, bit-exact to the
reference's golden fixtures) under Node on this host at 1 thread and at the host's CPU share, plus
the C port, each on a bounded crop of the same workload.
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
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 counter passes (N=1 roofline)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mp-mode", default="ranks", choices=["ranks", "inproc"],
                    help="N>1: one process per GPU (torch.distributed) or one process over rt_settings.devices")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks on fewer GPUs (rank -> device LOCAL_RANK %% device count, sums "
                         "reduced through host memory); never a measurement")
    ap.add_argument("--bands", type=int, default=0,
                    help="ranks mode: reduce the sums band by band as the bands complete (rt_trace_device_bands); "
                         "0 (default): one reduce after the trace (DESIGN.md §6: the one-GPU rehearsal measured the "
                         "banded trace 1.1 %% slower, and the RCCL kernels cannot run beside the persistent trace waves)")
    ap.add_argument("--dump", help="rank 0 writes the frame's float64 sums and RGBA8 here (.npz) after the timed steps")
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


# JS CPU baseline crops (side of the centred square crop, at full resolution, spp and depth): about
# 10 s for one thread; the multi-thread run renders a crop twice the side.  Config 1 (the
# reference's own CPU-runnable case) is timed on its whole 256x256 frame.
JS_CROP = {"sample_scene": 256, "cornell": 48, "rtow": 32, "rtow4k": 24, "mesh50k": 4}


def js_cpu_baseline(cfg_name, cfg, seed, workers, side):
    """The reference's JS CPU path (oracle/js/pt_cpu.mjs, bit-exact to the reference on every golden
    fixture) under Node on this host: `workers` worker_threads over row bands of a centred crop."""
    import shutil
    import subprocess
    import tempfile
    node = shutil.which("node")
    if node is None:
        return {"error": "node not found"}
    w, h = cfg["w"], cfg["h"]
    side = min(side, w, h)
    x0, y0 = (w - side) // 2, (h - side) // 2
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(load_scene_json(cfg["scene"]), f)
        path = f.name
    try:
        args = dict(scene=path, width=w, height=h, spp=cfg["spp"], depth=cfg["depth"], seed=seed,
                    crop=[x0, y0, side, side], workers=workers)
        r = subprocess.run([node, os.path.join(ROOT, "oracle", "js", "cpu_tool.mjs"), "bench", json.dumps(args)],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            return {"error": r.stderr[-300:]}
        out = json.loads(r.stdout)
    finally:
        os.unlink(path)
    return {"value": round(out["msamples_per_s"], 6), "unit": "Msamples/s", "cores": out["workers"],
            "nproc": out["nproc"], "kind": "js",
            "sample": f"{side}x{side} crop at ({x0},{y0}) of the {w}x{h} frame, {cfg['spp']} spp, maxDepth "
                      f"{cfg['depth']}: {out['samples']} samples in {out['render_s']:.1f} s (slowest worker; {out['wall_s']:.1f} s wall with worker start-up) (oracle/js/pt_cpu.mjs "
                      f"under Node {out['node']}, {out['workers']} worker thread(s) over interleaved rows)"}


def cpu_baseline(rt, cfg_name, cfg, seed, side):
    """CPU baselines on this host: the JS CPU path at 1 thread (the reference's own model: one Node
    event loop) and at the host's CPU share, plus the C port (oracle/pt_oracle.c, 1 thread)."""
    from oracle import binding
    js_side = JS_CROP.get(cfg_name, 32)
    one = js_cpu_baseline(cfg_name, cfg, seed, 1, js_side)
    ncores = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS") or (os.cpu_count() or 1)))
    many = js_cpu_baseline(cfg_name, cfg, seed, ncores, 2 * js_side)
    w, h = cfg["w"], cfg["h"]
    side = min(side, w, h)
    x0, y0 = (w - side) // 2, (h - side) // 2
    st = rt.settings(crop=(x0, y0, side, side))
    binding.lib()
    t = time.perf_counter()
    binding.render(rt.packed(), st)
    dt = time.perf_counter() - t
    samples = side * side * st.samples
    port = {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"{side}x{side} crop at ({x0},{y0}) of the {w}x{h} frame, {st.samples} spp, "
                      f"maxDepth {cfg['depth']}: {samples} samples in {dt:.1f} s (oracle/pt_oracle.c, 1 thread)"}
    res = dict(one) if "error" not in one else dict(port)
    res["js_multi_core"] = many
    res["c_port"] = port
    return res


# VALU issue ceiling: 256 CUs x 4 SIMD-32s, a wave64 VALU instruction holds its SIMD for 2 cycles (a
# binary64 one for 4: FP64 vector is half the FP32 rate) at 2.4 GHz (MI355X_MICROARCH.md)
VALU_ISSUE_PEAK_GSLOTS = 256 * 4 * 2.4 / 2
# the trace step: one launch each per frame ("trace_pool": trace_pool_kernel, or trace_pool_lds_kernel for
# binary32 sphere scenes)
TRACE_KERNELS = ("trace_pool", "reduce_kernel")
# the vector-memory data path (TA address / TD data units, vector L1 = TCP, L2 = TCC): TA 1 of 2, TD 1 of 2,
# TCP 2 of 4, TCC 2 of 4, GRBM 1 of 2 counters per pass
VMEM_COUNTERS = ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum",
                 "TCC_HIT_sum", "TCC_MISS_sum", "GRBM_GUI_ACTIVE")
SQ_COUNTERS = ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_INSTS_VALU_ADD_F64",
               "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


# Instruction-floor model: the VALU issue slots per segment that the
# reference's arithmetic needs (wave64 binary32 / integer VALU instruction = 1 slot, binary64 = 2, as
# VALU_ISSUE_PEAK_GSLOTS counts them), from the events the kernel's own code performs per segment (counted
# on the CPU, tests/hostcheck RT_HCOUNT) and a per-event cost in gfx950 instructions: binary64 sqrt =
# the 20-instruction v_rsq_f64 + Newton expansion (~32 slots), binary64 division = v_div_scale x2 /
# v_rcp / 5 FMA / v_div_fmas / v_div_fixup (~22 slots).  Addressing, loop control and lane bookkeeping
# are not counted: this is the arithmetic floor, at lane utilization 1.
FLOOR_COST = {
    "walk_step_grid": 12,       # 3D-DDA cell step, binary32 (pt_core.h closest_hit_grid)
    "walk_step_bvh": 24,        # two-child node: 6 packed FMA slab planes + min/max + child choice (binary32)
    "filter_tests": 12,         # binary32 sphere pre-filter (pt_core.h sphere_filter_pass)
    "f64_sphere_tests": 36,     # oc, halfB, c, discriminant: 17 binary64 ops + compare (geometry.js:16-22)
    "disc_nonneg": 58,          # sqrt + (-halfB - sqrtd) / a + tMin test (geometry.js:24-26)
    "second_root": 26,          # (-halfB + sqrtd) / a + test (geometry.js:27-28)
    "tri_filter_tests": 52,     # binary32 triangle pre-filter: 21 FMA-chain ops + bounds + 6 tests (pt_core.h)
    "tri_tests": 102,           # Moller-Trumbore: 2 cross, 4 dot, 1 division (geometry.js:148-188)
    "plane_tests": 50,          # dot, (p - o).n / denom (geometry.js:56-74)
    "box_tests": 150,           # six divisions + slab logic (geometry.js:85-117)
    "hit": 100,                 # ray.at(t), (p - c) / radius (3 divisions), setFaceNormal (math.js:41,55-58)
    "segment": 108,             # one normalize per segment: length (sqrt) + 3 divisions (math.js:18)
    "lambertian": 12,           # n + unit, attenuation (materials.js:20-25)
    "metal": 54,                # reflect + fuzz * p + dot test (materials.js:36-41)
    "dielectric": 118,          # ratio, cos, sin (sqrt), refract/reflect (materials.js:51-83)
    "dielectric_schlick": 68,   # r0, pow5 (10 binary64 ops), draw and compare (materials.js:79-83)
    "emissive": 6,              # emission x throughput (materials.js:87-96)
    "miss": 34,                 # skyGradient x intensity x throughput (world.js:35-44)
    "sphere_draw_rounds": 45,   # 3 keyed draws + integer |p|^2 < 1 test (math.js:22-26)
    "disk_draw_rounds": 30,     # 2 keyed draws + integer test (math.js:27-31)
    "samples": 151,             # sample key, 2 AA draws, (i + r) / width x 2, camera ray (camera.js:38-51)
}


def instruction_floor(rt, cfg, side=32, spp=8):
    """The instruction floor of the workload (FLOOR_COST over the kernel's events per segment on three
    crops of the frame at `spp`, counted on the CPU by the kernel's own code)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    import hostcheck_binding as hb
    packed = rt.packed()
    n3, regs, use_grid = (ctypes.c_int * 3)(), ctypes.c_longlong(), ctypes.c_int()
    hb.lib().ptc_grid_info(ctypes.byref(packed.desc), n3, ctypes.byref(regs), ctypes.byref(use_grid))
    prims = sum(o.count if k in ("mesh", "triangle") else 1 if k == "sphere" else 0
                for k, o in zip(packed.kinds, packed.objects))
    walk = "grid" if use_grid.value else ("bvh" if prims >= 8 else "brute")
    w, h = cfg["w"], cfg["h"]
    sts = []
    for fx, fy in ((0.5, 0.5), (0.25, 0.7), (0.75, 0.3)):
        st = rt.settings(crop=(int(fx * (w - side)), int(fy * (h - side)), side, side))
        st.samples = spp
        sts.append(st)
    ev = hb.event_counts(packed, sts, walk)
    ev["plane_tests"] = float(sum(1 for k in packed.kinds if k == "plane"))
    ev["box_tests"] = float(sum(1 for k in packed.kinds if k == "box"))
    ev["hit"] = 1.0 - ev["miss"]
    ev["segment"] = 1.0
    ev["walk_step_" + ("grid" if walk == "grid" else "bvh")] = ev["walk_steps"] if walk != "brute" else 0.0
    slots = {k: FLOOR_COST[k] * ev.get(k, 0.0) for k in FLOOR_COST}
    return {"walk": walk, "events_per_segment": {k: round(v, 4) for k, v in ev.items()},
            "lane_slots_per_segment": round(sum(slots.values()), 1),
            "lane_slots_by_event": {k: round(v, 1) for k, v in slots.items() if v},
            "sample": f"3 crops of {side}x{side} at {spp} spp, the kernel's code on the CPU (tests/hostcheck RT_HCOUNT)"}


def pmc_child(args):
    """--pmc-child: one frame of the workload through rt_render (the same trace launches as a bench
    step), run under rocprofv3 --pmc by pmc_passes()."""
    rt = make_tracer(CONFIGS[args.config], args.precision, args.seed, 0, args.accel)
    rt.render()
    rt.close()


def pmc_passes(args, outdir):
    """rocprofv3 --pmc passes (one counter group per process, as MI355X_MICROARCH.md prescribes) over
    one frame; returns {counter: value summed over the trace step's kernels} per pass, or an error."""
    import csv
    import glob
    import shutil
    import subprocess
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    child = [sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", args.config, "--precision",
             args.precision, "--seed", str(args.seed), "--accel", args.accel]
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    res = {}
    for name, counters in (("fetch", ("FETCH_SIZE",)), ("write", ("WRITE_SIZE",)), ("sq", SQ_COUNTERS),
                           ("vmem", VMEM_COUNTERS)):
        d = os.path.join(outdir, name)
        cmd = ["timeout", "-s", "KILL", "240", prof, "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run",
               "--", *child]
        r = subprocess.run(cmd, capture_output=True, text=True, env=env)
        if r.returncode != 0:
            return {"error": f"{name} pass exit {r.returncode}: {r.stderr[-300:]}"}
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            return {"error": f"{name} pass wrote no counter_collection.csv"}
        tot, per_kernel, names = {}, {}, []
        for row in csv.DictReader(open(files[0])):
            k = next((k for k in TRACE_KERNELS if k in row["Kernel_Name"]), None)
            if k is None:
                continue
            if row["Kernel_Name"] not in names:
                names.append(row["Kernel_Name"])
            v = float(row["Counter_Value"])
            tot[row["Counter_Name"]] = tot.get(row["Counter_Name"], 0.0) + v
            per_kernel.setdefault(k, {})
            per_kernel[k][row["Counter_Name"]] = per_kernel[k].get(row["Counter_Name"], 0.0) + v
        res[name] = {"total": tot, "per_kernel": per_kernel, "names": names, "csv": os.path.relpath(files[0], ROOT)}
    return res


def node_end_to_end(cfg, args):
    """The Node drop-in end to end (scripts/node_e2e.mjs): GpuRayTracer.render() through rt_napi.node,
    scene resident from the first call, timed on the second."""
    import shutil
    import subprocess
    import tempfile
    node = shutil.which("node")
    if node is None or not os.path.exists(os.path.join(ROOT, "blenderraytracer_amd", "lib", "rt_napi.node")):
        return {"error": "node or rt_napi.node not available"}
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(load_scene_json(cfg["scene"]), f)
        path = f.name
    try:
        a = dict(scene=path, width=cfg["w"], height=cfg["h"], spp=cfg["spp"], depth=cfg["depth"], seed=args.seed,
                 precision=args.precision)
        r = subprocess.run([node, os.path.join(ROOT, "scripts", "node_e2e.mjs"), json.dumps(a)], capture_output=True,
                           text=True, timeout=600)
        if r.returncode != 0:
            return {"error": r.stderr[-300:]}
        out = json.loads(r.stdout)
    finally:
        os.unlink(path)
    return {"value": round(out["value"], 3), "unit": "Msamples/s", "wall_ms": round(out["wall_ms"], 3),
            "walls_ms": [round(w, 3) for w in out["walls_ms"]], "reps": out["reps"],
            "first_call_ms": round(out["first_call_ms"], 3), "kernel_ms": round(out["kernel_ms"], 3),
            "rt_render_wall_ms": round(out["rt_render_wall_ms"], 3),
            "progress_calls": out["progress_calls"], "no_preview_wall_ms": round(out["no_preview_wall_ms"], 3),
            "one_batch_wall_ms": round(out["one_batch_wall_ms"], 3), "one_batch_kernel_ms": round(out["one_batch_kernel_ms"], 3),
            "what": "GpuRayTracer.render() from Node (the installGpuRender path): scene resident from the first call "
                    "(first_call_ms includes its upload and BVH build), pack + compare, trace in 16 progressive "
                    "sample batches (onProgress + the running frame in imageData after each), epilogue, RGBA8 "
                    "into imageData (what the reference's render() produces); median of `reps` after a warm-up; "
                    "no_preview / one_batch: the same frame without preview frames / as one sample batch"}


def build_provenance():
    """The commit / source digest librt_hip.so was built from (lib/build_info.json, written by the build)
    and whether the sources in this tree still hash the same (the GPU box has no .git)."""
    from blenderraytracer_amd import build as B
    info = B.read_build_info() or {}
    tree = B.source_digest()
    return {"commit": info.get("commit"), "sources_modified_at_build": info.get("sources_modified"),
            "library_source_digest": info.get("source_digest"), "tree_source_digest": tree,
            "library_matches_tree": info.get("source_digest") == tree}


def spawn_ranks(args):
    """`python bench.py --gpus N` without a launcher: start N rank processes (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* in their environment, as torch.distributed.run sets them) and wait for them.
    This process never touches a GPU (it only starts children); it exits with the first failing rank's
    status, stopping the other ranks (by their own PIDs) if one fails."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    status = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            rc = p.poll()
            if rc is None:
                continue
            pending.remove(p)
            if rc != 0 and status == 0:
                status = rc
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return status


def main():
    args = parse()
    if args.pmc_child:
        return pmc_child(args)
    cfg = CONFIGS[args.config]
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.mp_mode == "ranks":
        raise SystemExit(spawn_ranks(args))
    inproc = args.gpus > 1 and args.mp_mode == "inproc"
    # under torch.distributed.run (WORLD_SIZE set) the process group is up at every world size, 1
    # included: the sums then go through the RCCL reduce even on one GPU (tests/test_gpu_parity.py)
    distributed = not inproc and "WORLD_SIZE" in os.environ
    world = 1 if inproc else int(os.environ.get("WORLD_SIZE", "1"))
    rank = 0 if inproc else int(os.environ.get("RANK", "0"))
    local = 0 if inproc else int(os.environ.get("LOCAL_RANK", "0"))
    if not inproc and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if args.dist_backend == "gloo":
        local %= ndev
    torch.cuda.set_device(local)
    if distributed:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    rt = make_tracer(cfg, args.precision, args.seed, local, args.accel)
    packed = rt.packed()
    flops_per_segment = sum(FLOPS[k] * (o.count if k in ("mesh", "triangle") else 1)
                            for k, o in zip(packed.kinds, packed.objects))

    cpu = None
    if rank == 0 and args.gpus == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(rt, args.config, cfg, args.seed, args.cpu_crop)

    inproc_devices = [k % ndev for k in range(args.gpus)] if inproc else None
    if inproc:
        from blenderraytracer_amd.distributed import InProcessRender
        job = InProcessRender(rt, inproc_devices)
    else:
        job = ShardedRender(rt, rank=rank, world=world, device=torch.device("cuda", local), bands=args.bands)
    for _ in range(args.warmup):
        job.step()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    # ranks: no host synchronization inside a timed step — the trace's duration comes from HIP events
    # recorded around it on the stream it runs on (torch's current stream, handed to rt_trace_device);
    # inproc: rt_render is synchronous and reports its own HIP-event time
    kernel_ms = []
    events = [] if inproc else [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                                for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        if inproc:
            job.step()
            kernel_ms.append(job.stats.kernel_ms)
        else:
            job.step(stats=False, events=events[k])
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not inproc:
        kernel_ms = [a.elapsed_time(b) for a, b in events]
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if args.dist_backend == "nccl" else "cpu")
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    # the work counters of the frame (identical in every step): one more, untimed step with stats
    job.step()
    torch.cuda.synchronize()
    segs, abytes = [job.stats.segments], [job.stats.algorithmic_bytes]
    work = [(job.stats.node_visits, job.stats.sphere_tests, job.stats.tri_tests)]
    progressive = None
    if inproc:
        # the Node drop-in's default: 16 progressive batches with a running frame and a progress call
        # after each (gpu-ray-tracer.mjs DEFAULT_PROGRESS_STEPS), timed over the same number of steps
        from blenderraytracer_amd.distributed import InProcessRender
        pj = InProcessRender(rt, inproc_devices, progress_steps=16)
        pj.step()
        tp = time.perf_counter()
        for _ in range(args.steps):
            pj.step()
        pt = time.perf_counter() - tp
        progressive = {"value": round(cfg["w"] * cfg["h"] * rt.settings().samples * args.steps / pt / 1e6, 3),
                       "unit": "Msamples/s", "ms_per_step": round(pt / args.steps * 1e3, 3), "batches": 16,
                       "batch_samples": pj.batch, "progress_calls_per_step": pj.progress_calls // (args.steps + 1),
                       "what": "rt_render with rt_settings.devices as the Node drop-in ships it: 16 sample batches "
                               "dealt round-robin to the devices, the running frame into a preview buffer and a "
                               "progress callback after each batch"}
    if args.dump and rank == 0:
        import numpy as np
        torch.cuda.synchronize()
        if inproc:      # rt_render's checkpoint holds the frame's merged float64 sums
            sums, done = rt.checkpoint()
            np.savez(args.dump, sum=sums.reshape(-1), rgba8=job.rgba8, samples=done)
        else:
            np.savez(args.dump, sum=job.sum.cpu().numpy(), rgba8=job.rgba8.cpu().numpy(), samples=job.samples)

    e2e = e2e_node = None
    if rank == 0 and args.gpus == 1 and not args.no_end_to_end:
        # RayTracer.render as the drop-in boundary runs it (rt_render): sums zeroed on device, the
        # trace, the epilogue, Float32 post-gamma + RGBA8 frames copied back over PCIe
        rt.render()
        t1 = time.perf_counter()
        rt.render()
        wall = time.perf_counter() - t1
        e2e = {"value": round(cfg["w"] * cfg["h"] * rt.settings().samples / wall / 1e6, 3), "unit": "Msamples/s",
               "wall_ms": round(wall * 1e3, 3), "kernel_ms": round(rt.last_stats.kernel_ms, 3),
               "what": "one rt_render call from Python: trace + tone map/gamma/RGBA8 + Float32 and RGBA8 readback"}
        e2e_node = node_end_to_end(cfg, args)

    if rank == 0:
        total_samples = cfg["w"] * cfg["h"] * rt.settings().samples * args.steps
        value = total_samples / elapsed / 1e6
        k_ms = sum(kernel_ms) / len(kernel_ms)
        a_bytes = sum(abytes) / len(abytes)
        seg_launch = sum(segs) / len(segs)
        nodes, sph, tri = (sum(w[k] for w in work) / len(work) for k in range(3))
        bvh = nodes > 0
        if bvh:   # BVH: slab test 12 flops/node + per-test flops of the leaves + brute planes/boxes
            brute = sum(FLOPS[k] for k in packed.kinds if k in ("plane", "box"))
            flops = 12 * nodes + FLOPS["sphere"] * sph + FLOPS["triangle"] * tri + seg_launch * brute
        else:
            flops = seg_launch * flops_per_segment
        rank_samples = cfg["w"] * cfg["h"] * (job.range[1] - job.range[0])
        # the walk this render ran (rt_scene_walk): BVH nodes or grid cells are its walk steps
        walk = {0: "world_order", 1: "bvh", 2: "uniform_grid"}.get(
            capi.load_library().rt_scene_walk(rt.scene_handle(), capi.RT_PREC_F32 if args.precision == "f32" else capi.RT_PREC_F64,
                                              {"auto": capi.RT_ACCEL_AUTO, "brute": capi.RT_ACCEL_BRUTE, "bvh": capi.RT_ACCEL_BVH}[args.accel]),
            "error")
        kernel_desc = ("trace step of the " + walk + " walk: " +
                       ("trace_pool_lds_kernel (the grid's cell offsets and filters in LDS, when they fit)"
                        if walk == "uniform_grid" else "trace_pool_kernel / trace_pool_lds_kernel") +
                       " + reduce_kernel, one launch each per frame; the counter pass names the kernels it saw")
        roofline = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                    "traffic": None, "kernel": kernel_desc, "kernel_ms": round(k_ms, 3)}
        binding = vmem = None
        if args.gpus == 1 and not args.no_pmc:
            import tempfile
            keep = os.environ.get("BENCH_PMC_KEEP")      # scripts/profile_round.sh keeps the counter CSVs
            if keep:
                pmc = pmc_passes(args, keep)
            else:
                with tempfile.TemporaryDirectory(prefix="bench_pmc_", dir=os.environ.get("TMPDIR", "/tmp")) as d:
                    pmc = pmc_passes(args, d)
            if "error" in pmc:
                roofline["pmc_error"] = pmc["error"]
            else:
                roofline["kernel"] = " + ".join(pmc["fetch"]["names"]) + " (the kernels the counter passes saw)"
                fetch = 2.0 * pmc["fetch"]["total"].get("FETCH_SIZE", 0.0) * 1024   # gfx950: x2, KiB
                write = pmc["write"]["total"].get("WRITE_SIZE", 0.0) * 1024
                hbm = fetch + write
                gbs = hbm / (k_ms * 1e-3) / 1e9
                roofline.update({"achieved": round(gbs, 3), "frac": round(gbs / HBM_PEAK_GBS, 6), "traffic": hbm,
                                 "traffic_read": fetch, "traffic_write": write,
                                 "counters_per_kernel": {k: {**pmc["fetch"]["per_kernel"].get(k, {}),
                                                             **pmc["write"]["per_kernel"].get(k, {})}
                                                         for k in TRACE_KERNELS},
                                 "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes over one "
                                           "frame run by this bench invocation (FETCH x2 per the gfx950 correction, "
                                           "KiB x1024) / this run's HIP-event trace-step time",
                                 "commit": build_provenance()["commit"]})
                sq = pmc["sq"]["total"]
                f64 = sum(sq.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
                slots = sq.get("SQ_INSTS_VALU", 0.0) + f64
                gslots = slots / (k_ms * 1e-3) / 1e9
                binding = {"bound": "valu_issue", "achieved": round(gslots, 1), "peak": VALU_ISSUE_PEAK_GSLOTS,
                           "unit": "G issue slots/s (wave64 VALU instruction = 1 slot, binary64 = 2)",
                           "frac": round(gslots / VALU_ISSUE_PEAK_GSLOTS, 4),
                           "lane_utilization": round(sq["SQ_THREAD_CYCLES_VALU"] / (64.0 * sq["SQ_ACTIVE_INST_VALU"]), 4)
                           if sq.get("SQ_ACTIVE_INST_VALU") else None,
                           "valu_insts_per_launch": sq.get("SQ_INSTS_VALU"), "f64_insts_per_launch": f64,
                           "waves_per_launch": sq.get("SQ_WAVES"),
                           "source": "rocprofv3 --pmc SQ_* pass over one frame run by this bench invocation / this "
                                     "run's HIP-event trace-step time"}
                vm = pmc["vmem"]["per_kernel"].get("trace_pool", {})
                grbm = vm.get("GRBM_GUI_ACTIVE", 0.0)
                cu_cycles = 256 * grbm / 8       # rocprofv3's GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles
                if cu_cycles > 0:
                    acc = vm.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0)
                    hit, miss = vm.get("TCC_HIT_sum", 0.0), vm.get("TCC_MISS_sum", 0.0)
                    vmem = {"bound": "vector_memory", "kernel": "trace_pool_kernel / trace_pool_lds_kernel",
                            "td_busy": round(vm.get("TD_TD_BUSY_sum", 0.0) / cu_cycles, 4),
                            "ta_busy": round(vm.get("TA_TA_BUSY_sum", 0.0) / cu_cycles, 4),
                            "l1_hit": round(1 - vm.get("TCP_TCC_READ_REQ_sum", 0.0) / acc, 4) if acc else None,
                            "l2_hit": round(hit / (hit + miss), 4) if hit + miss else None,
                            "clock_ghz": round(grbm / 8 / (k_ms * 1e-3) / 1e9, 3),
                            "counters": vm,
                            "definition": "TA/TD busy cycles summed over the 256 CUs / (256 x GRBM_GUI_ACTIVE / 8): "
                                          "rocprofv3's GRBM_GUI_ACTIVE is the sum over the 8 XCDs "
                                          "(MI355X_MICROARCH.md); l1_hit = 1 - TCP_TCC_READ_REQ / TCP accesses",
                            "source": "rocprofv3 --pmc pass over one frame run by this bench invocation"}
        floor = None
        if args.gpus == 1:
            try:
                floor = instruction_floor(rt, cfg)
                fl_ms = seg_launch * floor["lane_slots_per_segment"] / 64.0 / (VALU_ISSUE_PEAK_GSLOTS * 1e9) * 1e3
                floor.update({"floor_ms": round(fl_ms, 3), "kernel_ms": round(k_ms, 3), "frac": round(fl_ms / k_ms, 4),
                              "peak": VALU_ISSUE_PEAK_GSLOTS, "unit": "G issue slots/s at lane utilization 1",
                              "definition": "the reference arithmetic's VALU issue slots (FLOOR_COST x the kernel's "
                                            "events per segment) x this frame's segments / 64 lanes / peak; frac = "
                                            "floor_ms / the measured trace-step time"})
            except Exception as e:      # the host-check library is test infrastructure: report, do not fail
                floor = {"error": f"{type(e).__name__}: {e}"}
            if binding is not None:
                binding["floor"] = floor
        roofline.update({
            "cache_served_bytes": a_bytes,
            "cache_served_GBps": round(a_bytes / (k_ms * 1e-3) / 1e9, 2),
            "algorithmic_frac": round(a_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_frac_definition": "cache_served_GBps / 8000: the SURVEY 8d bytes of the work done, served "
                                           "from LDS/L1/L2, NOT HBM traffic (that is `frac`)",
            "cache_served_definition": ("SURVEY 8d algorithmic bytes, BVH form: 64 B/node visited (8 B/cell for the "
                                        "uniform-grid walk) + 16 B/sphere + 36 B/triangle tested + segments x 24 "
                                        "B/plane|box + 12 B/pixel; read from L1/L2 (the trees are cache-resident), "
                                        "not HBM" if bvh else
                                        "SURVEY 8d algorithmic bytes: segments x sum(prim record bytes: sphere 16, "
                                        "plane 24, box 24, tri 36) + 12 B/pixel; scalar (SGPR) loads, not HBM"),
            "walk": walk,
            "walk_steps_per_segment": round(nodes / seg_launch, 3) if bvh else None,
            "prim_tests_per_segment": round((sph + tri) / seg_launch, 3) if bvh else None})
        if distributed:
            mp_mode = {"mode": "ranks", "world_size": dist.get_world_size(), "backend": dist.get_backend(),
                       "launcher": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ else "bench.py spawn",
                       "reduce_bands": job.bands}
            parallelism = (f"sample-split x{world} + RCCL reduce" if args.dist_backend == "nccl" and world > 1 else
                           "1 GPU, RCCL reduce at world size 1" if args.dist_backend == "nccl" else
                           f"REHEARSAL sample-split x{world} over {ndev} GPU(s), gloo host reduce: not a measurement")
        elif inproc:
            mp_mode = {"mode": "inproc", "devices": inproc_devices}
            parallelism = (f"in-process whole-batch split x{args.gpus} (rt_settings.devices {inproc_devices}: batch k "
                           "on device k % N, chunk partials copied over xGMI and reduced in batch order on device 0)" +
                           ("" if len(set(inproc_devices)) == args.gpus else
                            f": REHEARSAL on {ndev} GPU(s), not a measurement"))
        else:
            mp_mode = None
            parallelism = "1 GPU"
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": args.gpus,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic",
            "config": {"workload": f"config{cfg['cfg']}_{args.config}_{cfg['w']}x{cfg['h']}_{cfg['spp']}spp",
                       "scene": cfg["scene"], "width": cfg["w"], "height": cfg["h"], "spp": cfg["spp"],
                       "max_depth": cfg["depth"], "primitives": packed.primitives_per_segment(), "accel": args.accel,
                       "parallelism": parallelism},
            "mp_mode": mp_mode,
            "progressive_16": progressive,
            "roofline": roofline,
            "roofline_binding": binding if binding is not None else ({"floor": floor} if floor else None),
            "roofline_vmem": vmem,
            "valu_flops": {"achieved": round(flops / (k_ms * 1e-3) / 1e12, 3), "peak": VALU_PEAK_TFLOPS[args.precision],
                           "unit": "TFLOP/s", "frac": round(flops / (k_ms * 1e-3) / 1e12 / VALU_PEAK_TFLOPS[args.precision], 4),
                           "flops_per_segment": round(flops / seg_launch, 2),
                           "definition": "SURVEY 8d canonical flops (12/node, 23/sphere, 51/triangle test)"},
            "segments_per_sample": round(seg_launch / rank_samples, 4),
            "kernel_msamples_per_s": round(rank_samples / (k_ms * 1e-3) / 1e6, 3),
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "end_to_end_node": e2e_node,
            "build": build_provenance(),
        }
        print(json.dumps(line), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
