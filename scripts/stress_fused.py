"""Fused-batch stress (DEV TOOL): many progressive renders with random batch sizes, previews and random
cancels (a quarter of them 1080p, where the pool's chunk rule matters); every finished render must equal
the same render in one batch up to the pool's summation order (SUM_RTOL), every cancelled one must leave a checkpoint that resumes to the uninterrupted sums
bit for bit.  A third of the renders deal their batches to devices=[0, 0] or [0, 0, 0] (the whole-batch
split, one fused launch per device since round 5; bit-identical to one device).
usage: python scripts/stress_fused.py [renders]"""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402
from blenderraytracer_amd.renderer import GpuRayTracer  # noqa: E402
from blenderraytracer_amd.scene import load_scene_json  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rnd = random.Random(5)
scenes = {name: load_scene_json(name) for name in ("rtow.json", "cornell.json", "mesh50k")}
t0 = time.time()
bad = 0
for i in range(n):
    name = rnd.choice(list(scenes))
    w, h = rnd.choice([(160, 90), (320, 180), (96, 64), (1920, 1080)])
    # 1080p: >= 64k pool items, where the chunk rule leaves its floor of 4 samples, so a resume's chunks
    # differ unless they follow the whole render's rule (round 5's one-batch-left bug)
    spp = rnd.choice([8, 12, 24, 32]) if w < 1920 else rnd.choice([24, 32, 48])
    batch = rnd.choice([1, 2, 3, 4, 5, 8]) if w < 1920 else rnd.choice([8, 12, 16])
    rt = GpuRayTracer(w, h, seed=i)
    assert rt.load_from_json(scenes[name])
    rt.update_render_settings({"samples": spp, "maxBounces": 5})
    ref = rt.render(want=("mean",), batch_samples=batch)["mean"]          # fused (or not) progressive
    devices = rnd.choice([None, None, [0, 0], [0, 0, 0]])
    if devices:
        # the whole-batch split deals batches of min(batch, ceil(spp / N)) samples (rt_capi.cpp): the same
        # sums bit for bit as those batches on one device
        batch = min(batch, -(-spp // len(devices)))
        ref = rt.render(want=("mean",), batch_samples=batch)["mean"]
        split = rt.render(want=("mean",), batch_samples=batch, devices=devices)["mean"]
        if not np.array_equal(split, ref, equal_nan=True):
            bad += 1
            print(f"render {i}: {name} {w}x{h} spp {spp} batch {batch} devices {devices}: split != one device", flush=True)
    calls = []
    stop_at = rnd.randint(1, max(1, spp // batch))
    try:
        rt.render(want=("mean", "preview"), batch_samples=batch, devices=devices,
                  on_progress=lambda f: calls.append(f) or len(calls) >= stop_at)
        cancelled = False
    except RuntimeError as e:
        cancelled = "CANCELLED" in str(e)
        if not cancelled:
            raise
    if cancelled:
        sums, done = rt.checkpoint()
        res = rt.render(want=("mean",), batch_samples=batch, resume=(sums, done), devices=devices)["mean"]
        ok = np.array_equal(res, ref, equal_nan=True)
    else:
        ok = True
    if not ok:
        bad += 1
        print(f"render {i}: {name} {w}x{h} spp {spp} batch {batch}: resumed != uninterrupted", flush=True)
    rt.close()
    if i % 20 == 0:
        print(f"{i} renders, {time.time() - t0:.1f} s, {bad} bad", flush=True)
print(f"done: {n} renders, {bad} bad, {time.time() - t0:.1f} s", flush=True)
sys.exit(1 if bad else 0)
