"""Diagnose the progressive preview after a cancel (DEV TOOL): checkpoint sums and preview frame of a
cancelled render vs a render of exactly the checkpointed samples."""
import sys
import numpy as np
sys.path.insert(0, ".")
import torch  # noqa: F401
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json


def mk(spp):
    rt = GpuRayTracer(128, 72, seed=6)
    assert rt.load_from_json(load_scene_json("rtow.json"))
    rt.update_render_settings({"maxBounces": 5, "samples": spp})
    return rt


rt = mk(32)
calls = []
try:
    rt.render(want=("preview",), batch_samples=2, on_progress=lambda f: calls.append(f) or len(calls) >= 5)
except RuntimeError as e:
    print("cancelled:", e)
sums, done = rt.checkpoint()
prev = rt.image_data.copy()
print("done", done, "calls", calls)
rt2 = mk(done)
ref = rt2.render(batch_samples=2, want=("mean",))
s2, d2 = rt2.checkpoint()
print("sums equal", np.array_equal(sums, s2), "max rel", np.max(np.abs(sums - s2) / np.maximum(1e-300, np.abs(s2))))
print("preview == ref rgba8", np.array_equal(prev, ref["rgba8"]), "differing bytes", int(np.sum(prev != ref["rgba8"])))
# preview vs finalize of the checkpoint (host approximation of reinhard + gamma)
m = sums / done
g = np.power(np.maximum(0, m / (1 + m)), 1 / 2.2)
u8 = np.minimum(255, np.maximum(0, np.floor(g * 255))).astype(np.uint8)
print("preview vs host finalize(ckpt) differing bytes", int(np.sum(prev[..., :3] != u8)))
print("ref vs host finalize(ckpt2) differing bytes", int(np.sum(ref["rgba8"][..., :3] != u8)))
for k in range(8, 16, 2):
    s3 = mk(k).render(batch_samples=2)["rgba8"]
    print(f"preview vs render of {k} samples: {int(np.sum(prev != s3))} bytes differ")
