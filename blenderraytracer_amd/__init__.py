"""MI355X-native backend for the per-pixel path-tracing loop of Shinzef/BlenderRayTracer.

Layout:
  csrc/          HIP kernels for gfx950 + the extern "C" ABI (include/rt_hip.h) + the N-API addon
  js/            Node host: GpuRayTracer drop-in for RayTracer.render, keyed RNG, scene packer
  capi.py        ctypes mirror of include/rt_hip.h (loads lib/librt_hip.so, no CPU fallback)
  scene.py       scene-JSON semantics (js/scene-loader.js, js/camera.js) -> rt_scene_desc
  renderer.py    GpuRayTracer, the Python twin of the RayTracer surface
  distributed.py sample-range sharding over ranks + RCCL reduce of the per-pixel sums
  build.py       hipcc build of librt_hip.so and the N-API addon
"""
from . import capi  # noqa: F401
from .renderer import GpuRayTracer, settings_struct  # noqa: F401
