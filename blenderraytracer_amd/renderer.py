"""GpuRayTracer — Python mirror of the reference's RayTracer surface (js/ray-tracer.js), rendering
through librt_hip.so.  The JS twin for Node lives in blenderraytracer_amd/js/gpu-ray-tracer.mjs.

Mirrored members: width/height, maxBounces/samples/gamma/exposure/toneMapping/antiAliasing/denoising
(defaults ray-tracer.js:23-33), load_from_json (:305-334), update_render_settings (:554-566),
update_background (:568-585), resize_canvas (:598-614), render(on_progress) (:166-281) -> image_data.
Randomness: Math.random is replaced by the keyed RNG; `seed` selects the stream.
"""
import ctypes as C

import numpy as np

from . import capi
from .jsmath import js_exp
from .scene import PackedScene, default_scene, load_from_json, setup_camera, keyed_permutation, js_or, truthy


def settings_struct(width, height, samples, max_bounces, anti_aliasing, tone_mapping, exposure, gamma, seed,
                    crop=None, precision=capi.RT_PREC_F64, sample_range=None, batch_samples=0, denoising=False,
                    denoise_strength=0.5, accel=capi.RT_ACCEL_AUTO, devices=None, sum_order=capi.RT_SUM_POOL):
    """rt_settings from RayTracer fields, resolving sampleCount (ray-tracer.js:201) and the string
    switches of getAntiAliasSample (:125-149) and toneMap (:151-161)."""
    s = capi.Settings()
    s.width, s.height = int(width), int(height)
    s.samples = 1 if anti_aliasing == "none" else int(samples)
    s.max_depth = int(max_bounces)
    s.aa_mode = {"stochastic": capi.RT_AA_STOCHASTIC, "supersampling": capi.RT_AA_SUPERSAMPLING}.get(
        anti_aliasing, capi.RT_AA_CENTER)
    s.tone_map = {"aces": capi.RT_TM_ACES, "linear": capi.RT_TM_LINEAR}.get(tone_mapping, capi.RT_TM_REINHARD)
    s.exposure, s.gamma = float(exposure), float(gamma)
    s.seed = int(seed) & 0xFFFFFFFF
    if sample_range is not None:
        s.sample_begin, s.sample_end = int(sample_range[0]), int(sample_range[1])
    if crop is not None:
        s.crop_x0, s.crop_y0, s.crop_w, s.crop_h = (int(v) for v in crop)
    s.precision = int(precision)
    s.batch_samples = int(batch_samples)
    s.accel = int(accel)
    s.sum_order = int(sum_order)
    if devices:                 # multi-GPU sample split (rt_settings.devices)
        if len(devices) > capi.RT_MAX_DEVICES:
            raise ValueError(f"at most {capi.RT_MAX_DEVICES} devices")
        s.device_count = len(devices)
        for k, d in enumerate(devices):
            s.devices[k] = int(d)
    if truthy(denoising):
        # post-processor.js:55: Math.exp(-(kx*kx + ky*ky) / (2 * strength * strength)) for kx^2+ky^2 = 1, 2
        st = float(denoise_strength)
        s.denoise = 1
        s.denoise_weights[:] = (js_exp(-1 / (2 * st * st)), js_exp(-2 / (2 * st * st)))   # V8's Math.exp (jsmath.py)
    return s


class GpuRayTracer:
    def __init__(self, width, height, seed=0, device=0, precision=capi.RT_PREC_F64, accel=capi.RT_ACCEL_AUTO,
                 sum_order=capi.RT_SUM_POOL):
        self.width, self.height = int(width), int(height)
        self.seed = seed
        self.device = device
        self.precision = precision
        self.accel = accel
        self.sum_order = sum_order
        self.max_bounces, self.samples, self.gamma, self.exposure = 5, 4, 2.2, 1.0
        self.tone_mapping, self.anti_aliasing = "reinhard", "supersampling"
        self.denoising, self.denoise_strength = False, 0.5
        self.world, self.camera = default_scene(self.width, self.height, keyed_permutation(seed))
        self.image_data = np.zeros((self.height, self.width, 4), dtype=np.uint8)
        self.float_data = None
        self.last_stats = None
        self._scene = None
        self._packed = None
        self._dirty = True

    # ---- RayTracer API --------------------------------------------------------------------------
    def load_from_json(self, data):
        try:
            world, camera, dims = load_from_json(data, self.width, self.height, keyed_permutation(self.seed))
        except Exception:   # ray-tracer.js:330-333: errors -> false
            return False
        self.world = world
        if camera is not None:
            self.camera = camera
        if dims is not None:
            self.resize_canvas(*dims)
        self._dirty = True
        return True

    def resize_canvas(self, width, height):
        self.width, self.height = int(width), int(height)
        self.image_data = np.zeros((self.height, self.width, 4), dtype=np.uint8)
        if self.camera is not None:
            self.camera = setup_camera(self.camera, self.width, self.height)
        self._dirty = True

    def update_render_settings(self, params):
        g = params.get
        self.max_bounces = js_or(g("maxBounces"), 5)
        self.samples = js_or(g("samples"), 4)
        self.gamma = js_or(g("gamma"), 2.2)
        self.exposure = js_or(g("exposure"), 1.0)
        self.tone_mapping = js_or(g("toneMapping"), "reinhard")
        self.anti_aliasing = js_or(g("antiAliasing"), "supersampling")
        self.denoising = js_or(g("denoising"), False)
        self.denoise_strength = js_or(g("denoiseStrength"), 0.5)

    def update_background(self, type, intensity=1.0):
        self.world.sky_intensity = intensity
        self.world.background = {"solid": capi.RT_BG_SOLID, "hdri": capi.RT_BG_HDRI,
                                 "procedural_sky": capi.RT_BG_PROCEDURAL_SKY}.get(type, capi.RT_BG_GRADIENT)
        self.world.solid_color = (0.1, 0.1, 0.1)
        self._dirty = True

    # ---- packing / rendering --------------------------------------------------------------------
    def packed(self):
        if self._dirty or self._packed is None:
            self._packed = PackedScene(self.world, self.camera)
        return self._packed

    def settings(self, crop=None, sample_range=None, batch_samples=0, devices=None):
        return settings_struct(self.width, self.height, self.samples, self.max_bounces, self.anti_aliasing,
                               self.tone_mapping, self.exposure, self.gamma, self.seed, crop=crop,
                               precision=self.precision, sample_range=sample_range, batch_samples=batch_samples,
                               denoising=self.denoising, denoise_strength=self.denoise_strength, accel=self.accel,
                               devices=devices, sum_order=self.sum_order)

    def scene_handle(self):
        lib = capi.load_library()
        if self._dirty or self._scene is None:
            self.close()
            h = C.c_void_p()
            capi.check(lib.rt_scene_create(C.byref(self.packed().desc), self.device, C.byref(h)))
            self._scene = h
            self._dirty = False
        return self._scene

    def render(self, on_progress=None, crop=None, want=("rgba8",), batch_samples=0, resume=None, devices=None):
        """RayTracer.render: fills image_data (RGBA8) and float_data (post-gamma RGBA float).
        Returns a dict of the requested host arrays (mean, post, rgba8, segments, draws, preview).
        resume: a checkpoint() result to continue from (rt_render_resume).
        devices: HIP ordinals to deal the sample batches to (multi-GPU; may repeat a device).
        "preview" in want (with batch_samples): when on_progress runs, image_data (full frame) and the
        returned "preview" array hold the frame of the samples done so far (rt_output.preview_rgba8); a
        cancel (on_progress returning True, or rt_cancel) leaves the frame of the checkpointed samples
        there and raises RuntimeError(RT_ERR_CANCELLED)."""
        lib = capi.load_library()
        scene = self.scene_handle()
        st = self.settings(crop=crop, batch_samples=batch_samples, devices=devices)
        cw = st.crop_w or self.width
        ch = st.crop_h or self.height
        n = cw * ch
        res = {}
        out = capi.Output()
        if "mean" in want:
            res["mean"] = np.zeros((ch, cw, 3), dtype=np.float64)
            out.mean = res["mean"].ctypes.data_as(C.POINTER(C.c_double))
        res["post"] = np.zeros((ch, cw, 4), dtype=np.float32)
        out.post = res["post"].ctypes.data_as(C.POINTER(C.c_float))
        res["rgba8"] = np.zeros((ch, cw, 4), dtype=np.uint8)
        out.rgba8 = res["rgba8"].ctypes.data_as(C.POINTER(C.c_uint8))
        if "segments" in want:
            res["segments"] = np.zeros((ch, cw), dtype=np.uint32)
            out.segments = res["segments"].ctypes.data_as(C.POINTER(C.c_uint32))
        if "draws" in want:
            res["draws"] = np.zeros((ch, cw), dtype=np.uint32)
            out.draws = res["draws"].ctypes.data_as(C.POINTER(C.c_uint32))
        if "preview" in want:
            res["preview"] = np.zeros((ch, cw, 4), dtype=np.uint8)
            out.preview_rgba8 = res["preview"].ctypes.data_as(C.POINTER(C.c_uint8))
            if crop is None:                 # the running frame, as the reference's canvas between rows
                self.image_data = res["preview"]
        stats = capi.Stats()
        cb = capi.PROGRESS_FN(lambda f, u: int(bool(on_progress(f)) if on_progress else 0))
        if resume is None:
            rc = lib.rt_render(scene, C.byref(st), C.byref(out), cb, None, C.byref(stats))
        else:
            sums, done = resume
            sums = np.ascontiguousarray(sums, dtype=np.float64)
            assert sums.size == 3 * n, "checkpoint of another frame size"
            rc = lib.rt_render_resume(scene, C.byref(st), sums.ctypes.data_as(C.POINTER(C.c_double)), int(done),
                                      C.byref(out), cb, None, C.byref(stats))
        if rc == -4 and "preview" in want and crop is None:    # cancelled: the frame of the checkpoint stays
            self.image_data = res["preview"]
        capi.check(rc)
        self.last_stats = stats
        if crop is None:
            self.image_data = res["rgba8"]
            self.float_data = res["post"]
        if on_progress:
            on_progress(1.0)
        assert n == res["rgba8"].shape[0] * res["rgba8"].shape[1]
        return res

    def checkpoint(self, crop=None):
        """(per-pixel float64 sums (h, w, 3), samples_done) of the last render, finished or
        cancelled (rt_render_checkpoint); pass it to render(resume=...) to continue."""
        lib = capi.load_library()
        st = self.settings(crop=crop)
        cw, ch = st.crop_w or self.width, st.crop_h or self.height
        sums = np.zeros((ch, cw, 3), dtype=np.float64)
        done = C.c_int32()
        capi.check(lib.rt_render_checkpoint(self.scene_handle(), sums.ctypes.data_as(C.POINTER(C.c_double)), sums.size,
                                            C.byref(done)))
        return sums, done.value

    def close(self):
        if self._scene is not None:
            capi.load_library().rt_scene_destroy(self._scene)
            self._scene = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
