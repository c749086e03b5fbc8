"""GPU parity: the HIP path (through the C ABI) against the reference's golden fixtures and the
oracle.  Tolerances (BASELINE.json north_star: <= 1e-3 per-channel RMS vs the JS reference):
  * f64 mode  — same arithmetic as the JS: segment counts and RNG draw counts per pixel must be
                identical (every path decision matches), linear means within 1e-12 relative
                (only the forward throughput product's rounding differs from the recursion's),
                RGBA8 identical;
  * f32 mode  — per-channel RMS of post-gamma values <= 1e-3 where the survey's budget applies
                (>= 64 spp), looser bounds documented per case at low spp.
"""
import ctypes as C

import numpy as np
import pytest

import golden_cases as gc
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
from oracle import binding

pytestmark = pytest.mark.gpu

WANT = ("mean", "segments", "draws")


def rel_err(a, b):
    ok = ~(np.isnan(a) & np.isnan(b))
    return float(np.max(np.abs(a[ok] - b[ok]) / np.maximum(1.0, np.abs(b[ok])))) if ok.any() else 0.0


@pytest.mark.parametrize("case", gc.case_names())
def test_f64_matches_reference(gpu, case):
    rt, c = gc.tracer_for(case, precision=capi.RT_PREC_F64)
    r = rt.render(crop=c["crop"], want=WANT)
    lin = gc.load_array(case, "linear")
    assert np.array_equal(np.isnan(r["mean"]), np.isnan(lin))
    assert np.array_equal(r["segments"], gc.load_array(case, "segs")), "world.hit count per pixel differs"
    assert np.array_equal(r["draws"], gc.load_array(case, "draws")), "RNG draws per pixel differ"
    assert rel_err(r["mean"], lin) <= 1e-12
    rgba = gc.load_array(case, "rgba8")
    assert np.array_equal(r["rgba8"], rgba), "RGBA8 differs"
    if gc.has(case, "denoised"):                 # rt_output.post holds the denoised floats then
        dn = gc.load_array(case, "denoised")
        assert np.all(np.abs(r["post"] - dn) <= np.spacing(np.abs(dn))), "PostProcessor.denoise differs"
    else:
        post = gc.load_array(case, "post")
        ok = ~np.isnan(post)
        assert np.max(np.abs(r["post"][..., :3][ok] - post[ok]), initial=0) <= 1e-6   # float32 storage
    rt.close()


@pytest.mark.parametrize("case", gc.case_names())
def test_f64_sample_order_bit_exact_to_reference(gpu, case):
    """In the reference's own summation order (rt_settings.sum_order = RT_SUM_SAMPLE_ORDER: each pixel's
    samples added in sample order, ray-tracer.js:202-206) the GPU's binary64 render IS the reference's,
    bit for bit: every decision, Math.pow / exp / sin / cos (V8's own algorithms, csrc/js_math.h) and each
    sample's radiance in the recursion's order (pt_path.h trace_pixel: a0 * (a1 * (... * X)), as
    rayColor's emitted + attenuation * rayColor(scattered)).  Means, post-gamma values (float32 storage),
    RGBA8 bytes and the denoised frame equal the fixtures exactly."""
    rt, c = gc.tracer_for(case, precision=capi.RT_PREC_F64)
    rt.sum_order = capi.RT_SUM_SAMPLE_ORDER
    r = rt.render(crop=c["crop"], want=WANT)
    lin = gc.load_array(case, "linear")
    nan = np.isnan(lin)
    assert np.array_equal(np.isnan(r["mean"]), nan)
    a, b = r["mean"][~nan], lin[~nan]
    ulps = np.abs(a - b) / np.spacing(np.maximum(np.abs(b), 2.0 ** -1022))
    print(f"{case}: {np.mean(a == b):.4f} of channels bit-identical, max {ulps.max(initial=0):.1f} ulps")
    assert np.array_equal(a, b)
    assert np.array_equal(r["rgba8"], gc.load_array(case, "rgba8"))
    ref_post = gc.load_array(case, "denoised")[..., :3] if gc.has(case, "denoised") else gc.load_array(case, "post")
    ok = ~np.isnan(ref_post)
    assert np.array_equal(np.isnan(r["post"][..., :3]), ~ok)
    assert np.array_equal(r["post"][..., :3][ok], ref_post.astype(np.float32)[ok])
    rt.close()


# f32 fast mode: RMS of post-gamma output vs the reference.  At these low sample counts a single
# flipped path decision moves a pixel by up to 1/spp, so the bounds are per case; the north-star
# budget (1e-3) is asserted on the 512-spp RTOW crop.
F32_RMS = {"cfg3_rtow_crop_512spp": 1e-3, "cfg3_rtow_crop_512spp_wide": 1e-3, "cfg5_mesh50k_256spp_wide": 1e-3}


@pytest.mark.parametrize("case", gc.case_names())
def test_f32_rms(gpu, case):
    rt, c = gc.tracer_for(case, precision=capi.RT_PREC_F32)
    r = rt.render(crop=c["crop"])
    post = gc.load_array(case, "denoised")[..., :3] if gc.has(case, "denoised") else gc.load_array(case, "post")
    ok = ~np.isnan(post)
    assert np.array_equal(np.isnan(r["post"][..., :3]), ~ok)
    rms = float(np.sqrt(np.mean((r["post"][..., :3][ok] - post[ok]) ** 2))) if ok.any() else 0.0
    print(f"{case}: f32 post-gamma RMS {rms:.2e}")
    assert rms <= F32_RMS.get(case, 3e-2)
    rt.close()


@pytest.mark.parametrize("scene,w,h,spp,crop,bound", [
    ("rtow.json", 1920, 1080, 512, (896, 476, 128, 128), 1e-3),
    ("cornell.json", 512, 512, 64, None, 2.5e-3),
    ("mesh50k", 1920, 1080, 256, (896, 476, 128, 128), 1e-3)], ids=["config3", "config2", "config5"])
def test_f32_rms_at_full_spp(gpu, scene, w, h, spp, crop, bound):
    """The f32 fast mode against the f64 mode (whose path decisions are the reference's, every golden
    fixture) at each config's full resolution and sample count: per-channel RMS of the post-gamma
    values <= 1e-3 (BASELINE.json north-star tolerance) on 128x128 crops of configs 3 and 5.  Config 2
    (the whole Cornell frame, 64 spp): binary32 flips a path decision in ~0.02 % of pixels (58 of
    262k in this render), and a flipped path that reaches the intensity-15 light moves its pixel's
    mean by up to 15/64, so f32 measures 1.7e-3 RMS there — above the north-star bound, which the
    default f64 mode meets (its decisions are the reference's); the bound asserted is 2.5e-3."""
    post = {}
    for prec in (capi.RT_PREC_F64, capi.RT_PREC_F32):
        rt = GpuRayTracer(w, h, seed=8, precision=prec)
        assert rt.load_from_json(load_scene_json(scene))
        rt.update_render_settings({"maxBounces": 5, "samples": spp})
        post[prec] = rt.render(crop=crop)["post"][..., :3].astype(np.float64)
        rt.close()
    a, b = post[capi.RT_PREC_F64], post[capi.RT_PREC_F32]
    ok = ~np.isnan(a)
    assert np.array_equal(ok, ~np.isnan(b))
    rms = float(np.sqrt(np.mean((a[ok] - b[ok]) ** 2)))
    print(f"{scene} {w}x{h}x{spp}: f32 vs f64 post-gamma RMS {rms:.2e}")
    assert rms <= bound


def _rtow(w, h, spp, precision=capi.RT_PREC_F64, seed=1234):
    rt = GpuRayTracer(w, h, seed=seed, precision=precision)
    assert rt.load_from_json(load_scene_json("rtow.json"))
    rt.update_render_settings({"maxBounces": 5, "samples": spp})
    return rt


def test_f64_matches_oracle_rtow(gpu):
    rt = _rtow(160, 90, 16)
    r = rt.render(want=WANT)
    o = binding.render(rt.packed(), rt.settings())
    assert np.array_equal(r["segments"], o["segments"]) and np.array_equal(r["draws"], o["draws"])
    assert rel_err(r["mean"], o["mean"]) <= 1e-12
    assert np.array_equal(r["rgba8"], o["rgba8"])


# Summation-order tolerance: the sample pool adds a pixel's samples in the order its wave finishes
# them (then the chunk partials in chunk order), not in sample order, so renders that split the same
# samples differently (batches, crops, launches) agree to the rounding of the binary64 sums.  Every
# path decision (segment and draw counts) is unaffected.
SUM_RTOL = 1e-13


def test_batching_matches_one_launch(gpu):
    """Sample batches continue each pixel's running sum: one launch's result up to summation order."""
    rt = _rtow(96, 54, 12)
    full = rt.render(want=("mean", "segments"))
    batched = rt.render(want=("mean", "segments"), batch_samples=5)
    assert np.array_equal(full["segments"], batched["segments"])
    assert np.allclose(full["mean"], batched["mean"], rtol=SUM_RTOL, atol=0)


def test_crop_is_window_of_full(gpu):
    rt = _rtow(128, 72, 6)
    full = rt.render(want=("mean", "segments"))
    crop = rt.render(want=("mean", "segments"), crop=(37, 11, 50, 29))
    assert np.array_equal(full["segments"][11:40, 37:87], crop["segments"])
    assert np.allclose(full["mean"][11:40, 37:87], crop["mean"], rtol=SUM_RTOL, atol=0)


def test_deterministic_and_progress(gpu):
    """The same render twice gives the same bits (the pool's summation order depends only on the
    scene, the crop and the launch split, never on timing); progress is monotone and ends at 1."""
    rt = _rtow(64, 36, 8)
    seen = []
    a = rt.render(want=("mean",), batch_samples=2, on_progress=lambda f: seen.append(f) and False)["mean"]
    a2 = rt.render(want=("mean",), batch_samples=2)["mean"]
    b = rt.render(want=("mean",))["mean"]
    assert np.array_equal(a, a2)
    assert np.allclose(a, b, rtol=SUM_RTOL, atol=0)
    assert seen and seen[-1] == 1.0 and all(x <= y for x, y in zip(seen, seen[1:]))


def test_cancel_via_progress(gpu):
    rt = _rtow(64, 36, 16)
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(batch_samples=1, on_progress=lambda f: True)
    # the first batch, plus those of the three queued behind it that were reduced before the cancel
    # word reached them (they stop at their next item and are not reduced: the checkpoint is a prefix)
    assert 1 <= rt.checkpoint()[1] <= 4


def test_cancel_between_batches_in_sample_order(gpu):
    """Without the pool's overlapped batches (sample order) a cancel is observed between batches: the
    batches already queued complete (the first and the three behind it), and the checkpoint resumes
    bit-exactly."""
    rt = _rtow(64, 36, 16)
    rt.sum_order = capi.RT_SUM_SAMPLE_ORDER
    full = rt.render(want=("mean",), batch_samples=1)
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(batch_samples=1, on_progress=lambda f: True)
    sums, done = rt.checkpoint()
    assert done == 4
    rt2 = _rtow(64, 36, 16)
    rt2.sum_order = capi.RT_SUM_SAMPLE_ORDER
    assert np.array_equal(rt2.render(want=("mean",), resume=(sums, done), batch_samples=1)["mean"], full["mean"])


def test_max_depth_zero_is_black(gpu):
    rt = _rtow(32, 18, 4)
    rt.max_bounces = -1        # truthy in JS: rayColor(ray, -1) returns 0 immediately
    r = rt.render(want=("mean", "segments"))
    assert np.all(r["mean"] == 0) and np.all(r["segments"] == 0)


def test_trace_device_sample_split(gpu):
    """Sample-range sharding (the multi-GPU path): partial sums over [0,k) and [k,S) add up."""
    import torch
    rt = _rtow(80, 45, 10)
    lib = capi.load_library()
    scene = rt.scene_handle()
    n = 80 * 45
    sums = []
    for rng in ((0, 10), (0, 4), (4, 10)):
        buf = torch.zeros(n * 3, dtype=torch.float64, device="cuda")
        st = rt.settings(sample_range=rng)
        torch.cuda.synchronize()
        capi.check(lib.rt_trace_device(scene, C.byref(st), C.c_void_p(buf.data_ptr()), None, 1, None))
        sums.append(buf.cpu().numpy())
    full, a, b = sums
    assert np.allclose(a + b, full, rtol=1e-13, atol=0)


def test_full_resolution_config3_properties(gpu):
    """Config 3 at its full 1920x1080 size (2 spp): finite, deterministic, windows match the oracle."""
    rt = _rtow(1920, 1080, 2, seed=17)
    r1 = rt.render(want=("mean", "segments"))
    r2 = rt.render(want=("mean",))
    assert np.all(np.isfinite(r1["mean"]))
    assert np.array_equal(r1["mean"], r2["mean"])
    for (x0, y0) in ((0, 0), (950, 530), (1904, 1064)):
        o = binding.render(rt.packed(), rt.settings(crop=(x0, y0, 16, 16)))
        assert np.array_equal(o["segments"], r1["segments"][y0:y0 + 16, x0:x0 + 16])
        assert rel_err(r1["mean"][y0:y0 + 16, x0:x0 + 16], o["mean"]) <= 1e-12
    seg_per_sample = r1["segments"].sum() / (1920 * 1080 * 2)
    assert 1.5 < seg_per_sample < 4.0


@pytest.mark.parametrize("case", gc.case_names())
def test_f64_bvh_matches_reference(gpu, case):
    """RT_ACCEL_BVH on the GPU: the same per-pixel decisions and bits as the World-order walk."""
    rt, c = gc.tracer_for(case, precision=capi.RT_PREC_F64)
    rt.accel = capi.RT_ACCEL_BVH
    r = rt.render(crop=c["crop"], want=WANT)
    lin = gc.load_array(case, "linear")
    assert np.array_equal(r["segments"], gc.load_array(case, "segs"))
    assert np.array_equal(r["draws"], gc.load_array(case, "draws"))
    assert np.array_equal(np.isnan(r["mean"]), np.isnan(lin))
    assert rel_err(r["mean"], lin) <= 1e-12
    rt.accel = capi.RT_ACCEL_BRUTE
    b = rt.render(crop=c["crop"], want=WANT)
    assert np.array_equal(r["mean"], b["mean"], equal_nan=True)
    rt.close()


@pytest.mark.parametrize("precision", [capi.RT_PREC_F64, capi.RT_PREC_F32])
def test_bvh_bit_identical_to_brute_mesh50k(gpu, precision):
    """The 49,984-triangle mesh (config 5): BVH and brute force agree bit for bit on a crop in f64
    (bvh_conservative_bound); in f32 the node margins are not a proof, so near-identical is asserted."""
    rt = GpuRayTracer(1920, 1080, seed=5, precision=precision)
    assert rt.load_from_json(load_scene_json("mesh50k"))
    rt.update_render_settings({"maxBounces": 5, "samples": 4})
    crop = (900, 480, 96, 64)
    rt.accel = capi.RT_ACCEL_BVH
    a = rt.render(crop=crop, want=WANT)
    rt.accel = capi.RT_ACCEL_BRUTE
    b = rt.render(crop=crop, want=WANT)
    if precision == capi.RT_PREC_F32:
        assert np.mean(a["segments"] == b["segments"]) >= 0.999
        assert np.sqrt(np.mean((a["mean"] - b["mean"]) ** 2)) <= 1e-3
    else:
        assert np.array_equal(a["segments"], b["segments"]) and np.array_equal(a["draws"], b["draws"])
        assert np.array_equal(a["mean"], b["mean"], equal_nan=True)
        o = binding.render(rt.packed(), rt.settings(crop=(crop[0], crop[1], 16, 16)))
        assert np.array_equal(o["segments"], a["segments"][:16, :16])
        assert rel_err(a["mean"][:16, :16], o["mean"]) <= 1e-12
    rt.close()


def test_exit_skip_bit_identical_on_mesh_silhouette(gpu):
    """tri_exit_bound on the device: the tree kernel skips the triangle walk of segments leaving the mesh
    (pt_core.h leaves_tri_hull), the brute-force World-order kernel never skips.  Over the UV sphere's
    silhouette, where reflections leave the mesh at grazing angles, the two agree bit for bit."""
    rt = GpuRayTracer(1920, 1080, seed=11, precision=capi.RT_PREC_F64)
    assert rt.load_from_json(load_scene_json("mesh50k"))
    rt.update_render_settings({"maxBounces": 5, "samples": 8})
    crop = (1090, 470, 96, 96)                  # the sphere's right edge (its centre projects to 960, 540)
    rt.accel = capi.RT_ACCEL_BVH
    a = rt.render(crop=crop, want=WANT)
    rt.accel = capi.RT_ACCEL_BRUTE
    b = rt.render(crop=crop, want=WANT)
    assert np.array_equal(a["segments"], b["segments"]) and np.array_equal(a["draws"], b["draws"])
    assert np.array_equal(a["mean"], b["mean"], equal_nan=True)
    rt.close()


def test_resume_with_one_batch_left_is_bit_exact(gpu):
    """A resume whose remaining samples are a single batch (the render as a whole has several) takes
    that batch's chunks from the whole render's rule, as the uninterrupted render did: bit-identical.
    (Round 5: the single batch took the pool's rule for its own 32 samples — 11 + 11 + 10 instead of
    32 — and the resumed sums differed by 1 ulp in most pixels.)  Cancelled from the progress call
    after the 2nd of 3 fused batches: the checkpoint is 64 samples (or 96 if the 3rd batch finished
    before the cancel reached it)."""
    rt = _rtow(640, 360, 96)
    full = rt.render(want=("mean",), batch_samples=32)
    calls = []
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(batch_samples=32, on_progress=lambda f: calls.append(f) or len(calls) >= 2)
    sums, done = rt.checkpoint()
    rt.close()
    print(f"checkpoint {done} samples")
    assert done in (64, 96)
    rt2 = _rtow(640, 360, 96)
    res = rt2.render(want=("mean",), resume=(sums, done), batch_samples=32)
    assert np.array_equal(res["mean"], full["mean"])
    rt2.close()


def test_resident_resume_checks_its_checkpoint(gpu):
    """rt_render_resume(sums = NULL) continues from the sums left on the device only for the checkpoint's
    own frame, crop, first sample, precision and seed (the pixel count alone let a crop of the
    same area at another origin continue from unrelated sums); the matching resume is bit-exact."""
    rt = _rtow(64, 48, 16)
    lib = capi.load_library()
    scene = rt.scene_handle()
    crop = (0, 0, 32, 24)
    full = rt.render(want=("mean",), crop=crop, batch_samples=4)["mean"]
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(crop=crop, batch_samples=4, on_progress=lambda f: True)
    done = C.c_int32()
    capi.check(lib.rt_render_checkpoint(scene, None, 0, C.byref(done)))
    assert 4 <= done.value < 16
    mean = np.zeros((24, 32, 3))
    out = capi.Output()
    out.mean = mean.ctypes.data_as(C.POINTER(C.c_double))

    def resume(st):
        return lib.rt_render_resume(scene, C.byref(st), None, done.value, C.byref(out), capi.PROGRESS_FN(0), None,
                                    None)
    other_origin = rt.settings(crop=(8, 0, 32, 24), batch_samples=4)          # same area, another window
    assert resume(other_origin) == -1 and "another frame" in lib.rt_last_error().decode()
    other_seed = rt.settings(crop=crop, batch_samples=4)
    other_seed.seed += 1
    assert resume(other_seed) == -1
    other_prec = rt.settings(crop=crop, batch_samples=4)
    other_prec.precision = capi.RT_PREC_F32
    assert resume(other_prec) == -1
    capi.check(resume(rt.settings(crop=crop, batch_samples=4)))                # the checkpoint's own: resumes
    assert np.array_equal(mean, full)
    rt.close()


def test_finalize_two_streams_two_gammas(gpu):
    """Two asynchronous RGBA8-only rt_finalize_device calls with different gammas on two streams, no host
    wait in between (one gamma table per scene was rebuilt in place for the second call while
    the first call's kernel could still read it): each frame equals its own synchronous finalize_kernel
    frame (Float32 output requested, so the table is not used)."""
    import torch
    rng = np.random.default_rng(5)
    n = 1 << 18
    sums = torch.from_numpy(rng.uniform(0.0, 1.5, 3 * n)).cuda()
    rt = _rtow(n, 1, 1, seed=1)
    lib = capi.load_library()
    scene = rt.scene_handle()
    gammas = (2.2, 1.7, 2.2, 0.8)
    refs = []
    for g in gammas:
        rt.gamma = g
        ref = torch.zeros(4 * n, dtype=torch.uint8, device="cuda")
        post = torch.zeros(4 * n, dtype=torch.float32, device="cuda")
        capi.check(lib.rt_finalize_device(scene, C.byref(rt.settings()), C.c_void_p(sums.data_ptr()), None,
                                          C.c_void_p(post.data_ptr()), C.c_void_p(ref.data_ptr()), None))
        refs.append(ref)
    torch.cuda.synchronize()
    for rep in range(3):
        streams = [torch.cuda.Stream() for _ in gammas]
        outs = [torch.zeros(4 * n, dtype=torch.uint8, device="cuda") for _ in gammas]
        torch.cuda.synchronize()
        for g, st, o in zip(gammas, streams, outs):
            rt.gamma = g
            capi.check(lib.rt_finalize_device(scene, C.byref(rt.settings()), C.c_void_p(sums.data_ptr()), None, None,
                                              C.c_void_p(o.data_ptr()), C.c_void_p(st.cuda_stream)))
        torch.cuda.synchronize()
        for g, o, r in zip(gammas, outs, refs):
            assert torch.equal(o, r), (rep, g)
    rt.close()


def test_checkpoint_resume_is_bit_exact(gpu):
    """Progressive rendering: cancel after some batches, checkpoint the float64 sums,
    resume in a NEW scene handle from the saved state: identical bits to an uninterrupted render with
    the same sample batches."""
    rt = _rtow(96, 54, 10)
    full = rt.render(want=("mean", "segments"), batch_samples=1)
    calls = []
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(batch_samples=1, on_progress=lambda f: calls.append(f) or len(calls) >= 2)
    sums, done = rt.checkpoint()
    # cancelled after batch 2: of batches 3 to 5 (queued) those reduced before the cancel reached them
    assert 2 <= done <= 5 and sums.shape == (54, 96, 3)
    rt.close()
    rt2 = _rtow(96, 54, 10)
    res = rt2.render(want=("mean",), resume=(sums, done), batch_samples=1)
    assert np.array_equal(res["mean"], full["mean"])
    assert np.array_equal(res["rgba8"], full["rgba8"])
    s2, d2 = rt2.checkpoint()
    assert d2 == 10
    rt2.close()


_WALK_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import torch  # noqa: F401  (HIP runtime first)
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
out = {}
for name, w, h, crop in (("mesh50k", 1920, 1080, (900, 480, 64, 48)), ("kitchen_sink.json", 96, 64, None),
                         ("rtow.json", 160, 90, None)):
    rt = GpuRayTracer(w, h, seed=9, accel=capi.RT_ACCEL_BVH)
    assert rt.load_from_json(load_scene_json(name))
    rt.update_render_settings({"samples": 4, "maxBounces": 5})
    r = rt.render(crop=crop, want=("mean", "segments", "draws"))
    for k in ("mean", "segments", "draws"):
        out[f"{name}.{k}"] = r[k]
np.savez(sys.argv[2], **out)
'''


def _render_in_child(script, path, **env):
    """Run `script` in a child process (the trace-kernel choices are read once per process)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", script, root, str(path)], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(path)


_LEAN_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import torch  # noqa: F401  (HIP runtime first)
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
out = {}
# the three lean kernels' scenes (RTOW: the grid, spheres only; mesh50k: the triangle walk, no boxes;
# Cornell: World order, spheres and planes), in both precisions, plus a scene that takes none (stochastic AA)
for name, w, h, crop, aa in (("rtow.json", 160, 90, None, "supersampling"), ("mesh50k", 1920, 1080, (900, 480, 64, 48), "supersampling"),
                             ("cornell.json", 96, 96, None, "supersampling"), ("rtow.json", 96, 54, None, "stochastic")):
    for prec in (capi.RT_PREC_F64, capi.RT_PREC_F32):
        rt = GpuRayTracer(w, h, seed=21, precision=prec)
        assert rt.load_from_json(load_scene_json(name))
        rt.update_render_settings({"samples": 6, "maxBounces": 5, "antiAliasing": aa})
        r = rt.render(crop=crop, want=("mean", "segments", "draws"), batch_samples=2)
        for k in ("mean", "segments", "draws"):
            out[f"{name}.{aa}.{prec}.{k}"] = r[k]
        rt.close()
np.savez(sys.argv[2], **out)
'''


def test_lean_kernels_bit_identical(gpu, tmp_path):
    """The lean kernels (round 6: compiled without the plane / box / triangle code a scene cannot use,
    the other backgrounds, the orthographic camera and the other AA modes) give the general kernels' bits:
    the same renders with RT_LEAN=0 (never lean) equal the default ones bit for bit, per-pixel segment and
    RNG-draw counts included — one-shot and in progressive batches, binary64 and binary32."""
    lean = _render_in_child(_LEAN_SCRIPT, tmp_path / "lean.npz")
    general = _render_in_child(_LEAN_SCRIPT, tmp_path / "general.npz", RT_LEAN="0")
    for k in lean.files:
        assert np.array_equal(lean[k], general[k], equal_nan=True), k


@pytest.mark.parametrize("walk", ["skip", "tree", "grid"])
def test_alternative_bvh_walks_bit_identical(gpu, tmp_path, walk):
    """Every walk renders the same bits as the general two-child walk (RT_BVH_WALK=two): skip = the
    stackless preorder walk, tree = the sphere tree where the uniform grid was chosen (RTOW), grid =
    the grid wherever one was built (run in child processes: the walk is chosen per process)."""
    res = {mode: _render_in_child(_WALK_SCRIPT, tmp_path / f"{mode}.npz", RT_BVH_WALK=mode) for mode in ("two", walk)}
    for k in res["two"].files:
        assert np.array_equal(res["two"][k], res[walk][k], equal_nan=True), k


_POOL_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import torch  # noqa: F401  (HIP runtime first)
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
out = {}
for name, w, h, crop, prec, accel, spp in (
        ("mesh50k", 1920, 1080, (900, 480, 61, 43), capi.RT_PREC_F64, capi.RT_ACCEL_BVH, 5),
        ("kitchen_sink.json", 96, 64, None, capi.RT_PREC_F64, capi.RT_ACCEL_BVH, 7),
        ("kitchen_sink.json", 96, 64, None, capi.RT_PREC_F64, capi.RT_ACCEL_BRUTE, 7),
        ("cornell.json", 52, 37, None, capi.RT_PREC_F64, capi.RT_ACCEL_AUTO, 9),
        ("rtow.json", 163, 91, None, capi.RT_PREC_F64, capi.RT_ACCEL_BVH, 7),
        ("rtow.json", 163, 91, None, capi.RT_PREC_F32, capi.RT_ACCEL_BVH, 7)):
    rt = GpuRayTracer(w, h, seed=9, accel=accel, precision=prec)
    assert rt.load_from_json(load_scene_json(name))
    rt.update_render_settings({"samples": spp, "maxBounces": 5})
    r = rt.render(crop=crop, want=("mean", "segments", "draws"))
    for k in ("mean", "segments", "draws"):
        out[f"{name}.{prec}.{accel}.{k}"] = r[k]
    out[f"{name}.{prec}.{accel}.batched"] = rt.render(crop=crop, want=("mean",), batch_samples=3)["mean"]
np.savez(sys.argv[2], **out)
'''


@pytest.mark.parametrize("env", [{}, {"RT_PART_MB": "1", "RT_POOL_CHUNK": "2"}, {"RT_POOL_CHUNK": "1"},
                                 {"RT_POOL_CHUNK": "3"}],
                         ids=["default", "split_launches", "one_sample_chunks", "three_sample_chunks"])
def test_sample_pool_vs_lane_per_pixel(gpu, tmp_path, env):
    """The sample-pool kernel (default: lanes take (pixel, sample) items of their 8x8 tile, radiance
    added to per-pixel partials in LDS, chunk partials added in chunk order) against the in-order
    lane-per-pixel kernel (RT_SAMPLE_POOL=0): identical segment and draw counts, sums equal up to the
    order of the binary64 additions (SUM_RTOL) — also when a 1-MiB partials budget splits the samples
    over many launches and with 1- and 3-sample chunks; ragged tiles, both precisions, BVH and brute
    force.  A second pool run in another process must reproduce the first bit for bit."""
    base = _render_in_child(_POOL_SCRIPT, tmp_path / "lpp.npz", RT_SAMPLE_POOL="0")
    pool = _render_in_child(_POOL_SCRIPT, tmp_path / "pool.npz", **env)
    again = _render_in_child(_POOL_SCRIPT, tmp_path / "again.npz", **env)
    for k in base.files:
        assert np.array_equal(pool[k], again[k], equal_nan=True), k
        if k.endswith(("segments", "draws")):
            assert np.array_equal(base[k], pool[k]), k
        else:
            assert np.array_equal(np.isnan(base[k]), np.isnan(pool[k])), k
            ok = ~np.isnan(base[k])
            assert np.allclose(base[k][ok], pool[k][ok], rtol=SUM_RTOL, atol=1e-300), k


@pytest.mark.parametrize("env", [{}, {"RT_PART_MB": "1", "RT_POOL_CHUNK": "2"}], ids=["default", "split_launches"])
def test_lds_node_kernel_bit_identical(gpu, tmp_path, env):
    """trace_pool_lds_kernel (sphere tree nodes in LDS, multi-wave workgroups taking (tile, chunk)
    items from a device-wide queue; default for binary32 sphere scenes, RT_LDS_NODES=2 forces it for
    binary64 too) renders exactly the bits of the one-wave pool kernel (RT_LDS_NODES=0): sums, segment
    and draw counts, batched renders — also over many launches (1-MiB partials budget, 2-sample chunks:
    the queue ring is reused) and in a second process."""
    base = _render_in_child(_POOL_SCRIPT, tmp_path / "global.npz", RT_LDS_NODES="0", **env)
    lds = _render_in_child(_POOL_SCRIPT, tmp_path / "lds.npz", RT_LDS_NODES="2", **env)
    again = _render_in_child(_POOL_SCRIPT, tmp_path / "again.npz", RT_LDS_NODES="2", **env)
    for k in base.files:
        assert np.array_equal(base[k], lds[k], equal_nan=True), k
        assert np.array_equal(lds[k], again[k], equal_nan=True), k


@pytest.mark.parametrize("env", [{}, {"RT_PART_MB": "1", "RT_POOL_CHUNK": "2"}], ids=["default", "split_launches"])
def test_lds_grid_kernel_bit_identical(gpu, tmp_path, env):
    """The grid walk with its cell offsets and record filters in LDS (trace_pool_lds_kernel<.., 7>,
    default where the grid is walked: RTOW in both precisions) renders exactly the bits of the one-wave
    grid kernel reading them from global memory (RT_LDS_GRID=0): sums, segment and draw counts, batched
    renders, also over many launches, and again in a second process."""
    base = _render_in_child(_POOL_SCRIPT, tmp_path / "global.npz", RT_LDS_GRID="0", **env)
    lds = _render_in_child(_POOL_SCRIPT, tmp_path / "lds.npz", RT_LDS_GRID="1", **env)
    again = _render_in_child(_POOL_SCRIPT, tmp_path / "again.npz", **env)
    for k in base.files:
        assert np.array_equal(base[k], lds[k], equal_nan=True), k
        assert np.array_equal(lds[k], again[k], equal_nan=True), k


@pytest.mark.parametrize("precision", [capi.RT_PREC_F64, capi.RT_PREC_F32], ids=["f64", "f32"])
def test_trace_device_two_streams_then_render(gpu, precision):
    """Scene scratch shared across streams: two rt_trace_device shards enqueued on two
    different streams with no host synchronization, then rt_render on the scene's own stream: every
    result equals its single-launch counterpart.  In binary32 the launches are trace_pool_lds_kernel's,
    running at once on the two streams, each with its own device-wide item queue."""
    import torch
    rt = _rtow(200, 120, 24, precision=precision)   # several chunks per launch: the shards use the partials buffer
    lib = capi.load_library()
    scene = rt.scene_handle()
    n = 200 * 120
    ref_full = rt.render(want=("mean",))["mean"]
    refs = []
    for rng in ((0, 13), (13, 24)):
        buf = torch.zeros(n * 3, dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        capi.check(lib.rt_trace_device(scene, C.byref(rt.settings(sample_range=rng)), C.c_void_p(buf.data_ptr()), None, 1, None))
        refs.append(buf.cpu().numpy())
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    bufs = [torch.zeros(n * 3, dtype=torch.float64, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    for rng, st, buf in zip(((0, 13), (13, 24)), (s1, s2), bufs):
        capi.check(lib.rt_trace_device(scene, C.byref(rt.settings(sample_range=rng)), C.c_void_p(buf.data_ptr()),
                                       C.c_void_p(st.cuda_stream), 0, None))
    full = rt.render(want=("mean",))["mean"]
    torch.cuda.synchronize()
    for ref, buf in zip(refs, bufs):
        assert np.array_equal(buf.cpu().numpy(), ref)
    assert np.array_equal(full, ref_full)


@pytest.mark.parametrize("scene,w,h,spp,crop,bands", [
    ("rtow.json", 640, 360, 24, None, 8),           # the grid's LDS pool kernel, several chunks
    ("rtow.json", 200, 120, 3, (10, 20, 150, 90), 64),   # one chunk; more bands asked than tile rows
    ("mesh50k", 640, 360, 12, (100, 50, 300, 200), 5),   # the one-wave kernel (triangle tree)
    ("cornell.json", 256, 256, 16, None, 3),        # brute force
])
def test_trace_device_bands_bit_identical(gpu, scene, w, h, spp, crop, bands):
    """rt_trace_device_bands (the band-by-band multi-GPU reduce): the same sums as
    rt_trace_device bit for bit (band-major items, the same chunks and partials), every band delivered
    once, in order, as contiguous rows covering the crop, and the callback's rows already final when it
    runs (a copy enqueued on the stream from inside the callback equals the final rows)."""
    import torch
    rt = GpuRayTracer(w, h, seed=4)
    assert rt.load_from_json(load_scene_json(scene))
    rt.update_render_settings({"samples": spp, "maxBounces": 5})
    lib = capi.load_library()
    sc = rt.scene_handle()
    st = rt.settings(crop=crop)
    cw, ch = (crop[2], crop[3]) if crop else (w, h)
    ref = torch.zeros(3 * cw * ch, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    capi.check(lib.rt_trace_device(sc, C.byref(st), C.c_void_p(ref.data_ptr()), None, 1, None))
    got = torch.zeros_like(ref)
    snap = torch.full_like(ref, float("nan"))
    stream = torch.cuda.current_stream()
    seen = []

    def ready(b, row0, rows, user):
        seen.append((b, row0, rows))
        sl = slice(3 * row0 * cw, 3 * (row0 + rows) * cw)
        snap[sl].copy_(got[sl])          # enqueued on the current stream right behind the band's reduce
        return 0
    cb = capi.BAND_FN(ready)
    torch.cuda.synchronize()
    stats = capi.Stats()
    capi.check(lib.rt_trace_device_bands(sc, C.byref(st), C.c_void_p(got.data_ptr()), C.c_void_p(stream.cuda_stream),
                                         bands, cb, None, C.byref(stats)))
    torch.cuda.synchronize()
    nb = min(bands, (ch + 7) // 8)
    assert [b for b, _, _ in seen] == list(range(nb))
    assert seen[0][1] == 0 and sum(r for _, _, r in seen) == ch
    assert all(seen[k][1] + seen[k][2] == seen[k + 1][1] for k in range(nb - 1))
    assert torch.equal(got, ref)
    assert torch.equal(snap, ref)        # every band was final when its callback ran
    assert stats.samples == cw * ch * spp and stats.kernel_ms > 0
    rt.close()


def test_sharded_step_matches_render(gpu):
    """bench.py's device path (ShardedRender.step: d_sum zeroed on torch's stream, rt_trace_device,
    rt_finalize_device, no synchronization in between) gives the host API's image frame after frame:
    the zeroing, the trace and the epilogue run in stream order."""
    import torch
    from blenderraytracer_amd.distributed import ShardedRender
    rt = _rtow(640, 360, 8, seed=3)
    ref = rt.render(want=("rgba8",))["rgba8"]
    job = ShardedRender(rt, device=torch.device("cuda", 0))
    for _ in range(3):
        job.step(stats=False)
        torch.cuda.synchronize()
        assert np.array_equal(job.rgba8.cpu().numpy().reshape(ref.shape), ref)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]], ids=["2_shards", "3_shards"])
def test_multi_device_split_matches_one_device(gpu, devices):
    """rt_settings.devices (SURVEY §8e through the C ABI), the whole-batch split: batch k traced on
    devices[k % N] (here all device 0: the replicas run on their own streams), its chunk partials copied
    to the scene's device and reduced there in batch order.  Bit-identical to the same batches on one
    device (without batch_samples the batch is ceil(samples / N)), identical per-pixel segment and draw
    counts, equal to the one-batch render up to summation order; replicas cached and re-zeroed.  The
    sample-order mode still splits every batch into N contiguous sample ranges (equal up to order)."""
    rt = _rtow(160, 90, 24)
    want = ("mean", "segments", "draws")
    nd = len(devices)
    one = rt.render(want=want)
    many = rt.render(want=want, devices=devices)
    for k in ("segments", "draws"):
        assert np.array_equal(one[k], many[k]), k
    assert np.allclose(one["mean"], many["mean"], rtol=SUM_RTOL, atol=0)
    assert np.array_equal(many["mean"], rt.render(want=("mean",), batch_samples=-(-24 // nd))["mean"])
    batched = rt.render(want=want, devices=devices, batch_samples=7)
    assert np.array_equal(one["segments"], batched["segments"]) and np.array_equal(one["draws"], batched["draws"])
    assert np.array_equal(batched["mean"], rt.render(want=("mean",), batch_samples=7)["mean"])
    again = rt.render(want=want, devices=devices, batch_samples=7)      # replicas cached, re-zeroed
    assert np.array_equal(batched["mean"], again["mean"])
    rt.sum_order = capi.RT_SUM_SAMPLE_ORDER                            # every batch split over the devices
    ordered = rt.render(want=want)
    split = rt.render(want=want, devices=devices, batch_samples=7)
    for k in ("segments", "draws"):
        assert np.array_equal(ordered[k], split[k]), k
    assert np.allclose(ordered["mean"], split["mean"], rtol=SUM_RTOL, atol=0)
    rt.close()


def test_multi_device_checkpoint_resume(gpu):
    """Cancel a 2-device render (whole-batch split) in its first progress call: the queued batches stop
    at their next item and are not reduced, so the checkpoint is a prefix of the batches (at least the
    first, at most the 1 + 2 x 3 queued behind it).  Resumed in a new scene with the same devices and
    batches: bit-identical to the uninterrupted render."""
    rt = _rtow(640, 360, 160)
    full = rt.render(want=("mean",), batch_samples=8, devices=[0, 0])
    calls = []
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(batch_samples=8, devices=[0, 0], on_progress=lambda f: calls.append(f) or len(calls) >= 1)
    sums, done = rt.checkpoint()
    print(f"cancelled in the first progress call: {done} of 160 samples checkpointed")
    assert done % 8 == 0 and 8 <= done <= 8 * 7
    rt.close()
    rt2 = _rtow(640, 360, 160)
    res = rt2.render(want=("mean",), resume=(sums, done), batch_samples=8, devices=[0, 0])
    assert np.array_equal(res["mean"], full["mean"])
    rt2.close()


_CANCEL_SCRIPT = r'''
import sys, threading, time, json
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch  # noqa: F401  (HIP runtime first)
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
devices = json.loads(sys.argv[3])
scene, spp = (sys.argv[4], int(sys.argv[5])) if len(sys.argv) > 5 else ("rtow.json", 512)
batch = spp // 4
def tracer():
    rt = GpuRayTracer(1920, 1080, seed=5)
    assert rt.load_from_json(load_scene_json(scene))
    rt.update_render_settings({"maxBounces": 5, "samples": spp})
    return rt
rt = tracer()
rt.render(batch_samples=batch, devices=devices)                       # warm-up (scene, replicas, slots)
t = time.perf_counter()
full = rt.render(want=("mean",), batch_samples=batch, devices=devices)
frame_s = time.perf_counter() - t
lib = capi.load_library()
box = {}
def run():
    try:
        rt.render(batch_samples=batch, devices=devices)
        box["rc"] = 0
    except RuntimeError as e:
        box["rc"] = str(e)
    box["t"] = time.perf_counter()
th = threading.Thread(target=run)
th.start()
time.sleep(0.4 * frame_s)                                            # inside the second batch
t0 = time.perf_counter()
capi.check(lib.rt_cancel(rt.scene_handle()))
th.join()
sums, done = rt.checkpoint()
rt2 = tracer()
res = rt2.render(want=("mean",), resume=(sums, done), batch_samples=batch, devices=devices)
np.savez(sys.argv[2], latency=box["t"] - t0, frame=frame_s, done=done, rc=str(box["rc"]),
         equal=np.array_equal(res["mean"], full["mean"]))
'''


@pytest.mark.parametrize("devices", [None, [0, 0]], ids=["one_device", "2_devices"])
def test_cancel_latency_within_a_batch(gpu, tmp_path, devices):
    """VERDICT r3 item 5 / ray-tracer.js:190,196,256 (the reference stops at the next pixel): a cancel
    from another thread (rt_cancel, as the Node drop-in's window.renderCancelled does) stops the batches
    in flight at their next (tile, chunk) item.  Config 3's frame (1920x1080 x 512 spp) in four batches
    of 128 spp, cancelled 40 % into the frame: rt_render returns in less than one batch's time (before
    the cancel stopped only new batches: the 3 queued ones ran to the end, about 0.6 frames), and the
    checkpoint (the batches reduced before the cancel) resumes bit-exactly."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _CANCEL_SCRIPT, root, str(tmp_path / "c.npz"), json.dumps(devices)],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = np.load(tmp_path / "c.npz")
    latency, frame, done = float(r["latency"]), float(r["frame"]), int(r["done"])
    print(f"cancel-to-return {latency * 1e3:.2f} ms; frame {frame * 1e3:.1f} ms (batch {frame * 250:.1f} ms); "
          f"checkpoint {done} samples; render: {r['rc']}")
    assert "CANCELLED" in str(r["rc"])
    assert done in (0, 128, 256, 384)
    assert latency < frame / 4
    assert bool(r["equal"])


_TWO_RENDERS_SCRIPT = r'''
import sys, threading, time
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch  # noqa: F401  (HIP runtime first)
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
def tracer(seed):
    rt = GpuRayTracer(960, 540, seed=seed)
    assert rt.load_from_json(load_scene_json("rtow.json"))
    rt.update_render_settings({"maxBounces": 5, "samples": 256})
    return rt
a, b = tracer(3), tracer(4)
ref_a = a.render(want=("mean",), batch_samples=32)["mean"]
ref_b = b.render(want=("mean",), batch_samples=32)["mean"]
lib = capi.load_library()
box = {}
calls = []
def cancel_a(f):                      # A's 3rd progress call cancels A through rt_cancel, B still running
    calls.append(f)
    if len(calls) == 3:
        capi.check(lib.rt_cancel(a.scene_handle()))
    return False
def run(name, rt, cb):
    try:
        box[name] = rt.render(want=("mean",), batch_samples=32, on_progress=cb)["mean"]
    except RuntimeError as e:
        box[name] = str(e)
ta = threading.Thread(target=run, args=("a", a, cancel_a))
tb = threading.Thread(target=run, args=("b", b, None))
tb.start(); ta.start()
ta.join(); tb.join()
sums, done = a.checkpoint()
res_a = tracer(3).render(want=("mean",), resume=(sums, done), batch_samples=32)["mean"]
diff = np.abs(res_a - ref_a)
print("done", done, "a:", box["a"] if isinstance(box["a"], str) else "finished", "resume max|diff|", float(diff.max()),
      "pixels differing", int(np.count_nonzero(diff)), file=sys.stderr)
np.savez(sys.argv[2], a_cancelled=isinstance(box["a"], str) and "cancel" in box["a"].lower(),
         b_equal=(not isinstance(box["b"], str)) and np.array_equal(box["b"], ref_b),
         a_resume_equal=np.array_equal(res_a, ref_a), done=done)
'''


def test_cancel_one_of_two_concurrent_renders(gpu, tmp_path):
    """The in-flight launches a cancel moves are those of the cancelled render only (cancel_pool_launches
    keys them by the scene's cancel word): two progressive renders of two scenes run at once on two
    threads, one is cancelled mid-frame (rt_cancel from its 3rd progress call) — the other finishes
    bit-identical to its own uninterrupted render, and the cancelled one's checkpoint resumes
    bit-exactly."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _TWO_RENDERS_SCRIPT, root, str(tmp_path / "t.npz")],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = np.load(tmp_path / "t.npz")
    print(p.stderr[-600:])
    print(f"cancelled render's checkpoint: {int(r['done'])} samples")
    assert bool(r["a_cancelled"])
    assert bool(r["b_equal"])
    assert bool(r["a_resume_equal"])


_QUEUES_SCRIPT = r'''
import sys, threading, time, ctypes as C
sys.path.insert(0, sys.argv[1])
import numpy as np
import torch
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
def tracer(w, h, spp, seed):
    rt = GpuRayTracer(w, h, seed=seed)
    assert rt.load_from_json(load_scene_json("rtow.json"))
    rt.update_render_settings({"maxBounces": 5, "samples": spp})
    return rt
lib = capi.load_library()
# the long render: 64 one-tile items of 20000 samples each (RT_POOL_CHUNK=20000 in this process), so its
# LDS launch holds its queue pair for a long time on only 16 workgroups, and the small launches run and
# complete beside it: the queue pairs are handed out again and again while it holds its own
big, small = tracer(64, 64, 20000, 7), tracer(32, 32, 2, 9)
assert lib.rt_scene_walk(small.scene_handle(), capi.RT_PREC_F64, 0) == 2      # the grid: LDS pool launches
ref_big = big.render(want=("mean",))["mean"]
n, N = 32 * 32, int(sys.argv[3])
st = small.settings()
one = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
torch.cuda.synchronize()
capi.check(lib.rt_trace_device(small.scene_handle(), C.byref(st), C.c_void_p(one.data_ptr()), None, 1, None))
ref_small = one.cpu().numpy()
bufs = torch.zeros((N, 3 * n), dtype=torch.float64, device="cuda")
side = torch.cuda.Stream()
torch.cuda.synchronize()
box = {}
def long_render():
    box["big"] = big.render(want=("mean",))["mean"]
    box["t"] = time.perf_counter()
th = threading.Thread(target=long_render)
th.start()
time.sleep(0.02)
enq = []
for k in range(N):              # every call enqueues one LDS pool launch on `side`, no host wait
    capi.check(lib.rt_trace_device(small.scene_handle(), C.byref(st), C.c_void_p(bufs[k].data_ptr()),
                                   C.c_void_p(side.cuda_stream), 0, None))
    enq.append(time.perf_counter())
th.join()
torch.cuda.synchronize()
out = bufs.cpu().numpy()
bad = sum(not np.array_equal(out[k], ref_small) for k in range(N))
during = sum(t < box["t"] for t in enq)
print(f"{during} of {N} small launches enqueued while the long render ran; {bad} differ", file=sys.stderr)
np.savez(sys.argv[2], big_equal=np.array_equal(box["big"], ref_big), bad=bad, during=during)
'''


def test_lds_queues_owned_under_concurrent_launches(gpu, tmp_path):
    """every LDS pool launch holds a work queue of its own (queue_slots.h).  One long
    render (one LDS launch of 16 workgroups that runs for a fraction of a second) on one thread, while
    another thread enqueues 2048 small LDS-pool launches of another scene (rt_trace_device, asynchronous,
    on a side stream), which run and complete beside it — twice the 1024 queue pairs, so round 5's ring
    handed the long launch's pair to a small one (whose waves then found its counter past their items).
    Both the long render and every small one are bit-identical to their solo renders."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _QUEUES_SCRIPT, root, str(tmp_path / "q.npz"), "2048"],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, RT_POOL_CHUNK="20000"))
    assert p.returncode == 0, p.stderr[-2000:]
    print(p.stderr[-400:])
    r = np.load(tmp_path / "q.npz")
    assert int(r["during"]) > 1024          # the pairs went round more than once while it ran
    assert int(r["bad"]) == 0
    assert bool(r["big_equal"])


def test_cancel_latency_triangle_scene(gpu, tmp_path):
    """The same in-batch cancel on config 5 (mesh50k 1920x1080 x 256 spp in four batches): its walk runs
    in the one-wave pool kernel, whose workgroups read the cancel word as their item starts (the LDS
    kernels' queue move does not apply).  Round 5: 25 ms against a 114-ms frame — the fused launch's
    remaining one-wave workgroups (~400k) passed through the dispatcher, each reading the word over PCIe
    and writing the host `aborted` word.  Round 6: the word is a device-memory copy set from a
    high-priority stream (an L2 read) and skipping workgroups write nothing: 5 ms (scripts/probe_cancel.py).
    Asserted: rt_render returns within an eighth of a frame and the checkpoint
    resumes bit-exactly."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", _CANCEL_SCRIPT, root, str(tmp_path / "c.npz"), "null", "mesh50k", "256"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = np.load(tmp_path / "c.npz")
    latency, frame, done = float(r["latency"]), float(r["frame"]), int(r["done"])
    print(f"cancel-to-return {latency * 1e3:.2f} ms; frame {frame * 1e3:.1f} ms; checkpoint {done} samples; {r['rc']}")
    assert "CANCELLED" in str(r["rc"])
    assert done in (0, 64, 128, 192)
    assert latency < frame / 8
    assert bool(r["equal"])


def test_config4_rtow_4k_1024spp_sharded(gpu):
    """Config 4 at its full size: RTOW 3840x2160 x 1024 spp (8.5e9 samples).  (1) Through
    rt_trace_device, 8 sample-range shards (the per-GPU work of the 8-GPU split, run one after another
    on this GPU) add up to the single-launch sums (ray-tracer.js:202-206 is a per-pixel sum over
    samples, so only the summation order may differ).  (2) Through rt_render with devices=[0]*8 (the
    C ABI's own split).  (3) Three 16x16 windows of the sharded frame match the oracle at full 1024 spp
    (segment counts identical, means within 1e-12)."""
    import torch
    W, H, S = 3840, 2160, 1024
    rt = _rtow(W, H, S, seed=4)
    lib = capi.load_library()
    scene = rt.scene_handle()
    n = W * H
    full = torch.zeros(n * 3, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    capi.check(lib.rt_trace_device(scene, C.byref(rt.settings()), C.c_void_p(full.data_ptr()), None, 1, None))
    shards = torch.zeros(n * 3, dtype=torch.float64, device="cuda")
    part = torch.zeros(n * 3, dtype=torch.float64, device="cuda")
    for k in range(8):
        part.zero_()
        torch.cuda.synchronize()
        rng = (k * S // 8, (k + 1) * S // 8)
        capi.check(lib.rt_trace_device(scene, C.byref(rt.settings(sample_range=rng)), C.c_void_p(part.data_ptr()), None, 1, None))
        shards += part
    torch.cuda.synchronize()
    a, b = full.cpu().numpy().reshape(H, W, 3), shards.cpu().numpy().reshape(H, W, 3)
    assert np.all(np.isfinite(a))
    assert np.allclose(a, b, rtol=SUM_RTOL, atol=0)
    del full, shards, part
    r = rt.render(want=("mean",), devices=[0] * 8)
    assert np.allclose(r["mean"], a / S, rtol=SUM_RTOL, atol=0)
    for (x0, y0) in ((0, 0), (1900, 1060), (3824, 2144)):
        o = binding.render(rt.packed(), rt.settings(crop=(x0, y0, 16, 16)))
        g = rt.render(want=("mean", "segments"), crop=(x0, y0, 16, 16))
        assert np.array_equal(o["segments"], g["segments"])
        assert rel_err(b[y0:y0 + 16, x0:x0 + 16] / S, o["mean"]) <= 1e-12
    rt.close()


@pytest.mark.parametrize("world,launch", [(2, "torchrun"), (3, "torchrun"), (2, "spawn"), (2, "inproc")])
def test_bench_multi_rank_rehearsal(gpu, tmp_path, world, launch):
    """bench.py's N>1 branches run end to end on the one GPU.  torchrun / spawn: `world` ranks sharing
    device 0 (--dist-backend gloo: RCCL refuses two ranks on one device, so the sums are reduced through
    host memory; everything else — the sample-range split, the barriers, the max-over-ranks time, rank
    0's epilogue and JSON line — is the RCCL path's code), launched by torch.distributed.run or by
    bench.py itself as a plain `python bench.py --gpus N` (spawn).  inproc: one process,
    rt_settings.devices = [0, 0] (the Node drop-in's split: replicas, peer copies, add on device 0).
    Rank 0's frame equals the 1-rank bench's frame up to the order of the partial-sum additions."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--config", "cornell", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-end-to-end", "--no-pmc"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    bench = os.path.join(root, "bench.py")
    one = subprocess.run([sys.executable, bench, *common, "--dump", str(tmp_path / "n1.npz")],
                         env=env, capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stderr[-2000:]
    dump = ["--dump", str(tmp_path / "nw.npz")]
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(29611 + world), bench, "--gpus", str(world),
               "--dist-backend", "gloo", "--bands", "8", *common, *dump]      # the band-by-band reduce
    elif launch == "spawn":
        cmd = [sys.executable, bench, "--gpus", str(world), "--dist-backend", "gloo", *common, *dump]
    else:
        cmd = [sys.executable, bench, "--gpus", str(world), "--mp-mode", "inproc", *common, *dump]
    multi = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert multi.returncode == 0, multi.stderr[-3000:]
    line = json.loads([ln for ln in multi.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world and line["value"] > 0 and "REHEARSAL" in line["config"]["parallelism"]
    if launch == "inproc":
        assert line["mp_mode"] == {"mode": "inproc", "devices": [0] * world}
        pg = line["progressive_16"]                 # the Node drop-in's 16 progressive batches, also timed
        assert pg["batches"] == 16 and pg["value"] > 0 and pg["progress_calls_per_step"] == 15, pg
    else:
        assert line["mp_mode"]["mode"] == "ranks" and line["mp_mode"]["world_size"] == world
        assert line["mp_mode"]["reduce_bands"] == (8 if launch == "torchrun" else 0)
    a, b = np.load(tmp_path / "n1.npz"), np.load(tmp_path / "nw.npz")
    assert int(a["samples"]) == int(b["samples"]) == 64
    assert np.allclose(a["sum"], b["sum"], rtol=SUM_RTOL, atol=1e-300)
    flips = int(np.sum(a["rgba8"] != b["rgba8"]))    # summation order only: as test_sample_order_vs_pool_rgba8_full_size
    print(f"RGBA8 bytes differing from the 1-rank frame: {flips} of {a['rgba8'].size}")
    assert flips <= 1e-5 * a["rgba8"].size


def test_bench_rccl_world_size_1(gpu, tmp_path):
    """bench.py's RCCL branch on the one GPU.  Under torch.distributed.run with one
    rank, init_process_group("nccl", device_id=cuda:0) and dist.reduce of the CUDA float64 sums run
    through RCCL exactly as at N=8 (distributed.reduce_sums); the frame equals the plain 1-GPU bench's
    bit for bit (a one-rank reduce is the identity)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bench = os.path.join(root, "bench.py")
    common = ["--config", "cornell", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-end-to-end", "--no-pmc"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    one = subprocess.run([sys.executable, bench, *common, "--dump", str(tmp_path / "n1.npz")],
                         env=env, capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stderr[-2000:]
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    for bands in (0, 8):        # 8: the N > 1 default, every band reduced through RCCL as it completes
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
               "127.0.0.1", "--master-port", str(port + bands), bench, "--gpus", "1", "--dist-backend", "nccl",
               *common, "--bands", str(bands), "--dump", str(tmp_path / "r1.npz")]
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        assert line["mp_mode"]["mode"] == "ranks" and line["mp_mode"]["world_size"] == 1
        assert line["mp_mode"]["reduce_bands"] == bands
        assert line["mp_mode"]["backend"] == "nccl" and line["n_gpus"] == 1 and line["value"] > 0
        a, b = np.load(tmp_path / "n1.npz"), np.load(tmp_path / "r1.npz")
        assert np.array_equal(a["sum"], b["sum"]) and np.array_equal(a["rgba8"], b["rgba8"]), bands


def test_multi_device_distinct_gpus(gpu):
    """rt_settings.devices over DISTINCT devices (peer access enabled by the library, sums copied over
    xGMI): equal to one device up to summation order.  Needs >= 2 visible GPUs."""
    n = C.c_int()
    capi.check(capi.load_library().rt_device_count(C.byref(n)))
    if n.value < 2:
        pytest.skip(f"{n.value} HIP device visible: the distinct-device split needs 2 (the 8-GPU node's run)")
    rt = _rtow(160, 90, 24)
    want = ("mean", "segments", "draws")
    one = rt.render(want=want)
    devs = list(range(min(n.value, 8)))
    many = rt.render(want=want, devices=devs, batch_samples=5)
    for k in ("segments", "draws"):
        assert np.array_equal(one[k], many[k]), k
    assert np.allclose(one["mean"], many["mean"], rtol=SUM_RTOL, atol=0)
    rt.close()


_TREE_PROOF_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
import torch  # noqa: F401  (HIP runtime first)
import hostcheck_binding as hb
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
from test_gpu_parity import _closest_hits
rt = GpuRayTracer(64, 36, seed=3)
assert rt.load_from_json(load_scene_json("rtow.json"))
r, ht, hk, hi = hb.bvh_rays(rt.packed(), 200000, 99, 0)
bt, bk, bi = _closest_hits(rt, r, capi.RT_PREC_F64, capi.RT_ACCEL_BRUTE)
vt, vk, vi = _closest_hits(rt, r, capi.RT_PREC_F64, capi.RT_ACCEL_BVH)
np.savez(sys.argv[2], bt=bt, bk=bk, bi=bi, vt=vt, vk=vk, vi=vi)
'''


@pytest.mark.parametrize("walk", ["tree", "grid", "grid_global"])
def test_rtow_walks_closest_hit_identical_on_device(gpu, tmp_path, walk):
    """RTOW's two sphere walks, each forced in a child process (the trace kernel uses the grid there,
    its records in LDS; grid_global: read from global memory, RT_LDS_GRID=0), on the host check's 200k
    adversarial rays through rt_closest_hits: device walk == device World order, bit for bit (t, kind,
    index)."""
    env = {"RT_BVH_WALK": walk.split("_")[0]}
    if walk == "grid_global":
        env["RT_LDS_GRID"] = "0"
    res = _render_in_child(_TREE_PROOF_SCRIPT, tmp_path / f"{walk}.npz", **env)
    assert (res["bk"] >= 0).sum() > len(res["bk"]) // 10
    assert np.array_equal(res["bk"], res["vk"]) and np.array_equal(res["bi"], res["vi"])
    assert np.array_equal(res["bt"].view(np.uint64), res["vt"].view(np.uint64))


def _closest_hits(rt, rays, precision, accel):
    lib = capi.load_library()
    n = len(rays)
    rays = np.ascontiguousarray(rays, dtype=np.float64)
    t = np.zeros(n)
    kind = np.zeros(n, dtype=np.int32)
    idx = np.zeros(n, dtype=np.int32)
    capi.check(lib.rt_closest_hits(rt.scene_handle(), precision, accel, rays.ctypes.data_as(C.POINTER(C.c_double)), n,
                                   t.ctypes.data_as(C.POINTER(C.c_double)), kind.ctypes.data_as(C.POINTER(C.c_int32)),
                                   idx.ctypes.data_as(C.POINTER(C.c_int32))))
    return t, kind, idx


@pytest.mark.parametrize("scene,rays,host_rays", [("rtow.json", 200_000, 200_000), ("kitchen_sink.json", 200_000, 200_000),
                                                  ("sample_mesh.json", 200_000, 200_000), ("cornell.json", 200_000, 200_000),
                                                  ("mesh50k", 200_000, 4_000)])
def test_bvh_closest_hit_identical_on_device(gpu, scene, rays, host_rays):
    """The BVH's bit-identity proof (bvh_conservative_bound, sphere_filter_bound) checked on the
    instructions the GPU runs — v_rcp_f32 / v_rsq_f32 in the binary32 pre-tests, the device's binary64
    sqrt and division: tests/test_hostcheck.py's adversarial rays (near-tangent spheres, triangle edges
    and vertices) through rt_closest_hits.  Device BVH == device World-order walk, bit for bit, on every
    ray; the device World-order walk == the host's (the kernel's code compiled for the CPU) on the first
    `host_rays`.  Binary32 mode is reported, not proven: these rays are near-tangent to 1e-2 .. 1e-12,
    far below binary32's resolution, where a binary32 root (error ~2^-12 relative near tangency) falls
    outside the node margins sized for binary64 ones — 9 % of RTOW's rays differ, while rendered images
    agree (test_bvh_bit_identical_to_brute_mesh50k, test_f32_rms*); >= 80 % is asserted as a sanity
    bound."""
    import hostcheck_binding as hb
    rt = GpuRayTracer(64, 36, seed=3)
    assert rt.load_from_json(load_scene_json(scene))
    r, ht, hk, hi = hb.bvh_rays(rt.packed(), rays, 99, host_rays)
    assert len(r) > rays * 0.9
    bt, bk, bi = _closest_hits(rt, r, capi.RT_PREC_F64, capi.RT_ACCEL_BRUTE)
    vt, vk, vi = _closest_hits(rt, r, capi.RT_PREC_F64, capi.RT_ACCEL_BVH)
    hit = bk >= 0
    print(f"{scene}: {len(r)} rays, {int(hit.sum())} hits")
    assert hit.sum() > len(r) // 10
    assert np.array_equal(bk, vk) and np.array_equal(bi, vi)
    assert np.array_equal(bt.view(np.uint64), vt.view(np.uint64))
    m = min(host_rays, len(r))
    assert np.array_equal(hk[:m], bk[:m]) and np.array_equal(hi[:m], bi[:m])
    assert np.array_equal(ht[:m].view(np.uint64), bt[:m].view(np.uint64))
    ft, fk, fi = _closest_hits(rt, r, capi.RT_PREC_F32, capi.RT_ACCEL_BRUTE)
    gt, gk, gi = _closest_hits(rt, r, capi.RT_PREC_F32, capi.RT_ACCEL_BVH)
    same32 = (fk == gk) & (fi == gi) & (ft.view(np.uint64) == gt.view(np.uint64))
    print(f"{scene}: binary32 BVH vs brute force differ on {int((~same32).sum())} of {len(r)} rays")
    assert same32.mean() >= 0.8
    rt.close()


def test_sample_order_mode(gpu):
    """rt_settings.sum_order = RT_SUM_SAMPLE_ORDER (one lane per pixel adding its samples in sample
    order, the reference's loop order, ray-tracer.js:202-206): the sums do not depend on how the samples
    are batched (bit-identical with and without batches, and to the RT_SAMPLE_POOL=0 kernel), the path
    decisions equal the pool's, and the sums differ from the pool's only by summation order."""
    rt = _rtow(96, 54, 12)
    pool = rt.render(want=("mean", "segments", "draws"))
    rt.sum_order = capi.RT_SUM_SAMPLE_ORDER
    a = rt.render(want=("mean", "segments", "draws"))
    b = rt.render(want=("mean",), batch_samples=5)
    assert np.array_equal(a["mean"], b["mean"])
    assert np.array_equal(a["segments"], pool["segments"]) and np.array_equal(a["draws"], pool["draws"])
    assert np.allclose(a["mean"], pool["mean"], rtol=SUM_RTOL, atol=0)
    rt.close()


def test_sample_order_vs_pool_rgba8_full_size(gpu):
    """how often the pool's summation order flips an RGBA8 byte against the sample-order sum,
    measured on config 3's full 1920x1080 frame (64 spp: the same pool chunking rule as 512).  A flip
    needs a pixel's binary64 mean within ~1e-16 relative of a floor(c*255) boundary after tone mapping
    and gamma; bound asserted: <= 1e-5 of the bytes (observed count printed)."""
    rt = _rtow(1920, 1080, 64, seed=21)
    pool = rt.render(want=("mean",))
    rt.sum_order = capi.RT_SUM_SAMPLE_ORDER
    ordered = rt.render(want=("mean",))
    diff = int(np.sum(pool["rgba8"] != ordered["rgba8"]))
    print(f"RGBA8 bytes differing, pool vs sample order, 1920x1080x64: {diff} of {pool['rgba8'].size}")
    assert np.allclose(pool["mean"], ordered["mean"], rtol=SUM_RTOL, atol=0)
    assert diff <= 1e-5 * pool["rgba8"].size
    rt.close()


def test_progressive_preview_and_cancel(gpu):
    """The reference repaints after every row and stops on window.renderCancelled leaving the rows done
    (ray-tracer.js:224-264).  Here: 16 sample batches give 16 monotone progress calls; the preview frame
    (rt_output.preview_rgba8) at the last progress call (30 of 32 samples) equals a render of exactly
    those 30 samples with the same batches; a cancel leaves the frame of the checkpointed samples, again
    equal to a render of exactly those samples."""
    rt = _rtow(128, 72, 32, seed=6)
    fr = []
    res = rt.render(want=("preview",), batch_samples=2, on_progress=lambda f: fr.append(f) and False)
    assert len(fr) >= 16 and all(x < y for x, y in zip(fr, fr[1:])) and fr[-1] == 1.0
    rt30 = _rtow(128, 72, 30, seed=6)
    # running frames come from preview_kernel (gamma thresholds instead of a binary64 pow, pt_trace.hip):
    # the same bytes as the exact epilogue
    assert np.array_equal(res["preview"], rt30.render(batch_samples=2)["rgba8"])
    assert not np.array_equal(res["preview"], res["rgba8"])
    rt30.close()
    calls = []
    with pytest.raises(RuntimeError, match="CANCELLED"):
        rt.render(want=("preview",), batch_samples=2, on_progress=lambda f: calls.append(f) or len(calls) >= 5)
    sums, done = rt.checkpoint()
    assert done % 2 == 0 and 10 <= done <= 16                    # 5 batches + those of the 3 queued reduced first
    cancelled = rt.image_data.copy()
    rt2 = _rtow(128, 72, done, seed=6)                           # exactly the checkpointed samples
    ref = rt2.render(batch_samples=2)
    assert np.array_equal(cancelled, ref["rgba8"])
    assert np.array_equal(sums, rt2.checkpoint()[0])
    rt.close()
    rt2.close()


_BATCH_SCRIPT = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import torch  # noqa: F401  (HIP runtime first)
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
out = {}
for name, w, h, spp, batch, devices in (("rtow.json", 160, 90, 24, 3, None), ("rtow.json", 160, 90, 24, 5, None),
                                        ("rtow.json", 160, 90, 24, 5, [0, 0]),
                                        ("mesh50k", 1920, 1080, 8, 2, None), ("cornell.json", 64, 48, 17, 4, None)):
    rt = GpuRayTracer(w, h, seed=12)
    assert rt.load_from_json(load_scene_json(name))
    rt.update_render_settings({"samples": spp, "maxBounces": 5})
    crop = (900, 480, 64, 48) if name == "mesh50k" else None
    r = rt.render(crop=crop, want=("mean",), batch_samples=batch, devices=devices)
    out[f"{name}.{batch}.{devices}"] = r["mean"]
np.savez(sys.argv[2], **out)
'''


def test_overlapped_batches_equal_serial_batches(gpu, tmp_path):
    """Batches traced in one fused launch (items batch-major, each batch reduced once its items are done)
    and batches traced on three streams into their own chunk partials (RT_FUSED_BATCHES=0: the next
    batch's waves fill the CUs while this one drains; reduces in batch order) give the same bits as the
    same batches run one after the other (forced here by a 1-MiB partials budget, too small for two
    slots): ragged last batches, a triangle BVH, and the whole-batch split over two devices (== the same
    batches one after the other on one device)."""
    over = _render_in_child(_BATCH_SCRIPT, tmp_path / "over.npz")                 # one device: fused batches
    unfused = _render_in_child(_BATCH_SCRIPT, tmp_path / "unfused.npz", RT_FUSED_BATCHES="0")   # a launch per batch
    serial = _render_in_child(_BATCH_SCRIPT, tmp_path / "serial.npz", RT_PART_MB="1")
    two = "rtow.json.5.[0, 0]"          # the whole-batch split (two devices) == the same batches on one
    for k in over.files:
        ref = serial["rtow.json.5.None"] if k == two else serial[k]
        assert np.array_equal(over[k], ref, equal_nan=True), k
        assert np.array_equal(unfused[k], ref, equal_nan=True), k


@pytest.mark.parametrize("gamma", [2.2, 1.0, 0.45, 3.7, 0.25, 4.0, 50.0])
def test_preview_thresholds_match_finalize(gpu, gamma):
    """preview_kernel's RGBA8 bytes (the count of gamma thresholds T_k <= tm, T_k computed with the
    device's own binary64 pow) against finalize_kernel's floor(255 pow(max(0, tm), 1/gamma)) on tone-mapped
    values within +-3000 ulps of every threshold (where a non-monotone pow or an off-by-one search would
    show), plus random, negative, zero, huge, infinite and NaN values: rt_finalize_device with RGBA8 only
    takes the threshold kernel, with the Float32 frame requested too finalize_kernel (linear tone map,
    exposure 1, one sample: tm = the sum).  0.25 and 4.0 are the ends of the range whose tables are used
    (kGammaMin / kGammaMax, pt_launch.h); gamma 50 lies outside it, so both calls take finalize_kernel
    (a non-monotone region wider than the exception scan would otherwise go unseen)."""
    import torch
    k = np.arange(1, 256, dtype=np.float64)
    approx = (k / 255.0) ** gamma                                  # T_k up to a few ulps
    steps = np.arange(-3000, 3001, dtype=np.int64)
    near = (approx.view(np.int64)[:, None] + steps[None, :]).ravel().view(np.float64)
    rng = np.random.default_rng(2)
    extra = np.concatenate([rng.uniform(-0.5, 1.5, 200_000), 10.0 ** rng.uniform(-30, 30, 100_000),
                            [0.0, -0.0, -1.0, 1.0, np.inf, -np.inf, np.nan, 5e-324, 1e300]])
    tm = np.concatenate([near, extra])
    n = -(-tm.size // 3)
    tm = np.concatenate([tm, np.zeros(3 * n - tm.size)])
    lib = capi.load_library()
    rt = _rtow(n, 1, 1, seed=1)
    rt.tone_mapping, rt.exposure, rt.gamma = "linear", 1.0, gamma
    scene = rt.scene_handle()
    st = rt.settings()
    d_sum = torch.from_numpy(tm).cuda()
    fast = torch.zeros(4 * n, dtype=torch.uint8, device="cuda")
    exact = torch.zeros(4 * n, dtype=torch.uint8, device="cuda")
    post = torch.zeros(4 * n, dtype=torch.float32, device="cuda")
    capi.check(lib.rt_finalize_device(scene, C.byref(st), C.c_void_p(d_sum.data_ptr()), None, None,
                                      C.c_void_p(fast.data_ptr()), None))
    capi.check(lib.rt_finalize_device(scene, C.byref(st), C.c_void_p(d_sum.data_ptr()), None,
                                      C.c_void_p(post.data_ptr()), C.c_void_p(exact.data_ptr()), None))
    torch.cuda.synchronize()
    f, e = fast.cpu().numpy(), exact.cpu().numpy()
    assert np.array_equal(f, e), int(np.count_nonzero(f != e))
    assert len(np.unique(e)) == 256                                 # every byte value was exercised
    rt.close()

