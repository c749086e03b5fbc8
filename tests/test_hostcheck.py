"""The GPU kernel's own per-lane code (pt_path.h / pt_core.h / scene_pack.h), compiled for the CPU
by tests/hostcheck, against the reference's golden fixtures.  This separates algorithm bugs (caught
here, on CPU) from GPU code-generation problems (caught only by tests/test_gpu_parity.py)."""
import ctypes as C
import math
import numpy as np
import pytest

import golden_cases as gc
import hostcheck_binding as hb
from blenderraytracer_amd import capi
from oracle import binding


@pytest.mark.parametrize("case", gc.case_names(heavy=False))   # heavy cases: the BVH walks below
def test_kernel_logic_f64_matches_reference(case):
    rt, c = gc.tracer_for(case)
    r = hb.render(rt.packed(), rt.settings(crop=c["crop"]))
    assert np.array_equal(r["segments"], gc.load_array(case, "segs"))
    assert np.array_equal(r["draws"], gc.load_array(case, "draws"))
    lin = gc.load_array(case, "linear")
    assert np.array_equal(np.isnan(r["mean"]), np.isnan(lin))
    ok = ~np.isnan(lin)
    assert np.array_equal(r["mean"][ok], lin[ok])     # bit for bit (trace_pixel: the recursion's order)


def test_kernel_logic_sample_ranges_and_crops():
    rt, c = gc.tracer_for("kitchen_sink")
    full = hb.render(rt.packed(), rt.settings())
    st = rt.settings(crop=(7, 5, 20, 11))
    crop = hb.render(rt.packed(), st)
    assert np.array_equal(full["mean"][5:16, 7:27], crop["mean"])
    a = hb.render(rt.packed(), rt.settings(sample_range=(0, 3)))
    b = hb.render(rt.packed(), rt.settings(sample_range=(3, rt.samples)))
    assert np.allclose(a["mean"] + b["mean"], full["mean"], rtol=1e-13, atol=1e-15)
    assert np.array_equal(a["segments"] + b["segments"], full["segments"])


def test_kernel_logic_f32_close_to_oracle():
    rt, c = gc.tracer_for("rtow_small", precision=capi.RT_PREC_F32)
    r = hb.render(rt.packed(), rt.settings())
    o = binding.render(rt.packed(), rt.settings())
    assert np.all(np.isfinite(r["mean"]))
    assert np.sqrt(np.mean((r["mean"] - o["mean"]) ** 2)) < 0.05


@pytest.mark.parametrize("walk", ["two-child", "stackless"])
@pytest.mark.parametrize("case", gc.case_names())
def test_kernel_logic_bvh_matches_reference(case, walk):
    """RT_ACCEL_BVH (closest_hit_bvh: the ordered two-child walk of the kernel, and the stackless
    preorder walk) gives the same decisions as World.hit on every golden case."""
    rt, c = gc.tracer_for(case)
    rt.accel = {"two-child": capi.RT_ACCEL_BVH, "stackless": 3}[walk]   # 3: hostcheck-only
    r = hb.render(rt.packed(), rt.settings(crop=c["crop"]))
    assert np.array_equal(r["segments"], gc.load_array(case, "segs"))
    assert np.array_equal(r["draws"], gc.load_array(case, "draws"))
    lin = gc.load_array(case, "linear")
    assert np.array_equal(np.isnan(r["mean"]), np.isnan(lin))
    ok = ~np.isnan(lin)
    assert np.array_equal(r["mean"][ok], lin[ok])     # bit for bit (trace_pixel: the recursion's order)


@pytest.mark.parametrize("scene,rays", [("rtow.json", 200_000), ("kitchen_sink.json", 200_000),
                                        ("sample_mesh.json", 200_000), ("cornell.json", 200_000), ("mesh50k", 4_000)])
def test_bvh_closest_hit_identical_on_adversarial_rays(scene, rays):
    """Near-tangent sphere rays and rays through triangle edges/vertices: the BVH walk returns the
    bit-identical (t, primitive) of the World-order walk (bvh_conservative_bound in pt_core.h)."""
    from blenderraytracer_amd.renderer import GpuRayTracer
    from blenderraytracer_amd.scene import load_scene_json
    rt = GpuRayTracer(64, 36, seed=3)
    assert rt.load_from_json(load_scene_json(scene))
    bad, hits = hb.bvh_check(rt.packed(), rays, 99)
    assert hits > rays // 10
    assert bad == 0


def test_bvh_depth_cap_forces_median_splits():
    """The builder keeps every leaf within the traversal stack (RT_BVH_STACK entries): with the cap
    lowered to 10 (hostcheck variant) the 486-sphere RTOW tree (one sphere per leaf) is re-split to
    depth <= 10 and still renders bit-identically to the World-order walk."""
    from blenderraytracer_amd.renderer import GpuRayTracer
    from blenderraytracer_amd.scene import load_scene_json
    import ctypes as C
    rt = GpuRayTracer(64, 36, seed=3)
    assert rt.load_from_json(load_scene_json("rtow.json"))
    depth_full = hb.bvh_info(rt.packed())[0]
    capped = hb.lib(("RT_BVH_STACK=10",))
    depth_cap = hb.bvh_info(rt.packed(), capped)[0]
    assert depth_full > 10 >= depth_cap
    hits = C.c_longlong()
    assert capped.ptc_bvh_check(C.byref(rt.packed().desc), 50_000, 7, C.byref(hits)) == 0 and hits.value > 5000


def test_dominant_spheres_rtow():
    """scene_pack.h peel_big_spheres: on RTOW the spheres above 1/64 of the other spheres' box area are
    the R = 1000 ground and the three r = 1 spheres, taken out of the tree largest first (tested before
    the walk); every other sphere stays in the tree.  The closest hit is unchanged (the BVH-vs-World
    checks above run on the same build)."""
    from blenderraytracer_amd.renderer import GpuRayTracer
    from blenderraytracer_amd.scene import load_scene_json
    rt = GpuRayTracer(64, 36, seed=3)
    assert rt.load_from_json(load_scene_json("rtow.json"))
    p = rt.packed()
    radii = [o.g[3] for o in p.objects if o.type == 0]
    big = hb.bvh_shape(p)[2]
    assert [abs(radii[i]) for i in big] == [1000.0, 1.0, 1.0, 1.0]
    assert max(abs(r) for i, r in enumerate(radii) if i not in big) < 1.0


def test_away_rejection_is_exact():
    """sphere_candidate's early rejections (origin outside or on the sphere moving away; origin just
    inside it moving away, the far root then below tMin — pt_core.h `leave`) never change the decision or
    t of the reference's full binary64 test (geometry.js:15-45, restated in the host check): 2 M rays,
    half of them leaving a sphere from a binary64 hit point (a quarter nearly tangent), radii from 1e-3 to
    1e7 including the RTOW ground's R = 1000 and negative radii."""
    import ctypes as C
    taken = C.c_longlong()
    assert hb.lib().ptc_away_check(2_000_000, 11, C.byref(taken)) == 0
    assert taken.value > 300_000          # the shortcut is exercised


def test_pow5_correctly_rounded():
    """pow5_rn (Schlick's Math.pow(1 - cosine, 5) in the kernel, pt_path.h) is the correctly rounded
    x^5 (exact rational arithmetic) on 100k arguments 1 - c over the dielectric's range of cosines,
    tiny and exact ones.  libm pow (glibc, <= 0.52 ulp; V8's fdlibm pow is likewise not always
    correctly rounded) differs by 1 ulp in <= 0.1 % of near-midpoint cases, as the device pow did."""
    from fractions import Fraction
    L = hb.lib()
    L.ptc_pow5.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_longlong]
    rng = np.random.default_rng(5)
    c = np.concatenate([rng.uniform(-1.0, 1.0, 60_000), 1.0 - rng.uniform(0, 1e-3, 20_000),
                        rng.uniform(0, 1, 20_000) ** 8])
    x = np.concatenate([1.0 - c, [0.0, 1.0, 2.0, 2.0 ** -53, 0.5, 1.5, 1e-16]])
    out = np.empty_like(x)
    L.ptc_pow5(x.ctypes.data_as(C.POINTER(C.c_double)), out.ctypes.data_as(C.POINTER(C.c_double)), len(x))
    exact = np.array([float(Fraction(v) ** 5) for v in x])      # float(Fraction) rounds correctly
    assert np.array_equal(out, exact), int(np.sum(out != exact))
    libm = np.array([math.pow(v, 5) for v in x])
    diff = out != libm
    assert diff.mean() <= 1e-3
    assert np.all(np.abs(out[diff] - libm[diff]) <= np.spacing(np.abs(libm[diff])))

