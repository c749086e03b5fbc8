"""The GPU kernel's own per-lane code (pt_path.h / pt_core.h / scene_pack.h), compiled for the CPU
by tests/hostcheck, against the reference's golden fixtures.  This separates algorithm bugs (caught
here, on CPU) from GPU code-generation problems (caught only by tests/test_gpu_parity.py)."""
import numpy as np
import pytest

import golden_cases as gc
import hostcheck_binding as hb
from blenderraytracer_amd import capi
from oracle import binding


@pytest.mark.parametrize("case", gc.case_names())
def test_kernel_logic_f64_matches_reference(case):
    rt, c = gc.tracer_for(case)
    r = hb.render(rt.packed(), rt.settings(crop=c["crop"]))
    assert np.array_equal(r["segments"], gc.load_array(case, "segs"))
    assert np.array_equal(r["draws"], gc.load_array(case, "draws"))
    lin = gc.load_array(case, "linear")
    assert np.array_equal(np.isnan(r["mean"]), np.isnan(lin))
    ok = ~np.isnan(lin)
    assert np.all(np.abs(r["mean"][ok] - lin[ok]) <= 1e-12 * np.maximum(1, np.abs(lin[ok])))


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
