"""Diagnose GPU-vs-reference differences on golden cases: mismatching pixels, segment/draw diffs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import golden_cases as gc  # noqa: E402
from blenderraytracer_amd import capi  # noqa: E402

prec = capi.RT_PREC_F64 if os.environ.get("PREC", "f64") == "f64" else capi.RT_PREC_F32
for case in sys.argv[1:] or gc.case_names():
    rt, c = gc.tracer_for(case, precision=prec)
    r = rt.render(crop=c["crop"], want=("mean", "segments", "draws"))
    lin = gc.load_array(case, "linear")
    segs, draws = gc.load_array(case, "segs"), gc.load_array(case, "draws")
    nan_bad = np.argwhere(np.isnan(r["mean"][..., 0]) != np.isnan(lin[..., 0]))
    seg_bad = np.argwhere(r["segments"] != segs)
    draw_bad = np.argwhere(r["draws"] != draws)
    ok = ~(np.isnan(lin) | np.isnan(r["mean"]))
    err = np.max(np.abs(r["mean"][ok] - lin[ok])) if ok.any() else 0
    print(f"{case}: nan-mismatch {len(nan_bad)} seg-mismatch {len(seg_bad)} draw-mismatch {len(draw_bad)} max|d| {err:.2e}")
    for y, x in seg_bad[:5]:
        print(f"   pixel crop({x},{y}) segs gpu {r['segments'][y, x]} ref {segs[y, x]} draws gpu {r['draws'][y, x]} ref {draws[y, x]}")
    rt.close()
