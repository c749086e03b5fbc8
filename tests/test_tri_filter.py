"""The binary32 triangle pre-filter of the exact (f64) mode never rejects a triangle the binary64 test
accepts (pt_core.h tri_filter_bound): adversarial rays through edges and vertices, at the |A| = 1e-4
threshold, at t = tmin and at the current best hit's t, over 7 decades of scale."""
import ctypes as C

import hostcheck_binding as hb


def test_tri_filter_is_conservative():
    lib = hb.lib()
    lib.ptc_tri_filter_check.argtypes = [C.c_longlong, C.c_uint, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.ptc_tri_filter_check.restype = C.c_longlong
    rej, passed = C.c_double(), C.c_double()
    violations = lib.ptc_tri_filter_check(3_000_000, 2024, C.byref(rej), C.byref(passed))
    assert violations == 0
    # the filter must also be useful: most binary64 rejections of these near-boundary cases are its too
    assert rej.value > 0.5
    print(f"binary64 rejections also rejected by the filter: {rej.value:.3f}; passed: {passed.value:.3f}")
