"""The binary32 sphere pre-filter of the exact (f64) mode never rejects a sphere the binary64 test
accepts (pt_core.h sphere_filter_bound): adversarial near-tangent rays over 7 decades of scale."""
import ctypes as C

import hostcheck_binding as hb


def test_filter_bound_is_conservative():
    lib = hb.lib()
    lib.ptc_sphere_filter_check.argtypes = [C.c_longlong, C.c_uint, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    worst, frac = C.c_double(), C.c_double()
    violations = lib.ptc_sphere_filter_check(2_000_000, 12345, C.byref(worst), C.byref(frac))
    assert violations == 0
    # the analysis gives |X - Y| <= 27 u Q (u = 2^-24, pt_core.h sphere_filter_bound); the margin is 128 u Q
    assert worst.value <= 27 * 2.0 ** -24
    print(f"max |X-Y|/Q = {worst.value / 2.0 ** -24:.2f} u; near-tangent misses rejected {frac.value:.3f}")
