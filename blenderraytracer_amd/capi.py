"""ctypes mirror of include/rt_hip.h and the loader for the in-tree librt_hip.so.

The product path has no CPU fallback: if the HIP library is missing or no GPU is visible,
every entry point raises (RuntimeError) instead of computing anything on the host.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "librt_hip.so")

RT_ABI_VERSION = 3
RT_MAX_DEVICES = 8

# enums (include/rt_hip.h)
RT_OBJ_SPHERE, RT_OBJ_PLANE, RT_OBJ_BOX, RT_OBJ_TRIANGLE, RT_OBJ_MESH = range(5)
RT_MAT_LAMBERTIAN, RT_MAT_METAL, RT_MAT_DIELECTRIC, RT_MAT_EMISSIVE = range(4)
RT_BG_GRADIENT, RT_BG_SOLID, RT_BG_HDRI, RT_BG_PROCEDURAL_SKY, RT_BG_NAN = range(5)
RT_CAM_PERSPECTIVE, RT_CAM_ORTHOGRAPHIC = range(2)
RT_AA_SUPERSAMPLING, RT_AA_STOCHASTIC, RT_AA_CENTER = range(3)
RT_TM_REINHARD, RT_TM_ACES, RT_TM_LINEAR = range(3)
RT_PREC_F64, RT_PREC_F32 = range(2)
RT_ACCEL_AUTO, RT_ACCEL_BRUTE, RT_ACCEL_BVH = range(3)
RT_SUM_POOL, RT_SUM_SAMPLE_ORDER = range(2)

STATUS = {0: "RT_OK", -1: "RT_ERR_INVALID", -2: "RT_ERR_DEVICE", -3: "RT_ERR_NOMEM",
          -4: "RT_ERR_CANCELLED", -5: "RT_ERR_NO_DEVICE"}


class MaterialDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("_pad", C.c_int32), ("albedo", C.c_double * 3),
                ("roughness", C.c_double), ("ior", C.c_double), ("emission", C.c_double * 3)]


class ObjectDesc(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("first", C.c_int32),
                ("count", C.c_int32), ("g", C.c_double * 6)]


class CameraDesc(C.Structure):
    _fields_ = [("origin", C.c_double * 3), ("lower_left", C.c_double * 3), ("horizontal", C.c_double * 3),
                ("vertical", C.c_double * 3), ("u", C.c_double * 3), ("v", C.c_double * 3),
                ("w", C.c_double * 3), ("lens_radius", C.c_double), ("type", C.c_int32), ("_pad", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("num_objects", C.c_int32), ("objects", C.POINTER(ObjectDesc)),
                ("num_materials", C.c_int32), ("num_triangles", C.c_int32),
                ("materials", C.POINTER(MaterialDesc)), ("triangles", C.POINTER(C.c_double)),
                ("camera", CameraDesc), ("background", C.c_int32), ("_pad", C.c_int32),
                ("sky_intensity", C.c_double), ("solid_color", C.c_double * 3), ("perm", C.c_int32 * 512)]


class Settings(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("samples", C.c_int32), ("max_depth", C.c_int32),
                ("aa_mode", C.c_int32), ("tone_map", C.c_int32), ("exposure", C.c_double), ("gamma", C.c_double),
                ("seed", C.c_uint32), ("sample_begin", C.c_int32), ("sample_end", C.c_int32),
                ("crop_x0", C.c_int32), ("crop_y0", C.c_int32), ("crop_w", C.c_int32), ("crop_h", C.c_int32),
                ("precision", C.c_int32), ("batch_samples", C.c_int32), ("denoise", C.c_int32),
                ("denoise_weights", C.c_double * 2), ("accel", C.c_int32), ("device_count", C.c_int32),
                ("devices", C.c_int32 * 8), ("sum_order", C.c_int32)]


class Output(C.Structure):
    _fields_ = [("mean", C.POINTER(C.c_double)), ("post", C.POINTER(C.c_float)), ("rgba8", C.POINTER(C.c_uint8)),
                ("segments", C.POINTER(C.c_uint32)), ("draws", C.POINTER(C.c_uint32)),
                ("preview_rgba8", C.POINTER(C.c_uint8)), ("preview_samples", C.POINTER(C.c_int32))]


class Stats(C.Structure):
    _fields_ = [("kernel_ms", C.c_double), ("finalize_ms", C.c_double), ("wall_ms", C.c_double),
                ("samples", C.c_uint64), ("segments", C.c_uint64), ("prim_tests", C.c_uint64),
                ("algorithmic_bytes", C.c_double), ("node_visits", C.c_uint64),
                ("sphere_tests", C.c_uint64), ("tri_tests", C.c_uint64)]


PROGRESS_FN = C.CFUNCTYPE(C.c_int, C.c_double, C.c_void_p)
BAND_FN = C.CFUNCTYPE(C.c_int, C.c_int32, C.c_int32, C.c_int32, C.c_void_p)   # rt_band_fn

# every symbol include/rt_hip.h declares (checked by tests/test_capi_symbols.py)
EXPORTS = {
    "rt_abi_version": (C.c_int, []),
    "rt_last_error": (C.c_char_p, []),
    "rt_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "rt_scene_create": (C.c_int, [C.POINTER(SceneDesc), C.c_int, C.POINTER(C.c_void_p)]),
    "rt_scene_destroy": (None, [C.c_void_p]),
    "rt_render": (C.c_int, [C.c_void_p, C.POINTER(Settings), C.POINTER(Output), PROGRESS_FN, C.c_void_p,
                            C.POINTER(Stats)]),
    "rt_trace_device": (C.c_int, [C.c_void_p, C.POINTER(Settings), C.c_void_p, C.c_void_p, C.c_int,
                                  C.POINTER(Stats)]),
    "rt_trace_device_bands": (C.c_int, [C.c_void_p, C.POINTER(Settings), C.c_void_p, C.c_void_p, C.c_int32, BAND_FN,
                                        C.c_void_p, C.POINTER(Stats)]),
    "rt_finalize_device": (C.c_int, [C.c_void_p, C.POINTER(Settings), C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p]),
    "rt_cancel": (C.c_int, [C.c_void_p]),
    "rt_closest_hits": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_double), C.c_size_t,
                                  C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rt_scene_walk": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "rt_render_checkpoint": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_size_t, C.POINTER(C.c_int32)]),
    "rt_render_resume": (C.c_int, [C.c_void_p, C.POINTER(Settings), C.POINTER(C.c_double), C.c_int32,
                                   C.POINTER(Output), PROGRESS_FN, C.c_void_p, C.POINTER(Stats)]),
    # include/rt_scene_json.h (host-only scene-JSON loader)
    "rt_json_scene_load": (C.c_int, [C.c_char_p, C.c_size_t, C.c_int32, C.c_int32, C.c_uint32, C.POINTER(C.c_void_p)]),
    "rt_json_scene_desc": (C.POINTER(SceneDesc), [C.c_void_p]),
    "rt_json_scene_size": (None, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "rt_json_scene_destroy": (None, [C.c_void_p]),
}

_lib = None


def load_library(path=None):
    """Load librt_hip.so (built by __graft_entry__.build() / blenderraytracer_amd/build.py)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("RT_HIP_LIB", LIB_PATH)
    try:
        # torch ships its own libamdhip64.so (same soname): load it first so that this process has
        # ONE HIP runtime and torch device pointers are valid inside librt_hip.so
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(p):
        raise RuntimeError(f"librt_hip.so not found at {p}: run `python -m blenderraytracer_amd.build` "
                           "(the HIP backend has no CPU fallback)")
    lib = C.CDLL(p)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != RT_ABI_VERSION:
        raise RuntimeError("librt_hip.so ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(status, lib=None):
    if status != 0:
        lib = lib or _lib
        msg = lib.rt_last_error().decode() if lib is not None else ""
        raise RuntimeError(f"{STATUS.get(status, status)}: {msg}")
    return status
