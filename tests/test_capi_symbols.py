"""librt_hip.so loads on a machine without a GPU, exports every function include/rt_hip.h declares,
and refuses to compute without a device (no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

from blenderraytracer_amd import capi
from blenderraytracer_amd.scene import PackedScene, default_scene
from blenderraytracer_amd.rng import permutation

INCLUDE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADER = os.path.join(INCLUDE, "rt_hip.h")


def declared_functions():
    """Every function declared by include/*.h."""
    names = set()
    for h in sorted(os.listdir(INCLUDE)):
        src = re.sub(r"/\*.*?\*/", "", open(os.path.join(INCLUDE, h)).read(), flags=re.S)
        names |= set(re.findall(r"^\s*(?:int|void|const char\*|const rt_\w+\*)\s+(rt_\w+)\s*\(", src, flags=re.M))
    return names


def test_header_and_binding_agree():
    assert declared_functions() == set(capi.EXPORTS)


def test_library_exports_every_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.rt_abi_version() == capi.RT_ABI_VERSION


def test_struct_layout_matches_c_compiler(tmp_path):
    """sizeof/offsetof of every ABI struct as gcc lays it out == the ctypes mirror."""
    structs = {"rt_material_desc": capi.MaterialDesc, "rt_object_desc": capi.ObjectDesc,
               "rt_camera_desc": capi.CameraDesc, "rt_scene_desc": capi.SceneDesc, "rt_settings": capi.Settings,
               "rt_output": capi.Output, "rt_stats": capi.Stats}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'printf("{cname}.{f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-o", str(exe), str(src)])
    got = dict(l.rsplit(" ", 1) for l in subprocess.check_output([str(exe)]).decode().split("\n") if l)
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for f in py._fields_:
            assert int(got[f"{cname}.{f[0]}"]) == getattr(py, f[0]).offset, (cname, f[0])


def test_no_device_means_error_not_fallback(lib):
    from conftest import gpu_available
    if gpu_available():
        return  # on the GPU box this is covered by the parity tests
    n = C.c_int(-1)
    assert lib.rt_device_count(C.byref(n)) == -5 and n.value == 0
    w, cam = default_scene(8, 8, permutation(0))
    p = PackedScene(w, cam)
    h = C.c_void_p()
    assert lib.rt_scene_create(C.byref(p.desc), 0, C.byref(h)) == -5
    assert b"no HIP device" in lib.rt_last_error()


def test_invalid_descriptor_rejected(lib):
    w, cam = default_scene(8, 8, permutation(0))
    p = PackedScene(w, cam)
    p.desc.abi_version = 99
    h = C.c_void_p()
    assert lib.rt_scene_create(C.byref(p.desc), 0, C.byref(h)) == -1
    assert lib.rt_scene_create(None, 0, C.byref(h)) == -1


def test_library_records_the_sources_it_was_built_from(lib):
    """lib/build_info.json (written by the build next to librt_hip.so) names the commit and the digest
    of csrc/ + include/; bench.py reports both, so a profile names the sources it measured."""
    from blenderraytracer_amd import build as B
    info = B.read_build_info()
    assert info is not None and len(info["source_digest"]) == 16
    lib_mtime = os.path.getmtime(os.path.join(B.LIBDIR, "librt_hip.so"))
    srcs = [os.path.join(d, f) for d in (B.CSRC, INCLUDE) for f in os.listdir(d)]
    if all(os.path.getmtime(s) <= lib_mtime for s in srcs):     # library built after the last edit
        assert info["source_digest"] == B.source_digest()
