"""Build librt_hip.so (HIP kernels + C ABI) for gfx950, in-tree, with plain hipcc.

    python -m blenderraytracer_amd.build [--napi]

Flags: -ffp-contract=off keeps every binary64 operation unfused, like JavaScript; no fast-math
(NaN/Inf semantics are part of Box.hit and the JSON-solid background, SURVEY §7 hard part 1).
The N-API addon (csrc/napi_addon.cpp, for the Node host) is built with --napi when Node headers exist.
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
REPO = os.path.dirname(HERE)
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")

SOURCES = ["pt_trace.hip", "pt_onewave.hip", "rt_capi.cpp", "scene_json.cpp"]
# per-source flags: the one-wave pool and lane-per-pixel kernels (pt_onewave.hip) with LLVM's AMDGPU
# register-pressure trackers during scheduling (mesh50k +1.0 %, Cornell +1.4 %; the LDS kernels -3.6 %
# with it, so not for pt_trace.hip)
SOURCE_FLAGS = {"pt_onewave.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]}
# -structurizecfg-skip-uniform-regions: branches the compiler proves wave-uniform stay plain scalar
# branches instead of exec-mask regions (RTOW +0.9 %, mesh50k +0.5 %, identical images)
HIP_FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC",
             "-mllvm", "-structurizecfg-skip-uniform-regions=1",
             "-Wall", "-Wno-unused-function", "-I", os.path.join(REPO, "include")]


def _run(cmd):
    print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def source_digest():
    """sha256 (16 hex digits) over the library's sources (csrc/ and include/, names and bytes) and its
    compile flags (without the machine-specific include path)."""
    h = hashlib.sha256()
    h.update(" ".join(f for f in HIP_FLAGS if not os.path.isabs(f)).encode())
    for d in (CSRC, os.path.join(REPO, "include")):
        for f in sorted(os.listdir(d)):
            p = os.path.join(d, f)
            if os.path.isfile(p):
                h.update(f.encode())
                with open(p, "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


def _git(*args):
    try:
        return subprocess.run(["git", "-C", REPO, *args], capture_output=True, text=True, timeout=10).stdout.strip()
    except Exception:
        return ""


def write_build_info():
    """lib/build_info.json: the commit and source digest librt_hip.so was built from (travels with the
    library; bench.py reports it, so a profile names the sources it measured)."""
    info = {"commit": _git("rev-parse", "--short", "HEAD") or None,
            "sources_modified": bool(_git("status", "--porcelain", "--", CSRC, os.path.join(REPO, "include"),
                                          os.path.abspath(__file__))),
            "source_digest": source_digest()}
    with open(os.path.join(LIBDIR, "build_info.json"), "w") as f:
        json.dump(info, f)
    return info


def read_build_info():
    try:
        with open(os.path.join(LIBDIR, "build_info.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def build_lib(force=False):
    os.makedirs(LIBDIR, exist_ok=True)
    target = os.path.join(LIBDIR, "librt_hip.so")
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(REPO, "include", f) for f in os.listdir(os.path.join(REPO, "include"))]
    if not force and not _stale(target, deps):
        return target
    objs, procs = [], []
    for src in SOURCES:                  # the translation units compile in parallel
        obj = os.path.join(LIBDIR, os.path.splitext(src)[0] + ".o")
        cmd = [HIPCC, *HIP_FLAGS, *SOURCE_FLAGS.get(src, []), "-c", os.path.join(CSRC, src), "-o", obj]
        print(" ".join(cmd), flush=True)
        procs.append((cmd, subprocess.Popen(cmd)))
        objs.append(obj)
    failed = [cmd for cmd, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    _run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", target, *objs])
    write_build_info()
    return target


def build_napi(force=False):
    """Node N-API addon: plain g++ against node_api.h, links librt_hip.so by rpath."""
    node_inc = os.environ.get("NODE_INCLUDE", "/usr/include/node")
    if not os.path.exists(os.path.join(node_inc, "node_api.h")):
        print("node_api.h not found: skipping the N-API addon")
        return None
    target = os.path.join(LIBDIR, "rt_napi.node")
    src = os.path.join(CSRC, "napi_addon.cpp")
    if not os.path.exists(src):
        return None
    if not force and not _stale(target, [src, os.path.join(REPO, "include", "rt_hip.h"), os.path.join(LIBDIR, "librt_hip.so")]):
        return target
    _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", node_inc, "-I", os.path.join(REPO, "include"),
          src, "-o", target, "-L", LIBDIR, "-lrt_hip", "-Wl,-rpath,$ORIGIN"])
    return target


def build_cli(force=False):
    """rt_render_cli: the Node-free front end (scene JSON -> rt_json_scene_load -> rt_render)."""
    target = os.path.join(LIBDIR, "rt_render_cli")
    src = os.path.join(CSRC, "rt_cli.cpp")
    deps = [src, os.path.join(LIBDIR, "librt_hip.so")] + [os.path.join(REPO, "include", f)
                                                          for f in os.listdir(os.path.join(REPO, "include"))]
    if not force and not _stale(target, deps):
        return target
    _run(["g++", "-O2", "-std=c++17", "-Wall", "-I", os.path.join(REPO, "include"), src, "-o", target,
          "-L", LIBDIR, "-lrt_hip", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath-link,/opt/rocm/lib"])
    return target


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    force = "--force" in argv
    print(build_lib(force))
    print(build_cli(force))
    if "--napi" in argv:
        print(build_napi(force))


if __name__ == "__main__":
    main()
