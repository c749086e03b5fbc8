"""Static spill-reload census of one kernel, per loop (DEV TOOL): compiles
csrc/pt_trace.hip (or pt_onewave.hip) to gfx950 assembly and, for every block, takes LLVM's own loop
annotation (`; Loop: Header=BBx Depth=n`), then sums per loop the instructions, VALU and binary64
instructions, `v_readlane_b32` (SGPR-spill reloads), `v_writelane_b32` and scratch accesses.  Static
counts: a block inside a loop counts once, whichever of its branches a wave takes.
usage: python scripts/isa_loops.py <mangled kernel name> [pt_trace.hip|pt_onewave.hip]"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
fn = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else "pt_trace.hip"
extra = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"] if src == "pt_onewave.hip" else []
with tempfile.TemporaryDirectory() as d:
    out = os.path.join(d, "k.s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                           "-fPIC", "-mllvm", "-structurizecfg-skip-uniform-regions=1", *extra, "-I",
                           os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-o", out,
                           os.path.join(ROOT, "blenderraytracer_amd", "csrc", src)], stderr=subprocess.DEVNULL)
    lines = open(out).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(fn + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur = [], {"depth": 0, "hdr": None, "ins": []}
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)", l)
    if m:
        blocks.append(cur)
        d = re.search(r"Depth=(\d+)", m.group(2))
        h = re.search(r"Header=(BB\d+_\d+)", m.group(2))
        cur = {"lab": m.group(1), "hdr": h.group(1) if h else None, "depth": int(d.group(1)) if d else 0, "ins": []}
        continue
    if "This Inner Loop Header" in l or "This Loop Header" in l:
        cur["depth"] = int(re.search(r"Depth=(\d+)", l).group(1))
        cur["hdr"] = cur.get("lab", "").lstrip(".L")
        continue
    if "in Loop: Header" in l and cur["hdr"] is None:
        cur["depth"] = int(re.search(r"Depth=(\d+)", l).group(1))
        cur["hdr"] = re.search(r"Header=(BB\d+_\d+)", l).group(1)
    t = l.strip()
    if t and not t.startswith(";") and not t.startswith("."):
        cur["ins"].append(t)
blocks.append(cur)
by = collections.defaultdict(collections.Counter)
for b in blocks:
    c = collections.Counter(t.split()[0] for t in b["ins"])
    k = (b["depth"], b["hdr"])
    by[k]["instrs"] += len(b["ins"])
    by[k]["valu"] += sum(v for op, v in c.items() if op.startswith("v_"))
    by[k]["f64"] += sum(v for op, v in c.items() if op.endswith("_f64"))
    by[k]["readlane"] += c["v_readlane_b32"]
    by[k]["writelane"] += c["v_writelane_b32"]
    by[k]["scratch"] += sum(v for op, v in c.items() if op.startswith("scratch_"))
print(f"# {fn} ({src}): static counts per loop (depth, LLVM loop header)")
for k in sorted(by, key=lambda k: (k[0], str(k[1]))):
    v = by[k]
    print(f"depth {k[0]} header {k[1]}: instrs {v['instrs']:5d} valu {v['valu']:5d} f64 {v['f64']:4d} "
          f"v_readlane {v['readlane']:3d} v_writelane {v['writelane']:3d} scratch {v['scratch']}")
