#!/bin/bash
# Node end-to-end diagnosis (DEV TOOL): the drop-in's 16 progressive batches vs one batch on config 3 with
# the current library, round 4's (variants/r4.so) and the fence-free commit (variants/fence0.so) swapped in
# for lib/librt_hip.so (the addon loads it by rpath), plus the progress hand-off trace of the current one
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r5_node_diag.log
: > $L
python3 - <<'PY' > /tmp/rtow_scene.json
import json, sys
sys.path.insert(0, '.')
from blenderraytracer_amd.scene import load_scene_json
json.dump(load_scene_json('rtow.json'), sys.stdout)
PY
A='{"scene": "/tmp/rtow_scene.json", "width": 1920, "height": 1080, "spp": 512, "depth": 5, "seed": 1, "reps": 5}'
cp blenderraytracer_amd/lib/librt_hip.so /tmp/librt_hip_cur.so
for v in cur r4 fence0 cur r4; do
  if [ $v = cur ]; then cp /tmp/librt_hip_cur.so blenderraytracer_amd/lib/librt_hip.so; else cp blenderraytracer_amd/lib/variants/$v.so blenderraytracer_amd/lib/librt_hip.so; fi
  echo "== $v $(timeout -k 10 200 node scripts/node_e2e.mjs "$A")" >> $L || exit 1
done
cp /tmp/librt_hip_cur.so blenderraytracer_amd/lib/librt_hip.so
RT_NAPI_TRACE=1 timeout -k 10 200 node scripts/node_e2e.mjs "$A" > gpurun_out/r5_node_trace.out 2> gpurun_out/r5_node_trace.err
