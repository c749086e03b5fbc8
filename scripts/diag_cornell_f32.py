import sys, numpy as np
sys.path.insert(0, '.')
import torch  # noqa
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json
res = {}
for prec in (capi.RT_PREC_F64, capi.RT_PREC_F32):
    rt = GpuRayTracer(512, 512, seed=8, precision=prec)
    rt.load_from_json(load_scene_json('cornell.json')); rt.update_render_settings({'maxBounces': 5, 'samples': 64})
    res[prec] = rt.render(want=('mean', 'segments', 'draws'))
a, b = res[0], res[1]
d = np.abs(a['post'][..., :3].astype(float) - b['post'][..., :3])
print('segs equal', np.mean(a['segments'] == b['segments']), 'draws equal', np.mean(a['draws'] == b['draws']))
print('rms', np.sqrt(np.mean(d ** 2)), 'max', d.max())
bad = np.argwhere(a['segments'] != b['segments'])
print('n bad pixels', len(bad), bad[:10])
rows = np.sqrt(np.mean(d ** 2, axis=(1, 2)))
print('worst rows', np.argsort(rows)[-10:], rows[np.argsort(rows)[-10:]])
cols = np.sqrt(np.mean(d ** 2, axis=(0, 2)))
print('worst cols', np.argsort(cols)[-10:])
