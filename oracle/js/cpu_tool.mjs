// Driver of the JS CPU path (pt_cpu.mjs).  TEST INFRASTRUCTURE / CPU BASELINE ONLY.
//   node cpu_tool.mjs golden <outdir> <case>...    -> <case>.{sum,segs,draws}.bin for tests/test_js_cpu.py
//   node cpu_tool.mjs bench <json args>             -> one JSON line: the JS CPU path timed on a crop
//        {"scene": path, "width", "height", "spp", "depth", "seed", "crop": [x0,y0,w,h], "workers": N}
//        1 worker = the reference's own model (one thread); N workers = worker_threads over interleaved
//        rows (the keyed RNG makes rows independent).  Reports the render time and Msamples/s.
import fs from 'fs';
import os from 'os';
import path from 'path';
import { fileURLToPath } from 'url';
import { Worker, isMainThread, parentPort, workerData } from 'worker_threads';
import { GpuRayTracer, settingsOf } from '../../blenderraytracer_amd/js/gpu-ray-tracer.mjs';
import { packScene } from '../../blenderraytracer_amd/js/pack.mjs';
import { makeScene, renderCrop } from './pt_cpu.mjs';

const HERE = path.dirname(fileURLToPath(import.meta.url));
const REPO = path.resolve(HERE, '..', '..');

function tracer(width, height, seed, sceneJson, settingsIn, backgroundIn) {
    const rt = new GpuRayTracer({ width, height }, { seed });
    if (!rt.loadFromJSON(sceneJson)) throw new Error('loadFromJSON failed');
    if (settingsIn) rt.updateRenderSettings(settingsIn);
    if (backgroundIn) rt.updateBackground(backgroundIn.type, backgroundIn.intensity);
    return rt;
}

function golden(outdir, names) {
    const manifest = JSON.parse(fs.readFileSync(path.join(REPO, 'tests', 'golden', 'manifest.json'), 'utf8'));
    for (const name of names) {
        const c = manifest.cases[name];
        const file = path.join(REPO, 'scenes', c.scene.endsWith('.json') ? c.scene : c.scene + '.json');
        const rt = tracer(c.requested[0], c.requested[1], c.seed, JSON.parse(fs.readFileSync(file, 'utf8')), c.settings_in, c.background_in);
        const st = settingsOf(rt, { seed: c.seed });
        const r = renderCrop(makeScene(packScene(rt.world, rt.camera)), st, c.crop || null);
        for (const k of ['sum', 'segs', 'draws']) fs.writeFileSync(path.join(outdir, `${name}.${k}.bin`), Buffer.from(r[k].buffer));
    }
}

function runBand(job) {
    const rt = tracer(job.width, job.height, job.seed, JSON.parse(fs.readFileSync(job.scene, 'utf8')), { samples: job.spp, maxBounces: job.depth });
    if (rt.width !== job.width || rt.height !== job.height) rt.resizeCanvas(job.width, job.height);
    const st = settingsOf(rt, { seed: job.seed });
    const S = makeScene(packScene(rt.world, rt.camera));
    const t0 = process.hrtime.bigint();
    const r = renderCrop(S, st, job.crop, job.rows);
    const secs = Number(process.hrtime.bigint() - t0) * 1e-9;
    let check = 0, segs = 0;
    for (let i = 0; i < r.sum.length; i++) check += r.sum[i];
    for (let i = 0; i < r.segs.length; i++) segs += r.segs[i];
    return { secs, check, segs, samples: r.segs.length * st.samples };
}

async function bench(args) {
    const workers = Math.max(1, args.workers || 1);
    const ch = args.crop[3];
    const bands = [];                                     // worker w: rows w, w + N, w + 2N, ...
    for (let w = 0; w < Math.min(workers, ch); w++) bands.push([w, ch, workers]);
    const t0 = process.hrtime.bigint();
    let parts;
    if (bands.length === 1) {
        parts = [runBand({ ...args, rows: bands[0] })];
    } else {
        parts = await Promise.all(bands.map((rows) => new Promise((resolve, reject) => {
            const w = new Worker(fileURLToPath(import.meta.url), { workerData: { ...args, rows } });
            w.once('message', resolve);
            w.once('error', reject);
        })));
    }
    const wall = Number(process.hrtime.bigint() - t0) * 1e-9;
    const samples = parts.reduce((a, p) => a + p.samples, 0);
    // timed region: the render loops (each band's own clock; the slowest band ends the frame), not the
    // workers' start-up and scene load
    const render = Math.max(...parts.map((p) => p.secs));
    process.stdout.write(JSON.stringify({
        wall_s: wall, render_s: render, samples, msamples_per_s: samples / render / 1e6, workers: bands.length,
        nproc: os.cpus().length,
        segments: parts.reduce((a, p) => a + p.segs, 0), checksum: parts.reduce((a, p) => a + p.check, 0),
        node: process.version,
    }) + '\n');
}

if (!isMainThread) {
    parentPort.postMessage(runBand(workerData));
} else {
    const [cmd, ...rest] = process.argv.slice(2);
    if (cmd === 'golden') golden(rest[0], rest.slice(1));
    else if (cmd === 'bench') bench(JSON.parse(rest[0])).catch((e) => { process.stderr.write(String(e.stack || e) + '\n'); process.exit(1); });
    else { process.stderr.write('usage: cpu_tool.mjs golden|bench ...\n'); process.exit(2); }
}
