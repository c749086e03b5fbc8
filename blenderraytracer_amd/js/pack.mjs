// Packs a World + Camera into the rt_scene_desc records of include/rt_hip.h.
//
// Duck-typed on the reference's object protocol (SURVEY §1 L4), so it accepts both the reference's
// own js/world.js / js/geometry.js / js/materials.js / js/camera.js instances (the browser drop-in)
// and the restated model of scene-model.mjs (Node).  World.objects order is preserved: it decides
// ties (js/world.js:24-30).
const OBJ = { sphere: 0, plane: 1, box: 2, triangle: 3, mesh: 4 };
const MAT = { lambertian: 0, metal: 1, dielectric: 2, emissive: 3 };
export const BG_CODE = { gradient: 0, solid: 1, hdri: 2, procedural_sky: 3, nan: 4 };
export const OBJECT_BYTES = 64;
export const MATERIAL_BYTES = 72;

function materialRecord(m) {
    if (m == null) throw new Error('object without material');
    if (m.texture !== undefined) throw new Error('textured materials are not reachable from render() (SURVEY §0) and not supported');
    if (m.refractionIndex !== undefined) return { type: MAT.dielectric, ior: m.refractionIndex };
    if (m.intensity !== undefined && m.color !== undefined) {
        // materials.js:95: emitted = color.mul(intensity), evaluated in double exactly as the reference does
        const e = typeof m.emitted === 'function' ? m.emitted(0, 0, null) : { x: m.color.x * m.intensity, y: m.color.y * m.intensity, z: m.color.z * m.intensity };
        return { type: MAT.emissive, emit: [e.x, e.y, e.z] };
    }
    if (m.albedo !== undefined && m.roughness !== undefined) return { type: MAT.metal, albedo: [m.albedo.x, m.albedo.y, m.albedo.z], roughness: m.roughness };
    if (m.albedo !== undefined) return { type: MAT.lambertian, albedo: [m.albedo.x, m.albedo.y, m.albedo.z] };
    throw new Error('unsupported material');
}

// World.background is a function in the reference; recover which one (ray-tracer.js:568-585,
// scene-loader.js:38-51).  Our own World carries backgroundKind directly.
function backgroundOf(world) {
    if (world.backgroundKind !== undefined) {
        const c = world.solidColor || { x: 0.1, y: 0.1, z: 0.1 };
        return { code: world.backgroundKind, solid: [c.x, c.y, c.z] };
    }
    const fn = world.background;
    const name = fn && fn.name;
    if (name === 'bound skyGradient') return { code: BG_CODE.gradient, solid: [0, 0, 0] };
    if (name === 'bound proceduralSky') return { code: BG_CODE.procedural_sky, solid: [0, 0, 0] };
    if (name === 'bound solidBackground' || name === 'bound hdriBackground') return { code: BG_CODE.nan, solid: [0, 0, 0] };
    if (typeof fn === 'function' && fn.length === 0) {            // solidBackground(color) closure
        const saved = world.skyIntensity;
        world.skyIntensity = 1;
        const c = fn();
        world.skyIntensity = saved;
        return { code: BG_CODE.solid, solid: [c.x, c.y, c.z] };
    }
    if (typeof fn === 'function' && fn.length === 1) return { code: BG_CODE.hdri, solid: [0, 0, 0] };  // hdriBackground() closure
    throw new Error('unsupported world.background');
}

function triangleRecord(t, out, k) {
    out.set([t.v0.x, t.v0.y, t.v0.z, t.v1.x, t.v1.y, t.v1.z, t.v2.x, t.v2.y, t.v2.z, t.normal.x, t.normal.y, t.normal.z], 12 * k);
}

export function packScene(world, camera) {
    const mats = [];
    const matIndex = new Map();
    const matOf = (m) => {
        if (!matIndex.has(m)) { matIndex.set(m, mats.length); mats.push(materialRecord(m)); }
        return matIndex.get(m);
    };
    let ntri = 0;
    for (const o of world.objects) if (o.triangles) ntri += o.triangles.length; else if (o.v0) ntri += 1;
    const tris = new Float64Array(Math.max(1, ntri) * 12);
    const objects = new ArrayBuffer(OBJECT_BYTES * world.objects.length);
    const ov = new DataView(objects);
    let k = 0;
    world.objects.forEach((o, i) => {
        const base = i * OBJECT_BYTES;
        const g = (vals) => vals.forEach((v, j) => ov.setFloat64(base + 16 + 8 * j, v, true));
        let type, mat, first = 0, count = 0;
        if (o.triangles) {                                            // TriangleMesh
            type = OBJ.mesh;
            first = k; count = o.triangles.length;
            mat = count ? matOf(o.triangles[0].material) : matOf(o.material || { albedo: { x: 0, y: 0, z: 0 } });
            for (const t of o.triangles) {
                if (t.material !== o.triangles[0].material) throw new Error('mesh triangles with different materials');
                triangleRecord(t, tris, k++);
            }
        } else if (o.v0) {                                            // Triangle
            type = OBJ.triangle; mat = matOf(o.material); first = k; count = 1;
            triangleRecord(o, tris, k++);
        } else if (o.center !== undefined && o.radius !== undefined) {
            type = OBJ.sphere; mat = matOf(o.material); g([o.center.x, o.center.y, o.center.z, o.radius]);
        } else if (o.point !== undefined && o.normal !== undefined) {
            type = OBJ.plane; mat = matOf(o.material); g([o.point.x, o.point.y, o.point.z, o.normal.x, o.normal.y, o.normal.z]);
        } else if (o.min !== undefined && o.max !== undefined) {
            type = OBJ.box; mat = matOf(o.material); g([o.min.x, o.min.y, o.min.z, o.max.x, o.max.y, o.max.z]);
        } else {
            throw new Error(`world.objects[${i}]: unsupported object`);
        }
        ov.setInt32(base, type, true);
        ov.setInt32(base + 4, mat, true);
        ov.setInt32(base + 8, first, true);
        ov.setInt32(base + 12, count, true);
    });
    const materials = new ArrayBuffer(MATERIAL_BYTES * Math.max(1, mats.length));
    const mv = new DataView(materials);
    mats.forEach((m, i) => {
        const b = i * MATERIAL_BYTES;
        mv.setInt32(b, m.type, true);
        (m.albedo || [0, 0, 0]).forEach((v, j) => mv.setFloat64(b + 8 + 8 * j, v, true));
        mv.setFloat64(b + 32, m.roughness || 0, true);
        mv.setFloat64(b + 40, m.ior || 0, true);
        (m.emit || [0, 0, 0]).forEach((v, j) => mv.setFloat64(b + 48 + 8 * j, v, true));
    });
    const c = camera;
    const cam = new Float64Array(22);
    [c.origin, c.lowerLeftCorner, c.horizontal, c.vertical, c.u, c.v, c.w].forEach((v, j) => cam.set([v.x, v.y, v.z], 3 * j));
    cam[21] = c.lensRadius;
    const bg = backgroundOf(world);
    return {
        objects: new Uint8Array(objects),
        materials: new Uint8Array(materials, 0, MATERIAL_BYTES * mats.length),
        triangles: tris.subarray(0, ntri * 12),
        camera: cam,
        cameraType: c.type === 'orthographic' ? 1 : 0,        // getRay branches on === 'orthographic'
        background: bg.code,
        skyIntensity: world.skyIntensity,
        solidColor: new Float64Array(bg.solid),
        perm: Int32Array.from(world.cloudNoise.p),
    };
}
