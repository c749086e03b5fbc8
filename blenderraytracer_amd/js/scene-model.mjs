// Scene model for the Node host: a clean-room restatement of the reference's scene objects and
// JSON loader, producing objects with the SAME duck-typed shape as the reference's classes, so the
// packer (pack.mjs) handles either.  All arithmetic is JS double, evaluated in the reference's order:
//   Vec3                       js/math.js:6-32
//   Camera constructor         js/camera.js:8-36
//   Plane / Triangle / Mesh    js/geometry.js:50-53, 140-146, 193-237
//   materials                  js/materials.js:14-96
//   World + backgrounds        js/world.js:8-16 (background kinds are tagged, see backgroundKind)
//   SceneLoader.loadFromJSON   js/scene-loader.js:20-284
import { permutation } from './keyed-rng.mjs';

export class Vec3 {
    constructor(x = 0, y = 0, z = 0) { this.x = x; this.y = y; this.z = z; }
    add(v) { return new Vec3(this.x + v.x, this.y + v.y, this.z + v.z); }
    sub(v) { return new Vec3(this.x - v.x, this.y - v.y, this.z - v.z); }
    mul(s) { return new Vec3(this.x * s, this.y * s, this.z * s); }
    div(s) { return new Vec3(this.x / s, this.y / s, this.z / s); }
    dot(v) { return this.x * v.x + this.y * v.y + this.z * v.z; }
    cross(v) { return new Vec3(this.y * v.z - this.z * v.y, this.z * v.x - this.x * v.z, this.x * v.y - this.y * v.x); }
    length() { return Math.sqrt(this.x * this.x + this.y * this.y + this.z * this.z); }
    normalize() { const l = this.length(); return l > 0 ? this.div(l) : new Vec3(); }
}

export class Camera {
    constructor(lookFrom, lookAt, vup, vfov, aspect, aperture, focusDist, type = 'perspective') {
        this.type = type;
        this.aperture = aperture;
        this.focusDist = focusDist;
        this.fov = vfov;
        const theta = vfov * Math.PI / 180;
        const h = Math.tan(theta / 2);
        const viewportHeight = 2.0 * h;
        const viewportWidth = aspect * viewportHeight;
        this.w = lookFrom.sub(lookAt).normalize();
        this.u = vup.cross(this.w).normalize();
        this.v = this.w.cross(this.u);
        this.origin = lookFrom;
        if (type === 'perspective') {
            this.horizontal = this.u.mul(viewportWidth * focusDist);
            this.vertical = this.v.mul(viewportHeight * focusDist);
            this.lowerLeftCorner = this.origin.sub(this.horizontal.div(2)).sub(this.vertical.div(2)).sub(this.w.mul(focusDist));
        } else {
            this.horizontal = this.u.mul(viewportWidth);
            this.vertical = this.v.mul(viewportHeight);
            this.lowerLeftCorner = this.origin.sub(this.horizontal.div(2)).sub(this.vertical.div(2));
        }
        this.lensRadius = aperture / 2;
    }
}

// materials: same fields as the reference classes
export class Lambertian { constructor(albedo) { this.albedo = albedo; } }
export class Metal { constructor(albedo, roughness = 0) { this.albedo = albedo; this.roughness = Math.min(roughness, 1); } }
export class Dielectric { constructor(ior) { this.refractionIndex = ior; } }
export class Emissive {
    constructor(color, intensity = 1) { this.color = color; this.intensity = intensity; }
    emitted() { return this.color.mul(this.intensity); }
}

// geometry: same fields as the reference classes
export class Sphere { constructor(center, radius, material) { this.center = center; this.radius = radius; this.material = material; } }
export class Plane { constructor(point, normal, material) { this.point = point; this.normal = normal.normalize(); this.material = material; } }
export class Box { constructor(min, max, material) { this.min = min; this.max = max; this.material = material; } }
export class Triangle {
    constructor(v0, v1, v2, material) {
        this.v0 = v0; this.v1 = v1; this.v2 = v2; this.material = material;
        this.normal = v1.sub(v0).cross(v2.sub(v0)).normalize();
    }
}
export class TriangleMesh {
    constructor(vertices, indices, material) {
        this.triangles = [];
        if (!Array.isArray(vertices) || !Array.isArray(indices)) return;
        for (let i = 0; i < indices.length; i += 3) {
            if (i + 2 >= indices.length) continue;                        // incomplete triangle
            const idx = [indices[i], indices[i + 1], indices[i + 2]];
            if (idx.some((k) => k >= vertices.length)) continue;         // out-of-range index
            const vs = idx.map((k) => (vertices[k] instanceof Vec3 ? vertices[k] : new Vec3(0, 0, 0)));
            this.triangles.push(new Triangle(vs[0], vs[1], vs[2], material));
        }
    }
}

export const BG = { gradient: 0, solid: 1, hdri: 2, procedural_sky: 3, nan: 4 };

export class World {
    constructor(perm) {
        this.objects = [];
        this.lights = [];
        this.backgroundKind = BG.gradient;
        this.solidColor = new Vec3(0.1, 0.1, 0.1);
        this.skyIntensity = 1.0;
        this.cloudNoise = { p: perm };
    }
    add(o) { this.objects.push(o); }
}

const parseVec3 = (a) => (Array.isArray(a) && a.length >= 3 ? new Vec3(a[0], a[1], a[2]) : new Vec3(0, 0, 0));

function createMaterial(m) {
    if (!m || !m.type) return new Lambertian(new Vec3(0.8, 0.8, 0.8));
    switch (m.type.toLowerCase()) {
        case 'lambertian': return new Lambertian(parseVec3(m.color));
        case 'metal': return new Metal(parseVec3(m.color), m.roughness !== undefined ? m.roughness : 0.0);
        case 'dielectric': return new Dielectric(m.ior !== undefined ? m.ior : 1.5);
        case 'emissive': return new Emissive(parseVec3(m.color), m.intensity !== undefined ? m.intensity : 1.0);
        default: return new Lambertian(new Vec3(0.8, 0.8, 0.8));
    }
}

function createObject(o) {
    if (!o.type) return null;
    const material = createMaterial(o.material || { type: 'lambertian', color: [0.8, 0.8, 0.8] });
    switch (o.type.toLowerCase()) {
        case 'sphere': return new Sphere(parseVec3(o.center), o.radius || 1.0, material);
        case 'plane': return new Plane(parseVec3(o.point), parseVec3(o.normal), material);
        case 'box': return new Box(parseVec3(o.min), parseVec3(o.max), material);
        case 'triangle': return new Triangle(parseVec3(o.v0), parseVec3(o.v1), parseVec3(o.v2), material);
        case 'mesh':
            if (!o.vertices || !o.indices) return null;
            return new TriangleMesh(o.vertices.map(parseVec3), o.indices, material);
        default: return null;
    }
}

export function createCamera(cam, aspect) {
    const position = parseVec3(cam.position || [0, 0, 5]);
    let lookAt = parseVec3(cam.lookAt || [0, 0, 0]);
    const up = parseVec3(cam.up || [0, 1, 0]);
    const fov = cam.fov !== undefined ? cam.fov : 45;
    const aperture = cam.aperture !== undefined ? cam.aperture : 0.0;
    if (position.sub(lookAt).length() < 1.0) {
        const direction = position.sub(lookAt).normalize().mul(-1);
        lookAt = position.add(direction.mul(100));
    }
    let focusDist = cam.focusDist;
    if (focusDist === undefined) focusDist = position.sub(lookAt).length();
    return new Camera(position, lookAt, up, fov, cam.aspect || aspect, aperture, focusDist, cam.type || 'perspective');
}

// SceneLoader.loadFromJSON: perm = World.cloudNoise.p for the new World (reference: Math.random
// shuffle at construction; here passed in so that it can come from the keyed RNG).
export function loadFromJSON(json, width, height, perm) {
    let newDimensions = null;
    if (json.camera && json.camera.resolution) {
        newDimensions = { width: json.camera.resolution[0], height: json.camera.resolution[1] };
        width = newDimensions.width;
        height = newDimensions.height;
    }
    const world = new World(perm);
    if (json.background) {
        const t = json.background.type;
        world.backgroundKind = t === 'solid' || t === 'hdri' ? BG.nan : t === 'procedural_sky' ? BG.procedural_sky : BG.gradient;
        if (json.background.intensity !== undefined) world.skyIntensity = json.background.intensity;
    }
    if (Array.isArray(json.objects)) for (const o of json.objects) { const obj = createObject(o); if (obj) world.add(obj); }
    // lights (scene-loader.js:69-76) are parsed but never rendered; _createLight calls
    // lightData.type.toLowerCase() (:187), which throws for a truthy non-string type: the load fails
    if (json.lights && Array.isArray(json.lights))
        for (const l of json.lights) if (l && l.type) l.type.toLowerCase();
    const camera = json.camera ? createCamera(json.camera, width / height) : null;
    return { world, camera, newDimensions };
}

// RayTracer.setupDefaultScene (ray-tracer.js:42-77)
export function defaultScene(width, height, perm) {
    const w = new World(perm);
    w.add(new Plane(new Vec3(0, -0.5, 0), new Vec3(0, 1, 0), new Lambertian(new Vec3(0.5, 0.5, 0.5))));
    w.add(new Sphere(new Vec3(0, 0, -1), 0.5, new Lambertian(new Vec3(0.7, 0.3, 0.3))));
    w.add(new Sphere(new Vec3(-1, 0, -1), 0.5, new Dielectric(1.5)));
    w.add(new Sphere(new Vec3(1, 0, -1), 0.5, new Metal(new Vec3(0.8, 0.8, 0.9), 0.1)));
    w.add(new Sphere(new Vec3(0, 1.5, -1), 0.3, new Emissive(new Vec3(1, 1, 1), 5)));
    const cam = new Camera(new Vec3(3, 2, 2), new Vec3(0, 0, -1), new Vec3(0, 1, 0), 45, width / height, 0.0, 10.0);
    return { world: w, camera: cam };
}

// RayTracer.setupCamera after a resize (ray-tracer.js:439-474)
export function setupCamera(camera, width, height) {
    const lookAt = camera.origin.sub(camera.w.mul(camera.focusDist));
    return new Camera(camera.origin, lookAt, camera.v, camera.fov || 45, width / height, camera.aperture || 0.0,
        camera.focusDist || 10.0, camera.type || 'perspective');
}

export { permutation };
