'use strict';
// Node host mirror of the reference's TypeScript surface (src/gpu_context.ts, src/renderer.ts,
// src/camera.ts), driving the MI355X renderer through the N-API addon (../lib/gsplat_napi.node).
// Same names, argument meaning and error behaviour as the reference:
//   * GpuContext.create() / Renderer.requestContext() reject with a STRING when no device exists
//     (src/gpu_context.ts:12-26, src/renderer.ts:79-100);
//   * new Renderer(canvas, camera, gaussians, context, fpsCounter) throws Error when the surface is
//     missing (src/renderer.ts:119-122), copies the AoS scene once (:139-146) and starts the frame
//     loop with requestAnimationFrame(() => this.animate(true)) (:278);
//   * animate(forceDraw?) packs the 160-B uniform block from camera.getCamera() and draws only when
//     the camera is dirty or forced (:332-387); draw(cb) renders and schedules cb (:301-330);
//   * destroy() resolves after the next frame (:103-107, :281-292); resize() reallocates the
//     W x H state (:293-299).
// Headless conventions (SURVEY §8b): canvas = {width, height, present?, onFrame?}; after every
// frame renderer.framebuffer (and canvas.framebuffer) holds SimpleRender.framebuffer's contents
// (W*H premultiplied RGBA float32, row 0 = top) and, with canvas.present, canvas.image holds the
// PostProcessRenderer output; fpsCounter = {innerText, style}; requestAnimationFrame = setImmediate
// unless the host provides one.
const path = require('path');

let native = null;
function addon() {
    if (native === null) {
        const p = process.env.GSPLAT_NAPI || path.join(__dirname, '..', 'lib', 'gsplat_napi.node');
        native = require(p);  // throws if the addon was not built: there is no other backend
    }
    return native;
}

const raf = (cb) => (typeof requestAnimationFrame === 'function' ? requestAnimationFrame(cb) : setImmediate(cb));
const now = () => Number(process.hrtime.bigint()) / 1e6;
const FOV = 1.04719755;  // 60 degrees (src/camera.ts:4)

const GS_ACCUM_FP32 = 0, GS_ACCUM_FP16_TARGET = 1, GS_OUT_RGBA_F32 = 0, GS_OUT_RGBA_F16 = 1;
// host-readback frames in flight: the event loop's hand-off from the copy's waiting thread back
// to the frame loop takes ~0.1 ms, so two in flight left the GPU idle between frames
// (GSPLAT_READBACK_DEPTH overrides; clamped to [1, 7]: the C library's readback ring holds 8
// copies, gs_ctx::kReadbacks, and a deeper frame loop would wait on a slot a newer copy reused)
const kReadbackDepth = Math.min(7, Math.max(1, parseInt(process.env.GSPLAT_READBACK_DEPTH, 10) || 3));

// ---------------------------------------------------------------------------- GpuContext
class GpuContext {
    constructor(gpu, adapter, device) {
        this.gpu = gpu;          // {api: 'hip'}
        this.adapter = adapter;  // {deviceIndex, deviceCount}
        this.device = device;    // native context handle (gs_ctx*)
    }

    // deviceIndex: one HIP device, or an array of devices (a device group: the frame is split into
    // K-balanced row strips, one per device, and each strip is sent to the first device -- RCCL
    // send/receive pairs over distinct devices, peer copies when the list repeats one -- where the
    // image lands)
    static async create(deviceIndex = 0) {
        let n = 0;
        try {
            n = addon().deviceCount();
        } catch (e) {
            return Promise.reject('gsplat addon not available: ' + e.message);
        }
        if (n <= 0) return Promise.reject('No HIP device available (gs_device_count = 0)');
        try {
            const device = addon().ctxCreate(deviceIndex);
            return new GpuContext({api: 'hip'}, {deviceIndex, deviceCount: n}, device);
        } catch (e) {
            return Promise.reject(String(e.message));
        }
    }

    destroy() {
        if (this.device) addon().ctxDestroy(this.device);
        this.adapter = null;
        this.device = null;
    }
}

// ---------------------------------------------------------------------------- scene input
// The reference's PackedGaussians (src/ply.ts:249-257): AoS records of 64 + 16 * nShCoeffs bytes.
class PackedGaussians {
    constructor(gaussiansBuffer, numGaussians, nShCoeffs = 16) {
        this.gaussiansBuffer = gaussiansBuffer instanceof ArrayBuffer ? gaussiansBuffer : gaussiansBuffer.buffer;
        this.numGaussians = numGaussians;
        this.nShCoeffs = nShCoeffs;
        this.sphericalHarmonicsDegree = Math.sqrt(nShCoeffs) - 1;
        this.gaussianArrayLayout = {size: numGaussians * (64 + 16 * nShCoeffs)};
        this.min_pos = [99999, 99999, 99999];
        this.max_pos = [-99999, -99999, -99999];
    }

    // new PackedGaussians(plyArrayBuffer) of the reference (src/ply.ts:200-355), parsed natively
    // with the same semantics (gs_ply_parse); throws Error like the reference on a bad file
    static fromPly(plyArrayBuffer) {
        const r = addon().plyParse(plyArrayBuffer);
        const g = new PackedGaussians(r.aos, r.numGaussians, r.nShCoeffs);
        g.sphericalHarmonicsDegree = r.shDegree;
        g.min_pos = r.minPos;
        g.max_pos = r.maxPos;
        return g;
    }
}

// ---------------------------------------------------------------------------- cameras
// Camera fields as src/camera.ts:56-138 (matrices Float32Array(16), column-major).
class Camera {
    constructor(height, width, viewMatrix, perspective, focalX, focalY, scaleModifier) {
        this.height = height;
        this.width = width;
        this.viewMatrix = viewMatrix;
        this.perspective = perspective;
        this.focalX = focalX;
        this.focalY = focalY;
        this.scaleModifier = scaleModifier;
    }

    // Camera.default (src/camera.ts:101-111) for a canvas of width x height
    static default(width, height) {
        return new Camera(height, width, addon().lookAt([0, 0, -5], [0, 0, 0], [0, 1, 0]),
                          addon().perspective(FOV, width / height, 0.03, 1000), width, height, 1);
    }

    static lookAt(eye, target, width, height, fovy = FOV, near = 0.03, far = 1000) {
        return new Camera(height, width, addon().lookAt(eye, target, [0, 1, 0]),
                          addon().perspective(fovy, width / height, near, far), width, height, 1);
    }

    // cameraFromJSON (src/camera.ts:476-503): an INRIA cameras.json entry for a canvasW x canvasH
    // canvas (+z forward, getProjectionMatrix(0.2, 100, fovX, fovY)); focalX/focalY = H/W as there
    static fromJSON(rawCamera, canvasW, canvasH) {
        const c = addon().cameraFromJSON(rawCamera, canvasW, canvasH);
        return new Camera(canvasH, canvasW, c.viewMatrix, c.perspective, c.focalX, c.focalY, 1);
    }

    // translation of inverse(view) (src/camera.ts:135-138)
    getPosition() {
        return addon().cameraPosition(this.viewMatrix);
    }
}

// InteractiveCamera's contract as used by Renderer.animate: isDirty() / getCamera().
class HeadlessCamera {
    constructor(camera) {
        this.camera = camera;
        this.dirty = true;
    }

    setNewCamera(camera) {
        this.camera = camera;
        this.dirty = true;
    }

    setDirty() {
        this.dirty = true;
    }

    isDirty() {
        return this.dirty;
    }

    getCamera() {
        this.dirty = false;
        return this.camera;
    }
}

// ---------------------------------------------------------------------------- Renderer
class Renderer {
    static async requestContext(gaussians, deviceIndex = 0) {
        if (!gaussians || !gaussians.gaussiansBuffer) return Promise.reject('requestContext: no gaussians');
        return GpuContext.create(deviceIndex);
    }

    // destroy the renderer; resolves when it's done (after the next frame)
    async destroy() {
        return new Promise((resolve) => {
            this.destroyCallback = resolve;
        });
    }

    constructor(canvas, interactiveCamera, gaussians, context, fpsCounter, options = {}) {
        if (!canvas || !(canvas.width > 0) || !(canvas.height > 0)) {
            throw new Error('Render surface not found! (canvas needs width and height)');
        }
        if (!context || !context.device) throw new Error('GpuContext is not initialised');
        this.canvas = canvas;
        this.interactiveCamera = interactiveCamera;
        this.context = context;
        this.fpsCounter = fpsCounter || {innerText: '', style: {}};
        this.lastDraw = now();
        this.numGaussians = gaussians.numGaussians;
        this.destroyCallback = null;
        // options: accum, outFormat, tMin, deviceResident (frames stay in HBM; readback() on request)
        this.opts = Object.assign({accum: GS_ACCUM_FP32, outFormat: GS_OUT_RGBA_F32, tMin: 1e-4, deviceResident: false},
                                  options);
        this.deviceFramebuffer = null;
        this.frames = 0;
        // host-readback frames in flight (see draw): kReadbackDepth device framebuffers, one more
        // page-locked host array, frames delivered in order through one promise chain
        this.devFbs = null;
        this.hostFbs = null;
        this.slot = 0;
        this.inflight = 0;
        this.waiting = null;
        this.delivered = Promise.resolve();
        // the AoS record buffer is borrowed for this call only (copied into HBM as SoA)
        this.scene = addon().sceneUpload(context.device, gaussians.gaussiansBuffer, gaussians.numGaussians,
                                         gaussians.nShCoeffs);
        this.resize();
        raf(() => this.animate(true));
    }

    destroyImpl() {
        if (this.destroyCallback === null) throw new Error('destroyImpl called without destroyCallback set!');
        if (this.deviceFramebuffer && this.context.device) addon().fbFree(this.context.device, this.deviceFramebuffer);
        this.deviceFramebuffer = null;
        this.releaseReadback();
        if (this.scene && this.context.device) addon().sceneFree(this.scene);
        this.scene = null;
        this.context.destroy();
        this.destroyCallback();
    }

    // host-readback buffers: unpinned and freed (no readback in flight: see draw / animate)
    releaseReadback() {
        if (this.hostFbs && this.context.device)
            for (const b of this.hostFbs) addon().hostUnregister(this.context.device, b);
        if (this.devFbs && this.context.device)
            for (const f of this.devFbs) addon().fbFree(this.context.device, f);
        this.hostFbs = null;
        this.devFbs = null;
    }

    // reallocate the W x H-dependent state (src/renderer.ts:293-299)
    resize() {
        this.width = this.canvas.width;
        this.height = this.canvas.height;
        const px = this.width * this.height * 4;
        this.releaseReadback();
        if (this.opts.deviceResident) {
            // the frame stays in HBM like the reference's framebuffer texture; readback() copies it
            if (this.deviceFramebuffer) addon().fbFree(this.context.device, this.deviceFramebuffer);
            this.fbBytes = px * (this.opts.outFormat === GS_OUT_RGBA_F16 ? 2 : 4);
            this.deviceFramebuffer = addon().fbAlloc(this.context.device, this.fbBytes);
            this.framebuffer = null;
            this.image = null;
            return;
        }
        // host readback: like the reference's draw, a frame is submitted and the next animation
        // frame requested without waiting for it; its copy to the host runs on a copy stream while
        // the next frame renders (kReadbackDepth device framebuffers, one more page-locked host array)
        const f16 = this.opts.outFormat === GS_OUT_RGBA_F16;
        this.fbBytes = px * (f16 ? 2 : 4);
        this.hostFbs = Array.from({length: kReadbackDepth + 1}, () => (f16 ? new Uint16Array(px) : new Float32Array(px)));
        this.devFbs = Array.from({length: kReadbackDepth}, () => addon().fbAlloc(this.context.device, this.fbBytes));
        for (const b of this.hostFbs) addon().hostRegister(this.context.device, b);
        this.slot = 0;
        this.framebuffer = this.hostFbs[0];
        this.image = this.canvas.present ? new Float32Array(px) : null;
    }

    // device-resident mode: the last frame's framebuffer (W x H RGBA, f32 or f16 as outFormat) copied
    // into `target` (allocated when absent) once the frames in flight are done
    readback(target) {
        if (!this.deviceFramebuffer) throw new Error('readback: the renderer is not device-resident');
        const px = this.width * this.height * 4;
        const out = target || (this.opts.outFormat === GS_OUT_RGBA_F16 ? new Uint16Array(px) : new Float32Array(px));
        addon().fbRead(this.context.device, this.deviceFramebuffer, out);
        return out;
    }

    // render one frame (depth keys + sort + tile composite), then schedule nextFrameCallback
    draw(nextFrameCallback) {
        if (this.canvas.width !== this.width || this.canvas.height !== this.height) {
            if (this.inflight > 0) {  // resize once the frames in flight have landed
                this.waiting = () => this.draw(nextFrameCallback);
                return;
            }
            this.resize();
        }
        if (this.opts.deviceResident) {
            // enqueue the frame (frames in flight, no readback) and go on: the reference's draw
            // submits to the GPU queue and returns the same way
            try {
                addon().renderDevice(this.context.device, this.scene, this.uniforms, this.width, this.height, this.opts,
                                     this.deviceFramebuffer, this.fbBytes);
                this.frames++;
                if (typeof this.canvas.onFrame === 'function') this.canvas.onFrame(this);
            } catch (err) {
                this.lastError = err;
                if (typeof this.canvas.onError === 'function') this.canvas.onError(err);
            }
            raf(nextFrameCallback);
            return;
        }
        // host readback, up to kReadbackDepth frames in flight: render into device framebuffer
        // f % D, copy it out asynchronously into host array f % (D + 1), and request the next frame
        // at once unless D are already in flight.  Frames are delivered (renderer.framebuffer,
        // canvas.onFrame) in order, each when its copy has landed; the delivered frame's array is
        // not written again before the next frame is delivered.
        const D = kReadbackDepth;
        const k = this.slot % D, h = this.slot % (D + 1);
        this.slot = (this.slot + 1) % (D * (D + 1));
        let copied;
        try {
            addon().renderDevice(this.context.device, this.scene, this.uniforms, this.width, this.height, this.opts,
                                 this.devFbs[k], this.fbBytes);
            copied = addon().readbackAsync(this.context.device, this.devFbs[k], this.hostFbs[h]);
        } catch (err) {
            this.lastError = err;
            if (typeof this.canvas.onError === 'function') this.canvas.onError(err);
            raf(nextFrameCallback);
            return;
        }
        const host = this.hostFbs[h];
        this.inflight++;
        const landed = () => {
            this.inflight--;
            const w = this.waiting;
            this.waiting = null;
            if (w) raf(w);
        };
        this.delivered = this.delivered.then(() => copied).then(() => {
            this.frames++;
            this.framebuffer = host;
            this.canvas.framebuffer = host;
            if (this.image) {
                addon().present(host, this.width, this.height, this.image);
                this.canvas.image = this.image;
            }
            if (typeof this.canvas.onFrame === 'function') this.canvas.onFrame(this);
            landed();
        }, (err) => {
            this.lastError = err;
            if (typeof this.canvas.onError === 'function') this.canvas.onError(err);
            landed();
        });
        if (this.inflight < kReadbackDepth) raf(nextFrameCallback);
        else this.waiting = nextFrameCallback;
    }

    animate(forceDraw) {
        const t = now();
        const fps = 1000 / (t - this.lastDraw);
        this.lastDraw = t;
        this.fpsCounter.innerText = 'FPS: ' + fps.toFixed(2);
        if (this.fpsCounter.style) this.fpsCounter.style.display = 'block';

        if (this.destroyCallback !== null) {
            if (this.inflight > 0) {  // the frames in flight land first (their buffers are freed)
                this.waiting = () => this.animate();
                return;
            }
            this.destroyImpl();
            return;
        }
        if (!this.interactiveCamera.isDirty() && !forceDraw) {
            raf(() => this.animate());
            return;
        }
        const camera = this.interactiveCamera.getCamera();
        const position = camera.getPosition();
        const tanHalfFovX = 0.5 * this.canvas.width / camera.focalX;
        const tanHalfFovY = 0.5 * this.canvas.height / camera.focalY;
        this.uniforms = addon().packUniforms(camera.viewMatrix, camera.perspective, position, tanHalfFovX, tanHalfFovY,
                                             camera.focalX, camera.focalY, camera.scaleModifier);
        this.draw(() => this.animate());
    }

    timings() {
        return addon().timings(this.context.device);
    }
}

module.exports = {
    GpuContext, Renderer, PackedGaussians, Camera, HeadlessCamera, addon,
    GS_ACCUM_FP32, GS_ACCUM_FP16_TARGET, GS_OUT_RGBA_F32, GS_OUT_RGBA_F16,
};
