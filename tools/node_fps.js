'use strict';
// Frame rate of the Node drop-in: the reference's frame loop (GpuContext.create -> new Renderer ->
// animate/draw via the rAF shim) on the seeded synthetic scene at the bench camera, every frame
// forced through the full path (the camera stays dirty, as a moving one: frames are requested back
// to back), measured in JS from the fifth frame's callback to the last.  Two modes: deviceResident (frames stay in HBM, as the reference's
// framebuffer texture; frames in flight) and host readback (renderAsync + a D2H copy per frame).
// The device-resident mode's last frame is read back and compared with the host mode's.
// Usage: node tools/node_fps.js <n> <seed> <W> <H> <frames>   -> one JSON line
const path = require('path');
const gs = require(path.join(__dirname, '..', 'gaussian-splatting-web_amd', 'js'));
// warm-up frames before timing: the chunk controller's statistics reach the host a few frames
// late, so the first frames of a scene run with a seeded or a stale split (with 5 warm-up frames
// and 100 timed ones the Node line read ~0.43 ms per frame against ~0.30 ms at steady state)
const kWarm = 20;

async function run(gaussians, W, H, frames, options) {
    const a = gs.addon();
    const cam = gs.Camera.lookAt([0, 0, 0], [0, 0, -1], W, H);
    // a camera that stays dirty until the measured frames are drawn (a moving camera, as under
    // user input): frames are requested back to back, not each after the last one's callback
    const icam = new gs.HeadlessCamera(cam);
    let drawn = 0;
    icam.getCamera = function () {
        if (++drawn >= frames + kWarm) this.dirty = false;
        return this.camera;
    };
    const context = await gs.Renderer.requestContext(gaussians, 0);
    const canvas = {width: W, height: H};
    let seen = 0, t0 = 0n, t1 = 0n;
    const done = new Promise((resolve, reject) => {
        canvas.onError = reject;
        canvas.onFrame = (r) => {
            seen++;
            if (seen === kWarm) t0 = process.hrtime.bigint();  // warm-up frames (bench.py's count)
            if (seen >= frames + kWarm) { t1 = process.hrtime.bigint(); resolve(r); }
        };
    });
    const renderer = new gs.Renderer(canvas, icam, gaussians, context, null, options);
    const r = await done;
    let img;
    if (options.deviceResident) {
        img = r.readback();  // waits for the frames in flight
        t1 = process.hrtime.bigint();
    } else {
        img = r.framebuffer.slice();
    }
    const ms = Number(t1 - t0) / 1e6 / frames;
    await renderer.destroy();
    void a;
    return {ms, img};
}

async function main() {
    const [n, seed, W, H, frames] = process.argv.slice(2).map(Number);
    const buf = gs.addon().synthAos(n, seed, W, H);
    const gaussians = new gs.PackedGaussians(buf, n, 16);
    const opts = {outFormat: gs.GS_OUT_RGBA_F16};
    const dev = await run(gaussians, W, H, frames, Object.assign({deviceResident: true}, opts));
    const host = await run(gaussians, W, H, frames, opts);
    let same = dev.img.length === host.img.length;
    for (let i = 0; same && i < dev.img.length; ++i) same = dev.img[i] === host.img[i];
    console.log(JSON.stringify({n, W, H, frames, device_resident_fps: 1000 / dev.ms, device_resident_ms: dev.ms,
                                host_readback_fps: 1000 / host.ms, host_readback_ms: host.ms, same_image: same}));
}

main().catch((e) => {
    console.error('FAILED', e);
    process.exit(1);
});
