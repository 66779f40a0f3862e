'use strict';
// GPU: the reference's frame loop through the Node host.  Loads an AoS scene file, renders with
// Renderer (GpuContext.create -> new Renderer -> animate/draw loop -> destroy) at a fixture
// camera, and writes the framebuffer of frame `frames` to a file.
// Usage: node render_frames.js <aos.bin> <n> <nsh> <uniforms160.bin> <W> <H> <out.f32> [frames] [devices]
// devices: comma-separated device list for a device group (e.g. 0,0,0 on one GPU).
const fs = require('fs');
const path = require('path');
const gs = require(path.join(__dirname, '..', '..', 'gaussian-splatting-web_amd', 'js'));

async function main() {
    const [aosPath, n, nsh, uniPath, W, H, outPath, framesArg, devArg] = process.argv.slice(2);
    const devices = devArg ? devArg.split(',').map(Number) : 0;
    const frames = Number(framesArg || 3);
    const aos = fs.readFileSync(aosPath);
    const gaussians = new gs.PackedGaussians(aos.buffer.slice(aos.byteOffset, aos.byteOffset + aos.byteLength),
                                             Number(n), Number(nsh));
    const ub = fs.readFileSync(uniPath);  // small files come from Node's buffer pool: honour the offset
    const uni = new Float32Array(ub.buffer.slice(ub.byteOffset, ub.byteOffset + ub.byteLength));
    // a camera whose getCamera() yields exactly the fixture's matrices
    const cam = new gs.Camera(Number(H), Number(W), uni.slice(0, 16), uni.slice(16, 32), Number(W), Number(H), 1);
    const icam = new gs.HeadlessCamera(cam);
    const context = await gs.Renderer.requestContext(gaussians, devices);
    const canvas = {width: Number(W), height: Number(H), present: true};
    const fps = {innerText: '', style: {}};
    let seen = 0;
    const done = new Promise((resolve, reject) => {
        canvas.onError = reject;
        canvas.onFrame = (r) => {
            seen++;
            if (seen < frames) icam.setDirty();  // force the next frames through the full path
            else resolve(r);
        };
    });
    const renderer = new gs.Renderer(canvas, icam, gaussians, context, fps);
    const r = await done;
    fs.writeFileSync(outPath, Buffer.from(r.framebuffer.buffer));
    fs.writeFileSync(outPath + '.present', Buffer.from(canvas.image.buffer));
    await renderer.destroy();
    console.log(JSON.stringify({frames: seen, fps: fps.innerText, destroyed: context.device === null}));
}

main().catch((e) => {
    console.error('FAILED', e);
    process.exit(1);
});
