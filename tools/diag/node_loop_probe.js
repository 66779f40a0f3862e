'use strict';
// Node: where the host-readback frame loop spends its time (wraps the addon calls the Renderer
// makes and times them).   node tools/diag/node_loop_probe.js [n]
const path = require('path');
const gs = require(path.join(__dirname, '..', '..', 'gaussian-splatting-web_amd', 'js'));

async function main() {
    const n = Number(process.argv[2] || 6100000), W = 1920, H = 1080;
    const a = gs.addon();
    const now = () => Number(process.hrtime.bigint()) / 1e3;
    const acc = {};
    for (const name of ['renderDevice', 'readbackAsync', 'packUniforms', 'cameraPosition', 'hostRegister']) {
        const f = a[name];
        a[name] = (...args) => {
            const t0 = now();
            const r = f(...args);
            const d = now() - t0;
            acc[name] = acc[name] || {n: 0, us: 0, max: 0};
            acc[name].n++;
            acc[name].us += d;
            acc[name].max = Math.max(acc[name].max, d);
            return r;
        };
    }
    const buf = a.synthAos(n, 6, W, H);
    const gaussians = new gs.PackedGaussians(buf, n, 16);
    const cam = gs.Camera.lookAt([0, 0, 0], [0, 0, -1], W, H);
    const icam = new gs.HeadlessCamera(cam);
    const context = await gs.Renderer.requestContext(gaussians, 0);
    const canvas = {width: W, height: H};
    let seen = 0, t0 = 0;
    const frames = 100;
    const done = new Promise((resolve) => {
        canvas.onFrame = (r) => {
            seen++;
            if (seen === 5) t0 = now();
            if (seen < frames + 5) icam.setDirty(); else resolve(r);
        };
    });
    const renderer = new gs.Renderer(canvas, icam, gaussians, context, null, {outFormat: gs.GS_OUT_RGBA_F16});
    await done;
    const per = (now() - t0) / frames;
    await renderer.destroy();
    for (const k of Object.keys(acc)) acc[k].mean = acc[k].us / acc[k].n;
    console.log(JSON.stringify({frame_us: per, calls: acc}));
}
main().catch((e) => { console.error('FAILED', e); process.exit(1); });
