'use strict';
// Node: where the device-resident frame loop spends its time.  The Renderer's addon calls are
// wrapped and timed (mean/max), and the loop's period is split into time inside renderDevice and
// the rest (JS frame loop + rAF shim).   node tools/diag/node_dev_probe.js [n] [frames]
const path = require('path');
const gs = require(path.join(__dirname, '..', '..', 'gaussian-splatting-web_amd', 'js'));

async function main() {
    const n = Number(process.argv[2] || 6100000), frames = Number(process.argv[3] || 300), W = 1920, H = 1080;
    const a = gs.addon();
    const now = () => Number(process.hrtime.bigint()) / 1e3;
    const acc = {};
    for (const name of ['renderDevice', 'packUniforms']) {
        const f = a[name];
        a[name] = (...args) => {
            const t0 = now();
            const r = f(...args);
            const d = now() - t0;
            const e = acc[name] = acc[name] || {n: 0, us: 0, max: 0, samples: []};
            e.n++;
            e.us += d;
            e.max = Math.max(e.max, d);
            e.samples.push(d);
            return r;
        };
    }
    const buf = a.synthAos(n, 6, W, H);
    const gaussians = new gs.PackedGaussians(buf, n, 16);
    const cam = gs.Camera.lookAt([0, 0, 0], [0, 0, -1], W, H);
    const icam = new gs.HeadlessCamera(cam);
    let drawn = 0;
    icam.getCamera = function () {
        if (++drawn >= frames + 5) this.dirty = false;
        return this.camera;
    };
    const context = await gs.Renderer.requestContext(gaussians, 0);
    const canvas = {width: W, height: H};
    let seen = 0, t0 = 0, t1 = 0;
    const done = new Promise((resolve) => {
        canvas.onFrame = (r) => {
            seen++;
            if (seen === 5) {
                t0 = now();
                for (const k in acc) acc[k] = {n: 0, us: 0, max: 0, samples: []};
            }
            if (seen >= frames + 5) { t1 = now(); resolve(r); }
        };
    });
    const renderer = new gs.Renderer(canvas, icam, gaussians, context, null,
                                     {outFormat: gs.GS_OUT_RGBA_F16, deviceResident: true});
    const r = await done;
    r.readback();
    const per = (t1 - t0) / frames;
    const out = {node: process.version, frames, us_per_frame: per};
    for (const k in acc) {
        const s = acc[k].samples.sort((x, y) => x - y);
        out[k] = {mean: acc[k].us / acc[k].n, p50: s[s.length >> 1], p90: s[Math.floor(s.length * 0.9)], max: acc[k].max};
    }
    out.outside_render_us = per - out.renderDevice.mean;
    console.log(JSON.stringify(out));
    await renderer.destroy();
}
main().catch((e) => { console.error('FAILED', e); process.exit(1); });
