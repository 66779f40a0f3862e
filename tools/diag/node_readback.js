'use strict';
// Node: time the host side of readbackAsync (gs_readback_start) with and without hostRegister,
// and the copy's landing, for a W x H f16 framebuffer.   node tools/diag/node_readback.js
const path = require('path');
const gs = require(path.join(__dirname, '..', '..', 'gaussian-splatting-web_amd', 'js'));

async function main() {
    const a = gs.addon();
    const W = 1920, H = 1080, px = W * H * 4, bytes = px * 2;
    const ctx = a.ctxCreate(0);
    const fb = a.fbAlloc(ctx, bytes);
    const now = () => Number(process.hrtime.bigint()) / 1e3;
    for (const reg of [false, true]) {
        const host = new Uint16Array(px);
        if (reg) a.hostRegister(ctx, host);
        let tStart = 0, tAll = 0;
        const N = 50;
        for (let i = 0; i < N; ++i) {
            const t0 = now();
            const p = a.readbackAsync(ctx, fb, host);
            const t1 = now();
            await p;
            const t2 = now();
            tStart += t1 - t0;
            tAll += t2 - t0;
        }
        console.log(JSON.stringify({registered: reg, start_us: tStart / N, landed_us: tAll / N,
                                    GBs: bytes / (tAll / N) / 1e3}));
        if (reg) a.hostUnregister(ctx, host);
    }
    a.fbFree(ctx, fb);
    a.ctxDestroy(ctx);
}
main().catch((e) => { console.error('FAILED', e); process.exit(1); });
