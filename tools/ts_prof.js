// The TS zero-copy loop alone, for `node --cpu-prof` (where the JS thread's
// time goes per batch).  node --cpu-prof tools/ts_prof.js [iters]
'use strict';
const path = require('path');
const seg = require(path.join(__dirname, '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));
async function main() {
  const it = Number(process.argv[2] || 2000);
  const b = 8, h = 480, w = 640;
  const s = new seg.Segmenter({ maxBatch: b, maxFrameWidth: w, maxFrameHeight: h, queueDepth: 4 });
  const frames = [];
  for (let i = 0; i < b; i++) frames.push({ data: new Uint8Array(h * w * 3).fill(i * 20), width: w, height: h, channels: 3 });
  for (let i = 0; i < 150; i++) await s.segmentFrames(frames);
  const t0 = process.hrtime.bigint();
  let zs = [];
  for (let i = 0; i < it; i++) {
    if (zs.length === s.queueDepth) { await zs[0]; zs = zs.slice(1); }
    const lease = s.acquireFrames();
    zs.push(s.segmentLease(lease, b, w, h));
  }
  for (const p of zs) await p;
  const el = Number(process.hrtime.bigint() - t0) / 1e9;
  console.log(JSON.stringify({ frames_per_s: Math.round(b * it / el), ms_per_batch: el * 1e3 / it }));
  s.close();
}
main().catch((e) => { console.error(e); process.exit(1); });
