// The TS copy path (segmentFrames with separate per-frame Uint8Arrays), timed
// with the JS thread's own share: the synchronous part of each addon.segment
// call (staging copy + queueing) vs the whole batch interval.  Run with
// VSS_TIME_SUBMIT=1 for the library's submit phases.
//   node tools/ts_copy_probe.js [iters] [window]
'use strict';
const path = require('path');
const seg = require(path.join(__dirname, '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));
async function main() {
  const it = Number(process.argv[2] || 400);
  const b = 8, h = 480, w = 640;
  const s = new seg.Segmenter({ maxBatch: b, maxFrameWidth: w, maxFrameHeight: h, queueDepth: 4 });
  const win = Number(process.argv[3] || 2 * s.queueDepth);
  const frames = [];
  for (let i = 0; i < b; i++) frames.push({ data: new Uint8Array(h * w * 3).fill(i * 20), width: w, height: h, channels: 3 });
  for (let i = 0; i < 150; i++) await s.segmentFrames(frames);
  // wrap the addon call the Segmenter makes to time its synchronous part
  const orig = s.submitBatch.bind(s);
  let inCall = 0;
  s.submitBatch = function (f) {
    const t = process.hrtime.bigint();
    const p = orig(f);
    inCall += Number(process.hrtime.bigint() - t);
    return p;
  };
  for (let rep = 0; rep < 2; rep++) {
    inCall = 0;
    const t0 = process.hrtime.bigint();
    let ps = [];
    for (let i = 0; i < it; i++) {
      ps.push(s.segmentFrames(frames));
      if (ps.length === win) { await ps[0]; ps = ps.slice(1); }
    }
    await Promise.all(ps);
    const el = Number(process.hrtime.bigint() - t0);
    console.log(JSON.stringify({ rep: rep, window: win, frames_per_s: Math.round(b * it / (el / 1e9)),
                                 us_per_batch: el / it / 1e3, submit_call_us: inCall / it / 1e3 }));
  }
  s.close();
}
main().catch((e) => { console.error(e); process.exit(1); });
