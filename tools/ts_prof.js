// Phase table of the TypeScript host (VERDICT r5 #2): where one segmentFrame /
// segmentFrames call's wall time goes, from the JS call to the resumed await.
//   node tools/ts_prof.js [iters] [--zero-copy]
// Runs with VSS_NAPI_TRACE=1 (the addon stamps every batch, vss_napi.cc
// TracePoint; the stamps share process.hrtime's CLOCK_MONOTONIC) and prints one
// JSON line: per mode, the median / p90 of each phase in microseconds, plus the
// pipelined throughput of segmentFrames (queueDepth batches in flight).
//   js_call      segmentFrames() entered -> the addon's segment() entered (segment.ts)
//   addon_call   segment(): arguments, result block, references, enqueue
//   thread_hop   enqueue -> the handle's submit thread picks the batch up
//   submit       vss_submit_list_async: staging copy into pinned memory + enqueue
//   device       H2D -> forward -> D2H -> completion callback (library's thread)
//   deliver_hop  completion callback -> the JS thread runs the delivery (tsfn)
//   settle       Float32Array + promise resolve
//   js_resume    resolve -> the caller's await resumes (segment.ts's ordered chain)
'use strict';
process.env.VSS_NAPI_TRACE = '1';
const path = require('path');
const seg = require(path.join(__dirname, '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));
const addon = require(path.join(__dirname, '..', 'video-stream-segmenetation_amd', 'ts', 'addon', 'vss_napi.node'));

const NP = 8;  // TracePoint count + frames, vss_napi.cc
const PH = ['js_call', 'addon_call', 'thread_hop', 'submit', 'device', 'deliver_hop', 'settle', 'js_resume'];

function stats(v) {
  const a = v.slice().sort((x, y) => x - y);
  const q = (p) => Math.round(a[Math.min(a.length - 1, Math.floor(p * a.length))] * 10) / 10;
  return { p50: q(0.5), p90: q(0.9) };
}

// rows of the addon's trace + the JS stamps (ns) of the same calls, in order
function table(js) {
  const t = addon.traceDump();
  const n = Math.min(js.length, t.length / NP);
  const ph = PH.map(() => []);
  const total = [];
  for (let i = 0; i < n; i++) {
    const r = t.subarray(i * NP, (i + 1) * NP);
    const [j0, j1] = js[i];
    const pts = [j0, r[0], r[1], r[2], r[3], r[4], r[5], r[6], j1];
    for (let k = 0; k < PH.length; k++) ph[k].push((pts[k + 1] - pts[k]) / 1e3);
    total.push((j1 - j0) / 1e3);
  }
  const out = { calls: n, total_us: stats(total), pool: addon.poolStats() };
  PH.forEach((p, k) => { out[p + '_us'] = stats(ph[k]); });
  return out;
}

async function main() {
  const args = process.argv.slice(2);
  const it = Number(args.find((a) => /^\d+$/.test(a)) || 400);
  const b = 8, h = 480, w = 640;
  const st = Number(process.env.TS_PROF_STAGING_THREADS || 0);  // 0: the library's default (8)
  const s = new seg.Segmenter({ maxBatch: b, maxFrameWidth: w, maxFrameHeight: h, queueDepth: 4, stagingThreads: st });
  const frames = [];
  for (let i = 0; i < b; i++) frames.push({ data: new Uint8Array(h * w * 3).fill(i * 20), width: w, height: h, channels: 3 });
  for (let i = 0; i < 150; i++) await s.segmentFrames(frames);
  addon.traceDump();
  const now = () => Number(process.hrtime.bigint());
  const res = {};
  // one frame per call, one call at a time (the reference's processFrame loop)
  let js = [];
  for (let i = 0; i < it; i++) {
    const t0 = now();
    await s.segmentFrame(frames[i % b]);
    js.push([t0, now()]);
  }
  res.segmentFrame = table(js);
  // a batch of 8 per call, one call at a time
  js = [];
  for (let i = 0; i < it; i++) {
    const t0 = now();
    await s.segmentFrames(frames);
    js.push([t0, now()]);
  }
  res.segmentFrames_serial = table(js);
  // pipelined: calls fired ahead (a window of 2 x queueDepth), as bench_ts.js
  const win = 2 * s.queueDepth;
  js = [];
  const t0 = now();
  let ps = [];
  for (let i = 0; i < it; i++) {
    const c = now();
    const p = s.segmentFrames(frames).then(() => { js[i] = [c, now()]; });
    ps.push(p);
    if (ps.length === win) { await ps[0]; ps = ps.slice(1); }
  }
  await Promise.all(ps);
  const el = (now() - t0) / 1e9;
  res.segmentFrames_pipelined = table(js);
  res.segmentFrames_pipelined.frames_per_s = Math.round(b * it / el);
  s.close();
  console.log(JSON.stringify(res));
}
main().catch((e) => { console.error(e); process.exit(1); });
