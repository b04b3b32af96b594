// The TypeScript host timed end to end (SURVEY.md §8(d): segmentFrames call ->
// promise resolve, including staging, H2D, the forward and D2H), the way the
// reference times `Latency` (session.run, frameProcessorTest.ts:90-92) and
// `Total Frame` (:180-185, shown at main.ts:96-105).  Run by bench.py as its
// own child process:
//   node bench_ts.js <height> <width> <batch> <iters> [queueDepth]
// prints one JSON line: throughput with every call fired at once (the queue
// keeps queueDepth batches in flight) and the latency of one call at a time.
'use strict';
const path = require('path');
const seg = require(path.join(__dirname, '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));

function synthetic(n, h, w) {
  const frames = [];
  for (let i = 0; i < n; i++) {
    const data = new Uint8Array(h * w * 3);
    let s = 20251024 + i;
    for (let k = 0; k < data.length; k++) {
      s = (s * 1664525 + 1013904223) >>> 0;
      data[k] = s >>> 24;
    }
    frames.push({ data: data, width: w, height: h, channels: 3 });
  }
  return frames;
}

async function main() {
  const [h, w, b, it, depth] = process.argv.slice(2).map(Number);
  const frames = synthetic(b, h, w);
  const s = new seg.Segmenter({ maxBatch: b, maxFrameWidth: w, maxFrameHeight: h, queueDepth: depth || 0 });
  // warm-up: long enough for V8 to collect results and their pinned blocks to
  // come back to the addon's pool (the steady state of a video loop)
  for (let i = 0; i < 150; i++) await s.segmentFrames(frames);
  // latency: one call at a time (the reference's serialised loop)
  const lat = [];
  for (let i = 0; i < Math.max(20, it / 5); i++) {
    const t0 = process.hrtime.bigint();
    await s.segmentFrames(frames);
    lat.push(Number(process.hrtime.bigint() - t0) / 1e6);
  }
  lat.sort((a, c) => a - c);
  // one frame per call, one call at a time: the reference's own usage
  // (processFrame -> runModnetExclusive, main.ts:18-22, 66-74), whose overlay
  // shows session.run's wall time as `Latency` (frameProcessorTest.ts:90-92)
  for (let i = 0; i < 50; i++) await s.segmentFrame(frames[0]);
  const lat1 = [];
  const n1 = Math.max(200, it);
  const t1 = process.hrtime.bigint();
  for (let i = 0; i < n1; i++) {
    const t0 = process.hrtime.bigint();
    await s.segmentFrame(frames[i % b]);
    lat1.push(Number(process.hrtime.bigint() - t0) / 1e6);
  }
  const el1 = Number(process.hrtime.bigint() - t1) / 1e9;
  lat1.sort((a, c) => a - c);
  const pct = (a, q) => Math.round(a[Math.min(a.length - 1, Math.floor(q * a.length))] * 1e4) / 1e4;
  // throughput: calls fired ahead of their results (a window of 2 x the queue
  // depth outstanding, so resolved results are dropped as a consumer would)
  const win = 2 * s.queueDepth;
  async function copyLoop(n) {
    const t0 = process.hrtime.bigint();
    let ps = [];
    for (let i = 0; i < n; i++) {
      ps.push(s.segmentFrames(frames));
      if (ps.length === win) { await ps[0]; ps = ps.slice(1); }
    }
    await Promise.all(ps);
    return Number(process.hrtime.bigint() - t0) / 1e9;
  }
  // zero-copy: frames decoded straight into leased pinned staging (the
  // synthetic decoder fills each slot's buffer once; later leases find them)
  const filled = new Set();
  const fb = h * w * 3;
  let last = null;
  async function zeroCopyLoop(n) {
    const z0 = process.hrtime.bigint();
    let zs = [];
    for (let i = 0; i < n; i++) {
      if (zs.length === s.queueDepth) { last = await zs[0]; zs = zs.slice(1); }  // a slot's batch is done
      const lease = s.acquireFrames();
      if (!filled.has(lease.slot)) {
        for (let k = 0; k < b; k++) lease.data.set(frames[k].data, k * fb);
        filled.add(lease.slot);
      }
      zs.push(s.segmentLease(lease, b, w, h));
    }
    for (const p of zs) last = await p;
    return Number(process.hrtime.bigint() - z0) / 1e9;
  }
  // each loop runs untimed once first: the first few hundred batches of a
  // cold pipelined loop run up to 1.5x slower (copy threads, DMA queues)
  await copyLoop(it);
  const el = await copyLoop(it);
  await zeroCopyLoop(it);
  const zel = await zeroCopyLoop(it);
  const ref = (await s.segmentFrames(frames)).masks;
  const zsame = last.masks.every((v, k) => v === ref[k]);
  console.log(JSON.stringify({ value: Math.round(b * it / el * 10) / 10, unit: 'frames/s',
                               ms_per_batch: Math.round(el * 1e3 / it * 1e4) / 1e4, iters: it,
                               latency_ms_p50: Math.round(lat[lat.length >> 1] * 1e4) / 1e4,
                               latency_ms_min: Math.round(lat[0] * 1e4) / 1e4, latency_ms_p99: pct(lat, 0.99),
                               queue_depth: s.queueDepth,
                               single_frame: { entry: 'Segmenter.segmentFrame, one 640x480 frame per call, one call at a time',
                                               calls: n1, latency_ms_p50: pct(lat1, 0.5), latency_ms_p99: pct(lat1, 0.99),
                                               latency_ms_min: Math.round(lat1[0] * 1e4) / 1e4,
                                               frames_per_s: Math.round(n1 / el1 * 10) / 10 },
                               entry: 'Segmenter.segmentFrames (TS -> N-API -> vss_submit_list / vss_wait)',
                               zero_copy: { value: Math.round(b * it / zel * 10) / 10,
                                            ms_per_batch: Math.round(zel * 1e3 / it * 1e4) / 1e4,
                                            masks_equal_copy_path: zsame,
                                            entry: 'Segmenter.acquireFrames + segmentLease (decode into pinned staging)' } }));
  s.close();
}
main().catch((e) => { console.error(e); process.exit(1); });
