// Driver for tests/test_ts.py: the queued Segmenter.  Fires every call at once
// (more than queueDepth, so some wait in the JS queue) and records the order
// the promises resolve in; writes each call's masks.
//   node run_queue.js <frames.bin> <n> <height> <width> <channels> <outPrefix> <queueDepth> [deviceIds]
'use strict';
const fs = require('fs');
const path = require('path');
const seg = require(path.join(__dirname, '..', '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));

async function main() {
  const [framesPath, n, h, w, c, outPrefix, depth, ids] = process.argv.slice(2);
  const N = +n, H = +h, W = +w, C = +c;
  const raw = fs.readFileSync(framesPath);
  const bytes = H * W * C;
  const frames = [];
  for (let i = 0; i < N; i++) {
    frames.push({ data: new Uint8Array(raw.buffer, raw.byteOffset + i * bytes, bytes), width: W, height: H, channels: C });
  }
  const opts = { maxBatch: N, maxFrameWidth: W, maxFrameHeight: H, queueDepth: +depth };
  if (ids) opts.deviceIds = ids.split(',').map(Number);
  const s = new seg.Segmenter(opts);
  const order = [];
  // calls: each frame alone, then the whole batch, then the batch reversed
  const calls = frames.map((f) => [f]);
  calls.push(frames);
  calls.push(frames.slice().reverse());
  const ps = calls.map((fs_, i) => s.segmentFrames(fs_).then((r) => { order.push(i); return r; }));
  ps.push(s.segmentFrames([]).then(() => 'accepted', (e) => (e instanceof RangeError ? 'rejected' : String(e))));
  const res = await Promise.all(ps);
  for (let i = 0; i < calls.length; i++) {
    const m = res[i].masks;
    fs.writeFileSync(outPrefix + '.' + i, Buffer.from(m.buffer, m.byteOffset, m.byteLength));
  }
  // zero-copy leases (single-GPU handles): frames decoded into pinned staging
  let leaseEqual = null;
  if (!ids) {
    const whole = res[N].masks;
    const lease = s.acquireFrames();
    for (let i = 0; i < N; i++) lease.data.set(frames[i].data, i * bytes);
    const other = s.segmentFrames(frames);  // runs on another slot meanwhile
    const r = await s.segmentLease(lease, N, W, H, C);
    await other;
    leaseEqual = r.count === N && r.masks.every((v, i) => v === whole[i]);
    s.releaseFrames(s.acquireFrames());  // a lease given back unused
  }
  console.log(JSON.stringify({ order: order, calls: calls.length, empty: res[calls.length],
                               queueDepth: s.queueDepth, nGpus: s.nGpus, leaseEqual: leaseEqual }));
  s.close();
}
main().catch((e) => { console.error(e); process.exit(1); });
