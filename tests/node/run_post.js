// Driver for tests/test_ts.py: the post-processing chain through the TypeScript
// host (PostChain in segment.js): two calls on one stream, then a knob change.
//   node run_post.js <frames.bin> <n> <height> <width> <channels> <out prefix> <dtype>
'use strict';
const fs = require('fs');
const path = require('path');
const seg = require(path.join(__dirname, '..', '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));

async function main() {
  const [framesPath, n, h, w, c, outPrefix, dtype] = process.argv.slice(2);
  const N = +n, H = +h, W = +w, C = +c;
  const raw = fs.readFileSync(framesPath);
  const bytes = H * W * C;
  const frames = [];
  for (let i = 0; i < N; i++) {
    frames.push({ data: new Uint8Array(raw.buffer, raw.byteOffset + i * bytes, bytes), width: W, height: H, channels: C });
  }
  const s = new seg.Segmenter({ dtype: dtype, maxBatch: N, maxFrameWidth: W, maxFrameHeight: H });
  const post = new seg.PostChain(s, {});
  const half = N >> 1;
  const a = await post.processFrames(frames.slice(0, half));
  const b = await post.processFrames(frames.slice(half));
  await post.reset();
  await post.setConfig({ USE_BILATERAL: false, GAMMA: 1.0 });
  const d = await post.processFrames(frames);
  await post.reset();
  await post.setConfig({});
  const comp = await post.compositeFrames(frames);
  fs.writeFileSync(outPrefix + '_rgba.u8', Buffer.from(comp.rgba.buffer, comp.rgba.byteOffset, comp.rgba.byteLength));
  let rejected = false;
  try { await post.setConfig({ BILATERAL_SIGMA_RANGE: 0 }); } catch (e) { rejected = e.code === '-1'; }
  const cat = (x, y, T) => { const o = new T(x.length + y.length); o.set(x, 0); o.set(y, x.length); return o; };
  const alpha = cat(a.alpha, b.alpha, Float32Array), u8 = cat(a.alphaU8, b.alphaU8, Uint8Array);
  fs.writeFileSync(outPrefix + '.f32', Buffer.from(alpha.buffer));
  fs.writeFileSync(outPrefix + '.u8', Buffer.from(u8.buffer));
  fs.writeFileSync(outPrefix + '_nobil.f32', Buffer.from(d.alpha.buffer, d.alpha.byteOffset, d.alpha.byteLength));
  console.log(JSON.stringify({ width: a.width, height: a.height, count: a.count + b.count, badConfigRejected: rejected }));
  post.close();
  s.close();
}
main().catch((e) => { console.error(e); process.exit(1); });
