// Driver for tests/test_ts.py: the post chain with the face stabiliser's inputs
// through the TypeScript host (PostChain.processFrames(frames, faces)).
//   node run_face.js <frames.bin> <n> <height> <width> <channels> <faces.json> <out prefix>
'use strict';
const fs = require('fs');
const path = require('path');
const seg = require(path.join(__dirname, '..', '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));

async function main() {
  const [framesPath, n, h, w, c, facesPath, outPath] = process.argv.slice(2);
  const N = +n, H = +h, W = +w, C = +c;
  const raw = fs.readFileSync(framesPath);
  const bytes = H * W * C;
  const frames = [];
  for (let i = 0; i < N; i++) {
    frames.push({ data: new Uint8Array(raw.buffer, raw.byteOffset + i * bytes, bytes), width: W, height: H, channels: C });
  }
  const faces = JSON.parse(fs.readFileSync(facesPath, 'utf8'));
  const s = new seg.Segmenter({ dtype: 'bf16x2', maxBatch: N, maxFrameWidth: W, maxFrameHeight: H });
  const post = new seg.PostChain(s, {});
  const r = await post.processFrames(frames, faces);
  let mismatchRejected = false;
  try { await post.processFrames(frames, faces.slice(1)); } catch (e) { mismatchRejected = e instanceof RangeError; }
  fs.writeFileSync(outPath + '.f32', Buffer.from(r.alpha.buffer, r.alpha.byteOffset, r.alpha.byteLength));
  fs.writeFileSync(outPath + '.u8', Buffer.from(r.alphaU8.buffer, r.alphaU8.byteOffset, r.alphaU8.byteLength));
  console.log(JSON.stringify({ count: r.count, width: r.width, height: r.height, mismatchRejected }));
  post.close();
  s.close();
}
main().catch((e) => { console.error(e); process.exit(1); });
