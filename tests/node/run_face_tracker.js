// Driver for tests/test_ts.py: the GPU face stage through the TypeScript host
// (segment.js FaceTracker over two InferenceSessions), its faces fed to a
// PostChain as processFrame would.
//   node run_face_tracker.js <detector.onnx> <landmarks.onnx> <frames.bin> <n> <h> <w> <c> <out prefix>
// Prints the per-frame FaceInputs as JSON; writes the post chain's alpha to <out prefix>.f32.
'use strict';
const fs = require('fs');
const path = require('path');
const vss = require(path.join(__dirname, '..', '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));

async function main() {
  const [detPath, lmkPath, framesPath, n_, h_, w_, c_, outPrefix] = process.argv.slice(2);
  const n = +n_, h = +h_, w = +w_, c = +c_;
  const det = await vss.InferenceSession.create(detPath, {});
  const lmk = await vss.InferenceSession.create(lmkPath, {});
  const tracker = new vss.FaceTracker(det, lmk, { interval: 3 });
  const raw = fs.readFileSync(framesPath);
  const frames = [];
  for (let t = 0; t < n; t++) {
    frames.push({ data: new Uint8Array(raw.buffer, raw.byteOffset + t * h * w * c, h * w * c), width: w, height: h,
                  channels: c });
  }
  const seg = new vss.Segmenter({ modelHeight: 48, modelWidth: 64, dtype: 'f32', maxBatch: 8, maxFrameHeight: h,
                                  maxFrameWidth: w, autotune: false });
  // two calls: the stage's frame index and lastAffine carry across them
  const a = await tracker.track(frames.slice(0, 4), seg.maskWidth, seg.maskHeight);
  const b = await tracker.track(frames.slice(4), seg.maskWidth, seg.maskHeight);
  const faces = a.concat(b);
  const post = new vss.PostChain(seg);
  const r = await post.processFrames(frames, faces);
  fs.writeFileSync(outPrefix + '.f32', Buffer.from(r.alpha.buffer, r.alpha.byteOffset, r.alpha.byteLength));
  let releaseBlocked = false;
  try { await det.release(); } catch (e) { releaseBlocked = true; }  // the tracker still uses it
  await tracker.release();
  let releasedRejects = false;
  try { await tracker.track(frames, seg.maskWidth, seg.maskHeight); } catch (e) { releasedRejects = true; }
  await det.release();
  await lmk.release();
  post.close();
  seg.close();
  console.log(JSON.stringify({ faces, releaseBlocked, releasedRejects }));
}

main().catch((e) => { console.error(e); process.exit(1); });
