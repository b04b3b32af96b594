// Driver for tests/test_ts.py: run an ONNX model through the TypeScript host's
// onnxruntime-web surface (segment.js InferenceSession / Tensor) and write the
// outputs back.
//   node run_onnx.js <model.onnx> <inputs.bin> <out prefix> [<unsupported.onnx> [<precision>]]
// inputs.bin holds every input's float32 data, in the session's input order;
// output k is written to <out prefix>_<k>.bin.
'use strict';
const fs = require('fs');
const path = require('path');
const ort = require(path.join(__dirname, '..', '..', 'video-stream-segmenetation_amd', 'ts', 'segment.js'));

async function main() {
  const [modelPath, inputsPath, outPrefix, badModel, precision] = process.argv.slice(2);
  // from bytes, as a bundler-fetched ArrayBuffer would arrive
  const session = await ort.InferenceSession.create(new Uint8Array(fs.readFileSync(modelPath)),
                                                    { executionProviders: ['wasm'], precision: precision || 'f32' });
  const raw = fs.readFileSync(inputsPath);
  const all = new Float32Array(raw.buffer.slice(raw.byteOffset, raw.byteOffset + raw.byteLength));
  const feeds = {};
  let off = 0;
  session.inputNames.forEach((name, i) => {
    const dims = session.inputShapes[i];
    const n = dims.reduce((a, b) => a * b, 1);
    feeds[name] = new ort.Tensor('float32', all.subarray(off, off + n).slice(), dims);
    off += n;
  });
  // two concurrent runs are serialised on the session; graph replay is deterministic
  const [a, b] = await Promise.all([session.run(feeds), session.run(feeds)]);
  let replaySame = true;
  session.outputNames.forEach((name, k) => {
    const t = a[name];
    fs.writeFileSync(`${outPrefix}_${k}.bin`, Buffer.from(t.data.buffer, t.data.byteOffset, t.data.byteLength));
    replaySame = replaySame && t.data.every((v, i) => v === b[name].data[i]);
  });
  // a wrongly shaped feed rejects without breaking later runs
  let badDimsRejected = false;
  const name0 = session.inputNames[0];
  const wrong = {};
  wrong[name0] = new ort.Tensor('float32', new Float32Array(4), [1, 1, 2, 2]);
  try { await session.run(wrong); } catch (e) { badDimsRejected = e instanceof RangeError; }
  const again = await session.run(feeds);
  const afterReject = again[session.outputNames[0]].data.every((v, i) => v === a[session.outputNames[0]].data[i]);
  let unsupported = null;
  if (badModel) {
    try { await ort.InferenceSession.create(badModel); } catch (e) { unsupported = { code: e.code, message: e.message }; }
  }
  await session.release();
  let releasedRejects = false;
  try { await session.run(feeds); } catch (e) { releasedRejects = true; }
  console.log(JSON.stringify({
    inputNames: session.inputNames, outputNames: session.outputNames,
    outputDims: session.outputNames.map((n) => a[n].dims), outputTypes: session.outputNames.map((n) => a[n].type),
    replaySame, badDimsRejected, afterReject, unsupported, releasedRejects,
  }));
}
main().catch((e) => { console.error(e); process.exit(1); });
