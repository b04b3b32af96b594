"""Real-weight ONNX fixtures for the GPU ONNX sessions (run in the build
container, where /root/reference exists; the GPU box only reads the .npz).

The reference ships two intact ORT models it creates sessions for
(client/src/core/main.ts:7-8, model.ts:36-67): MediaPipeFaceDetector.onnx and
MediaPipeFaceLandmarkDetector.onnx (client/src/assets/).  This script parses
each with oracle/onnx_ref.py, stores its graph (nodes and attributes as JSON,
initializers as arrays, in a compressed .npz — a re-encoding, not the file),
a seeded input image tensor in [0, 1] (what preprocessToNCHW feeds,
frameProcessorTest.ts:374-393) and the oracle's outputs for it.  The source
file's sha256 is recorded.  tests/onnx_models.py:load_golden rebuilds the
ONNX bytes from the .npz for the sessions under test.

    python tests/golden/make_onnx_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import onnx_ref as R  # noqa: E402

ASSETS = "/root/reference/client/src/assets"
MODELS = {"mediapipe_face_detector": "MediaPipeFaceDetector.onnx",
          "mediapipe_face_landmarks": "MediaPipeFaceLandmarkDetector.onnx"}


def _jsonable(v):
    if isinstance(v, np.ndarray):
        return None  # stored as an array
    return v


def main():
    for key, fname in MODELS.items():
        path = os.path.join(ASSETS, fname)
        data = open(path, "rb").read()
        m = R.load(data)
        arrays = {}
        nodes = []
        for k, nd in enumerate(m.nodes):
            attrs = {}
            for an, av in nd["attrs"].items():
                if isinstance(av, np.ndarray):
                    arrays[f"attr_{k}_{an}"] = av
                    attrs[an] = {"tensor": f"attr_{k}_{an}"}
                else:
                    attrs[an] = {"value": av}
            nodes.append({"op": nd["op"], "inputs": nd["inputs"], "outputs": nd["outputs"], "attrs": attrs})
        init_names = list(m.inits)
        for k, n in enumerate(init_names):
            arrays[f"init_{k}"] = m.inits[n]
        rng = np.random.default_rng(20251024)
        feeds = {}
        for (name, _, dims) in m.inputs:
            feeds[name] = rng.random(dims, dtype=np.float32)
        want = R.run(m, feeds)
        meta = {"source": f"client/src/assets/{fname}", "sha256": hashlib.sha256(data).hexdigest(),
                "opset": m.opset, "nodes": nodes, "inits": init_names,
                "inputs": [[n, e, d] for n, e, d in m.inputs], "outputs": [[n, e, d] for n, e, d in m.outputs],
                "feeds": list(feeds), "expected": list(want)}
        for k, (n, v) in enumerate(feeds.items()):
            arrays[f"feed_{k}"] = v
        for k, (n, v) in enumerate(want.items()):
            arrays[f"want_{k}"] = v
        arrays["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
        out = os.path.join(HERE, key + ".npz")
        np.savez_compressed(out, **arrays)
        print(f"{out}: {len(nodes)} nodes, {len(init_names)} initializers, "
              f"outputs {[(k, v.shape) for k, v in want.items()]}, {os.path.getsize(out) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
