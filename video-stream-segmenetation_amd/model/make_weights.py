"""Seeded weight generator for the build-defined network (spec.json).

The reference's segmentation weights (`client/src/assets/model_q4f16.onnx`) are
absent (`/root/reference/.MISSING_LARGE_BLOBS:7`), so the network is the
build's own and its weights come from numpy PCG64 with a
fixed seed.  The blob written here is the ONE weights file both the HIP
library (`csrc/vss_capi.hip`) and the CPU oracle (`oracle/vss_oracle.c`)
interpret: a self-describing layer table followed by f32 tensors.

Blob layout (little endian):
    header  8 x u32 : magic 'VSSW', version, n_layers, n_floats, eps(f32 bits), 0, 0, 0
    layers  n_layers x 16 x u32 :
            kind, cin, chid, cout, stride, flags, src, skip,
            off_w1, off_b1, off_wdw, off_bdw, off_w2, off_b2, off_gamma, off_beta
    data    n_floats x f32
kind: 1 stem, 2 ir (inverted residual), 3 dec (decoder), 4 head.
flags: 1 EXPAND, 2 RESIDUAL.  Offsets are float indices into `data`, NONE = 0xFFFFFFFF.
Pointwise weights (ir w1/w2, dec w2) are bf16-exact.
Tensor layouts (PyTorch OIHW order): stem w1 [cout][3][3][3]; ir w1 [chid][cin],
wdw [chid][9], w2 [cout][chid]; dec wdw [cin+cskip][9], w2 [cout][cin+cskip];
head w2 [1][cin].  For dec, `chid` holds cskip.
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys

import numpy as np

MAGIC = 0x57535356  # 'VSSW'
VERSION = 1
NONE = 0xFFFFFFFF
KIND = {"stem": 1, "ir": 2, "dec": 3, "head": 4}
F_EXPAND, F_RESIDUAL = 1, 2

HERE = os.path.dirname(os.path.abspath(__file__))
SPEC_PATH = os.path.join(HERE, "spec.json")
DEFAULT_BLOB = os.path.join(HERE, "vss_weights_seed7.bin")


def load_spec(path: str = SPEC_PATH) -> dict:
    with open(path) as f:
        return json.load(f)


def generate(spec: dict, seed: int | None = None):
    """Return (layer_records, data f32 array, eps). Deterministic in `seed`."""
    seed = spec["weights"]["seed"] if seed is None else seed
    eps = float(spec["weights"]["norm_eps"])
    rng = np.random.Generator(np.random.PCG64(seed))
    names = [l["name"] for l in spec["layers"]]
    chunks: list[np.ndarray] = []
    n_floats = 0

    def put(a: np.ndarray) -> int:
        nonlocal n_floats
        a = np.ascontiguousarray(a, dtype=np.float32).ravel()
        off = n_floats
        chunks.append(a)
        n_floats += a.size
        return off

    def he(shape, fan_in, gain=2.0):
        return rng.standard_normal(shape) * np.sqrt(gain / fan_in)

    def bias(n, s=0.05):
        return rng.standard_normal(n) * s

    def bf16_exact(a):
        # Pointwise (MFMA) weights are stored bf16-representable so the f32 and
        # the bf16-MFMA paths compute ONE model (like the reference's q4f16 blob
        # ships pre-quantised weights).  RNE on the f32 bit pattern.
        u = np.asarray(a, np.float32).view(np.uint32).astype(np.uint64)
        u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
        return u.astype(np.uint32).view(np.float32)

    records = []
    for l in spec["layers"]:
        kind = l["kind"]
        offs = [NONE] * 8  # w1 b1 wdw bdw w2 b2 gamma beta
        cin, cout = l["cin"], l["cout"]
        chid, stride, flags = 0, 1, 0
        src = names.index(l["src"]) if "src" in l else -1
        skip = names.index(l["skip"]) if "skip" in l else -1
        if kind == "stem":
            stride = l["stride"]
            offs[0] = put(he((cout, cin, 3, 3), cin * 9))
            offs[1] = put(bias(cout, 0.1))
        elif kind == "ir":
            chid, stride = l["chid"], l["stride"]
            if l["expand"]:
                flags |= F_EXPAND
                offs[0] = put(bf16_exact(he((chid, cin), cin)))
                offs[1] = put(bias(chid))
            if l["residual"]:
                flags |= F_RESIDUAL
            offs[2] = put(he((chid, 9), 9))
            offs[3] = put(bias(chid))
            # linear projection: unit-gain init, halved on residual blocks
            offs[4] = put(bf16_exact(he((cout, chid), chid, gain=0.5 if l["residual"] else 1.0)))
            offs[5] = put(bias(cout))
        elif kind == "dec":
            chid = l["cskip"]
            ccat = cin + chid
            offs[2] = put(he((ccat, 9), 9, gain=1.0))
            offs[3] = put(bias(ccat))
            offs[4] = put(bf16_exact(he((cout, ccat), ccat, gain=1.0)))
            offs[5] = put(bias(cout))
            offs[6] = put(1.0 + 0.1 * rng.standard_normal(cout))
            offs[7] = put(0.1 * rng.standard_normal(cout))
        elif kind == "head":
            # Analytic calibration (no forward pass): the head input is
            # relu(instance-normed d3 * gamma + beta) -> per-channel mean
            # E[relu(z)], z ~ N(beta, gamma^2). Aim at logit std ~2 around 0 so the
            # mask is neither saturated nor flat.
            src_l = spec["layers"][src]
            assert src_l["kind"] == "dec"
            w = rng.standard_normal((1, cin)) * 0.9
            offs[4] = put(w)
            # gamma ~ 1, beta ~ 0 for d3 -> E[relu(z)] ~ 1/sqrt(2*pi)
            mean_a = 1.0 / np.sqrt(2.0 * np.pi)
            offs[5] = put(np.array([-float(w.sum()) * mean_a]))
        else:
            raise ValueError(kind)
        records.append([KIND[kind], cin, chid, cout, stride, flags,
                        src & 0xFFFFFFFF, skip & 0xFFFFFFFF] + offs)
    data = np.concatenate(chunks).astype(np.float32)
    return records, data, eps


def pack(records, data, eps) -> bytes:
    eps_bits = struct.unpack("<I", struct.pack("<f", eps))[0]
    out = bytearray(struct.pack("<8I", MAGIC, VERSION, len(records), data.size, eps_bits, 0, 0, 0))
    for r in records:
        out += struct.pack("<16I", *r)
    out += data.astype("<f4").tobytes()
    return bytes(out)


def write_blob(path: str = DEFAULT_BLOB, seed: int | None = None) -> str:
    records, data, eps = generate(load_spec(), seed)
    blob = pack(records, data, eps)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(blob)
    os.replace(tmp, path)
    return hashlib.sha256(blob).hexdigest()


def parse_blob(blob: bytes):
    """Inverse of pack (used by tests and the Python host for metadata)."""
    magic, ver, nl, nf, eps_bits = struct.unpack_from("<5I", blob, 0)
    assert magic == MAGIC and ver == VERSION, "bad weights blob"
    eps = struct.unpack("<f", struct.pack("<I", eps_bits))[0]
    recs = [list(struct.unpack_from("<16I", blob, 32 + 64 * i)) for i in range(nl)]
    data = np.frombuffer(blob, dtype="<f4", count=nf, offset=32 + 64 * nl)
    return recs, data, eps


if __name__ == "__main__":
    p = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_BLOB
    print(p, write_blob(p))
