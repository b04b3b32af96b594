"""Synthetic ONNX models for the GPU ONNX sessions (test infrastructure):
built with oracle/onnx_ref.py's writer from seeded weights, so every test
run sees the same bytes.  `modnet_like` follows the public MODNet layout the
reference's absent model_q4f16.onnx is named after:
MobileNetV2 inverted residuals with ReLU6 (Clip), an SE block (GAP ->
Gemm -> Relu -> Gemm -> Sigmoid -> Mul), IBNorm (half the channels
BatchNormalization, half InstanceNormalization: Split / Concat), bilinear
Resize x2 with skip Concat, and a sigmoid matte at input resolution."""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import onnx_ref as R  # noqa: E402


class Builder:
    def __init__(self, seed=0):
        self.rng = np.random.default_rng(seed)
        self.nodes, self.inits, self.k = [], {}, 0

    def name(self, p="t"):
        self.k += 1
        return f"{p}{self.k}"

    def w(self, *shape, scale=None):
        n = self.name("w")
        fan = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        s = scale if scale is not None else (2.0 / max(fan, 1)) ** 0.5
        self.inits[n] = (self.rng.standard_normal(shape) * s).astype(np.float32)
        return n

    def const(self, arr):
        n = self.name("c")
        self.inits[n] = np.asarray(arr)
        return n

    def op(self, op, inputs, n_out=1, **attrs):
        outs = [self.name(op.lower()) for _ in range(n_out)]
        self.nodes.append(R.make_node(op, inputs, outs, **attrs))
        return outs[0] if n_out == 1 else outs

    def conv(self, x, cin, cout, k, stride=1, pads=None, group=1, dil=1, bias=True):
        p = pads if pads is not None else [k // 2 * dil] * 4
        ins = [x, self.w(cout, cin // group, k, k)]
        if bias:
            ins.append(self.w(cout, scale=0.1))
        return self.op("Conv", ins, kernel_shape=[k, k], strides=[stride, stride], pads=p, group=group,
                       dilations=[dil, dil])

    def model(self, inputs, outputs, opset=13):
        return R.make_model(self.nodes, self.inits, inputs, outputs, opset=opset)


def conv_zoo(h=64, w=80):
    """Every convolution shape class the face models and MODNet use, with the
    epilogue fusions (BatchNormalization folding, residual Add, activations).
    At 64x80 the two depthwise -> 1x1 pairs run as k_conv_dwpw and the rest as
    k_conv_small; at 512x512 the stem has >= 1024 64x64 tiles and runs as
    k_conv_gemm (test_gpu_onnx checks the choice)."""
    b = Builder(1)
    x = "x"
    a = b.conv(x, 3, 24, 5, stride=2, pads=[1, 1, 2, 2])                  # MediaPipe stem: 5x5 s2 asym pads
    a = b.op("Relu", [a])
    d = b.conv(a, 24, 24, 3, group=24)                                     # depthwise 3x3
    p = b.conv(d, 24, 24, 1)                                               # 1x1
    r = b.op("Add", [p, a])                                                # residual
    r = b.op("Relu", [r])
    s2 = b.conv(r, 24, 24, 3, stride=2, pads=[0, 0, 2, 2], group=24)       # depthwise s2, pads (0,0,2,2)
    s2 = b.conv(s2, 24, 32, 1)
    sl = b.w(32, 1, 1, scale=0.3)
    s2 = b.op("PRelu", [s2, sl])                                           # per-channel PRelu (landmarks)
    g = b.conv(s2, 32, 32, 3, group=2)                                     # grouped
    bn = b.op("BatchNormalization", [g, b.const(b.rng.random(32).astype(np.float32) + 0.5),
                                     b.const(b.rng.standard_normal(32).astype(np.float32) * 0.1),
                                     b.const(b.rng.standard_normal(32).astype(np.float32) * 0.1),
                                     b.const(b.rng.random(32).astype(np.float32) + 0.5)], epsilon=1e-5)
    c6 = b.op("Clip", [bn, b.const(np.array(0, np.float32)), b.const(np.array(6, np.float32))])
    dl = b.conv(c6, 32, 40, 3, dil=2)                                      # dilated
    dl = b.op("LeakyRelu", [dl], alpha=0.1)
    v = b.conv(dl, 40, 16, 3, pads=[0, 0, 0, 0], bias=False)               # valid padding, no bias
    nb = b.w(16, 40 // 1, 1, 1)
    v2 = b.op("Conv", [dl, nb], kernel_shape=[1, 1], auto_pad="SAME_UPPER", strides=[2, 2])
    h2, w2 = (h // 2 - 1) // 2 + 1, (w // 2 - 1) // 2 + 1
    return b.model([("x", [1, 3, h, w])], [(v, [1, 16, h2 - 2, w2 - 2]), (v2, [1, 16, (h2 + 1) // 2, (w2 + 1) // 2])])


def ops_zoo():
    """The non-convolution operators, incl. the shape arithmetic exporters emit."""
    b = Builder(2)
    x = "x"                                                                # [2, 8, 12, 16]
    mp = b.op("MaxPool", [x], kernel_shape=[2, 2], strides=[2, 2])
    ap = b.op("AveragePool", [x], kernel_shape=[3, 3], strides=[2, 2], pads=[1, 1, 1, 1], count_include_pad=0)
    cat = b.op("Concat", [mp, ap], axis=1)                                  # [2, 16, 6, 8]
    pad = b.op("Pad", [cat, b.const(np.array([0, 0, 1, 0, 0, 4, 0, 2], np.int64)), b.const(np.array(0.5, np.float32))],
               mode="constant")                                             # channel + spatial pad [2, 20, 7, 10]
    sp = b.op("Split", [pad, b.const(np.array([5, 15], np.int64))], n_out=2, axis=1)
    sm = b.op("Sigmoid", [sp[0]])
    th = b.op("Tanh", [sp[1]])
    mul = b.op("Mul", [th, b.const(b.rng.standard_normal((15, 1, 1)).astype(np.float32))])
    sub = b.op("Sub", [mul, b.const(np.array(0.25, np.float32))])
    div = b.op("Div", [sm, b.const(np.array(192.0, np.float32))])
    cat2 = b.op("Concat", [div, sub], axis=1)                               # [2, 20, 7, 10]
    sl = b.op("Slice", [cat2, b.const(np.array([1, 0], np.int64)), b.const(np.array([7, 10], np.int64)),
                        b.const(np.array([2, 3], np.int64)), b.const(np.array([2, 3], np.int64))])  # [2, 20, 3, 4]
    tr = b.op("Transpose", [sl], perm=[0, 2, 3, 1])                         # NHWC like the face heads
    # shape arithmetic: reshape to [N, -1, 4] via Shape -> Gather -> Unsqueeze -> Concat
    shp = b.op("Shape", [tr])
    n0 = b.op("Gather", [shp, b.const(np.array(0, np.int64))], axis=0)
    n0 = b.op("Unsqueeze", [n0, b.const(np.array([0], np.int64))])
    tgt = b.op("Concat", [n0, b.const(np.array([-1, 4], np.int64))], axis=0)
    rs = b.op("Reshape", [tr, tgt])                                         # [2, 60, 4]
    smx = b.op("Softmax", [rs], axis=-1)
    up = b.op("Resize", [x, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
              coordinate_transformation_mode="half_pixel")                  # [2, 8, 24, 32]
    upn = b.op("Resize", [x, "", "", b.const(np.array([2, 8, 18, 24], np.int64))], mode="nearest",
               coordinate_transformation_mode="asymmetric", nearest_mode="floor")
    upa = b.op("Resize", [x, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
               coordinate_transformation_mode="align_corners")
    # rows of a width that is not a multiple of 4: k_resize's one-output-per-thread form
    upo = b.op("Resize", [x, "", "", b.const(np.array([2, 8, 15, 21], np.int64))], mode="linear",
               coordinate_transformation_mode="pytorch_half_pixel")
    upc = b.op("Resize", [x, "", "", b.const(np.array([2, 8, 7, 10], np.int64))], mode="nearest",
               coordinate_transformation_mode="half_pixel", nearest_mode="round_prefer_ceil")
    inn = b.op("InstanceNormalization", [up, b.const(b.rng.random(8).astype(np.float32) + 0.5),
                                         b.const(b.rng.standard_normal(8).astype(np.float32))], epsilon=1e-5)
    gap = b.op("GlobalAveragePool", [x])                                    # [2, 8, 1, 1]
    fl = b.op("Flatten", [gap], axis=1)                                     # [2, 8]
    gm = b.op("Gemm", [fl, b.w(12, 8), b.w(12, scale=0.1)], transB=1)      # [2, 12]
    mm = b.op("MatMul", [gm, b.w(12, 5)])                                   # [2, 5]
    sq = b.op("Unsqueeze", [mm, b.const(np.array([1], np.int64))])          # [2, 1, 5]
    sq = b.op("Squeeze", [sq, b.const(np.array([1], np.int64))])            # [2, 5]
    return b.model([("x", [2, 8, 12, 16])],
                   [(smx, [2, 60, 4]), (inn, [2, 8, 24, 32]), (upn, [2, 8, 18, 24]), (upa, [2, 8, 24, 32]),
                    (sq, [2, 5]), (upo, [2, 8, 15, 21]), (upc, [2, 8, 7, 10])])


def modnet_like(h=64, w=96):
    """A small MODNet-shaped matting net (see module docstring)."""
    b = Builder(3)
    x = "input"
    s = b.op("Clip", [b.conv(x, 3, 16, 3, stride=2), b.const(np.array(0, np.float32)), b.const(np.array(6, np.float32))])

    def ir(t, cin, cout, stride, e=4):
        hdn = b.op("Clip", [b.conv(t, cin, cin * e, 1), b.const(np.array(0, np.float32)),
                            b.const(np.array(6, np.float32))])
        d = b.op("Clip", [b.conv(hdn, cin * e, cin * e, 3, stride=stride, group=cin * e),
                          b.const(np.array(0, np.float32)), b.const(np.array(6, np.float32))])
        o = b.conv(d, cin * e, cout, 1)
        return b.op("Add", [o, t]) if stride == 1 and cin == cout else o

    e1 = ir(s, 16, 16, 1)          # /2
    e2 = ir(e1, 16, 24, 2)         # /4
    e3 = ir(e2, 24, 24, 1)
    e4 = ir(e3, 24, 32, 2)         # /8
    # SE block
    gp = b.op("GlobalAveragePool", [e4])
    f = b.op("Flatten", [gp])
    f = b.op("Relu", [b.op("Gemm", [f, b.w(8, 32), b.w(8, scale=0.1)], transB=1)])
    f = b.op("Sigmoid", [b.op("Gemm", [f, b.w(32, 8), b.w(32, scale=0.1)], transB=1)])
    f = b.op("Reshape", [f, b.const(np.array([1, 32, 1, 1], np.int64))])
    se = b.op("Mul", [e4, f])
    # IBNorm: half BatchNorm, half InstanceNorm
    c = b.conv(se, 32, 32, 3)
    parts = b.op("Split", [c, b.const(np.array([16, 16], np.int64))], n_out=2, axis=1)
    bn = b.op("BatchNormalization", [parts[0], b.const(b.rng.random(16).astype(np.float32) + 0.5),
                                     b.const(b.rng.standard_normal(16).astype(np.float32) * 0.1),
                                     b.const(b.rng.standard_normal(16).astype(np.float32) * 0.1),
                                     b.const(b.rng.random(16).astype(np.float32) + 0.5)])
    inn = b.op("InstanceNormalization", [parts[1], b.const(np.ones(16, np.float32)), b.const(np.zeros(16, np.float32))])
    ib = b.op("Relu", [b.op("Concat", [bn, inn], axis=1)])
    # decoder
    u = b.op("Resize", [ib, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
             coordinate_transformation_mode="half_pixel")                  # /4
    u = b.op("Relu", [b.conv(b.op("Concat", [u, e3], axis=1), 56, 24, 3)])
    u = b.op("Resize", [u, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
             coordinate_transformation_mode="half_pixel")                  # /2
    u = b.op("Relu", [b.conv(b.op("Concat", [u, e1], axis=1), 40, 16, 3)])
    u = b.op("Resize", [u, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
             coordinate_transformation_mode="half_pixel")                  # /1
    m = b.op("Sigmoid", [b.conv(u, 16, 1, 3)])
    return b.model([(x, [1, 3, h, w])], [(m, [1, 1, h, w])])


def q4f16_like(h=64, w=96):
    """A MODNet-shaped net in the form of a q4f16 export (the reference's
    absent model_q4f16.onnx, model.ts:13): float32 input Cast to float16,
    float16 weights and biases, a convolution whose weights are int4 blocks
    behind DequantizeLinear (opset 21, block_size along the input channels),
    the SE block's fully connected layers as com.microsoft MatMulNBits (4-bit
    blocks with packed zero points, a partial last block, a bias), and a
    float32 Cast of the matte."""
    b = Builder(4)
    rng = b.rng
    x = "input"

    def w16(*shape, scale=None):
        n = b.w(*shape, scale=scale)
        b.inits[n] = b.inits[n].astype(np.float16)
        return n

    def conv16(t, cin, cout, k, stride=1, group=1, wname=None):
        ins = [t, wname or w16(cout, cin // group, k, k), w16(cout, scale=0.1)]
        return b.op("Conv", ins, kernel_shape=[k, k], strides=[stride, stride], pads=[k // 2] * 4, group=group)

    def relu6(t):
        return b.op("Clip", [t, b.const(np.array(0, np.float16)), b.const(np.array(6, np.float16))])

    def nbits(t, K, N, bs, bias):
        kb = -(-K // bs)
        n = b.name("q")
        b.inits[n] = rng.integers(0, 256, (N, kb, bs // 2), dtype=np.uint8)
        sc = b.const((rng.random(N * kb) * 0.1 + 0.02).astype(np.float16))
        zp = b.const(rng.integers(0, 256, (N * (-(-kb // 2)),), dtype=np.uint8))
        ins = [t, n, sc, zp] + (["", b.const((rng.standard_normal(N) * 0.1).astype(np.float16))] if bias else [])
        return b.op("MatMulNBits", ins, domain="com.microsoft", K=K, N=N, bits=4, block_size=bs)

    h16 = b.op("Cast", [x], to=R.DT_FLOAT16)
    s = relu6(conv16(h16, 3, 16, 3, stride=2))                               # /2
    qn = b.name("qw")
    b.inits[qn] = R.Packed4(rng.integers(-8, 8, (24, 16, 3, 3)), signed=True)
    dq = b.op("DequantizeLinear", [qn, b.const((rng.random((24, 2, 3, 3)) * 0.05 + 0.01).astype(np.float16))],
              axis=1, block_size=8)
    e = relu6(conv16(s, 16, 24, 3, stride=2, wname=dq))                      # /4
    e = relu6(conv16(e, 24, 24, 3, group=24))
    gp = b.op("Flatten", [b.op("GlobalAveragePool", [e])])                   # [1, 24]
    f = b.op("Relu", [nbits(gp, 24, 8, 16, bias=False)])                     # K 24 = 16 + partial 8
    f = b.op("Sigmoid", [nbits(f, 8, 24, 16, bias=True)])                    # one partial block
    f = b.op("Reshape", [f, b.const(np.array([1, 24, 1, 1], np.int64))])
    e = b.op("Mul", [e, f])
    u = b.op("Resize", [e, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
             coordinate_transformation_mode="half_pixel")                    # /2
    u = b.op("Relu", [conv16(b.op("Concat", [u, s], axis=1), 40, 16, 3)])
    u = b.op("Resize", [u, "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
             coordinate_transformation_mode="half_pixel")                    # /1
    m = b.op("Cast", [b.op("Sigmoid", [conv16(u, 16, 1, 3)])], to=R.DT_FLOAT)
    return b.model([(x, [1, 3, h, w])], [(m, [1, 1, h, w])], opset=21)


def modnet(h=288, w=512, hr=32, q4f16=False, seed=7, in_eps=1e-5, taps=None, export=()):
    """The public MODNet topology (Ke et al., "MODNet: Real-Time Trimap-Free
    Portrait Matting via Objective Decomposition", AAAI 2022; the authors'
    src/models/modnet.py) at inference, the graph an ONNX export of the
    reference's model_q4f16.onnx holds (model.ts:12-29, run at 288x512 by
    frameProcessorTest.ts:91), with seeded weights (the real ones are absent):
      backbone  MobileNetV2 1.0 (stem 3x3 s2 32, inverted residuals
                t,c,n,s = 1,16,1,1 / 6,24,2,2 / 6,32,3,2 / 6,64,4,2 / 6,96,3,1 /
                6,160,3,2 / 6,320,1,1, 1x1 320 -> 1280; ReLU6 as Clip; BN folded
                into the conv as the exporter does); enc2x 16ch, enc4x 24ch,
                enc32x 1280ch
      LR        SE block on enc32x (GAP -> MatMul 1280x320 -> Relu -> MatMul
                320x1280 -> Sigmoid -> Mul), x2 bilinear -> Conv-IBNorm-Relu 5x5
                1280 -> 96, x2 -> 5x5 96 -> 32 (lr8x)
      HR        img/2, img/4 (bilinear); 1x1 16 -> hr on enc2x, 3x3 s2 (hr+3) ->
                hr; 1x1 24 -> hr on enc4x, 3x3 2hr -> 2hr; lr8x x2; 3x3 (3hr+3)
                -> 2hr -> 2hr -> hr; x2; 3x3 2hr -> 2hr -> hr -> hr -> hr (hr2x)
      fusion    lr8x x2 -> 5x5 32 -> hr; x2; 3x3 2hr -> hr; x2; 3x3 (hr+3) ->
                hr/2; 1x1 hr/2 -> 1; Sigmoid (the matte)
    IBNorm = Slice -> BatchNormalization (first half) / InstanceNormalization
    (second half, affine=False) -> Concat.  q4f16=True gives the export's form:
    float16 weights, the input Cast to FLOAT16 and the matte back to FLOAT, the
    SE's two MatMuls as com.microsoft MatMulNBits (4-bit, block 32).
    taps: a dict filled with {stage name: value name} (enc2x .. fu); export:
    [(value name, shape)] made graph outputs too (a per-stage diagnostic,
    tools/modnet_taps.py)."""
    b = Builder(seed)
    rng = b.rng
    x = "input"
    dt = np.float16 if q4f16 else np.float32

    def cst(v):
        return b.const(np.array(v, dt))

    def wt(*shape, scale=None):
        n = b.w(*shape, scale=scale)
        b.inits[n] = b.inits[n].astype(dt)
        return n

    def conv(t, cin, cout, k, stride=1, group=1):
        ins = [t, wt(cout, cin // group, k, k), wt(cout, scale=0.1)]
        return b.op("Conv", ins, kernel_shape=[k, k], strides=[stride, stride], pads=[k // 2] * 4, group=group)

    def relu6(t):
        return b.op("Clip", [t, cst(0), cst(6)])

    def ir(t, cin, cout, stride, e):
        hd = cin * e
        u = relu6(conv(t, cin, hd, 1)) if e != 1 else t
        u = relu6(conv(u, hd, hd, 3, stride=stride, group=hd))
        o = conv(u, hd, cout, 1)
        return b.op("Add", [o, t]) if stride == 1 and cin == cout else o

    def ibn_relu(t, cin, cout, k, stride=1):
        c = conv(t, cin, cout, k, stride)
        nb = cout // 2
        lo = b.op("Slice", [c, b.const(np.array([0], np.int64)), b.const(np.array([nb], np.int64)),
                            b.const(np.array([1], np.int64))])
        hi = b.op("Slice", [c, b.const(np.array([nb], np.int64)), b.const(np.array([cout], np.int64)),
                            b.const(np.array([1], np.int64))])
        bn = b.op("BatchNormalization", [lo, b.const((rng.random(nb) + 0.5).astype(dt)),
                                         b.const((rng.standard_normal(nb) * 0.1).astype(dt)),
                                         b.const((rng.standard_normal(nb) * 0.1).astype(dt)),
                                         b.const((rng.random(nb) + 0.5).astype(dt))], epsilon=1e-5)
        inn = b.op("InstanceNormalization", [hi, b.const(np.ones(cout - nb, dt)), b.const(np.zeros(cout - nb, dt))],
                   epsilon=in_eps)
        return b.op("Relu", [b.op("Concat", [bn, inn], axis=1)])

    def resize(t, s):
        return b.op("Resize", [t, "", b.const(np.array([1, 1, s, s], np.float32))], mode="linear",
                    coordinate_transformation_mode="pytorch_half_pixel")

    def matmul(t, K, N):
        if not q4f16:
            return b.op("MatMul", [t, b.w(K, N, scale=(2.0 / K) ** 0.5)])
        bs = 32
        kb = -(-K // bs)
        n = b.name("q")
        b.inits[n] = rng.integers(0, 256, (N, kb, bs // 2), dtype=np.uint8)
        sc = b.const((rng.random(N * kb) * (0.4 / K ** 0.5) + 0.01 / K ** 0.5).astype(np.float16))
        zp = b.const(np.full((N * (-(-kb // 2)),), 0x88, np.uint8))
        return b.op("MatMulNBits", [t, n, sc, zp], domain="com.microsoft", K=K, N=N, bits=4, block_size=bs)

    img = b.op("Cast", [x], to=R.DT_FLOAT16) if q4f16 else x
    # MobileNetV2 backbone
    t = relu6(conv(img, 3, 32, 3, stride=2))
    cin, enc = 32, {}
    for i, (e, c, n, s) in enumerate(((1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1),
                                      (6, 160, 3, 2), (6, 320, 1, 1))):
        for j in range(n):
            t = ir(t, cin, c, s if j == 0 else 1, e)
            cin = c
        enc[i] = t
    enc2x, enc4x = enc[0], enc[1]
    enc32x = relu6(conv(t, 320, 1280, 1))
    tap = taps if taps is not None else {}
    tap.update({"enc2x": enc2x, "enc4x": enc4x, "enc8x": enc[2], "enc16x": enc[4], "enc32x": enc32x})
    # LR branch
    gp = b.op("Flatten", [b.op("GlobalAveragePool", [enc32x])])
    f = b.op("Relu", [matmul(gp, 1280, 320)])
    f = b.op("Sigmoid", [matmul(f, 320, 1280)])
    f = b.op("Reshape", [f, b.const(np.array([-1, 1280, 1, 1], np.int64))])
    lr = b.op("Mul", [enc32x, f])
    lr16x = ibn_relu(resize(lr, 2), 1280, 96, 5)
    lr8x = ibn_relu(resize(lr16x, 2), 96, 32, 5)
    tap.update({"se": lr, "lr16x": lr16x, "lr8x": lr8x})
    # HR branch
    img2x, img4x = resize(img, 0.5), resize(img, 0.25)
    e2 = ibn_relu(enc2x, 16, hr, 1)
    hr4x = ibn_relu(b.op("Concat", [img2x, e2], axis=1), hr + 3, hr, 3, stride=2)
    e4 = ibn_relu(enc4x, 24, hr, 1)
    hr4x = ibn_relu(b.op("Concat", [hr4x, e4], axis=1), 2 * hr, 2 * hr, 3)
    lr4x = resize(lr8x, 2)
    u = ibn_relu(b.op("Concat", [hr4x, lr4x, img4x], axis=1), 3 * hr + 3, 2 * hr, 3)
    u = ibn_relu(u, 2 * hr, 2 * hr, 3)
    hr4x = ibn_relu(u, 2 * hr, hr, 3)
    u = b.op("Concat", [resize(hr4x, 2), e2], axis=1)
    u = ibn_relu(u, 2 * hr, 2 * hr, 3)
    u = ibn_relu(u, 2 * hr, hr, 3)
    u = ibn_relu(u, hr, hr, 3)
    hr2x = ibn_relu(u, hr, hr, 3)
    tap.update({"e2": e2, "e4": e4, "hr4x": hr4x, "hr2x": hr2x})
    # fusion branch
    l4 = ibn_relu(resize(lr8x, 2), 32, hr, 5)
    f2x = ibn_relu(b.op("Concat", [resize(l4, 2), hr2x], axis=1), 2 * hr, hr, 3)
    fu = ibn_relu(b.op("Concat", [resize(f2x, 2), img], axis=1), hr + 3, hr // 2, 3)
    m = b.op("Sigmoid", [conv(fu, hr // 2, 1, 1)])
    tap.update({"l4": l4, "f2x": f2x, "fu": fu})
    if q4f16:
        m = b.op("Cast", [m], to=R.DT_FLOAT)
    return b.model([(x, [1, 3, h, w])], [(m, [1, 1, h, w])] + list(export), opset=21 if q4f16 else 13)


def conv_tiles():
    """Every k_conv_tile form (vso_conv.hip) on odd-sized batch-2 inputs, each
    convolution reading a graph input so 16-bit operand rounding is the
    oracle's exactly: a 1x1 (k_conv_small), 3x3 (M 16 / 70: one and two channel tiles), 5x5,
    3x3 stride 2, channel counts off the 32-channel chunk (40), a K split over
    workgroups (x2: 200 channels at 9x16, 5x5) with a residual Add and Relu in
    the reduction's epilogue, and Clip / Sigmoid epilogues."""
    b = Builder(8)
    x, x2 = "x", "x2"
    c1 = b.op("Relu", [b.conv(x, 40, 24, 1)])
    c3 = b.conv(x, 40, 16, 3)
    c3b = b.op("Clip", [b.conv(x, 40, 70, 3), b.const(np.array(-0.5, np.float32)), b.const(np.array(0.5, np.float32))])
    c5 = b.op("Sigmoid", [b.conv(x, 40, 32, 5)])
    s2 = b.conv(x, 40, 24, 3, stride=2)
    k1 = b.conv(x2, 200, 48, 5)
    k2 = b.conv(x2, 200, 48, 3)
    ks = b.op("Relu", [b.op("Add", [k1, k2])])
    return b.model([(x, [2, 40, 37, 70]), (x2, [2, 200, 9, 16])],
                   [(c1, [2, 24, 37, 70]), (c3, [2, 16, 37, 70]), (c3b, [2, 70, 37, 70]), (c5, [2, 32, 37, 70]),
                    (s2, [2, 24, 19, 35]), (ks, [2, 48, 9, 16])])


def norm_planes():
    """InstanceNormalization on every k_norm_plane form (vso_kernels.hip) and
    past it: planes of 2590 (scalar loads, 256 threads x 16), 9216 (float4,
    256 x 48), 36750 (scalar, 1024 x 36) and 40000 elements (the statistics +
    apply pair), with and without a following Relu (fused)."""
    b = Builder(13)
    outs = []
    for name, shape, relu in (("a", [2, 3, 37, 70], False), ("b", [2, 4, 72, 128], True),
                              ("c", [1, 2, 150, 245], True), ("d", [1, 2, 200, 200], False)):
        C = shape[1]
        y = b.op("InstanceNormalization", [name, b.const(b.rng.random(C).astype(np.float32) + 0.5),
                                           b.const(b.rng.standard_normal(C).astype(np.float32))], epsilon=1e-5)
        if relu:
            y = b.op("Relu", [y])
        outs.append((y, shape))
    return b.model([("a", [2, 3, 37, 70]), ("b", [2, 4, 72, 128]), ("c", [1, 2, 150, 245]), ("d", [1, 2, 200, 200])],
                   outs)


def se_forms():
    """The SE chain's kernel forms (vso_kernels.hip): GlobalAveragePool on
    short planes (k_gap_wave: 24 and 35 elements) and a long one (k_gap:
    1600), Gemm + Relu / Sigmoid / LeakyRelu in the GEMM epilogue, Gemm +
    PRelu left as its own launch, and the channel gate Mul on the float4
    per-plane form (inner 24) and the general broadcast (inner 35)."""
    b = Builder(21)
    outs = []
    for name, shape in (("a", [2, 6, 4, 6]), ("c", [2, 6, 5, 7])):
        C = shape[1]
        gp = b.op("Flatten", [b.op("GlobalAveragePool", [name])])
        f = b.op("Relu", [b.op("Gemm", [gp, b.w(4, C), b.w(4, scale=0.1)], transB=1)])
        f = b.op("Sigmoid", [b.op("Gemm", [f, b.w(C, 4), b.w(C, scale=0.1)], transB=1)])
        f = b.op("Reshape", [f, b.const(np.array([shape[0], C, 1, 1], np.int64))])
        outs.append((b.op("Mul", [name, f]), shape))
    gl = b.op("Flatten", [b.op("GlobalAveragePool", ["l"])])
    outs.append((b.op("LeakyRelu", [b.op("Gemm", [gl, b.w(5, 3), b.w(5, scale=0.1)], transB=1)], alpha=0.2), [2, 5]))
    outs.append((b.op("PRelu", [b.op("Gemm", [gl, b.w(5, 3)], transB=1),
                                b.const((b.rng.random(5) * 0.3).astype(np.float32))]), [2, 5]))
    return b.model([("a", [2, 6, 4, 6]), ("c", [2, 6, 5, 7]), ("l", [2, 3, 40, 40])], outs)


def conv_thin():
    """1x1 heads of <= 4 outputs on k_conv_thin (vso_kernels.h): 3 outputs
    with a Sigmoid on a 37x70 plane (scalar pixel path), 4 outputs with a
    fused residual Add on 36x64 (float4 path), 2 outputs plain."""
    b = Builder(15)
    h1 = b.op("Sigmoid", [b.conv("x", 24, 3, 1)])
    h2 = b.op("Add", [b.conv("x2", 16, 4, 1), "r"])
    h3 = b.conv("x2", 16, 2, 1)
    return b.model([("x", [2, 24, 37, 70]), ("x2", [2, 16, 36, 64]), ("r", [2, 4, 36, 64])],
                   [(h1, [2, 3, 37, 70]), (h2, [2, 4, 36, 64]), (h3, [2, 2, 36, 64])])


def conv_up():
    """The 2x linear Resize computed inside its consumer convolution
    (k_conv_tile_up, vso_conv.hip; 16-bit operands): through a Concat with a
    skip input (half_pixel, 3x3, 24 output channels), straight into a 5x5
    (pytorch_half_pixel by sizes, 16 output channels), and one it must not
    take (a 3x3 of 70 output channels: two channel tiles, the Resize keeps its
    launch).  Odd low-resolution sizes put the edge clamps inside tiles."""
    b = Builder(9)
    up = b.op("Resize", ["lo", "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
              coordinate_transformation_mode="half_pixel")                  # [2, 64, 18, 34]
    cat = b.op("Concat", [up, "skip"], axis=1)                              # [2, 69, 18, 34]
    a = b.op("Relu", [b.conv(cat, 69, 24, 3)])
    up2 = b.op("Resize", ["lo2", "", "", b.const(np.array([2, 32, 22, 26], np.int64))], mode="linear",
               coordinate_transformation_mode="pytorch_half_pixel")
    c = b.conv(up2, 32, 16, 5)
    up3 = b.op("Resize", ["lo2", "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
               coordinate_transformation_mode="half_pixel")
    d = b.conv(up3, 32, 70, 3)
    return b.model([("lo", [2, 64, 9, 17]), ("skip", [2, 5, 18, 34]), ("lo2", [2, 32, 11, 13])],
                   [(a, [2, 24, 18, 34]), (c, [2, 16, 22, 26]), (d, [2, 70, 22, 26])])


def ir_chain():
    """MobileNetV2 inverted residuals (1x1 expand -> Clip -> 3x3 depthwise ->
    Clip -> 1x1 project [+ input]) of every k_ir form (vso_ir.hip): stride 1
    with the residual, stride 2, widening stride-1 blocks, on an odd-sized
    batch-2 input (edge tiles, a partial last tile row) whose deep blocks have
    few tiles, so the hidden channels split over workgroups (ks > 1) — and a
    block whose project output is also a graph output (still fused: the Add's
    input is kept)."""
    b = Builder(13)
    one = lambda: b.const(np.array(0, np.float32))
    six = lambda: b.const(np.array(6, np.float32))

    def ir(t, cin, cout, stride, e=6):
        hd = cin * e
        u = b.op("Clip", [b.conv(t, cin, hd, 1), one(), six()])
        u = b.op("Clip", [b.conv(u, hd, hd, 3, stride=stride, group=hd), one(), six()])
        o = b.conv(u, hd, cout, 1)
        return b.op("Add", [o, t]) if stride == 1 and cin == cout else o

    t = ir("x", 16, 24, 2)          # 38x67 -> 19x34
    t = ir(t, 24, 24, 1)
    t = ir(t, 24, 32, 2)            # -> 10x17
    t = ir(t, 32, 32, 1)
    t = ir(t, 32, 64, 2)            # -> 5x9
    t = ir(t, 64, 64, 1)
    t = ir(t, 64, 96, 1)
    t = ir(t, 96, 96, 1)
    t2 = ir(t, 96, 160, 2)          # -> 3x5
    t3 = ir(t2, 160, 160, 1)
    t4 = ir(t3, 160, 320, 1)
    return b.model([("x", [2, 16, 38, 67])], [(t, [2, 96, 5, 9]), (t4, [2, 320, 3, 5])])


def dw_separable_chain():
    """MobileNetV1-style depthwise-separable blocks with ReLU6 (dw 3x3 -> Clip
    -> 1x1 -> Clip, twice, then a stride-2 pair): the first 1x1's input is a
    depthwise output that the planner leaves to its 1x1 consumer (no launch of
    its own), and the 1x1 -> Clip -> dw -> Clip -> 1x1 after it has the shape of
    an inverted residual, which must not take the fused k_ir form over an input
    nothing wrote."""
    b = Builder(21)
    zero = lambda: b.const(np.array(0, np.float32))
    six = lambda: b.const(np.array(6, np.float32))
    clip = lambda t: b.op("Clip", [t, zero(), six()])
    t = clip(b.conv("x", 32, 32, 3, group=32))
    t = clip(b.conv(t, 32, 64, 1))
    t = clip(b.conv(t, 64, 64, 3, group=64))
    t = clip(b.conv(t, 64, 64, 1))
    t = clip(b.conv(t, 64, 64, 3, stride=2, group=64))
    t = b.conv(t, 64, 48, 1)
    return b.model([("x", [2, 32, 30, 44])], [(t, [2, 48, 15, 22])])


def conv_up_thin():
    """A pending 2x Resize through an in-place Concat into a thin 1x1 head
    (<= 4 outputs, k_conv_thin: computes no upsample itself), so the planner
    must launch the Resize in front of it (the thin path flushed
    only its direct input, and the plan failed with 'Resize ... never
    launched').  32-channel upsampled range, a 3-output Sigmoid head."""
    b = Builder(10)
    up = b.op("Resize", ["lo", "", b.const(np.array([1, 1, 2, 2], np.float32))], mode="linear",
              coordinate_transformation_mode="half_pixel")                  # [2, 32, 18, 34]
    cat = b.op("Concat", [up, "skip"], axis=1)                              # [2, 48, 18, 34]
    h = b.op("Sigmoid", [b.conv(cat, 48, 3, 1)])
    return b.model([("lo", [2, 32, 9, 17]), ("skip", [2, 16, 18, 34])], [(h, [2, 3, 18, 34])])


def face_detector_like(S=256, A=896, score_bias=3.0, seed=5):
    """A stand-in with the I/O of the reference's face detector
    (MediaPipeFaceDetector.onnx: image [1,3,S,S] -> box_coords [1,A,16],
    box_scores [1,A,1]) whose best anchor is a confident, frame-dependent box:
    the image's channel means through a Gemm onto seeded per-anchor boxes.
    Drives the face stage through its has-box path, which the real detector
    does not reach on synthetic frames."""
    b = Builder(seed)
    rng = b.rng
    gp = b.op("Flatten", [b.op("GlobalAveragePool", ["image"])])             # [1, 3]
    cx, cy = rng.uniform(0.3, 0.7, A), rng.uniform(0.3, 0.7, A)
    sw, sh = rng.uniform(0.1, 0.3, A), rng.uniform(0.1, 0.3, A)
    cb = rng.uniform(0, 1, (A, 16))
    cb[:, 0], cb[:, 1], cb[:, 2], cb[:, 3] = cx - sw / 2, cy - sh / 2, cx + sw / 2, cy + sh / 2
    wc = b.const((rng.standard_normal((A * 16, 3)) * 0.05).astype(np.float32))
    co = b.op("Gemm", [gp, wc, b.const(cb.reshape(-1).astype(np.float32))], transB=1)
    sb = rng.standard_normal(A) - 2.0
    sb[A // 2 + 17] = score_bias
    ws = b.const((rng.standard_normal((A, 3)) * 0.2).astype(np.float32))
    sc = b.op("Sigmoid", [b.op("Gemm", [gp, ws, b.const(sb.astype(np.float32))], transB=1)])
    b.nodes.append(R.make_node("Reshape", [co, b.const(np.array([1, A, 16], np.int64))], ["box_coords"]))
    b.nodes.append(R.make_node("Reshape", [sc, b.const(np.array([1, A, 1], np.int64))], ["box_scores"]))
    return b.model([("image", [1, 3, S, S])], [("box_coords", [1, A, 16]), ("box_scores", [1, A, 1])])


def face_landmarks_like(LH=192, LW=192, score_bias=2.0, seed=6):
    """A stand-in with the I/O of the reference's landmark model
    (MediaPipeFaceLandmarkDetector.onnx: image [1,3,LH,LW] -> scores [1],
    landmarks [1,468,3]): seeded points, the five anchors the affine uses
    near their face positions, moved by the ROI's channel means."""
    b = Builder(seed)
    rng = b.rng
    gp = b.op("Flatten", [b.op("GlobalAveragePool", ["image"])])             # [1, 3]
    pts = rng.uniform(0.2, 0.8, (468, 3))
    for i, (x, y) in zip((33, 263, 1, 13, 14), ((0.3, 0.4), (0.7, 0.41), (0.5, 0.56), (0.6, 0.72), (0.41, 0.7))):
        pts[i, :2] = (x, y)
    wl = b.const((rng.standard_normal((1404, 3)) * 0.05).astype(np.float32))
    lm = b.op("Gemm", [gp, wl, b.const(pts.reshape(-1).astype(np.float32))], transB=1)
    ws = b.const((rng.standard_normal((1, 3)) * 0.2).astype(np.float32))
    sc = b.op("Sigmoid", [b.op("Gemm", [gp, ws, b.const(np.array([score_bias], np.float32))], transB=1)])
    b.nodes.append(R.make_node("Reshape", [sc, b.const(np.array([1], np.int64))], ["scores"]))
    b.nodes.append(R.make_node("Reshape", [lm, b.const(np.array([1, 468, 3], np.int64))], ["landmarks"]))
    return b.model([("image", [1, 3, LH, LW])], [("scores", [1]), ("landmarks", [1, 468, 3])])


MODELS = {"conv_zoo": (conv_zoo, {"x": (1, 3, 64, 80)}),
          "conv_zoo_512": (lambda: conv_zoo(512, 512), {"x": (1, 3, 512, 512)}),
          "ops_zoo": (ops_zoo, {"x": (2, 8, 12, 16)}),
          "modnet_like": (modnet_like, {"input": (1, 3, 64, 96)}),
          "q4f16_like": (q4f16_like, {"input": (1, 3, 64, 96)})}


def feeds_for(name, seed=0):
    rng = np.random.default_rng(100 + seed)
    return {k: rng.random(s, dtype=np.float32) for k, s in MODELS[name][1].items()}


def load_golden(path):
    """(model bytes, feeds, expected outputs, meta) of a tests/golden/*.npz
    written by tests/golden/make_onnx_golden.py (the ONNX re-encoded from the
    stored graph with onnx_ref's writer)."""
    import json
    z = np.load(path, allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    nodes = []
    for nd in meta["nodes"]:
        attrs = {}
        for an, av in nd["attrs"].items():
            attrs[an] = z[av["tensor"]] if "tensor" in av else av["value"]
        nodes.append(R.make_node(nd["op"], nd["inputs"], nd["outputs"], **attrs))
    inits = {n: z[f"init_{k}"] for k, n in enumerate(meta["inits"])}
    model = R.make_model(nodes, inits, [(n, d, e) for n, e, d in meta["inputs"]],
                         [(n, [v if isinstance(v, int) else 1 for v in d], e) for n, e, d in meta["outputs"]],
                         opset=meta["opset"])
    feeds = {n: z[f"feed_{k}"] for k, n in enumerate(meta["feeds"])}
    want = {n: z[f"want_{k}"] for k, n in enumerate(meta["expected"])}
    return model, feeds, want, meta
