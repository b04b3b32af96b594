"""ONNX sessions on the GPU (include/vso.h) — the host mirror of
onnxruntime-web's InferenceSession as the reference uses it:

    session = await ort.InferenceSession.create(url, opts)        # model.ts:14, :38, :61
    const outputs = await session.run({ image: tensor })          # frameProcessorTest.ts:406, :478

becomes

    session = InferenceSession(path_or_bytes)                      # vso_create
    outputs = session.run({"image": array})                        # vso_run -> {name: np.ndarray}

Tensors are float32 NCHW numpy arrays.  Fails loudly (VsoError) when the
library or an operator is missing: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import lib as _vss_lib

VSO_OK, VSO_E_INVALID_ARG, VSO_E_HIP, VSO_E_PARSE, VSO_E_UNSUPPORTED, VSO_E_OOM = 0, -1, -2, -3, -4, -5
PRECISIONS = {"f32": 0, "bf16": 1, "f16": 2}  # vso_options.conv_precision


class Options(ctypes.Structure):
    _fields_ = [("conv_precision", ctypes.c_int), ("reserved", ctypes.c_int * 7)]

_bound = False


class VsoError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vso error {code}: {msg}")
        self.code = code


def lib():
    global _bound
    L = _vss_lib()
    if not _bound:
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        I64P = ctypes.POINTER(ctypes.c_int64)
        sig = {
            "vso_create": ([P, S, I64P, I, I, ctypes.POINTER(P)], I),
            "vso_create_ex": ([P, S, I64P, I, I, ctypes.POINTER(Options), ctypes.POINTER(P)], I),
            "vso_options_default": ([ctypes.POINTER(Options)], None),
            "vso_tile_conv_count": ([P], I),
            "vso_ir_block_count": ([P], I),
            "vso_lane_count": ([P], I),
            "vso_destroy": ([P], None),
            "vso_last_error": ([P], ctypes.c_char_p),
            "vso_io_count": ([P, ctypes.POINTER(I), ctypes.POINTER(I)], I),
            "vso_input_name": ([P, I, ctypes.c_char_p, I], I),
            "vso_output_name": ([P, I, ctypes.c_char_p, I], I),
            "vso_input_shape": ([P, I, I64P, I], I),
            "vso_output_shape": ([P, I, I64P, I], I),
            "vso_run": ([P, ctypes.POINTER(P), ctypes.POINTER(P)], I),
            "vso_run_device": ([P, ctypes.POINTER(P), ctypes.POINTER(P), P], I),
            "vso_launch_count": ([P], I),
            "vso_launch_name": ([P, I, ctypes.c_char_p, I], I),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _bound = True
    return L


def _check(rc, handle=None):
    if rc < 0:
        msg = lib().vso_last_error(handle)
        raise VsoError(rc, msg.decode() if msg else "")
    return rc


class InferenceSession:
    """One ONNX model on one GPU with a fixed input shape.  precision: the
    dense convolutions' operands ("f32" exact, "bf16", "f16"; vso_options)."""

    def __init__(self, model, input_shape=None, device_id: int = 0, precision: str = "f32"):
        if isinstance(model, (bytes, bytearray)):
            data = bytes(model)
        else:
            with open(model, "rb") as f:
                data = f.read()
        self._model = data
        dims = None
        nd = 0
        if input_shape is not None:
            nd = len(input_shape)
            dims = (ctypes.c_int64 * nd)(*input_shape)
        if precision not in PRECISIONS:
            raise VsoError(VSO_E_INVALID_ARG, f"precision must be one of {sorted(PRECISIONS)}")
        opts = Options()
        lib().vso_options_default(ctypes.byref(opts))
        opts.conv_precision = PRECISIONS[precision]
        self.precision = precision
        h = ctypes.c_void_p()
        _check(lib().vso_create_ex(data, len(data), dims, nd, device_id, ctypes.byref(opts), ctypes.byref(h)), None)
        self._h = h
        ni, no = ctypes.c_int(), ctypes.c_int()
        _check(lib().vso_io_count(self._h, ctypes.byref(ni), ctypes.byref(no)), self._h)
        self.input_names = [self._name(lib().vso_input_name, i) for i in range(ni.value)]
        self.output_names = [self._name(lib().vso_output_name, i) for i in range(no.value)]
        self.input_shapes = [self._shape(lib().vso_input_shape, i) for i in range(ni.value)]
        self.output_shapes = [self._shape(lib().vso_output_shape, i) for i in range(no.value)]

    def _name(self, fn, i):
        buf = ctypes.create_string_buffer(512)
        _check(fn(self._h, i, buf, 512), self._h)
        return buf.value.decode()

    def _shape(self, fn, i):
        dims = (ctypes.c_int64 * 8)()
        n = _check(fn(self._h, i, dims, 8), self._h)
        return tuple(dims[k] for k in range(n))

    def run(self, feeds: dict, output_names=None) -> dict:
        """session.run(feeds) -> {output name: float32 array} (host memory)."""
        ins = []
        for name, shape in zip(self.input_names, self.input_shapes):
            if name not in feeds:
                raise VsoError(VSO_E_INVALID_ARG, f"missing feed '{name}'")
            a = np.ascontiguousarray(feeds[name], dtype=np.float32)
            if tuple(a.shape) != shape:
                raise VsoError(VSO_E_INVALID_ARG, f"feed '{name}' has shape {a.shape}, session expects {shape}")
            ins.append(a)
        outs = [np.empty(s, np.float32) for s in self.output_shapes]
        pin = (ctypes.c_void_p * len(ins))(*[a.ctypes.data for a in ins])
        pout = (ctypes.c_void_p * len(outs))(*[o.ctypes.data for o in outs])
        _check(lib().vso_run(self._h, pin, pout), self._h)
        res = dict(zip(self.output_names, outs))
        return {k: res[k] for k in (output_names or self.output_names)}

    def run_device(self, in_ptrs, out_ptrs, stream: int = 0):
        """HBM pointers (one per input / output), enqueued on `stream`."""
        pin = (ctypes.c_void_p * len(in_ptrs))(*in_ptrs)
        pout = (ctypes.c_void_p * len(out_ptrs))(*out_ptrs)
        _check(lib().vso_run_device(self._h, pin, pout, stream or None), self._h)

    def launches(self):
        """Kernel names of one run, in launch order (as rocprofv3 names them)."""
        n = _check(lib().vso_launch_count(self._h), self._h)
        return [self._name(lib().vso_launch_name, k) for k in range(n)]

    def tile_convs(self) -> int:
        """Convolutions planned on the LDS-tiled MFMA kernel (k_conv_tile)."""
        return _check(lib().vso_tile_conv_count(self._h), self._h)

    def ir_blocks(self) -> int:
        """Inverted residual blocks planned as one fused launch each (k_ir)."""
        return _check(lib().vso_ir_block_count(self._h), self._h)

    def lanes(self) -> int:
        """Capture lanes of the session's graph (0 before its first run)."""
        return _check(lib().vso_lane_count(self._h), self._h)

    def close(self):
        if getattr(self, "_h", None):
            lib().vso_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
