"""Python host mirror of the segmentation seam over libvss.so (include/vss.h).

Reference seam (/root/reference/client/src/core/frameProcessorTest.ts:78-97):

    frame -> tf.browser.fromPixels -> resizeBilinear -> /255 -> NCHW  (:79-85)
          -> session.run({input})                                      (:91)
          -> squeezeMaskTo2D -> (alphaRaw, maskW, maskH)               (:94-97)

`Session.segment_frame(frame)` returns exactly that triple (mask as a float32
array of maskH*maskW, plus maskW, maskH); `segment_frames` does a batch.  The
TypeScript surface (segmentFrame/segmentFrames) is in ts/ over the same C ABI.

Errors mirror ORT-web's rejecting `session.run`: every failing call raises
VssError carrying the C code and vss_last_error().  There is no CPU fallback:
if libvss.so is missing or no HIP device is present, creating a Session raises.

A Session owns `queue_depth` slots: `submit(frames)` returns a ticket at once
(the host -> device copy, forward and device -> host copy of consecutive
batches overlap) and `wait(ticket)` returns the masks; `Session(device_ids=
[...])` shards every batch over those GPUs and all-gathers the masks over RCCL.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
import weakref

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# VSS_LIBRARY selects another build of the same ABI (e.g. lib/libvss_trace.so
# for tools/trace_phases.py); the default is the in-tree product library.
LIB_PATH = os.environ.get("VSS_LIBRARY") or os.path.join(HERE, "lib", "libvss.so")
DEFAULT_WEIGHTS = os.path.join(HERE, "model", "vss_weights_seed7.bin")
HEADER = os.path.join(os.path.dirname(HERE), "include", "vss.h")

VSS_OK, VSS_E_INVALID_ARG, VSS_E_HIP, VSS_E_RCCL, VSS_E_BUSY, VSS_E_OOM, VSS_E_IO, VSS_E_UNSUPPORTED = (
    0, -1, -2, -3, -4, -5, -6, -7)
DTYPES = {"f32": 0, "bf16x2": 1}
VSS_OPT_USE_GRAPH, VSS_OPT_PROFILE, VSS_OPT_KEEP_STEM, VSS_OPT_ROW_FETCH = 1, 2, 6, 7
VSS_OPT_GRAPH_BUILDS, VSS_OPT_GRAPH_PATCHES, VSS_OPT_COMM_RANKS, VSS_OPT_GATHER_CALLS = 8, 9, 10, 11  # read-only
VSS_OPT_GATHER_FORM = 12  # settable until comm_init_rank
VSS_GATHER_ORDERED, VSS_GATHER_CONCURRENT = 0, 1
GATHER_FORMS = {"ordered": VSS_GATHER_ORDERED, "concurrent": VSS_GATHER_CONCURRENT}
VSS_CREATE_NO_AUTOTUNE = 1
VSS_OUT_MODEL, VSS_OUT_FRAME = 0, 1


class VssError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vss error {code}: {msg}")
        self.code = code


class _Config(ctypes.Structure):
    _fields_ = [("model_h", ctypes.c_int), ("model_w", ctypes.c_int), ("dtype", ctypes.c_int),
                ("device_id", ctypes.c_int), ("max_batch", ctypes.c_int), ("max_frame_h", ctypes.c_int),
                ("max_frame_w", ctypes.c_int), ("weights_path", ctypes.c_char_p), ("flags", ctypes.c_int),
                ("n_gpus", ctypes.c_int), ("device_ids", ctypes.POINTER(ctypes.c_int)), ("queue_depth", ctypes.c_int),
                ("staging_threads", ctypes.c_int)]


class _Info(ctypes.Structure):
    _fields_ = [("mask_h", ctypes.c_int), ("mask_w", ctypes.c_int), ("n_layers", ctypes.c_int),
                ("dtype", ctypes.c_int), ("device_bytes", ctypes.c_size_t), ("n_gpus", ctypes.c_int),
                ("queue_depth", ctypes.c_int), ("rccl", ctypes.c_int)]


class PostConfig(ctypes.Structure):
    """vss_post_config: the reference's post-processing knobs
    (frameProcessorTest.ts:12-18; defaults = defaultConfig :20-28)."""
    _fields_ = [("ema", ctypes.c_double), ("noise_cutoff", ctypes.c_double), ("high_threshold", ctypes.c_double),
                ("gamma", ctypes.c_double), ("sigma_spatial", ctypes.c_double), ("sigma_range", ctypes.c_double),
                ("use_bilateral", ctypes.c_int)]
    # the reference's config keys -> fields
    KEYS = {"EMA": "ema", "NOISE_CUTOFF": "noise_cutoff", "HIGH_THRESHOLD": "high_threshold", "GAMMA": "gamma",
            "BILATERAL_SIGMA_SPATIAL": "sigma_spatial", "BILATERAL_SIGMA_RANGE": "sigma_range",
            "USE_BILATERAL": "use_bilateral"}

    @classmethod
    def default(cls, **overrides):
        c = cls()
        lib().vss_post_config_default(ctypes.byref(c))
        for k, v in overrides.items():
            setattr(c, cls.KEYS.get(k, k), int(v) if cls.KEYS.get(k, k) == "use_bilateral" else float(v))
        return c


CALLBACK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)
_lib = None
_lock = threading.Lock()


def build(force: bool = False) -> str:
    """Compile libvss.so for gfx950 in-tree (hipcc cross-compiles without a GPU).
    Always runs make: its dependency tracking rebuilds exactly what changed, so
    a library built from older sources is never reused."""
    cmd = ["make", "-s", "-j", str(min(8, os.cpu_count() or 1)), "-C", os.path.join(HERE, "csrc")]
    if force:
        cmd.insert(2, "-B")
    subprocess.run(cmd, check=True)
    return LIB_PATH


def ensure_weights(path: str = DEFAULT_WEIGHTS) -> str:
    if not os.path.exists(path):
        import importlib.util
        spec = importlib.util.spec_from_file_location("vss_make_weights", os.path.join(HERE, "model", "make_weights.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        mod.write_blob(path)
    return path


def lib() -> ctypes.CDLL:
    """Load libvss.so; raises (never falls back) when the HIP library is absent."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise VssError(VSS_E_IO, f"libvss.so not built at {LIB_PATH} (run build())")
            L = ctypes.CDLL(LIB_PATH)
            P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
            sig = {
                "vss_version": ([], I),
                "vss_create": ([ctypes.POINTER(_Config), ctypes.POINTER(P)], I),
                "vss_destroy": ([P], None),
                "vss_last_error": ([P], ctypes.c_char_p),
                "vss_get_info": ([P, ctypes.POINTER(_Info)], I),
                "vss_segment": ([P, P, I, I, I, I, S, P, I], I),
                "vss_segment_async": ([P, P, I, I, I, I, S, P, I, CALLBACK, P], I),
                "vss_submit": ([P, P, I, I, I, I, S, P, I, ctypes.POINTER(ctypes.c_uint64)], I),
                "vss_wait": ([P, ctypes.c_uint64], I),
                "vss_query": ([P, ctypes.c_uint64], I),
                "vss_staging_acquire": ([P, ctypes.POINTER(I), ctypes.POINTER(P), ctypes.POINTER(S)], I),
                "vss_staging_release": ([P, I], I),
                "vss_submit_staged": ([P, I, I, I, I, I, S, P, I, CALLBACK, P, ctypes.POINTER(ctypes.c_uint64)], I),
                "vss_submit_list": ([P, ctypes.POINTER(P), I, I, I, I, S, P, I, ctypes.POINTER(ctypes.c_uint64)], I),
                "vss_segment_device": ([P, P, I, I, I, I, S, S, P, P], I),
                "vss_prepare_device": ([P, I, I, I, I, S, S], I),
                "vss_slot_stream": ([P, I, ctypes.POINTER(P)], I),
                "vss_shard_plan": ([I, I, I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)], I),
                "vss_gather_runs": ([I, I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)], I),
                "vss_host_alloc": ([S, ctypes.POINTER(P)], I),
                "vss_host_free": ([P], I),
                "vss_comm_unique_id": ([P, P, S, ctypes.POINTER(S)], I),
                "vss_comm_init_rank": ([P, I, I, P, S], I),
                "vss_segment_gather_device": ([P, P, I, I, I, I, S, S, P, P], I),
                "vss_comm_status": ([P, ctypes.POINTER(I), I, ctypes.POINTER(I), ctypes.POINTER(ctypes.c_uint64)], I),
                "vss_block_lds_bytes": ([I] * 9, I),
                "vss_preprocess_device": ([P, P, I, I, I, I, S, S, P, P], I),
                "vss_mask_to_frame_device": ([P, P, I, I, I, P, P], I),
                "vss_synchronize": ([P], I),
                "vss_set_option": ([P, I, I], I),
                "vss_get_option": ([P, I, ctypes.POINTER(I)], I),
                "vss_layer_shape": ([P, I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I)], I),
                "vss_read_layer": ([P, I, I, P], I),
                "vss_profile_read": ([P, ctypes.POINTER(ctypes.c_double), I, ctypes.POINTER(I)], I),
                "vss_layer_kernel": ([P, I, ctypes.c_char_p, I], I),
                "vss_layer_tiles": ([P, I, ctypes.POINTER(I), ctypes.POINTER(I), I], I),
                "vss_layer_tile_kernel": ([P, I, I, ctypes.c_char_p, I], I),
                "vss_layer_occupancy": ([P, I, ctypes.POINTER(I), ctypes.POINTER(I)], I),
                "vss_post_config_default": ([ctypes.POINTER(PostConfig)], None),
                "vss_post_create": ([P, ctypes.POINTER(PostConfig), ctypes.POINTER(P)], I),
                "vss_post_destroy": ([P], None),
                "vss_post_reset": ([P], I),
                "vss_post_set_config": ([P, ctypes.POINTER(PostConfig)], I),
                "vss_post_set_faces": ([P, P, I], I),
                "vss_post_set_faces_device": ([P, P, I], I),
                "vss_postprocess_device": ([P, P, I, I, I, I, S, S, P, P, P, P], I),
                "vss_segment_post": ([P, P, P, I, I, I, I, S, P, P], I),
                "vss_composite_device": ([P, P, I, I, I, I, S, S, P, P, S, S, P], I),
                "vss_segment_composite": ([P, P, P, I, I, I, I, S, P], I),
            }
            for name, (args, res) in sig.items():
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = res
            _lib = L
        return _lib


def _check(rc: int, handle=None):
    if rc != VSS_OK:
        msg = lib().vss_last_error(handle)
        raise VssError(rc, msg.decode() if msg else "")


def _as_frames(frames: np.ndarray) -> np.ndarray:
    """[H,W,C] or [N,H,W,C] uint8, C in {3,4} (tf.browser.fromPixels input)."""
    a = np.asarray(frames)
    if a.dtype != np.uint8:
        raise VssError(VSS_E_INVALID_ARG, "frames must be uint8")
    if a.ndim == 3:
        a = a[None]
    if a.ndim != 4 or a.shape[3] not in (3, 4):
        raise VssError(VSS_E_INVALID_ARG, "frames must be [N,H,W,3|4]")
    return np.ascontiguousarray(a)


class Session:
    """One GPU, one model resolution: the MI355X stand-in for an ORT
    InferenceSession of the segmentation model (model.ts:12-29)."""

    def __init__(self, model_h: int = 144, model_w: int = 256, dtype: str = "bf16x2", device_id: int = 0,
                 max_batch: int = 8, max_frame_h: int = 1080, max_frame_w: int = 1920,
                 weights_path: str | None = None, autotune: bool = True, device_ids=None, queue_depth: int = 0,
                 staging_threads: int = 0):
        """device_ids: one handle over these GPUs (batches sharded, masks all-gathered over
        RCCL; a list of one GPU still takes the RCCL path); queue_depth: batches in flight."""
        if dtype not in DTYPES:
            raise VssError(VSS_E_INVALID_ARG, f"dtype must be one of {sorted(DTYPES)}")
        self.weights_path = ensure_weights(weights_path or DEFAULT_WEIGHTS)
        ids = None
        if device_ids is not None:
            ids = (ctypes.c_int * max(1, len(device_ids)))(*[int(d) for d in device_ids])
        cfg = _Config(model_h, model_w, DTYPES[dtype], device_id, max_batch, max_frame_h, max_frame_w,
                      self.weights_path.encode(), 0 if autotune else 1,
                      len(device_ids) if device_ids is not None else 0,
                      ctypes.cast(ids, ctypes.POINTER(ctypes.c_int)) if ids is not None else None,
                      queue_depth, staging_threads)
        h = ctypes.c_void_p()
        _check(lib().vss_create(ctypes.byref(cfg), ctypes.byref(h)), None)
        self._h = h
        info = _Info()
        _check(lib().vss_get_info(self._h, ctypes.byref(info)), self._h)
        self.mask_h, self.mask_w, self.n_layers = info.mask_h, info.mask_w, info.n_layers
        self.device_bytes = info.device_bytes
        self.n_gpus, self.queue_depth, self.rccl = info.n_gpus, info.queue_depth, bool(info.rccl)
        self.dtype, self.max_batch = dtype, max_batch
        self._pending = []
        self._tickets = {}
        self._posts = []

    # -- lifecycle --------------------------------------------------------
    def close(self):
        for p in getattr(self, "_posts", []):
            p.close()
        if getattr(self, "_h", None):
            lib().vss_destroy(self._h)
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

    # -- the seam -----------------------------------------------------------
    def segment_frames(self, frames: np.ndarray, output_size: str = "model"):
        """frames [N,H,W,3|4] uint8 -> (masks float32 [N, maskH*maskW], maskW, maskH); with
        output_size="frame" the masks come upsampled on the GPU: ([N, H*W], W, H)."""
        f = _as_frames(frames)
        n, hh, ww, c = f.shape
        if output_size not in ("model", "frame"):
            raise VssError(VSS_E_INVALID_ARG, "output_size must be 'model' or 'frame'")
        frame = output_size == "frame"
        out = np.empty((n, hh * ww if frame else self.mask_h * self.mask_w), np.float32)
        _check(lib().vss_segment(self._h, f.ctypes.data, n, hh, ww, c, ww * c, out.ctypes.data,
                                 VSS_OUT_FRAME if frame else VSS_OUT_MODEL), self._h)
        return (out, ww, hh) if frame else (out, self.mask_w, self.mask_h)

    def segment_frame(self, frame: np.ndarray):
        """One frame -> (alphaRaw float32[maskH*maskW], maskW, maskH)  (frameProcessorTest.ts:95-97)."""
        masks, mw, mh = self.segment_frames(frame)
        return masks[0], mw, mh

    def segment_frames_async(self, frames: np.ndarray, callback):
        """Queued: returns once the frames are staged; callback(masks, maskW, maskH, status)
        fires when done, in submission order.  Raises VssError(VSS_E_BUSY) when queue_depth
        batches are in flight."""
        f = _as_frames(frames)
        n, hh, ww, c = f.shape
        out = np.empty((n, self.mask_h * self.mask_w), np.float32)

        def _done(_user, status, _out=out):
            callback(_out, self.mask_w, self.mask_h, status)

        cb = CALLBACK(_done)
        self._pending.append((cb, out))
        if len(self._pending) > 4 * max(1, self.queue_depth):
            self._pending = self._pending[-2 * max(1, self.queue_depth):]  # callbacks long since fired
        _check(lib().vss_segment_async(self._h, f.ctypes.data, n, hh, ww, c, ww * c, out.ctypes.data,
                                       VSS_OUT_MODEL, cb, None), self._h)
        return out

    def submit(self, frames: np.ndarray, output_size: str = "model", out: np.ndarray | None = None) -> int:
        """Queued host call: returns the batch's ticket once its frames are staged
        (VssError(VSS_E_BUSY) when queue_depth batches are in flight); wait(ticket)
        returns (masks, maskW, maskH).  out: where the masks go (e.g. host_empty()
        memory, which the D2H fills directly); a new array by default."""
        f = _as_frames(frames)
        n, hh, ww, c = f.shape
        frame = output_size == "frame"
        shape = (n, hh * ww if frame else self.mask_h * self.mask_w)
        if out is None:
            out = np.empty(shape, np.float32)
        elif out.dtype != np.float32 or out.size < shape[0] * shape[1] or not out.flags.c_contiguous:
            raise VssError(VSS_E_INVALID_ARG, f"out must be a C-contiguous float32 array of >= {shape} elements")
        t = ctypes.c_uint64()
        _check(lib().vss_submit(self._h, f.ctypes.data, n, hh, ww, c, ww * c, out.ctypes.data,
                                VSS_OUT_FRAME if frame else VSS_OUT_MODEL, ctypes.byref(t)), self._h)
        self._tickets[t.value] = (out, (ww, hh) if frame else (self.mask_w, self.mask_h))
        return t.value

    def wait(self, ticket: int):
        """Block until batch `ticket` is done -> (masks, maskW, maskH)."""
        _check(lib().vss_wait(self._h, ticket), self._h)
        out, (mw, mh) = self._tickets.pop(ticket)
        return out, mw, mh

    def query(self, ticket: int) -> bool:
        rc = lib().vss_query(self._h, ticket)
        if rc < 0:
            _check(rc, self._h)
        return rc == 1

    def staging_acquire(self):
        """Zero-copy input (the decode -> infer loop): reserve a free slot and return
        (slot, its pinned staging buffer as a writable uint8 array); decode frames into
        it, then submit_staged(slot, ...)."""
        k, p, cap = ctypes.c_int(), ctypes.c_void_p(), ctypes.c_size_t()
        _check(lib().vss_staging_acquire(self._h, ctypes.byref(k), ctypes.byref(p), ctypes.byref(cap)), self._h)
        return k.value, np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint8)), shape=(cap.value,))

    def staging_release(self, slot: int):
        _check(lib().vss_staging_release(self._h, slot), self._h)

    def submit_staged(self, slot: int, n: int, h: int, w: int, c: int, out: np.ndarray | None = None,
                      row_stride: int = 0) -> int:
        """Queue the n frames written into `slot`'s staging buffer; wait(ticket) -> masks."""
        if out is None:
            out = np.empty((n, self.mask_h * self.mask_w), np.float32)
        t = ctypes.c_uint64()
        _check(lib().vss_submit_staged(self._h, slot, n, h, w, c, row_stride or w * c, out.ctypes.data,
                                       VSS_OUT_MODEL, CALLBACK(), None, ctypes.byref(t)), self._h)
        self._tickets[t.value] = (out, (self.mask_w, self.mask_h))
        return t.value

    # -- one GPU per process: an RCCL clique over the processes ---------------
    def comm_unique_id(self) -> bytes:
        buf = ctypes.create_string_buffer(4096)
        n = ctypes.c_size_t()
        _check(lib().vss_comm_unique_id(self._h, buf, 4096, ctypes.byref(n)), self._h)
        return buf.raw[:n.value]

    def comm_init_rank(self, nranks: int, rank: int, ids: bytes):
        buf = ctypes.create_string_buffer(ids, len(ids))
        _check(lib().vss_comm_init_rank(self._h, nranks, rank, buf, len(ids)), self._h)

    def comm_status(self) -> dict:
        """{'async_errors': per slot (0 ok, 7 in progress, -1 no communicator,
        else an RCCL error), 'gather_calls': n} — lock-free (vss_comm_status),
        for a watchdog thread."""
        errs = (ctypes.c_int * 64)()
        ns = ctypes.c_int()
        calls = ctypes.c_uint64()
        _check(lib().vss_comm_status(self._h, errs, 64, ctypes.byref(ns), ctypes.byref(calls)), self._h)
        return {"async_errors": list(errs[:min(ns.value, 64)]), "gather_calls": int(calls.value),
                "slots": ns.value}

    def segment_gather_device(self, frames_ptr: int, n: int, h: int, w: int, c: int, row_stride: int,
                              frame_stride: int, gathered_ptr: int, stream: int = 0):
        """This rank's n frames -> every rank's masks [nranks * n][maskH * maskW] (RCCL all-gather)."""
        _check(lib().vss_segment_gather_device(self._h, frames_ptr, n, h, w, c, row_stride, frame_stride,
                                               gathered_ptr, stream or None), self._h)

    # -- device-resident path (bench, multi-GPU host) ----------------------
    def segment_device(self, frames_ptr: int, n: int, h: int, w: int, c: int, row_stride: int, frame_stride: int,
                       masks_ptr: int, stream: int = 0):
        _check(lib().vss_segment_device(self._h, frames_ptr, n, h, w, c, row_stride, frame_stride, masks_ptr,
                                        stream or None), self._h)

    def prepare_device(self, n: int, h: int, w: int, c: int, row_stride: int, frame_stride: int):
        """Build every slot's executable graph for this batch shape now (no launch)."""
        _check(lib().vss_prepare_device(self._h, n, h, w, c, row_stride, frame_stride), self._h)

    def slot_stream(self, k: int) -> int:
        """Slot k's hipStream_t (device call i takes slot i % queue_depth)."""
        p = ctypes.c_void_p()
        _check(lib().vss_slot_stream(self._h, k, ctypes.byref(p)), self._h)
        return p.value

    @property
    def graph_builds(self) -> int:
        """Executable graphs built so far (one per slot and batch shape)."""
        return self.get_option(VSS_OPT_GRAPH_BUILDS)

    @property
    def graph_patches(self) -> int:
        """Replays that patched a graph's buffer pointers (callers rotating buffers)."""
        return self.get_option(VSS_OPT_GRAPH_PATCHES)

    @property
    def gather_form(self) -> str:
        """How segment_gather_device issues its all-gathers: "ordered" (one
        communicator and one gather stream: one total order of collectives per
        rank, the default) or "concurrent" (one communicator per slot)."""
        v = self.get_option(VSS_OPT_GATHER_FORM)
        return next(k for k, f in GATHER_FORMS.items() if f == v)

    @gather_form.setter
    def gather_form(self, form: str):
        self.set_option(VSS_OPT_GATHER_FORM, GATHER_FORMS[form])

    @property
    def comm_ranks(self) -> int:
        """Ranks of the handle's RCCL clique (ncclCommCount), 1 without one."""
        return self.get_option(VSS_OPT_COMM_RANKS)

    def mask_to_frame_device(self, masks_ptr: int, n: int, frame_h: int, frame_w: int, out_ptr: int,
                             stream: int = 0):
        """HBM masks [n][maskH][maskW] -> [n][frame_h][frame_w] (VSS_OUT_FRAME's upsample)."""
        _check(lib().vss_mask_to_frame_device(self._h, masks_ptr, n, frame_h, frame_w, out_ptr, stream or None),
               self._h)

    def preprocess_device(self, frames_ptr: int, n: int, h: int, w: int, c: int, row_stride: int,
                          frame_stride: int, out_ptr: int, stream: int = 0):
        _check(lib().vss_preprocess_device(self._h, frames_ptr, n, h, w, c, row_stride, frame_stride, out_ptr,
                                           stream or None), self._h)

    def synchronize(self):
        _check(lib().vss_synchronize(self._h), self._h)
        self._pending.clear()

    def set_option(self, option: int, value: int):
        _check(lib().vss_set_option(self._h, option, value), self._h)

    def get_option(self, option: int) -> int:
        v = ctypes.c_int()
        _check(lib().vss_get_option(self._h, option, ctypes.byref(v)), self._h)
        return v.value

    # -- introspection -----------------------------------------------------
    def layer_shape(self, layer: int):
        c, h, w = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().vss_layer_shape(self._h, layer, ctypes.byref(c), ctypes.byref(h), ctypes.byref(w)), self._h)
        return c.value, h.value, w.value

    def layer_tiles(self, layer: int):
        """The compiled output tiles (th, tw) of `layer`'s shape ([] for stem / head)."""
        th, tw = (ctypes.c_int * 64)(), (ctypes.c_int * 64)()
        n = lib().vss_layer_tiles(self._h, layer, th, tw, 64)
        if n < 0:
            _check(n, self._h)
        return [(th[k], tw[k]) for k in range(n)]

    def layer_tile_kernel(self, layer: int, idx: int) -> str:
        """The kernel of candidate `idx` of layer_tiles(layer) (pin it with VSS_TILE="layer:#idx")."""
        buf = ctypes.create_string_buffer(256)
        n = lib().vss_layer_tile_kernel(self._h, layer, idx, buf, 256)
        if n < 0:
            _check(n, self._h)
        return buf.value.decode()

    def tile_spec(self) -> str:
        """The VSS_TILE spec ("layer:#idx,...") that pins this handle's kernels."""
        spec = []
        for li in range(self.n_layers):
            want = self.layer_kernel(li)
            for k in range(len(self.layer_tiles(li))):
                if self.layer_tile_kernel(li, k) == want:
                    spec.append(f"{li}:#{k}")
                    break
        return ",".join(spec)

    def layer_occupancy(self, layer: int):
        """(workgroups per CU, LDS bytes per workgroup) of `layer`'s kernel."""
        w, b = ctypes.c_int(), ctypes.c_int()
        _check(lib().vss_layer_occupancy(self._h, layer, ctypes.byref(w), ctypes.byref(b)), self._h)
        return w.value, b.value

    def layer_kernel(self, layer: int) -> str:
        """The kernel running `layer`, named as rocprofv3 reports it."""
        buf = ctypes.create_string_buffer(256)
        rc = lib().vss_layer_kernel(self._h, layer, buf, 256)
        if rc < 0:
            _check(rc, self._h)
        return buf.value.decode()

    def read_layer(self, layer: int, n: int) -> np.ndarray:
        """Layer output of the latest forward as NCHW float32 (oracle layout)."""
        c, h, w = self.layer_shape(layer)
        out = np.empty((n, h, w, c), np.float32)
        _check(lib().vss_read_layer(self._h, layer, n, out.ctypes.data), self._h)
        return out.transpose(0, 3, 1, 2).copy()

    def profile_read(self):
        """(mean ms per layer over profiled forwards, count)."""
        arr = (ctypes.c_double * self.n_layers)()
        cnt = ctypes.c_int()
        _check(lib().vss_profile_read(self._h, arr, self.n_layers, ctypes.byref(cnt)), self._h)
        return list(arr), cnt.value


class FaceFrame(ctypes.Structure):
    """vss_face_frame: one frame's face-stabiliser inputs (processFrame's
    opts.lastAffine and its detection box, frameProcessorTest.ts:99-114, :131-166)."""
    _fields_ = [("has_affine", ctypes.c_int), ("affine", ctypes.c_double * 6), ("has_box", ctypes.c_int),
                ("box", ctypes.c_double * 4), ("video_w", ctypes.c_int), ("video_h", ctypes.c_int)]

    @classmethod
    def make(cls, affine=None, box=None, video_wh=(0, 0)):
        """affine = (a11, a12, tx, a21, a22, ty) or None; box = (x0, y0, x1, y1) video pixels or None."""
        f = cls()
        if affine is not None:
            f.has_affine = 1
            f.affine[:] = [float(v) for v in affine]
        if box is not None:
            f.has_box = 1
            f.box[:] = [float(v) for v in box]
        f.video_w, f.video_h = (int(v) for v in video_wh)
        return f


class PostChain:
    """The reference's per-stream mask post-processing (processFrame
    frameProcessorTest.ts:115-169: temporalEMA -> morphologicalOpening ->
    jointBilateral3x3 -> refineAlphaOnce -> alphaToImageData) on the GPU.

    One PostChain per video stream: it holds that stream's prevAlpha (:47);
    feed it the stream's frames in order.  reset() = the next frame is first."""

    def __init__(self, session: Session, config: PostConfig | None = None, **overrides):
        self.session = session
        self.config = config if config is not None else PostConfig.default(**overrides)
        st = ctypes.c_void_p()
        _check(lib().vss_post_create(session._h, ctypes.byref(self.config), ctypes.byref(st)), session._h)
        self._st = st
        session._posts.append(self)

    def close(self):
        if getattr(self, "_st", None):
            lib().vss_post_destroy(self._st)
            self._st = None

    def reset(self):
        _check(lib().vss_post_reset(self._st), self.session._h)

    def set_config(self, config: PostConfig | None = None, **overrides):
        """Live knob change (the settings sliders, client/script.ts:16-25)."""
        c = config if config is not None else PostConfig.default()
        if config is None:
            for f, _ in PostConfig._fields_:
                setattr(c, f, getattr(self.config, f))
            for k, v in overrides.items():
                f = PostConfig.KEYS.get(k, k)
                setattr(c, f, int(v) if f == "use_bilateral" else float(v))
        _check(lib().vss_post_set_config(self._st, ctypes.byref(c)), self.session._h)
        self.config = c

    def segment(self, frames: np.ndarray):
        """Consecutive frames [N,H,W,3|4] u8 -> (refinedAlpha f32 [N, maskH*maskW],
        alpha bytes u8 [N, maskH*maskW], maskW, maskH)."""
        s = self.session
        f = _as_frames(frames)
        n, hh, ww, c = f.shape
        a = np.empty((n, s.mask_h * s.mask_w), np.float32)
        u = np.empty((n, s.mask_h * s.mask_w), np.uint8)
        _check(lib().vss_segment_post(s._h, self._st, f.ctypes.data, n, hh, ww, c, ww * c, a.ctypes.data,
                                      u.ctypes.data), s._h)
        return a, u, s.mask_w, s.mask_h

    def composite(self, frames: np.ndarray) -> np.ndarray:
        """Consecutive frames [N,H,W,3|4] u8 -> the output canvas after compositing
        (frameProcessorTest.ts:170-178): RGBA u8 [N,H,W,4]."""
        s = self.session
        f = _as_frames(frames)
        n, hh, ww, c = f.shape
        out = np.empty((n, hh, ww, 4), np.uint8)
        _check(lib().vss_segment_composite(s._h, self._st, f.ctypes.data, n, hh, ww, c, ww * c, out.ctypes.data),
               s._h)
        return out

    def set_faces(self, faces):
        """The face inputs (a list of FaceFrame, one per frame) of the NEXT call."""
        arr = (FaceFrame * len(faces))(*faces)
        _check(lib().vss_post_set_faces(self._st, arr, len(faces)), self.session._h)

    def set_faces_device(self, faces_ptr: int, n: int):
        """The same from a device array of n vss_face_frame (e.g. the GPU face stage's output)."""
        _check(lib().vss_post_set_faces_device(self._st, faces_ptr, n), self.session._h)

    def process_device(self, frames_ptr: int, n: int, h: int, w: int, c: int, row_stride: int, frame_stride: int,
                       masks_ptr: int, alpha_ptr: int = 0, alpha_u8_ptr: int = 0, stream: int = 0):
        _check(lib().vss_postprocess_device(self._st, frames_ptr or None, n, h, w, c, row_stride, frame_stride,
                                            masks_ptr, alpha_ptr or None, alpha_u8_ptr or None, stream or None),
               self.session._h)


def composite_device(session: Session, frames_ptr: int, n: int, h: int, w: int, c: int, row_stride: int,
                     frame_stride: int, alpha_u8_ptr: int, out_ptr: int, out_row_stride: int = 0,
                     out_frame_stride: int = 0, stream: int = 0):
    """HBM in/out compositing: frames + mask alpha bytes -> RGBA frames."""
    ors = out_row_stride or w * 4
    _check(lib().vss_composite_device(session._h, frames_ptr, n, h, w, c, row_stride, frame_stride, alpha_u8_ptr,
                                      out_ptr, ors, out_frame_stride or ors * h, stream or None), session._h)


class _PinnedBlock:
    """A vss_host_alloc block, freed with its last numpy view."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        _check(lib().vss_host_alloc(max(16, nbytes), ctypes.byref(p)))
        self.ptr = p.value
        weakref.finalize(self, lib().vss_host_free, ctypes.c_void_p(p.value))


def host_empty(shape, dtype=np.float32) -> np.ndarray:
    """An uninitialised array in pinned host memory (vss_host_alloc): as the masks
    `out` of Session.submit / submit_staged the batch's D2H lands in it directly
    (no copy on the completion path)."""
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    blk = _PinnedBlock(count * dt.itemsize)
    buf = (ctypes.c_uint8 * max(16, count * dt.itemsize)).from_address(blk.ptr)
    buf._block = blk  # the memory lives as long as any view of it
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


def shard_plan(n: int, nranks: int, rank: int):
    """(first, count, per_rank) of `rank`'s contiguous shard of an n-frame batch
    (vss_shard_plan); the gathered [nranks][per_rank] rows hold
    frame i at row i.  Host-only: no GPU needed."""
    f, c, m = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().vss_shard_plan(n, nranks, rank, ctypes.byref(f), ctypes.byref(c), ctypes.byref(m)))
    return f.value, c.value, m.value


def gather_runs(n: int, nranks: int):
    """The multi-GPU copy-out of an n-frame batch (vss_gather_runs): a list of
    (src_row, dst_row, rows) runs moving the all-gathered [nranks][per_rank]
    rows to frame order.  Host-only: no GPU needed."""
    a, b, c = (ctypes.c_int * max(1, nranks))(), (ctypes.c_int * max(1, nranks))(), (ctypes.c_int * max(1, nranks))()
    k = lib().vss_gather_runs(n, nranks, a, b, c)
    _check(min(k, 0))
    return [(a[j], b[j], c[j]) for j in range(k)]


def version() -> int:
    return lib().vss_version()


def block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, stem_in=0) -> int:
    """block_lds() of csrc/vss_kernels.h through the library (no GPU needed)."""
    return lib().vss_block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, stem_in)
