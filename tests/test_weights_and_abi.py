"""CPU tests: the weights blob, the layer table, and the C-ABI library surface
(loads, exports every symbol include/vss.h declares, validates arguments) —
no compute calls without a GPU."""
import ctypes
import hashlib
import json
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_blob_regenerates_bit_identically(pkg, blob, tmp_path):
    import importlib.util
    spec = importlib.util.spec_from_file_location("mw", os.path.join(pkg.HERE, "model", "make_weights.py"))
    mw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mw)
    p = tmp_path / "w.bin"
    sha = mw.write_blob(str(p))
    assert sha == hashlib.sha256(blob).hexdigest()
    g = np.load(os.path.join(ROOT, "tests", "golden", "vga_2f_144x256.npz"), allow_pickle=False)
    assert sha == str(g["weights_sha256"])
    recs, data, eps = mw.parse_blob(blob)
    spec_json = json.load(open(os.path.join(pkg.HERE, "model", "spec.json")))
    assert len(recs) == len(spec_json["layers"])
    assert abs(eps - 1e-5) < 1e-12
    kinds = {1: "stem", 2: "ir", 3: "dec", 4: "head"}
    for r, l in zip(recs, spec_json["layers"]):
        assert kinds[r[0]] == l["kind"] and r[1] == l["cin"] and r[3] == l["cout"]
        # pointwise (MFMA) weights are bf16-exact: low 16 bits zero
        for oi, cnt in ((0, r[2] * r[1]), (4, r[3] * (r[2] if r[0] == 2 else r[1] + r[2]))):
            if r[0] in (2, 3) and r[8 + oi] != 0xFFFFFFFF and cnt:
                w = data[r[8 + oi]:r[8 + oi] + cnt].view(np.uint32)
                assert not np.any(w & 0xFFFF)


def _declared_symbols():
    syms = set()
    for h in ("vss.h", "vso.h", "vsf.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"\b(vs[sof]_[a-z_]+)\s*\(", src))
    return sorted(syms)


def test_library_exports_header_symbols(pkg):
    pkg.build()
    L = ctypes.CDLL(pkg.LIB_PATH)
    syms = _declared_symbols()
    assert len(syms) >= 14 + 12 + 9
    for s in syms:
        assert hasattr(L, s), f"libvss.so does not export {s}"


def test_version_and_argument_validation(pkg):
    pkg.build()
    assert pkg.version() == 30000
    # invalid configs are rejected before any HIP call
    with pytest.raises(pkg.VssError) as e:
        pkg.Session(model_h=100, model_w=256)
    assert e.value.code == pkg.VSS_E_INVALID_ARG and "multiples of 16" in str(e.value)
    with pytest.raises(pkg.VssError) as e:
        pkg.Session(dtype="f16")
    assert e.value.code == pkg.VSS_E_INVALID_ARG
    with pytest.raises(pkg.VssError):
        pkg.Session(max_batch=0)
    # pinned result blocks: bad arguments and pointers vss_host_alloc did not
    # return are refused from the registry alone (no HIP call)
    import ctypes
    L = pkg.lib()
    p = ctypes.c_void_p()
    assert L.vss_host_alloc(0, ctypes.byref(p)) == pkg.VSS_E_INVALID_ARG
    assert L.vss_host_alloc(64, None) == pkg.VSS_E_INVALID_ARG
    buf = ctypes.create_string_buffer(64)
    assert L.vss_host_free(ctypes.cast(buf, ctypes.c_void_p)) == pkg.VSS_E_INVALID_ARG
    assert L.vss_host_free(None) == pkg.VSS_OK


def test_no_silent_cpu_fallback(pkg):
    # On a host without a GPU the product must fail loudly, never compute on CPU.
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.VssError) as e:
        pkg.Session()
    assert e.value.code == pkg.VSS_E_HIP


def test_product_never_imports_oracle():
    pkg_dir = os.path.join(ROOT, "video-stream-segmenetation_amd")
    for dp, _, fns in os.walk(pkg_dir):
        for fn in fns:
            if fn.endswith((".py", ".hip", ".h", ".cpp", ".cc", ".ts", ".js")):
                txt = open(os.path.join(dp, fn), errors="ignore").read()
                assert "oracle_py" not in txt and "liboracle" not in txt and "torch_ref" not in txt, fn
