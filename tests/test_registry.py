"""The registry generator's LDS formula (tools/gen_registry.py) must equal the
kernels' own carve (block_lds in csrc/vss_kernels.h, exported by libvss as
vss_block_lds_bytes) for every compiled shape, so its MAX_LDS filter never
lets a tile through that would fail to launch."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_registry", os.path.join(ROOT, "tools", "gen_registry.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_lds_formula_matches_kernel_carve(pkg):
    gen = _gen()
    spec = json.load(open(gen.SPEC))
    checked = 0
    for name, mode, stride, cin, cskip, chid, cout, flags in gen.shapes(spec):
        for th, tw in gen.CANDIDATES:
            py, _ = gen.block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, bool(flags & 256))
            if py is None:
                continue
            c = pkg.block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, 1 if flags & 256 else 0)
            assert py == c, (name, th, tw, py, c)
            checked += 1
    assert checked > 100


def test_registry_is_regenerated():
    """The committed vss_registry.inc is what the generator writes today."""
    gen = _gen()
    spec = json.load(open(gen.SPEC))
    want = set()
    for name, mode, stride, cin, cskip, chid, cout, flags in gen.shapes(spec):
        for th, tw in gen.CANDIDATES:
            lds, nacc = gen.block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, bool(flags & 256))
            if lds is None or nacc > gen.MAX_ACC or lds > gen.MAX_LDS or (th * tw) % 16:
                continue
            want.add((mode, stride, th, tw, cin, cskip, chid, cout, flags))
    got = set()
    inc = os.path.join(ROOT, "video-stream-segmenetation_amd", "csrc", "vss_registry.inc")
    for line in open(inc):
        if line.startswith("VSS_BLOCK("):
            got.add(tuple(int(v) for v in line[len("VSS_BLOCK("):line.index(")")].split(",")))
    assert got == want
