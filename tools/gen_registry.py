"""Generate csrc/vss_registry.inc: the k_block shapes compiled into libvss.so.

One line per (layer shape, output tile, split variant):
    VSS_BLOCK(mode, stride, TH, TW, cin, cskip, chid, cout, flags)
mode 0 = inverted residual with expand, 1 = inverted residual without expand,
2 = decoder; flags = block_flags(norm_in, residual, XP, SP, KS) (vss_kernels.h):
an expand layer whose hidden channels can be split (ks_max > 1) is compiled
unsplit and split KS = ks_max ways (chid = the slice width), and every
consumer of it for XP / SP = 1 and its producer's KS.
Tiles are every candidate that fits the kernel's limits (<= 16 accumulator
tiles per wave, <= 160 KiB LDS); the host planner picks among them at run
time for the handle's model resolution and batch.  The LDS formula mirrors
block_lds() in csrc/vss_kernels.h (tests/test_registry.py checks the two
against each other through libvss's vss_block_lds_bytes).

    python tools/gen_registry.py [spec.json]   # writes csrc/vss_registry*.inc
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPEC = os.path.join(ROOT, "video-stream-segmenetation_amd", "model", "spec.json")
CANDIDATES = [(8, 16), (6, 16), (4, 16), (3, 16), (8, 8), (6, 8), (4, 8), (2, 16), (2, 8), (1, 16)]
MAX_ACC, MAX_LDS = 16, 160 * 1024
HID_STRIDE = 20  # hid_stride() in csrc/vss_kernels.h
SHARDS = 6  # compile units for the block shapes (csrc/Makefile: VSS_SHARDS)


def r4(v):
    return (v + 3) & ~3


# VSS_SWZ in csrc/vss_kernels.h: the round-5 bank-conflict-free LDS layouts
# (env VSS_SWZ=0: round 4's, for a -DVSS_SWZ=0 build: tools/build_variant.sh)
SWZ = os.environ.get("VSS_SWZ", "1") != "0"


def stem_xwp(iw):
    """stem_xwp() in csrc/vss_kernels.h: the fused stem's x0 row pitch."""
    if not SWZ:
        return 2 * iw + 2
    x = 2 * iw + 1
    while (x - (iw + 1)) % 32:
        x += 1
    return x


def stem_in_lds(ih, iw):
    return r4(3 * (2 * ih + 1) * stem_xwp(iw)) + 27 * 16 + 16


def dw_run(tw, npb, pw):
    """dw_run() in csrc/vss_kernels.h: pixels per lane run of the dw stage."""
    if tw % 4 == 0 and 16 % (tw // 4) == 0 and npb % 4 == 0 and (npb // 4) % pw == 0:
        return 4
    if tw % 2 == 0 and 16 % (tw // 2) == 0 and npb % 2 == 0 and (npb // 2) % pw == 0:
        return 2
    return 1


def block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, stem_in=False):
    ih = 2 * th + 1 if stride == 2 else th + 2
    iw = 2 * tw + 1 if stride == 2 else tw + 2
    p_in_pad = (ih * iw + 15) & ~15
    p_out = th * tw
    cx = cin + cskip if mode == 2 else cin
    npb = p_out // 16
    nchunk = chid // 16
    cs = 4 if nchunk >= 4 else (2 if nchunk >= 2 else 1)   # chunk groups: channels only (tile-invariant sums)
    pw = 4 // cs
    if npb % pw:
        return None, None
    npbw = npb // pw
    nacc = npbw * (cout // 16)
    sr, sc = (th + 1) // 2 + 3, (tw + 1) // 2 + 3
    # xt: quad-major planes (direct), swizzled unpadded pixels (expand), or
    # pixel-major rows padded to 8 mod 16 floats (16-wide decoder tiles)
    xqm = SWZ and mode == 1
    xs = (cx + 4) if not SWZ else (4 if xqm else ((cx + (8 if tw == 16 else 4)) if mode == 2 else cx))
    xt_floats = p_in_pad * cx if xqm else r4(p_in_pad * xs)
    rs = cout if SWZ else cout + 4
    xr1 = dw_run(tw, npb, 1) == 1
    hid = 16 * 4 * (p_in_pad + (1 if stride == 2 else 0)) if (SWZ and xr1) else 4 * p_in_pad * HID_STRIDE
    f = xt_floats
    f += r4(p_out * cin) if (mode == 0 and stride == 1 and cin == cout) else 0
    f += r4(chid * (cin + 8) // 2) if mode == 0 else 0
    f += r4(cout * (chid + 8) // 2) + r4(9 * chid) + r4(chid) + (r4(chid) if mode == 0 else 0) + r4(cout)
    f += r4(2 * cin) if mode == 2 else 0
    f += 4 * p_in_pad if mode == 2 and (th % 2 or tw % 2) else 0  # the decoder's upsample tap records (L.uc; odd tiles)
    # work: expand scratch / slabs / (decoder) the low-res src region; the
    # decoder's slabs go into xt when they fit (its stats scratch then in work)
    slab_in_xt = mode == 2 and cs * p_out * rs <= xt_floats
    f += max(hid if mode == 0 else 1024, 0 if slab_in_xt else cs * p_out * rs,
             r4(sr * sc * cin) if mode == 2 else 0, stem_in_lds(ih, iw) if stem_in else 0)
    return f * 4, nacc


def ks_max(layer):
    """Largest hidden split of an expand layer leaving every wave >= 1 chunk
    of 16 channels (mirrors ks_max() in csrc/vss_capi.hip)."""
    if layer["kind"] != "ir" or not layer["expand"]:
        return 1
    nchunk = layer["chid"] // 16
    for k in (4, 3, 2):
        if nchunk % k == 0 and nchunk // k >= 4:
            return k
    return 1


def flags_of(norm_in, residual, xp, sp, ks, stem_in=False):
    return ((1 if norm_in else 0) | (2 if residual else 0) | ((xp - 1) << 2) | ((sp - 1) << 4) | ((ks - 1) << 6) |
            (256 if stem_in else 0))


def shapes(spec):
    layers = spec["layers"]
    names = [l["name"] for l in layers]
    ks_opts = {l["name"]: sorted({1, ks_max(l)}) for l in layers}
    out = []
    for l in layers:
        if l["kind"] == "ir":
            mode = 0 if l["expand"] else 1
            chid = l["chid"] if l["expand"] else l["cin"]
            for ks in ks_opts[l["name"]]:
                for xp in ks_opts[l["src"]]:
                    out.append((l["name"], mode, l["stride"], l["cin"], 0, chid // ks, l["cout"],
                                flags_of(False, l["residual"], xp, 1, ks)))
            src = layers[names.index(l["src"])]
            if src["kind"] == "stem" and not l["expand"] and l["stride"] == 1 and l["cin"] == src["cout"] == 16:
                # the stem fused into its consumer's prologue (STEM_IN)
                out.append((l["name"], mode, 1, l["cin"], 0, chid, l["cout"],
                            flags_of(False, l["residual"], 1, 1, 1, stem_in=True)))
        elif l["kind"] == "dec":
            src = layers[names.index(l["src"])]
            for xp in ks_opts[l["src"]]:
                for sp in ks_opts[l["skip"]]:
                    out.append((l["name"], 2, 1, l["cin"], l["cskip"], l["cin"] + l["cskip"], l["cout"],
                                flags_of(src["kind"] == "dec", False, xp, sp, 1)))
    return out


def main():
    spec = json.load(open(sys.argv[1] if len(sys.argv) > 1 else SPEC))
    entries = []
    seen = set()
    for name, mode, stride, cin, cskip, chid, cout, flags in shapes(spec):
        for th, tw in CANDIDATES:
            lds, nacc = block_lds_bytes(mode, stride, th, tw, cin, cskip, chid, cout, bool(flags & 256))
            if lds is None or nacc > MAX_ACC or lds > MAX_LDS or (th * tw) % 16:
                continue
            key = (mode, stride, th, tw, cin, cskip, chid, cout, flags)
            if key in seen:
                continue
            seen.add(key)
            entries.append((name, key, lds, nacc))
    head = f"// generated by tools/gen_registry.py from {os.path.basename(SPEC)} ({spec['name']}); do not edit"
    lines = [head]
    for name, key, lds, nacc in entries:
        args = ", ".join(str(v) for v in key)
        lines.append(f"VSS_BLOCK({args})  // {name}: {lds // 1024} KiB LDS, {nacc} acc")
    csrc = os.environ.get("VSS_REGISTRY_DIR") or os.path.join(ROOT, "video-stream-segmenetation_amd", "csrc")
    open(os.path.join(csrc, "vss_registry.inc"), "w").write("\n".join(lines) + "\n")
    # the same lines dealt round-robin to the shard files the Makefile compiles in parallel
    for k in range(SHARDS):
        part = [head + f" (shard {k} of {SHARDS})"] + lines[1 + k::SHARDS]
        open(os.path.join(csrc, f"vss_registry_{k}.inc"), "w").write("\n".join(part) + "\n")
    open(os.path.join(csrc, "vss_registry_shards.inc"), "w").write(
        "\n".join([head] + [f"VSS_SHARD_FN({k})" for k in range(SHARDS)]) + "\n")


if __name__ == "__main__":
    main()
