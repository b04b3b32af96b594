"""Every LDS access site of the hot block kernels, lane by lane, costed with
gfx950's bank rules (/opt/skills/guides/MI355X_MICROARCH.md §LDS), per wave
and per layer — the full-kernel successor of tools/lds_model.py (which covers
the main loops only).  Sites follow csrc/vss_kernels.hip's block_body
statement by statement (prologue commits, the fused stem of b1, the
decoder's 2x upsample, the main loop, the epilogue and the decoder's norm
statistics); each yields (site, kind, 64 byte addresses or None per lane).

Kinds (lane groups / bank of dword address d):
  r32, w32       : {0-31}, {32-63}; d % 32
  r64            : {0-31}, {32-63}; d % 64, 2 dwords per lane
  r128           : {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32); d % 64, 4 dwords
  w128           : 8 groups of 8 contiguous lanes; d % 32, 4 dwords
  r2_64          : two accesses (offset0/offset1), each 4 groups of 16 contiguous; d % 32
  w2_32 / r2_32  : two b32 accesses
Extra cycles = per group, the largest number of distinct dwords on one bank,
minus 1 — the quantity SQ_LDS_BANK_CONFLICT counts.

    python tools/lds_sites.py [--layer b1|b3|d3|all] [--xs-pad 4] [--hs1 20] [--perm]
"""
from __future__ import annotations

import argparse
from collections import defaultdict

B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
               [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
B128_GROUPS = B128_GROUPS + [[l + 32 for l in g] for g in B128_GROUPS]
HALVES = [list(range(32)), list(range(32, 64))]


def _groups_cost(groups, width, nb, addrs):
    cyc = extra = 0
    for g in groups:
        bank = defaultdict(set)
        for lane in g:
            a = addrs[lane]
            if a is None:
                continue
            assert a % 4 == 0, a
            for d in range(width):
                dw = a // 4 + d
                bank[dw % nb].add(dw)
        if bank:
            cyc += 1
            extra += max(len(v) for v in bank.values()) - 1
    return cyc, extra


def cost(kind, addrs):
    if kind in ("r32", "w32"):
        return _groups_cost(HALVES, 1, 32, addrs)
    if kind == "r64":
        return _groups_cost(HALVES, 2, 64, addrs)
    if kind == "r128":
        return _groups_cost(B128_GROUPS, 4, 64, addrs)
    if kind == "w128":
        return _groups_cost([list(range(8 * k, 8 * k + 8)) for k in range(8)], 4, 32, addrs)
    if kind == "r2_64":  # each half-access: 4 x 16 contiguous lanes
        return _groups_cost([list(range(16 * k, 16 * k + 16)) for k in range(4)], 2, 32, addrs)
    raise ValueError(kind)


def r4(v):
    return (v + 3) & ~3


class Lds:
    """block_lds() of csrc/vss_kernels.h, in floats."""

    def __init__(self, mode, stride, TH, TW, cin, cskip, chid, cout, stem_in=False, xs_pad=4, hs1=20, quads=True,
                 swz=False):
        self.mode, self.S, self.TH, self.TW = mode, stride, TH, TW
        self.stem_in = stem_in
        self.cin, self.cskip, self.CH, self.cout = cin, cskip, chid, cout
        self.IH = 2 * TH + 1 if stride == 2 else TH + 2
        self.IW = 2 * TW + 1 if stride == 2 else TW + 2
        self.P_in = self.IH * self.IW
        self.P_in_pad = (self.P_in + 15) & ~15
        self.P_out = TH * TW
        self.CX = cin + cskip if mode == 2 else cin
        self.XS = self.CX + xs_pad
        self.LD1, self.LD2 = cin + 8, chid + 8
        self.SR, self.SC = (TH + 1) // 2 + 3, (TW + 1) // 2 + 3
        self.NCB, self.NPB, self.NCHUNK = cout // 16, self.P_out // 16, chid // 16
        self.CS = 4 if self.NCHUNK >= 4 else (2 if self.NCHUNK >= 2 else 1)
        self.PW = 4 // self.CS
        self.NPBW = self.NPB // self.PW
        self.slab_stride = self.P_out * (cout + 4)
        self.HSD = (20 if hs1 == 20 else hs1) if stride == 2 else hs1
        o = 0
        self.xt = o; o += r4(self.P_in_pad * self.XS)
        self.xr = o; o += r4(self.P_out * cin) if (mode == 0 and stride == 1 and cin == cout) else 0
        self.w1 = o; o += r4(chid * self.LD1 // 2) if mode == 0 else 0
        self.w2 = o; o += r4(cout * self.LD2 // 2)
        self.wdw = o; o += r4(9 * chid)
        self.bdw = o; o += r4(chid)
        self.b1 = o; o += r4(chid) if mode == 0 else 0
        self.b2 = o; o += r4(cout)
        self.wimg_end = o
        xt_floats = r4(self.P_in_pad * self.XS)
        slab_in_xt = mode == 2 and self.CS * self.slab_stride <= xt_floats
        self.work = self.lr = o
        stem = r4(3 * (2 * self.IH + 1) * (2 * self.IW + 2)) + 27 * 16 + 16 if stem_in else 0
        o += max(4 * self.P_in_pad * self.HSD if mode == 0 else 1024, 0 if slab_in_xt else self.CS * self.slab_stride,
                 r4(self.SR * self.SC * cin) if mode == 2 else 0, stem)
        self.nrm = o; o += r4(2 * cin) if mode == 2 else 0
        self.quads = quads and TH % 2 == 0 and TW % 2 == 0
        self.uc = o; o += 4 * self.P_in_pad if (mode == 2 and not self.quads) else 0
        self.slab = self.xt if slab_in_xt else self.work
        self.stt = self.work if slab_in_xt else self.xt
        self.total = o
        self.RS = cout + 4
        # quad swizzles (pixel -> XOR of the channel-quad index), identity by default
        self.sx = self.sh = self.ss = self.sr = (lambda pix: 0)
        self.xqm = self.hqm = self.skp = False
        self.stem_t, self.xwp = False, None
        if swz:
            self.set_swz()

    def set_swz(self):
        """The round-5 layouts of block_lds() with VSS_SWZ=1 (csrc/vss_kernels.h)."""
        def gray(m):
            return lambda p: (p ^ (p >> 1)) & (m - 1)

        def p2(q):
            return 16 if q % 16 == 0 else 8 if q % 8 == 0 else 4 if q % 4 == 0 else 2 if q % 2 == 0 else 1
        mode, S = self.mode, self.S
        self.xqm = mode == 1
        self.XS = 4 if self.xqm else (self.CX + (8 if self.TW == 16 else 4) if mode == 2 else self.CX)
        self.XPL = 4 * self.P_in_pad
        self.sx = gray(p2(self.CX // 4)) if mode == 0 else (lambda p: 0)
        self.hqm = mode == 0 and dw_run(self.TW, self.NPB, 1) == 1
        self.skp = mode == 2 and self.cskip == 16 and (self.XS // 4) % 4 == 2
        self.HPL = 4 * (self.P_in_pad + (1 if S == 2 else 0))
        self.RS = self.cout
        self.ss = gray(p2(self.cout // 4))
        m = p2(self.cin // 4)
        self.sr = lambda p: p & (m - 1)
        self.slab_stride = self.P_out * self.RS
        self.stem_t = True
        x = 2 * self.IW + 1
        while (x - (self.IW + 1)) % 32:
            x += 1
        self.xwp = x
        # the carve (offsets only matter mod 64 dwords for the banks: recompute like block_lds)
        o = 0
        xt_floats = self.P_in_pad * self.CX if self.xqm else r4(self.P_in_pad * self.XS)
        self.xt = o; o += xt_floats
        self.xr = o; o += r4(self.P_out * self.cin) if (mode == 0 and S == 1 and self.cin == self.cout) else 0
        self.w1 = o; o += r4(self.CH * self.LD1 // 2) if mode == 0 else 0
        self.w2 = o; o += r4(self.cout * self.LD2 // 2)
        self.wdw = o; o += r4(9 * self.CH)
        self.bdw = o; o += r4(self.CH)
        self.b1 = o; o += r4(self.CH) if mode == 0 else 0
        self.b2 = o; o += r4(self.cout)
        self.wimg_end = o
        slab_in_xt = mode == 2 and self.CS * self.slab_stride <= xt_floats
        self.work = self.lr = o
        stem = r4(3 * (2 * self.IH + 1) * self.xwp) + 27 * 16 + 16 if self.stem_in else 0
        o += max((16 * self.HPL if self.hqm else 4 * self.P_in_pad * self.HSD) if mode == 0 else 1024, 0 if slab_in_xt else self.CS * self.slab_stride,
                 r4(self.SR * self.SC * self.cin) if mode == 2 else 0, stem)
        self.nrm = o; o += r4(2 * self.cin) if mode == 2 else 0
        self.uc = o; o += 4 * self.P_in_pad if (mode == 2 and not self.quads) else 0
        self.slab = self.xt if slab_in_xt else self.work
        self.stt = self.work if slab_in_xt else self.xt
        self.total = o

    @staticmethod
    def _sw(stride, s, pix, ch):
        return pix * stride + 4 * ((ch >> 2) ^ s(pix)) + (ch & 3)

    def xt_at(self, pix, ch):
        if self.xqm:
            return self.xt + (ch >> 2) * self.XPL + 4 * pix + (ch & 3)
        return self.xt + self._sw(self.XS, self.sx, pix, ch)

    def hid_at(self, base, pix, ch):
        if self.hqm:
            return base + (ch >> 2) * self.HPL + 4 * pix + (ch & 3)
        return base + self._sw(self.HSD, self.sh, pix, ch)

    def slab_at(self, s_, pix, ch):
        return self.slab + s_ * self.slab_stride + self._sw(self.RS, self.ss, pix, ch)

    def xr_at(self, pix, ch):
        return self.xr + self._sw(self.cin, self.sr, pix, ch)


def dw_run(TW, NPB, PW):
    if TW % 4 == 0 and 16 % (TW // 4) == 0 and NPB % 4 == 0 and (NPB // 4) % PW == 0:
        return 4
    if TW % 2 == 0 and 16 % (TW // 2) == 0 and NPB % 2 == 0 and (NPB // 2) % PW == 0:
        return 2
    return 1


def lanes(fn):
    """64 byte addresses from fn(lane) -> float offset or None."""
    out = []
    for l in range(64):
        v = fn(l)
        out.append(None if v is None else 4 * v)
    return out


def tid_lanes(w, fn):
    return lanes(lambda l: fn(64 * w + l))


def sites(L, tile, img, stem_geo=None):
    """Sites of one workgroup (4 waves) of layer shape L at tile (bx, by) of an
    image of img = (H, W) input pixels (IR: the input; DEC: skip/output), i.e.
    the block_body code path for that tile."""
    bx, by = tile
    H, W = img
    TH, TW, IW, XS, S = L.TH, L.TW, L.IW, L.XS, L.S
    oy0, ox0 = by * TH, bx * TW
    iy0, ix0 = S * oy0 - 1, S * ox0 - 1
    Ho, Wo = (H, W) if L.mode == 2 else ((H + S - 1) // S, (W + S - 1) // S)
    wimg_f4 = (L.wimg_end - L.w1) // 4
    out = []

    def emit(site, kind, w, fn):
        out.append((site, kind, w, tid_lanes(w, fn)))

    if L.mode == 2:
        CL, C4L, SR, SC = L.cin, L.cin // 4, L.SR, L.SC
        GL, GS = CL // 16, L.cskip // 16
        # norm slots staged in xt (16-B items) then summed by tid < CL reading b64
        nslot16 = 4 * 2 * CL // 2
        for u in range((nslot16 + 255) // 256):
            for w in range(4):
                emit("dec: norm slots -> xt (w128)", "w128", w, lambda t, u=u: 4 * (t + 256 * u) if t + 256 * u < nslot16 else None)
        for k in range(4):
            for part in (0, 1):  # s_fx, q_fx reads, int64 (compiler: b64 reads)
                for w in range(4):
                    emit("dec: norm slot sums (r64)", "r64", w,
                         lambda t, k=k, part=part: 2 * (k * 2 * CL + part * CL + t) if t < CL else None)
        for w in range(4):
            emit("dec: scale/shift writes (w32)", "w32", w, lambda t: L.nrm + t if t < CL else None)
            emit("dec: scale/shift writes (w32)", "w32", w, lambda t: L.nrm + CL + t if t < CL else None)
        # lr commit (float4 j -> lane j % 256): lr[4 * item + k] = lr f4 index j
        tot = 4 * SR * SC * GL
        for u in range((tot + 255) // 256):
            for w in range(4):
                emit("dec: src region commit (w128)", "w128", w,
                     lambda t, u=u: L.lr + 4 * (t + 256 * u) if t + 256 * u < tot else None)
            # norm scale/shift reads on commit (two f4 per item, by channel group)
            for w in range(4):
                for base in (0, CL):
                    emit("dec: commit scale/shift (r128)", "r128", w,
                         lambda t, u=u, base=base: L.nrm + base + 4 * (((t + 256 * u) >> 2) % GL * 4 + ((t + 256 * u) & 3))
                         if t + 256 * u < tot else None)
        tot = 4 * L.P_in_pad * GS
        for u in range((tot + 255) // 256):
            for w in range(4):
                def sk(t, u=u):
                    j = t + 256 * u
                    if j >= tot:
                        return None
                    i, k = j >> 2, j & 3
                    pix, gq = i // GS, i % GS
                    if L.skp:
                        pix = (pix & ~3) | ((pix & 1) << 1) | ((pix >> 1) & 1)
                    return L.xt_at(pix, CL + 16 * gq + 4 * k)
                emit("dec: skip commit (w128)", "w128", w, sk)
        for u in range((wimg_f4 + 255) // 256):
            for w in range(4):
                emit("weight image commit (w128)", "w128", w,
                     lambda t, u=u: L.w1 + 4 * (t + 256 * u) if t + 256 * u < wimg_f4 else None)
        assert L.quads
        QH, QW = L.IH // 2, IW // 2
        NQI = QH * QW * C4L
        sy0, sx0 = max(0, (oy0 - 1) // 2 - 1), max(0, (ox0 - 1) // 2 - 1)
        j0, i0 = (iy0 - 1) // 2 if iy0 >= 1 else -1, (ix0 - 1) // 2 if ix0 >= 1 else -1
        jr, ic = j0 - sy0, i0 - sx0
        for k in range((NQI + 255) // 256):
            def quad(t, k=k):
                it = t + 256 * k
                if it >= NQI:
                    return None
                c4, qq = it % C4L, it // C4L
                return c4, qq % QW, qq // QW
            for w in range(4):
                for dr, dc in ((0, 0), (0, 1), (1, 0), (1, 1)):
                    def rd(t, dr=dr, dc=dc):
                        q = quad(t)
                        if q is None:
                            return None
                        c4, qx, qy = q
                        ra = min(max(qy + jr + dr, 0), SR - 1)
                        ca = min(max(qx + ic + dc, 0), SC - 1)
                        return L.lr + ra * (SC * CL) + 4 * c4 + ca * CL
                    emit("dec: upsample tap reads (r128)", "r128", w, rd)
                for dy, dx in ((0, 0), (0, 1), (1, 0), (1, 1)):
                    def wr(t, dy=dy, dx=dx):
                        q = quad(t)
                        if q is None:
                            return None
                        c4, qx, qy = q
                        return L.xt_at((2 * qy + dy) * IW + 2 * qx + dx, 4 * c4)
                    emit("dec: upsample writes (w128)", "w128", w, wr)
    elif stem_geo is not None:
        # fused stem (b1): x0 region resize writes, stem weights, MFMA taps, xt writes
        Hm, Wm = stem_geo
        XH, XW = 2 * L.IH + 1, 2 * IW + 1
        XWP = getattr(L, "xwp", None) or XW + 1
        x0s, sws = L.work, L.work + r4(3 * XH * XWP)
        sbs = sws + 27 * 16
        HW2 = (XW + 1) // 2
        NPAIR = XH * HW2
        for u in range((NPAIR + 255) // 256):
            for e in (0, 1):
                for c in range(3):
                    for w in range(4):
                        def xw(t, u=u, e=e, c=c):
                            i = t + 256 * u
                            if i >= NPAIR:
                                return None
                            ly, lx = i // HW2, i % HW2 + e * HW2
                            return x0s + (c * XH + ly) * XWP + lx if lx < XW else None
                        emit("b1: resized region writes (w32)", "w32", w, xw)
        for u in range(2):
            for w in range(4):
                if getattr(L, "stem_t", False):  # thread i writes sws[i] (the load reads w transposed)
                    emit("b1: stem weight writes (w32)", "w32", w,
                         lambda t, u=u: sws + t + 256 * u if t + 256 * u < 432 else None)
                else:
                    emit("b1: stem weight writes (w32)", "w32", w,
                         lambda t, u=u: sws + ((t + 256 * u) % 27) * 16 + (t + 256 * u) // 27 if t + 256 * u < 432 else None)
        for w in range(4):
            emit("b1: stem bias write (w32)", "w32", w, lambda t: sbs + t if t < 16 else None)
        for u in range((wimg_f4 + 255) // 256):
            for w in range(4):
                emit("weight image commit (w128)", "w128", w,
                     lambda t, u=u: L.w1 + 4 * (t + 256 * u) if t + 256 * u < wimg_f4 else None)
        # the taps' weights: 7 b32 reads (compiled as 3 read2st64 + 1 b32) + the bias
        for w in range(4):
            for s_ in range(7):
                emit("b1: stem tap weights (r32)", "r32", w, lambda t, s_=s_: sws + (4 * s_ + (t % 64) // 16) * 16 + t % 16)
            emit("b1: stem bias read (r32)", "r32", w, lambda t: sbs + t % 16)
        plane, row = XH * XWP, XWP
        offs = []
        for k in range(28):
            offs.append((k // 9) * plane + ((k % 9) // 3) * row + k % 3 if k < 27 else 0)
        for w in range(4):
            for blk in range(w, L.P_in_pad // 16, 4):
                def corner(t, blk=blk):
                    r = t % 16
                    pa = min(blk * 16 + r, L.P_in - 1)
                    py, px = pa // IW, pa % IW
                    return x0s + 2 * py * XWP + 2 * px
                for s_ in range(7):
                    emit("b1: stem MFMA taps (r32)", "r32", w,
                         lambda t, s_=s_: corner(t) + offs[4 * s_ + (t % 64) // 16])
                if getattr(L, "stem_t", False):  # transposed MFMA: lane (r, g) = pixel r, channels 4g..4g+3
                    emit("b1: stem out -> xt (w128)", "w128", w,
                         lambda t, blk=blk: L.xt_at(blk * 16 + t % 16, 4 * ((t % 64) // 16)))
                    continue
                for i in range(0, 4, 2):  # ds_write2_b32: pixels 4g+i, 4g+i+1 (stride XS)
                    for ii in (i, i + 1):
                        emit("b1: stem out -> xt (w2_32)", "w32", w,
                             lambda t, blk=blk, ii=ii: L.xt_at(blk * 16 + 4 * ((t % 64) // 16) + ii, t % 16))
        interior = iy0 >= 0 and iy0 + L.IH <= H and ix0 >= 0 and ix0 + IW <= W
        if not interior:
            for u in range((L.P_in * 4 + 255) // 256):
                for w in range(4):
                    def zw(t, u=u):
                        i = t + 256 * u
                        if i >= L.P_in * 4:
                            return None
                        q, e = (i // L.P_in, i % L.P_in) if L.xqm else (i & 3, i >> 2)
                        qy, qx = e // IW, e % IW
                        yy, xx = iy0 + qy, ix0 + qx
                        if 0 <= yy < H and 0 <= xx < W:
                            return None
                        return L.xt_at(qy * IW + qx, 4 * q)
                    a = tid_lanes(w, zw)
                    if any(v is not None for v in a):
                        out.append(("b1: edge zeroing (w128)", "w128", w, a))
    else:
        GI = L.cin // 16
        tot = L.P_in_pad * GI  # whole 16-channel items per lane (VSS_STAGE16)
        for u in range((tot + 255) // 256):
            for k in range(4):
                for w in range(4):
                    def xc(t, u=u, k=k):
                        i = t + 256 * u
                        if i >= tot:
                            return None
                        pix, gq = i // GI, i % GI
                        return L.xt_at(pix, 4 * (gq * 4 + k))
                    emit("ir: input tile commit (w128)", "w128", w, xc)
                    if L.mode == 0 and L.S == 1 and L.cin == L.cout:
                        def rc(t, u=u, k=k):
                            i = t + 256 * u
                            if i >= tot:
                                return None
                            pix, gq = i // GI, i % GI
                            py, px = pix // IW, pix % IW
                            if 1 <= py <= TH and 1 <= px <= TW:
                                return L.xr_at((py - 1) * TW + px - 1, 4 * (gq * 4 + k))
                            return None
                        a = tid_lanes(w, rc)
                        if any(v is not None for v in a):
                            out.append(("ir: residual centre commit (w128)", "w128", w, a))
        for u in range((wimg_f4 + 255) // 256):
            for w in range(4):
                emit("weight image commit (w128)", "w128", w,
                     lambda t, u=u: L.w1 + 4 * (t + 256 * u) if t + 256 * u < wimg_f4 else None)
    # ---- main ----
    XR = dw_run(TW, L.NPB, 1 if L.mode == 0 else L.PW)

    def run_pix(sb, j, r):
        if XR == 1:
            return sb * 16 + r
        return (sb * (16 * XR // TW) + r // (TW // XR)) * TW + (r % (TW // XR)) * XR + j

    for w in range(4):
        pw, cw = w % L.PW, w // L.PW
        chunks = list(range(w, L.NCHUNK, 4)) if L.mode == 0 else list(range(cw, L.NCHUNK, L.CS))
        for ck in chunks:
            c0 = ck * 16
            if L.mode == 0:
                NK = L.cin // 16
                for s_ in range(NK):  # aw: lds_a rows (b64)
                    emit("ir: expand A frags (r64)", "r64", w,
                         lambda t, s_=s_: L.w1 + ((c0 + t % 16) * L.LD1 + 16 * s_ + 4 * ((t % 64) // 16)) // 2)
                emit("ir: expand bias (r128)", "r128", w, lambda t: L.b1 + c0 + 4 * ((t % 64) // 16))
                hid = L.work + w * (4 * L.HPL if L.hqm else L.P_in_pad * L.HSD)
                for cb in range(L.P_in_pad // 16):
                    for s_ in range(NK):
                        emit("ir: expand B reads (r128)", "r128", w,
                             lambda t, cb=cb, s_=s_: L.xt_at(cb * 16 + t % 16, 16 * s_ + 4 * ((t % 64) // 16)))
                    emit("ir: hidden chunk writes (w128)", "w128", w,
                         lambda t, cb=cb: L.hid_at(hid, cb * 16 + t % 16, 4 * ((t % 64) // 16)))
                at, npbw, cbase = (lambda pix, ch, hid=hid: L.hid_at(hid, pix, ch)), L.NPB, 0
            else:
                at, npbw, cbase = L.xt_at, L.NPBW, c0
            for tt in range(9):
                emit("dw tap weights (r128)", "r128", w, lambda t, tt=tt: L.wdw + tt * L.CH + c0 + 4 * ((t % 64) // 16))
            emit("dw bias (r128)", "r128", w, lambda t: L.bdw + c0 + 4 * ((t % 64) // 16))
            for cb in range(L.NCB):
                emit("project A frags (r64)", "r64", w,
                     lambda t, cb=cb: L.w2 + ((cb * 16 + t % 16) * L.LD2 + c0 + 4 * ((t % 64) // 16)) // 2)
            nq = (L.NPB if L.mode == 0 else npbw) // XR
            for q in range(nq):
                sb = q if L.mode == 0 else pw + q * L.PW
                NT = S * (XR - 1) + 3
                for ky in range(3):
                    for u in range(NT):
                        def tap(t, ky=ky, u=u, sb=sb):
                            p0 = run_pix(sb, 0, t % 16)
                            ly, lx0 = p0 // TW, p0 % TW
                            return at((S * ly + ky) * IW + S * lx0 + u, cbase + 4 * ((t % 64) // 16))
                        emit("dw taps (r128)", "r128", w, tap)
    # ---- epilogue ----
    C4O = L.cout // 4
    if L.mode == 1 and L.CS == 1:
        for w in range(4):
            emit("epilogue bias (r128)", "r128", w, lambda t: L.b2 + 4 * ((t % 64) // 16))
            for q in range(L.NPBW // XR):
                for j in range(XR):
                    def ctr(t, q=q, j=j):
                        pix = run_pix(w % L.PW + q * L.PW, j, t % 16)
                        ly, lx = pix // TW, pix % TW
                        return L.xt_at((ly + 1) * IW + lx + 1, 4 * ((t % 64) // 16))
                    emit("residual centre (r128)", "r128", w, ctr)
        return out
    RS = L.RS
    for w in range(4):
        pw, cw = w % L.PW, w // L.PW
        nsb = (L.NPB if L.mode == 0 else L.NPBW) // XR
        for q in range(nsb):
            for j in range(XR):
                for cb in range(L.NCB):
                    def sw_(t, q=q, j=j, cb=cb, pw=pw, cw=cw):
                        sb = q if L.mode == 0 else pw + q * L.PW
                        return L.slab_at(cw, run_pix(sb, j, t % 16), cb * 16 + 4 * ((t % 64) // 16))
                    emit("slab writes (w128)", "w128", w, sw_)
    nout = (L.P_out * C4O + 255) // 256
    for k in range(nout):
        for w in range(4):
            def it(t, k=k):
                i = t + 256 * k
                return (i // C4O, i % C4O) if i < L.P_out * C4O else None
            for s_ in range(L.CS):
                emit("slab sum reads (r128)", "r128", w,
                     lambda t, s_=s_: None if it(t) is None else
                     L.slab_at(s_, it(t)[0], 4 * it(t)[1]))
            emit("epilogue bias (r128)", "r128", w, lambda t: None if it(t) is None else L.b2 + 4 * it(t)[1])
            if L.mode == 0 and L.S == 1 and L.cin == L.cout:
                emit("residual centre (r128)", "r128", w,
                     lambda t: None if it(t) is None else L.xr_at(it(t)[0], 4 * it(t)[1]))
            if L.mode == 2:
                emit("dec: slab write-back (w128)", "w128", w,
                     lambda t: None if it(t) is None else L.slab_at(0, it(t)[0], 4 * it(t)[1]))
    if L.mode == 2:
        G = 256 // L.cout
        for w in range(4):
            for pix in range(0, L.P_out, G):
                emit("dec: stats slab reads (r32)", "r32", w,
                     lambda t, pix=pix: L.slab_at(0, pix + t // L.cout, t % L.cout)
                     if t // L.cout < G and pix + t // L.cout < L.P_out else None)
            for part in (0, 1):
                emit("dec: stats int64 writes (r64/w)", "r64", w,
                     lambda t, part=part: L.stt + 2 * (256 * part + (t // L.cout) * L.cout + t % L.cout)
                     if t // L.cout < G else None)
            for k in range(G):
                emit("dec: stats int64 reads (r64)", "r64", w,
                     lambda t, k=k: L.stt + 2 * ((t if t < L.cout else 256 + t - L.cout) + k * L.cout)
                     if t < 2 * L.cout else None)
    return out


LAYERS = {  # the bench's tiles (r04q): name -> (mode, stride, TH, TW, cin, cskip, chid, cout, stem_in, H, W)
    "b1": (1, 1, 4, 16, 16, 0, 16, 16, True, 72, 128),
    "b2": (0, 2, 2, 8, 16, 0, 64, 32, False, 72, 128),
    "b3": (0, 1, 3, 16, 32, 0, 128, 32, False, 36, 64),
    "b4": (0, 2, 2, 8, 32, 0, 128, 48, False, 36, 64),
    "b5": (0, 1, 4, 8, 48, 0, 192, 48, False, 18, 32),
    "b6": (0, 2, 2, 8, 48, 0, 192, 64, False, 18, 32),
    "b7": (0, 1, 2, 8, 64, 0, 256, 64, False, 9, 16),
    "d1": (2, 1, 4, 8, 64, 48, 112, 48, False, 18, 32),
    "d2": (2, 1, 4, 8, 48, 32, 80, 32, False, 36, 64),
    "d3": (2, 1, 6, 16, 32, 16, 48, 16, False, 72, 128),
}
MEASURED = {  # r04q SQ pass per wave: (LDS instructions, conflict cycles)
    "b1": (238096 / 4608, 577152 / 4608), "b3": (186240 / 1536, 445440 / 1536), "d3": (267304 / 3072, 602873 / 3072),
}


def model(name, xs_pad=4, hs1=20, verbose=True, swz=False):
    mode, S, TH, TW, cin, cskip, chid, cout, stem_in, H, W = LAYERS[name]
    L = Lds(mode, S, TH, TW, cin, cskip, chid, cout, stem_in, xs_pad, hs1, swz=swz)
    Ho, Wo = (H, W) if mode == 2 else ((H + S - 1) // S, (W + S - 1) // S)
    tiles = [(bx, by) for by in range((Ho + TH - 1) // TH) for bx in range((Wo + TW - 1) // TW)]
    per = defaultdict(lambda: [0, 0, 0])
    for t in tiles:
        for site, kind, w, ad in sites(L, t, (H, W), (2 * H, 2 * W) if stem_in else None):
            if all(a is None for a in ad):
                continue
            c, e = cost(kind, ad)
            per[site][0] += 1
            per[site][1] += c
            per[site][2] += e
    nw = 4 * len(tiles)
    ti = sum(v[0] for v in per.values()) / nw
    te = sum(v[2] for v in per.values()) / nw
    if verbose:
        mi, me = MEASURED.get(name, (0, 0))
        print(f"{name}: LDS {L.total * 4} B; per wave {ti:.1f} LDS instr, {te:.1f} conflict cycles "
              f"({te / max(ti, 1e-9):.2f} per instr); measured {mi:.1f} / {me:.1f} ({me / max(mi, 1e-9):.2f})")
        for site, (n, c, e) in sorted(per.items(), key=lambda kv: -kv[1][2]):
            print(f"    {site:36s} instr/wave {n / nw:6.2f}  extra/wave {e / nw:7.2f}  ({e / max(n, 1):.2f} per instr)")
    return ti, te, L.total * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="all")
    ap.add_argument("--xs-pad", type=int, default=4)
    ap.add_argument("--hs1", type=int, default=20)
    ap.add_argument("--swz", action="store_true", help="the round-5 layouts (VSS_SWZ=1)")
    a = ap.parse_args()
    for n in (LAYERS if a.layer == "all" else [a.layer]):
        model(n, a.xs_pad, a.hs1, swz=a.swz)


if __name__ == "__main__":
    main()
