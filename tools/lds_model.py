"""Bank-conflict model of k_block's LDS access sites (csrc/vss_kernels.hip).

For each layer shape of the plan, every LDS access site of the kernel is
enumerated the way the kernel issues it (wave-instruction by wave-instruction,
lane addresses), and its LDS cycles are costed with the gfx950 rules of
/opt/skills/guides/MI355X_MICROARCH.md §LDS:
  ds_read_b128 : 4 lane groups of 16 ({0-3,12-15,20-27}, ...), bank = (a/4) % 64,
                 1 cycle per group + 1 per extra distinct address on a bank;
  ds_read_b64  : 2 groups of 32, bank (a/4) % 64 (2 dwords per lane);
  ds_read_b32  : 2 groups of 32, bank (a/4) % 32;
  ds_write_b128: 8 groups of 8 contiguous lanes, bank (a/4) % 32.
Prints per site: wave-instructions per workgroup, conflict-free cycles, extra
(conflict) cycles — the same quantity as SQ_LDS_BANK_CONFLICT.

    python tools/lds_model.py [--hid-stride 20] [--xs-pad 4] [--rs-pad 4]
"""
from __future__ import annotations

import argparse
from collections import defaultdict

B128_GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
               [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
B128_GROUPS = B128_GROUPS + [[l + 32 for l in g] for g in B128_GROUPS]


def cost(kind, addrs):
    """addrs: 64 byte addresses (None = inactive lane) -> (cycles, extra)."""
    if kind == "r128":
        groups, width, nb = B128_GROUPS, 4, 64
    elif kind == "r64":
        groups, width, nb = [list(range(32)), list(range(32, 64))], 2, 64
    elif kind == "r32":
        groups, width, nb = [list(range(32)), list(range(32, 64))], 1, 32
    elif kind == "w128":
        groups, width, nb = [list(range(8 * k, 8 * k + 8)) for k in range(8)], 4, 32
    else:
        raise ValueError(kind)
    cyc = extra = 0
    for g in groups:
        bank_addrs = defaultdict(set)
        for lane in g:
            a = addrs[lane]
            if a is None:
                continue
            for d in range(width):
                dw = a // 4 + d
                bank_addrs[dw % nb].add(dw)
        if not bank_addrs:
            continue
        deg = max(len(v) for v in bank_addrs.values())
        cyc += 1
        extra += deg - 1
    return cyc, extra


def r4(v):
    return (v + 3) & ~3


def perm(r, on):
    """Lane r's pixel within its 16-pixel block: with `on`, lanes {0-3, 12-15}
    take pixels 0-7 and lanes {4-11} pixels 8-15 (the b128 lane groups then
    always pair a first-half pixel with a second-half one)."""
    if not on:
        return r
    return r if r < 4 else (r + 4 if r < 12 else r - 8)


class Shape:
    def __init__(self, name, mode, stride, th, tw, cin, cskip, chid, cout, hid_stride, xs_pad, rs_pad, pm=False):
        self.name, self.mode, self.S, self.TH, self.TW = name, mode, stride, th, tw
        self.cin, self.cskip, self.CH, self.cout = cin, cskip, chid, cout
        self.IH = 2 * th + 1 if stride == 2 else th + 2
        self.IW = 2 * tw + 1 if stride == 2 else tw + 2
        self.P_in = self.IH * self.IW
        self.P_in_pad = (self.P_in + 15) & ~15
        self.P_out = th * tw
        self.CX = cin + cskip if mode == 2 else cin
        self.XS = self.CX + xs_pad
        self.HS = hid_stride
        self.RS = cout + rs_pad
        nchunk = chid // 16
        self.CS = 4 if nchunk >= 4 else (2 if nchunk >= 2 else 1)
        self.PW = 4 // self.CS
        self.NPB = self.P_out // 16
        self.NPBW = self.NPB // self.PW
        self.NCB = cout // 16
        self.NCHUNK = nchunk
        self.pm = pm


def sites(sh):
    """Yield (site, kind, [64 addresses]) for one workgroup of shape sh (waves 0..3)."""
    XS, HS, RS = sh.XS, sh.HS, sh.RS
    # prologue commit of the input tile (IR): thread i -> pixel i // C4, c4 = i % C4
    C4 = sh.cin // 4
    tot = sh.P_in_pad * C4
    for u in range((tot + 255) // 256):
        for w in range(4):
            ad = []
            for l in range(64):
                i = 256 * u + 64 * w + l
                ad.append((i // C4 * XS + 4 * (i % C4)) * 4 if i < tot else None)
            yield "commit x (w128)", "w128", ad
    if sh.mode == 0:
        # expand: per wave chunk ck: MFMA B reads over all input pixel blocks, hid writes
        NK = sh.cin // 16
        for w in range(4):
            for ck in range(w, sh.NCHUNK, 4):
                for cb in range(sh.P_in_pad // 16):
                    for s in range(NK):
                        ad = [((cb * 16 + (l & 15)) * XS + 16 * s + 4 * (l >> 4)) * 4 for l in range(64)]
                        yield "expand B (r128)", "r128", ad
                    ad = [((cb * 16 + (l & 15)) * HS + 4 * (l >> 4)) * 4 for l in range(64)]
                    yield "hid write (w128)", "w128", ad
                # dw taps from hid
                for pb in range(sh.NPB):
                    for ky in range(3):
                        for kx in range(3):
                            ad = []
                            for l in range(64):
                                pix = pb * 16 + perm(l & 15, sh.pm)
                                ly, lx = pix // sh.TW, pix % sh.TW
                                sp = (sh.S * ly + ky) * sh.IW + sh.S * lx + kx
                                ad.append((sp * HS + 4 * (l >> 4)) * 4)
                            yield "dw taps hid (r128)", "r128", ad
    else:
        for w in range(4):
            pw, cw = w % sh.PW, w // sh.PW
            for ck in range(cw, sh.NCHUNK, sh.CS):
                c0 = ck * 16
                for i in range(sh.NPBW):
                    pb = pw + i * sh.PW
                    for ky in range(3):
                        for kx in range(3):
                            ad = []
                            for l in range(64):
                                pix = pb * 16 + perm(l & 15, sh.pm)
                                ly, lx = pix // sh.TW, pix % sh.TW
                                ad.append((((ly + ky) * sh.IW + lx + kx) * XS + c0 + 4 * (l >> 4)) * 4)
                            yield "dw taps xt (r128)", "r128", ad
    # epilogue slab writes: wave (pw, cw) acc[i][cb] -> slab cw, pixel (pb*16 + r), channel cb*16 + 4g
    for w in range(4):
        pw, cw = w % sh.PW, w // sh.PW
        for i in range(sh.NPBW):
            pb = pw + i * sh.PW
            for cb in range(sh.NCB):
                ad = [(cw * sh.P_out * RS + (pb * 16 + (l & 15)) * RS + cb * 16 + 4 * (l >> 4)) * 4 for l in range(64)]
                yield "slab write (w128)", "w128", ad
    # epilogue reads: i = tid + 256k -> pix = i // C4O, c4 = i % C4O, CS slabs
    C4O = sh.cout // 4
    tot = sh.P_out * C4O
    for k in range((tot + 255) // 256):
        for w in range(4):
            for s in range(sh.CS):
                ad = []
                for l in range(64):
                    i = 256 * k + 64 * w + l
                    ad.append((s * sh.P_out * RS + (i // C4O) * RS + 4 * (i % C4O)) * 4 if i < tot else None)
                yield "slab read (r128)", "r128", ad


PLAN = [  # the autotuned tiles at 144x256, batch 8 (bench r02b)
    ("b1", 1, 1, 4, 16, 16, 0, 16, 16),
    ("b2", 0, 2, 2, 8, 16, 0, 64, 32),
    ("b3", 0, 1, 3, 16, 32, 0, 128, 32),
    ("b4", 0, 2, 2, 8, 32, 0, 128, 48),
    ("b5", 0, 1, 4, 8, 48, 0, 64, 48),
    ("b6", 0, 2, 2, 8, 48, 0, 64, 64),
    ("b7", 0, 1, 6, 8, 64, 0, 64, 64),
    ("d1", 2, 1, 2, 8, 64, 48, 112, 48),
    ("d2", 2, 1, 4, 8, 48, 32, 80, 32),
    ("d3", 2, 1, 6, 16, 32, 16, 48, 16),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hid-stride", type=int, default=20)
    ap.add_argument("--xs-pad", type=int, default=4)
    ap.add_argument("--rs-pad", type=int, default=4)
    ap.add_argument("--hid-stride2", type=int, default=0, help="hid stride of stride-2 layers (0: --hid-stride)")
    ap.add_argument("--perm", action="store_true", help="lane -> pixel permutation of the 16-pixel blocks")
    args = ap.parse_args()
    grand = [0, 0]
    for row in PLAN:
        hs = args.hid_stride2 if (args.hid_stride2 and row[2] == 2) else args.hid_stride
        sh = Shape(*row, hs, args.xs_pad, args.rs_pad, args.perm)
        per = defaultdict(lambda: [0, 0, 0])
        for site, kind, ad in sites(sh):
            c, e = cost(kind, ad)
            per[site][0] += 1
            per[site][1] += c
            per[site][2] += e
        tot_i = sum(v[0] for v in per.values())
        tot_e = sum(v[2] for v in per.values())
        grand[0] += tot_i
        grand[1] += tot_e
        print(f"{row[0]}: {tot_i} LDS wave-instr (modelled sites), {tot_e} conflict cycles, ratio {tot_e / max(tot_i, 1):.2f}")
        for site, (n, c, e) in sorted(per.items(), key=lambda kv: -kv[1][2]):
            print(f"    {site:22s} n={n:6d} cycles={c:7d} extra={e:7d}")
    print(f"total modelled: {grand[0]} instr, {grand[1]} conflict cycles per set of workgroups")


if __name__ == "__main__":
    main()
