"""Static instruction mix of one kernel in a device assembly file (hipcc -S
--cuda-device-only): counts by class, and the VALU opcodes.  Static counts
(loops counted once) — a guide to where a kernel's VALU issue goes, next to
the SQ_INSTS_VALU PMC counts of tools/prof_run.sh.
  python tools/isa_stats.py FILE.s SYMBOL_SUBSTRING [--top N] [--dump]"""
import collections
import re
import sys


def body(path, sym):
    lines = open(path).read().split("\n")
    out, on = [], False
    for ln in lines:
        if not on and re.match(r"^_Z\S*:", ln) and sym in ln.split(":")[0]:
            on = True
            continue
        if on:
            if ln.startswith(".Lfunc_end") or re.match(r"^\s*\.size\s", ln):
                break
            out.append(ln)
    return out


def main():
    path, sym = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    b = body(path, sym)
    ops = []
    for ln in b:
        t = ln.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        ops.append(t.split()[0])
    cls = collections.Counter()
    valu = collections.Counter()
    for o in ops:
        if o.startswith("v_mfma"):
            cls["mfma"] += 1
        elif o.startswith("v_"):
            cls["valu"] += 1
            valu[o] += 1
        elif o.startswith("ds_"):
            cls["lds"] += 1
        elif o.startswith(("global_", "buffer_", "flat_", "scratch_")):
            cls["vmem"] += 1
        elif o.startswith("s_"):
            cls["salu/ctl"] += 1
        else:
            cls["other"] += 1
    print(dict(cls), "total", len(ops))
    for o, c in valu.most_common(top):
        print(f"{c:6d} {o}")
    if "--dump" in sys.argv:
        print("\n".join(b))


if __name__ == "__main__":
    main()


def loops(path, sym):
    """VALU count inside each loop (from its header label to its back-edge branch)."""
    b = body(path, sym)
    labels = {}
    for i, ln in enumerate(b):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            labels[m.group(1)] = i
    out = []
    for i, ln in enumerate(b):
        m = re.match(r"^\s*s_cbranch_\w+\s+(\.LBB\S+)|^\s*s_branch\s+(\.LBB\S+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                seg = b[labels[tgt]:i + 1]
                v = sum(1 for x in seg if x.strip().startswith("v_") and not x.strip().startswith("v_mfma"))
                out.append((tgt, labels[tgt], i, v))
    return out


if __name__ == "__main__" and "--loops" in sys.argv:
    for t, a, z, v in loops(sys.argv[1], sys.argv[2]):
        print(f"loop {t}: lines {a}-{z}, VALU {v}")


def phases(path, sym):
    """VALU per segment between workgroup barriers (s_barrier)."""
    b = body(path, sym)
    seg, out = 0, []
    for ln in b:
        t = ln.strip()
        if t.startswith("s_barrier"):
            out.append(seg)
            seg = 0
        elif t.startswith("v_") and not t.startswith("v_mfma"):
            seg += 1
    out.append(seg)
    return out


if __name__ == "__main__" and "--phases" in sys.argv:
    print("VALU between barriers:", phases(sys.argv[1], sys.argv[2]))
