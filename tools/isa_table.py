"""Static VALU per wave of the bench's 11 forward kernels (bf16x2), from the
device assembly of every k_block shard (tools/isa_shard.sh), with an
estimated dynamic count: loop bodies counted (trips - 1) more times, where an
expand layer's chunk loop runs NCHUNK / 4 times per wave.  A CPU-side guide
to SQ_INSTS_VALU (the PMC pass) while editing the kernels.
  python tools/isa_table.py [OUTDIR] [--no-build]"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_stats  # noqa: E402

# (name, template args) as bench.py's autotuned set (profiles/r03q/bench.json)
KERNELS = [("b1", (1, 1, 4, 16, 16, 0, 16, 16, 258)), ("b2", (0, 2, 2, 8, 16, 0, 64, 32, 0)),
           ("b3", (0, 1, 3, 16, 32, 0, 128, 32, 2)), ("b4", (0, 2, 2, 8, 32, 0, 128, 48, 0)),
           ("b5", (0, 1, 4, 8, 48, 0, 64, 48, 130)), ("b6", (0, 2, 2, 8, 48, 0, 64, 64, 136)),
           ("b7", (0, 1, 4, 8, 64, 0, 64, 64, 202)), ("d1", (2, 1, 2, 8, 64, 48, 112, 48, 44)),
           ("d2", (2, 1, 4, 8, 48, 32, 80, 32, 1)), ("d3", (2, 1, 6, 16, 32, 16, 48, 16, 1))]
# waves per launch at batch 8, 144x256 (tiles x frames x KS x 4 waves)
WAVES = {"b1": 1152 * 4, "b2": 1152 * 4, "b3": 384 * 4, "b4": 288 * 4, "b5": 480 * 4, "b6": 240 * 4,
         "b7": 192 * 4, "d1": 288 * 4, "d2": 576 * 4, "d3": 768 * 4}


def shard_of(args):
    pat = "VSS_BLOCK(" + ", ".join(str(a) for a in args) + ")"
    for k in range(6):
        if pat in open(os.path.join(ROOT, "video-stream-segmenetation_amd/csrc", f"vss_registry_{k}.inc")).read():
            return k
    raise KeyError(args)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "/tmp/isa"
    os.makedirs(out, exist_ok=True)
    shards = sorted({shard_of(a) for _, a in KERNELS})
    if "--no-build" not in sys.argv:
        with ThreadPoolExecutor(6) as ex:
            list(ex.map(lambda k: subprocess.run(["bash", os.path.join(ROOT, "tools/isa_shard.sh"), str(k),
                                                  f"{out}/s{k}.s"], check=True), shards))
    tot = 0.0
    for name, a in KERNELS:
        sym = "ILi" + "ELi".join(str(x) for x in a) + "ELi1E"
        f = f"{out}/s{shard_of(a)}.s"
        ops = [ln.strip().split()[0] for ln in isa_stats.body(f, sym)
               if ln.strip() and not ln.strip().startswith((";", ".", "//")) and not ln.strip().endswith(":")]
        valu = sum(1 for o in ops if o.startswith("v_") and not o.startswith("v_mfma"))
        lds = sum(1 for o in ops if o.startswith("ds_"))
        lp = isa_stats.loops(f, sym)
        dyn = valu
        if a[0] == 0:  # expand: the chunk loop
            trips = a[6] // 16 // 4
            for _, _, _, v in lp:
                dyn += v * (trips - 1)
        tot += dyn * WAVES[name]
        print(f"{name}: static VALU {valu:5d}  LDS {lds:4d}  loops {[v for *_, v in lp]}  est. dynamic/wave {dyn:5d}"
              f"  est. per launch {dyn * WAVES[name] / 1e6:.2f} M")
    print(f"blocks total est. {tot / 1e6:.2f} M VALU per 8-frame forward (+ head)")


if __name__ == "__main__":
    main()
