"""Summarise a tools/prof_run.sh output directory into profiles/.

Reads the rocprofv3 kernel-trace stats (mean duration per kernel) and the two
PMC passes (FETCH_SIZE, WRITE_SIZE per dispatch) and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats table as collected
  profiles/<tag>_summary.md         per-kernel duration, HBM bytes, GB/s
  profiles/<tag>_traffic.json       {kernel name: {...}} read by bench.py

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md §HBM and
cdna_hip_programming.md §7: FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  Infinity-Cache hits are
counted by these memory-side counters (they are L2-miss traffic, not strictly
DRAM traffic) — stated in the summary.

    python tools/prof_summary.py gpurun_out/prof_r01 r01
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, tag = sys.argv[1], sys.argv[2]
    command = sys.argv[3] if len(sys.argv) > 3 else f"bash tools/prof_run.sh {tag} ..."
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    pmc = defaultdict(lambda: defaultdict(list))
    for kind in ("fetch", "write", "mfma"):
        p = os.path.join(src, kind, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    traffic = {}
    for s in stats:
        name = s["Name"]
        avg_ns = float(s["AverageNs"])
        f = pmc.get(name, {}).get("FETCH_SIZE", [])
        w = pmc.get(name, {}).get("WRITE_SIZE", [])
        fetch_b = 2.0 * 1024.0 * (sum(f) / len(f)) if f else None
        write_b = 1024.0 * (sum(w) / len(w)) if w else None
        tb = (fetch_b or 0.0) + (write_b or 0.0) if (f or w) else None
        rows.append((name, int(s["Calls"]), avg_ns, fetch_b, write_b, tb))
        traffic[name] = {"avg_ns": avg_ns, "calls": int(s["Calls"]), "fetch_bytes": fetch_b,
                         "write_bytes": write_b, "traffic_bytes": tb,
                         "traffic_GBps": (tb / avg_ns) if tb else None}
        mf = {c: sum(v) / len(v) for c, v in pmc.get(name, {}).items() if c not in ("FETCH_SIZE", "WRITE_SIZE") and v}
        if mf:
            traffic[name]["sq"] = mf
            g = mf.get("GRBM_GUI_ACTIVE")
            if g and "SQ_VALU_MFMA_BUSY_CYCLES" in mf:
                # MFMA pipe busy over every SIMD's active cycles: GRBM_GUI_ACTIVE is
                # summed over the 8 XCDs (MI355X_MICROARCH.md), 32 CUs x 4 SIMDs each
                traffic[name]["mfma_util"] = mf["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8.0 * 256 * 4)
    # bench.py times its dominant kernel with launch events in a separate pass
    # that runs one batch at a time after the timed region (4 in flight);
    # the rocprof average above mixes both.  The mean of each kernel's last
    # `steps` dispatches is that isolated pass: the number to compare with the
    # bench line's roofline.mean_kernel_ms.
    log = open(os.path.join(src, "trace.log")).read().strip().splitlines()
    steps = None
    for l in reversed(log):
        if l.startswith("{"):
            try:
                steps = json.loads(l).get("steps")
            except ValueError:
                pass
            break
    iso = {}
    tpath = os.path.join(src, "trace", "run_kernel_trace.csv")
    if steps and os.path.exists(tpath):
        durs = defaultdict(list)
        for r in csv.DictReader(open(tpath)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for name, d in durs.items():
            if len(d) >= 2 * steps:
                iso[name] = sum(d[-steps:]) / steps
                if name in traffic:
                    traffic[name]["avg_ns_isolated_pass"] = iso[name]
    json.dump(traffic, open(os.path.join(out, f"{tag}_traffic.json"), "w"), indent=1)
    bench_lines = [l for l in log if l.startswith("{")]
    bench_line = "\n".join(bench_lines[-4:]) if "prof_onnx" in command else (bench_lines[-1] if bench_lines else "")
    with open(os.path.join(out, f"{tag}_summary.md"), "w") as fh:
        fh.write(f"# rocprofv3 summary `{tag}`\n\n")
        fh.write("Command: `" + command + "` (kernel trace + stats pass; separate FETCH_SIZE "
                 "and WRITE_SIZE PMC passes).  HBM bytes = 2 x FETCH_SIZE KiB + WRITE_SIZE KiB (gfx950 "
                 "correction); memory-side counters include Infinity-Cache hits.\n\n")
        if iso:
            fh.write(f"`mean us` is over every dispatch (the timed region runs 4 batches in flight, so kernels "
                     f"overlap and last longer); `isolated us` is the mean of each kernel's last {steps} dispatches "
                     f"= bench.py's one-batch-at-a-time event pass, the duration its roofline uses.\n\n")
        fh.write("| kernel | calls | mean us | isolated us | HBM read MB/launch | HBM write MB/launch | GB/s (PMC) | "
                 "MFMA util | MFMA insts | VALU insts | LDS insts | LDS bank conflicts |\n")
        fh.write("|---|---|---|---|---|---|---|---|---|---|---|---|\n")
        for name, calls, ns, fb, wb, tb in rows:
            t = traffic[name]
            sq = t.get("sq", {})
            mu = t.get("mfma_util")
            fmt = lambda k: f"{sq[k]:.0f}" if k in sq else "-"
            isu = f"{iso[name] / 1e3:.2f}" if name in iso else "-"
            fh.write(f"| `{name}` | {calls} | {ns / 1e3:.2f} | {isu} | {fb / 1e6 if fb else 0:.3f} | "
                     f"{wb / 1e6 if wb else 0:.3f} | {tb / ns if tb else 0:.0f} | "
                     f"{'-' if mu is None else f'{100 * mu:.2f}%'} | {fmt('SQ_INSTS_MFMA')} | {fmt('SQ_INSTS_VALU')} | "
                     f"{fmt('SQ_INSTS_LDS')} | {fmt('SQ_LDS_BANK_CONFLICT')} |\n")
        if bench_line:
            fh.write("\nbench line of the traced run:\n\n```\n" + bench_line + "\n```\n")
    print(open(os.path.join(out, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main()
