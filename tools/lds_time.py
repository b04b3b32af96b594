"""LDS x lifetime of one forward, per layer, from a bench JSON line (the
steady-state model of DESIGN.md §3 "What bounds 4 batches in flight").

At 4 batches in flight the CUs are LDS-full (tools/trace_inflight.py: ~3.3
workgroups per CU, ~4 % idle), so a layer costs the chip roughly
    workgroups x LDS bytes x workgroup lifetime
of its 256 x 160 KiB of LDS, and one forward's sum over the layers divided by
the chip's LDS predicts the steady-state step.  A workgroup's lifetime is the
kernel's duration (one batch at a time, the bench's event pass) over its rounds
of workgroups (ceil(workgroups / (CUs x workgroups per CU))).

  python3 tools/lds_time.py BENCH.json [--batch 8] [--model 144x256]
"""
from __future__ import annotations

import argparse
import json
import math
import re

CUS, LDS_CU = 256, 160 * 1024
GRANULE = 2048


def layer_out(kind_stride_res, hm, wm):
    d = {"/2": 2, "/4": 4, "/8": 8, "/16": 16}[kind_stride_res]
    return -(-hm // d), -(-wm // d)


RES = {1: "/2", 2: "/4", 3: "/4", 4: "/8", 5: "/8", 6: "/16", 7: "/16", 8: "/8", 9: "/4", 10: "/2"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--model", default="144x256")
    a = ap.parse_args()
    raw = open(a.bench).read()
    try:
        d = json.loads(raw)
    except json.JSONDecodeError:  # a log: its last JSON line
        d = json.loads(next(x for x in reversed(raw.strip().splitlines()) if x.startswith("{")))
    if "run" in d and "stdout_tail" in d["run"]:  # a driver record (BENCH_rNN.json)
        d = json.loads([x for x in d["run"]["stdout_tail"].splitlines() if x.startswith("{")][-1])
    hm, wm = (int(v) for v in a.model.split("x"))
    rows, total = [], 0.0
    for k in d["kernels"]:
        m = re.search(r"k_block<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", k["kernel"])
        if not m or not k.get("lds_bytes"):
            continue
        th, tw, flags = int(m.group(3)), int(m.group(4)), int(m.group(9))
        ks = ((flags >> 6) & 3) + 1
        ho, wo = layer_out(RES[k["layer"]], hm, wm)
        wgs = math.ceil(ho / th) * math.ceil(wo / tw) * a.batch * ks
        lds = math.ceil(k["lds_bytes"] / GRANULE) * GRANULE
        per_cu = k["wg_per_cu"] or 1
        rounds = math.ceil(wgs / (CUS * per_cu))
        life_us = k["ms"] * 1e3 / rounds
        cost = wgs * lds * life_us / 1e6  # MB x us
        total += cost
        rows.append((k["layer"], f"{th}x{tw}", wgs, per_cu, k["lds_bytes"], rounds, round(k["ms"] * 1e3, 2),
                     round(life_us, 2), round(cost, 1)))
    print(f"{'layer':>5} {'tile':>6} {'WGs':>5} {'WG/CU':>5} {'LDS B':>7} {'rounds':>6} {'kernel us':>9} "
          f"{'life us':>7} {'MB*us':>7}")
    for r in rows:
        print(f"{r[0]:>5} {r[1]:>6} {r[2]:>5} {r[3]:>5} {r[4]:>7} {r[5]:>6} {r[6]:>9} {r[7]:>7} {r[8]:>7}")
    chip = CUS * LDS_CU / 1e6
    print(f"sum {total:.0f} MB*us over {chip:.1f} MB of LDS: predicted step >= {total / chip:.1f} us "
          f"(+ the head and the stem-less layers); measured median step "
          f"{(d.get('median_step_ms') or 0) * 1e3:.1f} us, the window's {d['ms_per_step'] * 1e3:.1f} us")


if __name__ == "__main__":
    main()
