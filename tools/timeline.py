"""Per-queue timeline of a rocprofv3 kernel trace (run_kernel_trace.csv):
for the forward launches of the bench's timed region, the busy time of each
hardware queue, the gaps between a queue's consecutive kernels, and how many
queues were running a kernel at each instant (concurrency histogram).
Usage: python tools/timeline.py gpurun_out/tl/run_kernel_trace.csv [first_dispatch_frac]"""
import collections
import csv
import sys

import numpy as np


def main(path, skip=0.3):
    rows = [r for r in csv.DictReader(open(path)) if "k_block" in r["Kernel_Name"] or "k_head" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * skip):int(len(rows) * 0.6)]  # a steady stretch of the timed region
    t0 = int(rows[0]["Start_Timestamp"])
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r["Queue_Id"]].append((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"]))
    span = max(e for q in byq.values() for _, e, _ in q) - min(s for q in byq.values() for s, _, _ in q)
    print(f"{len(rows)} kernels over {span / 1e3:.1f} us on queues {sorted(byq)}")
    for q, ks in sorted(byq.items()):
        busy = sum(e - s for s, e, _ in ks)
        gaps = [ks[i + 1][0] - ks[i][1] for i in range(len(ks) - 1)]
        print(f"queue {q}: {len(ks)} kernels, busy {busy / span * 100:.0f}% of the span, mean kernel "
              f"{busy / len(ks) / 1e3:.2f} us, gap median {np.median(gaps) / 1e3:.2f} us mean {np.mean(gaps) / 1e3:.2f} us")
    # concurrency: queues with a kernel running, sampled every 100 ns
    ts = np.arange(0, span, 100)
    conc = np.zeros_like(ts)
    for ks in byq.values():
        for s, e, _ in ks:
            conc[(ts >= s) & (ts < e)] += 1
    h = np.bincount(conc, minlength=5)
    print("fraction of time with k queues running:", {k: round(float(v) / len(ts), 3) for k, v in enumerate(h)})
    # per-kernel duration by layer kind (name)
    dur = collections.defaultdict(list)
    for ks in byq.values():
        for s, e, n in ks:
            dur[n].append(e - s)
    for n, v in sorted(dur.items(), key=lambda kv: -np.mean(kv[1])):
        print(f"  {np.mean(v) / 1e3:6.2f} us  x{len(v):4d}  {n[:90]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.3)
