"""Per-kernel means of the SQ counters of one rocprofv3 --pmc pass (csv), the
forward's 11 kernels first, and the per-forward VALU total.
  python tools/sq_table.py run_counter_collection.csv"""
import csv
import sys
from collections import defaultdict


def main():
    d = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(sys.argv[1])):
        d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, c in d.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        rows.append((k, len(c.get("SQ_INSTS_VALU", [])), m))
    rows.sort(key=lambda x: -x[1])
    # The timed forwards' kernels: every hot kernel has (about) the same dispatch
    # count; autotune candidates and one-off launches have far fewer.
    hot = [n for k, n, m in rows if "k_block" in k or "k_head" in k or "k_stem" in k]
    thr = 0.8 * max(hot) if hot else 0
    tot = 0.0
    for k, n, m in rows:
        if "k_block" in k or "k_head" in k or "k_stem" in k:
            if n >= thr:
                tot += m.get("SQ_INSTS_VALU", 0)
            print(f"{n:5d} VALU {m.get('SQ_INSTS_VALU', 0) / 1e6:7.3f} M  LDS {m.get('SQ_INSTS_LDS', 0) / 1e3:8.1f} k"
                  f"  MFMA {m.get('SQ_INSTS_MFMA', 0) / 1e3:7.1f} k  bankc {m.get('SQ_LDS_BANK_CONFLICT', 0) / 1e3:8.1f} k"
                  f"  waves {m.get('SQ_WAVES', 0):8.0f}  {k[:90]}")
    print(f"forward VALU (kernels with >= {thr:.0f} dispatches): {tot / 1e6:.3f} M")


if __name__ == "__main__":
    main()
