"""Per-kernel MFMA utilisation table of one rocprofv3 --pmc pass (csv) over
SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA, SQ_INSTS_VALU, SQ_INSTS_LDS,
SQ_LDS_BANK_CONFLICT and GRBM_GUI_ACTIVE (tools/prof_onnx.sh / prof_run.sh's
"mfma" pass): per dispatch averages,
  util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs)
(GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles; MFMA busy counts every SIMD's
MFMA pipe cycles).  Sorted by the kernel's total GRBM cycles.
  python3 tools/pmc_table.py run_counter_collection.csv [top]"""
import csv
import sys
from collections import defaultdict


def main():
    d = defaultdict(lambda: defaultdict(list))
    disp = defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        k = r["Kernel_Name"]
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows = []
    for k, c in d.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        g = m.get("GRBM_GUI_ACTIVE", 0.0)
        rows.append((g * len(disp[k]), k, len(disp[k]), m))
    rows.sort(key=lambda x: -x[0])
    print(f"{'kernel':58s} {'disp':>5s} {'GRBM/8':>8s} {'MFMA busy':>10s} {'util':>6s} {'MFMA':>8s} {'VALU':>9s} "
          f"{'LDS':>8s} {'bankc':>8s}")
    for _, k, n, m in rows[:top]:
        g8 = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        util = busy / (g8 * 256 * 4) if g8 > 0 else 0.0
        name = k.split("(")[0].replace("void ", "")[:58]
        print(f"{name:58s} {n:5d} {g8:8.0f} {busy:10.0f} {util:6.3f} {m.get('SQ_INSTS_MFMA', 0):8.0f} "
              f"{m.get('SQ_INSTS_VALU', 0):9.0f} {m.get('SQ_INSTS_LDS', 0):8.0f} {m.get('SQ_LDS_BANK_CONFLICT', 0):8.0f}")


if __name__ == "__main__":
    main()
