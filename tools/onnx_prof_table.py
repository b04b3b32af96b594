"""Per (kernel, grid) table of one tools/prof_onnx.sh directory: launches per
run, mean duration in the kernel-trace pass, and the FETCH_SIZE / WRITE_SIZE
passes' bytes per launch (FETCH_SIZE doubled: gfx950 counts 64 B per 128-B
request, MI355X_MICROARCH.md §HBM; calibrated on k_conv_tile's buffer loads,
tools/conv_probe.py), sorted by total time.  The passes run the kernels one
at a time (PMC) or as the session's lanes issue them (trace).
    python tools/onnx_prof_table.py gpurun_out/prof_TAG [runs] [top]"""
import csv
import glob
import sys
from collections import defaultdict


def rows(root, sub):
    for f in glob.glob(f"{root}/{sub}/**/*.csv", recursive=True):
        if f.endswith("run_kernel_trace.csv") or f.endswith("run_counter_collection.csv"):
            yield from csv.DictReader(open(f))


def main():
    root = sys.argv[1]
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 70
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    dur, fetch, write = defaultdict(list), defaultdict(list), defaultdict(list)
    for r in rows(root, "trace"):
        g = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y") or 1) * int(r.get("Grid_Size_Z") or 1)
        k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), str(g))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for sub, dst in (("fetch", fetch), ("write", write)):
        for r in rows(root, sub):
            k = (r["Kernel_Name"].split("(")[0].replace("void ", ""), str(int(float(r["Grid_Size"]))))
            dst[k].append(float(r["Counter_Value"]) * 1024 * (2 if sub == "fetch" else 1))
    tot = sum(sum(v) for v in dur.values()) / runs
    out = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    print(f"kernel time per run {tot:.1f} us ({runs} runs)")
    print(f"{'kernel':56s} {'grid':>8s} {'/run':>5s} {'us':>7s} {'us/run':>7s} {'fetch MB':>9s} {'write MB':>9s} {'TB/s':>6s}")
    for k, v in out[:top]:
        m = sum(v) / len(v)
        f = sum(fetch[k]) / len(fetch[k]) / 1e6 if fetch.get(k) else float("nan")
        w = sum(write[k]) / len(write[k]) / 1e6 if write.get(k) else float("nan")
        print(f"{k[0][:56]:56s} {k[1]:>8s} {len(v) / runs:5.1f} {m:7.2f} {sum(v) / runs:7.1f} {f:9.2f} {w:9.2f} "
              f"{(f + w) / m if m else 0:6.2f}")


if __name__ == "__main__":
    main()
