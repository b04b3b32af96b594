"""Mean duration per (kernel, grid) of the k_conv_tile 5x5 launches in a rocprofv3 kernel-trace directory."""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_conv_tile" in r["Kernel_Name"] and ", 5, 1," in r["Kernel_Name"]:
            d[(r["Kernel_Name"].split("(")[0][10:], r["Grid_Size_X"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    print(f"  {k[0]} grid {k[1]}: {len(v)} launches, mean {sum(v) / len(v):.1f} us")
