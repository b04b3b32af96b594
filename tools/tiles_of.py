"""The VSS_TILE spec ("layer:THxTW,...") of the kernels a bench.py JSON line
timed (its per-layer `kernels` entries): python tools/tiles_of.py bench.json"""
import json
import re
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
if d.get("tile_spec"):  # by candidate index (bench.py >= round 3): exact for every kernel variant
    print(d["tile_spec"])
    sys.exit(0)
spec = []
for k in d["kernels"]:
    m = re.search(r"k_block<\s*\d+,\s*\d+,\s*(\d+),\s*(\d+),", k["kernel"])
    if m:
        spec.append(f"{k['layer']}:{m.group(1)}x{m.group(2)}")
print(",".join(spec))
