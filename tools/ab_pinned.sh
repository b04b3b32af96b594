#!/bin/bash
# A/B of library builds (same ABI) with the layer tiles pinned, interleaved:
#   bash tools/ab_pinned.sh LIB [LIB...]     (the in-tree libvss.so is always included)
export VSS_TILE=${VSS_TILE:-"1:4x16,2:2x8,3:3x16,4:2x8,5:4x8,6:2x8,7:6x8,8:2x8,9:4x8,10:6x16"}
for r in 1 2; do
  for lib in video-stream-segmenetation_amd/lib/libvss.so "$@"; do
    VSS_LIBRARY=$lib timeout -k 10 120 python bench.py --no-cpu --no-host --no-ts --no-post --no-sweep --steps 400 \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib'.split('/')[-1], d['value'], [round(k['ms']*1000,2) for k in d['kernels']])" || exit 1
  done
done
