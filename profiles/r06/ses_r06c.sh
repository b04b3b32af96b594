#!/bin/bash
# Round-6 session c: the copy pool's protocol A/B (the bench's TS and host
# legs, new vs VSS_COPY_WAIT_ALL=1, interleaved x2) and the TS phase table per
# arm; then the MODNet b8 PMC passes (bf16, f16: MFMA busy per kernel) and the
# seam's MFMA pass.
TAG=${1:-r06c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "step rc=$1: stopping"; exit $1;; esac; }
for i in 1 2; do
  for arm in new waitall; do
    if [ $arm = waitall ]; then export VSS_COPY_WAIT_ALL=1; else unset VSS_COPY_WAIT_ALL; fi
    timeout -k 10 300 python bench.py --steps 400 --no-cpu --no-post --no-sweep --no-latency > gpurun_out/${TAG}_${arm}_$i.log 2>&1; rc=$?; fatal $rc
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_${arm}_$i.log').read().splitlines()[-1]);h=d['host_path']['vga'];t=d['ts_path'];print('$arm',$i,'value',d['value'],'C copy',h['copy']['value'],'pinned',h['copy_pinned_out']['value'],'zc',h['zero_copy']['value'],'TS',t['value'],'TSzc',t['zero_copy']['value'],'frame p50',t['single_frame']['latency_ms_p50'])"
    timeout -k 10 300 node tools/ts_prof.js 400 > gpurun_out/${TAG}_${arm}_tsprof_$i.json 2>&1; rc=$?; fatal $rc
    python3 -c "
import json;d=json.load(open('gpurun_out/${TAG}_${arm}_tsprof_$i.json'))
for m,v in d.items(): print('  ',m,{k:v[k]['p50'] for k in v if k.endswith('_us')}, v.get('frames_per_s',''))"
  done
done
unset VSS_COPY_WAIT_ALL
for c in b8_bf16 b8_f16; do
  bash tools/prof_onnx.sh ${TAG}_modnet_$c --only-modnet --batch 8 --iters 50 --cases $c > gpurun_out/${TAG}_modnet_$c.log 2>&1; rc=$?; fatal $rc
  echo "== MODNet $c"; python3 tools/pmc_table.py gpurun_out/prof_${TAG}_modnet_$c/mfma/run_counter_collection.csv 22
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --output-format csv -d "$R/gpurun_out/prof_${TAG}_seam/mfma" -o run -- \
  python3 "$R/bench.py" --no-cpu --no-host --no-ts --no-sweep --no-post --no-latency --steps 200 --warmup 5 > "$R/gpurun_out/${TAG}_seam_mfma.log" 2>&1; rc=$?
cd "$R"; fatal $rc
echo "== seam"; python3 tools/pmc_table.py gpurun_out/prof_${TAG}_seam/mfma/run_counter_collection.csv 14
