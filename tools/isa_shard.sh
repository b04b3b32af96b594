#!/bin/bash
# Device assembly of one k_block shard (no in-tree build): tools/isa_shard.sh K OUT.s [extra hipcc flags]
K=$1; OUT=$2; shift 2
cd "$(dirname "$0")/../video-stream-segmenetation_amd/csrc" && \
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form=1 -DVSS_SHARD=$K \
  --cuda-device-only -S vss_kernels.hip -o "$OUT" "$@" 2>&1 | grep -v "argument unused" 
exit 0
