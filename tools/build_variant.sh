#!/bin/bash
# Build libvss.so from the current sources with extra compile flags into
# abvar/libvss_<name>.so (a separate tree under /tmp; the in-tree build is
# untouched).  Usage: tools/build_variant.sh NAME "-DVSS_X=1 ..."
set -e
NAME=$1; FLAGS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/vssvar_$NAME
rm -rf "$T"; mkdir -p "$T/video-stream-segmenetation_amd" "$R/abvar"
cp -r "$R/include" "$T/"
cp -r "$R/video-stream-segmenetation_amd/csrc" "$T/video-stream-segmenetation_amd/"
mkdir -p "$T/video-stream-segmenetation_amd/lib"
# a -DVSS_SWZ=0 build needs the registry's LDS sizes of round 4's layouts
case "$FLAGS" in *-DVSS_SWZ=0*)
  VSS_SWZ=0 VSS_REGISTRY_DIR="$T/video-stream-segmenetation_amd/csrc" python3 "$R/tools/gen_registry.py";;
esac
make -s -j8 -C "$T/video-stream-segmenetation_amd/csrc" HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form=1 $FLAGS" 2>&1 | grep -E "rror" || true
cp "$T/video-stream-segmenetation_amd/lib/libvss.so" "$R/abvar/libvss_$NAME.so"
echo "abvar/libvss_$NAME.so"
