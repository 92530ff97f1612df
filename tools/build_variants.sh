#!/bin/bash
# Build A/B variants of libpsfm_hip.so (git-ignored build/variants/, travels with gpurun) from
# "name:-DFLAG=.. -DFLAG=.." specs, for tools/kbench.py --lib.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build/variants"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -I "$ROOT/include" $flags \
    "$ROOT"/packnet-sfm-resnet-san_amd/csrc/*.hip -o "$ROOT/build/variants/$name.so" &
done
wait
ls "$ROOT/build/variants"
