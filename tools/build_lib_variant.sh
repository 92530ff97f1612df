#!/bin/bash
# Build a whole-library A/B variant from a directory holding replacement csrc files:
#   tools/build_lib_variant.sh NAME DIR   -> build/k12var/NAME.so (travels with gpurun; git-ignored)
# Files in DIR replace same-named files of packnet-sfm-resnet-san_amd/csrc; per-TU flags as build().
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; DIR=$2
T=$(mktemp -d "$ROOT/build/var-XXXX")
trap 'rm -rf "$T"' EXIT
cp "$ROOT"/packnet-sfm-resnet-san_amd/csrc/* "$T/"
cp "$DIR"/* "$T/"
sed -i "s#\"../../include/#\"$ROOT/include/#" "$T"/*.hip "$T"/*.h
mkdir -p "$ROOT/build/k12var"
for f in "$T"/*.hip; do
  extra=""; [ "$(basename "$f")" = "psfm_photometric.hip" ] && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall $extra -DPSFM_SRC_HASH="\"var-$NAME\"" \
    -I "$ROOT/include" -c "$f" -o "$f.o" 2>/dev/null &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$T"/*.o -o "$ROOT/build/k12var/$NAME.so"
ls -la "$ROOT/build/k12var/$NAME.so"
