#!/bin/bash
# K12 variants for tools/kbench.py --lib: copies csrc/ with edited compile-time constants of
# psfm_fused.h (WAVES) and builds build/variants/<name>.so.  Specs: name:WAVES[:probe[+probe]]
# (probes: tools/k12_probe_patch.py — timing-only builds)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build/variants"
for spec in "$@"; do
  IFS=: read -r name waves probes <<< "$spec"
  d="$ROOT/build/variants/src_$name/a/b"; rm -rf "$ROOT/build/variants/src_$name"; mkdir -p "$d"
  cp -r "$ROOT/packnet-sfm-resnet-san_amd/csrc" "$d/"
  sed -i "s/^constexpr int WAVES = [0-9]*;/constexpr int WAVES = $waves;/" "$d/csrc/psfm_fused.h"
  for pr in ${probes//+/ }; do python3 "$ROOT/tools/k12_probe_patch.py" "$d/csrc/psfm_fused.h" "$pr"; done
  sed -i 's#"../../include/#"../../../../../../include/#' "$d"/csrc/*.hip "$d"/csrc/*.h
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -I "$ROOT/include" "$d"/csrc/*.hip \
    -o "$ROOT/build/variants/$name.so" &
done
wait
rm -rf "$ROOT"/build/variants/src_*
ls "$ROOT/build/variants"
