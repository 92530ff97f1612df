#!/bin/bash
# A/B builds for tools/kbench.py --lib: build/variants/<name>.so from the csrc/ + include/ of a git
# revision (or "WORKTREE" for the working tree).  Specs: name:rev
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build/variants"
for spec in "$@"; do
  IFS=: read -r name rev <<< "$spec"
  d="$ROOT/build/variants/rev_$name"; rm -rf "$d"; mkdir -p "$d"
  if [ "$rev" = WORKTREE ]; then
    cp -r "$ROOT/include" "$d/"; mkdir -p "$d/pkg"; cp -r "$ROOT/packnet-sfm-resnet-san_amd/csrc" "$d/pkg/"
  else
    (cd "$ROOT" && git archive "$rev" include packnet-sfm-resnet-san_amd/csrc) | tar -x -C "$d"
    mv "$d/packnet-sfm-resnet-san_amd" "$d/pkg"
  fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -I "$d/include" "$d"/pkg/csrc/*.hip \
    -o "$ROOT/build/variants/$name.so" &
done
wait
rm -rf "$ROOT"/build/variants/rev_*
ls -la "$ROOT/build/variants"
