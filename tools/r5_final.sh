#!/bin/bash
# Final evidence for a list of configs on the current library: stamped PMC passes
# (tools/gpu_pmc_bench.sh -> gpurun_out/pmc/<key>/<key>.json) then a bench line + rocprof step summary
# (tools/r5_bench.sh --prof).  usage: tools/r5_final.sh TAG config [config ...]
set -u
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_cache
mkdir -p "$ROOT/gpurun_out/$TAG"
(for i in $(seq 1 300); do date >> "$ROOT/gpurun_out/$TAG/heartbeat_final.txt"; sleep 15; done) & hb=$!
trap 'kill $hb 2>/dev/null' EXIT
for cfg in "$@"; do
  PMC_EXTRA=--no-miopen-find bash "$ROOT/tools/gpu_pmc_bench.sh" --config "$cfg" || exit $?
done
bash "$ROOT/tools/r5_bench.sh" "$TAG" --prof "$@"
