#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$ROOT/tools/gpu_r2r.sh"; bash "$ROOT/tools/gpu_r2s.sh"
