#!/bin/bash
# Round-3 closing evidence: gpu_full.sh (tests, smoke, bench, kernel traces, PMC) then the
# per-config lines, kernel traces and PMC (gpu_configs.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
tag=${1:-r03b}
bash tools/gpu_full.sh $tag || exit 1
bash tools/gpu_configs.sh $tag c3,c3spec,c4fm,c4tx,c5,c5fir || exit 1
