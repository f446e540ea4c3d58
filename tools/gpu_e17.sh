#!/bin/bash
# C2 A/B: front block 8 vs 16, schedule pipe vs fused
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
WL=c2 bash tools/gpu_lib_ab.sh e17 "r8||" "r16||--front-block 16" "fused||--schedule fused" "r8b||" "r16b||--front-block 16"
