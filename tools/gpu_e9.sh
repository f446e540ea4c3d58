#!/bin/bash
# GPU suite on the working tree, north-star lines (R = 8 / 16, EXACT / FMA), then the
# north-star PMC passes of the working tree (tools/gpu_pmc.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/e9_pytest.log 2>&1 || { tail -60 gpurun_out/e9_pytest.log; exit 1; }
tail -1 gpurun_out/e9_pytest.log
bash tools/gpu_lib_ab.sh e9 "r8||--schedule fused" "r16||--schedule fused --front-block 16" "r8fma||--schedule fused --precision fma" "r16fma||--schedule fused --front-block 16 --precision fma" || exit 1
bash tools/gpu_pmc.sh ns --workload northstar --steps 20 --warmup 3 --schedule fused
