#!/bin/bash
# GPU suite on the working tree, then north-star lines and the rx_front LDS PMC pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/e13_pytest.log 2>&1 || { tail -60 gpurun_out/e13_pytest.log; exit 1; }
tail -1 gpurun_out/e13_pytest.log
bash tools/gpu_lib_ab.sh e13 "r8||--schedule fused" "r8fma||--schedule fused --precision fma" "r8b||--schedule fused" "r8fmab||--schedule fused --precision fma" "chain||--schedule chain" || exit 1
true
