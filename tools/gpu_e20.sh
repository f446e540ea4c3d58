#!/bin/bash
# pipelined RX parity tests, host submission cost, C2 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_schedules.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/e20_pytest.log 2>&1 || { tail -40 gpurun_out/e20_pytest.log; exit 1; }
tail -1 gpurun_out/e20_pytest.log
timeout -k 10 200 python tools/host_cost.py || exit 1
WL=c2 bash tools/gpu_lib_ab.sh e20 "c2||" "c2b||" "serial||--serial"
