#!/bin/bash
# RX check: the RX + spectrum parity tests, then the C3 SAM and C4 FM lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_paths.py tests/test_gpu_pipelined.py tests/test_gpu_fma.py tests/test_status.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rxc_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/rxc_pytest.log
[ $rc -eq 0 ] || { grep -m5 -B5 -A30 "Error\|FAIL" gpurun_out/rxc_pytest.log | head -80; exit $rc; }
timeout -k 10 300 python tools/bench_configs.py --only c3,c4fm > gpurun_out/rxc_cfg.jsonl 2> gpurun_out/rxc_cfg.err || { tail -20 gpurun_out/rxc_cfg.err; exit 1; }
cut -c1-300 gpurun_out/rxc_cfg.jsonl
